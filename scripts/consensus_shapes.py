"""The one-block consensus call in every shape go/cda makes it (bench.one_block_fresh): roots only with fresh shares,
pooled share / EDS slabs (cda_host_register), fresh EDS buffers with and without the huge-page opt-in, pinned.
Prints one JSON line; `python scripts/consensus_shapes.py [reps] [rounds]`."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
import cda  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 25
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ctx = cda.Context(0)
ods = bench.gen_ods(128, 0xC0FFEE)
for r in range(rounds):
    res = bench.one_block_fresh(ctx, ods, reps=reps)
    print(json.dumps({"round": r, **{k: v for k, v in res.items() if k != "note"}}), flush=True)
