"""bench.repair_measure's C4 sequence with libcda's per-phase host trace (CDA_REPAIR_TRACE=1 on the command
line): which phase moves when a host-buffer repair is slow."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import cda  # noqa: E402

torch.cuda.init()
ctx = cda.Context(0)
for rep in range(2):
    print(json.dumps(bench.repair_measure(ctx, reps=9)), flush=True)
