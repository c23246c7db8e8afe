"""cda_extend_commit_nodes alone (k=128: every row tree's nodes, as go/cda.Nodes and pkg/inclusion's subtree cacher
take them; optionally the column trees too): per-call times.  python scripts/node_export_probe.py [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
import cda  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ctx = cda.Context(0)
ods = bench.gen_ods(128, 0xC0FFEE)
out = {}
for label, kw in (("rows", dict(rows=True, cols=False, dah_tree=False)),
                  ("rows_dah", dict(rows=True, cols=False, dah_tree=True)),
                  ("rows_cols_dah", dict(rows=True, cols=True, dah_tree=True))):
    ctx.extend_commit_nodes(ods, **kw)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.extend_commit_nodes(ods, **kw)
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    out[label] = {"min_ms": round(ts[0], 3), "median_ms": round(ts[len(ts) // 2], 3)}
print(json.dumps(out))
