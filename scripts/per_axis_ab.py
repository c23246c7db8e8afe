"""Same-box A/B of the per-axis seams (bench.py per_axis_measure): each libcda build given on the command line, then
the CPU restatement (oracle) in the same shapes.  python scripts/per_axis_ab.py [lib.so ...] > out.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402

libs = sys.argv[1:] or [os.path.join(ROOT, "celestia-app_amd", "cda", "libcda.so")]
out = {}
for lib in libs:
    try:
        out[os.path.basename(lib)] = bench.per_axis_measure("cda", lib)
    except Exception as e:  # noqa: BLE001
        out[os.path.basename(lib)] = {"error": f"{type(e).__name__}: {e}"}
    print(json.dumps({os.path.basename(lib): out[os.path.basename(lib)]}), flush=True)
out["oracle"] = bench.per_axis_measure("oracle", os.path.join(ROOT, "oracle", "liboracle.so"), reps=3, reps_repair=2,
                                       reps_single=100)
print(json.dumps(out), flush=True)
