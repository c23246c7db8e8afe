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
for arg in libs:  # lib.so or lib.so@VAR=value (a knob of the test-hooks build, set for that run only)
    lib, _, assign = arg.partition("@")
    name = os.path.basename(lib) + (f"@{assign}" if assign else "")
    var, _, val = assign.partition("=")
    if var:
        os.environ[var] = val
    try:
        out[name] = bench.per_axis_measure("cda", lib)
    except Exception as e:  # noqa: BLE001
        out[name] = {"error": f"{type(e).__name__}: {e}"}
    finally:
        if var:
            del os.environ[var]
    print(json.dumps({name: out[name]}), flush=True)
out["oracle"] = bench.per_axis_measure("oracle", os.path.join(ROOT, "oracle", "liboracle.so"), reps=3, reps_repair=2,
                                       reps_single=100)
print(json.dumps(out), flush=True)
