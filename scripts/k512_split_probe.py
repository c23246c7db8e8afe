"""Config C5 on one GPU: bench.k512_measure alone (block path, C-ABI split G=1 / G=8 replicas, python split)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import cda  # noqa: E402

dev = torch.device("cuda", 0)
ctx = cda.Context(0)
print(json.dumps(bench.k512_measure(ctx, dev, reps=int(sys.argv[1]) if len(sys.argv) > 1 else 3)), flush=True)
ctx.close()
