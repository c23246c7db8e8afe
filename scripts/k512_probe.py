"""Config C5 probe: bench.k512_measure on cuda:0 (one JSON line)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
import cda  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ctx = cda.Context(0)
print(json.dumps(bench.k512_measure(ctx, dev)), flush=True)
