"""Config C2 probe: one k=128 block, device-resident latency and per-kernel split (bench.single_block_measure)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import torch  # noqa: E402,F401  (first: libcda then resolves HIP through torch's runtime)
import bench  # noqa: E402
import cda  # noqa: E402

print(json.dumps(bench.single_block_measure(cda.Context(0), torch.device("cuda", 0))))
