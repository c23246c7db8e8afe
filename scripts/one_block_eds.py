"""One k=128 block with its EDS through host buffers (cda_extend_commit_batch, nblocks = 1), 8 calls, for tracing."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import bench  # noqa: E402
import cda  # noqa: E402

ctx = cda.Context(0)
k, w = 128, 256
ods = bench.gen_ods(k, 1).reshape(1, k * k, 512)
out = np.zeros((1, w * w, 512), np.uint8)
for i in range(8):
    t0 = time.perf_counter()
    ctx.extend_commit_batch(ods, True, out)
    print(round((time.perf_counter() - t0) * 1e3, 3))
