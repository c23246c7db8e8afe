"""First-process D2H on a fresh box: one k=128 block into pinned buffers (cda_host_alloc), median of 10 calls,
every ~2 s for `secs` seconds, plus a 256 MiB pinned D2H copy rate each time -- does a slow first process recover
within the process (box warm-up) or stay slow (process state)?"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
import cda  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60
ctx = cda.Context(0)
k, w = 128, 256
ods = bench.gen_ods(k, 0xC0FFEE).reshape(k * k, 512)
pb_ods, pb_eds = ctx.pinned((1, k * k, 512)), ctx.pinned((1, w * w, 512))
pb_ods.array[0] = ods
h = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
d = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
t_start = time.time()
while time.time() - t_start < secs:
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        ctx.extend_commit_batch(pb_ods.array, eds_out=pb_eds.array)
        ts.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    d2h = h.numel() / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    h2d = h.numel() / (time.perf_counter() - t0) / 1e9
    print(json.dumps({"t_s": round(time.time() - t_start, 1), "pinned_one_block_ms": round(float(np.median(ts)), 3),
                      "d2h_gbs": round(d2h, 1), "h2d_gbs": round(h2d, 1)}), flush=True)
    time.sleep(2)
