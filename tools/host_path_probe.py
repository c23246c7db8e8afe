"""Probe: PCIe-inclusive cda_extend_commit_batch with different host output buffers (fresh, reused, pinned)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import cda  # noqa: E402
from bench import gen_ods  # noqa: E402

k, nb = 128, 16
ctx = cda.Context(0)
ods = np.stack([gen_ods(k, 0xC0FFEE + (b % 4)) for b in range(nb)])


def timed(fn, reps=3):
    fn()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return round(nb / best, 1), round(best * 1e3, 2)


print("fresh np.empty:", timed(lambda: ctx.extend_commit_batch(ods, want_eds=True)))
reuse = np.ones((nb, 4 * k * k, 512), np.uint8)
print("reused touched:", timed(lambda: ctx.extend_commit_batch(ods, eds_out=reuse)))
pinned = torch.empty((nb, 4 * k * k, 512), dtype=torch.uint8, pin_memory=True).numpy()
pinned[:] = 1
ods_p = torch.from_numpy(ods).pin_memory().numpy()
print("pinned out:", timed(lambda: ctx.extend_commit_batch(ods, eds_out=pinned)))
print("pinned in+out:", timed(lambda: ctx.extend_commit_batch(ods_p, eds_out=pinned)))
print("roots only, pinned in:", timed(lambda: ctx.extend_commit_batch(ods_p, want_eds=False)))
