"""Config C4 probe: where cda_repair's time goes (per-kernel HIP-event profile + wall time), k=128."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
import cda  # noqa: E402

ctx = cda.Context(0)
k, w = 128, 256
ods = bench.gen_ods(k, 0xC0FFEE)
eds, rr, cr, _ = ctx.extend_commit(ods)
out = {}
for name, frac, seed in (("random50", 0.5, 7), ("random60", 0.6, 8), ("q0_only", None, 0)):
    if frac is None:
        pres = np.zeros((w, w), np.uint8)
        pres[:k, :k] = 1
        pres = pres.reshape(-1)
    else:
        pres = (np.random.default_rng(seed).random(w * w) < frac).astype(np.uint8)
    damaged = eds.copy()
    damaged[pres == 0] = 0
    ctx.repair(damaged, pres, rr, cr)
    ctx.profile_reset()
    ctx.profile_enable(True)
    t0 = time.perf_counter()
    got, _ = ctx.repair(damaged, pres, rr, cr)
    d2, p2 = damaged.copy(), pres.copy()
    el = time.perf_counter() - t0
    ctx.profile_enable(False)
    prof = ctx.profile_read()
    assert np.array_equal(got, eds)
    ctx.profile_reset()
    t0 = time.perf_counter()
    ctx.repair(d2, p2, rr, cr, inplace=True)
    el2 = time.perf_counter() - t0
    assert np.array_equal(d2, eds)
    out[name] = {"ms_profiled": round(el * 1e3, 2), "ms": round(el2 * 1e3, 2),
                 "kernels": {n: [round(ms, 3), cnt] for n, (ms, cnt) in prof.items()}}
print(json.dumps(out, indent=1))
