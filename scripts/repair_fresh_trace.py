import os, sys, time
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "celestia-app_amd"))
import numpy as np, torch, bench, cda
ctx = cda.Context(0)
k, w = 128, 256
eds, rr, cr, _ = ctx.extend_commit(bench.gen_ods(k, 1).reshape(k * k, 512))
pres = (np.random.default_rng(7).random(w * w) < 0.5).astype(np.uint8)
dam = eds.copy(); dam[pres == 0] = 0
for i in range(10):
    b = np.empty_like(dam); np.copyto(b, dam); p = pres.copy()
    t0 = time.perf_counter(); ctx.repair(b, p, rr, cr, inplace=True); print("ms", round((time.perf_counter()-t0)*1e3, 2), file=sys.stderr)
