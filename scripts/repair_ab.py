"""C4 host-buffer repair, fresh and reused caller buffers, for A/B of library builds (CDA_LIB)."""
import json
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
eds, rr, cr, _ = ctx.extend_commit(bench.gen_ods(k, 1).reshape(k * k, 512))
out = {"lib": os.environ.get("CDA_LIB", "default")}
for name, frac in (("random", 0.5), ("q0", None)):
    if frac is None:
        q = np.zeros((w, w), np.uint8)
        q[:k, :k] = 1
        pres = q.reshape(-1)
    else:
        pres = (np.random.default_rng(7).random(w * w) < frac).astype(np.uint8)
    dam = eds.copy()
    dam[pres == 0] = 0
    keep = dam.copy()
    for mode in ("reused", "fresh"):
        ts = []
        for i in range(9):
            if mode == "fresh":
                b = np.empty_like(dam)
            else:
                b = keep
            np.copyto(b, dam)
            p = pres.copy()
            t0 = time.perf_counter()
            ctx.repair(b, p, rr, cr, inplace=True)
            ts.append((time.perf_counter() - t0) * 1e3)
        out[f"{name}_{mode}"] = [round(min(ts[1:]), 2), round(float(np.median(ts[1:])), 2)]
print(json.dumps(out))
