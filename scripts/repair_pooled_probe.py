"""cda_repair in place on one page-locked buffer (go/cda Repair's pooled slab), config C4 (k=128, random 50 % and
Q0-only): per-call times; with the test-hooks library and CDA_REPAIR_TRACE=1 each call's host phases go to stderr.
python scripts/repair_pooled_probe.py [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cda  # noqa: E402
import oracle_lib as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
k, w = 128, 256
ctx = cda.Context(0)
ods = O.gen_ods(k, 0xC0FFEE)
rc, eds, rr, cr, _ = O.extend_commit(ods)
rng = np.random.default_rng(5)
pooled = np.empty_like(eds)
ctx.host_register(pooled)
out = {}
try:
    for case in ("random", "q0_only"):
        ts = []
        for i in range(reps + 2):
            if case == "random":
                present = (rng.random(w * w) < 0.5).astype(np.uint8)
            else:
                present = np.zeros((w, w), np.uint8)
                present[:k, :k] = 1
                present = present.reshape(-1)
            np.copyto(pooled, np.where(present[:, None] == 1, eds, 0).astype(np.uint8))
            t0 = time.perf_counter()
            ctx.repair(pooled, present.copy(), rr, cr, inplace=True)
            t = (time.perf_counter() - t0) * 1e3
            assert np.array_equal(pooled, eds)
            if i >= 2:
                ts.append(t)
        out[case] = {"min_ms": round(min(ts), 3), "median_ms": round(float(np.median(ts)), 3)}
finally:
    ctx.host_unregister(pooled)
print(json.dumps(out))
