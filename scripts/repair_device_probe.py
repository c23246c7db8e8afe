"""cda_repair_device alone (config C4, k=128, random 50 % and Q0-only), for a kernel trace of the device-resident
repair: python scripts/repair_device_probe.py [reps].  Prints per-call times; run under rocprofv3 --kernel-trace."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
import cda  # noqa: E402
import oracle_lib as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
k, w = 128, 256
ctx = cda.Context(0)
ods = O.gen_ods(k, 0xC0FFEE)
rc, eds, rr, cr, _ = O.extend_commit(ods)
rng = np.random.default_rng(3)
out = {}
for case in ("random", "q0_only"):
    ts = []
    for i in range(reps + 2):
        if case == "random":
            present = (rng.random(w * w) < 0.5).astype(np.uint8)
        else:
            present = np.zeros((w, w), np.uint8)
            present[:k, :k] = 1
            present = present.reshape(-1)
        damaged = np.where(present[:, None] == 1, eds, 0).astype(np.uint8)
        d_eds = torch.from_numpy(damaged).cuda()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc, _, _ = ctx.repair_device(k, d_eds.data_ptr(), present.copy(), rr, cr)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) * 1e3
        assert rc == 0 and np.array_equal(d_eds.cpu().numpy(), eds)
        if i >= 2:
            ts.append(t)
    out[case] = {"min_ms": round(min(ts), 3), "median_ms": round(float(np.median(ts)), 3)}
print(json.dumps(out))
