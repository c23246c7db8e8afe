"""Phase timeline of trees_lds_kernel for ONE k=128 block (config C2), diagnostic library built with
-DCDA_TREES_TRACE=1 (CDA_LIB=ab/libcda_ttr.so): per workgroup s_memrealtime (100 MHz) and s_memtime (shader clock)
at kernel entry, after the leaf records are in LDS, after each of the 8 levels, after the roots' DAH leaf digests,
after the block counter, and (last workgroup) around the DAH fold.  Prints medians of each phase in us and the
effective shader clock of each phase (d memtime / d realtime x 100 MHz)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
k, w = 128, 256
NWG = w  # 2k trees... trees_lds: one workgroup per two trees -> 4k / 2 = 2w workgroups per block
NWG = 2 * w
trace = torch.zeros(NWG * 32 * 2, dtype=torch.int64, device=dev)
os.environ["CDA_TREES_TRACE_PTR"] = str(trace.data_ptr())
import bench  # noqa: E402
import cda  # noqa: E402

ctx = cda.Context(0)
ods = torch.from_numpy(bench.gen_ods(k, 0xC0FFEE)).to(dev)
eds = torch.empty((1, w * w, 512), dtype=torch.uint8, device=dev)
roots = torch.empty((1, 2 * w, 96), dtype=torch.uint8, device=dev)
dah = torch.empty((1, 32), dtype=torch.uint8, device=dev)
st = torch.empty((1,), dtype=torch.int64, device=dev)
s = torch.cuda.current_stream(dev)
out = []
for rep in range(12):
    trace.zero_()
    ctx.extend_commit_device(k, 1, ods.data_ptr(), eds.data_ptr(), roots.data_ptr(), dah.data_ptr(), st.data_ptr(),
                             s.cuda_stream)
    s.synchronize()
    if rep < 2:
        continue
    t = trace.cpu().numpy().reshape(NWG, 32, 2).astype(np.float64)
    rt, ck = t[:, :, 0], t[:, :, 1]
    ok = rt[:, 0] > 0
    t0 = rt[ok, 0].min()
    last = int(np.argmax(rt[:, 29]))
    med = lambda a: round(float(np.median(a)), 2)  # noqa: E731
    row = {"leaf_load_us": med((rt[ok, 1] - rt[ok, 0]) / 100)}
    prev = rt[ok, 1]
    lv = []
    for l in range(1, 9):
        a, b, c = rt[ok, 2 + 3 * (l - 1)], rt[ok, 3 + 3 * (l - 1)], rt[ok, 4 + 3 * (l - 1)]
        if l == 1:
            lv.append({"total": med((c - prev) / 100)})
        else:
            lv.append({"block0": med((a - prev) / 100), "barrier": med((b - a) / 100), "kw2": med((c - b) / 100),
                       "total": med((c - prev) / 100)})
        prev = c
    row["levels_us"] = lv
    row["digest_us"] = med((rt[ok, 26] - prev) / 100)
    row["counter_us"] = med((rt[ok, 27] - rt[ok, 26]) / 100)
    row["fold_us"] = float((rt[last, 29] - rt[last, 28]) / 100)
    row["total_us"] = float((rt[last, 29] - t0) / 100)
    out.append(row)
best = min(out, key=lambda r: r["total_us"])
worst = max(out, key=lambda r: r["total_us"])
print(json.dumps({"best": best, "worst": worst, "totals_us": [round(r["total_us"], 1) for r in out]}), flush=True)
ctx.close()
