"""Per-workgroup phase timeline of the half-slice GF(2^16) encoder (diagnostic library built with
-DCDA_RS16_H2_TRACE=1, CDA_LIB=ab/libcda_h2tr*.so): one k=512 column pass, s_memrealtime (100 MHz) at the loop top,
after the state is built (loads consumed), after the transforms and after the stores are issued, for the first 8
items of every workgroup; plus where each workgroup ran (XCC, SE, CU).  Prints phase medians and how the two
workgroups of each CU overlap."""
import collections
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
G = 2 * torch.cuda.get_device_properties(0).multi_processor_count
trace = torch.zeros(G * 33, dtype=torch.int64, device=dev)
os.environ["CDA_H2_TRACE_PTR"] = str(trace.data_ptr())
import cda  # noqa: E402

ctx = cda.Context(0)
k, S = 512, 512
w = 2 * k
E = torch.randint(0, 256, (w, w, S), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev)
base, pitch = E.data_ptr(), w * S
for _ in range(3):
    trace.zero_()
    ctx.rs_encode_device(k, S, w, base, S, pitch, base + k * pitch, S, pitch, s.cuda_stream)
    s.synchronize()
t = trace.cpu().numpy()
ph = t[:G * 32].reshape(G, 8, 4).astype(np.float64)
hw = t[G * 32:]
t0 = ph[ph > 0].min()
us = (ph - t0) / 100.0  # 100 MHz -> us
valid = ph[:, :, 0] > 0
items = valid.sum(1)
load = (us[:, :, 1] - us[:, :, 0])[valid]
comp = (us[:, :, 2] - us[:, :, 1])[valid]
stor = (us[:, :, 3] - us[:, :, 2])[valid]
nxt = (us[:, 1:, 0] - us[:, :-1, 3])[valid[:, 1:]]
end = np.where(valid, us[:, :, 3], 0).max(1)
out = {"grid": G, "items_per_wg": dict(collections.Counter(items.tolist())),
       "median_us": {"load": float(np.median(load)), "compute": float(np.median(comp)),
                     "store_issue": float(np.median(stor)), "to_next_top": float(np.median(nxt)) if nxt.size else None},
       "p10_p90_us": {"load": [float(np.percentile(load, 10)), float(np.percentile(load, 90))],
                      "compute": [float(np.percentile(comp, 10)), float(np.percentile(comp, 90))]},
       "first_top_us": [float(np.percentile(us[:, 0, 0], q)) for q in (0, 50, 100)],
       "wg_end_us": [float(np.percentile(end, q)) for q in (0, 50, 100)]}
# pair the workgroups by CU: (xcc, se, sh, cu) from HW_ID
cu_of = {}
for b in range(G):
    h = int(hw[b]) & 0xFFFFFFFF
    xcc = int(hw[b]) >> 32
    key = (xcc & 0xF, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 0xF)
    cu_of.setdefault(key, []).append(b)
sizes = collections.Counter(len(v) for v in cu_of.values())
out["wgs_per_cu"] = dict(sizes)
# overlap: for CUs with two workgroups, the fraction of A's compute time during which B also computes
fr = []
for key, bs in cu_of.items():
    if len(bs) != 2:
        continue
    a, b = bs
    ca = [(us[a, i, 1], us[a, i, 2]) for i in range(8) if valid[a, i]]
    cb = [(us[b, i, 1], us[b, i, 2]) for i in range(8) if valid[b, i]]
    tot = sum(e - s_ for s_, e in ca)
    ov = sum(max(0.0, min(e1, e2) - max(s1, s2)) for s1, e1 in ca for s2, e2 in cb)
    fr.append(ov / tot if tot else 0)
out["compute_overlap_of_cu_pairs"] = [float(np.percentile(fr, q)) for q in (10, 50, 90)] if fr else None
ex = cu_of[sorted(cu_of)[0]]
out["example_cu"] = {str(b): [[round(float(x), 1) for x in us[b, i]] for i in range(8) if valid[b, i]] for b in ex}
print(json.dumps(out), flush=True)
ctx.close()
