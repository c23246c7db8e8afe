"""Per-workgroup phase timeline of the whole-codeword GF(2^16) encoder (diagnostic library built with
-DCDA_RS16_TRACE=1, CDA_LIB=ab/libcda_r16tr.so): one k=512 row pass and one column pass, s_memrealtime (100 MHz) by
wave 0 when the codeword is in registers (top part done), after the last LDS exchange, after the transforms and
after the store phase, for the first 8 codewords of each persistent workgroup.  Prints phase medians in us."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
G = torch.cuda.get_device_properties(0).multi_processor_count
trace = torch.zeros(G * 32, dtype=torch.int64, device=dev)
os.environ["CDA_RS16_TRACE_PTR"] = str(trace.data_ptr())
import cda  # noqa: E402

ctx = cda.Context(0)
k, S = 512, 512
w = 2 * k
E = torch.randint(0, 256, (w, w, S), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev)
base, pitch = E.data_ptr(), w * S
passes = {"rows": lambda: ctx.rs_encode_device(k, S, k, base, pitch, S, base + k * S, pitch, S, s.cuda_stream),
          "cols": lambda: ctx.rs_encode_device(k, S, w, base, S, pitch, base + k * pitch, S, pitch, s.cuda_stream)}
out = {}
for name, fn in passes.items():
    for _ in range(3):
        trace.zero_()
        fn()
        s.synchronize()
    ph = trace.cpu().numpy().reshape(G, 8, 4).astype(np.float64)
    valid = ph[:, :, 0] > 0
    t0 = ph[ph > 0].min()
    us = (ph - t0) / 100.0
    d01 = (us[:, :, 1] - us[:, :, 0])[valid]
    d12 = (us[:, :, 2] - us[:, :, 1])[valid]
    d23 = (us[:, :, 3] - us[:, :, 2])[valid]
    top = (us[:, 1:, 0] - us[:, :-1, 3])[valid[:, 1:]]
    end = np.where(valid, us[:, :, 3], 0).max(1)
    med = lambda a: round(float(np.median(a)), 2) if a.size else None  # noqa: E731
    out[name] = {"codewords_per_wg": int(valid.sum(1).max()),
                 "first_in_registers_us": med(us[:, 0, 0]),
                 "median_us": {"top_to_last_exchange": med(d01), "fft_tail": med(d12), "store_phase": med(d23),
                               "next_top_part": med(top)},
                 "wg_end_us": [round(float(np.percentile(end, q)), 1) for q in (0, 50, 100)],
                 "example_wg0": [[round(float(x), 1) for x in us[0, i]] for i in range(8) if valid[0, i]]}
print(json.dumps(out), flush=True)
ctx.close()
