"""GF(2^16) encoder alone at k=512 (config C5's RS passes): rows (Q0 -> Q0 copy + Q1) and columns (top half ->
bottom half) of one square through cda_rs_encode_device, timed with HIP events on the launch stream.
CDA_RS16=lds selects the LDS encoder."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import cda  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ctx = cda.Context(0)
k, S = 512, 512
w = 2 * k
E = torch.randint(0, 256, (w, w, S), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev)
base, pitch = E.data_ptr(), w * S


def rows():
    ctx.rs_encode_device(k, S, k, base, pitch, S, base + k * S, pitch, S, s.cuda_stream)


def cols():
    ctx.rs_encode_device(k, S, w, base, S, pitch, base + k * pitch, S, pitch, s.cuda_stream)


out = {}
for name, fn, nbytes in (("rows", rows, 2 * k * k * S), ("cols", cols, 2 * w * k * S)):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    ms = a.elapsed_time(b) / reps
    out[name] = {"ms_per_square": round(ms, 4), "gbs": round(nbytes / ms / 1e6, 1)}
out["encoder"] = os.environ.get("CDA_RS16", "reg")
print(json.dumps(out), flush=True)
ctx.close()
