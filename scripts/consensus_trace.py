"""Phase trace of the one-block consensus path with page-locked buffers (csrc/consensus.cpp, CDA_CONS_TRACE=1: host
timestamps of each phase on stderr).  Warms the D2H path up first (pinned one-block calls until 10 calls in a row are
within 10 % of their median, at most 12 s), then 30 traced calls per output shape; prints one JSON line with the
median of every phase (us from the call's start) plus the warm-up length and a plain 24 MiB D2H for reference."""
import json
import os
import re
import statistics as st
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.environ.get("CDA_CONS_TRACE") is None:  # re-run self with the trace on, stderr captured (no GPU touched yet)
    env = dict(os.environ, CDA_CONS_TRACE="1")
    p = subprocess.run([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env, capture_output=True,
                       text=True, timeout=600)
    rows = {}
    cur = None
    for line in p.stderr.splitlines():
        if line.startswith("== "):
            cur = line[3:].strip()
        elif line.startswith("cons_trace") and cur:
            rows.setdefault(cur, []).append({k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", line)})
    out = {}
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            out.update(json.loads(line))
    for shape, r in rows.items():
        r = r[-30:]
        out[shape + "_phases_us"] = {f: round(st.median(x[f] for x in r), 1) for f in r[0]}
    print(json.dumps(out), flush=True)
    sys.exit(p.returncode)

sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import cda  # noqa: E402

torch.cuda.init()
ctx = cda.Context(0)
k = 128
ods = bench.gen_ods(k, 0xC0FFEE)
pin_in, pin_out = ctx.pinned((1, k * k, 512)), ctx.pinned((1, 4 * k * k, 512))
pin_in.array[0] = ods
res, ts, t0 = {}, [], time.perf_counter()
sys.stderr.write("== warmup\n"); sys.stderr.flush()
while time.perf_counter() - t0 < 12:
    a = time.perf_counter()
    ctx.extend_commit_batch(pin_in.array, eds_out=pin_out.array)
    ts.append((time.perf_counter() - a) * 1e3)
    if len(ts) >= 10 and max(ts[-10:]) < 1.1 * st.median(ts[-10:]):
        break
res["warmup"] = {"s": round(time.perf_counter() - t0, 2), "calls": len(ts), "first_ms": round(ts[0], 3),
                 "last10_median_ms": round(st.median(ts[-10:]), 3)}
reg = np.empty((1, 4 * k * k, 512), np.uint8)
ctx.host_register(reg)
for name, src, out in (("pinned", pin_in.array, pin_out.array), ("registered_out", ods[None].copy(), reg),
                       ("roots_only", ods[None].copy(), None)):
    sys.stderr.write(f"== {name}\n")
    sys.stderr.flush()
    ms = []
    for i in range(30):
        a = time.perf_counter()
        ctx.extend_commit_batch(src, eds_out=out, want_eds=out is not None)
        ms.append((time.perf_counter() - a) * 1e3)
    res[name + "_ms_median"] = round(st.median(ms), 3)
ctx.host_unregister(reg)
d = torch.empty(24 << 20, dtype=torch.uint8, device="cuda")
h = torch.empty(24 << 20, dtype=torch.uint8).pin_memory()
for _ in range(3):
    h.copy_(d, non_blocking=True)
torch.cuda.synchronize()
a = time.perf_counter()
for _ in range(20):
    h.copy_(d, non_blocking=True)
torch.cuda.synchronize()
res["d2h_24mib_ms"] = round((time.perf_counter() - a) * 1e3 / 20, 3)
print(json.dumps(res), flush=True)
