"""Pageable vs pinned host<->device copy rate by chunk size (what cda_repair's EDS copies can reach)."""
import json
import time

import numpy as np
import torch

N = 32 << 20
a = np.random.default_rng(0).integers(0, 256, N, dtype=np.uint8)
b = np.empty_like(a)
d = torch.empty(N, dtype=torch.uint8, device="cuda")
ta, tb = torch.from_numpy(a), torch.from_numpy(b)
pa = torch.empty(N, dtype=torch.uint8).pin_memory()
pa.copy_(ta)
out = {}
for name, src, dst in (("pageable", ta, tb), ("pinned", pa, pa)):
    for chunk in (N, 8 << 20, 4 << 20, 1 << 20):
        for direction in ("h2d", "d2h"):
            best = 1e9
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for o in range(0, N, chunk):
                    if direction == "h2d":
                        d[o:o + chunk].copy_(src[o:o + chunk], non_blocking=True)
                    else:
                        dst[o:o + chunk].copy_(d[o:o + chunk], non_blocking=True)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            out[f"{name}_{direction}_{chunk >> 20}MiB"] = round(N / best / 1e9, 1)
# fresh host arrays per copy (as a caller handing over a newly filled square)
for direction in ("h2d", "d2h"):
    best = 1e9
    for _ in range(5):
        fresh = torch.from_numpy(a.copy())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if direction == "h2d":
            d.copy_(fresh, non_blocking=True)
        else:
            fresh.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    out[f"pageable_fresh_{direction}_32MiB"] = round(N / best / 1e9, 1)
print(json.dumps(out, indent=1))

# raw HIP: hipMemcpyAsync on a non-blocking stream vs the null stream, fresh pageable source (cda_repair's copy)
import ctypes  # noqa: E402
import os  # noqa: E402

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
st = ctypes.c_void_p()
assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
dp = ctypes.c_void_p(d.data_ptr())
raw = {}
for sname, sv in (("nonblocking", st), ("null", ctypes.c_void_p(0))):
    for direction, kind in (("h2d", 1), ("d2h", 2)):
        for sync in ("async", "sync"):
            best = 1e9
            for _ in range(5):
                h = a.copy()
                hp = ctypes.c_void_p(h.ctypes.data)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                src, dst = (hp, dp) if kind == 1 else (dp, hp)
                if sync == "async":
                    rc = hip.hipMemcpyAsync(dst, src, ctypes.c_size_t(N), kind, sv)
                else:
                    rc = hip.hipMemcpy(dst, src, ctypes.c_size_t(N), kind)
                assert rc == 0 and hip.hipStreamSynchronize(sv) == 0
                best = min(best, time.perf_counter() - t0)
            raw[f"{sname}_{direction}_{sync}"] = round(N / best / 1e9, 1)
print(json.dumps(raw, indent=1))
