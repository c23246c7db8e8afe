"""H2D from the Q0 rows of a page-locked EDS buffer: is a 2-D copy whose HOST side is strided (64 KiB rows at a
128 KiB pitch, k = 128) as fast as a contiguous one?  hipMemcpy2DAsync / hipMemcpyAsync through ctypes on buffers
from hipHostMalloc and from hipHostRegister (the Go pools' slabs), and a pageable contiguous copy for reference.
One JSON line, ms per 8 MiB (whole square) and per 2 MiB band."""
import ctypes
import json
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
for f in ("hipMalloc", "hipHostMalloc", "hipHostRegister", "hipStreamCreate", "hipStreamSynchronize",
          "hipMemcpyAsync", "hipMemcpy2DAsync", "hipSetDevice", "hipDeviceSynchronize"):
    getattr(hip, f).restype = ctypes.c_int
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
H2D = 1


def ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: HIP error {rc}")


ok(hip.hipSetDevice(0), "hipSetDevice")
k, S = 128, 512
row, erow = k * S, 2 * k * S
ods_b, eds_b = k * row, 2 * k * erow
d = ctypes.c_void_p()
ok(hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(ods_b)), "hipMalloc")
st = ctypes.c_void_p()
ok(hip.hipStreamCreate(ctypes.byref(st)), "hipStreamCreate")
hm = ctypes.c_void_p()
ok(hip.hipHostMalloc(ctypes.byref(hm), ctypes.c_size_t(eds_b), 0), "hipHostMalloc")
reg = np.ones(eds_b + 4096, np.uint8)
reg_p = (reg.ctypes.data + 4095) & ~4095
ok(hip.hipHostRegister(ctypes.c_void_p(reg_p), ctypes.c_size_t(eds_b), 0), "hipHostRegister")
pageable = np.ones(ods_b, np.uint8)
ctypes.memset(hm, 1, eds_b)


def timed(fn, reps=30):
    fn()
    ok(hip.hipStreamSynchronize(st), "sync")
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ok(hip.hipStreamSynchronize(st), "sync")
        ts.append((time.perf_counter() - t) * 1e3)
    return round(float(np.median(ts)), 4)


def contig(src, n):
    return lambda: ok(hip.hipMemcpyAsync(d, ctypes.c_void_p(src), n, H2D, st), "memcpy")


def strided(src, rows):
    return lambda: ok(hip.hipMemcpy2DAsync(d, row, ctypes.c_void_p(src), erow, row, rows, H2D, st), "memcpy2d")


def banded(src, two_d):
    def run():
        for b in range(4):
            if two_d:
                ok(hip.hipMemcpy2DAsync(ctypes.c_void_p(d.value + b * 32 * row), row, ctypes.c_void_p(src + b * 32 * erow),
                                        erow, row, 32, H2D, st), "memcpy2d")
            else:
                ok(hip.hipMemcpyAsync(ctypes.c_void_p(d.value + b * 32 * row), ctypes.c_void_p(src + b * 32 * row),
                                      32 * row, H2D, st), "memcpy")
    return run


out = {
    "hostmalloc_contig_8mib": timed(contig(hm.value, ods_b)),
    "hostmalloc_2d_q0_8mib": timed(strided(hm.value, k)),
    "registered_contig_8mib": timed(contig(reg_p, ods_b)),
    "registered_2d_q0_8mib": timed(strided(reg_p, k)),
    "registered_2d_q0_4bands": timed(banded(reg_p, True)),
    "registered_contig_4bands": timed(banded(reg_p, False)),
    "pageable_contig_8mib": timed(contig(pageable.ctypes.data, ods_b)),
    "pageable_contig_4bands": timed(banded(pageable.ctypes.data, False)),
}
print(json.dumps(out), flush=True)
