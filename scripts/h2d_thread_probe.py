"""Pageable 32 MiB H2D: torch copy, raw hipMemcpyAsync on a non-blocking stream from the main thread and from
another OS thread, into a reused vs a fresh host buffer (what cda_repair's upload does)."""
import ctypes
import os
import threading
import time

import numpy as np
import torch

N = 32 << 20
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
st = ctypes.c_void_p()
assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
d = torch.empty(N, dtype=torch.uint8, device="cuda")
dp = ctypes.c_void_p(d.data_ptr())
a = np.random.default_rng(0).integers(0, 256, N, dtype=np.uint8)


def copy(h):
    assert hip.hipMemcpyAsync(dp, ctypes.c_void_p(h.ctypes.data), ctypes.c_size_t(N), 1, st) == 0
    assert hip.hipStreamSynchronize(st) == 0


def timed(fn, reps=8):
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        out.append((time.perf_counter() - t0) * 1e3)
    return [round(x, 2) for x in out]


reused = a.copy()
print("main reused ", timed(lambda: copy(reused)))
print("main fresh  ", timed(lambda: copy(a.copy())))


def in_thread(h):
    t = threading.Thread(target=copy, args=(h,))
    t.start()
    t.join()


print("thread reused", timed(lambda: in_thread(reused)))
print("thread fresh ", timed(lambda: in_thread(a.copy())))
print("torch reused ", timed(lambda: (d.copy_(torch.from_numpy(reused)), torch.cuda.synchronize())))
