"""Do an H2D and a D2H on two streams overlap (PCIe full duplex through the DMA engines), and how fast is a strided
2-D D2H (the consensus path's Q1 bands)?  Pinned host buffers (torch), one JSON line."""
import json
import time

import torch

torch.cuda.init()
dev = torch.device("cuda", 0)
MiB = 1 << 20
h_in = torch.empty(8 * MiB, dtype=torch.uint8).pin_memory()
h_out = torch.empty(24 * MiB, dtype=torch.uint8).pin_memory()
d_in = torch.empty(8 * MiB, dtype=torch.uint8, device=dev)
d_out = torch.empty(24 * MiB, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) * 1e3 / reps, 3)


def h2d():
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_out, non_blocking=True)


def both():
    h2d()
    d2h()


def d2h_2d():  # Q1 of 128 rows: 64 KiB of every 128 KiB row
    with torch.cuda.stream(s2):
        h_out.view(128, -1)[:, :64 * 1024].copy_(d_out.view(128, -1)[:, 64 * 1024:128 * 1024], non_blocking=True)


def d2h_2d_src():  # strided device source -> contiguous host
    with torch.cuda.stream(s2):
        h_out[:8 * MiB].view(128, -1).copy_(d_out.view(128, -1)[:, 64 * 1024:128 * 1024], non_blocking=True)


def d2h_2d_dst():  # contiguous device source -> strided host
    with torch.cuda.stream(s2):
        h_out.view(128, -1)[:, 64 * 1024:128 * 1024].copy_(d_out[:8 * MiB].view(128, -1), non_blocking=True)


d_stage = torch.empty(8 * MiB, dtype=torch.uint8, device=dev)


def d2d_then_d2h():  # on-device gather into a contiguous stage, then one contiguous D2H
    with torch.cuda.stream(s2):
        d_stage.view(128, -1).copy_(d_out.view(128, -1)[:, 64 * 1024:128 * 1024], non_blocking=True)
        h_out[:8 * MiB].copy_(d_stage, non_blocking=True)


def d2h_8mib():
    with torch.cuda.stream(s2):
        h_out[:8 * MiB].copy_(d_out[:8 * MiB], non_blocking=True)


out = {"h2d_8mib_ms": timed(h2d), "d2h_24mib_ms": timed(d2h), "both_concurrent_ms": timed(both),
       "d2h_2d_8mib_ms": timed(d2h_2d), "d2h_8mib_ms": timed(d2h_8mib), "d2h_2d_src_strided_ms": timed(d2h_2d_src),
       "d2h_2d_dst_strided_ms": timed(d2h_2d_dst), "d2d_gather_then_d2h_ms": timed(d2d_then_d2h)}
out["overlap"] = "yes" if out["both_concurrent_ms"] < 0.8 * (out["h2d_8mib_ms"] + out["d2h_24mib_ms"]) else "no"
print(json.dumps(out), flush=True)
