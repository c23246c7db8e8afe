import torch, time
d = torch.device("cuda", 0)
for n in (1 << 30, 4 << 30):
    a = torch.empty(n, dtype=torch.uint8, device=d).fill_(1)
    b = torch.empty_like(a)
    for _ in range(3): b.copy_(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): b.copy_(a)
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"copy {n>>20} MiB: {2*n/ms/1e6:.0f} GB/s (read+write)")
    s.record()
    for _ in range(10): b.fill_(3)
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"fill {n>>20} MiB: {n/ms/1e6:.0f} GB/s")
    s.record()
    for _ in range(10): x = a.sum(dtype=torch.int64)
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"read(sum) {n>>20} MiB: {n/ms/1e6:.0f} GB/s")
