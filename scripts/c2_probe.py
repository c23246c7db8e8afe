"""Config C2 probe: one k=128 block, device-resident latency and per-kernel split (bench.single_block_measure),
plus the GPU-side span of one call (HIP events on the launch stream) against the host wall time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import torch  # noqa: E402  (first: libcda then resolves HIP through torch's runtime)
import bench  # noqa: E402
import cda  # noqa: E402

dev = torch.device("cuda", 0)
ctx = cda.Context(0)
r = bench.single_block_measure(ctx, dev)
k, w = 128, 256
ods = torch.from_numpy(bench.gen_ods(k, 0xC0FFEE)).to(dev)
eds = torch.empty((1, w * w, 512), dtype=torch.uint8, device=dev)
roots = torch.empty((1, 2 * w, 96), dtype=torch.uint8, device=dev)
dah = torch.empty((1, 32), dtype=torch.uint8, device=dev)
st = torch.empty((1,), dtype=torch.int64, device=dev)
s = torch.cuda.Stream(dev)
gpu, host = [], []
for i in range(60):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        a.record(s)
        t0 = time.perf_counter()
        ctx.extend_commit_device(k, 1, ods.data_ptr(), eds.data_ptr(), roots.data_ptr(), dah.data_ptr(),
                                 st.data_ptr(), s.cuda_stream)
        b.record(s)
    s.synchronize()
    host.append(time.perf_counter() - t0)
    if i >= 10:
        gpu.append(a.elapsed_time(b))
r["gpu_span_ms_min"] = round(min(gpu), 4)
r["gpu_span_ms_median"] = round(sorted(gpu)[len(gpu) // 2], 4)
r["host_ms_min_created_stream"] = round(min(host[10:]) * 1e3, 4)
r["graph"] = os.environ.get("CDA_GRAPH", "1")
print(json.dumps(r))
