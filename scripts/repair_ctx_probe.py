"""C4 host-buffer repair timed after different kinds of prior work in the same process (what the bench runs
before it), to separate process-state effects from the repair itself."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import cda  # noqa: E402

ctx = cda.Context(0)
dev = torch.device("cuda", 0)


def rep(tag):
    r = bench.repair_measure(ctx)
    print(tag, r["random"]["ms"], r["q0_only"]["ms"], r["random"]["device_resident_ms"], flush=True)


rep("fresh")
big = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
big.fill_(1)
torch.cuda.synchronize()
rep("after_4GiB_torch_alloc")
k = 128
w = 2 * k
ods = torch.from_numpy(bench.gen_ods(k, 1)).to(dev)
eds = torch.empty((1, w * w, 512), dtype=torch.uint8, device=dev)
roots = torch.empty((1, 2 * w, 96), dtype=torch.uint8, device=dev)
dah = torch.empty((1, 32), dtype=torch.uint8, device=dev)
st = torch.empty((1,), dtype=torch.int64, device=dev)
s = torch.cuda.current_stream(dev)
ctx.extend_commit_device(k, 1, ods.data_ptr(), eds.data_ptr(), roots.data_ptr(), dah.data_ptr(), st.data_ptr(),
                         s.cuda_stream)
torch.cuda.synchronize()
rep("after_extend_commit_device")
ctx.extend_commit(bench.gen_ods(k, 2).reshape(k * k, 512))
rep("after_extend_commit")
