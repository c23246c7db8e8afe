"""Config C2 latency (one k=128 block, device-resident) and small batches B = 1, 2, 4 through
cda_extend_commit_device: prints best-of-N ms per call and the per-kernel split.  Run once with the default and once
with CDA_TREES_LDS=0 (the batched level kernels + dah_kernel) to compare the two tree paths."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import cda  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ctx = cda.Context(0)
out = {"mode": os.environ.get("CDA_TREES_LDS", "default"), "c2": bench.single_block_measure(ctx, dev)}
for k in (128, 256):
    w = 2 * k
    for B in (1, 2, 4):
        ods = torch.from_numpy(np.stack([bench.gen_ods(k, 0xC0FFEE + b) for b in range(B)])).to(dev)
        eds = torch.empty((B, w * w, 512), dtype=torch.uint8, device=dev)
        roots = torch.empty((B, 2 * w, 96), dtype=torch.uint8, device=dev)
        dah = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        st = torch.empty((B,), dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream(dev)
        best = 1e9
        for it in range(30):
            t0 = time.perf_counter()
            ctx.extend_commit_device(k, B, ods.data_ptr(), eds.data_ptr(), roots.data_ptr(), dah.data_ptr(),
                                     st.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize(dev)
            best = min(best, time.perf_counter() - t0)
        want = [ctx.extend_commit(bench.gen_ods(k, 0xC0FFEE + b))[3] for b in range(B)]
        ok = all(bytes(dah[b].cpu().numpy()) == want[b] for b in range(B))
        out[f"k{k}_B{B}"] = {"ms": round(best * 1e3, 3), "dah_ok": ok}
print(json.dumps(out), flush=True)
