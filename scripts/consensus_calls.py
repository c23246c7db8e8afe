"""N one-block k=128 calls through page-locked buffers (cda_host_alloc shares and EDS), after a D2H warm-up: the
command a rocprofv3 kernel + memory-copy trace of the consensus path runs (scripts/gpu_r05.sh constrace_prof)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
import cda  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
mode = sys.argv[2] if len(sys.argv) > 2 else "pinned"  # pinned: cda_host_alloc in/out; inplace: cda_extend_commit_eds
ctx = cda.Context(0)
k = 128
pin_in, pin_out = ctx.pinned((1, k * k, 512)), ctx.pinned((1, 4 * k * k, 512))
ods = bench.gen_ods(k, 0xC0FFEE)
pin_in.array[0] = ods
pin_out.array[0].reshape(2 * k, 2 * k, 512)[:k, :k] = ods.reshape(k, k, 512)
if mode == "inplace":
    def call():
        ctx.extend_commit_eds(pin_out.array[0])
else:
    def call():
        ctx.extend_commit_batch(pin_in.array, eds_out=pin_out.array)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 3:
    call()
ts = []
for _ in range(n):
    a = time.perf_counter()
    call()
    ts.append((time.perf_counter() - a) * 1e3)
ts.sort()
print("consensus_calls median_ms", round(ts[len(ts) // 2], 3), flush=True)
