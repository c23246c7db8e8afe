"""The consensus-path call as go/cda.ExtendSharesOn makes it (go/cda/extend.go:42-48): one k=128 block per
cda_extend_commit call, the shares freshly copied into a new flat buffer (outside the timed call, as Go's flatten
runs before the cgo call) and a NEW, untouched 32 MiB EDS buffer per call (np.empty: fresh mmap'd pages, as a large
Go make()).  Reports min / median per form, plus host first-touch copy rates into fresh pages by thread count and
the box's transparent-huge-page setting -- what bounds a fresh-buffer D2H."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import bench  # noqa: E402
import cda  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = cda.Context(0)
k, w = 128, 256
ods = bench.gen_ods(k, 0xC0FFEE).reshape(k * k, 512)
eds_ref, rr_ref, cr_ref, dah_ref = ctx.extend_commit(ods)


def series(want_eds, fresh_out):
    """fresh_out: a NEW never-touched output buffer per call (np.empty, allocated before the timed call and kept alive
    until the series ends -- freeing a 32 MiB buffer unmaps it, which a Go caller does not pay inside the call)."""
    out = []
    keep = np.ones((1, w * w, 512), np.uint8)
    bufs = [np.empty((1, w * w, 512), np.uint8) for _ in range(reps + 2)] if (fresh_out and want_eds) else None
    for i in range(reps + 2):
        src = ods.copy()[None]
        dst = (bufs[i] if fresh_out else keep) if want_eds else None
        t0 = time.perf_counter()
        eds, rr, cr, dah = ctx.extend_commit_batch(src, want_eds=want_eds, eds_out=dst)
        el = (time.perf_counter() - t0) * 1e3
        if bytes(dah[0]) != dah_ref:
            raise RuntimeError("DAH mismatch")
        if want_eds and i == reps + 1 and not np.array_equal(dst.reshape(eds_ref.shape), eds_ref):
            raise RuntimeError("EDS mismatch")
        if i >= 2:
            out.append(el)
    del bufs
    return {"min": round(min(out), 3), "median": round(float(np.median(out)), 3), "max": round(max(out), 3)}


res = {"reps": reps, **{v: os.environ[v] for v in ("CDA_CONSENSUS", "CDA_CONS_IN", "CDA_CONS_OUT") if v in os.environ}}
res["fresh_with_eds"] = series(True, True)
res["fresh_roots_only"] = series(False, True)
res["reused_with_eds"] = series(True, False)
res["reused_roots_only"] = series(False, False)


def pinned_series():
    """A caller that keeps pinned buffers (cda_host_alloc) for the shares and the EDS: both DMAs direct."""
    pb_ods, pb_eds = ctx.pinned((1, k * k, 512)), ctx.pinned((1, w * w, 512))
    pin_ods, pin_eds = pb_ods.array, pb_eds.array
    out = []
    for i in range(reps + 2):
        pin_ods[0] = ods
        t0 = time.perf_counter()
        _, _, _, dah = ctx.extend_commit_batch(pin_ods, eds_out=pin_eds)
        el = (time.perf_counter() - t0) * 1e3
        if bytes(dah[0]) != dah_ref:
            raise RuntimeError("DAH mismatch")
        if i >= 2:
            out.append(el)
    if not np.array_equal(pin_eds.reshape(eds_ref.shape), eds_ref):
        raise RuntimeError("EDS mismatch")
    pb_ods.free()
    pb_eds.free()
    return {"min": round(min(out), 3), "median": round(float(np.median(out)), 3), "max": round(max(out), 3)}


res["pinned_with_eds"] = pinned_series()
try:  # where the process runs relative to the GPU (host placement moves the D2H rate between boxes)
    pr = torch.cuda.get_device_properties(0)
    bdf = "%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id, pr.pci_device_id)
    res["gpu_numa_node"] = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
except Exception as e:  # noqa: BLE001
    res["gpu_numa_node"] = repr(e)[:80]
cpus = sorted(os.sched_getaffinity(0))
res["cpus"] = f"{len(cpus)}: {cpus[0]}-{cpus[-1]}" if cpus else "none"
print(json.dumps(res), flush=True)
if os.environ.get("CDA_CONSENSUS", "1") != "0" and os.environ.get("CDA_PROBE_SWEEP"):  # copy-pool size sweep (a context reads CDA_COPY_THREADS at its first call)
    sweep = {}
    for T in (3, 7, 11, 15):
        os.environ["CDA_COPY_THREADS"] = str(T)
        ctx.close()
        ctx = cda.Context(0)
        sweep[str(T)] = series(True, True)
    os.environ.pop("CDA_COPY_THREADS")
    print(json.dumps({"copy_threads_sweep_fresh_with_eds": sweep}), flush=True)

if not os.environ.get("CDA_PROBE_HOST"):
    sys.exit(0)
# host side: first-touch copies into fresh pages
N = 32 << 20
src = torch.empty(N, dtype=torch.uint8).pin_memory().numpy()
src[:] = 7
host = {}
for T in (1, 2, 4, 8, 12, 16):
    times = []
    for _ in range(5):
        dst = np.empty(N, np.uint8)
        bounds = [(N * i // T, N * (i + 1) // T) for i in range(T)]
        t0 = time.perf_counter()
        ths = [threading.Thread(target=lambda lo, hi: np.copyto(dst[lo:hi], src[lo:hi]), args=b) for b in bounds]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        times.append(time.perf_counter() - t0)
        del dst
    host[str(T)] = {"fresh_gbs_best": round(N / min(times) / 1e9, 1), "fresh_gbs_median": round(N / float(np.median(times)) / 1e9, 1)}
warm = np.empty(N, np.uint8)
warm.fill(1)
t0 = time.perf_counter()
np.copyto(warm, src)
host["1_warm_gbs"] = round(N / (time.perf_counter() - t0) / 1e9, 1)
thp = {}
for f in ("enabled", "defrag"):
    try:
        thp[f] = open(f"/sys/kernel/mm/transparent_hugepage/{f}").read().strip()
    except OSError:
        thp[f] = None
print(json.dumps({"host_first_touch_copy": host, "thp": thp, "affinity": len(os.sched_getaffinity(0))}), flush=True)
