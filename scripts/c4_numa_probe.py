"""C4 host-buffer repair spread vs host-thread placement: the NUMA nodes of the box, the GPU's local CPUs, then
15 repairs (fresh caller buffer each, random 50 %) with the process's threads on (a) the default affinity, (b) the
GPU-local node, (c) a remote node -- a new context per mode so its helper threads start under that mask.
CDA_REPAIR_TRACE=1 adds libcda's per-phase host times."""
import glob
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


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


nodes = {}
for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
    nodes[int(d.rsplit("node", 1)[1])] = cpulist(open(d + "/cpulist").read())
allowed = sorted(os.sched_getaffinity(0))
torch.cuda.init()
info = {"nodes": {n: [c[0], c[-1], len(c)] for n, c in nodes.items()}, "allowed": len(allowed)}
gpu_node = None
for p in glob.glob("/sys/class/drm/card*/device"):
    try:
        node = int(open(p + "/numa_node").read())
        local = open(p + "/local_cpulist").read().strip()
        info.setdefault("drm", []).append([os.path.realpath(p).rsplit("/", 1)[1], node, local])
    except OSError:
        continue
info["visible"] = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
print(json.dumps(info), flush=True)
props = torch.cuda.get_device_properties(0)
for bdf_s, node, _ in info.get("drm", []):  # "0000:f1:00.0": bus 0xf1 = props.pci_bus_id
    if int(bdf_s.split(":")[1], 16) == props.pci_bus_id:
        gpu_node = node
print(json.dumps({"gpu_bus": props.pci_bus_id, "gpu_node": gpu_node}), flush=True)

k, w = 128, 256
ods = bench.gen_ods(k, 0xC0FFEE).reshape(k * k, 512)
c0 = cda.Context(0)
eds, rr, cr, _ = c0.extend_commit(ods)
c0.close()
rng = np.random.default_rng(7)


Q0 = np.zeros((w, w), np.uint8)
Q0[:k, :k] = 1


def run(mode, cpus, q0=False):
    if cpus:
        os.sched_setaffinity(0, cpus)
    ctx = cda.Context(0)
    ms = []
    for it in range(17):
        present = Q0.reshape(-1).copy() if q0 else (rng.random(w * w) < 0.5).astype(np.uint8)
        damaged = np.empty_like(eds)
        np.copyto(damaged, eds)
        damaged[present == 0] = 0
        t0 = time.perf_counter()
        ctx.repair(damaged, present, rr, cr, inplace=True)
        el = (time.perf_counter() - t0) * 1e3
        if it >= 2:
            ms.append(el)
    ctx.close()
    os.sched_setaffinity(0, allowed)
    print(json.dumps({"mode": mode + ("_q0" if q0 else ""), "ncpus": len(cpus) if cpus else len(allowed), "min": round(min(ms), 2),
                      "median": round(float(np.median(ms)), 2), "ms": [round(x, 2) for x in ms]}), flush=True)


run("default", None)
run("default", None, q0=True)
if gpu_node is not None and len(nodes) > 1:
    local = [c for c in nodes[gpu_node] if c in set(allowed)]
    remote = [c for n, cs in nodes.items() if n != gpu_node for c in cs if c in set(allowed)]
    run("gpu_local_node", local)
    run("remote_node", remote)
    run("gpu_local_16", local[:16])
    run("default_again", None)
