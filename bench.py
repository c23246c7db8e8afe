#!/usr/bin/env python3
"""bench.py — ODS -> EDS + 4k NMT roots + DAH throughput on MI355X.

Metric (BASELINE.json): "ODS\u2192EDS+DAH blocks/sec at k=128 (1/8 GPU); achieved HBM GB/s".
A step = one pass of the hot path (da.ExtendShares + NewDataAvailabilityHeader
restated: RS rows, RS columns, leaf hashing, NMT levels, DAH) over a batch of B
independent k=128 blocks per GPU, inputs already resident in HBM.  N GPUs shard
independent blocks (weak scaling, no collective on the data path); the only
collectives are the timing barrier and the max-over-ranks of the elapsed time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--k 128] [--batch B]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

# Algorithmic work per block, k = ODS width.
def block_bytes(k):  # read ODS + write EDS + 4k roots + DAH
    return 512 * k * k + 512 * 4 * k * k + 4 * k * 90 + 32


def block_compressions_ref(k):  # SHA-256 compressions the reference performs
    return 96 * k * k + 4 * k - 2


def block_compressions_engine(k):  # each EDS cell hashed once (row & col leaf data identical)
    w = 2 * k
    return 9 * w * w + 3 * (2 * w) * (w - 1) + 2 * (2 * w) + 2 * (2 * w - 1)


def kernel_step_bytes(name, k, B):
    """Algorithmic HBM bytes one bench step moves through kernel `name` (B blocks of width k).

    rows: read Q0, write the Q0 copy + Q1; cols: read the top half, write the
    bottom half; leaf_hash: read every EDS cell, write a 90-B leaf node;
    NMT levels: read 2 child nodes, write 1 (90 B each); dah: read 4k roots.
    """
    w, S, N = 2 * k, 512, 90
    if name.endswith("_rows"):
        return B * 3 * k * k * S
    if name.endswith("_cols"):
        return B * 2 * w * k * S
    if name == "leaf_hash":
        return B * w * w * (S + N)
    if name == "nmt_levels_1":  # levels 1-2 in one launch: read the leaves, write levels 1 and 2
        return B * 2 * w * ((w // 2) * 2 * N + (w // 2) * N + (w // 4) * N)
    if name == "nmt_levels":  # levels 3..log2(w): read level 2, write every later level
        n, tot = w // 4, 2 * w * (w // 4) * N
        while n > 1:
            tot += 2 * w * (n // 2) * N
            n //= 2
        return B * tot
    if name == "dah":
        return B * (2 * w * N + 32)
    return None


# What bounds each kernel: the SHA-256 kernels issue VALU work (their HBM traffic is a small fraction
# of 8 TB/s), the Reed-Solomon encoders stream HBM (read + write) with the GF arithmetic beside it.
KERNEL_KIND = {"leaf_hash": "valu", "nmt_levels_1": "valu", "nmt_levels": "valu", "dah": "latency",
               "rs_encode8_rows": "hbm", "rs_encode8_cols": "hbm", "rs_encode16_rows": "hbm", "rs_encode16_cols": "hbm"}
# SHA-256 compressions per launch of the hashing kernels (B blocks of width k): leaf = 9 per EDS cell, levels 1-2 =
# 3 per node of the first two levels of all 4k trees, levels 3.. = 3 per remaining inner node
def kernel_compressions(name, k, B):
    w = 2 * k
    if name == "leaf_hash":
        return 9 * B * w * w
    if name == "nmt_levels_1":
        return 3 * B * 2 * w * (w // 2 + w // 4)
    return None


SHA_UBENCH_GCOMP_S = 28.7  # register-only SHA-256 on MI355X (profiles/r02_sha_ubench.txt): the issue-bound ceiling
VALU_CLK = 2.4e9  # peak engine clock (MI355X_MICROARCH.md)


def hbm_ceilings(device):
    """Measured HBM ceilings of this box (tools/copy_bw.hip, hand-written dwordx4 streaming kernels over 1 GiB
    buffers): copy (read + write, the RS encoders' traffic shape), read-only, write-only, in GB/s of bytes moved."""
    import ctypes
    path = os.path.join(ROOT, "tools", "libcopybw.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.copybw_measure.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    out = (ctypes.c_double * 3)()
    cfg = (ctypes.c_int * 3)()
    if L.copybw_measure(device, 1 << 30, 10, out, cfg) != 0:
        return None
    names = ("copy", "read", "write")
    return {**{f"{n}_gbs": round(out[i], 1) for i, n in enumerate(names)},
            "best_config": {n: {"accesses_per_thread": cfg[i] // 10000, "workgroup": cfg[i] % 10000}
                            for i, n in enumerate(names)},
            "note": "tools/copy_bw.hip: 16 B per lane per access (global_load/store_dwordx4), 1 GiB buffers (4x the "
                    "Infinity Cache), best of U in {1,2,4,8} x workgroup {256,512,1024}; copy counts read + written "
                    "bytes"}


def isa_mix():
    """Static VALU mix of the kernels (scripts/isa_mix.sh -> profiles/r*_isa_mix.json, newest)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_isa_mix.json")))
    if not files:
        return {}, None
    mix = json.load(open(files[-1]))
    return mix, os.path.relpath(files[-1], ROOT)


def avg_cycles_per_valu(mix, kernel_symbol_part):
    for name, v in mix.items():
        if kernel_symbol_part in name:
            return v["avg_cycles_per_valu"]
    return None


def splitmix_bytes(seed, n_u64):
    """SplitMix64 stream (same generator as the test oracle's ora_gen_ods)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n_u64 + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)


def gen_ods(k, seed):
    """Namespace-sorted synthetic ODS: v0 ns (0x00*19 ‖ 10 random) ‖ 483 random, sorted."""
    n = k * k
    rnd = splitmix_bytes(seed, n * 62).reshape(n, 496)
    ods = np.zeros((n, 512), np.uint8)
    ods[:, 19:29] = rnd[:, :10]
    ods[:, 29:] = rnd[:, 10:493]
    v = np.ascontiguousarray(ods).view(np.dtype((np.void, 512))).ravel()
    return np.sort(v).view(np.uint8).reshape(n, 512)


def _host_cpu():
    model, flags = "unknown", []
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and model == "unknown":
                model = line.split(":", 1)[1].strip()
            if line.startswith("flags") and not flags:
                f = line.split(":", 1)[1].split()
                flags = [x for x in ("avx2", "avx512f", "gfni", "sha_ni", "vaes") if x in f]
    except OSError:
        pass
    return model, flags


def _host_topology():
    """nproc, the bench process's affinity, physical cores and the cgroup CPU quota of this host."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    phys = set()
    try:
        pid = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                pid = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                core = line.split(":", 1)[1].strip()
                phys.add((pid, core))
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": aff, "physical_cores": len(phys) or None, "cgroup_cpu_quota": quota}


def _best_ms(fn, reps):
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        el = (time.perf_counter() - t0) * 1e3
        best = el if best is None else min(best, el)
    return best


def cpu_baseline(k, seconds, gpu=None):
    """The CPU restatement (oracle/, 'port': the Go reference cannot run here) on this host's cores, in the shapes
    SURVEY.md §8d prescribes, each next to its GPU number (`gpu`: the GPU extras of this run):
    * throughput (`value`): whole single-threaded ExtendShares+NewDataAvailabilityHeader calls on independent k=128
      blocks, one per worker thread, swept over 1 / 16 / 64 / all threads of the affinity mask;
    * single_block_ms: ONE k=128 block (the consensus path handles one block at a time,
      app/process_proposal.go:137,143) with rsmt2d's axis fan-out -- one task per row / column in every phase
      (oracle/da.c parallel_for) -- on 1, 16, the cgroup quota and all threads;
    * repair_c4_ms: config C4 (k=128 Repair, random 50 % and Q0-only) single-threaded like rsmt2d's solveCrossword,
      with klauspost's Leopard reconstruct as the decoder (ora_leo_decode_fft);
    * k512_ms: config C5 (one k=512 square, GF(2^16)) with axis fan-out;
    * blob_commitments: go-square CreateCommitment of 64 KiB blobs on one thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    topo = _host_topology()
    allt = topo["affinity"]
    quota = int(topo["cgroup_cpu_quota"]) if topo["cgroup_cpu_quota"] else allt
    ods = gen_ods(k, 0xC0FFEE)
    counts = sorted({1, min(16, allt), min(64, allt), allt})
    sweep, total_blocks = {}, {}
    for n in counts:
        blocks, el = O.extend_commit_throughput(ods, n, seconds / len(counts))
        sweep[str(n)] = round(blocks / el, 2)
        total_blocks[str(n)] = (blocks, round(el, 2))
    model, flags = _host_cpu()
    best = max(sweep, key=lambda n: sweep[n])
    phys = topo["physical_cores"] or allt
    out = {"value": sweep[best], "unit": "blocks/s", "cores": int(best), "kind": "port",
           "single_thread_value": sweep["1"], "sweep_threads_blocks_per_s": sweep,
           "all_threads": {"threads": allt, "value": sweep[str(allt)]},
           "full_host_linear_extrapolation": {"cores": phys, "value": round(sweep["1"] * phys, 1),
                                              "note": "single-thread rate x physical cores: an upper bound for "
                                                      "the whole host, not a measurement (the bench process is "
                                                      "limited by its cgroup CPU quota)"},
           "host": dict(topo, cpu=model, simd=flags)}
    # one block, axis fan-out (EDS written: da.ExtendShares returns it)
    lat_threads = sorted({1, min(16, allt), min(quota, allt), allt})
    out["single_block_ms"] = {str(n): round(_best_ms(lambda: O.extend_commit(ods, nthreads=n), 3 if n > 1 else 2), 2)
                              for n in lat_threads}
    # config C4 on the CPU
    w = 2 * k
    rc, eds, rr, cr, _ = O.extend_commit(ods, nthreads=min(quota, allt))
    rng = np.random.default_rng(7)
    q0 = np.zeros((w, w), np.uint8)
    q0[:k, :k] = 1
    c4 = {}
    for name, pres in (("random", (rng.random(w * w) < 0.5).astype(np.uint8)), ("q0_only", q0.reshape(-1))):
        damaged = eds.copy()
        damaged[pres == 0] = 0
        res = {}
        c4[name] = round(_best_ms(lambda: res.setdefault("r", O.repair(damaged, pres, rr, cr, fft=True)), 2), 1)
        if res["r"][0] != 0 or not np.array_equal(res["r"][1], eds):
            raise RuntimeError(f"CPU repair ({name}) did not restore the square")
    out["repair_c4_ms"] = dict(c4, note="k=128, single thread (rsmt2d's crossword is sequential), decoder = "
                                        "Leopard reconstruct (ora_leo_decode_fft); same damaged squares as repair_c4")
    # config C5 on the CPU
    ods512 = gen_ods(512, 0xC0FFEE)
    nq = min(quota, allt)
    k5 = {}
    r5 = {}
    k5[str(nq)] = round(_best_ms(lambda: r5.setdefault("r", O.extend_commit(ods512, want_eds=True, nthreads=nq)), 2), 1)
    k5["1"] = round(_best_ms(lambda: O.extend_commit(ods512, want_eds=False, nthreads=1), 1), 1)
    out["k512_ms"] = dict(k5, note="one k=512 square (GF(2^16)), EDS written, axis fan-out; keys = threads")
    out["k512_dah"] = r5["r"][4].hex()
    # blob share commitments on one thread, the bench's blobs; equal to the GPU's when this run computed them
    ns, data, offs = commitment_blobs()
    size = int(offs[1])
    n_cpu, t0 = 0, time.perf_counter()
    while n_cpu < len(offs) - 1 and time.perf_counter() - t0 < 2.0:
        rc, c = O.blob_commitment(ns[29 * n_cpu:29 * n_cpu + 29].tobytes(), data[n_cpu * size:(n_cpu + 1) * size].tobytes())
        if rc != 0 or (gpu and gpu.get("commitments") is not None and c != gpu["commitments"][n_cpu].tobytes()):
            raise RuntimeError("GPU blob commitment differs from the CPU restatement's")
        n_cpu += 1
    out["blob_commitments_1thread_per_s"] = round(n_cpu / (time.perf_counter() - t0), 1)
    # the per-axis shapes (rsmt2d over the CPU codec and wrapper tree) on the restatement, beside result["per_axis"]
    try:
        out["per_axis"] = per_axis_measure("oracle", os.path.join(ROOT, "oracle", "liboracle.so"), reps=3,
                                           reps_repair=2, reps_single=100)
    except Exception as e:
        out["per_axis"] = {"error": f"{type(e).__name__}: {e}"}
    out["sample"] = (f"k={k} ExtendShares+NewDataAvailabilityHeader (EDS written) via oracle/liboracle.so (C "
                     f"restatement, OpenSSL SHA-256 (SHA-NI), AVX2 Leopard; not the Go reference): throughput = "
                     f"independent blocks, one single-threaded call per worker thread, {seconds / len(counts):.1f} s "
                     f"per thread count over 1..{allt} threads (cgroup quota {topo['cgroup_cpu_quota']} CPUs), "
                     f"(blocks, s) per count: {total_blocks}; single_block_ms / repair_c4_ms / k512_ms: best of 1-3 "
                     f"calls; blob commitments: 64 KiB blobs")
    return out


AXES_DRIVER = os.path.join(ROOT, "tests", "abi_client", "rsmt2d_axes")


def _rfc6962_root(items):
    import hashlib
    if not items:
        return hashlib.sha256(b"").digest()
    if len(items) == 1:
        return hashlib.sha256(b"\x00" + items[0]).digest()
    s = 1
    while s * 2 < len(items):
        s *= 2
    return hashlib.sha256(b"\x01" + _rfc6962_root(items[:s]) + _rfc6962_root(items[s:])).digest()


def per_axis_measure(backend, lib_path, k=128, threads=8, reps_single=200, reps=5, reps_repair=5, seed=0xC0FFEE):
    """The per-axis drop-in seams -- what rsmt2d reaches when it runs with appconsts.DefaultCodec = cda.NewCodec and
    the GPU wrapper tree (go/pkg_da/extend_rocm.go): Codec.Encode / Decode (cda_rs_encode / cda_rs_decode) and the
    tree Root (cda_nmt_axis_root, pkg/wrapper/nmt_wrapper.go:118-124), each call through pageable host buffers as cgo
    passes Go slices.  tests/abi_client/rsmt2d_axes (a plain C caller, dlopen'ing `lib_path`) times:
    * single: one Encode (k x 512 B), one Decode (2k shards, half present), one Root (2k leaves);
    * extend: ComputeExtendedDataSquare + RowRoots/ColRoots in rsmt2d's shape -- erasureExtendSquare's 3k Encodes and
      computeRoots' 4k Roots, one task per axis ("goroutine") on `threads` OS threads;
    * repair_random / repair_q0_only: Repair in rsmt2d's shape (parallel prerepairSanityCheck, then the sequential
      crossword: Decode + Root per axis, Roots of newly completed orthogonal axes) of config C4's squares.
    backend "cda" = libcda (GPU), "oracle" = the CPU restatement (bench's cpu_baseline leg).  Every output is checked:
    the extension's DAH against tests/golden/bench_digests.json, each repair against the full square."""
    import subprocess
    import tempfile
    if not os.path.exists(AXES_DRIVER):
        raise RuntimeError("tests/abi_client/rsmt2d_axes not built (__graft_entry__.build())")
    w = 2 * k
    tmp = tempfile.mkdtemp(prefix="per_axis_")
    ods = gen_ods(k, seed).reshape(k * k, 512)
    ods_p = os.path.join(tmp, "ods.bin")
    ods.tofile(ods_p)

    def run(*args, timeout=600):
        p = subprocess.run([AXES_DRIVER, backend, lib_path] + [str(a) for a in args], capture_output=True, text=True,
                           timeout=timeout)
        if p.returncode != 0:
            raise RuntimeError(f"rsmt2d_axes {args[0]} failed ({p.returncode}): {p.stderr.strip()[-400:]}")
        return json.loads(p.stdout.strip().splitlines()[-1])

    out = {"k": k, "threads": threads, "backend": backend}
    out["single"] = run("single", k, reps_single, ods_p)
    # as Go runs it: errgroup starts one goroutine per axis and each blocks in cgo on its own OS thread
    out["extend_thread_per_axis"] = run("extend", k, 2 * k, reps, ods_p, tmp)
    out["extend"] = ext = run("extend", k, threads, reps, ods_p, tmp)
    eds = np.fromfile(os.path.join(tmp, "eds.bin"), np.uint8).reshape(w * w, 512)
    rr = np.fromfile(os.path.join(tmp, "row_roots.bin"), np.uint8).reshape(w, 90)
    cr = np.fromfile(os.path.join(tmp, "col_roots.bin"), np.uint8).reshape(w, 90)
    dah = _rfc6962_root([bytes(r) for r in rr] + [bytes(c) for c in cr]).hex()
    path = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
    want = json.load(open(path)).get(f"k{k}", {}).get(str(seed)) if os.path.exists(path) else None
    if want is not None and dah != want:
        raise RuntimeError(f"per-axis extension ({backend}) DAH {dah} != committed digest {want}")
    ext["dah_checked_vs_golden"] = want is not None
    roots_p = os.path.join(tmp, "roots.bin")
    np.concatenate([rr, cr]).tofile(roots_p)
    eds_p = os.path.join(tmp, "eds_full.bin")
    eds.tofile(eds_p)
    rng = np.random.default_rng(7)  # config C4's damaged squares (repair_measure / cpu_baseline: the same seed)
    q0 = np.zeros((w, w), np.uint8)
    q0[:k, :k] = 1
    for name, pres in (("random", (rng.random(w * w) < 0.5).astype(np.uint8)), ("q0_only", q0.reshape(-1))):
        pres_p = os.path.join(tmp, f"present_{name}.bin")
        pres.tofile(pres_p)
        r = run("repair", k, threads, reps_repair, eds_p, pres_p, roots_p, tmp)
        rep = np.fromfile(os.path.join(tmp, "repaired.bin"), np.uint8).reshape(w * w, 512)
        if r["rc"] != 0 or not np.array_equal(rep, eds):
            raise RuntimeError(f"per-axis repair ({backend}, {name}) rc {r['rc']} did not restore the square")
        out[f"repair_{name}"] = r
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)
    out["note"] = ("[min, median] over the timed calls; pageable malloc'd buffers (Go slices); extend/roots: one task per "
                   "axis on `threads` OS threads (extend_thread_per_axis: one thread per task, as Go's errgroup "
                   "goroutines each block in cgo on their own thread); repair: crossword sequential as in rsmt2d, the "
                   "sanity check's axes in parallel")
    return out


def repair_measure(ctx, k=128, survive=0.5, reps=9, warmup=2):
    """Config C4: rsmt2d Repair of a k=128 EDS from a random `survive` fraction of cells (host buffers in/out, repaired
    in place as through the C ABI), plus the Q0-only case (25 % of the cells: the structured repairable form of
    BASELINE's "25 % surviving"; random 25 % is unrepairable).  Each call gets a newly allocated
    (written) host square, as a cgo caller's; `warmup` untimed repairs precede the timed ones; min and median are
    reported."""
    import torch

    import cda
    w = 2 * k
    ods = gen_ods(k, 0xC0FFEE).reshape(k * k, 512)
    eds, rr, cr, _ = ctx.extend_commit(ods)
    rng = np.random.default_rng(7)
    out = {"k": k}
    q0 = np.zeros((w, w), np.uint8)
    q0[:k, :k] = 1
    d_eds = torch.empty(eds.shape, dtype=torch.uint8, device="cuda")
    for name, mk in (("random", lambda: (rng.random(w * w) < survive).astype(np.uint8)),
                     ("q0_only", lambda: q0.reshape(-1).copy())):
        cases = [mk() for _ in range(warmup + reps)]
        # device-resident form first (cda_repair_device on the square in HBM), as its own series
        dms = []
        for it, present in enumerate(cases):
            damaged = np.where(present[:, None] == 1, eds, 0).astype(np.uint8)
            d_eds.copy_(torch.from_numpy(damaged))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc, _, _ = ctx.repair_device(k, d_eds.data_ptr(), present, rr, cr)
            el_d = (time.perf_counter() - t0) * 1e3
            if rc != 0 or not np.array_equal(d_eds.cpu().numpy(), eds):
                raise RuntimeError("device repair produced a different EDS")
            if it >= warmup:
                dms.append(el_d)
        # then the host-buffer form, nothing else between the calls but building the next caller buffer
        ms, ok = [], True
        for it, present in enumerate(cases):
            damaged = np.empty_like(eds)  # a new caller buffer per call, as go/cda's Repair allocates one
            np.copyto(damaged, eds)
            damaged[present == 0] = 0
            t0 = time.perf_counter()
            try:
                ctx.repair(damaged, present, rr, cr, inplace=True)
                ok = True
            except cda.CdaError:
                ok = False
            el = (time.perf_counter() - t0) * 1e3
            if ok and not np.array_equal(damaged, eds):
                raise RuntimeError("repair produced a different EDS")
            if it >= warmup:
                ms.append(el)
        # go/cda's Repair: the present cells copied (8 goroutines) into a pooled page-locked slab that is reused, then
        # cda_repair on it; `ms` the call alone, `with_copy_ms` the copy on 8 threads + the call
        pooled = np.empty_like(eds)
        ctx.host_register(pooled)
        try:
            pms, pcms = [], []
            parts = np.array_split(np.arange(w * w), 8)

            from concurrent.futures import ThreadPoolExecutor
            ex = ThreadPoolExecutor(8)

            def fill(damaged):  # the copy into the slab on 8 threads (Go: present cells only, 8 goroutines)
                list(ex.map(lambda ix: np.copyto(pooled[ix[0]:ix[-1] + 1], damaged[ix[0]:ix[-1] + 1]), parts))

            for it, present in enumerate(cases):
                damaged = np.where(present[:, None] == 1, eds, 0).astype(np.uint8)
                t0 = time.perf_counter()
                fill(damaged)
                t1 = time.perf_counter()
                ctx.repair(pooled, present.copy(), rr, cr, inplace=True)
                t2 = time.perf_counter()
                if not np.array_equal(pooled, eds):
                    raise RuntimeError("pooled repair produced a different EDS")
                if it >= warmup:
                    pms.append((t2 - t1) * 1e3)
                    pcms.append((t2 - t0) * 1e3)
        finally:
            ex.shutdown()
            ctx.host_unregister(pooled)
        out[name] = {"ms": round(min(ms), 2), "ms_median": round(float(np.median(ms)), 2),
                     "device_resident_ms": round(min(dms), 2),
                     "device_resident_ms_median": round(float(np.median(dms)), 2), "repaired": ok,
                     "pooled_ms": round(min(pms), 2), "pooled_ms_median": round(float(np.median(pms)), 2),
                     "pooled_with_copy_ms_median": round(float(np.median(pcms)), 2)}
    out["survive"] = survive
    out["note"] = ("ms: cda_repair on host buffers, 32 MiB H2D + D2H of the EDS included (PCIe); device_resident_ms: "
                   "cda_repair_device on the square in HBM (presence and roots from the host); pooled_ms: cda_repair "
                   "on one page-locked buffer reused across calls (go/cda Repair's pooled slab), the damaged square "
                   "copied in beforehand (pooled_with_copy_ms_median: that copy on 8 threads included); "
                   f"{warmup} untimed + {reps} timed repairs per case, a new host buffer per call")
    return out


# bench kernel name -> rocprofv3 kernel name in profiles/*_counters.json
# (only kernels with ONE dispatch per step: the summaries average the counters over all dispatches of a kernel name,
# so the RS rows / columns launches and the tree-level launches would be mixed)
PMC_NAMES = {"leaf_hash": "leaf_hash_kernel", "dah": "dah_kernel"}
PMC_BATCH = 128  # scripts/profile.sh profiles the default bench step (B = 128 blocks)


def pmc_counters(kernel, B):
    """Per-launch PMC values of `kernel` from the newest committed rocprofv3 summary
    (profiles/r0*_counters.json; scripts/profile.sh + scripts/summarize_prof.py), scaled from the
    profiled batch to B.  hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (the gfx950 correction of
    MI355X_MICROARCH.md); valu_insts = SQ_INSTS_VALU (wave-instructions).  The NMT levels kernel runs
    with several grid sizes per step; summaries from round 4 on split its dispatches by grid
    ("nmt_levels_kernel@grid=N"): the largest grid is levels 1-2 (nmt_levels_1), the others the upper
    levels (nmt_levels, averaged per launch); the FF8 encoder's two launches likewise (columns: the larger grid).
    None if not covered."""
    import glob
    import re

    def order(f):  # r<round>_v<version>_counters.json, newest last
        m = re.match(r"r(\d+)(?:_v(\d+))?", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2) or 0)) if m else (0, 0)

    def per_grid(d, name):
        g = [(int(k.split("@grid=")[1]), v) for k, v in d.items() if k.startswith(name + "@grid=")]
        return sorted(g, key=lambda x: -x[0])

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_counters.json")), key=order)
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in PMC_NAMES:
            c, src = d.get(PMC_NAMES[kernel]), PMC_NAMES[kernel]
        elif kernel in ("nmt_levels_1", "nmt_levels"):
            g = per_grid(d, "nmt_levels_kernel")
            if len(g) < 2:
                continue
            if kernel == "nmt_levels_1":
                c, src = g[0][1], f"nmt_levels_kernel@grid={g[0][0]}"
            else:
                rest = [v for _, v in g[1:]]
                n = sum(v.get("dispatches", 1) for v in rest)
                c = {key: sum(v.get(key, 0) * v.get("dispatches", 1) for v in rest) / n
                     for key in ("hbm_bytes_corrected", "SQ_INSTS_VALU") if all(key in v for v in rest)}
                c["bench_batch"] = rest[0].get("bench_batch", PMC_BATCH)
                src = "nmt_levels_kernel@grid<" + str(g[0][0])
        elif kernel in ("rs_encode8_rows", "rs_encode8_cols"):
            g = per_grid(d, "rs_encode8_g2_kernel<7>")  # columns: twice the rows' workgroups (2k codewords)
            if len(g) != 2:
                continue
            c, src = g[0 if kernel == "rs_encode8_cols" else 1][1], \
                f"rs_encode8_g2_kernel<7>@grid={g[0 if kernel == 'rs_encode8_cols' else 1][0]}"
        else:
            return None
        if not c:
            continue
        scale = B / float(c.get("bench_batch", PMC_BATCH))
        return {"hbm_bytes": int(c["hbm_bytes_corrected"] * scale) if "hbm_bytes_corrected" in c else None,
                "valu_insts": c["SQ_INSTS_VALU"] * scale if "SQ_INSTS_VALU" in c else None,
                "source": f"{os.path.relpath(f, ROOT)} ({src}, B={c.get('bench_batch', PMC_BATCH)} "
                          f"profile scaled to B={B})"}
    return None


def single_block_measure(ctx, dev, k=128, reps=50):
    """Config C2: ONE k=128 block on one GPU, device-resident (the latency of one ExtendShares +
    NewDataAvailabilityHeader with the ODS already in HBM), with its per-kernel split.  One block fills few of the
    256 CUs (the tree levels and the DAH are chains of dependent SHA-256 compressions), so this is latency, not the
    batch throughput of the headline."""
    import torch
    w = 2 * k
    ods = torch.from_numpy(gen_ods(k, 0xC0FFEE)).to(dev)
    eds = torch.empty((1, w * w, 512), dtype=torch.uint8, device=dev)
    roots = torch.empty((1, 2 * w, 96), dtype=torch.uint8, device=dev)
    dah = torch.empty((1, 32), dtype=torch.uint8, device=dev)
    st = torch.empty((1,), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.extend_commit_device(k, 1, ods.data_ptr(), eds.data_ptr(), roots.data_ptr(), dah.data_ptr(),
                                 st.data_ptr(), stream.cuda_stream)
    step()
    torch.cuda.synchronize(dev)
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        best = min(best, time.perf_counter() - t0)
    ctx.profile_reset()
    ctx.profile_enable(True)
    step()
    torch.cuda.synchronize(dev)
    prof = ctx.profile_read()
    ctx.profile_enable(False)
    return {"k": k, "ms": round(best * 1e3, 3),
            "kernels_ms": {n: round(ms / max(1, cnt), 4) for n, (ms, cnt) in prof.items()},
            "note": "device-resident, best of %d; host-buffer latency: host_buffers.one_block_latency_ms" % reps}


def k512_measure(ctx, dev, reps=3):
    """Config C5 on ONE GPU: k=512 (GF(2^16) Leopard, 512 MiB EDS, 2,048 roots) through the device-resident block
    path (2 blocks per call), and through cda.split with a single rank (the multi-GPU code path at world size 1).
    FF16 parity is unpinned by reference data (no GF(2^16) vector in the reference; checked against the Lagrange
    oracle) -- see DESIGN.md §3."""
    import torch
    import cda
    from cda import split
    k, B = 512, 2
    w = 2 * k
    ods = torch.from_numpy(np.stack([gen_ods(k, 0xC0FFEE + b) for b in range(B)])).to(dev)
    eds = torch.empty((B, w * w, 512), dtype=torch.uint8, device=dev)
    roots = torch.empty((B, 2 * w, 96), dtype=torch.uint8, device=dev)
    dah = torch.empty((B, 32), dtype=torch.uint8, device=dev)
    st = torch.empty((B,), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.extend_commit_device(k, B, ods.data_ptr(), eds.data_ptr(), roots.data_ptr(), dah.data_ptr(),
                                 st.data_ptr(), stream.cuda_stream)
    step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / reps
    ctx.profile_reset()
    ctx.profile_enable(True)
    step()
    torch.cuda.synchronize(dev)
    prof = ctx.profile_read()
    ctx.profile_enable(False)
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")))["k512"]
    for b in range(B):
        if bytes(dah[b].cpu().numpy()).hex() != want[str(0xC0FFEE + b)]:
            raise RuntimeError(f"k=512 block {b} DAH differs from the committed digest")
    out = {"k": k, "blocks_per_call": B, "ms_per_block": round(el * 1e3 / B, 3), "blocks_per_s": round(B / el, 2),
           "dah_golden": want[str(0xC0FFEE)], "dahs_checked_vs_golden": B,
           "path_hbm_gbs": round(block_bytes(k) * B / el / 1e9, 1),
           "kernels_ms": {n: round(ms / max(1, cnt), 3) for n, (ms, cnt) in prof.items()},
           "parity": "GF(2^16) unpinned by reference data (Lagrange-oracle checked)"}
    # the same path with ONE square per call: the per-call fixed costs (the DAH's dependent chain, launch gaps) that
    # two squares per call share -- the like-for-like reference for the split entry below (one square per call)
    def step1():
        ctx.extend_commit_device(k, 1, ods.data_ptr(), eds.data_ptr(), roots.data_ptr(), dah.data_ptr(),
                                 st.data_ptr(), stream.cuda_stream)
    step1()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        step1()
    torch.cuda.synchronize(dev)
    out["one_square_per_call_ms"] = round((time.perf_counter() - t0) * 1e3 / reps, 3)
    del eds, roots
    # config C5's split path behind the C ABI (cda_multi_extend_commit_split_device): one square over the devices of
    # a handle.  On one GPU: G = 1 (the row slab is the column slab's top half, no exchange) and G = 8 replicas on
    # this device (the 8-device plan with device copies for the RCCL exchange -- a rehearsal, not a scaling number)
    want_dah = want[str(0xC0FFEE)]
    rows = ods[0].view(k, k, 512)
    for G in (1, 8):
        m = cda.MultiContext.replicas(dev.index, G)
        rp = k // G
        slabs = [rows[g * rp:(g + 1) * rp].contiguous() for g in range(G)]
        torch.cuda.synchronize(dev)
        ptrs = [sl.data_ptr() for sl in slabs]
        m.extend_commit_split_device(k, ptrs)
        t0 = time.perf_counter()
        for _ in range(reps):
            _, _, d = m.extend_commit_split_device(k, ptrs)
        el = (time.perf_counter() - t0) / reps
        if d.hex() != want_dah:
            raise RuntimeError(f"split (G={G}) DAH differs from the committed digest")
        prof = None
        if G == 1:
            c0 = m.context(0)
            c0.profile_reset()
            c0.profile_enable(True)
            m.extend_commit_split_device(k, ptrs)
            prof = {n: round(ms / max(1, cnt), 3) for n, (ms, cnt) in c0.profile_read().items()}
            c0.profile_enable(False)
        out[f"split_capi_G{G}_on_1gpu"] = {"ms_per_square": round(el * 1e3, 3), "dah_matches_golden": True,
                                            **({"kernels_ms": prof} if prof else {})}
        m.close()
    ops = split.DeviceOps(ctx)
    split.extend_commit_split(ops, k, rows)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        res = split.extend_commit_split(ops, k, rows)
    torch.cuda.synchronize(dev)
    out["split_py_on_1gpu"] = {"ms_per_square": round((time.perf_counter() - t0) * 1e3 / reps, 3),
                               "dah_matches_golden": res.dah.hex() == want_dah,
                               "note": "cda/split.py over torch.distributed (world 1), the cross-process form"}
    return out


def square_measure(ctx, reps=3):
    """square.Construct on the device (cda_construct_extend_commit): a k=128 block of BlobTxs (one 60 KiB blob each)
    planned on the host, only the payload bytes uploaded, the shares assembled in HBM, then the block path.  The
    host-side layout planning (Python) is outside the timed call."""
    from cda import square as S
    rng = np.random.default_rng(3)
    txs = []
    for i in range(120):
        ns_id = bytes(18) + bytes([1 + i % 255]) + bytes(rng.integers(0, 256, 9, dtype=np.uint8))
        data = bytes(rng.integers(0, 256, 60 * 1024, dtype=np.uint8))
        blob = b"\x0a" + S.varint(len(ns_id)) + ns_id + b"\x12" + S.varint(len(data)) + data
        tx = bytes(rng.integers(0, 256, 200, dtype=np.uint8))
        txs.append(b"\x0a" + S.varint(len(tx)) + tx + b"\x12" + S.varint(len(blob)) + blob + b"\x1a\x04BLOB")
    ss, segs, info = S.plan(txs, 128, 64)
    prepared = S.device_plan(segs)
    data = prepared[1]
    ctx.construct_extend_commit(ss, segs, want_eds=False, prepared=prepared)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.construct_extend_commit(ss, segs, want_eds=False, prepared=prepared)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return {"k": ss, "blobs": info["blobs"], "ms": round(best * 1e3, 3), "payload_bytes": int(data.size),
            "ods_bytes": ss * ss * 512,
            "note": "one cda_construct_extend_commit call (plan H2D, shares built on the GPU, extension, roots, DAH) "
                    "vs uploading the materialised ODS: compare host_buffers.one_block_latency_ms.roots_only"}


def proof_measure(ctx, k, reps=5):
    """pkg/proof NewShareInclusionProof for a 500-share range of a k=128 square (cda_share_inclusion_proof:
    extension + export of the proof's row trees + proof assembly, host ODS in)."""
    ods = gen_ods(k, 0xC0FFEE)
    ctx.share_inclusion_proof(ods, 1000, 1500)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = ctx.share_inclusion_proof(ods, 1000, 1500)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return {"k": k, "shares": 500, "rows": len(out["rows"]), "ms": round(best * 1e3, 2),
            "note": "one cda_share_inclusion_proof call: H2D of the ODS, extension, the nodes of the proof's rows "
                    "copied out, NMT range proofs + RFC-6962 aunts assembled from them"}


def host_path_measure(ctx, k, nblocks=48, reps=3):
    """The drop-in boundary with host buffers (cgo passes Go slices): cda_extend_commit_batch streams nblocks
    host ODS through the GPU (H2D / compute / D2H pipelined over three streams), with and without the EDS
    copy-out, from pageable and from pinned (cda_host_alloc) memory; plus one-block latency through
    cda_extend_commit.  PCIe-inclusive; reported beside, never as, the bench value."""
    ods = np.stack([gen_ods(k, 0xC0FFEE + b) for b in range(min(4, nblocks))])
    ods = np.ascontiguousarray(np.concatenate([ods] * (nblocks // len(ods)))).reshape(nblocks, k * k, 512)
    eds = np.ones((nblocks, 4 * k * k, 512), np.uint8)  # reused, already-touched output (a Go slice is zeroed)
    pin_in, pin_out = ctx.pinned(ods.shape), ctx.pinned(eds.shape)
    pin_in.array[:] = ods
    out = {}

    def best_of(fn):
        fn()
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        return best

    for mem, src, dst in (("pageable", ods, eds), ("pinned", pin_in.array, pin_out.array)):
        for want_eds in (True, False):
            el = best_of(lambda: ctx.extend_commit_batch(src, want_eds=want_eds, eds_out=dst if want_eds else None))
            moved = nblocks * (k * k * 512 + (4 * k * k * 512 if want_eds else 0))
            out[f"{mem}_{'with_eds' if want_eds else 'roots_only'}"] = {
                "blocks_per_s": round(nblocks / el, 1), "ms": round(el * 1e3, 2),
                "pcie_gbs": round(moved / el / 1e9, 1)}
    one, one_out = ods[0:1], eds[0:1]  # one block; the EDS lands in an already-touched buffer, as above
    out["one_block_latency_ms"] = {
        "roots_only": round(best_of(lambda: ctx.extend_commit_batch(one, want_eds=False)) * 1e3, 3),
        "with_eds": round(best_of(lambda: ctx.extend_commit_batch(one, want_eds=True, eds_out=one_out)) * 1e3, 3)}
    one_ods = ods[0].copy()
    pin_in.free()
    pin_out.free()
    del eds, one_out, ods, one  # the batch's 2 GB of host buffers are gone before the fresh-buffer series
    out["one_block_fresh"] = one_block_fresh(ctx, one_ods)
    import torch
    h = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
    d = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    el_h2d = best_of(lambda: (d.copy_(h, non_blocking=True), torch.cuda.synchronize()))
    el_d2h = best_of(lambda: (h.copy_(d, non_blocking=True), torch.cuda.synchronize()))
    out["pcie_copy_gbs"] = {"h2d": round(h.numel() / el_h2d / 1e9, 1), "d2h": round(h.numel() / el_d2h / 1e9, 1),
                            "note": "256 MiB pinned<->device copy (torch), the link's ceiling for this path"}
    out["note"] = (f"{nblocks} k={k} blocks per call (8 MiB in, + 32 MiB EDS out per block), output reused; bound: "
                   "PCIe Gen5 x16 (~50 GB/s per direction measured by hipMemcpy), H2D for roots_only, D2H with_eds")
    return out


def one_block_fresh(ctx, ods, reps=25, warmup=3):
    """The consensus call in the shapes go/cda makes it (app/prepare_proposal.go:65-93, app/process_proposal.go:137-151,
    app/extend_block.go:25; go/cda/extend.go).  One k=128 block per cda_extend_commit_batch call; min / median / max
    over `reps` calls after `warmup`; every DAH checked, and the EDS of the last call of each series.
      roots_only            ProcessProposal / PrepareProposal through the roots-only entry (da.NewDataAvailability-
                            HeaderFromShares, go/patches/0004): a fresh copy of the shares per call (np copy, outside
                            the timed call, like the Go caller's own flatten), no EDS.
      roots_only_pooled_in  the same with the shares flattened INTO a pooled page-locked slab inside the timed region
                            (go/cda's share pool: the flatten the Go caller does anyway, then a direct DMA).
      pooled_eds            ExtendShares / ExtendBlock (which must return the EDS): fresh shares (as roots_only), the
                            EDS written into one of two recycled page-locked slabs (go/cda's EDS pool: Go-heap slabs
                            registered once with cda_host_register and recycled through the garbage collector).
      pooled_both           pooled shares slab (flatten inside the timed region) + pooled EDS slab.
      pooled_eds_inplace    go/cda's ExtendShares: the shares flattened into Q0 of a pooled EDS slab (untimed, as the
                            fresh share copy of the other series), then cda_extend_commit_eds in place: no share
                            buffer, no host Q0 copy, the input bands are 2-D DMAs from page-locked memory.
      pooled_eds_inplace_flatten  the same with the flatten inside the timed region (the Go call end to end).
      with_eds              fresh shares and a NEW never-touched EDS buffer per call (np.empty, as a Go make()), no
                            huge-page hint (the release default: the library does not change caller page policy).
      with_eds_hugepages    the same on a context that opted in (cda_set_option(CDA_OPT_HUGE_PAGES, 1)).
      pinned_with_eds       cda_host_alloc buffers reused across calls."""
    import cda
    from cda import _native as N
    k = int(round(len(ods) ** 0.5))
    eds_ref, _, _, dah_ref = ctx.extend_commit(ods)
    res = {}
    # A fresh box's device-to-host path runs every with-EDS form at about twice its steady time for its first seconds
    # (profiles/r05_consensus_shapes_v1.log: rounds 0-1 1.44-1.66 ms, round 2 0.70-0.80 ms); a node
    # pays that once at start-up.  Pinned one-block calls until ten in a row are within 10 % of their median (at most
    # 12 s), recorded, before the timed series.
    pb_o, pb_e = ctx.pinned((1, k * k, 512)), ctx.pinned((1, 4 * k * k, 512))
    pb_o.array[0] = ods
    wts, t_w = [], time.perf_counter()
    while time.perf_counter() - t_w < 12:
        a = time.perf_counter()
        ctx.extend_commit_batch(pb_o.array, eds_out=pb_e.array)
        wts.append((time.perf_counter() - a) * 1e3)
        if len(wts) >= 10 and max(wts[-10:]) < 1.1 * float(np.median(wts[-10:])):
            break
    res["d2h_warmup"] = {"s": round(time.perf_counter() - t_w, 2), "calls": len(wts), "first_ms": round(wts[0], 3),
                         "settled_ms": round(float(np.median(wts[-10:])), 3)}
    pb_o.free()
    pb_e.free()

    def series(name, call, check_eds=None):
        ts = []
        for i in range(warmup + reps):
            prep = call(i)
            t0 = time.perf_counter()
            dah = prep()
            el = (time.perf_counter() - t0) * 1e3
            if bytes(dah) != dah_ref:
                raise RuntimeError(f"one-block DAH differs ({name})")
            if i >= warmup:
                ts.append(el)
        if check_eds is not None and not np.array_equal(check_eds(), eds_ref):
            raise RuntimeError(f"one-block EDS differs ({name})")
        res[name] = {"ms_min": round(min(ts), 3), "ms_median": round(float(np.median(ts)), 3),
                     "ms_max": round(max(ts), 3), "median_over_min": round(float(np.median(ts)) / min(ts), 3)}

    # roots only, fresh shares
    def roots_fresh(i):
        src = ods.copy()[None]
        return lambda: ctx.extend_commit_batch(src, want_eds=False)[3][0]
    series("roots_only", roots_fresh)
    # pooled (registered) share slabs and EDS slabs, recycled round-robin like go/cda's pools
    pool_in = [np.empty((1, k * k, 512), np.uint8) for _ in range(2)]
    pool_out = [np.empty((1, 4 * k * k, 512), np.uint8) for _ in range(2)]
    for b in pool_in + pool_out:
        ctx.host_register(b)
    try:
        def roots_pooled_in(i):
            slab = pool_in[i % 2]

            def run():
                np.copyto(slab[0], ods)  # the caller's flatten, into the pooled slab
                return ctx.extend_commit_batch(slab, want_eds=False)[3][0]
            return run
        series("roots_only_pooled_in", roots_pooled_in)
        last = {}

        def pooled_eds(i):
            src = ods.copy()[None]
            out = pool_out[i % 2]
            last["out"] = out
            return lambda: ctx.extend_commit_batch(src, eds_out=out)[3][0]
        series("pooled_eds", pooled_eds, lambda: last["out"][0])

        def pooled_both(i):
            slab, out = pool_in[i % 2], pool_out[i % 2]
            last["out"] = out

            def run():
                np.copyto(slab[0], ods)
                return ctx.extend_commit_batch(slab, eds_out=out)[3][0]
            return run
        series("pooled_both", pooled_both, lambda: last["out"][0])

        def q0(buf):
            return buf[0].reshape(2 * k, 2 * k, 512)[:k, :k]

        def pooled_inplace(i):
            out = pool_out[i % 2]
            q0(out)[:] = ods.reshape(k, k, 512)  # the caller's flatten, straight into Q0 of the pooled slab
            last["out"] = out
            return lambda: ctx.extend_commit_eds(out[0])[2]
        series("pooled_eds_inplace", pooled_inplace, lambda: last["out"][0])

        def pooled_inplace_flatten(i):
            out = pool_out[i % 2]
            last["out"] = out

            def run():
                q0(out)[:] = ods.reshape(k, k, 512)
                return ctx.extend_commit_eds(out[0])[2]
            return run
        series("pooled_eds_inplace_flatten", pooled_inplace_flatten, lambda: last["out"][0])
    finally:
        for b in pool_in + pool_out:
            ctx.host_unregister(b)
    # fresh, never-touched EDS buffers (allocated before the series, kept alive: freeing unmaps them)
    for name, c in (("with_eds", ctx), ("with_eds_hugepages", None)):
        if c is None:
            c = cda.Context(ctx.device)
            c.set_option(N.OPT_HUGE_PAGES, 1)
        bufs = [np.empty((1, 4 * k * k, 512), np.uint8) for _ in range(warmup + reps)]

        def fresh(i, c=c, bufs=bufs):
            src = ods.copy()[None]
            return lambda: c.extend_commit_batch(src, eds_out=bufs[i])[3][0]
        series(name, fresh, lambda bufs=bufs: bufs[-1][0])
        del bufs
        if c is not ctx:
            c.close()
    # a caller that recycles pinned buffers (cda_host_alloc) for the shares and the EDS: both DMAs direct
    pb_ods, pb_eds = ctx.pinned((1, k * k, 512)), ctx.pinned((1, 4 * k * k, 512))
    try:
        def pinned(i):
            pb_ods.array[0] = ods
            return lambda: ctx.extend_commit_batch(pb_ods.array, eds_out=pb_eds.array)[3][0]
        series("pinned_with_eds", pinned, lambda: pb_eds.array[0])
    finally:
        pb_ods.free()
        pb_eds.free()
    res["consensus_targets_ms"] = {"roots_only_median": 0.45, "pooled_eds_median": 0.70,
                                   "source": "VERDICT r04 next #1 (driver BENCH line)",
                                   "go_calls": {"PrepareProposal/ProcessProposal (patch 0004)": "roots_only",
                                                "ExtendShares/ExtendBlock (go/cda/pool.go)": "pooled_eds_inplace"}}
    res["note"] = (f"cda_extend_commit_batch, one k={k} block per call, {warmup} untimed + {reps} timed calls per "
                   f"series; csrc/consensus.cpp; pooled slabs: np.empty + cda_host_register, two per pool, "
                   f"round-robin (go/cda/pool.go)")
    return res


def commitment_blobs(nblobs=256, size=64 * 1024):
    """The bench's blob batch: random 64 KiB blobs under random v0 namespaces (seeded)."""
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, nblobs * size, dtype=np.uint8)
    ns = np.zeros((nblobs, 29), np.uint8)
    ns[:, 19:] = rng.integers(0, 256, (nblobs, 10), dtype=np.uint8)
    return ns.reshape(-1), data, np.arange(nblobs + 1, dtype=np.uint64) * size


def commitments_measure(ctx, reps=5):
    """x/blob share commitments (inclusion.CreateCommitments) of a batch of random blobs: one cda_blob_commitments
    call on pre-packed host arrays (H2D of the blob data included).  The CPU leg (cpu_baseline) recomputes the
    first ones with the oracle and compares."""
    ns, data, offs = commitment_blobs()
    nblobs, size = len(offs) - 1, int(offs[1])
    got = ctx.blob_commitments_packed(ns, data, offs)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.blob_commitments_packed(ns, data, offs)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return {"blobs": nblobs, "blob_bytes": size, "ms": round(best * 1e3, 3), "blobs_per_s": round(nblobs / best, 1),
            "mb_per_s": round(nblobs * size / best / 1e6, 1),
            "note": "one cda_blob_commitments call incl. H2D of the blob data (pageable), threshold 64"}, got


def launch_ranks(args):
    """bench.py --gpus N without torchrun: spawn N rank processes of this script (before anything
    touches the GPU), one per device, rank r -> device r % device_count; exit with the worst rank's code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


def dist_setup(world, local, dry_run):
    """Device for this rank and the process group.  Ranks that share a device (a 1-GPU lease running
    --gpus 2 as a logic check) or a dry run use gloo; one rank per device uses RCCL ("nccl")."""
    import torch
    import torch.distributed as dist
    if dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        return None, "gloo", False
    ndev = torch.cuda.device_count()  # does not initialise HIP on this image
    if ndev < 1:
        raise RuntimeError("no HIP device visible")
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    shared = world > ndev
    backend = "gloo" if shared else "nccl"
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return dev, backend, shared


def max_over_ranks(x, world, backend, dev):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world, backend, dev):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def rank_report(world, rank, backend, dev, cpu_group, ms_per_step=None, blocks=None, check=None):
    """Self-verification of a multi-rank run: `ranks_seen` = an all_reduce SUM of 1 over the
    run's own process group (RCCL when one rank per GPU), and every rank's own step time, device and output check,
    gathered over the CPU (gloo) group -- so the N-GPU line shows that each rank took part and on which GPU."""
    import torch.distributed as dist
    seen = sum_over_ranks(1.0, world, backend, dev)
    mine = {"rank": rank, "host": os.uname().nodename, "pid": os.getpid()}
    if dev is not None:
        import torch
        props = torch.cuda.get_device_properties(dev)
        mine.update(device=dev.index, device_name=props.name,
                    pci_bus_id=getattr(props, "pci_bus_id", None), pci_device_id=getattr(props, "pci_device_id", None),
                    visible_devices=os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES"))
    if ms_per_step is not None:
        mine["ms_per_step"] = round(ms_per_step, 4)
    if blocks is not None:
        mine["blocks"] = blocks
    if check is not None:
        mine["blocks_checked_vs_golden"] = check.get("blocks_checked_vs_golden")
    per = [mine]
    if world > 1:
        per = [None] * world
        dist.all_gather_object(per, mine, group=cpu_group)
    devs = [p.get("device") for p in per]
    return {"ranks_seen": int(seen), "backend": backend, "per_rank": per,
            "distinct_devices": len({(p.get("host"), p.get("pci_bus_id"), p.get("device")) for p in per})
            if dev is not None else None,
            "all_ranks_checked": all((p.get("blocks_checked_vs_golden") or 0) > 0 for p in per) if check else None,
            "devices": devs}


# ---- config C5's product path at N > 1: one k=512 square over all devices of the node, RCCL exchange ----------------
# The driver's multi-GPU command is `bench.py --gpus N` (one rank per GPU).  After the timed block-batch loop, rank 0
# hands one k=512 square to cda_multi_extend_commit_split_device over the devices the ranks use (ncclCommInitAll +
# one grouped send/recv exchange + a gather: csrc/split.cpp) and reports it beside G = 1.  It runs in a helper
# process that rank 0 starts BEFORE anything touches the GPU (no fork/exec from a GPU process), waiting on a pipe;
# the other ranks sit in a CPU (gloo) barrier meanwhile, so no RCCL kernel of theirs spins on the devices.  A
# failure or a hang of the helper becomes an "error" field, never the headline's exit code.
K512_SPLIT_TIMEOUT_S = 240


class SplitHelper:
    def __init__(self, ndev, dry_run):
        import subprocess
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
        cmd = [sys.executable, os.path.abspath(__file__), "--k512-split-helper", str(ndev)]
        if dry_run:
            cmd.append("--dry-run")
        self.p = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)

    def run(self, timeout=K512_SPLIT_TIMEOUT_S):
        import subprocess
        t0 = time.perf_counter()
        try:
            out, _ = self.p.communicate("go\n", timeout=timeout)
        except subprocess.TimeoutExpired:
            self.p.kill()
            self.p.communicate()
            return {"error": f"k=512 split helper timed out after {timeout} s (killed)"}
        lines = [l for l in out.splitlines() if l.startswith("{")]
        if self.p.returncode != 0 or not lines:
            return {"error": f"k=512 split helper exited {self.p.returncode}", "tail": out[-400:]}
        r = json.loads(lines[-1])
        r["helper_wall_s"] = round(time.perf_counter() - t0, 2)
        return r

    def close(self):
        if self.p.poll() is None:
            try:
                self.p.communicate("quit\n", timeout=30)
            except Exception:
                self.p.kill()


def split_measure(devices, k=512, reps=10, warmup=2, dev_mask_note=""):
    """One k-square over `devices` through cda_multi_extend_commit_split_device (G = len(devices)), and over the
    first device alone (G = 1), each with device-resident ODS slabs; per-call times (the call returns the 4k roots
    and the DAH on the host), the DAH checked against tests/golden/bench_digests.json."""
    import torch
    import cda
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")))[f"k{k}"][str(0xC0FFEE)]
    rows = gen_ods(k, 0xC0FFEE).reshape(k, k, 512)
    out = {"k": k, "devices": list(devices), "G": len(devices), "dah_golden": want}
    for label, devs in (("G1", devices[:1]), (f"G{len(devices)}", devices)):
        if label == "G1" and len(devices) == 1 and "G1" in out:
            continue
        G = len(devs)
        rp = k // G
        mask = 0
        for d in devs:
            mask |= 1 << d
        t0 = time.perf_counter()
        m = cda.MultiContext(mask)
        slabs = [torch.from_numpy(np.ascontiguousarray(rows[g * rp:(g + 1) * rp])).to(f"cuda:{d}")
                 for g, d in enumerate(devs)]
        for d in devs:
            torch.cuda.synchronize(d)
        ptrs = [s.data_ptr() for s in slabs]
        _, _, dah = m.extend_commit_split_device(k, ptrs)  # first call: ncclCommInitAll when G > 1
        first_s = time.perf_counter() - t0
        for _ in range(warmup):
            m.extend_commit_split_device(k, ptrs)
        ts = []
        for _ in range(reps):
            t1 = time.perf_counter()
            _, _, dah = m.extend_commit_split_device(k, ptrs)
            ts.append((time.perf_counter() - t1) * 1e3)
        out[label] = {"ms_per_square": round(min(ts), 3), "ms_median": round(float(np.median(ts)), 3),
                      "dah_matches_golden": dah.hex() == want, "init_and_first_call_s": round(first_s, 3)}
        m.close()
        del slabs
    gN = out.get(f"G{len(devices)}")
    if gN and len(devices) > 1:
        out["speedup_vs_G1"] = round(out["G1"]["ms_median"] / gN["ms_median"], 2)
    out["note"] = ("cda_multi_extend_commit_split_device: rows over devices, one RCCL grouped send/recv exchange of the "
                   "top half (shares + leaf records), column pass, gather + DAH on device 0; per-call host time, roots "
                   "and DAH returned to the host" + dev_mask_note)
    return out


def split_helper_main(args):
    """--k512-split-helper N: wait for "go" on stdin, then time config C5's split over devices 0..N-1."""
    line = sys.stdin.readline().strip()
    if line != "go":
        return
    if args.dry_run:
        print(json.dumps({"dry_run": True, "G": args.k512_split_helper}), flush=True)
        return
    try:
        res = split_measure(list(range(args.k512_split_helper)))
    except Exception as e:  # reported in the bench line, never raised into the bench's exit code
        res = {"error": f"{type(e).__name__}: {e}"}
    print(json.dumps(res), flush=True)


VALU_CYCLES_PER_WAVE_INSTR = 2  # wave64 on a SIMD-32 (MI355X_MICROARCH.md, execution model)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--batch", type=int, default=128,
                    help="independent blocks per GPU per step (128 = config C3: 1024 blocks over 8 GPUs)")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the repair/commitment/host-path/proof extras")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only (spawn, process group, max-over-ranks); no GPU work")
    ap.add_argument("--workload", choices=["block_batch", "split"], default="block_batch",
                    help="block_batch: B independent blocks per GPU (default, BASELINE metric); "
                         "split: ONE k-square split over all ranks with an RCCL all-to-all (config C5, --k 512)")
    ap.add_argument("--k512-split-helper", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--no-k512-split", action="store_true", help="skip config C5's split after the timed loop")
    args = ap.parse_args()
    if args.k512_split_helper:
        return split_helper_main(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.workload == "split":
        return bench_split(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # config C5 at N > 1: the helper process starts before this process touches the GPU (SplitHelper)
    helper = None
    if rank == 0 and world > 1 and not args.no_k512_split:
        helper = SplitHelper(split_devices(world), args.dry_run)
    try:
        return bench_main(args, world, rank, local, helper)
    finally:
        if helper is not None:
            helper.close()


def split_devices(world):
    """Distinct devices the ranks use (rank r -> device r % device_count; device_count does not initialise HIP)."""
    try:
        import torch
        ndev = torch.cuda.device_count()
    except Exception:
        ndev = 0
    n = min(world, ndev) if ndev else world
    while n & (n - 1):  # the split takes a power of two of devices
        n &= n - 1
    return max(1, n)


def bench_main(args, world, rank, local, helper):
    dev, backend, shared = dist_setup(world, local, args.dry_run)
    import torch
    import torch.distributed as dist
    cpu_group = dist.new_group(backend="gloo") if world > 1 else None
    if args.dry_run:
        if world > 1:
            dist.barrier()
        ranks = sum_over_ranks(1.0, world, backend, dev)
        t = max_over_ranks(float(rank), world, backend, dev)
        rep = rank_report(world, rank, backend, dev, cpu_group, ms_per_step=float(rank), blocks=0)
        split = None
        if world > 1:
            dist.barrier(group=cpu_group)
            if helper is not None:
                split = helper.run()
            dist.barrier(group=cpu_group)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": int(ranks), "max_rank": int(t),
                              "backend": backend, "ranks": rep, **({"k512_split": split} if split else {})}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    import cda
    ctx = cda.Context(dev.index)
    k, B = args.k, args.batch
    w = 2 * k
    # synthetic blocks, DISTINCT different squares per rank (seed = 0xC0FFEE + rank * B + b), replicated to fill B
    nd = min(B, DISTINCT_ODS)
    base = [gen_ods(k, 0xC0FFEE + rank * B + b) for b in range(nd)]
    ods_host = np.stack([base[b % nd] for b in range(B)])
    d_ods = torch.from_numpy(ods_host).to(dev)
    del ods_host
    d_eds = torch.empty((B, w * w, 512), dtype=torch.uint8, device=dev)
    d_roots = torch.empty((B, 2 * w, 96), dtype=torch.uint8, device=dev)
    d_dah = torch.empty((B, 32), dtype=torch.uint8, device=dev)
    d_status = torch.empty((B,), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.extend_commit_device(k, B, d_ods.data_ptr(), d_eds.data_ptr(), d_roots.data_ptr(), d_dah.data_ptr(),
                                 d_status.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if int(d_status.cpu().max()) != -1 or int(d_status.cpu().min()) != -1:
        raise RuntimeError("namespace-order status set on a sorted synthetic square")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    mine_s = time.perf_counter() - t0  # this rank's own steps (before the closing barrier)
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, backend, dev)

    blocks = world * B * args.steps
    value = blocks / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    # the timed steps' output: every block's DAH against the committed digests (tests/golden/bench_digests.json)
    check = check_dahs(d_dah.cpu().numpy(), k, B, rank, nd)
    ranks_rep = rank_report(world, rank, backend, dev, cpu_group, ms_per_step=1000.0 * mine_s / args.steps,
                            blocks=B * args.steps, check=check)

    # per-kernel durations: HIP events on the launch stream, separate pass (profiling adds event records)
    ctx.profile_reset()
    ctx.profile_enable(True)
    prof_steps = max(2, min(5, args.steps))
    for _ in range(prof_steps):
        step()
    torch.cuda.synchronize(dev)
    prof = ctx.profile_read()
    ctx.profile_enable(False)
    kern = {n: {"avg_ms": ms / max(1, cnt), "launches": cnt, "total_ms": ms} for n, (ms, cnt) in prof.items()}
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    ceil = hbm_ceilings(dev.index) if rank == 0 else None
    mix, mix_src = isa_mix()
    rooflines = {n: kernel_roofline(n, kern[n], k, B, prof_steps, ncu, ceil, mix) for n in kern}
    dom = max(kern, key=lambda n: kern[n]["total_ms"])
    roofline = dict(rooflines[dom], kernel=dom)
    path_gbs = block_bytes(k) * value / world / 1e9
    comp_per_s = block_compressions_engine(k) * value / world

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "blocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic (namespace-sorted random shares, SplitMix64 seed 0xC0FFEE+rank*B+b, {nd} distinct "
                f"squares per rank replicated to B)",
        "config": {"workload": f"k{k}_block_batch: da.ExtendShares+NewDataAvailabilityHeader on {B} independent "
                               f"k={k} blocks per GPU per step (configs[1] per block, batched as configs[2])",
                   "k": k, "blocks_per_gpu_per_step": B, "share_size": 512,
                   "parallelism": f"blocks x{world}" + (" (ranks share one device, gloo)" if shared else "")},
        "roofline": roofline,
        "kernel_rooflines": {n: v for n, v in rooflines.items() if n != dom},
        "hbm_ceilings": ceil,
        "isa_mix_source": mix_src,
        "output_check": check,
        "ranks": ranks_rep,
        "path_hbm_gbs": round(path_gbs, 1),
        "sha256_compressions_per_s": comp_per_s,
        "kernels_ms": {n: round(v["avg_ms"], 4) for n, v in kern.items()},
    }
    gpu = {}
    # config C5's product path: one k=512 square over every device the ranks use (G = N; helper process, RCCL) and
    # on one device (G = 1); at N = 1 in this process
    if world > 1:
        torch.cuda.synchronize(dev)
        dist.barrier(group=cpu_group)
        if helper is not None:
            result["k512_split"] = helper.run()
        dist.barrier(group=cpu_group)
    elif not args.no_k512_split:
        try:
            result["k512_split"] = split_measure([dev.index])
        except Exception as e:  # reported, never the headline's exit code
            result["k512_split"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0 and world == 1 and not args.no_extras:
        del d_eds, d_roots, d_ods
        torch.cuda.empty_cache()
        result["c2_single_block"] = single_block_measure(ctx, dev)
        result["repair_c4"] = repair_measure(ctx)
        result["blob_commitments"], gpu["commitments"] = commitments_measure(ctx)
        result["host_buffers"] = host_path_measure(ctx, k)
        result["share_proof"] = proof_measure(ctx, k)
        result["k512_single"] = k512_measure(ctx, dev)
        result["device_square"] = square_measure(ctx)
        try:  # the per-axis seams (rsmt2d over cda.NewCodec + the GPU tree): VERDICT r05 next #1
            from cda import _native
            result["per_axis"] = per_axis_measure("cda", _native.LIB_PATH)
        except Exception as e:  # reported, never the headline's exit code
            result["per_axis"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cb = cpu_baseline(k, args.cpu_seconds, gpu)
        result["gpu_vs_cpu"] = gpu_vs_cpu(result, value)
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


# BASELINE.json's metric, verbatim (the driver matches the line against it)
METRIC = "ODS\u2192EDS+DAH blocks/sec at k=128 (1/8 GPU); achieved HBM GB/s"
DISTINCT_ODS = 16  # distinct synthetic squares per rank (tests/golden/make_bench_digests.py covers ranks 0..7)


def check_dahs(dah, k, B, rank, nd):
    """Every block's DAH of the timed steps against tests/golden/bench_digests.json (oracle DAHs of the bench's
    seeds); replicas of one square must agree too."""
    path = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
    want = json.load(open(path)).get(f"k{k}", {}) if os.path.exists(path) else {}
    import cda
    info = cda.build_info()
    if not info.startswith("release"):  # the loaded library says it is a diagnostic build: timing only, no result
        return {"blocks_checked_vs_golden": 0, "skipped": f"diagnostic library ({info}), not a result"}
    checked = 0
    for b in range(B):
        got = bytes(dah[b]).hex()
        if got != bytes(dah[b % nd]).hex():
            raise RuntimeError(f"block {b} DAH differs from its replica {b % nd}")
        exp = want.get(str(0xC0FFEE + rank * B + b % nd))
        if exp is not None:
            if got != exp:
                raise RuntimeError(f"block {b} DAH {got} != committed digest {exp}")
            checked += 1
    return {"blocks_checked_vs_golden": checked, "distinct_squares": nd, "source": "tests/golden/bench_digests.json"}


def kernel_roofline(name, kv, k, B, prof_steps, ncu, ceil, mix):
    """Roofline of one kernel of the bench step, by what bounds it (KERNEL_KIND): HBM kernels against 8 TB/s and the
    measured copy ceiling; VALU kernels against the wave64 issue peak, cycle-weighted by their static instruction mix
    (tools/isa_count.py) and, for the SHA-256 kernels, against the register-only SHA-256 ceiling."""
    HBM_PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md
    kind = KERNEL_KIND.get(name, "hbm")
    launches_per_step = max(1, kv["launches"] // prof_steps)
    avg_s = kv["avg_ms"] * 1e-3
    step_bytes = kernel_step_bytes(name, k, B)
    launch_bytes = step_bytes // launches_per_step if step_bytes else None
    gbs = launch_bytes / avg_s / 1e9 if launch_bytes else None
    pmc = pmc_counters(name, B)
    r = {"bound": "valu" if kind in ("valu", "latency") else "hbm", "avg_launch_ms": round(kv["avg_ms"], 4),
         "bytes_per_launch": launch_bytes, "traffic": pmc["hbm_bytes"] if pmc else None}
    hbm = {"achieved": round(gbs, 1) if gbs else None, "peak": HBM_PEAK, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK, 4) if gbs else None}
    if ceil and gbs:
        hbm["measured_copy_ceiling"] = ceil["copy_gbs"]
        hbm["frac_of_measured_copy"] = round(gbs / ceil["copy_gbs"], 4)
    if r["bound"] == "hbm":
        r.update(achieved=hbm["achieved"], peak=HBM_PEAK, unit="GB/s", frac=hbm["frac"])
        if "frac_of_measured_copy" in hbm:
            r["frac_of_measured_copy"] = hbm["frac_of_measured_copy"]
            r["measured_copy_ceiling_gbs"] = hbm["measured_copy_ceiling"]
        return r
    r["hbm"] = hbm
    peak = ncu * 4 * VALU_CLK / VALU_CYCLES_PER_WAVE_INSTR * 64 / 1e12
    if pmc and pmc.get("valu_insts"):
        achieved = pmc["valu_insts"] * 64 / avg_s / 1e12
        r.update(achieved=round(achieved, 2), peak=round(peak, 2), unit="TOPS", frac=round(achieved / peak, 4),
                 valu_wave_instr_per_launch=int(pmc["valu_insts"]), counters_source=pmc["source"],
                 peak_def=f"{ncu} CU x 4 SIMD x 2.4 GHz / 2 cycles per wave64 VALU instruction x 64 lanes")
        sym = {"leaf_hash": "leaf_hash_kernel", "nmt_levels_1": "nmt_levels_kernel", "nmt_levels": "nmt_levels_kernel",
               "dah": "dah_kernel"}.get(name)
        cyc = avg_cycles_per_valu(mix, sym) if sym else None
        if cyc:
            # issue cycles the kernel's instructions occupy, priced with the measured per-instruction costs (2 or 4
            # cycles) at the static mix's average, over the SIMD-cycles of the launch at 2.4 GHz
            r["valu_cycle_weighted"] = {
                "avg_cycles_per_instr": cyc,
                "busy": round(pmc["valu_insts"] * cyc / (ncu * 4 * VALU_CLK * avg_s), 4),
                "def": "SQ_INSTS_VALU x static-mix cycles per instruction / (SIMDs x 2.4 GHz x launch time)"}
    comp = kernel_compressions(name, k, B)
    if comp:
        g = comp / launches_per_step / avg_s / 1e9 if name != "leaf_hash" else comp / avg_s / 1e9
        r["sha256"] = {"achieved_gcomp_s": round(g, 2), "ceiling_gcomp_s": SHA_UBENCH_GCOMP_S,
                       "frac": round(g / SHA_UBENCH_GCOMP_S, 4),
                       "ceiling_def": "register-only SHA-256 microbenchmark (profiles/r02_sha_ubench.txt)"}
    return r


def gpu_vs_cpu(result, value):
    cb = result["cpu_baseline"]
    out = {"throughput_measured_best": round(value / cb["value"], 1),
           "throughput_full_host_linear_extrapolation": round(value / cb["full_host_linear_extrapolation"]["value"], 1)}
    lat = cb.get("single_block_ms", {})
    if lat:
        best_cpu = min(lat.values())
        out["single_block_cpu_best_ms"] = best_cpu
        if "c2_single_block" in result:
            out["single_block_device_resident"] = round(best_cpu / result["c2_single_block"]["ms"], 1)
        hb = result.get("host_buffers", {}).get("one_block_latency_ms", {})
        if hb.get("with_eds"):
            out["single_block_host_buffers_with_eds"] = round(best_cpu / hb["with_eds"], 1)
        fr = result.get("host_buffers", {}).get("one_block_fresh", {})
        for key in ("roots_only", "pooled_eds", "pooled_eds_inplace", "pooled_both", "with_eds"):
            if fr.get(key):
                out[f"single_block_{key}_median"] = round(best_cpu / fr[key]["ms_median"], 1)
    c4 = cb.get("repair_c4_ms", {})
    g4 = result.get("repair_c4", {})
    for case in ("random", "q0_only"):
        if case in c4 and case in g4:
            out[f"repair_{case}_host_buffers"] = round(c4[case] / g4[case]["ms_median"], 1)
            out[f"repair_{case}_device_resident"] = round(c4[case] / g4[case]["device_resident_ms_median"], 1)
    pa, pc = result.get("per_axis", {}), cb.get("per_axis", {})
    if "single" in pa and "single" in pc:  # CPU median / GPU median per shape (> 1: the GPU seam is faster)
        pv = {f"single_{op}": round(pc["single"][f"{op}_us"][1] / pa["single"][f"{op}_us"][1], 2)
              for op in ("encode", "decode", "root")}
        pv["extend_and_roots"] = round(pc["extend"]["total_ms"][1] / pa["extend"]["total_ms"][1], 2)
        if "extend_thread_per_axis" in pa and "extend_thread_per_axis" in pc:
            pv["extend_and_roots_thread_per_axis"] = round(pc["extend_thread_per_axis"]["total_ms"][1] /
                                                           pa["extend_thread_per_axis"]["total_ms"][1], 2)
        for case in ("random", "q0_only"):
            pv[f"repair_{case}"] = round(pc[f"repair_{case}"]["repair_ms"][1] / pa[f"repair_{case}"]["repair_ms"][1], 2)
        out["per_axis_cpu_over_gpu"] = pv
    k5 = cb.get("k512_ms", {})
    g5 = result.get("k512_single", {})
    if k5 and g5:
        out["k512_block_path"] = round(min(v for kk, v in k5.items() if kk != "note") / g5["ms_per_block"], 1)
        if g5.get("dah_golden") and cb.get("k512_dah") != g5["dah_golden"]:
            raise RuntimeError("CPU k=512 DAH differs from the committed digest")
    return out


def bench_split(args):
    """Config C5: one k x k square (k=512: 128 MiB ODS, 512 MiB EDS, GF(2^16)) split over the ranks."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev, backend, shared = dist_setup(world, local, False)
    import cda
    from cda import split
    ctx = cda.Context(dev.index)
    ops = split.DeviceOps(ctx)
    k = args.k
    (r0, r1), _ = split.plan(k, world, rank)
    ods = gen_ods(k, 0xC0FFEE).reshape(k, k, 512)
    rows = torch.from_numpy(np.ascontiguousarray(ods[r0:r1])).to(dev)
    for _ in range(args.warmup):
        split.extend_commit_split(ops, k, rows)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = split.extend_commit_split(ops, k, rows)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, backend, dev)
    value = args.steps / elapsed
    result = {
        "metric": f"ODS->EDS+DAH squares/sec, one k={k} square split over {world} GPU(s)",
        "value": round(value, 3), "unit": "squares/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (namespace-sorted random shares, SplitMix64 seed 0xC0FFEE)",
        "config": {"workload": f"split_k{k}: cda.split.extend_commit_split (rows over ranks, one all-to-all, "
                               f"bottom-row subtree fold)", "k": k, "parallelism": f"rows x{world}"},
        "dah": out.dah.hex(),
        "path_hbm_gbs": round(block_bytes(k) * value / world / 1e9, 1),
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
