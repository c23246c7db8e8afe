"""The per-axis drop-in seams on the GPU: rsmt2d.Codec Encode / Decode (cda_rs_encode / cda_rs_decode) and the wrapper
tree Root (cda_nmt_axis_root), as upstream rsmt2d calls them one axis at a time when appconsts.DefaultCodec is the GPU
codec (pkg/appconsts/global_consts.go:92, go/pkg_da/extend_rocm.go; pkg/wrapper/nmt_wrapper.go:73-124).

Concurrent calls are coalesced in libcda's axis queue (csrc/axisq.cpp); every result must be the oracle's bytes
whichever batch it rode in.  The whole-square shapes -- ComputeExtendedDataSquare and Repair as upstream rsmt2d runs
them (cda.rsmt2d.compute_extended_data_square_axes / repair_axes, and the C caller tests/abi_client/rsmt2d_axes) --
are checked against the oracle's fused extension and its sequential Repair."""
import os
import subprocess
import threading

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "abi_client", "rsmt2d_axes")


def _run_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def test_concurrent_mixed_shapes_match_oracle(ctx):
    """48 threads x 4 calls of encodes (FF8 and FF16, odd k, 64-B and 512-B shards), decodes and roots (full,
    ragged and odd leaf counts) at once: batches mix shapes; each result is checked against the oracle."""
    rng = np.random.default_rng(11)
    jobs = []
    for t in range(48):
        kind = t % 3
        if kind == 0:
            k = [1, 3, 16, 17, 64, 128, 129, 256][t % 8]
            L = 64 if t % 5 == 0 else 512
            data = rng.integers(0, 256, (k, L), dtype=np.uint8)
            jobs.append(("enc", data, O.leo_encode(data)))
        elif kind == 1:
            k = [2, 16, 32, 100, 128, 200][t % 6]
            data = rng.integers(0, 256, (k, 512), dtype=np.uint8)
            full = np.concatenate([data, O.leo_encode(data)])
            present = np.zeros(2 * k, np.uint8)
            present[rng.choice(2 * k, k + t % 3, replace=False)] = 1
            jobs.append(("dec", (full, present), full))
        else:
            ss = [4, 16, 64, 128][t % 4]
            n = [2 * ss, 2 * ss, 5, 2 * ss - 1][(t // 3) % 4]
            axis = int(rng.integers(0, 2 * ss))
            leaves = rng.integers(0, 256, (n, 512), dtype=np.uint8)
            leaves[:, :29] = 0
            leaves[:, 19:29] = np.sort(rng.integers(0, 256, (n, 10), dtype=np.uint8), axis=0)
            leaves = leaves[np.lexsort(leaves[:, :29].T[::-1])]
            rc, want, _ = O.nmt_axis_root(ss, axis, [bytes(x) for x in leaves])
            assert rc == 0
            jobs.append(("root", (ss, axis, leaves), want))
    results = [[None] * 4 for _ in jobs]

    def worker(j):
        def run():
            kind, inp, _ = jobs[j]
            for rep in range(4):
                if kind == "enc":
                    results[j][rep] = ctx.rs_encode(inp)
                elif kind == "dec":
                    full, present = inp
                    damaged = np.where(present[:, None] == 1, full, 0).astype(np.uint8)
                    results[j][rep] = ctx.rs_decode(damaged, present)
                else:
                    ss, axis, leaves = inp
                    results[j][rep] = ctx.nmt_axis_root(ss, axis, [bytes(x) for x in leaves])
        return run

    _run_threads([worker(j) for j in range(len(jobs))])
    for j, (kind, _, want) in enumerate(jobs):
        for rep in range(4):
            got = results[j][rep]
            if kind == "root":
                assert got == want, f"job {j} rep {rep}"
            else:
                assert np.array_equal(got, want), f"job {j} ({kind}) rep {rep}"


def test_oversized_requests_beside_small_ones(ctx):
    """Requests larger than one batch slot's share of the staging (csrc/axisq.cpp: 64 MiB over 4 slots) run alone in
    a slot grown to fit them, while small requests keep flowing through the other slots; every result is the
    oracle's."""
    rng = np.random.default_rng(23)
    big = [rng.integers(0, 256, (32, 512 * 1024), dtype=np.uint8) for _ in range(2)]  # 16 MiB in + 16 MiB out each
    big_want = [O.leo_encode(d) for d in big]
    small = [rng.integers(0, 256, (16, 512), dtype=np.uint8) for _ in range(24)]
    small_want = [O.leo_encode(d) for d in small]
    got_big, got_small = [None] * len(big), [[None] * 8 for _ in small]

    def run_big(i):
        def f():
            got_big[i] = ctx.rs_encode(big[i])
        return f

    def run_small(i):
        def f():
            for rep in range(8):
                got_small[i][rep] = ctx.rs_encode(small[i])
        return f

    _run_threads([run_big(i) for i in range(len(big))] + [run_small(i) for i in range(len(small))])
    for i in range(len(big)):
        assert np.array_equal(got_big[i], big_want[i]), f"big {i}"
    for i in range(len(small)):
        for rep in range(8):
            assert np.array_equal(got_small[i][rep], small_want[i]), f"small {i} rep {rep}"


def test_axis_root_edge_cases_match_oracle(ctx):
    """Tree shapes the wrapper allows: one leaf, odd and ragged counts, a push-order violation (the reference's error
    with the offending leaf), and a tree wider than one workgroup's LDS (the generic level path)."""
    import cda
    from cda import _native as N
    rng = np.random.default_rng(5)
    for ss, n, axis in ((1, 1, 0), (3, 5, 1), (8, 16, 9), (128, 255, 3), (1024, 2048, 5)):
        leaves = rng.integers(0, 256, (n, 512), dtype=np.uint8)
        leaves[:, :29] = 0
        leaves = [bytes(x) for x in leaves]
        rc, want, _ = O.nmt_axis_root(ss, axis, leaves)
        assert rc == 0
        assert ctx.nmt_axis_root(ss, axis, leaves) == want, (ss, n, axis)
    leaves = [bytes([0] * 28 + [9]) + bytes(483), bytes([0] * 28 + [3]) + bytes(483)] + [bytes(512)] * 6
    rc, _, el = O.nmt_axis_root(4, 0, leaves)
    assert rc == O.E_NS_ORDER and el == 1
    with pytest.raises(cda.CdaError) as ei:
        ctx.nmt_axis_root(4, 0, leaves)
    assert ei.value.code == N.E_NS_ORDER and ei.value.leaf == 1


@pytest.mark.parametrize("k", [8, 32])
def test_upstream_shaped_extension_matches_oracle(ctx, k):
    """ComputeExtendedDataSquare axis by axis (3k Encodes, 4k tree Roots from 8 threads) = the oracle's square."""
    from cda import rsmt2d
    ods = O.gen_ods(k, 0x5EED + k)
    sq = rsmt2d.compute_extended_data_square_axes([bytes(r) for r in ods], rsmt2d.LeoRSCodec(ctx), workers=8)
    rc, eds, rr, cr, dah = O.extend_commit(ods)
    assert rc == 0
    assert np.array_equal(sq.cells, eds)
    assert [bytes(r) for r in rr] == sq.row_roots() and [bytes(c) for c in cr] == sq.col_roots()


@pytest.mark.parametrize("k,survive", [(8, 0.5), (16, 0.6)])
def test_upstream_shaped_repair_matches_oracle(ctx, k, survive):
    """Repair axis by axis (sanity check in parallel, crossword of Decode + Roots sequentially) restores the square
    the oracle restores; a square the oracle cannot repair is unrepairable here too."""
    from cda import rsmt2d
    ods = O.gen_ods(k, 0xAB + k)
    rc, eds, rr, cr, _ = O.extend_commit(ods)
    w = 2 * k
    rng = np.random.default_rng(k)
    for frac in (survive, 0.2):
        present = (rng.random(w * w) < frac).astype(np.uint8)
        orc, oeds, opres, _, _ = O.repair(np.where(present[:, None] == 1, eds, 0), present, rr, cr)
        sq = rsmt2d.import_extended_data_square([bytes(eds[i]) if present[i] else None for i in range(w * w)],
                                                rsmt2d.LeoRSCodec(ctx))
        if orc == 0:
            rsmt2d.repair_axes(sq, rr, cr)
            assert np.array_equal(sq.cells, eds)
        else:
            assert orc == O.E_UNREPAIRABLE
            with pytest.raises(rsmt2d.ErrUnrepairableDataSquare):
                rsmt2d.repair_axes(sq, rr, cr)
            assert np.array_equal(sq.present, opres)


def test_upstream_shaped_repair_byzantine_matches_oracle(ctx):
    """A corrupted present cell: the same ErrByzantineData axis / index as the oracle's sequential Repair, and as
    the batched cda_repair."""
    from cda import rsmt2d
    k = 8
    w = 2 * k
    ods = O.gen_ods(k, 0xB12)
    rc, eds, rr, cr, _ = O.extend_commit(ods)
    rng = np.random.default_rng(3)
    present = (rng.random(w * w) < 0.6).astype(np.uint8)
    bad = eds.copy()
    r, c = [(r, c) for r in range(w) for c in range(w) if present[r * w + c]][5]
    bad[r * w + c, 100] ^= 0x5A
    orc, _, _, oax, oidx = O.repair(np.where(present[:, None] == 1, bad, 0), present, rr, cr)
    assert orc == O.E_BYZANTINE
    sq = rsmt2d.import_extended_data_square([bytes(bad[i]) if present[i] else None for i in range(w * w)],
                                            rsmt2d.LeoRSCodec(ctx))
    with pytest.raises(rsmt2d.ErrByzantineData) as ei:
        rsmt2d.repair_axes(sq, rr, cr)
    assert (ei.value.axis, ei.value.index) == (oax, oidx)
    grc, _, _, err = ctx.repair_status(np.where(present[:, None] == 1, bad, 0), present, rr, cr)
    assert grc == O.E_BYZANTINE and (err.axis, err.index) == (oax, oidx)


def test_rsmt2d_axes_driver_on_gpu(tmp_path):
    """The C caller (tests/abi_client/rsmt2d_axes: rsmt2d's fan-out over OS threads, pageable buffers, the cgo
    call shapes) over libcda: its extension is the oracle's square and its Repair restores it."""
    from cda import _native
    k, w = 32, 64
    ods = O.gen_ods(k, 0xD21)
    (tmp_path / "ods.bin").write_bytes(ods.tobytes())
    run = lambda *a: subprocess.run([DRIVER, "cda", _native.LIB_PATH] + [str(x) for x in a], capture_output=True,  # noqa: E731
                                    text=True, timeout=120)
    p = run("extend", k, 16, 2, tmp_path / "ods.bin", tmp_path)
    assert p.returncode == 0, p.stderr
    rc, eds, rr, cr, _ = O.extend_commit(ods)
    assert np.array_equal(np.fromfile(tmp_path / "eds.bin", np.uint8).reshape(w * w, 512), eds)
    assert np.array_equal(np.fromfile(tmp_path / "row_roots.bin", np.uint8).reshape(w, 90), rr)
    assert np.array_equal(np.fromfile(tmp_path / "col_roots.bin", np.uint8).reshape(w, 90), cr)
    eds.tofile(tmp_path / "full.bin")
    np.concatenate([rr, cr]).tofile(tmp_path / "roots.bin")
    pres = (np.random.default_rng(1).random(w * w) < 0.5).astype(np.uint8)
    pres.tofile(tmp_path / "pres.bin")
    p = run("repair", k, 8, 1, tmp_path / "full.bin", tmp_path / "pres.bin", tmp_path / "roots.bin", tmp_path)
    assert p.returncode == 0, p.stderr
    assert '"rc": 0' in p.stdout
    assert np.array_equal(np.fromfile(tmp_path / "repaired.bin", np.uint8).reshape(w * w, 512), eds)
    p = run("single", k, 5, tmp_path / "ods.bin")
    assert p.returncode == 0, p.stderr
