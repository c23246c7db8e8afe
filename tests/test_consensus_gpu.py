"""The one-block host-buffer path (csrc/consensus.cpp): cda_extend_commit / cda_extend_commit_batch with one block,
as PrepareProposal / ProcessProposal call da.ExtendShares (app/prepare_proposal.go:65-93,
app/process_proposal.go:137-151).  The input goes up in row bands (or one copy for roots only), Q0 is copied host to
host by a copy pool, Q1 and the bottom half come back while the device hashes, and the output form follows the
caller's buffer (pinned / written before / fresh and untouched).  Every case is bit-exact against the oracle, and
against the serial form (a context opened with CDA_CONSENSUS=0) for the error reports.  The A/B switches exist only
in the test-hooks build (cda/libcda_hooks.so, same sources), so the forms below open their contexts on it; the release
library always takes the default form (test_one_block_fresh_buffers, test_one_block_registered_caller_buffers)."""
import threading

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def serial_ctx():
    import os

    import cda
    from cda import _native as N
    old = os.environ.get("CDA_CONSENSUS")
    os.environ["CDA_CONSENSUS"] = "0"
    try:
        c = cda.Context(0, lib_path=N.HOOKS_LIB_PATH)
    finally:
        if old is None:
            del os.environ["CDA_CONSENSUS"]
        else:
            os.environ["CDA_CONSENSUS"] = old
    yield c
    c.close()


def _check(ods, eds, rr, cr, dah, want_eds=True):
    rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
    assert rc == 0
    if want_eds:
        assert np.array_equal(eds.reshape(eds_o.shape), eds_o), "EDS bytes differ"
    assert np.array_equal(rr, rr_o) and np.array_equal(cr, cr_o), "roots differ"
    assert bytes(dah) == dah_o


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128, 256])
@pytest.mark.parametrize("want_eds", [True, False])
def test_one_block_fresh_buffers(ctx, k, want_eds):
    """cda_extend_commit with a fresh, never-touched EDS buffer (np.empty, as go/cda/extend.go allocates one)."""
    ods = O.gen_ods(k, 0xC0DE + k)
    eds, rr, cr, dah = ctx.extend_commit(ods.copy(), want_eds=want_eds)
    _check(ods, eds, rr, cr, dah, want_eds)


@pytest.mark.parametrize("cons_in,cons_out", [("1", "0"), ("2", "0"), ("1", "2"), ("2", "2")])
@pytest.mark.parametrize("stg", [None, "0", "3"])
@pytest.mark.parametrize("huge", [None, "1"])
def test_one_block_forms(monkeypatch, cons_in, cons_out, stg, huge):
    """Every input form (CDA_CONS_IN: four bands / one copy) with every pageable output form (CDA_CONS_OUT=0: chosen
    by residency -- fresh buffers are touched by the pool and sent in pieces; 2: the written-buffer form forced, so
    the runtime faults a fresh buffer in itself), bottom-half split (CDA_CONS_STG: default half staged through the
    pinned slab, 0 = all pageable, 3 MiB) and the opt-in huge-page hint (CDA_HUGE_PAGES), fresh and written output
    buffers, k = 16 and 128.  The knobs are read once at cda_init, so each form gets its own context."""
    import cda
    from cda import _native as N
    monkeypatch.setenv("CDA_CONS_IN", cons_in)
    monkeypatch.setenv("CDA_CONS_OUT", cons_out)
    if stg is not None:
        monkeypatch.setenv("CDA_CONS_STG", stg)
    if huge is not None:
        monkeypatch.setenv("CDA_HUGE_PAGES", huge)
    c = cda.Context(0, lib_path=N.HOOKS_LIB_PATH)
    try:
        for k in (16, 128):
            ods = O.gen_ods(k, 0xF0F0 + k)
            for buf in ("fresh", "written"):
                out = (np.empty((1, 4 * k * k, 512), np.uint8) if buf == "fresh"
                       else np.full((1, 4 * k * k, 512), 0x3C, np.uint8))
                eds, rr, cr, dah = c.extend_commit_batch(ods[None].copy(), eds_out=out)
                _check(ods, out[0], rr[0], cr[0], dah[0])
                _, rr2, cr2, dah2 = c.extend_commit_batch(ods[None].copy(), want_eds=False)
                assert np.array_equal(rr2, rr) and np.array_equal(cr2, cr) and bytes(dah2[0]) == bytes(dah[0])
    finally:
        c.close()


def test_one_block_registered_caller_buffers(ctx):
    """Caller memory page-locked once with cda_host_register and reused (go/cda's buffer pools): the shares and the
    EDS buffer take the direct DMA path, several calls in a row, every result exact; unregistered afterwards."""
    k = 128
    ods_buf = np.empty((1, k * k, 512), np.uint8)
    eds_buf = np.full((1, 4 * k * k, 512), 0x77, np.uint8)
    ctx.host_register(ods_buf)
    ctx.host_register(eds_buf)
    try:
        for seed in (0x301, 0x302, 0x303):
            ods = O.gen_ods(k, seed)
            ods_buf[0] = ods
            _, rr, cr, dah = ctx.extend_commit_batch(ods_buf, eds_out=eds_buf)
            _check(ods, eds_buf[0], rr[0], cr[0], dah[0])
            _, rr2, cr2, dah2 = ctx.extend_commit_batch(ods_buf, want_eds=False)
            assert bytes(dah2[0]) == bytes(dah[0])
    finally:
        ctx.host_unregister(ods_buf)
        ctx.host_unregister(eds_buf)


def test_set_option_validates(ctx):
    import cda
    from cda import _native as N
    ctx.set_option(N.OPT_HUGE_PAGES, 1)
    ctx.set_option(N.OPT_HUGE_PAGES, 0)
    with pytest.raises(cda.CdaError):
        ctx.set_option(12345, 1)


@pytest.mark.parametrize("k", [64, 128])
def test_one_block_output_fully_overwritten(ctx, k):
    """A reused output buffer full of other bytes: every byte of the EDS is written (Q0 by the host copy, Q1 and the
    bottom half from the device)."""
    ods = O.gen_ods(k, 0x5EED + k)
    out = np.full((1, 4 * k * k, 512), 0xAB, np.uint8)
    eds, rr, cr, dah = ctx.extend_commit_batch(ods[None], eds_out=out)
    _check(ods, out[0], rr[0], cr[0], dah[0])


@pytest.mark.parametrize("pin_in,pin_out", [(True, True), (True, False), (False, True)])
def test_one_block_pinned_caller_buffers(ctx, pin_in, pin_out):
    """Pinned caller memory (cda_host_alloc) takes the direct DMA, for the input, the output or both."""
    k = 128
    ods = O.gen_ods(k, 0x91 + 2 * pin_in + pin_out)
    bufs = []
    src = ods[None]
    if pin_in:
        p = ctx.pinned((1, k * k, 512))
        p.array[:] = src
        src = p.array
        bufs.append(p)
    out = None
    if pin_out:
        q = ctx.pinned((1, 4 * k * k, 512))
        q.array[:] = 0x5A
        out = q.array
        bufs.append(q)
    try:
        eds, rr, cr, dah = ctx.extend_commit_batch(src, eds_out=out)
        _check(ods, eds[0], rr[0], cr[0], dah[0])
    finally:
        for b in bufs:
            b.free()


def test_one_block_sizes_interleaved(ctx):
    """Growing and shrinking k between calls (pinned slabs grow; smaller calls reuse them), with and without the
    EDS: every call exact."""
    for k, want in ((16, True), (256, False), (8, True), (256, True), (128, False), (32, True), (128, True)):
        ods = O.gen_ods(k, 0x1234 + k + want)
        eds, rr, cr, dah = ctx.extend_commit(ods, want_eds=want)
        _check(ods, eds, rr, cr, dah, want)


@pytest.mark.parametrize("k,swap,axis", [(128, (130, 131), 0), (64, None, 1), (8, (3, 5), 0)])
def test_one_block_push_order_errors_match_serial(ctx, serial_ctx, k, swap, axis):
    """Namespace push-order errors come back with the same axis / index / leaf as the serial form."""
    import cda
    ods = O.gen_ods(k, 0x77 + k).copy()
    if swap is not None:
        ods[list(swap)] = ods[list(swap[::-1])]
    else:  # rows stay sorted, column 5 decreases between rows 9 and 10
        sq = ods.reshape(k, k, 512)
        sq[10, :, 19:29] = 0
        sq[10, :, 29:] = 0
        ods = np.sort(sq.view("S512").reshape(k, k), axis=1).view(np.uint8).reshape(k * k, 512)
    errs = []
    for c in (ctx, serial_ctx):
        with pytest.raises(cda.CdaError) as ei:
            c.extend_commit(ods)
        e = ei.value
        errs.append((e.code, e.axis, e.index, e.leaf))
    assert errs[0] == errs[1] and errs[0][0] == -5 and errs[0][1] == axis


def test_one_block_matches_serial_form(ctx, serial_ctx):
    k = 128
    ods = O.gen_ods(k, 0xABCD)
    a = ctx.extend_commit(ods)
    b = serial_ctx.extend_commit(ods)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]


def test_one_block_concurrent_callers(ctx):
    """Several host threads on one context (the ctx lock serialises them; the copy pool is per context)."""
    k = 64
    odss = [O.gen_ods(k, 0x4000 + i) for i in range(6)]
    want = [O.extend_commit(o)[4] for o in odss]
    got = [None] * len(odss)

    def run(i):
        for _ in range(3):
            got[i] = ctx.extend_commit(odss[i])[3]

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(odss))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert got == want


def test_one_block_copy_pool_fault_is_a_return_code(monkeypatch):
    """The copy pool's threads cannot start: CDA_E_INTERNAL, and the next call on the context works."""
    import cda
    from cda import _native as N
    c = cda.Context(0, lib_path=N.HOOKS_LIB_PATH)  # failure injection: the test-hooks build only
    try:
        ods = O.gen_ods(32, 9)
        monkeypatch.setenv("CDA_FAULT_INJECT", "thread")
        with pytest.raises(cda.CdaError) as ei:
            c.extend_commit(ods)
        assert ei.value.code == N.E_INTERNAL
        monkeypatch.delenv("CDA_FAULT_INJECT")
        eds, rr, cr, dah = c.extend_commit(ods)
        _check(ods, eds, rr, cr, dah)
    finally:
        c.close()


def _inplace_buffer(ods, k, fill=None):
    """A (4k^2, 512) EDS buffer with the ODS in Q0 (what go/cda's ExtendShares flattens into its pooled slab)."""
    eds = np.empty((4 * k * k, 512), np.uint8) if fill is None else np.full((4 * k * k, 512), fill, np.uint8)
    eds.reshape(2 * k, 2 * k, 512)[:k, :k] = ods.reshape(k, k, 512)
    return eds


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128, 256, 512])
def test_extend_commit_eds_in_place(ctx, k):
    """cda_extend_commit_eds: Q0 of the caller's buffer holds the ODS; Q1..Q3 written around it, bit-exact with the
    oracle (k <= 256: the consensus path without its Q0 copy, 2-D input DMAs; k = 512: the gathered fallback).  The
    rest of the buffer starts as other bytes, so every byte outside Q0 must be written."""
    ods = O.gen_ods(k, 0x1D0 + k)
    eds = _inplace_buffer(ods, k, fill=0xA5)
    rr, cr, dah = ctx.extend_commit_eds(eds)
    _check(ods, eds, rr, cr, dah)


@pytest.mark.parametrize("kind", ["registered", "pinned", "fresh_tail", "written"])
def test_extend_commit_eds_buffer_kinds(ctx, kind):
    """The in-place form on every kind of caller buffer at k = 128: registered once and reused (go/cda's EDS pool,
    several squares in a row), cda_host_alloc, a fresh buffer whose only written pages are Q0's, a written one."""
    k = 128
    seeds = (0x2A1, 0x2A2, 0x2A3)
    if kind == "registered":
        buf = np.full((4 * k * k, 512), 0x11, np.uint8)
        ctx.host_register(buf)
        try:
            for seed in seeds:
                ods = O.gen_ods(k, seed)
                buf.reshape(2 * k, 2 * k, 512)[:k, :k] = ods.reshape(k, k, 512)
                rr, cr, dah = ctx.extend_commit_eds(buf)
                _check(ods, buf, rr, cr, dah)
        finally:
            ctx.host_unregister(buf)
        return
    if kind == "pinned":
        p = ctx.pinned((4 * k * k, 512))
        try:
            ods = O.gen_ods(k, seeds[0])
            p.array[:] = 0x22
            p.array.reshape(2 * k, 2 * k, 512)[:k, :k] = ods.reshape(k, k, 512)
            rr, cr, dah = ctx.extend_commit_eds(p.array)
            _check(ods, p.array, rr, cr, dah)
        finally:
            p.free()
        return
    ods = O.gen_ods(k, seeds[1])
    eds = _inplace_buffer(ods, k, fill=None if kind == "fresh_tail" else 0x33)
    rr, cr, dah = ctx.extend_commit_eds(eds)
    _check(ods, eds, rr, cr, dah)


def test_extend_commit_eds_matches_extend_commit(ctx, serial_ctx):
    """Same roots and DAH as cda_extend_commit on the same shares, on the consensus context and on a serial one (the
    gathered fallback), and the same namespace push-order error."""
    import cda
    k = 64
    ods = O.gen_ods(k, 0x3B3)
    want = ctx.extend_commit(ods)
    for c in (ctx, serial_ctx):
        eds = _inplace_buffer(ods, k)
        rr, cr, dah = c.extend_commit_eds(eds)
        assert np.array_equal(eds, want[0].reshape(eds.shape))
        assert np.array_equal(rr, want[1]) and np.array_equal(cr, want[2]) and bytes(dah) == bytes(want[3])
    bad = ods.copy()
    bad[[5, 6]] = bad[[6, 5]]
    errs = []
    for c in (ctx, serial_ctx):
        with pytest.raises(cda.CdaError) as ei:
            c.extend_commit_eds(_inplace_buffer(bad, k))
        errs.append((ei.value.code, ei.value.axis, ei.value.index, ei.value.leaf))
    with pytest.raises(cda.CdaError) as ei:
        ctx.extend_commit(bad)
    assert errs[0] == errs[1] == (ei.value.code, ei.value.axis, ei.value.index, ei.value.leaf)


def test_extend_commit_eds_rejects_bad_shapes(ctx):
    with pytest.raises(ValueError):
        ctx.extend_commit_eds(np.zeros((3 * 3, 512), np.uint8))
    with pytest.raises(ValueError):
        ctx.extend_commit_eds(np.zeros((16, 256), np.uint8))
    with pytest.raises(ValueError):
        ctx.extend_commit_eds(np.zeros((16, 512), np.int8))
    with pytest.raises(ValueError):
        ctx.extend_commit_eds(np.zeros((16, 1024), np.uint8)[:, ::2])


def test_extend_commit_eds_concurrent_callers(ctx):
    """In-place calls from several host threads on one context, mixed with roots-only calls (the consensus handlers
    and ExtendBlock of one node): every square and DAH exact."""
    k = 64
    odss = [O.gen_ods(k, 0x5100 + i) for i in range(4)]
    want = [O.extend_commit(o) for o in odss]
    errs = []

    def run(i):
        try:
            for it in range(3):
                if (i + it) % 2:
                    eds = _inplace_buffer(odss[i], k)
                    rr, cr, dah = ctx.extend_commit_eds(eds)
                    assert np.array_equal(eds, want[i][1].reshape(eds.shape)) and dah == want[i][4]
                else:
                    assert ctx.extend_commit(odss[i], want_eds=False)[3] == want[i][4]
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errs.append(e)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(odss))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs


def test_extend_commit_eds_copy_pool_fault_is_a_return_code(monkeypatch):
    """In place with the copy pool's threads failing to start (test-hooks build): CDA_E_INTERNAL, the buffer's Q0 is
    untouched, and the next in-place call on the context is exact."""
    import cda
    from cda import _native as N
    c = cda.Context(0, lib_path=N.HOOKS_LIB_PATH)
    try:
        k = 32
        ods = O.gen_ods(k, 0x5200)
        eds = _inplace_buffer(ods, k, fill=0x44)
        monkeypatch.setenv("CDA_FAULT_INJECT", "thread")
        with pytest.raises(cda.CdaError) as ei:
            c.extend_commit_eds(eds)
        assert ei.value.code == N.E_INTERNAL
        assert np.array_equal(eds.reshape(2 * k, 2 * k, 512)[:k, :k], ods.reshape(k, k, 512))
        monkeypatch.delenv("CDA_FAULT_INJECT")
        rr, cr, dah = c.extend_commit_eds(eds)
        _check(ods, eds, rr, cr, dah)
    finally:
        c.close()
