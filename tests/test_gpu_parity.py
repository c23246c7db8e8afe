"""GPU parity: libcda (HIP, gfx950) vs the CPU oracle and the reference's KATs.

Every comparison is bit-exact (integer / byte / GF arithmetic; no tolerance).
"""
import numpy as np
import pytest

import kat
import oracle_lib as O

pytestmark = pytest.mark.gpu


# ---- reference known answers through the product path ----------------------------------
def test_min_data_availability_header(ctx):
    from cda import da
    dah = da.min_data_availability_header()
    assert dah.hash() == kat.MIN_DAH
    dah.validate_basic()


@pytest.mark.parametrize("k,expected", [(2, kat.TYPICAL_K2), (128, kat.MAX_K128)])
def test_new_data_availability_header(ctx, k, expected):
    from cda import da
    shares = [bytes(s) for s in kat.generate_shares(k * k)]
    eds = da.extend_shares(shares)
    got = da.new_data_availability_header(eds)
    assert len(got.row_roots) == 2 * k and len(got.column_roots) == 2 * k
    assert got.hash() == expected


@pytest.mark.parametrize("k,expected", [(1, None), (2, kat.TYPICAL_K2), (128, kat.MAX_K128)])
def test_dah_from_shares_roots_only(ctx, k, expected):
    """go/patches/0004's NewDataAvailabilityHeaderFromShares (mirror: da.new_data_availability_header_from_shares):
    the same roots and hash as NewDataAvailabilityHeader(ExtendShares(s)), which itself now extends in place."""
    from cda import da
    shares = da.min_shares() if k == 1 else [bytes(s) for s in kat.generate_shares(k * k)]
    full = da.new_data_availability_header(da.extend_shares(shares))
    fast = da.new_data_availability_header_from_shares(shares, ctx=ctx)
    assert fast.row_roots == full.row_roots and fast.column_roots == full.column_roots
    assert fast.hash() == full.hash() == (expected if expected is not None else kat.MIN_DAH)
    fast.validate_basic()


@pytest.mark.parametrize("count", [5, 8, 129 * 129])
def test_dah_from_shares_errors(ctx, count):
    from cda import da
    with pytest.raises(Exception):
        da.new_data_availability_header_from_shares([bytes(s) for s in kat.generate_shares(count)], ctx=ctx)
    with pytest.raises(Exception):
        da.extend_shares([bytes(s) for s in kat.generate_shares(count)])


def test_dah_validate_basic_cases(ctx):
    """Test_DAHValidateBasic (pkg/da/data_availability_header_test.go:135-215): min and max headers pass; too many
    roots, too few roots, a wrong hash and unequal root counts fail with the reference's messages."""
    from cda import appconsts, da
    max_size = appconsts.DEFAULT_SQUARE_SIZE_UPPER_BOUND ** 2
    big = da.new_data_availability_header(da.extend_shares([bytes(s) for s in kat.generate_shares(max_size)]))
    too_big = da.DataAvailabilityHeader(big.row_roots + [b"\x00"] * (max_size - len(big.row_roots)) + [b"\x01" * 32],
                                        big.column_roots + [b"\x00"] * (max_size - len(big.column_roots)) +
                                        [b"\x01" * 32], ctx=ctx)
    too_small = da.DataAvailabilityHeader([b"\x02" * 32], [b"\x02" * 32], ctx=ctx)
    bad_hash = da.min_data_availability_header()
    bad_hash._hash = bytes([1, 2, 3, 4])
    mismatch = da.min_data_availability_header()
    mismatch.column_roots.append(b"\x02" * 32)
    da.min_data_availability_header().validate_basic()
    big.validate_basic()
    for dah, msg in ((too_big, "maximum valid DataAvailabilityHeader has at most"),
                     (too_small, "minimum valid DataAvailabilityHeader has at least"),
                     (bad_hash, "wrong hash"),
                     (mismatch, "unequal number of row and column roots")):
        with pytest.raises(da.DAError) as ei:
            dah.validate_basic()
        assert msg in str(ei.value), (msg, str(ei.value))


def test_dah_square_size(ctx):
    """TestSquareSize (data_availability_header_test.go:217-240): 1 for the min header, the upper bound for the max."""
    from cda import appconsts, da
    assert da.min_data_availability_header().square_size() == 1
    n = appconsts.DEFAULT_SQUARE_SIZE_UPPER_BOUND
    big = da.new_data_availability_header(da.extend_shares([bytes(s) for s in kat.generate_shares(n * n)]))
    assert big.square_size() == n


def test_nil_dah_hash(ctx):
    from cda import da
    assert da.DataAvailabilityHeader().hash() == kat.EMPTY_HASH


@pytest.mark.parametrize("count", [5, 129 * 129])
def test_extend_shares_errors(ctx, count):
    from cda import da
    with pytest.raises(Exception):
        da.extend_shares([bytes(s) for s in kat.generate_shares(count)])


# ---- seeded random squares vs the oracle ---------------------------------------------------
@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128, 256, 512])
def test_extend_commit_matches_oracle(ctx, k):
    ods = O.gen_ods(k, 0xC0FFEE + k)
    rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
    assert rc == 0
    eds, rr, cr, dah = ctx.extend_commit(ods)
    assert np.array_equal(eds, eds_o), "EDS bytes differ"
    assert np.array_equal(rr, rr_o), "row roots differ"
    assert np.array_equal(cr, cr_o), "col roots differ"
    assert dah == dah_o


def test_batch_matches_single(ctx):
    k, nb = 32, 6
    ods = np.stack([O.gen_ods(k, 0xC0FFEE + b) for b in range(nb)])
    eds, rr, cr, dah = ctx.extend_commit_batch(ods)
    for b in range(nb):
        rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods[b])
        assert np.array_equal(eds[b], eds_o) and np.array_equal(rr[b], rr_o) and np.array_equal(cr[b], cr_o)
        assert dah[b].tobytes() == dah_o


def test_mainnet_block_408_data_hash(ctx):
    """Real block (reference fixture x/blob/test/testdata/block_response.json): GPU DAH == header data_hash."""
    import os
    from cda import da
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mainnet_h408.npz"))
    ods, want = z["ods"], z["data_hash"].tobytes()
    eds, rr, cr, dah = ctx.extend_commit(ods)
    assert dah == want
    rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
    assert np.array_equal(eds, eds_o) and np.array_equal(rr, rr_o) and np.array_equal(cr, cr_o)
    h = da.new_data_availability_header(da.extend_shares([bytes(s) for s in ods]))
    assert h.hash() == want
    # Repair from Q0 only reproduces the block's EDS
    w = 64
    present = np.zeros(w * w, np.uint8)
    present.reshape(w, w)[:32, :32] = 1
    damaged = eds.copy()
    damaged[present == 0] = 0
    out, pres = ctx.repair(damaged, present, rr, cr)
    assert np.array_equal(out, eds) and pres.all()


def test_batch_k128(ctx):
    """k=128 batch of 7 blocks through the host-buffer path: every block bit-exact."""
    k, nb = 128, 7
    ods = np.stack([O.gen_ods(k, 0xBEEF + b) for b in range(nb)])
    eds, rr, cr, dah = ctx.extend_commit_batch(ods)
    for b in range(nb):
        rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods[b])
        assert np.array_equal(eds[b], eds_o), f"block {b} EDS differs"
        assert np.array_equal(rr[b], rr_o) and np.array_equal(cr[b], cr_o), f"block {b} roots differ"
        assert dah[b].tobytes() == dah_o


@pytest.mark.parametrize("k,nb,want_eds", [(8, 2, True), (32, 5, True), (32, 33, False), (64, 9, True),
                                           (128, 2, True), (128, 13, True), (128, 13, False)])
def test_batch_host_pipeline(ctx, k, nb, want_eds):
    """cda_extend_commit_batch streams host buffers in chunks over three streams (H2D / compute / D2H, 3 device
    slots): every block's EDS, roots and DAH still equal the oracle's, for chunk counts below, at and above the
    slot count and a ragged last chunk."""
    ods = np.stack([O.gen_ods(k, 0xD00D + 7 * b + k) for b in range(nb)])
    eds, rr, cr, dah = ctx.extend_commit_batch(ods, want_eds=want_eds)
    for b in range(nb):
        rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods[b])
        if want_eds:
            assert np.array_equal(eds[b], eds_o), f"block {b} EDS differs"
        assert np.array_equal(rr[b], rr_o) and np.array_equal(cr[b], cr_o), f"block {b} roots differ"
        assert dah[b].tobytes() == dah_o


def test_batch_host_pipeline_pinned_buffers(ctx):
    """The same path with pinned host buffers (cda_host_alloc), as a cgo caller can allocate them."""
    k, nb = 64, 10
    src = np.stack([O.gen_ods(k, 0xAB + b) for b in range(nb)])
    pin_in = ctx.pinned(src.shape)
    pin_out = ctx.pinned((nb, 4 * k * k, 512))
    pin_in.array[:] = src
    eds, rr, cr, dah = ctx.extend_commit_batch(pin_in.array, eds_out=pin_out.array)
    for b in (0, nb // 2, nb - 1):
        rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(src[b])
        assert np.array_equal(eds[b], eds_o) and dah[b].tobytes() == dah_o
    pin_in.free()
    pin_out.free()


def test_batch_eds_out_is_validated(ctx):
    from cda import CdaError
    ods = np.stack([O.gen_ods(8, b) for b in range(2)])
    for bad in (np.empty((2, 256, 511), np.uint8), np.empty((2, 256, 512), np.int8),
                np.empty((2, 256, 1024), np.uint8)[:, :, ::2]):
        with pytest.raises(CdaError):
            ctx.extend_commit_batch(ods, eds_out=bad)


def test_multi_device_batch():
    """cda_multi over every visible device (device mask 0): contiguous block ranges per device, no collective;
    results equal the single-context batch.  On a one-GPU box this exercises the one-device path."""
    import cda
    m = cda.MultiContext(0)
    try:
        assert m.device_count >= 1
        k, nb = 32, 11
        ods = np.stack([O.gen_ods(k, 0x3A + b) for b in range(nb)])
        eds, rr, cr, dah = m.extend_commit_batch(ods)
        for b in range(nb):
            rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods[b])
            assert np.array_equal(eds[b], eds_o) and dah[b].tobytes() == dah_o
        ods[7, [1, 2]] = ods[7, [2, 1]]
        with pytest.raises(cda.CdaError) as ei:
            m.extend_commit_batch(ods, want_eds=False)
        assert (ei.value.code, ei.value.block) == (-5, 7)
    finally:
        m.close()


def test_batch_k128_push_error_block(ctx):
    """A push-order error in one block of a batch names that block, axis, index and leaf."""
    from cda import CdaError
    k, nb = 128, 5
    ods = np.stack([O.gen_ods(k, 0xFACE + b) for b in range(nb)])
    ods[3, [130, 131]] = ods[3, [131, 130]]  # row 1 leaves 2 and 3 swapped
    with pytest.raises(CdaError) as ei:
        ctx.extend_commit_batch(ods)
    e = ei.value
    assert (e.code, e.block, e.axis, e.index, e.leaf) == (-5, 3, 0, 1, 3)


def test_random_bytes_not_sorted_rows_are_rejected(ctx):
    from cda import CdaError
    k = 8
    ods = O.gen_ods(k, 99)
    ods[[3, 5]] = ods[[5, 3]]  # row 0: leaf 3 > leaf 4 after the swap
    with pytest.raises(CdaError) as ei:
        ctx.extend_commit(ods)
    assert ei.value.code == -5 and ei.value.axis == 0 and ei.value.index == 0


def test_column_order_violation(ctx):
    from cda import CdaError
    k = 4
    ods = O.gen_ods(k, 98).reshape(k, k, 512).copy()
    # make column 2 decrease between rows 1 and 2 while keeping every row sorted
    ods[2, :, 19:29] = 0
    ods[2, :, 29:] = 0
    ods[3, :, 19:29] = 0
    rows_sorted = np.sort(ods.reshape(k * k, 512).view("S512").reshape(k, k), axis=1)
    ods = rows_sorted.view(np.uint8).reshape(k * k, 512)
    rc, *_ = O.extend_commit(ods)
    with pytest.raises(CdaError) as ei:
        ctx.extend_commit(ods)
    assert ei.value.code == -5


# ---- codec ---------------------------------------------------------------------------------
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 7, 8, 15, 16, 33, 64, 100, 127, 128])
@pytest.mark.parametrize("L", [64, 512, 1024])
def test_rs_encode_matches_oracle(ctx, k, L):
    rng = np.random.default_rng(k * 1000 + L)
    d = rng.integers(0, 256, (k, L), dtype=np.uint8)
    assert np.array_equal(ctx.rs_encode(d), O.leo_encode(d))


@pytest.mark.parametrize("k", [129, 200, 256, 300, 512, 1000, 1024, 2048])
@pytest.mark.parametrize("L", [64, 512])
def test_rs_encode_ff16_matches_oracle(ctx, k, L):
    """GF(2^16) Leopard (2k > 256): lo/hi byte element layout per 64-byte block."""
    rng = np.random.default_rng(k * 7 + L)
    d = rng.integers(0, 256, (k, L), dtype=np.uint8)
    assert np.array_equal(ctx.rs_encode(d), O.leo_encode(d))


def test_codec_interface(ctx):
    from cda.rsmt2d import LeoRSCodec
    c = LeoRSCodec(ctx)
    assert c.name() == "Leopard" and c.max_chunks() == 32768 * 32768
    data = [bytes([i]) * 512 for i in range(4)]
    par = c.encode(data)
    assert par == [bytes(p) for p in O.leo_encode(np.stack([np.frombuffer(d, np.uint8) for d in data]))]


# ---- trees ---------------------------------------------------------------------------------
@pytest.mark.parametrize("k,axis,n", [(8, 0, 16), (8, 3, 16), (8, 9, 16), (8, 0, 8), (8, 0, 5), (128, 0, 256),
                                      (4, 1, 1), (1, 0, 2)])
def test_axis_root_matches_oracle(ctx, k, axis, n):
    ods = O.gen_ods(max(k, 4), k + axis + n)
    leaves = [bytes(ods[i % len(ods)]) for i in range(n)]
    leaves[:min(n, k)] = sorted(leaves[:min(n, k)])
    rc, want, _ = O.nmt_axis_root(k, axis, leaves)
    assert rc == 0
    assert ctx.nmt_axis_root(k, axis, leaves) == want


def test_wrapper_tree_roots(ctx):
    from cda.wrapper import new_constructor
    k = 8
    rc, eds, rr, cr, _ = O.extend_commit(O.gen_ods(k, 5))
    eds = eds.reshape(2 * k, 2 * k, 512)
    ctor = new_constructor(k, ctx)
    for r in (0, 5, 8, 15):
        t = ctor(0, r)
        for c in range(2 * k):
            t.push(bytes(eds[r, c]))
        assert t.root() == bytes(rr[r])


def _erasured_data(k, seed, codec):
    """generateErasuredData (nmt_wrapper_test.go:139-149): k random namespaced shares, sorted, then Codec.Encode."""
    raw = [bytes(s) for s in O.gen_ods(k, seed)[:k]]
    raw.sort()
    return raw + codec.encode(raw)


@pytest.mark.parametrize("k", [8, 128])
def test_push_erasured_data(ctx, k):
    """TestPushErasuredNamespacedMerkleTree (nmt_wrapper_test.go:19-42): 2k pushes of data + parity succeed, and the
    root equals the oracle's axis root of the same leaves (axis 0: the first k leaves keep their namespaces)."""
    from cda.rsmt2d import LeoRSCodec
    from cda.wrapper import ErasuredNamespacedMerkleTree
    data = _erasured_data(k, 0x77 + k, LeoRSCodec(ctx))
    t = ErasuredNamespacedMerkleTree(k, 0, ctx)
    for d in data:
        t.push(d)
    rc, want, _ = O.nmt_axis_root(k, 0, data)
    assert rc == 0 and t.root() == want


def test_push_errors_with_erasured_data(ctx):
    """TestErasureNamespacedMerkleTreePushErrors (nmt_wrapper_test.go:91-128), k = 16: pushing the erasured data of
    k + 1 shares, the erasured data in reverse order, or a 1-byte share fails."""
    from cda.rsmt2d import LeoRSCodec
    from cda.wrapper import ErasuredNamespacedMerkleTree, PushError
    codec = LeoRSCodec(ctx)
    over = _erasured_data(17, 0x91, codec)
    rev = sorted(_erasured_data(16, 0x92, codec), reverse=True)
    for data in (over, rev, [b"\x01"]):
        t = ErasuredNamespacedMerkleTree(16, 0, ctx)
        with pytest.raises(PushError):
            for d in data:
                t.push(d)


def test_erasured_tree_prove_range(ctx):
    """TestErasuredNamespacedMerkleTree_ProveRange (nmt_wrapper_test.go:152-182): for square sizes 1..16, the
    single-share proofs of every leaf of a tree of codec-erasured data are non-empty and verify against the tree's
    (GPU) root, under the share's namespace for i < k and the parity namespace above."""
    from cda.appconsts import PARITY_SHARES_NAMESPACE
    from cda.rsmt2d import LeoRSCodec
    from cda.wrapper import ErasuredNamespacedMerkleTree
    codec = LeoRSCodec(ctx)
    for k in range(1, 17):
        data = _erasured_data(k, 0x600 + k, codec)
        t = ErasuredNamespacedMerkleTree(k, 0, ctx)
        for d in data:
            t.push(d)
        root = t.root()
        for i in range(len(data)):
            p = t.prove_range(i, i + 1)
            assert p.nodes, (k, i)
            ns = data[i][:29] if i < k else PARITY_SHARES_NAMESPACE
            assert p.verify_inclusion(ns, [data[i]], root), (k, i)


def test_empty_tree_root(ctx):
    from cda.wrapper import ErasuredNamespacedMerkleTree
    r1 = ErasuredNamespacedMerkleTree(1, 0, ctx).root()
    r2 = ErasuredNamespacedMerkleTree(2, 1, ctx).root()
    assert r1 == r2 and r1[58:] == kat.EMPTY_HASH


@pytest.mark.parametrize("n", [1, 2, 3, 4, 6, 7, 256, 1000])
def test_dah_hash_any_count(ctx, n):
    rng = np.random.default_rng(n)
    rr = rng.integers(0, 256, (n, 90), dtype=np.uint8)
    cr = rng.integers(0, 256, (n, 90), dtype=np.uint8)
    assert ctx.dah_hash(rr, cr) == O.dah_hash(rr, cr)


# ---- decode (rsmt2d LeoRSCodec.Decode) -------------------------------------------------------
@pytest.mark.parametrize("k", [1, 2, 3, 4, 8, 16, 33, 64, 128, 129, 256, 300, 512])
def test_rs_decode_matches_oracle(ctx, k):
    rng = np.random.default_rng(1000 + k)
    L = 512 if k <= 256 else 128
    d = rng.integers(0, 256, (k, L), dtype=np.uint8)
    full = np.concatenate([d, O.leo_encode(d)])
    for trial in range(3):
        nkeep = k + trial * (k // 3)
        pres = np.zeros(2 * k, np.uint8)
        pres[rng.choice(2 * k, min(nkeep, 2 * k), replace=False)] = 1
        damaged = np.where(pres[:, None] == 1, full, 0x5C).astype(np.uint8)
        got = ctx.rs_decode(damaged, pres)
        assert np.array_equal(got, full), f"trial {trial}"


def test_rs_decode_too_few(ctx):
    from cda import CdaError
    k = 8
    pres = np.zeros(16, np.uint8)
    pres[:7] = 1
    with pytest.raises(CdaError) as ei:
        ctx.rs_decode(np.zeros((16, 64), np.uint8), pres)
    assert ei.value.code == -6


def test_codec_decode_interface(ctx):
    from cda.rsmt2d import LeoRSCodec
    c = LeoRSCodec(ctx)
    data = [bytes([i * 3 + 1]) * 512 for i in range(4)]
    full = data + c.encode(data)
    shards = [s if i in (1, 4, 6, 7) else None for i, s in enumerate(full)]
    assert c.decode(shards) == full


# ---- Repair (rsmt2d ExtendedDataSquare.Repair) ----------------------------------------------
def _square(k, seed):
    rc, eds, rr, cr, dah = O.extend_commit(O.gen_ods(k, seed))
    assert rc == 0
    return eds, rr, cr


def _check_repair(ctx, eds, rr, cr, pres):
    from cda import CdaError
    damaged = np.where(pres[:, None] == 1, eds, 0xEE).astype(np.uint8)
    rc_o, eds_o, p_o, ax_o, ix_o = O.repair(damaged, pres, rr, cr)
    try:
        got, p_g = ctx.repair(damaged, pres, rr, cr)
        rc_g, ax_g, ix_g = 0, -1, -1
    except CdaError as e:
        rc_g, ax_g, ix_g = e.code, e.axis, e.index
        got, p_g = None, None
    assert rc_g == rc_o, (rc_g, rc_o)
    if rc_o == 0:
        assert np.array_equal(got, eds) and p_g.all()
    elif rc_o == O.E_BYZANTINE:
        assert (ax_g, ix_g) == (ax_o, ix_o)
    return rc_o


@pytest.mark.parametrize("k", [2, 4, 16, 32, 128])
def test_repair_q0_only(ctx, k):
    eds, rr, cr = _square(k, 300 + k)
    w = 2 * k
    pres = np.zeros((w, w), np.uint8)
    pres[:k, :k] = 1
    assert _check_repair(ctx, eds, rr, cr, pres.reshape(-1)) == 0


@pytest.mark.parametrize("k,frac", [(8, 0.5), (32, 0.5), (128, 0.5), (128, 0.6), (32, 0.3), (128, 0.25)])
def test_repair_random(ctx, k, frac):
    eds, rr, cr = _square(k, 400 + k)
    rng = np.random.default_rng(k)
    pres = (rng.random(4 * k * k) < frac).astype(np.uint8)
    _check_repair(ctx, eds, rr, cr, pres)


@pytest.mark.parametrize("k,frac", [(32, 0.3), (128, 0.2)])
def test_repair_sparse_upload_leaves_zeros_where_unrepaired(ctx, k, frac):
    """A square with <= 75 % of its cells present goes up as runs of present cells only (repair.cpp, packed
    upload): an unrepairable one comes back with the oracle's presence and present cells, and zeros in every cell
    still missing where the packed form was used, the caller's own bytes where the whole square went up -- never
    bytes of an earlier square left on the device."""
    eds, rr, cr = _square(k, 700 + k)
    rng = np.random.default_rng(k)
    pres = (rng.random(4 * k * k) < frac).astype(np.uint8)
    ctx.repair_status(eds.copy(), np.ones_like(pres), rr, cr)  # leave a whole square in the device buffer
    damaged = np.where(pres[:, None] == 1, eds, 0xEE).astype(np.uint8)
    rc_o, eds_o, p_o, _, _ = O.repair(damaged, pres, rr, cr)
    rc_g, eds_g, p_g, _ = ctx.repair_status(damaged, pres, rr, cr)
    assert rc_g == rc_o == O.E_UNREPAIRABLE
    assert np.array_equal(p_g, p_o)
    m = p_o.astype(bool)
    assert np.array_equal(eds_g[m], eds_o[m])
    left = eds_g[~m]
    assert np.all((left == 0) | (left == 0xEE))


def test_repair_ff16(ctx):
    k = 256
    eds, rr, cr = _square(k, 7)
    rng = np.random.default_rng(5)
    pres = (rng.random(4 * k * k) < 0.9).astype(np.uint8)
    assert _check_repair(ctx, eds, rr, cr, pres) == 0


def test_repair_byzantine_complete_row(ctx):
    k = 8
    eds, rr, cr = _square(k, 21)
    w = 2 * k
    bad = eds.copy()
    bad[3 * w + 12, 200] ^= 0x10  # parity cell of complete row 3
    pres = np.ones(w * w, np.uint8)
    pres[5 * w + 1] = 0
    _check_repair(ctx, bad, rr, cr, pres)


def test_repair_byzantine_during_crossword(ctx):
    k = 8
    eds, rr, cr = _square(k, 22)
    w = 2 * k
    rng = np.random.default_rng(3)
    pres = (rng.random(w * w) < 0.6).astype(np.uint8)
    # corrupt one present cell so that its row/col decode fails verification
    idx = int(np.flatnonzero(pres)[17])
    bad = eds.copy()
    bad[idx, 50] ^= 0xFF
    rc = _check_repair(ctx, bad, rr, cr, pres)
    assert rc in (O.E_BYZANTINE, O.E_UNREPAIRABLE)


def test_rsmt2d_repair_api(ctx):
    from cda import rsmt2d
    k = 4
    eds, rr, cr = _square(k, 9)
    cells = [bytes(eds[i]) if (i // (2 * k) < k and i % (2 * k) < k) else None for i in range(4 * k * k)]
    sq = rsmt2d.import_extended_data_square(cells, rsmt2d.LeoRSCodec(ctx))
    sq.repair([bytes(r) for r in rr], [bytes(c) for c in cr])
    assert all(sq.get_cell(i // (2 * k), i % (2 * k)) == bytes(eds[i]) for i in range(4 * k * k))
    sq2 = rsmt2d.import_extended_data_square([None] * (4 * k * k), rsmt2d.LeoRSCodec(ctx))
    with pytest.raises(rsmt2d.ErrUnrepairableDataSquare):
        sq2.repair([bytes(r) for r in rr], [bytes(c) for c in cr])


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128, 256])
def test_extend_commit_matches_committed_digests(ctx, k):
    """Device EDS / roots / DAH against the committed oracle digests (tests/golden/oracle_digests.json)."""
    import hashlib
    import json
    import os
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                     "oracle_digests.json")))[str(k)]
    eds, rr, cr, dah = ctx.extend_commit(O.gen_ods(k, fx["seed"]))
    assert dah.hex() == fx["dah"]
    assert hashlib.sha256(eds.tobytes()).hexdigest() == fx["eds_sha256"]
    assert hashlib.sha256(rr.tobytes() + cr.tobytes()).hexdigest() == fx["roots_sha256"]


def test_concurrent_calls_on_one_context(ctx):
    """rsmt2d calls Codec.Encode / tree Root concurrently from per-axis goroutines (SURVEY.md §8b Threading):
    the ctx mutex keeps concurrent callers correct."""
    import threading
    rng = np.random.default_rng(21)
    jobs = [rng.integers(0, 256, (k, 512), dtype=np.uint8) for k in (16, 64, 128, 32, 8, 100)]
    want = [O.leo_encode(d) for d in jobs]
    ods = O.gen_ods(16, 77)
    rc, _, rr_o, _, dah_o = O.extend_commit(ods)
    errors = []

    def worker(i):
        try:
            for _ in range(3):
                assert np.array_equal(ctx.rs_encode(jobs[i]), want[i])
                _, rr, _, dah = ctx.extend_commit(ods)
                assert np.array_equal(rr, rr_o) and dah == dah_o
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(len(jobs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    assert not errors, errors


# ---- Repair under Byzantine input: batched GPU execution must equal rsmt2d's sequential order ------------
def _check_repair_exact(ctx, bad, pres, rr, cr):
    """rc, (axis, index), the presence map and every present cell of the partially repaired square equal the
    oracle's sequential rsmt2d restatement (oracle/da.c ora_repair)."""
    rc_o, eds_o, p_o, ax_o, ix_o = O.repair(bad, pres, rr, cr)
    rc_g, eds_g, p_g, err = ctx.repair_status(bad, pres, rr, cr)
    assert rc_g == rc_o, (rc_g, rc_o)
    if rc_o == O.E_BYZANTINE:
        assert (err.axis, err.index) == (ax_o, ix_o)
    assert np.array_equal(p_g, p_o)
    m = p_o.astype(bool)
    assert np.array_equal(eds_g[m], eds_o[m])
    return rc_o, (ax_o, ix_o)


def test_repair_byzantine_row_and_column_share_a_missing_cell(ctx):
    """row 0 (honest) and column 5 (one corrupted present cell) are both decodable in the first sweep
    and share the missing cell (0, 5).  rsmt2d repairs row 0 first and then reports column 5."""
    k = 8
    w = 2 * k
    eds, rr, cr = _square(k, 31)
    rng = np.random.default_rng(8)
    pres = (rng.random((w, w)) < 0.75).astype(np.uint8)
    pres[0, 5] = 0          # shared missing cell of row 0 and column 5
    pres[10, 5] = 1         # corrupted present cell, in a row processed after column 5
    pres[10, 11] = 0        # row 10 incomplete, so the sanity check does not see it
    pres[3, 5] = 0          # column 5 incomplete
    bad = eds.copy()
    bad[10 * w + 5, 100] ^= 0x5A
    rc, (ax, ix) = _check_repair_exact(ctx, bad, pres.reshape(-1), rr, cr)
    assert rc == O.E_BYZANTINE and (ax, ix) == (1, 5)


@pytest.mark.parametrize("k,frac,nbad,seed", [(8, 0.6, 1, 1), (8, 0.7, 2, 2), (16, 0.6, 1, 3), (32, 0.55, 2, 4),
                                              (32, 0.7, 3, 5), (128, 0.55, 1, 6), (128, 0.65, 2, 7),
                                              (128, 0.6, 1, 8)])
def test_repair_byzantine_random_matches_sequential(ctx, k, frac, nbad, seed):
    """Random erasures plus corrupted present cells: the GPU's batched crossword reports the same error, axis and
    index as the sequential oracle and leaves the same partially repaired square."""
    w = 2 * k
    eds, rr, cr = _square(k, 500 + seed)
    rng = np.random.default_rng(seed)
    pres = (rng.random(w * w) < frac).astype(np.uint8)
    bad = eds.copy()
    for idx in rng.choice(np.flatnonzero(pres), nbad, replace=False):
        bad[idx, rng.integers(0, 512)] ^= 1 + rng.integers(0, 255)
    _check_repair_exact(ctx, bad, pres, rr, cr)


def test_repair_randomised_sweep_matches_sequential(ctx):
    """Stress for the optimistic whole-repair execution (every sweep planned up front, one host wait, sequential
    replay from the first failing batch): 48 random squares, k = 4..64, survival 20..85 %, 0..3 corrupted present
    cells, some in complete rows / columns (sanity check) -- rc, axis/index, presence and present cells equal the
    sequential oracle in every case."""
    rng = np.random.default_rng(2024)
    outcomes = set()
    for case in range(48):
        k = int(rng.choice([4, 8, 16, 32, 64]))
        w = 2 * k
        eds, rr, cr = _square(k, 3000 + case)
        frac = float(rng.uniform(0.2, 0.85))
        pres = (rng.random(w * w) < frac).astype(np.uint8)
        if case % 6 == 0:  # complete a few rows so the sanity check has work
            for r in rng.choice(w, 2, replace=False):
                pres[r * w:(r + 1) * w] = 1
        bad = eds.copy()
        nbad = int(rng.integers(0, 4))
        if nbad and pres.any():
            for idx in rng.choice(np.flatnonzero(pres), min(nbad, int(pres.sum())), replace=False):
                bad[idx, rng.integers(0, 512)] ^= 1 + rng.integers(0, 255)
        rc, _ = _check_repair_exact(ctx, bad, pres, rr, cr)
        outcomes.add(rc)
    assert {0, O.E_BYZANTINE, O.E_UNREPAIRABLE} <= outcomes, outcomes


def test_compute_eds_honours_custom_tree_constructor(ctx):
    """A TreeConstructorFn other than wrapper.NewConstructor is called the rsmt2d way:
    one tree per axis, the axis's cells pushed in order; the roots are the custom trees' roots."""
    from cda import rsmt2d, wrapper
    k = 4
    ods = O.gen_ods(k, 5)
    calls = []

    class CountingTree(wrapper.ErasuredNamespacedMerkleTree):
        def push(self, data):
            calls.append((self.axis_index, self.share_index))
            super().push(data)

    def ctor(axis, index):
        return CountingTree(k, index, ctx)

    codec = rsmt2d.LeoRSCodec(ctx)
    sq = rsmt2d.compute_extended_data_square([bytes(r) for r in ods], codec, ctor)
    assert len(calls) == 2 * (2 * k) * (2 * k)
    ref = rsmt2d.compute_extended_data_square([bytes(r) for r in ods], codec, wrapper.new_constructor(k, ctx))
    assert sq.row_roots() == ref.row_roots() and sq.col_roots() == ref.col_roots()


_WORKSPACE_SCRIPT = r"""
import sys
import numpy as np
import torch  # first: libcda then resolves HIP through torch's runtime, as in bench.py
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import cda
import oracle_lib as O
ctx = cda.Context(0)
k, B = 32, 8
w = 2 * k
ods = np.stack([O.gen_ods(k, 900 + b) for b in range(B)])
dev = torch.device("cuda", 0)
d_ods = torch.from_numpy(ods).to(dev)
d_eds = torch.empty((B, w * w, 512), dtype=torch.uint8, device=dev)
d_roots = torch.empty((B, 2 * w, 96), dtype=torch.uint8, device=dev)
d_dah = torch.empty((B, 32), dtype=torch.uint8, device=dev)
d_status = torch.empty((B,), dtype=torch.int64, device=dev)
s = torch.cuda.Stream(dev)
other = O.gen_ods(64, 77)
dah_other = O.extend_commit(other)[4]
for _ in range(3):
    ctx.extend_commit_device(k, B, d_ods.data_ptr(), d_eds.data_ptr(), d_roots.data_ptr(), d_dah.data_ptr(),
                             d_status.data_ptr(), s.cuda_stream)
    assert ctx.extend_commit(other)[3] == dah_other  # synchronous, on the ctx's own stream
s.synchronize()
for b in range(B):
    assert d_dah[b].cpu().numpy().tobytes() == O.extend_commit(ods[b])[4], b
print("workspace ok")
"""


def test_device_and_sync_calls_share_the_workspace():
    """cda_extend_commit_device enqueues on the caller's stream and uses the ctx workspace; a
    synchronous call issued right after must not overwrite it before the device call's kernels ran.
    (Own process: torch must be imported before libcda there, as bench.py does.)"""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(os.path.dirname(here), "celestia-app_amd")
    out = subprocess.run([sys.executable, "-c", _WORKSPACE_SCRIPT, pkg, here], capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0 and "workspace ok" in out.stdout, out.stderr[-3000:]


_REPAIR_DEVICE_SCRIPT = r"""
import sys
import numpy as np
import torch  # first: libcda then resolves HIP through torch's runtime, as in bench.py
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import cda
import oracle_lib as O
ctx = cda.Context(0)
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
cases = [(16, 0.6, 0, 1), (32, 0.55, 1, 2), (128, 0.5, 0, 3), (128, 0.6, 2, 4), (128, 0.25, 0, 5)]
for k, frac, nbad, seed in cases:
    w = 2 * k
    rc, eds, rr, cr, _ = O.extend_commit(O.gen_ods(k, 700 + seed))
    rng = np.random.default_rng(seed)
    pres = (rng.random(w * w) < frac).astype(np.uint8)
    bad = eds.copy()
    for idx in rng.choice(np.flatnonzero(pres), nbad, replace=False):
        bad[idx, rng.integers(0, 512)] ^= 1 + rng.integers(0, 255)
    rc_o, eds_o, p_o, ax_o, ix_o = O.repair(bad, pres, rr, cr)
    d = torch.from_numpy(bad).to(dev)
    torch.cuda.synchronize()
    rc_g, p_g, err = ctx.repair_device(k, d.data_ptr(), pres, rr, cr, s.cuda_stream)
    got = d.cpu().numpy()
    assert rc_g == rc_o, (k, seed, rc_g, rc_o)
    if rc_o == O.E_BYZANTINE:
        assert (err.axis, err.index) == (ax_o, ix_o), (k, seed)
    assert np.array_equal(p_g, p_o), (k, seed)
    m = p_o.astype(bool)
    assert np.array_equal(got[m], eds_o[m]), (k, seed)
print("repair_device ok")
"""


def test_repair_device_matches_sequential():
    """cda_repair_device on a square in HBM (torch allocation, caller stream): rc, Byzantine axis/index, presence
    and every present cell equal the sequential oracle, for repairable, Byzantine and unrepairable squares."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(os.path.dirname(here), "celestia-app_amd")
    out = subprocess.run([sys.executable, "-c", _REPAIR_DEVICE_SCRIPT, pkg, here], capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0 and "repair_device ok" in out.stdout, out.stderr[-3000:]


def test_axis_root_order_error_wins_over_push_past(ctx):
    """the reference Push validates leaf by leaf, so an order violation at leaf 3 is reported even when
    the caller pushes more than 2k leaves; a sorted over-long push reports PUSH_PAST at leaf 2k."""
    from cda import CdaError
    k = 4
    ods = O.gen_ods(8, 41)
    leaves = sorted(bytes(r) for r in ods[:k])
    bad = leaves[:3] + [leaves[0]] + [bytes(ods[i]) for i in range(k, 2 * k + 3)]  # order broken at leaf 3
    rc_o, _, leaf_o = O.nmt_axis_root(k, 0, bad)
    assert rc_o == O.E_NS_ORDER and leaf_o == 3
    with pytest.raises(CdaError) as ei:
        ctx.nmt_axis_root(k, 0, bad)
    assert ei.value.code == O.E_NS_ORDER and ei.value.leaf == 3
    good = leaves + [bytes(ods[i]) for i in range(k, 2 * k + 2)]
    rc_o, _, leaf_o = O.nmt_axis_root(k, 0, good)
    assert rc_o == O.E_PUSH_PAST and leaf_o == 2 * k
    with pytest.raises(CdaError) as ei:
        ctx.nmt_axis_root(k, 0, good)
    assert ei.value.code == O.E_PUSH_PAST and ei.value.leaf == 2 * k


_RS_DEVICE_SCRIPT = r"""
import sys
import numpy as np
import torch  # first: libcda then resolves HIP through torch's runtime, as in bench.py
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import cda
import oracle_lib as O
ctx = cda.Context(0)
dev = torch.device("cuda", 0)
rng = np.random.default_rng(7)
for k, ncw, L in [(16, 4, 512), (17, 4, 512), (34, 6, 512), (64, 2, 1024), (100, 4, 512), (128, 6, 512),
                  (128, 3, 512), (126, 2, 512), (128, 65, 512), (64, 63, 512), (32, 101, 1024), (100, 33, 512)]:
    data = rng.integers(0, 256, (ncw, k, L), dtype=np.uint8)
    d_src = torch.from_numpy(data).to(dev)
    d_dst = torch.zeros((ncw, k, L), dtype=torch.uint8, device=dev)
    # codeword c = data[c]: shards contiguous (the rows of erasureExtendSquare)
    ctx.rs_encode_device(k, L, ncw, d_src.data_ptr(), k * L, L, d_dst.data_ptr(), k * L, L)
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy()
    for c in range(ncw):
        assert np.array_equal(got[c], O.leo_encode(data[c])), (k, ncw, L, c, "rows")
    # the same codewords read as columns of a k x ncw grid (the column pass: src_cw = shard, src_sh = pitch)
    grid = np.ascontiguousarray(data.transpose(1, 0, 2))  # [k][ncw][L]
    d_src = torch.from_numpy(grid).to(dev)
    d_dst = torch.zeros((k, ncw, L), dtype=torch.uint8, device=dev)
    ctx.rs_encode_device(k, L, ncw, d_src.data_ptr(), L, ncw * L, d_dst.data_ptr(), L, ncw * L)
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().transpose(1, 0, 2)
    for c in range(ncw):
        assert np.array_equal(got[c], O.leo_encode(data[c])), (k, ncw, L, c, "cols")
print("rs device ok")
"""


def test_rs_encode_device_batched_strided():
    """cda_rs_encode_device, the batched strided Codec.Encode of the split path: even k (register encoder, incl.
    non-powers of two whose padded elements are zero), odd k and odd codeword counts up to 101 (LDS encoder), row-
    and column-strided codewords, each codeword equal to the oracle's Leopard encode."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(os.path.dirname(here), "celestia-app_amd")
    out = subprocess.run([sys.executable, "-c", _RS_DEVICE_SCRIPT, pkg, here], capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0 and "rs device ok" in out.stdout, out.stderr[-3000:]
