"""GPU parity: blob share commitments, NMT node export and share inclusion proofs (libcda vs the oracle).

Every comparison is bit-exact. The mainnet block 408 fixtures (tests/test_inclusion.py)
pin the results on real data: the GPU reproduces the block's PFB share commitment
through CreateCommitment and through GetCommitment over its EDS, and its share
proofs verify against the block's data_hash.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from test_inclusion import GOLDEN, mainnet_blobs, mainnet_ods

pytestmark = pytest.mark.gpu


def test_blob_commitment_mainnet(ctx):
    from cda import inclusion as I
    blobs = mainnet_blobs()
    got = ctx.blob_commitments([b["ns"] for b in blobs], [b["data"] for b in blobs], [b["version"] for b in blobs], 64)
    assert got == [b["commitment"] for b in blobs]
    assert I.create_commitment(I.Blob(blobs[0]["ns"], blobs[0]["data"]), ctx=ctx) == blobs[0]["commitment"]


@pytest.mark.parametrize("threshold", [64, 8, 1])
def test_blob_commitments_random_vs_oracle(ctx, threshold):
    rng = np.random.default_rng(threshold)
    sizes = [1, 477, 478, 479, 960, 961, 5000, 40000, 171000, 300000, 1, 2, 3, 1_000_000]
    ns_list = [bytes(19) + rng.integers(0, 256, 10, dtype=np.uint8).tobytes() for _ in sizes]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    got = ctx.blob_commitments(ns_list, datas, None, threshold)
    for ns, d, g in zip(ns_list, datas, got):
        rc, want = O.blob_commitment(ns, d, 0, threshold)
        assert rc == 0 and g == want, len(d)


def test_blob_commitments_many_small(ctx):
    rng = np.random.default_rng(5)
    datas = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 3000, 500)]
    ns_list = [bytes(19) + rng.integers(0, 256, 10, dtype=np.uint8).tobytes() for _ in datas]
    got = ctx.blob_commitments(ns_list, datas, None, 64)
    assert got == [O.blob_commitment(n, d)[1] for n, d in zip(ns_list, datas)]


def test_blob_commitment_errors(ctx):
    from cda import CdaError
    with pytest.raises(CdaError) as e:
        ctx.blob_commitments([bytes(29)] * 2, [b"x", b""], None, 64)
    assert e.value.code == -14 and e.value.index == 1
    with pytest.raises(CdaError) as e:
        ctx.blob_commitments([bytes(29)], [b"x"], [1], 64)
    assert e.value.code == -13 and e.value.index == 0


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 200])
def test_merkle_roots_vs_oracle(ctx, n):
    rng = np.random.default_rng(n)
    sets = [[rng.integers(0, 256, 90, dtype=np.uint8).tobytes() for _ in range(m)] for m in (n, 1, n + 1)]
    got = ctx.merkle_roots(sets + [[]])
    assert got[:3] == [O.merkle_root(s) for s in sets]
    assert got[3] == O.sha256(b"")


@pytest.mark.parametrize("rows,cols", [(False, True), (True, False)])
def test_extend_commit_nodes_one_kind(ctx, rows, cols):
    """Only the column trees, or only the row trees, exported (the device-packed node lists of one kind)."""
    k = 8
    ods = O.gen_ods(k, 0xAC)
    out = ctx.extend_commit_nodes(ods, rows=rows, cols=cols, dah_tree=False)
    eds_o = O.extend(ods)
    for axis, key, want in ((0, "row_nodes", rows), (1, "col_nodes", cols)):
        if not want:
            assert out[key] is None
            continue
        for t in range(2 * k):
            assert np.array_equal(out[key][t], O.tree_levels(O.axis_leaf_nodes(eds_o, axis, t))), (axis, t)


@pytest.mark.parametrize("k", [1, 2, 4, 8, 32])
def test_extend_commit_nodes_vs_oracle(ctx, k):
    ods = O.gen_ods(k, 0xAB + k)
    out = ctx.extend_commit_nodes(ods, want_eds=True)
    rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
    assert rc == 0 and np.array_equal(out["eds"], eds_o)
    assert np.array_equal(out["row_roots"], rr_o) and np.array_equal(out["col_roots"], cr_o) and out["dah"] == dah_o
    w = 2 * k
    for axis, key in ((0, "row_nodes"), (1, "col_nodes")):
        for t in range(w):
            assert np.array_equal(out[key][t], O.tree_levels(O.axis_leaf_nodes(eds_o, axis, t))), (axis, t)
    items = [r.tobytes() for r in np.concatenate([rr_o, cr_o])]
    dn = out["dah_nodes"]
    assert dn[-1].tobytes() == dah_o
    for i in sorted({0, w - 1, w, 2 * w - 1}):
        assert dn[i].tobytes() == O.merkle_proof(items, i)[0]


def test_get_commitment_mainnet(ctx):
    from cda import inclusion as I
    cacher, dah = I.EDSSubTreeRootCacher.from_shares([bytes(s) for s in mainnet_ods()], ctx=ctx)
    assert dah.hash() == np.load(os.path.join(GOLDEN, "mainnet_h408.npz"))["data_hash"].tobytes()
    for b in mainnet_blobs():
        assert I.get_commitment(cacher, dah, b["start"], b["n"], 64, ctx=ctx) == b["commitment"]


def test_eds_sub_root_cacher(ctx):
    """TestEDSSubRootCacher (pkg/inclusion/nmt_caching_test.go:117-138), k = 8: for every ODS row, the subtree root
    three steps left of the row root is the NMT root of the row's first two shares pushed into a fresh tree (their
    own namespaces: quadrant zero)."""
    from cda import inclusion as I
    k = 8
    ods = O.gen_ods(k, 0xCAC4E)
    cacher, dah = I.EDSSubTreeRootCacher.from_shares([bytes(s) for s in ods], ctx=ctx)
    for i in range(k):
        rc, want, _ = O.nmt_axis_root(k, 0, [bytes(ods[i * k]), bytes(ods[i * k + 1])])
        assert rc == 0 and cacher.get_sub_tree_root(dah, i, [False, False, False]) == want, i


@pytest.mark.parametrize("k", [4, 16])
def test_get_commitment_random_vs_oracle(ctx, k):
    from cda import inclusion as I
    ods = O.gen_ods(k, 0x5EED + k)
    eds = O.extend(ods)
    cacher, dah = I.EDSSubTreeRootCacher.from_shares([bytes(s) for s in ods], ctx=ctx)
    for start, n in [(0, 1), (0, k * k), (3, 5), (k, 2 * k + 1), (0, k * k - 1)]:
        rc, want = O.get_commitment(eds, start, n, 64)
        assert rc == 0 and I.get_commitment(cacher, dah, start, n, 64, ctx=ctx) == want, (start, n)
    with pytest.raises(I.InclusionError):
        cacher.get_sub_tree_root(dah, 0, [False] * (2 * k).bit_length())


@pytest.mark.parametrize("k,ranges", [(1, [(0, 1)]), (4, [(0, 1), (0, 16), (3, 9), (5, 6), (15, 16)]),
                                      (16, [(0, 53), (17, 200), (255, 256), (16, 32), (0, 256)])])
def test_share_inclusion_proof_vs_oracle(ctx, k, ranges):
    """Row / NMT range proofs of ODS share ranges vs the oracle; (0, 256) at k = 16 is TestAllSharesInclusionProof's
    whole 256-share square (pkg/proof/proof_test.go:234-262)."""
    ods = O.gen_ods(k, 0xF00D + k)
    eds = O.extend(ods)
    rc, rr, cr, *_ = O.roots(eds)
    items = [r.tobytes() for r in np.concatenate([rr, cr])]
    for start, end in ranges:
        out = ctx.share_inclusion_proof(ods, start, end)
        assert (out["start_row"], out["end_row"], out["total"]) == (start // k, (end - 1) // k, 4 * k)
        for i, row in enumerate(out["rows"]):
            r = out["start_row"] + i
            assert row["row_root"] == rr[r].tobytes()
            leaf, aunts, root = O.merkle_proof(items, r)
            assert (row["leaf_hash"], row["aunts"], out["data_root"]) == (leaf, aunts, root)
            s = start % k if i == 0 else 0
            e = (end - 1) % k + 1 if r == out["end_row"] else k
            assert (row["start"], row["end"]) == (s, e)
            assert row["nodes"] == O.nmt_prove_range(O.axis_leaf_nodes(eds, 0, r), s, e)


def test_share_inclusion_proof_mainnet_verifies(ctx):
    """ShareProof.Validate semantics (share_proof.go:16-82) with the oracle verifiers against data_hash."""
    from cda import proof as P
    z = np.load(os.path.join(GOLDEN, "mainnet_h408.npz"))
    data_hash = z["data_hash"].tobytes()
    shares = [bytes(s) for s in z["ods"]]
    b = mainnet_blobs()[0]
    for start, end in [(b["start"], b["start"] + b["n"]), (0, 1), (b["start"] + 5, b["start"] + 40)]:
        ns = P.parse_namespace(shares, start, end)
        sp = P.new_share_inclusion_proof(shares, ns, start, end, ctx=ctx)
        assert sp.data_root == data_hash and len(sp.data) == end - start
        assert len(sp.share_proofs) == len(sp.row_proof.row_roots) == sp.row_proof.end_row - sp.row_proof.start_row + 1
        cursor = 0
        for nm, rp, rr in zip(sp.share_proofs, sp.row_proof.proofs, sp.row_proof.row_roots):
            assert O.merkle_verify(rp.total, rp.index, rp.leaf_hash, rp.aunts, data_hash, rr)
            used = nm.end - nm.start
            assert O.nmt_verify_inclusion(ns, sp.data[cursor:cursor + used], nm.start, nm.end, nm.nodes, rr)
            cursor += used
        assert cursor == end - start
        sp.validate(data_hash)  # ShareProof.Validate (cda.proof mirror) on the GPU-built proof
        with pytest.raises(P.ProofError):
            sp.validate(bytes(32))
    with pytest.raises(P.ProofError):
        P.parse_namespace(shares, 0, b["start"] + 1)  # spans several namespaces


def test_dah_proto_round_trip(ctx):
    from cda import da
    dahs = [da.min_data_availability_header(),
            da.new_data_availability_header(da.extend_shares([bytes(s) for s in O.gen_ods(8, 3)]))]
    for d in dahs:
        back = da.data_availability_header_from_proto(d.to_proto())
        assert back.row_roots == d.row_roots and back.column_roots == d.column_roots and back.hash() == d.hash()
    with pytest.raises(da.DAError):
        da.data_availability_header_from_proto(da.DataAvailabilityHeader([bytes(90)], [bytes(90)]).to_proto())


def test_max_square_nodes_and_proof_k128(ctx):
    """Production maximum (k=128, SquareSizeUpperBound): exported nodes of sampled trees and a proof spanning rows."""
    k = 128
    ods = O.gen_ods(k, 0x128)
    out = ctx.extend_commit_nodes(ods, want_eds=True)
    eds = out["eds"]
    for axis, key in ((0, "row_nodes"), (1, "col_nodes")):
        for t in (0, 127, 128, 255):
            assert np.array_equal(out[key][t], O.tree_levels(O.axis_leaf_nodes(eds, axis, t))), (axis, t)
    p = ctx.share_inclusion_proof(ods, 1000, 1500)
    assert p["data_root"] == out["dah"] and len(p["rows"]) == (1499 // k) - (1000 // k) + 1
    for i, row in enumerate(p["rows"]):
        r = p["start_row"] + i
        assert row["nodes"] == O.nmt_prove_range(O.axis_leaf_nodes(eds, 0, r), row["start"], row["end"])


def test_blob_commitment_largest_blob(ctx):
    """An ~8 MB blob (16 Ki shares: SubTreeWidth 128, 128 mountains) and a tiny one in one call."""
    rng = np.random.default_rng(8)
    datas = [rng.integers(0, 256, 16384 * 482 - 4, dtype=np.uint8).tobytes(), b"\x07"]
    ns = [bytes(19) + bytes(range(10)), bytes(19) + bytes(range(1, 11))]
    got = ctx.blob_commitments(ns, datas, None, 64)
    assert got == [O.blob_commitment(n, d)[1] for n, d in zip(ns, datas)]
