"""CPU tests: blob share commitments, subtree-root paths and proofs (oracle + host logic).

The oracle (oracle/inclusion.c) is pinned here against the reference's own data:
  * the share commitment of the blob in mainnet block 408
    (x/blob/test/testdata/block_response.json -> tests/golden/make_blob_commitments.py),
    through CreateCommitment and through GetCommitment over the block's EDS;
  * the valid ShareProof / RowProof of pkg/proof/share_proof_test.go:74-93 and
    row_proof_test.go:67-89 (tests/golden/make_share_proof_fixture.py).
The path planning of the Python mirror (cda.inclusion) is checked against
pkg/inclusion/paths_test.go.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from cda import inclusion as I

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
L, R = I.WALK_LEFT, I.WALK_RIGHT


def mainnet_blobs():
    z = np.load(os.path.join(GOLDEN, "mainnet_h408_blobs.npz"))
    offs = z["offsets"]
    return [dict(ns=z["namespaces"][i].tobytes(), data=z["data"][offs[i]:offs[i + 1]].tobytes(),
                 version=int(z["share_versions"][i]), start=int(z["starts"][i]), n=int(z["nshares"][i]),
                 commitment=z["commitments"][i].tobytes()) for i in range(len(offs) - 1)]


def mainnet_ods():
    return np.load(os.path.join(GOLDEN, "mainnet_h408.npz"))["ods"]


# ---- paths_test.go -------------------------------------------------------------------------
COORDS = [  # Test_calculateSubTreeRootCoordinates (paths_test.go:21-314): start, end, maxDepth, minDepth
    (0, 4, 3, 1, [(1, 0)]), (4, 8, 3, 1, [(1, 1)]), (3, 5, 3, 3, [(3, 3), (3, 4)]), (3, 4, 3, 3, [(3, 3)]),
    (3, 6, 3, 2, [(3, 3), (2, 2)]), (1, 7, 3, 2, [(3, 1), (2, 1), (2, 2), (3, 6)]),
    (1, 7, 3, 3, [(3, 1), (3, 2), (3, 3), (3, 4), (3, 5), (3, 6)]), (0, 5, 3, 1, [(1, 0), (3, 4)]),
    (0, 7, 3, 1, [(1, 0), (2, 2), (3, 6)]), (0, 8, 3, 0, [(0, 0)]), (0, 32, 7, 2, [(2, 0)]),
    (0, 33, 7, 2, [(2, 0), (7, 32)]), (0, 31, 7, 3, [(3, 0), (4, 2), (5, 6), (6, 14), (7, 30)]),
    (0, 64, 7, 1, [(1, 0)]), (0, 1, 2, 2, [(2, 0)]), (0, 19, 6, 3, [(3, 0), (3, 1), (5, 8), (6, 18)]),
]


@pytest.mark.parametrize("start,end,maxd,mind,want", COORDS)
def test_subtree_root_coordinates(start, end, maxd, mind, want):
    got = [(c.depth, c.position) for c in I.calculate_subtree_root_coordinates(maxd, mind, start, end)]
    assert got == want
    assert O.subtree_root_coords(maxd, mind, start, end) == want


@pytest.mark.parametrize("depth,pos,want", [(2, 0, [L, L]), (0, 0, []), (3, 0, [L, L, L]), (3, 1, [L, L, R]),
                                            (3, 2, [L, R, L]), (5, 16, [R, L, L, L, L])])
def test_gen_subtree_root_path(depth, pos, want):  # paths_test.go:321-339
    assert I.gen_subtree_root_path(depth, pos) == want


PATHS = [  # Test_calculateCommitPaths (paths_test.go:352-450): squareSize, start, blobLen, {index: (row, path)}
    (2, 2, 2, {0: (1, [L]), 1: (1, [R])}),
    (4, 2, 2, {0: (0, [R, L]), 1: (0, [R, R])}),
    (4, 3, 2, {0: (0, [R, R]), 1: (1, [L, L])}),
    (128, 8252, 1, {0: (64, [L, R, R, R, R, L, L])}),
    (128, 0, 8193, {31: (31, [])}),
    (128, 0, 8192, {31: (31, [])}),
    (128, 0, 64, {31: (0, [L, L, R, R, R, R, R])}),
    (128, 0, 65, {31: (0, [L, R, R, R, R, R]), 32: (0, [R, L, L, L, L, L, L])}),
]


@pytest.mark.parametrize("square,start,n,want", PATHS)
def test_calculate_commitment_paths(square, start, n, want):
    paths = I.calculate_commitment_paths(square, start, n, 64)
    for i, (row, instr) in want.items():
        assert (paths[i].row, paths[i].instructions) == (row, instr)
    keys = [(p.row, tuple(p.instructions)) for p in paths]
    assert len(keys) == len(set(keys))  # every path is unique


def test_share_arithmetic_mirror_matches_oracle():
    # data_square_layout.md:58: 172 shares, SRT 64 -> width 4, 43 mountains of 4
    assert I.sub_tree_width(172, 64) == O.subtree_width(172, 64) == 4
    assert I.merkle_mountain_range_sizes(172, 4) == O.mmr_sizes(172, 4) == [4] * 43
    for n in [1, 2, 3, 5, 17, 63, 64, 65, 127, 128, 129, 352, 1000, 4096, 8192, 8193, 16384]:
        for t in [1, 8, 64]:
            w = I.sub_tree_width(n, t)
            assert w == O.subtree_width(n, t)
            assert I.merkle_mountain_range_sizes(n, w) == O.mmr_sizes(n, w)
            assert sum(I.merkle_mountain_range_sizes(n, w)) == n
    for ln in [1, 477, 478, 479, 960, 961, 1_000_000]:
        assert I.sparse_shares_needed(ln) == O.sparse_shares_needed(ln)
    assert I.next_share_index(13, 4 * 64, 64) == 16


# ---- commitments pinned on mainnet block 408 ----------------------------------------------
def test_oracle_create_commitment_matches_mainnet_pfb():
    blobs = mainnet_blobs()
    assert blobs
    for b in blobs:
        rc, got = O.blob_commitment(b["ns"], b["data"], b["version"], 64)
        assert rc == 0 and got == b["commitment"]


def test_mainnet_blob_shares_sit_in_the_square():
    ods = mainnet_ods()
    for b in mainnet_blobs():
        shares = O.blob_to_shares(b["ns"], b["data"], b["version"])
        assert len(shares) == b["n"]
        assert np.array_equal(shares, ods[b["start"]:b["start"] + b["n"]])


def test_oracle_get_commitment_matches_mainnet_pfb():
    eds = O.extend(mainnet_ods())
    for b in mainnet_blobs():
        rc, got = O.get_commitment(eds, b["start"], b["n"], 64)
        assert rc == 0 and got == b["commitment"]


def test_oracle_commitment_errors():
    assert O.blob_commitment(bytes(29), b"", 0)[0] == O.E_BLOB_SIZE
    assert O.blob_commitment(bytes(29), b"x", 1)[0] == O.E_SHARE_VERSION


# ---- proof verifiers pinned on the reference's fixtures -----------------------------------
def _fixture():
    return json.load(open(os.path.join(GOLDEN, "share_proof_fixture.json")))


def test_reference_row_proof_verifies():
    fx = _fixture()
    p, rr = fx["row_proof"], bytes.fromhex(fx["row_roots"][0])
    aunts = [bytes.fromhex(a) for a in p["aunts"]]
    args = (p["total"], p["index"], bytes.fromhex(p["leaf_hash"]), aunts)
    assert O.merkle_verify(*args, bytes.fromhex(fx["root"]), rr)
    assert not O.merkle_verify(*args, bytes(32), rr)  # incorrectRoot (row_proof_test.go:70)


def test_reference_share_proof_verifies():
    fx = _fixture()
    rr = bytes.fromhex(fx["row_roots"][0])
    nid = bytes([fx["namespace_version"]]) + bytes.fromhex(fx["namespace_id"])
    data = [bytes.fromhex(d) for d in fx["data"]]
    nodes = [bytes.fromhex(x) for x in fx["nmt"]["nodes"]]
    s, e = fx["nmt"]["start"], fx["nmt"]["end"]
    assert O.nmt_verify_inclusion(nid, data, s, e, nodes, rr)
    bad = bytearray(data[0])
    bad[100] ^= 1
    assert not O.nmt_verify_inclusion(nid, [bytes(bad)], s, e, nodes, rr)
    assert not O.nmt_verify_inclusion(nid, data, s, e, nodes[:-1], rr)


@pytest.mark.parametrize("k", [1, 2, 4, 8])
def test_oracle_prove_range_round_trip(k):
    """ProveRange over real erasured rows verifies against the row root for every range."""
    eds = O.extend(O.gen_ods(k, 31 + k))
    rc, rr, cr, *_ = O.roots(eds)
    w = 2 * k
    for row in {0, k - 1, w - 1}:
        leaves = O.axis_leaf_nodes(eds, 0, row)
        assert O.tree_levels(leaves)[-1].tobytes() == rr[row].tobytes()
        cells = eds.reshape(w, w, 512)[row]
        for s in range(w):
            for e in range(s + 1, w + 1):
                nodes = O.nmt_prove_range(leaves, s, e)
                ns = leaves[s][:29].tobytes()
                if any(leaves[i][:29].tobytes() != ns for i in range(s, e)):
                    continue  # VerifyInclusion proves one namespace
                assert O.nmt_verify_inclusion(ns, [cells[i].tobytes() for i in range(s, e)], s, e, nodes,
                                              rr[row].tobytes())


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 16])
def test_oracle_merkle_proofs(n):
    rng = np.random.default_rng(n)
    items = [rng.integers(0, 256, 90, dtype=np.uint8).tobytes() for _ in range(n)]
    want_root = O.merkle_root(items)
    for i in range(n):
        leaf, aunts, root = O.merkle_proof(items, i)
        assert root == want_root
        assert O.merkle_verify(n, i, leaf, aunts, root, items[i])
        assert not O.merkle_verify(n, i, leaf, aunts, root, items[(i + 1) % n]) or n == 1


@pytest.mark.parametrize("start,end,msg", [(-1, 1, "should be positive"), (0, -1, "should be positive"),
                                           (10, 9, "cannot be lower than starting share"),
                                           (0, 1025, "is higher than block shares")])
def test_parse_namespace_rejects_bad_ranges(start, end, msg):
    """TestNewShareInclusionProof's error cases (pkg/proof/proof_test.go:98-232; querier.go ParseNamespace) on
    mainnet block 408's 32 x 32 square: negative start / end, end below start, end past the square's 1,024 shares;
    and a range spanning two namespaces."""
    from cda import proof as P
    shares = [bytes(s) for s in mainnet_ods()]
    with pytest.raises(P.ProofError) as ei:
        P.parse_namespace(shares, start, end)
    assert msg in str(ei.value)


def test_parse_namespace_single_namespace_ranges():
    from cda import proof as P
    shares = [bytes(s) for s in mainnet_ods()]
    b = mainnet_blobs()[0]
    assert P.parse_namespace(shares, 0, 1) == shares[0][:29]
    assert P.parse_namespace(shares, b["start"], b["start"] + b["n"]) == shares[b["start"]][:29]
    with pytest.raises(P.ProofError) as ei:
        P.parse_namespace(shares, b["start"] - 1, b["start"] + 1)
    assert "different namespaces" in str(ei.value)


# ---- pkg/proof Validate mirrors (cda.proof), on the reference's own fixtures ---------------------------------------
def _fixture_proofs():
    from cda import proof as P
    fx = _fixture()
    p = fx["row_proof"]
    pr = P.Proof(p["total"], p["index"], bytes.fromhex(p["leaf_hash"]), [bytes.fromhex(a) for a in p["aunts"]])
    rp = P.RowProof([bytes.fromhex(r) for r in fx["row_roots"]], [pr], fx["start_row"], fx["end_row"])
    nm = P.NMTProof(fx["nmt"]["start"], fx["nmt"]["end"], [bytes.fromhex(x) for x in fx["nmt"]["nodes"]])
    sp = P.ShareProof([bytes.fromhex(d) for d in fx["data"]], [nm], bytes.fromhex(fx["namespace_id"]), rp,
                      fx["namespace_version"])
    return bytes.fromhex(fx["root"]), rp, sp


def test_row_proof_validate_cases():
    """TestRowProofValidate (pkg/proof/row_proof_test.go:10-66) on its own vector."""
    import copy
    from cda import proof as P
    root, rp, _ = _fixture_proofs()
    rp.validate(root)  # "valid row proof returns no error"
    cases = {"empty": P.RowProof([], [], 0, 0)}
    cases["mismatched row roots"] = copy.deepcopy(rp)
    cases["mismatched row roots"].row_roots = []
    cases["mismatched proofs"] = copy.deepcopy(rp)
    cases["mismatched proofs"].proofs = []
    cases["mismatched rows"] = copy.deepcopy(rp)
    cases["mismatched rows"].end_row = 10
    for name, bad in cases.items():
        with pytest.raises(P.ProofError):
            bad.validate(root)
    with pytest.raises(P.ProofError):  # "valid row proof with incorrect root"
        rp.validate(bytes(32))


def test_share_proof_validate_cases():
    """TestShareProofValidate (pkg/proof/share_proof_test.go:9-60) on its own vector (33-byte namespace)."""
    import copy
    from cda import proof as P
    root, _, sp = _fixture_proofs()
    sp.validate(root)
    empty = P.ShareProof(None, [], b"", P.RowProof([], [], 0, 0), 0)
    fewer_proofs = copy.deepcopy(sp)
    fewer_proofs.share_proofs = []
    more_shares = copy.deepcopy(sp)
    more_shares.data = more_shares.data + [more_shares.data[0]]
    for bad in (empty, fewer_proofs, more_shares):
        with pytest.raises(P.ProofError):
            bad.validate(root)
    with pytest.raises(P.ProofError):
        sp.validate(bytes(32))
    tampered = copy.deepcopy(sp)
    d = bytearray(tampered.data[0])
    d[100] ^= 1
    tampered.data[0] = bytes(d)
    assert not tampered.verify_proof()


@pytest.mark.parametrize("k", [1, 2, 4])
def test_nmt_verify_inclusion_matches_oracle(k):
    """cda.proof's NMT inclusion verifier agrees with the oracle's on every single-namespace range of real erasured
    rows (ranges proved by the oracle's ProveRange), and rejects a proof with a node dropped."""
    from cda import proof as P
    eds = O.extend(O.gen_ods(k, 71 + k))
    rc, rr, *_ = O.roots(eds)
    w = 2 * k
    for row in {0, w - 1}:
        leaves = O.axis_leaf_nodes(eds, 0, row)
        cells = eds.reshape(w, w, 512)[row]
        for s in range(w):
            for e in range(s + 1, w + 1):
                ns = leaves[s][:29].tobytes()
                if any(leaves[i][:29].tobytes() != ns for i in range(s, e)):
                    continue
                nodes = O.nmt_prove_range(leaves, s, e)
                data = [cells[i].tobytes() for i in range(s, e)]
                assert P.NMTProof(s, e, nodes).verify_inclusion(ns, data, rr[row].tobytes())
                if nodes:
                    assert not P.NMTProof(s, e, nodes[:-1]).verify_inclusion(ns, data, rr[row].tobytes())


@pytest.mark.parametrize("k", [1, 2, 4, 8])
def test_wrapper_prove_range_matches_oracle(k):
    """wrapper ErasuredNamespacedMerkleTree.ProveRange (host, cda.wrapper) gives the oracle's proof nodes for every
    range of real erasured rows and columns, and each proof verifies against the oracle's root (cda.proof)."""
    from cda.wrapper import ErasuredNamespacedMerkleTree
    eds = O.extend(O.gen_ods(k, 91 + k))
    rc, rr, cr, *_ = O.roots(eds)
    w = 2 * k
    sq = eds.reshape(w, w, 512)
    for axis, idx in ((0, 0), (0, w - 1), (1, 0), (1, k)):
        cells = sq[idx] if axis == 0 else sq[:, idx]
        root = (rr if axis == 0 else cr)[idx].tobytes()
        leaves = O.axis_leaf_nodes(eds, axis, idx)
        t = ErasuredNamespacedMerkleTree(k, idx)
        for c in cells:
            t.push(c.tobytes())
        for s in range(w):
            for e in range(s + 1, w + 1):
                p = t.prove_range(s, e)
                assert p.nodes == O.nmt_prove_range(leaves, s, e), (axis, idx, s, e)
                ns = leaves[s][:29].tobytes()
                if all(leaves[i][:29].tobytes() == ns for i in range(s, e)):
                    assert p.verify_inclusion(ns, [cells[i].tobytes() for i in range(s, e)], root)
