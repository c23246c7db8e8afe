"""CPU tests: the oracle against the reference's known answers and the RS identities.

These pin the checker before it is used to judge the GPU path.
"""
import numpy as np
import pytest

import kat
import oracle_lib as O


def test_nil_dah_hash_is_sha256_empty():
    # TestNilDataAvailabilityHeaderHashDoesntCrash (data_availability_header_test.go:15-25)
    assert O.merkle_root([]) == kat.EMPTY_HASH
    assert O.sha256(b"") == kat.EMPTY_HASH


def test_min_data_availability_header():
    # TestMinDataAvailabilityHeader (:27-32)
    rc, _, rr, cr, dah = O.extend_commit(kat.tail_padding_share()[None])
    assert rc == 0 and dah == kat.MIN_DAH
    assert rr.shape == (2, 90)


@pytest.mark.parametrize("k,expected", [(2, kat.TYPICAL_K2), (128, kat.MAX_K128)])
def test_new_data_availability_header(k, expected):
    # TestNewDataAvailabilityHeader (:34-68)
    rc, _, rr, cr, dah = O.extend_commit(kat.generate_shares(k * k), want_eds=False)
    assert rc == 0
    assert len(rr) == 2 * k and len(cr) == 2 * k
    assert dah == expected


@pytest.mark.parametrize("count", [5, 129 * 129, 8])
def test_extend_shares_errors(count):
    # TestExtendShares (:70-99): non power of 2 -> error; 8 is pow2 but not square (rsmt2d)
    rc, *_ = O.extend_commit(kat.generate_shares(count), want_eds=False)
    assert rc in (O.E_NOT_POW2, O.E_NOT_SQUARE)


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 16, 33, 64, 100, 128, 129, 256, 300])
def test_leopard_fft_encode_equals_lagrange_decode(k):
    """FFT encoder (Appendix A) vs an independent Lagrange decoder in Leopard's field."""
    rng = np.random.default_rng(k)
    L = 64
    d = rng.integers(0, 256, (k, L), dtype=np.uint8)
    p = O.leo_encode(d)
    full = np.concatenate([d, p])
    for _ in range(3):
        pres = np.zeros(2 * k, np.uint8)
        pres[rng.choice(2 * k, k, replace=False)] = 1
        rc, rep = O.leo_decode(np.where(pres[:, None] == 1, full, 0xA5).astype(np.uint8), pres)
        assert rc == 0
        assert np.array_equal(rep, full)


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 64, 128, 256, 512])
def test_leopard_constant_to_constant(k):
    d = np.full((k, 64), 0x5A, np.uint8)
    assert np.all(O.leo_encode(d) == 0x5A)


def test_leopard_linearity():
    rng = np.random.default_rng(7)
    for k in (8, 100, 300):
        a = rng.integers(0, 256, (k, 64), dtype=np.uint8)
        b = rng.integers(0, 256, (k, 64), dtype=np.uint8)
        assert np.array_equal(O.leo_encode(a ^ b), O.leo_encode(a) ^ O.leo_encode(b))


def test_leopard_too_few_shards():
    d = np.zeros((4, 64), np.uint8)
    pres = np.array([1, 1, 1, 0, 0, 0, 0, 0], np.uint8)
    rc, _ = O.leo_decode(np.zeros((8, 64), np.uint8), pres)
    assert rc == O.E_TOO_FEW


def test_field_tables():
    # Leopard representation: 1 is the multiplicative identity; exp/log are inverse.
    for bits in (8, 16):
        order = 1 << bits
        for a in (1, 2, 3, 0x53, order - 1):
            assert O.lib().ora_leo_mul(bits, a, 1) == a
            assert O.lib().ora_leo_exp(bits, O.lib().ora_leo_log(bits, a)) == a


def test_eds_quadrant_layout_and_linearity():
    """Q0 = ODS; Q1/Q2 = row/col encodings; Q3 row- and column-consistent."""
    k = 8
    ods = O.gen_ods(k, 0xC0FFEE)
    eds = O.extend(ods).reshape(2 * k, 2 * k, 512)
    assert np.array_equal(eds[:k, :k].reshape(-1, 512), ods)
    for r in range(k):
        assert np.array_equal(eds[r, k:], O.leo_encode(eds[r, :k]))
    for c in range(2 * k):
        assert np.array_equal(eds[k:, c], O.leo_encode(eds[:k, c]))
    for r in range(k, 2 * k):
        assert np.array_equal(eds[r, k:], O.leo_encode(eds[r, :k]))


def test_nmt_erasured_root_differs_from_plain():
    # TestRootErasuredNamespacedMerkleTree (nmt_wrapper_test.go:49-73): k=8, 8 pushes on axis 0
    ods = O.gen_ods(8, 1)
    rc, root_erasured, _ = O.nmt_axis_root(8, 0, [bytes(ods[i]) for i in range(8)])
    # a plain NMT of the same leaves == erasured tree with all leaves inside Q0 (square size large)
    rc2, root_plain, _ = O.nmt_axis_root(1 << 20, 0, [bytes(ods[i]) for i in range(8)])
    assert rc == 0 and rc2 == 0
    assert root_erasured == root_plain  # 8 pushes on a k=8 axis are all Q0 leaves


def test_nmt_empty_roots_equal():
    # TestErasuredNamespacedMerkleTreeEmptyRoot (nmt_wrapper_test.go:76-89)
    _, r1, _ = O.nmt_axis_root(1, 0, [])
    _, r2, _ = O.nmt_axis_root(2, 1, [])
    assert r1 == r2 and r1[:58] == b"\x00" * 58 and r1[58:] == kat.EMPTY_HASH


def test_nmt_push_errors():
    # TestErasureNamespacedMerkleTreePushErrors (nmt_wrapper_test.go:91-128)
    k = 16
    ods = O.gen_ods(k, 3)
    leaves = [bytes(ods[i]) for i in range(2 * k + 2)]
    rc, _, _ = O.nmt_axis_root(k, 0, leaves)
    assert rc == O.E_PUSH_PAST
    rev = sorted([bytes(ods[i]) for i in range(2 * k)], reverse=True)
    rc, _, _ = O.nmt_axis_root(k, 0, rev)
    assert rc == O.E_NS_ORDER
    rc, _, _ = O.nmt_axis_root(k, 0, [b"\x01"])
    assert rc == O.E_NS_SHORT


def test_roots_namespace_order_error():
    k = 4
    ods = O.gen_ods(k, 5)
    ods[[1, 2]] = ods[[2, 1]]  # swap two shares in row 0
    rc, rr, cr, ax, ix = O.roots(O.extend(ods))
    assert rc == O.E_NS_ORDER and ax == 0 and ix == 0


def test_repair_structured_and_random():
    k = 8
    ods = O.gen_ods(k, 11)
    rc, eds, rr, cr, dah = O.extend_commit(ods)
    w = 2 * k
    # (i) only Q0 survives
    pres = np.zeros((w, w), np.uint8)
    pres[:k, :k] = 1
    rc, rep, p2, _, _ = O.repair(np.where(pres.reshape(-1, 1) == 1, eds, 0).astype(np.uint8), pres.reshape(-1), rr, cr)
    assert rc == 0 and np.array_equal(rep, eds) and p2.all()
    # (ii) random 50%
    rng = np.random.default_rng(2)
    ok = 0
    for _ in range(5):
        pres = (rng.random(w * w) < 0.5).astype(np.uint8)
        rc, rep, p2, _, _ = O.repair(np.where(pres[:, None] == 1, eds, 0).astype(np.uint8), pres, rr, cr)
        if rc == 0:
            ok += 1
            assert np.array_equal(rep, eds)
        else:
            assert rc == O.E_UNREPAIRABLE
    # (iii) 25% random: unrepairable
    pres = (rng.random(w * w) < 0.25).astype(np.uint8)
    rc, *_ = O.repair(np.where(pres[:, None] == 1, eds, 0).astype(np.uint8), pres, rr, cr)
    assert rc == O.E_UNREPAIRABLE


def test_repair_byzantine():
    k = 4
    ods = O.gen_ods(k, 12)
    rc, eds, rr, cr, dah = O.extend_commit(ods)
    w = 2 * k
    bad = eds.copy()
    bad[1 * w + 5, 100] ^= 1  # corrupt a parity cell of complete row 1
    pres = np.ones(w * w, np.uint8)
    pres[3 * w + 0] = 0
    rc, _, _, ax, ix = O.repair(bad, pres, rr, cr)
    assert rc == O.E_BYZANTINE and ax == 0 and ix == 1


def test_bench_generator_matches_oracle_generator():
    """bench.py's numpy generator == oracle ora_gen_ods (same SplitMix64 stream, memcmp sort)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for k in (1, 4, 16):
        assert np.array_equal(bench.gen_ods(k, 0xC0FFEE + k), O.gen_ods(k, 0xC0FFEE + k))


# ---- real-data pin: Celestia mainnet block 408 (reference fixture) -------------------------
def _mainnet():
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mainnet_h408.npz")
    z = np.load(p)  # allow_pickle=False (default): plain arrays written by tests/golden/make_mainnet_block.py
    return z["ods"], z["data_hash"].tobytes()


def test_oracle_reproduces_mainnet_block_408_data_hash():
    """ODS built from x/blob/test/testdata/block_response.json; its data_hash pins Leopard FF8 + NMT + DAH."""
    ods, want = _mainnet()
    assert ods.shape == (1024, 512)
    rc, eds, rr, cr, dah = O.extend_commit(ods)
    assert rc == 0 and dah == want
    # non-constant data: parity differs from the data it encodes
    e = eds.reshape(64, 64, 512)
    assert not np.array_equal(e[:32, 32:], e[:32, :32])


def test_oracle_matches_committed_digests():
    """Regression pin: the oracle's outputs on the seeded squares equal tests/golden/oracle_digests.json."""
    import hashlib
    import json
    import os
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_digests.json")))
    for ks in ("1", "8", "32", "64"):
        k = int(ks)
        rc, eds, rr, cr, dah = O.extend_commit(O.gen_ods(k, fx[ks]["seed"]))
        assert rc == 0 and dah.hex() == fx[ks]["dah"]
        assert hashlib.sha256(eds.tobytes()).hexdigest() == fx[ks]["eds_sha256"]
        assert hashlib.sha256(rr.tobytes() + cr.tobytes()).hexdigest() == fx[ks]["roots_sha256"]


def test_leopard_reconstruct_matches_lagrange():
    """ora_leo_decode_fft (klauspost's reconstruct restated: error locators, IFFT, formal derivative, FFT; the CPU
    baseline's decoder) returns the same shards as the independent Lagrange decoder, FF8 and FF16, ragged k."""
    rng = np.random.default_rng(5)
    for k in (1, 2, 3, 8, 33, 128, 129, 300):
        data = rng.integers(0, 256, (k, 64), dtype=np.uint8)
        sh = np.concatenate([data, O.leo_encode(data)])
        pres = np.zeros(2 * k, np.uint8)
        pres[rng.permutation(2 * k)[:k]] = 1
        bad = sh.copy()
        bad[pres == 0] = 0x5A
        rc1, a = O.leo_decode(bad, pres)
        rc2, b = O.leo_decode(bad, pres, fft=True)
        assert rc1 == rc2 == 0 and np.array_equal(a, sh) and np.array_equal(b, sh), k


def test_repair_fft_decoder_matches_lagrange():
    k, w = 16, 32
    rc, eds, rr, cr, dah = O.extend_commit(O.gen_ods(k, 77))
    pres = (np.random.default_rng(3).random(w * w) < 0.5).astype(np.uint8)
    d = eds.copy()
    d[pres == 0] = 0
    r0 = O.repair(d, pres, rr, cr)
    r1 = O.repair(d, pres, rr, cr, fft=True)
    assert r0[0] == r1[0] == 0 and np.array_equal(r0[1], eds) and np.array_equal(r1[1], eds)
