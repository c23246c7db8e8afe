"""Host logic of the upstream-shaped rsmt2d mirror (cda.rsmt2d.compute_extended_data_square_axes / repair_axes) on the
CPU: the same orchestration the GPU tests run over libcda's per-axis seams, here over a codec and a tree constructor
backed by the oracle, so the axis order, fan-out, crossword rules and error cases are checked without a device.  The
oracle is only the stand-in codec / tree and the checker here; the product path under test is the Python caller."""
import numpy as np
import pytest

import oracle_lib as O
from cda import _native as N
from cda import rsmt2d


class OracleCodec:
    """rsmt2d.Codec over the oracle (test stand-in for cda.rsmt2d.LeoRSCodec)."""

    def encode(self, data):
        return [bytes(p) for p in O.leo_encode(np.stack([np.frombuffer(bytes(d), np.uint8) for d in data]))]

    def decode(self, shards):
        if not any(s is not None for s in shards):
            raise N.CdaError(N.E_TOO_FEW)
        L = max(len(s) for s in shards if s is not None)
        arr = np.zeros((len(shards), L), np.uint8)
        pres = np.zeros(len(shards), np.uint8)
        for i, s in enumerate(shards):
            if s is not None:
                arr[i] = np.frombuffer(bytes(s), np.uint8)
                pres[i] = 1
        if pres.sum() < len(shards) // 2:
            raise N.CdaError(N.E_TOO_FEW)
        rc, out = O.leo_decode(arr, pres, fft=True)
        assert rc == 0
        return [bytes(r) for r in out]

    def max_chunks(self):
        return 32768 * 32768


class OracleTree:
    def __init__(self, k, idx):
        self.k, self.idx, self.leaves = k, idx, []

    def push(self, share):
        self.leaves.append(bytes(share))

    def root(self):
        rc, r, _ = O.nmt_axis_root(self.k, self.idx, self.leaves)
        if rc:
            raise ValueError(f"oracle tree rc {rc}")
        return r


def ctor(k):
    return lambda axis, idx: OracleTree(k, idx)


@pytest.mark.parametrize("k", [1, 4, 16])
def test_extension_axes_equals_fused_oracle(k):
    ods = O.gen_ods(k, 0x77 + k)
    sq = rsmt2d.compute_extended_data_square_axes([bytes(r) for r in ods], OracleCodec(), ctor(k), workers=4)
    rc, eds, rr, cr, _ = O.extend_commit(ods)
    assert rc == 0 and np.array_equal(sq.cells, eds)
    assert sq.row_roots() == [bytes(r) for r in rr] and sq.col_roots() == [bytes(c) for c in cr]


def test_extension_axes_rejects_non_square():
    with pytest.raises(ValueError):
        rsmt2d.compute_extended_data_square_axes([bytes(512)] * 3, OracleCodec(), ctor(2))


@pytest.mark.parametrize("k,frac", [(4, 0.5), (8, 0.55), (8, 0.2)])
def test_repair_axes_equals_oracle(k, frac):
    ods = O.gen_ods(k, 0x99 + k)
    rc, eds, rr, cr, _ = O.extend_commit(ods)
    w = 2 * k
    present = (np.random.default_rng(k + int(frac * 100)).random(w * w) < frac).astype(np.uint8)
    orc, oeds, opres, oax, oidx = O.repair(np.where(present[:, None] == 1, eds, 0), present, rr, cr)
    sq = rsmt2d.import_extended_data_square([bytes(eds[i]) if present[i] else None for i in range(w * w)],
                                            OracleCodec())
    if orc == 0:
        rsmt2d.repair_axes(sq, rr, cr, ctor(k))
        assert np.array_equal(sq.cells, eds)
    else:
        assert orc == O.E_UNREPAIRABLE
        with pytest.raises(rsmt2d.ErrUnrepairableDataSquare):
            rsmt2d.repair_axes(sq, rr, cr, ctor(k))
        assert np.array_equal(sq.present, opres)


@pytest.mark.parametrize("missing", [True, False])
def test_repair_axes_byzantine_equals_oracle(missing):
    """A corrupted cell, with cells missing (crossword) or in a complete square (prerepairSanityCheck)."""
    k, w = 4, 8
    ods = O.gen_ods(k, 0x31)
    rc, eds, rr, cr, _ = O.extend_commit(ods)
    present = (np.random.default_rng(9).random(w * w) < 0.6).astype(np.uint8) if missing else np.ones(w * w, np.uint8)
    bad = eds.copy()
    idx = int(np.flatnonzero(present)[3])
    bad[idx, 200] ^= 1
    orc, _, _, oax, oidx = O.repair(np.where(present[:, None] == 1, bad, 0), present, rr, cr)
    assert orc == O.E_BYZANTINE
    sq = rsmt2d.import_extended_data_square([bytes(bad[i]) if present[i] else None for i in range(w * w)],
                                            OracleCodec())
    with pytest.raises(rsmt2d.ErrByzantineData) as ei:
        rsmt2d.repair_axes(sq, rr, cr, ctor(k))
    assert (ei.value.axis, ei.value.index) == (oax, oidx)
