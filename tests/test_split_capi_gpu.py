"""One square split over devices behind the C ABI (cda_multi_extend_commit_split).

On a one-GPU box the G = 2 / 4 / 8 plans run through cda_multi_init_replicas: G contexts on the same device whose
exchanges are device copies, with the same plan and kernels as the RCCL transport.  Everything is bit-exact against
the CPU oracle (EDS bytes, all 4k roots, DAH) and against the block path; push-order errors match cda_extend_commit.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


def _multi(G):
    import cda
    return cda.MultiContext.replicas(0, G)


@pytest.mark.parametrize("k,G", [(2, 1), (2, 2), (8, 1), (8, 2), (8, 8), (16, 4), (64, 2), (128, 1), (128, 8),
                                 (256, 4), (512, 1), (512, 2), (512, 8)])
def test_split_matches_oracle(k, G):
    ods = O.gen_ods(k, 0x5EED + k + G)
    rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
    assert rc == 0
    m = _multi(G)
    try:
        for rep in range(2):  # second call reuses the handle's workspace
            eds, rr, cr, dah = m.extend_commit_split(ods)
            assert np.array_equal(rr, rr_o) and np.array_equal(cr, cr_o), f"roots differ (k={k}, G={G}, call {rep})"
            assert dah == dah_o
            assert np.array_equal(eds, eds_o), f"EDS differs (k={k}, G={G})"
    finally:
        m.close()


def test_split_roots_only_and_device_input():
    import torch
    k, G = 128, 4
    ods = O.gen_ods(k, 99)
    rc, _, rr_o, cr_o, dah_o = O.extend_commit(ods, want_eds=False)
    m = _multi(G)
    try:
        eds, rr, cr, dah = m.extend_commit_split(ods, want_eds=False)
        assert eds is None and dah == dah_o and np.array_equal(rr, rr_o) and np.array_equal(cr, cr_o)
        rows = torch.from_numpy(ods.reshape(k, k, 512)).cuda()
        rp = k // G
        slabs = [rows[g * rp:(g + 1) * rp].contiguous() for g in range(G)]
        torch.cuda.synchronize()
        rr2, cr2, dah2 = m.extend_commit_split_device(k, [s.data_ptr() for s in slabs])
        assert dah2 == dah_o and np.array_equal(rr2, rr_o) and np.array_equal(cr2, cr_o)
    finally:
        m.close()


@pytest.mark.parametrize("k,G", [(512, 8), (512, 4), (256, 8)])
def test_split_device_input_matches_oracle_dah(k, G):
    """cda_multi_extend_commit_split_device -- each device's ODS row slab already in its HBM, the form a multi-GPU
    node feeds config C5 with -- at k = 512 over G = 8: every root and the DAH equal the
    oracle's (the replica transport runs the same plan and kernels as RCCL)."""
    import torch
    ods = O.gen_ods(k, 0xC0FFEE)
    rc, _, rr_o, cr_o, dah_o = O.extend_commit(ods, want_eds=False)
    assert rc == 0
    m = _multi(G)
    try:
        rows = torch.from_numpy(ods.reshape(k, k, 512)).cuda()
        rp = k // G
        slabs = [rows[g * rp:(g + 1) * rp].contiguous() for g in range(G)]
        torch.cuda.synchronize()
        for _ in range(2):
            rr, cr, dah = m.extend_commit_split_device(k, [sl.data_ptr() for sl in slabs])
            assert dah == dah_o and np.array_equal(rr, rr_o) and np.array_equal(cr, cr_o)
    finally:
        m.close()


@pytest.mark.parametrize("G", [1, 2, 4])
def test_split_push_order_errors_match_block_path(ctx, G):
    """Swapped shares: a row violation, a column violation, a swap that breaks no axis order (row 4's last share
    with row 5's first) and one across the row blocks of two devices -- same outcome and error detail as
    cda_extend_commit."""
    import cda

    def outcome(fn, ods):
        try:
            fn(ods)
            return None
        except cda.CdaError as e:
            return (e.code, e.axis, e.index, e.leaf)
    k = 16
    m = _multi(G)
    try:
        seen_error = 0
        for swap in ((3 * k + 5, 3 * k + 6), (2 * k + 7, 3 * k + 7), (5 * k - 1, 5 * k), (7 * k + 2, 8 * k + 2)):
            ods = O.gen_ods(k, 1234)
            ods[list(swap)] = ods[list(swap[::-1])]
            want = outcome(ctx.extend_commit, ods)
            assert outcome(m.extend_commit_split, ods) == want, swap
            seen_error += want is not None
        assert seen_error == 3
    finally:
        m.close()


def test_split_over_visible_devices():
    """The RCCL transport over every visible device (device mask 0); on a one-GPU box this is G = 1."""
    import cda
    m = cda.MultiContext(0)
    try:
        G = m.device_count
        k = 64 if 64 % G == 0 else 128
        ods = O.gen_ods(k, 7)
        rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
        eds, rr, cr, dah = m.extend_commit_split(ods)
        assert dah == dah_o and np.array_equal(eds, eds_o)
    finally:
        m.close()


def test_split_rejects_bad_device_counts():
    import cda
    m = _multi(3)
    try:
        with pytest.raises(cda.CdaError) as ei:
            m.extend_commit_split(O.gen_ods(8, 1))
        assert ei.value.code == cda._native.E_ARG
    finally:
        m.close()
    m = _multi(4)
    try:
        with pytest.raises(cda.CdaError):
            m.extend_commit_split(O.gen_ods(2, 1))  # k = 2 < G
    finally:
        m.close()
