"""cda_repair on squares in page-locked caller memory (go/cda's pooled slabs, cda_host_register): a sparse square's
present runs are read by the scatter kernel straight from the registered memory (csrc/repair.cpp, staging.cpp
pinned_device_alias); a square only partly registered takes the staging ring.  Every outcome equals the oracle's
sequential Repair (repaired square, or the partial square and error of an unrepairable one)."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


def _square(k, seed):
    ods = O.gen_ods(k, seed)
    rc, eds, rr, cr, _ = O.extend_commit(ods)
    assert rc == 0
    return eds, rr, cr


@pytest.mark.parametrize("case", ["q0_only", "sparse_random", "unrepairable"])
@pytest.mark.parametrize("where", ["whole", "interior", "half_registered"])
def test_repair_in_registered_memory_matches_oracle(ctx, case, where):
    k, w = 64, 128
    eds, rr, cr = _square(k, 0x1234)
    rng = np.random.default_rng(hash((case, where)) & 0xFFFF)
    if case == "q0_only":
        present = np.zeros((w, w), np.uint8)
        present[:k, :k] = 1
        present = present.reshape(-1)
    else:
        present = (rng.random(w * w) < (0.45 if case == "sparse_random" else 0.2)).astype(np.uint8)
    damaged = np.where(present[:, None] == 1, eds, 0).astype(np.uint8)
    orc, oeds, opres, _, _ = O.repair(damaged, present, rr, cr)
    # the caller's slab: the square alone, inside a larger registered buffer, or with only its first half registered
    extra = 256 if where == "interior" else 0
    backing = np.zeros((w * w + 2 * extra, 512), np.uint8)
    square = backing[extra:extra + w * w]
    square[:] = damaged
    reg = backing if where != "half_registered" else backing[: (w * w) // 2]
    ctx.host_register(reg)
    try:
        pres = present.copy()
        rc, _, _, _ = ctx.repair_status(square, pres, rr, cr, inplace=True)
        assert rc == orc
        assert np.array_equal(pres, opres)
        assert np.array_equal(square[pres == 1], oeds[opres == 1])
        if orc == 0:
            assert np.array_equal(square, eds)
    finally:
        ctx.host_unregister(reg)


@pytest.mark.parametrize("where", ["whole", "half_registered"])
def test_one_block_output_in_registered_memory(ctx, where):
    """The one-block path with its EDS output page-locked whole (one DMA for the bottom half) or only in part (a
    partly registered range is treated as pageable): bit-exact either way."""
    k = 128
    ods = O.gen_ods(k, 0x4242)
    rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
    out = np.full((1, 4 * k * k, 512), 0x5A, np.uint8)
    reg = out if where == "whole" else out[0, : 2 * k * k]
    ctx.host_register(reg)
    try:
        _, rr, cr, dah = ctx.extend_commit_batch(ods[None].copy(), eds_out=out)
        assert np.array_equal(out[0], eds_o) and np.array_equal(rr[0], rr_o) and bytes(dah[0]) == dah_o
    finally:
        ctx.host_unregister(reg)
