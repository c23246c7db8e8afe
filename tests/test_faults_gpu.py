"""The C ABI's exception barrier on the device paths: a host allocation failure or a
helper thread that cannot start comes back as CDA_E_NOMEM / CDA_E_INTERNAL -- never std::terminate inside the
caller -- and the context stays usable.  Faults are injected with CDA_FAULT_INJECT (ctx.h: fault_point), which only
the test-hooks build honours (libcda_hooks.so, -DCDA_TEST_HOOKS=1); the release library ignores it (VERDICT r04 #3,
last test)."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


def test_injected_faults_return_codes_and_context_survives(monkeypatch):
    import cda
    from cda import _native as N
    c = cda.Context(0, lib_path=N.HOOKS_LIB_PATH)  # fresh context: its workspace is empty, so the first call grows it
    try:
        k = 16
        ods = O.gen_ods(k, 5)
        batch = np.stack([O.gen_ods(k, 40 + b) for b in range(6)])
        monkeypatch.setenv("CDA_FAULT_INJECT", "alloc")  # device workspace growth throws std::bad_alloc
        with pytest.raises(cda.CdaError) as ei:
            c.extend_commit(ods)
        assert ei.value.code == N.E_NOMEM
        monkeypatch.setenv("CDA_FAULT_INJECT", "thread")  # the pipeline's second helper thread fails to start
        with pytest.raises(cda.CdaError) as ei:
            c.extend_commit_batch(batch)
        assert ei.value.code == N.E_INTERNAL
        monkeypatch.delenv("CDA_FAULT_INJECT")
        eds, rr, cr, dah = c.extend_commit(ods)
        w = 2 * k
        present = np.zeros(w * w, np.uint8)
        present.reshape(w, w)[:k, :k] = 1
        damaged = eds.copy()
        damaged[present == 0] = 0
        monkeypatch.setenv("CDA_FAULT_INJECT", "thread")  # repair: thrown while its upload thread runs
        with pytest.raises(cda.CdaError) as ei:
            c.repair(damaged, present, rr, cr)
        assert ei.value.code == N.E_INTERNAL
        monkeypatch.delenv("CDA_FAULT_INJECT")
        # the same context afterwards: every path bit-exact again
        rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
        eds2, rr2, cr2, dah2 = c.extend_commit(ods)
        assert np.array_equal(eds2, eds_o) and dah2 == dah_o
        e3, r3, c3, d3 = c.extend_commit_batch(batch)
        for b in range(len(batch)):
            assert d3[b].tobytes() == O.extend_commit(batch[b])[4]
        out, pres = c.repair(damaged, present, rr, cr)
        assert np.array_equal(out, eds) and pres.all()
    finally:
        c.close()


def test_release_library_is_bit_exact_with_fault_injection_set(monkeypatch):
    """With CDA_FAULT_INJECT set to every site, the release libcda.so (no test hooks compiled in) grows a fresh
    context's workspace, runs the one-block path (copy-pool threads), a batch (helper threads) and a repair, and
    returns bit-exact results: no environment variable can make a release build fail."""
    import cda
    from cda import _native as N
    assert N.build_info().startswith("release gfx950")
    for site in ("alloc", "thread", "entry"):
        monkeypatch.setenv("CDA_FAULT_INJECT", site)
        c = cda.Context(0)  # fresh: every workspace buffer and helper thread is created under the variable
        try:
            k = 16
            ods = O.gen_ods(k, 77)
            rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(ods)
            eds, rr, cr, dah = c.extend_commit(ods)
            assert np.array_equal(eds, eds_o) and np.array_equal(rr, rr_o) and dah == dah_o
            batch = np.stack([O.gen_ods(k, 90 + b) for b in range(4)])
            _, _, _, d3 = c.extend_commit_batch(batch)
            for b in range(len(batch)):
                assert d3[b].tobytes() == O.extend_commit(batch[b])[4]
            w = 2 * k
            present = np.zeros(w * w, np.uint8)
            present.reshape(w, w)[:k, :k] = 1
            damaged = eds.copy()
            damaged[present == 0] = 0
            out, pres = c.repair(damaged, present, rr, cr)
            assert np.array_equal(out, eds) and pres.all()
        finally:
            c.close()
