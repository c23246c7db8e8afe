"""CPU tests of the C-ABI boundary: libcda.so loads and exports every symbol of include/cda.h.

No compute is called here (no GPU in the build container).
"""
import os
import re

import cda
from cda import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "cda.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cda_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_what_binding_binds():
    assert header_functions() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = cda.lib()
    for name in header_functions():
        assert hasattr(L, name), name


def test_pure_host_entry_points():
    L = cda.lib()
    assert L.cda_rs_name() == b"Leopard"
    assert L.cda_rs_max_chunks() == 32768 * 32768
    assert L.cda_rs_validate_chunk_size(512) == 0
    assert L.cda_rs_validate_chunk_size(100) == N.E_SHARD_SIZE
    assert N.strerror(N.E_NS_ORDER).startswith("pushed data")


def test_error_codes_match_header():
    src = open(os.path.join(ROOT, "include", "cda.h")).read()
    codes = dict((m[0], int(m[1])) for m in re.findall(r"(CDA_E_[A-Z0-9_]+)\s*=\s*(-?\d+)", src))
    for name, val in codes.items():
        assert getattr(N, name[4:]) == val, name


def test_wrapper_push_errors_without_gpu():
    # push-time checks mirror nmt_wrapper.go:93-114 and need no device
    from cda.wrapper import ErasuredNamespacedMerkleTree, PushError
    import pytest
    t = ErasuredNamespacedMerkleTree(16, 0)
    with pytest.raises(PushError):
        t.push(b"\x01")
    t = ErasuredNamespacedMerkleTree(2, 0)
    for _ in range(4):
        t.push(b"\x00" * 512)
    with pytest.raises(PushError):
        t.push(b"\x00" * 512)
    t = ErasuredNamespacedMerkleTree(4, 0)
    t.push(b"\x01" * 512)
    with pytest.raises(PushError):
        t.push(b"\x00" * 512)


def test_new_entry_points_reject_null_context_without_gpu():
    # argument checks run before any device work (include/cda.h contract: negative codes, no abort)
    L = cda.lib()
    assert L.cda_blob_commitments(None, 1, None, None, None, None, 64, None, None) == N.E_ARG
    assert L.cda_merkle_roots(None, 1, None, None, 90, None) == N.E_ARG
    assert L.cda_extend_commit_nodes(None, 4, 512, None, None, None, None, None, None, None, None, None) == N.E_ARG
    assert L.cda_share_inclusion_proof(None, 4, 512, None, 0, 1, None, None, None, None, None, None, None, None,
                                       None, None) == N.E_ARG
    assert N.strerror(N.E_BLOB_SIZE) == "cannot use zero blob size"
    assert N.strerror(N.E_SHARE_VERSION) == "unsupported share version"


def test_exception_barrier_without_gpu(monkeypatch):
    """No C++ exception crosses the C ABI (no abort; app/process_proposal.go:28-34 recovers Go panics
    only): an exception injected at entry (CDA_FAULT_INJECT=entry throws std::bad_alloc before the body runs) comes
    back as CDA_E_NOMEM from every kind of entry point, not as std::terminate.  Injection exists only in the
    test-hooks build (libcda_hooks.so)."""
    L = N.lib(N.HOOKS_LIB_PATH)
    assert "test_hooks" in N.build_info(N.HOOKS_LIB_PATH)
    monkeypatch.setenv("CDA_FAULT_INJECT", "entry")
    assert L.cda_merkle_roots(None, 1, None, None, 90, None) == N.E_NOMEM
    assert L.cda_repair(None, 8, None, None, None, None, None) == N.E_NOMEM
    assert L.cda_extend_commit(None, 4, 512, None, None, None, None, None, None) == N.E_NOMEM
    assert L.cda_multi_extend_commit_batch(None, 8, 1, None, None, None, None, None, None) == N.E_NOMEM
    monkeypatch.delenv("CDA_FAULT_INJECT")
    assert L.cda_merkle_roots(None, 1, None, None, 90, None) == N.E_ARG
    assert N.strerror(N.E_NOMEM) == "out of host memory"
    assert N.strerror(N.E_INTERNAL).startswith("internal error")


def test_release_library_ignores_fault_injection(monkeypatch):
    """the release libcda.so carries no test hook -- with CDA_FAULT_INJECT set at every site it still
    runs its argument checks (CDA_E_ARG for a null context, not the injected CDA_E_NOMEM) and says it is a release
    build.  The GPU side of this check (bit-exact results with the variable set) is tests/test_faults_gpu.py."""
    L = cda.lib()
    assert N.build_info().startswith("release gfx950")
    for site in ("entry", "alloc", "thread"):
        monkeypatch.setenv("CDA_FAULT_INJECT", site)
        assert L.cda_merkle_roots(None, 1, None, None, 90, None) == N.E_ARG
        assert L.cda_extend_commit(None, 4, 512, None, None, None, None, None, None) == N.E_ARG
        assert L.cda_set_option(None, N.OPT_HUGE_PAGES, 1) == N.E_ARG
        assert L.cda_host_register(None, None, 0) == N.E_ARG
        assert L.cda_extend_commit_eds(None, 8, None, None, None, None, None) == N.E_ARG


def test_release_library_reads_no_environment_per_call():
    """the product path reads its A/B knobs once at cda_init (ctx fields), never per call -- no getenv
    outside cda_init's knob block, a function-local static, the test hooks and the diagnostic builds' trace hooks."""
    import glob
    csrc = os.path.join(ROOT, "celestia-app_amd", "csrc")
    for path in glob.glob(os.path.join(csrc, "*.cpp")) + glob.glob(os.path.join(csrc, "*.hip")):
        src = open(path).read()
        for m in re.finditer(r"getenv\(", src):
            line_start = src.rfind("\n", 0, m.start()) + 1
            line = src[line_start:src.find("\n", m.start())]
            ctx_before = src[max(0, m.start() - 1500):m.start()]
            ok = ("static" in line or "static const" in ctx_before[-400:] or "cda_init" in ctx_before
                  or "CDA_TEST_HOOKS" in ctx_before or "TRACE" in line or "find_local_cpus" in ctx_before
                  or "CDA_NUMA_BIND" in line)
            assert ok, f"{os.path.basename(path)}: per-call getenv: {line.strip()}"


# The A/B switches of the measured experiments: test / diagnostic builds only.
AB_KNOBS = ("CDA_CONSENSUS", "CDA_CONS_IN", "CDA_CONS_OUT", "CDA_CONS_STG", "CDA_CONS_TRACE", "CDA_RS16",
            "CDA_RS16_LDS_KB", "CDA_RS8_LAT_U", "CDA_REPAIR_OVERLAP", "CDA_REPAIR_FUSED", "CDA_REPAIR_EARLY",
            "CDA_REPAIR_TRACE", "CDA_STAGING", "CDA_TREES_LDS", "CDA_HUGE_PAGES", "CDA_FAULT_INJECT", "CDA_AXIS_SLOTS")


def test_release_library_ignores_ab_knobs():
    """a release libcda.so cannot read an A/B switch -- none of their names is in the library (so no
    getenv of them can happen), while the test-hooks build that the A/B and fault tests load carries every one; the
    deployment options CDA_NUMA_BIND and CDA_COPY_THREADS are the release build's only environment inputs, and
    cda_build_info() names them."""
    rel = open(N.LIB_PATH, "rb").read()
    hooks = open(N.HOOKS_LIB_PATH, "rb").read()
    for name in AB_KNOBS:
        assert name.encode() + b"\0" not in rel, f"release library names {name}"
        assert name.encode() + b"\0" in hooks, f"test-hooks library lacks {name}"
    for name in ("CDA_NUMA_BIND", "CDA_COPY_THREADS"):
        assert name.encode() + b"\0" in rel
        assert name in N.build_info()
