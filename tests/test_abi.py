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
    back as CDA_E_NOMEM from every kind of entry point, not as std::terminate."""
    L = cda.lib()
    monkeypatch.setenv("CDA_FAULT_INJECT", "entry")
    assert L.cda_merkle_roots(None, 1, None, None, 90, None) == N.E_NOMEM
    assert L.cda_repair(None, 8, None, None, None, None, None) == N.E_NOMEM
    assert L.cda_extend_commit(None, 4, 512, None, None, None, None, None, None) == N.E_NOMEM
    assert L.cda_multi_extend_commit_batch(None, 8, 1, None, None, None, None, None, None) == N.E_NOMEM
    monkeypatch.delenv("CDA_FAULT_INJECT")
    assert L.cda_merkle_roots(None, 1, None, None, 90, None) == N.E_ARG
    assert N.strerror(N.E_NOMEM) == "out of host memory"
    assert N.strerror(N.E_INTERNAL).startswith("internal error")
