"""ctypes loader for the CPU oracle (oracle/liboracle.so).

Test infrastructure only: the oracle is the checker for parity tests and the
CPU baseline in bench.py; the product (libcda) never loads it.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None

SHARE = 512
NS = 29
NODE = 90

OK, E_NOT_POW2, E_NOT_SQUARE, E_SHARD_SIZE, E_NS_SHORT, E_NS_ORDER, E_TOO_FEW, \
    E_UNREPAIRABLE, E_BYZANTINE = 0, -1, -2, -3, -4, -5, -6, -7, -8
E_PUSH_PAST = -11
E_SHARE_VERSION, E_BLOB_SIZE = -13, -14


def lib():
    global _LIB
    if _LIB is None:
        # CDA_ORACLE_LIB: another build of the same sources (scripts/sanitize.sh: the ASan/UBSan one)
        path = os.environ.get("CDA_ORACLE_LIB") or os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.ora_sha256.argtypes = [P, ctypes.c_size_t, P]
        L.ora_leo_bits_for.argtypes = [ctypes.c_int]
        L.ora_leo_encode.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P]
        L.ora_leo_decode.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P]
        L.ora_leo_decode_fft.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P]
        L.ora_leo_mul.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_uint]
        L.ora_leo_mul.restype = ctypes.c_uint
        L.ora_leo_skew.argtypes = [ctypes.c_int, ctypes.c_int]
        L.ora_leo_log.argtypes = [ctypes.c_int, ctypes.c_uint]
        L.ora_leo_exp.argtypes = [ctypes.c_int, ctypes.c_uint]
        L.ora_nmt_axis_root.argtypes = [ctypes.c_uint64, ctypes.c_uint64, P, P, ctypes.c_int, P, P]
        L.ora_merkle_root.argtypes = [P, P, ctypes.c_int, P]
        L.ora_extend.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P, ctypes.c_int]
        L.ora_roots.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P, P, ctypes.c_int, P, P]
        L.ora_dah_hash.argtypes = [ctypes.c_int, P, P, P]
        L.ora_extend_commit.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P, P, P, P, ctypes.c_int]
        L.ora_extend_commit_throughput.argtypes = [ctypes.c_int, ctypes.c_size_t, P, ctypes.c_int, ctypes.c_double,
                                                   ctypes.POINTER(ctypes.c_double)]
        L.ora_extend_commit_throughput.restype = ctypes.c_long
        L.ora_repair.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P, P, P, P, P]
        L.ora_repair_ex.argtypes = [ctypes.c_int, ctypes.c_size_t, P, P, P, P, P, P, ctypes.c_int]
        L.ora_gen_ods.argtypes = [ctypes.c_int, ctypes.c_uint64, P]
        _bind_inclusion(L)
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ptr_array(rows):
    arr = (ctypes.c_void_p * len(rows))()
    for i, r in enumerate(rows):
        arr[i] = r.ctypes.data
    return arr


def sha256(b: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    buf = np.frombuffer(b, np.uint8).copy() if b else np.zeros(1, np.uint8)
    lib().ora_sha256(_p(buf), len(b), _p(out))
    return out.tobytes()


def gen_ods(k: int, seed: int) -> np.ndarray:
    """Namespace-sorted synthetic ODS (k*k, 512) — SURVEY §8d generator."""
    ods = np.zeros((k * k, SHARE), np.uint8)
    lib().ora_gen_ods(k, seed, _p(ods))
    return ods


def leo_encode(data: np.ndarray) -> np.ndarray:
    """data: (k, L) uint8 -> parity (k, L)."""
    data = np.ascontiguousarray(data, np.uint8)
    k, L = data.shape
    par = np.zeros_like(data)
    rows_d = [data[i] for i in range(k)]
    rows_p = [par[i] for i in range(k)]
    rc = lib().ora_leo_encode(k, L, _ptr_array(rows_d), _ptr_array(rows_p))
    if rc != 0:
        raise ValueError(f"ora_leo_encode rc={rc}")
    return par


def leo_decode(shards: np.ndarray, present: np.ndarray, fft: bool = False):
    """shards: (2k, L) with garbage where missing; returns (rc, repaired copy).  fft=False: the Lagrange decoder
    (independent check); fft=True: klauspost's Leopard reconstruct (error locators + IFFT/FFT)."""
    sh = np.ascontiguousarray(shards, np.uint8).copy()
    n, L = sh.shape
    pres = np.ascontiguousarray(present, np.uint8)
    rows = [sh[i] for i in range(n)]
    fn = lib().ora_leo_decode_fft if fft else lib().ora_leo_decode
    rc = fn(n // 2, L, _ptr_array(rows), _p(pres))
    return rc, sh


def extend(ods: np.ndarray, nthreads: int = 8) -> np.ndarray:
    n = ods.shape[0]
    k = int(round(n ** 0.5))
    L = ods.shape[1]
    eds = np.zeros((4 * k * k, L), np.uint8)
    lib().ora_extend(k, L, _p(np.ascontiguousarray(ods)), _p(eds), nthreads)
    return eds


def roots(eds: np.ndarray, nthreads: int = 8):
    n = eds.shape[0]
    w = int(round(n ** 0.5))
    k = w // 2
    rr = np.zeros((w, NODE), np.uint8)
    cr = np.zeros((w, NODE), np.uint8)
    ea = np.zeros(1, np.int32)
    ei = np.zeros(1, np.int32)
    rc = lib().ora_roots(k, eds.shape[1], _p(np.ascontiguousarray(eds)), _p(rr), _p(cr), nthreads, _p(ea), _p(ei))
    return rc, rr, cr, int(ea[0]), int(ei[0])


def dah_hash(row_roots: np.ndarray, col_roots: np.ndarray) -> bytes:
    out = np.zeros(32, np.uint8)
    lib().ora_dah_hash(row_roots.shape[0], _p(np.ascontiguousarray(row_roots)),
                       _p(np.ascontiguousarray(col_roots)), _p(out))
    return out.tobytes()


def extend_commit(shares: np.ndarray, want_eds: bool = True, nthreads: int = 8):
    """da.ExtendShares + NewDataAvailabilityHeader. Returns (rc, eds, row_roots, col_roots, dah)."""
    shares = np.ascontiguousarray(shares, np.uint8)
    count, L = shares.shape
    k = max(1, int(round(count ** 0.5)))
    eds = np.zeros((4 * k * k, L), np.uint8) if want_eds else None
    rr = np.zeros((2 * k, NODE), np.uint8)
    cr = np.zeros((2 * k, NODE), np.uint8)
    dah = np.zeros(32, np.uint8)
    rc = lib().ora_extend_commit(count, L, _p(shares), _p(eds) if eds is not None else None,
                                 _p(rr), _p(cr), _p(dah), nthreads)
    return rc, eds, rr, cr, dah.tobytes()


def extend_commit_throughput(shares: np.ndarray, nthreads: int, seconds: float):
    """Blocks/s of single-threaded ExtendShares+NewDataAvailabilityHeader calls run by `nthreads` workers
    on independent copies of one block for `seconds`. Returns (blocks, elapsed_s)."""
    shares = np.ascontiguousarray(shares, np.uint8)
    count, L = shares.shape
    el = ctypes.c_double(0.0)
    n = lib().ora_extend_commit_throughput(count, L, _p(shares), nthreads, seconds, ctypes.byref(el))
    if n < 0:
        raise RuntimeError(f"oracle throughput sample failed: {n}")
    return int(n), el.value


def nmt_axis_root(square_size: int, axis_index: int, leaves):
    arrs = [np.frombuffer(bytes(l), np.uint8).copy() if len(l) else np.zeros(1, np.uint8) for l in leaves]
    lens = np.array([len(l) for l in leaves], np.uint64) if leaves else np.zeros(1, np.uint64)
    root = np.zeros(NODE, np.uint8)
    err = np.zeros(1, np.int32)
    rc = lib().ora_nmt_axis_root(square_size, axis_index, _ptr_array(arrs) if arrs else None,
                                 _p(lens), len(leaves), _p(root), _p(err))
    return rc, root.tobytes(), int(err[0])


def merkle_root(items) -> bytes:
    arrs = [np.frombuffer(bytes(i), np.uint8).copy() if len(i) else np.zeros(1, np.uint8) for i in items]
    lens = np.array([len(i) for i in items], np.uint64) if items else np.zeros(1, np.uint64)
    out = np.zeros(32, np.uint8)
    lib().ora_merkle_root(_ptr_array(arrs) if arrs else None, _p(lens), len(items), _p(out))
    return out.tobytes()


def repair(eds: np.ndarray, present: np.ndarray, row_roots: np.ndarray, col_roots: np.ndarray, fft: bool = False):
    """rsmt2d Repair restated (sequential).  fft selects the decoder as in leo_decode."""
    eds = np.ascontiguousarray(eds, np.uint8).copy()
    pres = np.ascontiguousarray(present, np.uint8).copy()
    w = row_roots.shape[0]
    ea = np.zeros(1, np.int32)
    ei = np.zeros(1, np.int32)
    rc = lib().ora_repair_ex(w // 2, eds.shape[1], _p(eds), _p(pres), _p(np.ascontiguousarray(row_roots)),
                             _p(np.ascontiguousarray(col_roots)), _p(ea), _p(ei), 1 if fft else 0)
    return rc, eds, pres, int(ea[0]), int(ei[0])


# ---- blob share commitments, subtree roots and proofs (oracle/inclusion.c) ----------------
def _bind_inclusion(L):
    P, I, U32, SZ, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int64
    L.ora_sparse_shares_needed.argtypes = [U32]
    L.ora_blob_to_shares.argtypes = [P, P, U32, I, P]
    L.ora_subtree_width.argtypes = [I, I]
    L.ora_blob_min_square_size.argtypes = [I]
    L.ora_mmr_sizes.argtypes = [I, I, P]
    L.ora_blob_commitment.argtypes = [P, P, U32, I, I, P]
    L.ora_subtree_root_coords.argtypes = [I, I, I, I, P]
    L.ora_axis_leaf_nodes.argtypes = [I, P, I, I, P]
    L.ora_nmt_tree_levels.argtypes = [P, I, P]
    L.ora_get_commitment.argtypes = [I, P, I, I, I, P]
    L.ora_nmt_prove_range.argtypes = [P, I, I, I, P]
    L.ora_nmt_verify_inclusion.argtypes = [I, P, P, SZ, I, I, I, P, I, P]
    L.ora_merkle_proof.argtypes = [P, SZ, I, I, P, P, P]
    L.ora_merkle_verify.argtypes = [I64, I64, P, P, I, P, P, SZ]
    L.ora_nmt_hash_node_ns.argtypes = [I, P, P, P]
    L.ora_nmt_leaf_node.argtypes = [P, P, SZ, P]
    L.ora_nmt_root_of_nodes.argtypes = [P, I, P]


def _buf(b):
    b = bytes(b)
    return np.frombuffer(b, np.uint8).copy() if b else np.zeros(1, np.uint8)


def sparse_shares_needed(n):
    return lib().ora_sparse_shares_needed(n)


def blob_to_shares(ns, data, share_version=0):
    """go-square SparseShareSplitter.Write: (n, 512) shares of one blob."""
    n = lib().ora_sparse_shares_needed(len(data))
    out = np.zeros((max(n, 1), SHARE), np.uint8)
    lib().ora_blob_to_shares(_p(_buf(ns)), _p(_buf(data)), len(data), share_version, _p(out))
    return out[:n]


def subtree_width(share_count, threshold=64):
    return lib().ora_subtree_width(share_count, threshold)


def mmr_sizes(total, max_tree):
    n = lib().ora_mmr_sizes(total, max_tree, None)
    out = np.zeros(max(n, 1), np.int32)
    lib().ora_mmr_sizes(total, max_tree, _p(out))
    return [int(x) for x in out[:n]]


def blob_commitment(ns, data, share_version=0, threshold=64):
    """inclusion.CreateCommitment -> (rc, 32-byte commitment)."""
    out = np.zeros(32, np.uint8)
    rc = lib().ora_blob_commitment(_p(_buf(ns)), _p(_buf(data)), len(data), share_version, threshold, _p(out))
    return rc, out.tobytes()


def subtree_root_coords(max_depth, min_depth, start, end):
    n = lib().ora_subtree_root_coords(max_depth, min_depth, start, end, None)
    out = np.zeros(2 * n, np.int32)
    lib().ora_subtree_root_coords(max_depth, min_depth, start, end, _p(out))
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]


def axis_leaf_nodes(eds, axis, index):
    """Erasured leaf nodes (2k, 90) of one EDS row (axis 0) or column (axis 1)."""
    w = int(round(eds.shape[0] ** 0.5))
    out = np.zeros((w, NODE), np.uint8)
    lib().ora_axis_leaf_nodes(w // 2, _p(np.ascontiguousarray(eds)), axis, index, _p(out))
    return out


def tree_levels(leaf_nodes):
    """All levels of the perfect NMT over n leaf nodes: (2n-1, 90), leaves first, root last."""
    leaf_nodes = np.ascontiguousarray(leaf_nodes, np.uint8)
    n = leaf_nodes.shape[0]
    out = np.zeros((2 * n - 1, NODE), np.uint8)
    lib().ora_nmt_tree_levels(_p(leaf_nodes), n, _p(out))
    return out


def get_commitment(eds, start, blob_share_len, threshold=64):
    """pkg/inclusion GetCommitment over a full EDS -> (rc, 32 bytes)."""
    w = int(round(eds.shape[0] ** 0.5))
    out = np.zeros(32, np.uint8)
    rc = lib().ora_get_commitment(w // 2, _p(np.ascontiguousarray(eds)), start, blob_share_len, threshold, _p(out))
    return rc, out.tobytes()


def nmt_prove_range(leaf_nodes, start, end):
    """nmt ProveRange(start, end): list of 90-B proof nodes."""
    leaf_nodes = np.ascontiguousarray(leaf_nodes, np.uint8)
    out = np.zeros((128, NODE), np.uint8)
    c = lib().ora_nmt_prove_range(_p(leaf_nodes), leaf_nodes.shape[0], start, end, _p(out))
    if c < 0:
        raise ValueError("invalid proof range")
    return [out[i].tobytes() for i in range(c)]


def nmt_verify_inclusion(nid, leaves, start, end, nodes, root):
    """nmt Proof.VerifyInclusion (namespace size = len(nid))."""
    leaf_len = len(leaves[0]) if leaves else 0
    return bool(lib().ora_nmt_verify_inclusion(len(nid), _p(_buf(nid)), _p(_buf(b"".join(leaves))), leaf_len,
                                               len(leaves), start, end, _p(_buf(b"".join(nodes))), len(nodes),
                                               _p(_buf(root))))


def merkle_proof(items, index):
    """merkle.ProofsFromByteSlices(items)[index] -> (leaf_hash, aunts, root)."""
    leaf, root = np.zeros(32, np.uint8), np.zeros(32, np.uint8)
    aunts = np.zeros((100, 32), np.uint8)
    na = lib().ora_merkle_proof(_p(_buf(b"".join(items))), len(items[0]), len(items), index, _p(leaf), _p(aunts),
                                _p(root))
    return leaf.tobytes(), [aunts[i].tobytes() for i in range(na)], root.tobytes()


def merkle_verify(total, index, leaf_hash, aunts, root, item):
    """merkle.Proof{Total, Index, LeafHash, Aunts}.Verify(root, item)."""
    return bool(lib().ora_merkle_verify(total, index, _p(_buf(leaf_hash)), _p(_buf(b"".join(aunts))), len(aunts),
                                        _p(_buf(root)), _p(_buf(item)), len(item)))
