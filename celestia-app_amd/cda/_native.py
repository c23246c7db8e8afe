"""ctypes binding of libcda.so (include/cda.h).

The product path: every compute call goes through the HIP library.  There is
no CPU fallback — if libcda.so is missing or no GPU is visible the calls raise.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CDA_LIB: another build of the library (A/B measurements of kernel variants on one box)
LIB_PATH = os.environ.get("CDA_LIB") or os.path.join(_HERE, "libcda.so")
# the test-hooks build of the same sources (-DCDA_TEST_HOOKS=1, `make hooks`): failure injection through
# CDA_FAULT_INJECT, which a release libcda.so ignores.  Only the fault tests load it, beside the release library.
HOOKS_LIB_PATH = os.path.join(_HERE, "libcda_hooks.so")

SHARE_SIZE = 512
NAMESPACE_SIZE = 29
NODE_SIZE = 90
HASH_SIZE = 32
REC_BYTES = 96

OK = 0
E_NOT_POW2 = -1
E_NOT_SQUARE = -2
E_SHARD_SIZE = -3
E_NS_SHORT = -4
E_NS_ORDER = -5
E_TOO_FEW = -6
E_UNREPAIRABLE = -7
E_BYZANTINE = -8
E_ARG = -9
E_DEVICE = -10
E_PUSH_PAST = -11
E_UNSUPPORTED = -12
E_SHARE_VERSION = -13
E_BLOB_SIZE = -14
E_NOMEM = -15
E_INTERNAL = -16

AXIS_ROW = 0
AXIS_COL = 1

# Every symbol declared in include/cda.h (checked by tests/test_abi.py).
EXPORTS = [
    "cda_init", "cda_free", "cda_strerror", "cda_last_device_error", "cda_build_info",
    "cda_rs_encode", "cda_rs_decode", "cda_rs_max_chunks", "cda_rs_name", "cda_rs_validate_chunk_size",
    "cda_extend_commit", "cda_extend_commit_batch", "cda_extend_commit_device", "cda_commit_eds", "cda_extend_commit_eds",
    "cda_dah_hash", "cda_nmt_axis_root", "cda_repair", "cda_repair_device",
    "cda_rs_encode_device", "cda_nmt_roots_device", "cda_nmt_fold_device", "cda_dah_device",
    "cda_profile_enable", "cda_profile_read", "cda_profile_reset",
    "cda_blob_commitments", "cda_merkle_roots", "cda_extend_commit_nodes", "cda_share_inclusion_proof",
    "cda_host_alloc", "cda_host_free", "cda_multi_init", "cda_multi_free", "cda_multi_device_count",
    "cda_multi_context", "cda_multi_device", "cda_multi_extend_commit_batch", "cda_build_ods_device",
    "cda_construct_extend_commit", "cda_multi_extend_commit_split", "cda_multi_extend_commit_split_device",
    "cda_multi_init_replicas", "cda_set_option", "cda_host_register", "cda_host_unregister",
]

OPT_HUGE_PAGES = 1


class ErrInfo(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("axis", ctypes.c_int32), ("index", ctypes.c_int32),
                ("leaf", ctypes.c_int32), ("block", ctypes.c_int32)]


class ShareSegment(ctypes.Structure):
    """cda_share_segment (include/cda.h): one run of shares of a square plan."""
    _fields_ = [("kind", ctypes.c_uint32), ("first_share", ctypes.c_uint32), ("nshares", ctypes.c_uint32),
                ("share_version", ctypes.c_uint32), ("data_off", ctypes.c_uint64), ("data_len", ctypes.c_uint64),
                ("reserved_off", ctypes.c_uint32), ("ns", ctypes.c_uint8 * 29), ("pad_", ctypes.c_uint8 * 3)]


class ShareProofInfo(ctypes.Structure):
    _fields_ = [("start_row", ctypes.c_uint32), ("end_row", ctypes.c_uint32), ("nrows", ctypes.c_uint32),
                ("total", ctypes.c_uint32), ("naunts", ctypes.c_uint32), ("max_nodes", ctypes.c_uint32)]


class CdaError(Exception):
    """Error returned by libcda; `code` is a CDA_E_* value."""

    def __init__(self, code, msg="", axis=-1, index=-1, leaf=-1, block=-1):
        self.code, self.axis, self.index, self.leaf, self.block = code, axis, index, leaf, block
        super().__init__(f"{msg or strerror(code)} (code {code}, axis {axis}, index {index}, leaf {leaf})")


_libs = {}
_lib_lock = threading.Lock()


def lib(path=None):
    """Load libcda.so, or the build at `path` (raises if it was not built: no silent fallback)."""
    path = path or LIB_PATH
    with _lib_lock:
        if path not in _libs:
            if not os.path.exists(path):
                raise RuntimeError(f"libcda not built at {path}; run __graft_entry__.build()")
            L = ctypes.CDLL(path)
            P, U32, I32, U64, I64, SZ = (ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64,
                                          ctypes.c_int64, ctypes.c_size_t)
            sig = {
                "cda_init": (I32, [I32, ctypes.POINTER(P)]),
                "cda_free": (None, [P]),
                "cda_strerror": (ctypes.c_char_p, [I32]),
                "cda_last_device_error": (ctypes.c_char_p, [P]),
                "cda_build_info": (ctypes.c_char_p, []),
                "cda_rs_encode": (I32, [P, U32, U32, P, P]),
                "cda_rs_decode": (I32, [P, U32, U32, P, P]),
                "cda_rs_max_chunks": (I64, []),
                "cda_rs_name": (ctypes.c_char_p, []),
                "cda_rs_validate_chunk_size": (I32, [I64]),
                "cda_extend_commit": (I32, [P, U32, U32, P, P, P, P, P, P]),
                "cda_extend_commit_batch": (I32, [P, U32, U32, P, P, P, P, P, P]),
                "cda_extend_commit_device": (I32, [P, U32, U32, P, P, P, P, P, P]),
                "cda_commit_eds": (I32, [P, U32, P, P, P, P, P]),
                "cda_extend_commit_eds": (I32, [P, U32, P, P, P, P, P]),
                "cda_dah_hash": (I32, [P, U32, P, P, P]),
                "cda_nmt_axis_root": (I32, [P, U64, U64, U32, U32, P, P, P]),
                "cda_repair": (I32, [P, U32, P, P, P, P, P]),
                "cda_repair_device": (I32, [P, U32, P, P, P, P, P, P]),
                "cda_rs_encode_device": (I32, [P, U32, U32, U32, P, I64, I64, P, I64, I64, P]),
                "cda_nmt_roots_device": (I32, [P, U32, P, U32, U32, U32, U32, U32, P, P, P]),
                "cda_nmt_fold_device": (I32, [P, U32, U32, P, P, P]),
                "cda_dah_device": (I32, [P, U32, P, P, P]),
                "cda_profile_enable": (I32, [P, I32]),
                "cda_profile_read": (I32, [P, P, SZ, P, P, I32]),
                "cda_profile_reset": (I32, [P]),
                "cda_blob_commitments": (I32, [P, U32, P, P, P, P, U32, P, P]),
                "cda_merkle_roots": (I32, [P, U32, P, P, U32, P]),
                "cda_extend_commit_nodes": (I32, [P, U32, U32, P, P, P, P, P, P, P, P, P]),
                "cda_share_inclusion_proof": (I32, [P, U32, U32, P, U32, U32, P, P, P, P, P, P, P, P, P,
                                                      P]),
                "cda_host_alloc": (I32, [P, SZ, ctypes.POINTER(P)]),
                "cda_host_free": (I32, [P, P]),
                "cda_multi_init": (I32, [U32, ctypes.POINTER(P)]),
                "cda_multi_free": (None, [P]),
                "cda_multi_device_count": (I32, [P]),
                "cda_multi_context": (P, [P, I32]),
                "cda_multi_device": (I32, [P, I32]),
                "cda_multi_extend_commit_batch": (I32, [P, U32, U32, P, P, P, P, P, P]),
                "cda_multi_extend_commit_split": (I32, [P, U32, P, P, P, P, P, P]),
                "cda_multi_extend_commit_split_device": (I32, [P, U32, P, P, P, P, P]),
                "cda_multi_init_replicas": (I32, [I32, U32, ctypes.POINTER(P)]),
                "cda_build_ods_device": (I32, [P, U32, U32, P, P, U64, P, U32, P, P]),
                "cda_construct_extend_commit": (I32, [P, U32, U32, P, P, U64, P, U32, P, P, P, P, P, P]),
                "cda_set_option": (I32, [P, I32, I64]),
                "cda_host_register": (I32, [P, P, SZ]),
                "cda_host_unregister": (I32, [P, P]),
            }
            for name, (res, args) in sig.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _libs[path] = L
    return _libs[path]


def build_info(path=None):
    """cda_build_info(): "release gfx950", or "diagnostic gfx950 <tags>" for a diagnostic or test-hooks build."""
    return lib(path).cda_build_info().decode()


def strerror(code):
    return lib().cda_strerror(code).decode()


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _check(rc, err=None, ctx=None):
    if rc == OK:
        return
    if rc in (E_DEVICE, E_NOMEM, E_INTERNAL) and ctx is not None:
        raise CdaError(rc, strerror(rc) + ": " + ctx._L.cda_last_device_error(ctx._h).decode())
    if err is not None:
        raise CdaError(rc, axis=err.axis, index=err.index, leaf=err.leaf, block=err.block)
    raise CdaError(rc)


class Context:
    """One cda_ctx bound to one HIP device (one process per GPU)."""

    def pinned(self, shape, dtype=np.uint8):
        """Pinned host buffer (cda_host_alloc) for the host-buffer batch path."""
        return PinnedBuffer(self, shape, dtype)

    def __init__(self, device=0, lib_path=None):
        """lib_path: another build of libcda to bind this context to (the test-hooks library); default libcda.so."""
        self._L = lib(lib_path)
        h = ctypes.c_void_p()
        rc = self._L.cda_init(device, ctypes.byref(h))
        if rc != OK:
            raise CdaError(rc, "cda_init failed (no GPU visible?)")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None) and not getattr(self, "_borrowed", False):  # a MultiContext's view: not ours
            self._L.cda_free(self._h)
        self._h = None

    def set_option(self, option, value):
        """cda_set_option (include/cda.h), e.g. OPT_HUGE_PAGES."""
        _check(self._L.cda_set_option(self._h, option, int(value)), ctx=self)

    def host_register(self, array):
        """Page-lock a C-contiguous numpy array's memory for reuse as share / EDS buffers (cda_host_register)."""
        _check(self._L.cda_host_register(self._h, array.ctypes.data_as(ctypes.c_void_p), array.nbytes), ctx=self)

    def host_unregister(self, array):
        _check(self._L.cda_host_unregister(self._h, array.ctypes.data_as(ctypes.c_void_p)), ctx=self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- codec ----
    def rs_encode(self, data):
        data = np.ascontiguousarray(data, np.uint8)
        k, L = data.shape
        parity = np.empty_like(data)
        _check(self._L.cda_rs_encode(self._h, k, L, _p(data), _p(parity)), ctx=self)
        return parity

    def rs_decode(self, shards, present):
        sh = np.ascontiguousarray(shards, np.uint8).copy()
        pres = np.ascontiguousarray(present, np.uint8)
        n, L = sh.shape
        _check(self._L.cda_rs_decode(self._h, n // 2, L, _p(sh), _p(pres)), ctx=self)
        return sh

    # ---- block path ----
    def extend_commit(self, shares, want_eds=True):
        shares = np.ascontiguousarray(shares, np.uint8)
        count, L = shares.shape
        k = max(1, int(round(count ** 0.5)))
        eds = np.empty((4 * k * k, L), np.uint8) if want_eds else None
        rr = np.empty((2 * k, NODE_SIZE), np.uint8)
        cr = np.empty((2 * k, NODE_SIZE), np.uint8)
        dah = np.empty(32, np.uint8)
        err = ErrInfo()
        rc = self._L.cda_extend_commit(self._h, count, L, _p(shares), _p(eds), _p(rr), _p(cr), _p(dah),
                                     ctypes.byref(err))
        _check(rc, err, self)
        return eds, rr, cr, dah.tobytes()

    def extend_commit_batch(self, ods, want_eds=True, eds_out=None):
        """ods: (nblocks, k*k, 512); eds_out: optional preallocated (nblocks, 4k^2, 512) uint8 output."""
        ods, k, eds, rr, cr, dah = _batch_outputs(ods, want_eds, eds_out)
        nb = len(ods)
        err = ErrInfo()
        rc = self._L.cda_extend_commit_batch(self._h, k, nb, _p(ods), _p(eds), _p(rr), _p(cr), _p(dah),
                                           ctypes.byref(err))
        _check(rc, err, self)
        return eds, rr, cr, dah

    def construct_extend_commit(self, k, segs, want_ods=False, want_eds=True, prepared=None):
        """square.Construct + ExtendShares + NewDataAvailabilityHeader from a square plan (cda.square.plan):
        the shares are assembled on the device (cda_construct_extend_commit).  -> (ods, eds, rr, cr, dah).
        prepared: cda.square.device_plan(segs) computed beforehand (the C-ABI records)."""
        from .square import device_plan
        recs, data, reserved = prepared if prepared is not None else device_plan(segs)
        w = 2 * k
        ods = np.empty((k * k, SHARE_SIZE), np.uint8) if want_ods else None
        eds = np.empty((w * w, SHARE_SIZE), np.uint8) if want_eds else None
        rr = np.empty((w, NODE_SIZE), np.uint8)
        cr = np.empty((w, NODE_SIZE), np.uint8)
        dah = np.empty(32, np.uint8)
        err = ErrInfo()
        rc = self._L.cda_construct_extend_commit(self._h, k, len(recs), ctypes.cast(recs, ctypes.c_void_p), _p(data),
                                               sum(r.data_len for r in recs), _p(reserved), len(reserved), _p(ods),
                                               _p(eds), _p(rr), _p(cr), _p(dah), ctypes.byref(err))
        _check(rc, err, self)
        return ods, eds, rr, cr, dah.tobytes()

    def extend_commit_device(self, k, nblocks, d_ods, d_eds, d_roots, d_dah, d_status, stream=None):
        rc = self._L.cda_extend_commit_device(self._h, k, nblocks, ctypes.c_void_p(d_ods), ctypes.c_void_p(d_eds),
                                            ctypes.c_void_p(d_roots), ctypes.c_void_p(d_dah),
                                            ctypes.c_void_p(d_status), ctypes.c_void_p(stream or 0))
        _check(rc, ctx=self)

    # ---- device-resident building blocks (pointers are device addresses) ----
    def rs_encode_device(self, k, shard_len, ncw, d_src, src_cw, src_sh, d_dst, dst_cw, dst_sh, stream=None):
        rc = self._L.cda_rs_encode_device(self._h, k, shard_len, ncw, ctypes.c_void_p(d_src), src_cw, src_sh,
                                        ctypes.c_void_p(d_dst), dst_cw, dst_sh, ctypes.c_void_p(stream or 0))
        _check(rc, ctx=self)

    def nmt_roots_device(self, k, d_eds, axis, first_index, naxes, leaf_off, nleaves, d_roots, d_status,
                         stream=None):
        rc = self._L.cda_nmt_roots_device(self._h, k, ctypes.c_void_p(d_eds), axis, first_index, naxes, leaf_off,
                                        nleaves, ctypes.c_void_p(d_roots), ctypes.c_void_p(d_status),
                                        ctypes.c_void_p(stream or 0))
        _check(rc, ctx=self)

    def nmt_fold_device(self, ntrees, n, d_nodes, d_roots, stream=None):
        rc = self._L.cda_nmt_fold_device(self._h, ntrees, n, ctypes.c_void_p(d_nodes), ctypes.c_void_p(d_roots),
                                       ctypes.c_void_p(stream or 0))
        _check(rc, ctx=self)

    def dah_device(self, n_total, d_roots, d_dah, stream=None):
        rc = self._L.cda_dah_device(self._h, n_total, ctypes.c_void_p(d_roots), ctypes.c_void_p(d_dah),
                                  ctypes.c_void_p(stream or 0))
        _check(rc, ctx=self)

    def extend_commit_eds(self, eds):
        """In place (cda_extend_commit_eds): eds (4k^2, 512) uint8, C-contiguous, with the ODS in its top-left quadrant
        (row r of the ODS = eds[r * 2k : r * 2k + k]); Q1..Q3 are written around it.  -> (row_roots, col_roots, dah)."""
        if not (isinstance(eds, np.ndarray) and eds.dtype == np.uint8 and eds.flags.c_contiguous and eds.ndim == 2
                and eds.shape[1] == SHARE_SIZE):
            raise ValueError("eds must be a C-contiguous (4k^2, 512) uint8 array")
        w = int(round(eds.shape[0] ** 0.5))
        if w * w != eds.shape[0] or w % 2:
            raise ValueError(f"eds holds {eds.shape[0]} shares, not a (2k)^2 square")
        rr = np.empty((w, NODE_SIZE), np.uint8)
        cr = np.empty((w, NODE_SIZE), np.uint8)
        dah = np.empty(32, np.uint8)
        err = ErrInfo()
        _check(self._L.cda_extend_commit_eds(self._h, w // 2, _p(eds), _p(rr), _p(cr), _p(dah), ctypes.byref(err)),
               err, self)
        return rr, cr, dah.tobytes()

    def commit_eds(self, eds):
        eds = np.ascontiguousarray(eds, np.uint8)
        w = int(round(eds.shape[0] ** 0.5))
        rr = np.empty((w, NODE_SIZE), np.uint8)
        cr = np.empty((w, NODE_SIZE), np.uint8)
        dah = np.empty(32, np.uint8)
        err = ErrInfo()
        _check(self._L.cda_commit_eds(self._h, w // 2, _p(eds), _p(rr), _p(cr), _p(dah), ctypes.byref(err)), err, self)
        return rr, cr, dah.tobytes()

    def dah_hash(self, row_roots, col_roots):
        n = 0 if row_roots is None else len(row_roots)
        rr = np.ascontiguousarray(np.asarray(row_roots, np.uint8).reshape(n, NODE_SIZE)) if n else None
        cr = np.ascontiguousarray(np.asarray(col_roots, np.uint8).reshape(n, NODE_SIZE)) if n else None
        out = np.empty(32, np.uint8)
        _check(self._L.cda_dah_hash(self._h, n, _p(rr), _p(cr), _p(out)), ctx=self)
        return out.tobytes()

    def nmt_axis_root(self, square_size, axis_index, leaves):
        n = len(leaves)
        if n:
            lens = {len(x) for x in leaves}
            leaf_len = min(lens)
            if len(lens) != 1:
                raise CdaError(E_SHARD_SIZE, "leaves of unequal length")
            buf = np.frombuffer(b"".join(bytes(x) for x in leaves), np.uint8).copy()
        else:
            leaf_len, buf = 0, None
        root = np.empty(NODE_SIZE, np.uint8)
        err = ErrInfo()
        rc = self._L.cda_nmt_axis_root(self._h, square_size, axis_index, n, leaf_len, _p(buf), _p(root),
                                     ctypes.byref(err))
        _check(rc, err, self)
        return root.tobytes()

    def repair(self, eds, present, row_roots, col_roots, inplace=False):
        rc, eds, pres, err = self.repair_status(eds, present, row_roots, col_roots, inplace)
        _check(rc, err, self)
        return eds, pres

    def repair_status(self, eds, present, row_roots, col_roots, inplace=False):
        """cda_repair without raising: (rc, eds, present, err) where eds/present hold the square as far as
        it was repaired (rsmt2d leaves the square 'most repaired prior to the Byzantine axis').  inplace=True
        repairs the caller's C-contiguous uint8 arrays themselves (as the C ABI does) instead of copies."""
        if inplace:
            if not (isinstance(eds, np.ndarray) and eds.dtype == np.uint8 and eds.flags.c_contiguous
                    and isinstance(present, np.ndarray) and present.dtype == np.uint8 and present.flags.c_contiguous):
                raise CdaError(E_ARG, "inplace repair needs C-contiguous uint8 arrays")
            pres = present
        else:
            eds = np.ascontiguousarray(eds, np.uint8).copy()
            pres = np.ascontiguousarray(present, np.uint8).copy()
        w = len(row_roots)
        if eds.shape[0] != w * w or eds.size != w * w * SHARE_SIZE or pres.size != w * w:
            raise CdaError(E_ARG, "eds must be (2k)^2 x 512 bytes and present (2k)^2 flags")
        err = ErrInfo()
        rc = self._L.cda_repair(self._h, w // 2, _p(eds), _p(pres), _p(np.ascontiguousarray(row_roots, np.uint8)),
                              _p(np.ascontiguousarray(col_roots, np.uint8)), ctypes.byref(err))
        return rc, eds, pres, err

    def repair_device(self, k, d_eds, present, row_roots, col_roots, stream=None):
        """cda_repair_device: repairs the square at device address d_eds (4k^2 x 512 B) in place.
        -> (rc, present, err); present is a repaired copy of the caller's flags."""
        pres = np.ascontiguousarray(present, np.uint8).copy()
        w = 2 * k
        if pres.size != w * w or len(row_roots) != w or len(col_roots) != w:
            raise CdaError(E_ARG, "present must hold (2k)^2 flags and the roots 2k entries each")
        err = ErrInfo()
        rc = self._L.cda_repair_device(self._h, k, ctypes.c_void_p(d_eds), _p(pres),
                                     _p(np.ascontiguousarray(row_roots, np.uint8)),
                                     _p(np.ascontiguousarray(col_roots, np.uint8)), ctypes.byref(err),
                                     ctypes.c_void_p(stream or 0))
        return rc, pres, err

    # ---- blob share commitments, node export, proofs ----
    def blob_commitments(self, namespaces, datas, share_versions=None, subtree_root_threshold=64):
        """inclusion.CreateCommitments over many blobs in one call -> list of 32-byte commitments."""
        nb = len(datas)
        if nb == 0:
            return []
        ns = np.frombuffer(b"".join(bytes(n) for n in namespaces), np.uint8).copy()
        if ns.size != nb * NAMESPACE_SIZE:
            raise CdaError(E_ARG, "namespaces must be 29 bytes each")
        flat = b"".join(bytes(d) for d in datas)
        data = np.frombuffer(flat, np.uint8).copy() if flat else np.zeros(1, np.uint8)
        offs = np.zeros(nb + 1, np.uint64)
        offs[1:] = np.cumsum([len(d) for d in datas])
        sv = None if share_versions is None else np.ascontiguousarray(share_versions, np.uint8)
        return [bytes(o) for o in self.blob_commitments_packed(ns, data, offs, sv, subtree_root_threshold)]

    def blob_commitments_packed(self, namespaces, data, offsets, share_versions=None, subtree_root_threshold=64):
        """cda_blob_commitments on pre-packed arrays: namespaces (n*29,) uint8, data uint8, offsets (n+1,) uint64."""
        nb = len(offsets) - 1
        out = np.empty((nb, 32), np.uint8)
        err = ErrInfo()
        rc = self._L.cda_blob_commitments(self._h, nb, _p(namespaces), _p(data), _p(offsets), _p(share_versions),
                                        subtree_root_threshold, _p(out), ctypes.byref(err))
        _check(rc, err, self)
        return out

    def merkle_roots(self, sets):
        """merkle.HashFromByteSlices of each list of 90-byte NMT nodes."""
        offs = np.zeros(len(sets) + 1, np.uint32)
        offs[1:] = np.cumsum([len(x) for x in sets])
        flat = b"".join(bytes(x) for st in sets for x in st)
        items = np.frombuffer(flat, np.uint8).copy() if flat else None
        out = np.empty((len(sets), 32), np.uint8)
        _check(self._L.cda_merkle_roots(self._h, len(sets), _p(offs), _p(items), NODE_SIZE, _p(out)), ctx=self)
        return [bytes(o) for o in out]

    def extend_commit_nodes(self, shares, want_eds=False, rows=True, cols=True, dah_tree=True):
        """extend_commit plus every node of the row / column NMTs and of the DAH tree."""
        shares = np.ascontiguousarray(shares, np.uint8)
        count, L = shares.shape
        w = 2 * max(1, int(round(count ** 0.5)))
        eds = np.empty((w * w, L), np.uint8) if want_eds else None
        rr, cr = np.empty((w, NODE_SIZE), np.uint8), np.empty((w, NODE_SIZE), np.uint8)
        dah = np.empty(32, np.uint8)
        rn = np.empty((w, 2 * w - 1, NODE_SIZE), np.uint8) if rows else None
        cn = np.empty((w, 2 * w - 1, NODE_SIZE), np.uint8) if cols else None
        dn = np.empty((4 * w - 1, 32), np.uint8) if dah_tree else None
        err = ErrInfo()
        rc = self._L.cda_extend_commit_nodes(self._h, count, L, _p(shares), _p(eds), _p(rr), _p(cr), _p(dah), _p(rn),
                                           _p(cn), _p(dn), ctypes.byref(err))
        _check(rc, err, self)
        return {"eds": eds, "row_roots": rr, "col_roots": cr, "dah": dah.tobytes(), "row_nodes": rn,
                "col_nodes": cn, "dah_nodes": dn}

    def share_inclusion_proof(self, shares, start, end):
        """pkg/proof NewShareInclusionProof for ODS shares [start, end) (raw proof parts)."""
        shares = np.ascontiguousarray(shares, np.uint8)
        count, L = shares.shape
        k = max(1, int(round(count ** 0.5)))
        lg = (2 * k).bit_length() - 1
        info = ShareProofInfo()
        rr, lh = np.empty((k, NODE_SIZE), np.uint8), np.empty((k, 32), np.uint8)
        au = np.empty((k, lg + 1, 32), np.uint8)
        ns, ne, nc = np.empty(k, np.int32), np.empty(k, np.int32), np.empty(k, np.int32)
        nodes = np.empty((k, 2 * lg, NODE_SIZE), np.uint8)
        root = np.empty(32, np.uint8)
        err = ErrInfo()
        rc = self._L.cda_share_inclusion_proof(self._h, count, L, _p(shares), start, end, ctypes.byref(info), _p(rr),
                                             _p(lh), _p(au), _p(ns), _p(ne), _p(nc), _p(nodes), _p(root),
                                             ctypes.byref(err))
        _check(rc, err, self)
        rows = [{"row_root": rr[i].tobytes(), "leaf_hash": lh[i].tobytes(),
                 "aunts": [au[i, j].tobytes() for j in range(info.naunts)], "start": int(ns[i]), "end": int(ne[i]),
                 "nodes": [nodes[i, j].tobytes() for j in range(nc[i])]} for i in range(info.nrows)]
        return {"start_row": info.start_row, "end_row": info.end_row, "total": info.total, "rows": rows,
                "data_root": root.tobytes()}

    # ---- profiling ----
    def profile_enable(self, on=True):
        _check(self._L.cda_profile_enable(self._h, 1 if on else 0), ctx=self)

    def profile_reset(self):
        _check(self._L.cda_profile_reset(self._h), ctx=self)

    def profile_read(self):
        cap = 64
        names = ctypes.create_string_buffer(4096)
        ms = np.zeros(cap, np.float64)
        cnt = np.zeros(cap, np.int64)
        n = self._L.cda_profile_read(self._h, names, 4096, _p(ms), _p(cnt), cap)
        out, parts = {}, names.raw.split(b"\0")
        for i in range(n):
            out[parts[i].decode()] = (float(ms[i]), int(cnt[i]))
        return out


_default = None
_default_lock = threading.Lock()


def _batch_outputs(ods, want_eds, eds_out):
    """Shape checks shared by the batch entry points; returns (ods, k, eds, rr, cr, dah)."""
    ods = np.ascontiguousarray(ods, np.uint8)
    if ods.ndim != 3:
        raise CdaError(E_ARG, "ods must be (nblocks, k*k, 512)")
    nb, kk, L = ods.shape
    k = int(round(kk ** 0.5))
    if k * k != kk or L != SHARE_SIZE or nb == 0:
        raise CdaError(E_ARG, "ods must be (nblocks, k*k, 512) with nblocks > 0")
    if eds_out is not None:
        # the library writes nblocks * 4k^2 * 512 bytes through this pointer: it must be exactly that array
        if (not isinstance(eds_out, np.ndarray) or eds_out.dtype != np.uint8 or not eds_out.flags.c_contiguous
                or not eds_out.flags.writeable or eds_out.shape != (nb, 4 * k * k, L)):
            raise CdaError(E_ARG, f"eds_out must be a writeable C-contiguous uint8 array of shape {(nb, 4 * k * k, L)}")
    eds = eds_out if eds_out is not None else (np.empty((nb, 4 * k * k, L), np.uint8) if want_eds else None)
    rr = np.empty((nb, 2 * k, NODE_SIZE), np.uint8)
    cr = np.empty((nb, 2 * k, NODE_SIZE), np.uint8)
    dah = np.empty((nb, 32), np.uint8)
    return ods, k, eds, rr, cr, dah


class PinnedBuffer:
    """Pinned host memory from cda_host_alloc, viewed as a numpy array (freed with the object)."""

    def __init__(self, ctx, shape, dtype=np.uint8):
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        ptr = ctypes.c_void_p()
        _check(ctx._L.cda_host_alloc(ctx._h, nbytes, ctypes.byref(ptr)), ctx=ctx)
        self._ctx, self._ptr = ctx, ptr
        buf = (ctypes.c_uint8 * max(1, nbytes)).from_address(ptr.value)
        self.array = np.frombuffer(buf, np.uint8, count=nbytes).view(dtype).reshape(shape)

    def free(self):
        if self._ptr is not None and self._ctx._h:
            self._ctx._L.cda_host_free(self._ctx._h, self._ptr)
        self._ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class MultiContext:
    """cda_multi: one handle over several GPUs of this process (device mask; 0 = all visible).
    MultiContext.replicas(device, n): n contexts on one device whose split exchanges are device copies."""

    def __init__(self, device_mask=0, _handle=None):
        if _handle is not None:
            self._h = _handle
            return
        h = ctypes.c_void_p()
        rc = lib().cda_multi_init(device_mask, ctypes.byref(h))
        if rc != OK:
            raise CdaError(rc, "cda_multi_init failed")
        self._h = h

    @classmethod
    def replicas(cls, device, count):
        h = ctypes.c_void_p()
        rc = lib().cda_multi_init_replicas(device, count, ctypes.byref(h))
        if rc != OK:
            raise CdaError(rc, "cda_multi_init_replicas failed")
        return cls(_handle=h)

    def context(self, i):
        """Context view of device i's cda_ctx (owned by this handle)."""
        c = Context.__new__(Context)
        c._L = lib()
        c._h = ctypes.c_void_p(lib().cda_multi_context(self._h, i))
        c.device = lib().cda_multi_device(self._h, i)
        c._borrowed = True
        return c

    def extend_commit_split(self, ods, want_eds=True):
        """ONE k x k square (ods: (k*k, 512) uint8) split over the handle's devices (cda_multi_extend_commit_split).
        Returns (eds or None, row_roots, col_roots, dah bytes)."""
        ods = np.ascontiguousarray(ods, np.uint8)
        count = ods.shape[0]
        k = int(round(count ** 0.5))
        if k * k != count or ods.shape[1] != SHARE_SIZE:
            raise CdaError(E_ARG, "ods must be (k*k, 512)")
        eds = np.empty((4 * k * k, SHARE_SIZE), np.uint8) if want_eds else None
        rr = np.zeros((2 * k, NODE_SIZE), np.uint8)
        cr = np.zeros((2 * k, NODE_SIZE), np.uint8)
        dah = np.zeros(32, np.uint8)
        err = ErrInfo()
        rc = lib().cda_multi_extend_commit_split(self._h, k, _p(ods), _p(eds), _p(rr), _p(cr), _p(dah),
                                                 ctypes.byref(err))
        _check(rc, err, self.context(0))
        return eds, rr, cr, dah.tobytes()

    def extend_commit_split_device(self, k, slab_ptrs):
        """The split with device g's ODS rows already at device pointer slab_ptrs[g]; returns (rr, cr, dah)."""
        arr = (ctypes.c_void_p * len(slab_ptrs))(*slab_ptrs)
        rr = np.zeros((2 * k, NODE_SIZE), np.uint8)
        cr = np.zeros((2 * k, NODE_SIZE), np.uint8)
        dah = np.zeros(32, np.uint8)
        err = ErrInfo()
        rc = lib().cda_multi_extend_commit_split_device(self._h, k, arr, _p(rr), _p(cr), _p(dah), ctypes.byref(err))
        _check(rc, err, self.context(0))
        return rr, cr, dah.tobytes()

    @property
    def device_count(self):
        return lib().cda_multi_device_count(self._h)

    def extend_commit_batch(self, ods, want_eds=True, eds_out=None):
        ods, k, eds, rr, cr, dah = _batch_outputs(ods, want_eds, eds_out)
        err = ErrInfo()
        rc = lib().cda_multi_extend_commit_batch(self._h, k, len(ods), _p(ods), _p(eds), _p(rr), _p(cr), _p(dah),
                                                 ctypes.byref(err))
        _check(rc, err)
        return eds, rr, cr, dah

    def close(self):
        if getattr(self, "_h", None):
            lib().cda_multi_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def default_context():
    global _default
    with _default_lock:
        if _default is None:
            _default = Context(int(os.environ.get("LOCAL_RANK", "0")) if os.environ.get("CDA_USE_LOCAL_RANK") else 0)
    return _default
