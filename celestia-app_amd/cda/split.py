"""One data square extended and committed across G GPUs.

The single-GPU path (``Context.extend_commit*``) keeps a whole square on one
device.  A k=512 square (128 MiB ODS -> 512 MiB EDS, 2048 roots) can be split
over G ranks instead, with one process per GPU and ``torch.distributed``
(backend "nccl" = RCCL over xGMI). Rank g:

1. owns ODS rows [g*k/G, (g+1)*k/G). It row-encodes them (Q0 -> Q1) and computes
   their row roots. rsmt2d ``erasureExtendSquare`` runs this step for rows < k.
2. exchanges the top half in ONE all-to-all. Rank g receives columns
   [g*2k/G, (g+1)*2k/G) of rows 0..k-1.
3. column-encodes its columns (Q0|Q1 -> Q2|Q3, the same bytes as rsmt2d's
   Q3 = Enc(Q2 rows), by linearity) and computes their full column roots.
4. for each bottom row r >= k, computes the root of the NMT subtree over its own
   columns. The tree splits at powers of two (nmt_wrapper.go:118), so that
   subtree is a node of row r's tree. G x k subtree nodes (90 B each) are
   gathered and folded log2(G) levels into the bottom row roots. No second
   share transpose is needed.
5. gathers the 4k roots; every rank hashes the DAH.

The EDS stays distributed. On rank g the top-half rows it owns and its columns
are valid in ``E``. All compute runs in libcda's HIP kernels. The collectives
are the only data movement between GPUs.
"""
from dataclasses import dataclass

import numpy as np

from . import _native
from ._native import CdaError, E_NS_ORDER, NODE_SIZE

REC = 96  # device root record: 90-B NMT node + 6 zero bytes
ROW, COL = 0, 1


class DeviceOps:
    """Tensor-level wrappers over libcda's device entry points (include/cda.h)."""

    def __init__(self, ctx, stream=None):
        import torch
        self.torch = torch
        self.ctx = ctx
        self.device = torch.device("cuda", ctx.device)
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)

    def _s(self):
        return self.stream.cuda_stream

    def empty(self, shape, dtype=None):
        return self.torch.empty(shape, dtype=dtype or self.torch.uint8, device=self.device)

    def rs_encode_rows(self, E, k, r0, nrows):
        """Q1[r] = Enc(Q0[r]) for rows r0..r0+nrows (E: (2k, 2k, 512) uint8)."""
        pitch = E.stride(0)
        base = E.data_ptr()
        self.ctx.rs_encode_device(k, E.shape[2], nrows, base + r0 * pitch, pitch, E.shape[2],
                                  base + r0 * pitch + k * E.shape[2], pitch, E.shape[2], self._s())

    def rs_encode_cols(self, E, k, c0, ncols):
        """(Q2|Q3)[:, c] = Enc((Q0|Q1)[:, c]) for columns c0..c0+ncols."""
        pitch, S = E.stride(0), E.shape[2]
        base = E.data_ptr()
        self.ctx.rs_encode_device(k, S, ncols, base + c0 * S, S, pitch, base + k * pitch + c0 * S, S, pitch,
                                  self._s())

    def roots(self, E, k, axis, first, naxes, leaf_off, nleaves):
        out = self.empty((naxes, REC))
        st = self.empty((naxes,), self.torch.int64)
        self.ctx.nmt_roots_device(k, E.data_ptr(), axis, first, naxes, leaf_off, nleaves, out.data_ptr(),
                                  st.data_ptr(), self._s())
        return out, st

    def fold(self, nodes):
        """nodes: (ntrees, n, 96) -> (ntrees, 96)."""
        nodes = nodes.contiguous()
        out = self.empty((nodes.shape[0], REC))
        self.ctx.nmt_fold_device(nodes.shape[0], nodes.shape[1], nodes.data_ptr(), out.data_ptr(), self._s())
        return out

    def dah(self, roots):
        roots = roots.contiguous()
        out = self.empty((32,))
        self.ctx.dah_device(roots.shape[0], roots.data_ptr(), out.data_ptr(), self._s())
        return out


@dataclass
class SplitResult:
    row_roots: np.ndarray  # (2k, 90)
    col_roots: np.ndarray  # (2k, 90)
    dah: bytes
    eds: object  # this rank's (2k, 2k, 512) tensor; valid: rows [r0, r1) and columns [c0, c1)
    rows: tuple
    cols: tuple


def plan(k, world, rank):
    """Row / column ownership of `rank`."""
    if world < 1 or world & (world - 1) or k % world:
        raise ValueError(f"world size {world} must be a power of two dividing k={k}")
    rp, cp = k // world, 2 * k // world
    return (rank * rp, (rank + 1) * rp), (rank * cp, (rank + 1) * cp)


def _is_nccl(group):
    import torch.distributed as dist
    return dist.get_backend(group) == "nccl"


def _all_to_all(recv, send, group):
    import torch.distributed as dist
    if _is_nccl(group):
        dist.all_to_all_single(recv, send, group=group)
    else:  # gloo: host staging (CPU tests / multi-rank rehearsal on one GPU)
        r = recv.cpu()
        dist.all_to_all_single(r, send.cpu(), group=group)
        recv.copy_(r)


def _all_gather(t, group):
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if _is_nccl(group):
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t.contiguous(), group=group)
        return torch.stack(outs)
    tc = t.contiguous().cpu()
    outs = [torch.empty_like(tc) for _ in range(world)]
    dist.all_gather(outs, tc, group=group)
    return torch.stack(outs).to(t.device)


def _first_push_error(st_rows, st_cols, r_index, c_index):
    """Reference order: eds.RowRoots() first (row 0..), then ColRoots (data_availability_header.go:45-49)."""
    for st, idx, axis in ((st_rows, r_index, ROW), (st_cols, c_index, COL)):
        bad = np.flatnonzero(st != -1)
        if bad.size:
            j = int(bad[np.argmin(idx[bad])])
            return axis, int(idx[j]), int(st[j])
    return None


def extend_commit_split(ops, k, ods_rows, group=None):
    """Extend + commit one k x k square whose ODS rows are split over the ranks of `group`.

    ods_rows: this rank's (k/G, k, 512) uint8 tensor (rows plan(k)[0]) on ops.device.
    Returns SplitResult (identical roots / DAH on every rank). Raises CdaError
    (CDA_E_NS_ORDER with axis / index / leaf) like cda_extend_commit.
    """
    import torch
    if ops.device.type == "cuda":
        # every torch op and collective of the split on ops.stream, the stream the libcda calls use (a
        # collective orders itself after the CURRENT stream only)
        with torch.cuda.stream(ops.stream):
            return _extend_commit_split(ops, k, ods_rows, group)
    return _extend_commit_split(ops, k, ods_rows, group)


def _extend_commit_split(ops, k, ods_rows, group):
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    (r0, r1), (c0, c1) = plan(k, world, rank)
    w, S = 2 * k, ods_rows.shape[-1]
    if tuple(ods_rows.shape) != (r1 - r0, k, S):
        raise ValueError(f"ods_rows shape {tuple(ods_rows.shape)} != {(r1 - r0, k, S)}")
    E = ops.empty((w, w, S))
    # 1. own rows: Q0 copy + Q1, row roots of the top half rows it owns
    E[r0:r1, :k].copy_(ods_rows)
    ops.rs_encode_rows(E, k, r0, r1 - r0)
    top_roots, top_st = ops.roots(E, k, ROW, r0, r1 - r0, 0, w)
    # 2. one all-to-all of the top half: peer h gets rows [r0, r1) x its columns
    rp, cp = r1 - r0, c1 - c0
    if world > 1:
        send = E[r0:r1].view(rp, world, cp, S).permute(1, 0, 2, 3).contiguous()
        recv = torch.empty_like(send)
        ops.stream.synchronize()
        _all_to_all(recv, send, group)
        E[:k, c0:c1].copy_(recv.view(k, cp, S))
    # 3. own columns: Q2|Q3 and full column roots
    ops.rs_encode_cols(E, k, c0, cp)
    col_roots, col_st = ops.roots(E, k, COL, c0, cp, 0, w)
    # 4. bottom rows: subtree roots over own columns, gathered and folded
    sub, _ = ops.roots(E, k, ROW, k, k, c0, cp)
    if world > 1:
        ops.stream.synchronize()
        all_sub = _all_gather(sub, group)  # (G, k, 96)
        bottom = ops.fold(all_sub.permute(1, 0, 2))
        all_top = _all_gather(top_roots, group).reshape(k, REC)
        all_cols = _all_gather(col_roots, group).reshape(w, REC)
        st_rows = _all_gather(top_st, group).reshape(k)
        st_cols = _all_gather(col_st, group).reshape(w)
    else:
        bottom, all_top, all_cols, st_rows, st_cols = sub, top_roots, col_roots, top_st, col_st
    roots = torch.cat([all_top, bottom, all_cols])
    dah = ops.dah(roots)
    ops.stream.synchronize()
    err = _first_push_error(st_rows.cpu().numpy(), st_cols.cpu().numpy(), np.arange(k), np.arange(w))
    if err is not None:
        axis, index, leaf = err
        raise CdaError(E_NS_ORDER, axis=axis, index=index, leaf=leaf)
    r = roots.cpu().numpy()[:, :NODE_SIZE]
    return SplitResult(r[:w].copy(), r[w:].copy(), bytes(dah.cpu().numpy()), E, (r0, r1), (c0, c1))


__all__ = ["DeviceOps", "SplitResult", "plan", "extend_commit_split", "_native"]
