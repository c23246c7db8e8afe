"""Rank body for the split-square tests (tests/test_split.py): one process per rank, gloo.

`OracleOps` is a CPU test double of cda.split.DeviceOps: it answers the same
tensor-level calls through the C oracle so the distributed logic (ownership,
all-to-all layout, subtree fold, error order) can be exercised on CPU ranks.
It is test infrastructure only; the product path (DeviceOps) calls libcda.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

PARITY_NS = b"\xff" * 29


class _NullStream:
    cuda_stream = 0

    def synchronize(self):
        pass


class OracleOps:
    def __init__(self):
        import torch
        self.torch = torch
        self.device = torch.device("cpu")
        self.stream = _NullStream()

    def empty(self, shape, dtype=None):
        return self.torch.zeros(shape, dtype=dtype or self.torch.uint8)

    def rs_encode_rows(self, E, k, r0, nrows):
        import oracle_lib as O
        for r in range(r0, r0 + nrows):
            E[r, k:] = self.torch.from_numpy(O.leo_encode(E[r, :k].numpy()))

    def rs_encode_cols(self, E, k, c0, ncols):
        import oracle_lib as O
        for c in range(c0, c0 + ncols):
            E[k:, c] = self.torch.from_numpy(O.leo_encode(E[:k, c].numpy()))

    def roots(self, E, k, axis, first, naxes, leaf_off, nleaves):
        import oracle_lib as O
        out = self.empty((naxes, 96))
        st = self.torch.full((naxes,), -1, dtype=self.torch.int64)
        for t in range(naxes):
            idx = first + t
            cells = E[idx, leaf_off:leaf_off + nleaves] if axis == 0 else E[leaf_off:leaf_off + nleaves, idx]
            # the quadrant rule uses the global leaf index: shift the tree so that leaf
            # `leaf_off` is pushed at its own position only when the range starts at 0
            assert leaf_off == 0 or idx >= k, "sub-range trees are only taken over parity rows"
            rc, root, leaf = O.nmt_axis_root(k, idx, [bytes(c.numpy()) for c in cells])
            if rc != 0:
                st[t] = leaf
            out[t, :90] = self.torch.frombuffer(bytearray(root), dtype=self.torch.uint8)
        return out, st

    def fold(self, nodes):
        ntrees, n = nodes.shape[0], nodes.shape[1]
        cur = [[bytes(nodes[t, i, :90].numpy()) for i in range(n)] for t in range(ntrees)]
        while n > 1:
            nxt = []
            for lvl in cur:
                row = []
                for i in range(0, n, 2):
                    L, R = lvl[i], lvl[i + 1]
                    mx = L[29:58] if R[:29] == PARITY_NS else R[29:58]
                    row.append(L[:29] + mx + hashlib.sha256(b"\x01" + L + R).digest())
                nxt.append(row)
            cur, n = nxt, n // 2
        out = self.empty((ntrees, 96))
        for t in range(ntrees):
            out[t, :90] = self.torch.frombuffer(bytearray(cur[t][0]), dtype=self.torch.uint8)
        return out

    def dah(self, roots):
        import oracle_lib as O
        r = roots.numpy()[:, :90]
        w = r.shape[0] // 2
        return self.torch.frombuffer(bytearray(O.dah_hash(r[:w], r[w:])), dtype=self.torch.uint8)


def run_rank(rank, world, port, k, seed, use_gpu, outdir, unsorted=False):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cda import split
    import oracle_lib as O
    try:
        ods = O.gen_ods(k, seed).reshape(k, k, 512)
        if unsorted:  # swap two shares of row 1 -> push-order error on row 1 and a column
            ods = ods.copy()
            ods[1, [2, 3]] = ods[1, [3, 2]]
        (r0, r1), _ = split.plan(k, world, rank)
        if use_gpu:
            import cda
            ctx = cda.Context(0)
            ops = split.DeviceOps(ctx)
            rows = torch.from_numpy(np.ascontiguousarray(ods[r0:r1])).to(ops.device)
        else:
            ops = OracleOps()
            rows = torch.from_numpy(np.ascontiguousarray(ods[r0:r1]))
        res = {}
        try:
            out = split.extend_commit_split(ops, k, rows)
            E = out.eds.cpu().numpy() if use_gpu else out.eds.numpy()
            (a, b), (c, d) = out.rows, out.cols
            res = dict(rc=0, row_roots=out.row_roots, col_roots=out.col_roots,
                       dah=np.frombuffer(out.dah, np.uint8),
                       rows_sha=np.frombuffer(hashlib.sha256(E[a:b].tobytes()).digest(), np.uint8),
                       cols_sha=np.frombuffer(hashlib.sha256(np.ascontiguousarray(E[:, c:d]).tobytes()).digest(),
                                              np.uint8))
        except split.CdaError as e:
            res = dict(rc=e.code, axis=e.axis, index=e.index, leaf=e.leaf)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()
