"""pkg/proof mirror: share inclusion proofs over libcda (celestia-app @ 2025-02-13).

NewShareInclusionProof (pkg/proof/proof.go:55-167) re-extends the square and
rebuilds row trees on the CPU. Here one libcda call (cda_share_inclusion_proof)
extends the square on the GPU, keeps every tree node it computes and returns
the NMT range proof of each row the shares span plus the RFC-6962 proof of each
row root in the data root. ParseNamespace (querier.go:124-158) is host logic.
Verifying a proof (RowProof.Validate row_proof.go:10-50, ShareProof.Validate
share_proof.go:16-82) is the client's check of a few hashes: host code here, on
hashlib, pinned by the reference's own fixtures (row_proof_test.go,
share_proof_test.go) and run on every proof the GPU builds for block 408.
"""
import hashlib
from dataclasses import dataclass

import numpy as np

from . import _native as N
from . import appconsts


class ProofError(Exception):
    pass


def _sha256(*parts):
    h = hashlib.sha256()
    for x in parts:
        h.update(x)
    return h.digest()


def _split_point(n):
    """getSplitPoint / merkle getSplitPoint: the largest power of two strictly below n (0 for n = 1)."""
    k = 1 << (n.bit_length() - 1)
    return k >> 1 if k == n else k


MAX_AUNTS = 100  # go-square merkle proof.go


@dataclass
class NMTProof:
    """proof.pb.go NMTProof (Start, End, Nodes, LeafHash = nil for inclusion proofs)."""
    start: int
    end: int
    nodes: list
    leaf_hash: bytes = b""

    def verify_inclusion(self, namespace, leaves, root):
        """nmt Proof.VerifyInclusion(sha256, nid, leavesWithoutNamespace, root) with IgnoreMaxNamespace(true), as
        ShareProof.VerifyProof calls it: each leaf hashes as nid ‖ nid ‖ SHA256(0x00 ‖ nid ‖ leaf); the proof's nodes
        are consumed left to right while the root of the smallest power-of-two subtree holding [start, end) is
        recomputed, and the remaining nodes are right siblings up to the root.  False on any mismatch, including
        siblings out of namespace order."""
        nid = bytes(namespace)
        n = len(nid)
        if self.start < 0 or self.start >= self.end or self.end - self.start != len(leaves):
            return False
        if any(len(x) != 2 * n + 32 for x in self.nodes) or len(root) != 2 * n + 32:
            return False
        parity = b"\xff" * n
        hashes = [nid + nid + _sha256(b"\x00", nid, bytes(leaf)) for leaf in leaves]
        nodes = [bytes(x) for x in self.nodes]
        state = {"bad": False}

        def node(left, right):
            if left[n:2 * n] > right[:n]:
                state["bad"] = True  # nmt ValidateSiblings: left.max <= right.min
            mx = left[n:2 * n] if right[:n] == parity else right[n:2 * n]
            return left[:n] + mx + _sha256(b"\x01", left, right)

        def pop():
            return nodes.pop(0) if nodes else None

        def compute(lo, hi):
            if hi - lo == 1:
                if self.start <= lo < self.end:
                    return hashes.pop(0) if hashes else None
                return pop()
            if hi <= self.start or lo >= self.end:
                return pop()
            k = _split_point(hi - lo)
            left, right = compute(lo, lo + k), compute(lo + k, hi)
            if right is None:
                return left
            if left is None:
                state["bad"] = True
                return None
            return node(left, right)

        h = compute(0, max(1, _split_point(self.end) * 2))
        if h is None or hashes:
            return False
        while nodes:
            h = node(h, nodes.pop(0))
        return not state["bad"] and h == bytes(root)


@dataclass
class Proof:
    """merkle proof of one row root in the data root (proof.pb.go Proof)."""
    total: int
    index: int
    leaf_hash: bytes
    aunts: list

    def verify(self, root_hash, leaf):
        """Proof.Verify (row_proof.go:41-50) = go-square merkle Proof.Verify: RFC-6962 leaf hash, then the root
        rebuilt from the aunts (bottom-up).  Raises ProofError."""
        if self.total < 0:
            raise ProofError("proof total must be positive")
        if self.index < 0:
            raise ProofError("proof index cannot be negative")
        lh = _sha256(b"\x00", bytes(leaf))
        if lh != bytes(self.leaf_hash):
            raise ProofError(f"invalid leaf hash: wanted {lh.hex().upper()} got {bytes(self.leaf_hash).hex().upper()}")
        if len(self.aunts) > MAX_AUNTS:
            raise ProofError(f"expected no more than {MAX_AUNTS} aunts, got {len(self.aunts)}")

        def from_aunts(index, total, h, aunts):
            if index >= total or index < 0 or total <= 0:
                return None
            if total == 1:
                return h if not aunts else None
            if not aunts:
                return None
            k = _split_point(total)
            if index < k:
                sub = from_aunts(index, k, h, aunts[:-1])
                return None if sub is None else _sha256(b"\x01", sub, bytes(aunts[-1]))
            sub = from_aunts(index - k, total - k, h, aunts[:-1])
            return None if sub is None else _sha256(b"\x01", bytes(aunts[-1]), sub)

        got = from_aunts(self.index, self.total, lh, list(self.aunts))
        if got is None:
            raise ProofError("invalid proof: could not compute the root hash from the aunts")
        if got != bytes(root_hash):
            raise ProofError(f"invalid root hash: wanted {bytes(root_hash).hex().upper()} got {got.hex().upper()}")


@dataclass
class RowProof:
    row_roots: list
    proofs: list
    start_row: int
    end_row: int

    def validate(self, root):
        """RowProof.Validate (row_proof.go:10-24)."""
        if self.end_row - self.start_row + 1 != len(self.row_roots):
            raise ProofError(f"the number of rows {self.end_row - self.start_row + 1} must equal the number of row "
                             f"roots {len(self.row_roots)}")
        if len(self.proofs) != len(self.row_roots):
            raise ProofError(f"the number of proofs {len(self.proofs)} must equal the number of row roots "
                             f"{len(self.row_roots)}")
        if not self.verify_proof(root):
            raise ProofError("row proof failed to verify")

    def verify_proof(self, root):
        """RowProof.VerifyProof (:26-37)."""
        for p, rr in zip(self.proofs, self.row_roots):
            try:
                p.verify(root, rr)
            except ProofError:
                return False
        return True


@dataclass
class ShareProof:
    data: list
    share_proofs: list
    namespace_id: bytes
    row_proof: RowProof
    namespace_version: int
    data_root: bytes = b""  # the DAH hash the proof was built against (not a field of the reference type)

    def validate(self, root):
        """ShareProof.Validate (share_proof.go:16-51)."""
        if self.data is None:
            raise ProofError("empty share proof")
        in_proofs = sum(p.end - p.start for p in self.share_proofs)
        if len(self.share_proofs) != len(self.row_proof.row_roots):
            raise ProofError(f"the number of share proofs {len(self.share_proofs)} must equal the number of row "
                             f"roots {len(self.row_proof.row_roots)}")
        if len(self.data) != in_proofs:
            raise ProofError(f"the number of shares {len(self.data)} must equal the number of shares in share "
                             f"proofs {in_proofs}")
        for p in self.share_proofs:
            if p.start < 0:
                raise ProofError("proof index cannot be negative")
            if p.end - p.start <= 0:
                raise ProofError("proof total must be positive")
        self.row_proof.validate(root)
        if not self.verify_proof():
            raise ProofError("share proof failed to verify")

    def verify_proof(self):
        """ShareProof.VerifyProof (:53-82)."""
        cursor = 0
        for p, rr in zip(self.share_proofs, self.row_proof.row_roots):
            used = p.end - p.start
            if self.namespace_version > 255:
                return False
            ns = bytes([self.namespace_version]) + bytes(self.namespace_id)
            if not p.verify_inclusion(ns, self.data[cursor:cursor + used], rr):
                return False
            cursor += used
        return True


def parse_namespace(raw_shares, start_share, end_share):
    """ParseNamespace (querier.go:126-158): the one namespace of shares [start, end)."""
    if start_share < 0:
        raise ProofError(f"start share {start_share} should be positive")
    if end_share < 0:
        raise ProofError(f"end share {end_share} should be positive")
    if end_share < start_share:
        raise ProofError(f"end share {end_share} cannot be lower than starting share {start_share}")
    if end_share > len(raw_shares):
        raise ProofError(f"end share {end_share} is higher than block shares {len(raw_shares)}")
    ns = bytes(raw_shares[start_share][:appconsts.NAMESPACE_SIZE])
    for i in range(start_share, end_share):
        if bytes(raw_shares[i][:appconsts.NAMESPACE_SIZE]) != ns:
            raise ProofError(f"shares range contain different namespaces at index {i - start_share}")
    return ns


def new_share_inclusion_proof(data_square, namespace, start, end, ctx=None):
    """NewShareInclusionProof(dataSquare, namespace, shares.NewRange(start, end))."""
    ctx = ctx or N.default_context()
    arr = np.stack([np.frombuffer(bytes(s), np.uint8) for s in data_square])
    out = ctx.share_inclusion_proof(arr, start, end)
    k = int(round(len(data_square) ** 0.5))
    rows = out["rows"]
    row_proof = RowProof([r["row_root"] for r in rows],
                         [Proof(out["total"], out["start_row"] + i, r["leaf_hash"], r["aunts"])
                          for i, r in enumerate(rows)], out["start_row"], out["end_row"])
    data, share_proofs = [], []
    for i, r in enumerate(rows):
        row = out["start_row"] + i
        data += [arr[row * k + j].tobytes() for j in range(r["start"], r["end"])]
        share_proofs.append(NMTProof(r["start"], r["end"], r["nodes"]))
    namespace = bytes(namespace)
    return ShareProof(data, share_proofs, namespace[1:], row_proof, namespace[0], out["data_root"])
