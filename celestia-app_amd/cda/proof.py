"""pkg/proof mirror: share inclusion proofs over libcda (celestia-app @ 2025-02-13).

NewShareInclusionProof (pkg/proof/proof.go:55-167) re-extends the square and
rebuilds row trees on the CPU. Here one libcda call (cda_share_inclusion_proof)
extends the square on the GPU, keeps every tree node it computes and returns
the NMT range proof of each row the shares span plus the RFC-6962 proof of each
row root in the data root. ParseNamespace (querier.go:124-158) is host logic.
Verifying a proof (ShareProof.Validate, share_proof.go:16-82) is a client-side
CPU check and is not part of this engine; the tests verify with the oracle.
"""
from dataclasses import dataclass

import numpy as np

from . import _native as N
from . import appconsts


class ProofError(Exception):
    pass


@dataclass
class NMTProof:
    """proof.pb.go NMTProof (Start, End, Nodes, LeafHash = nil for inclusion proofs)."""
    start: int
    end: int
    nodes: list
    leaf_hash: bytes = b""


@dataclass
class Proof:
    """merkle proof of one row root in the data root (proof.pb.go Proof)."""
    total: int
    index: int
    leaf_hash: bytes
    aunts: list


@dataclass
class RowProof:
    row_roots: list
    proofs: list
    start_row: int
    end_row: int


@dataclass
class ShareProof:
    data: list
    share_proofs: list
    namespace_id: bytes
    row_proof: RowProof
    namespace_version: int
    data_root: bytes = b""  # the DAH hash the proof was built against (not a field of the reference type)


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
