//go:build rocm

// proof_rocm.go — goes to pkg/proof/ of celestia-app (with ../patches/0005 applied and ../cda copied to pkg/cda).
// Under -tags rocm NewShareInclusionProof (pkg/proof/proof.go:55-160: re-extend the square, rebuild the proven rows'
// trees, ProveRange, merkle.ProofsFromByteSlices over the 4k roots) is ONE cda_share_inclusion_proof call that
// extends the square, exports the nodes and assembles every proof on the GPU; the ShareProof it returns has the
// same fields and bytes (go/cda/cda_test.go TestShareInclusionProofMatchesCPUPath).
package proof

import (
	"github.com/celestiaorg/go-square/namespace"
	"github.com/celestiaorg/go-square/shares"
	"github.com/celestiaorg/go-square/square"

	"github.com/celestiaorg/celestia-app/v2/pkg/cda"
)

func init() {
	newShareInclusionProof = func(dataSquare square.Square, ns namespace.Namespace, shareRange shares.Range) (
		ShareProof, error) {
		ctx, err := cda.Default()
		if err != nil {
			return ShareProof{}, err
		}
		raw := shares.ToBytes(dataSquare)
		parts, err := cda.ShareInclusionProof(ctx, raw, shareRange.Start, shareRange.End)
		if err != nil {
			return ShareProof{}, err
		}
		rp := &RowProof{StartRow: uint32(parts.StartRow), EndRow: uint32(parts.EndRow)}
		var nmtProofs []*NMTProof
		for _, r := range parts.Rows {
			rp.RowRoots = append(rp.RowRoots, r.RowRoot)
			rp.Proofs = append(rp.Proofs, &Proof{Total: r.Total, Index: int64(r.Row), LeafHash: r.LeafHash,
				Aunts: r.Aunts})
			nmtProofs = append(nmtProofs, &NMTProof{Start: r.Start, End: r.End, Nodes: r.Nodes})
		}
		data := make([][]byte, 0, shareRange.End-shareRange.Start)
		for _, s := range raw[shareRange.Start:shareRange.End] {
			data = append(data, s)
		}
		return ShareProof{
			RowProof:         rp,
			Data:             data,
			ShareProofs:      nmtProofs,
			NamespaceId:      ns.ID,
			NamespaceVersion: uint32(ns.Version),
		}, nil
	}
}
