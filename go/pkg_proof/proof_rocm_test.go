//go:build rocm

package proof

import (
	"testing"

	"github.com/celestiaorg/go-square/shares"
	"github.com/celestiaorg/go-square/square"
	"github.com/stretchr/testify/require"

	"github.com/celestiaorg/celestia-app/v2/pkg/appconsts"
	"github.com/celestiaorg/celestia-app/v2/test/util/testfactory"
)

// TestShareInclusionProofMatchesCPUPath: the GPU route installed by proof_rocm.go returns the ShareProof the
// reference's CPU implementation builds, field for field, for ranges inside one row, across rows and over whole
// rows, and the proof validates against the data root (ShareProof.Validate, share_proof.go).
func TestShareInclusionProofMatchesCPUPath(t *testing.T) {
	txs := testfactory.GenerateRandomTxs(200, 600)
	dataSquare, err := square.Construct(txs.ToSliceOfBytes(), appconsts.DefaultSquareSizeUpperBound,
		appconsts.DefaultSubtreeRootThreshold)
	require.NoError(t, err)
	k := dataSquare.Size()
	for _, r := range []shares.Range{{Start: 0, End: 1}, {Start: 3, End: k - 1}, {Start: k - 2, End: 3 * k},
		{Start: 0, End: 2 * k}} {
		if r.End > k*k {
			continue
		}
		ns, err := dataSquare[r.Start].Namespace()
		require.NoError(t, err)
		want, err := newShareInclusionProofCPU(dataSquare, ns, r)
		require.NoError(t, err)
		got, err := NewShareInclusionProof(dataSquare, ns, r)
		require.NoError(t, err)
		require.Equal(t, want.Data, got.Data)
		require.Equal(t, want.RowProof.RowRoots, got.RowProof.RowRoots)
		require.Equal(t, want.RowProof.StartRow, got.RowProof.StartRow)
		require.Equal(t, want.RowProof.EndRow, got.RowProof.EndRow)
		for i := range want.RowProof.Proofs {
			require.Equal(t, *want.RowProof.Proofs[i], *got.RowProof.Proofs[i])
		}
		require.Len(t, got.ShareProofs, len(want.ShareProofs))
		for i := range want.ShareProofs {
			require.Equal(t, want.ShareProofs[i].Start, got.ShareProofs[i].Start)
			require.Equal(t, want.ShareProofs[i].End, got.ShareProofs[i].End)
			require.Equal(t, len(want.ShareProofs[i].Nodes), len(got.ShareProofs[i].Nodes))
			for j := range want.ShareProofs[i].Nodes {
				require.Equal(t, want.ShareProofs[i].Nodes[j], got.ShareProofs[i].Nodes[j])
			}
		}
		require.Equal(t, want.NamespaceId, got.NamespaceId)
		require.Equal(t, want.NamespaceVersion, got.NamespaceVersion)
	}
}
