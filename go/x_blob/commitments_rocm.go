//go:build rocm

// commitments_rocm.go — goes to x/blob/types/ of celestia-app (with ../patches/0003 applied and ../cda copied to
// pkg/cda).  Under -tags rocm ProcessProposal's pre-pass (types.PrecomputeCommitments) computes the share
// commitments of every BlobTx of a proposal in one cda_blob_commitments call on the GPU; ValidateBlobTx then
// compares each MsgPayForBlobs against them (x/blob/types/blob_tx.go:97-105), in the reference's order.
package types

import (
	"github.com/celestiaorg/go-square/blob"

	"github.com/celestiaorg/celestia-app/v2/pkg/cda"
)

func init() {
	BatchCommitments = func(blobs []*blob.Blob, subtreeRootThreshold int) ([][]byte, error) {
		ctx, err := cda.Default()
		if err != nil {
			return nil, err
		}
		return cda.CreateBlobCommitments(ctx, blobs, subtreeRootThreshold)
	}
}
