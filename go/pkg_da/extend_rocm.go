//go:build rocm

// extend_rocm.go — goes to pkg/da/ of celestia-app (with ../patches/0001, 0002 and 0004 applied and ../cda copied
// to pkg/cda).  Under -tags rocm the DA hot path runs on the GPU with every caller unchanged:
// PrepareProposal / ProcessProposal / ExtendBlock keep calling da.ExtendShares and
// da.NewDataAvailabilityHeader (app/prepare_proposal.go:65,77, app/process_proposal.go:137,143,
// app/extend_block.go:25), and code that uses rsmt2d directly gets the GPU codec from appconsts.DefaultCodec.
package da

import (
	"github.com/celestiaorg/celestia-app/v2/pkg/appconsts"
	"github.com/celestiaorg/celestia-app/v2/pkg/cda"
)

func init() {
	appconsts.DefaultCodec = cda.NewCodec
	extendShares = cda.ExtendShares
	// ../patches/0004: PrepareProposal / ProcessProposal take the data root without the EDS copied back
	dahFromShares = func(s [][]byte) (DataAvailabilityHeader, error) {
		rows, cols, hash, err := cda.DataAvailabilityHeaderFromShares(s)
		if err != nil {
			return DataAvailabilityHeader{}, err
		}
		return DataAvailabilityHeader{RowRoots: rows, ColumnRoots: cols, hash: hash}, nil
	}
}
