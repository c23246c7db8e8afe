//go:build rocm

// extend_rocm.go — goes to pkg/da/ of celestia-app (with ../patches/0001, 0002 and 0004 applied and ../cda copied
// to pkg/cda).  Under -tags rocm the DA hot path runs on the GPU with every caller unchanged:
// PrepareProposal / ProcessProposal / ExtendBlock keep calling da.ExtendShares and
// da.NewDataAvailabilityHeader (app/prepare_proposal.go:65,77, app/process_proposal.go:137,143,
// app/extend_block.go:25).
//
// appconsts.DefaultCodec is NOT replaced: rsmt2d callers outside the block path (ComputeExtendedDataSquare with
// appconsts.DefaultCodec(), (*ExtendedDataSquare).Repair) reach a codec one axis at a time, and measured per axis
// through host buffers the GPU codec and tree lose to the CPU ones or tie (bench.py per_axis, DESIGN.md §12.1: one
// Encode 31 vs 25 us, one tree Root 110 vs 92 us, an rsmt2d-shaped extension of k = 128 13.5 vs 3.2 ms with one
// thread per axis).  Those callers keep the reference's Leopard codec and wrapper trees; a caller that wants the
// GPU for a whole square calls cda.Repair (one call: ~1-3 ms against ~90-100 ms axis by axis) or installs
// cda.NewCodec itself (patch 0001 lets it).
package da

import (
	"github.com/celestiaorg/celestia-app/v2/pkg/cda"
)

func init() {
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
