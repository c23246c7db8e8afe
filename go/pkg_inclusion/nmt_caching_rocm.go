//go:build rocm

// nmt_caching_rocm.go — goes to pkg/inclusion/ of celestia-app (with ../patches/0005 applied and ../cda copied to
// pkg/cda).  Under -tags rocm NewSubtreeCacherFromShares fills the EDSSubTreeRootCacher (nmt_caching.go:76-124) from
// ONE cda_extend_commit_nodes call: every row tree's inner nodes, exported by the GPU, are recorded exactly as the
// rows' nmt.NodeVisitor would record them (parent -> its two children), so getSubTreeRoot / GetCommitment
// (get_commit.go:12-30) walk the same map with no host hashing.
package inclusion

import (
	"github.com/celestiaorg/celestia-app/v2/pkg/cda"
	"github.com/celestiaorg/celestia-app/v2/pkg/da"
)

func init() {
	NewSubtreeCacherFromShares = func(s [][]byte) (*EDSSubTreeRootCacher, da.DataAvailabilityHeader, error) {
		ctx, err := cda.Default()
		if err != nil {
			return nil, da.DataAvailabilityHeader{}, err
		}
		nodes, err := cda.ExtendCommitNodes(ctx, s, false, false)
		if err != nil {
			return nil, da.DataAvailabilityHeader{}, err
		}
		w := 2 * nodes.K
		cacher := NewSubtreeCacher(uint64(nodes.K))
		for row, tree := range nodes.RowNodes {
			for level, n := 1, w/2; n >= 1; level, n = level+1, n/2 {
				for pos := 0; pos < n; pos++ {
					cacher.Visit(uint(row), cda.Node(tree, w, level, pos), cda.Node(tree, w, level-1, 2*pos),
						cda.Node(tree, w, level-1, 2*pos+1))
				}
			}
		}
		dah := da.DataAvailabilityHeader{RowRoots: nodes.RowRoots, ColumnRoots: nodes.ColRoots}
		dah.Hash()
		return cacher, dah, nil
	}
}
