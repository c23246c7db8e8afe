//go:build rocm

package inclusion

import (
	"bytes"
	"math/rand"
	"sort"
	"testing"

	"github.com/celestiaorg/rsmt2d"
	"github.com/stretchr/testify/require"

	"github.com/celestiaorg/celestia-app/v2/pkg/appconsts"
	"github.com/celestiaorg/celestia-app/v2/pkg/da"
)

// TestSubtreeCacherFromSharesMatchesVisitor: the cacher filled from the GPU's exported nodes holds exactly the map
// the row trees' NodeVisitor fills on the CPU, and GetCommitment over it equals GetCommitment over the CPU cacher.
func TestSubtreeCacherFromSharesMatchesVisitor(t *testing.T) {
	r := rand.New(rand.NewSource(9))
	for _, k := range []int{4, 32} {
		raw := make([][]byte, k*k)
		for i := range raw {
			raw[i] = make([]byte, appconsts.ShareSize)
			r.Read(raw[i][19:])
		}
		sort.Slice(raw, func(i, j int) bool { return bytes.Compare(raw[i], raw[j]) < 0 })
		want := NewSubtreeCacher(uint64(k))
		eds, err := rsmt2d.ComputeExtendedDataSquare(raw, appconsts.DefaultCodec(), want.Constructor)
		require.NoError(t, err)
		wantDAH, err := da.NewDataAvailabilityHeader(eds)
		require.NoError(t, err)
		got, gotDAH, err := NewSubtreeCacherFromShares(raw)
		require.NoError(t, err)
		require.Equal(t, wantDAH.Hash(), gotDAH.Hash())
		require.Equal(t, len(want.caches), len(got.caches))
		for row, c := range want.caches {
			require.Equal(t, c.cache, got.caches[row].cache, "k=%d row %d", k, row)
		}
		for start := 0; start+4 <= k*k; start += k + 3 {
			cw, err := GetCommitment(want, wantDAH, start, 4, appconsts.DefaultSubtreeRootThreshold)
			require.NoError(t, err)
			cg, err := GetCommitment(got, gotDAH, start, 4, appconsts.DefaultSubtreeRootThreshold)
			require.NoError(t, err)
			require.Equal(t, cw, cg, "k=%d start %d", k, start)
		}
	}
}
