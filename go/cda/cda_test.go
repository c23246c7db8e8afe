//go:build rocm

// Tests a maintainer runs where Go, the module cache and a GPU exist (CGO_ENABLED=1 go test -tags rocm
// ./pkg/cda/): they pin the GPU path against the reference's own CPU code -- rsmt2d.NewLeoRSCodec and
// wrapper.NewConstructor -- on non-constant data, which the container this engine was built in could not do
// (no Go toolchain; see DESIGN.md §3).
package cda_test

import (
	"bytes"
	"crypto/sha256"
	"math/rand"
	"runtime"
	"sort"
	"testing"
	"time"
	"unsafe"

	"github.com/celestiaorg/go-square/blob"
	"github.com/celestiaorg/go-square/inclusion"
	"github.com/celestiaorg/go-square/merkle"
	appns "github.com/celestiaorg/go-square/namespace"
	"github.com/celestiaorg/go-square/shares"
	"github.com/celestiaorg/go-square/square"
	"github.com/celestiaorg/rsmt2d"
	"github.com/stretchr/testify/require"

	"github.com/celestiaorg/celestia-app/v2/pkg/cda"
	"github.com/celestiaorg/celestia-app/v2/pkg/da"
	"github.com/celestiaorg/celestia-app/v2/pkg/wrapper"
)

// sortedShares: v0 namespaces (0x00 x 19 ‖ 10 random bytes) ‖ 483 random bytes, sorted (SURVEY.md §8d).
func sortedShares(r *rand.Rand, n int) [][]byte {
	s := make([][]byte, n)
	for i := range s {
		b := make([]byte, cda.ShareSize)
		r.Read(b[19:])
		for j := 0; j < 19; j++ {
			b[j] = 0
		}
		s[i] = b
	}
	sort.Slice(s, func(i, j int) bool { return bytes.Compare(s[i], s[j]) < 0 })
	return s
}

// constantShares is pkg/da's generateShares (data_availability_header_test.go:247-263).
func constantShares(n int) [][]byte {
	ns := append(make([]byte, 19), bytes.Repeat([]byte{1}, 10)...)
	s := make([][]byte, n)
	for i := range s {
		s[i] = append(append([]byte{}, ns...), bytes.Repeat([]byte{0xFF}, cda.ShareSize-len(ns))...)
	}
	return s
}

// rfc6962 is go-square merkle.HashFromByteSlices.
func rfc6962(items [][]byte) []byte {
	switch len(items) {
	case 0:
		h := sha256.Sum256(nil)
		return h[:]
	case 1:
		h := sha256.Sum256(append([]byte{0}, items[0]...))
		return h[:]
	}
	k := 1
	for k*2 < len(items) {
		k *= 2
	}
	l, r := rfc6962(items[:k]), rfc6962(items[k:])
	h := sha256.Sum256(append(append([]byte{1}, l...), r...))
	return h[:]
}

func TestExtendSharesReferenceKATs(t *testing.T) {
	for _, tc := range []struct {
		k    int
		want []byte
	}{ // pkg/da/data_availability_header_test.go:34-68
		{2, []byte{0xb5, 0x6e, 0x4d, 0x25, 0x1a, 0xc2, 0x66, 0xf4, 0xb9, 0x1c, 0xc5, 0x46, 0x4b, 0x3f, 0xc7, 0xef,
			0xcb, 0xdc, 0x88, 0x80, 0x64, 0x64, 0x74, 0x96, 0xd1, 0x31, 0x33, 0xf0, 0xdc, 0x65, 0xac, 0x25}},
		{128, []byte{0xb, 0xd3, 0xab, 0xee, 0xac, 0xfb, 0xb0, 0xb9, 0x2d, 0xfb, 0xda, 0xc4, 0xa1, 0x54, 0x86, 0x8e,
			0x3c, 0x4e, 0x79, 0x66, 0x6f, 0x7f, 0xcf, 0x6c, 0x62, 0xb, 0xb9, 0xd, 0xd3, 0xa0, 0xdc, 0xf0}},
	} {
		eds, err := cda.ExtendShares(constantShares(tc.k * tc.k))
		require.NoError(t, err)
		rows, err := eds.RowRoots()
		require.NoError(t, err)
		cols, err := eds.ColRoots()
		require.NoError(t, err)
		require.Equal(t, tc.want, rfc6962(append(rows, cols...)))
	}
}

func TestCodecMatchesLeoRSCodec(t *testing.T) {
	r := rand.New(rand.NewSource(1))
	gpu, cpu := cda.NewCodec(), rsmt2d.NewLeoRSCodec()
	for _, k := range []int{1, 2, 3, 5, 16, 100, 128, 129, 256, 512} { // 2k > 256: GF(2^16)
		data := make([][]byte, k)
		for i := range data {
			data[i] = make([]byte, 512)
			r.Read(data[i])
		}
		want, err := cpu.Encode(data)
		require.NoError(t, err)
		got, err := gpu.Encode(data)
		require.NoError(t, err)
		require.Equal(t, want, got, "k=%d", k)
		shards := append(append([][]byte{}, data...), want...)
		for _, i := range r.Perm(2 * k)[:k] {
			shards[i] = nil
		}
		dec, err := gpu.Decode(append([][]byte{}, shards...))
		require.NoError(t, err)
		require.Equal(t, append(append([][]byte{}, data...), want...), dec, "decode k=%d", k)
	}
}

func TestExtendSharesMatchesCPUPath(t *testing.T) {
	r := rand.New(rand.NewSource(2))
	for _, k := range []int{1, 2, 4, 8, 16, 32, 64, 128, 256} {
		s := sortedShares(r, k*k)
		want, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
		require.NoError(t, err)
		got, err := cda.ExtendShares(s)
		require.NoError(t, err)
		require.Equal(t, want.Flattened(), got.Flattened(), "k=%d", k)
		wr, _ := want.RowRoots()
		gr, _ := got.RowRoots()
		wc, _ := want.ColRoots()
		gc, _ := got.ColRoots()
		require.Equal(t, wr, gr, "k=%d", k)
		require.Equal(t, wc, gc, "k=%d", k)
	}
}

// TestDataAvailabilityHeaderFromSharesMatchesCPUPath: the roots-only consensus entry (../patches/0004) equals
// da.NewDataAvailabilityHeader(rsmt2d.ComputeExtendedDataSquare(...)) on the reference's CPU code, and fails where
// it fails (not a power of two; a namespace-order violation).
func TestDataAvailabilityHeaderFromSharesMatchesCPUPath(t *testing.T) {
	r := rand.New(rand.NewSource(6))
	for _, k := range []int{1, 2, 8, 32, 64, 128} {
		s := sortedShares(r, k*k)
		eds, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
		require.NoError(t, err)
		want, err := da.NewDataAvailabilityHeader(eds)
		require.NoError(t, err)
		rows, cols, hash, err := cda.DataAvailabilityHeaderFromShares(s)
		require.NoError(t, err)
		require.Equal(t, want.RowRoots, rows, "k=%d", k)
		require.Equal(t, want.ColumnRoots, cols, "k=%d", k)
		require.Equal(t, want.Hash(), hash, "k=%d", k)
		got, err := da.NewDataAvailabilityHeaderFromShares(s) // the pkg/da wrapper installed by extend_rocm.go
		require.NoError(t, err)
		require.Equal(t, want.Hash(), got.Hash(), "k=%d", k)
	}
	_, _, _, err := cda.DataAvailabilityHeaderFromShares(make([][]byte, 5))
	require.Error(t, err)
	s := sortedShares(r, 64)
	s[3], s[40] = s[40], s[3]
	_, _, _, err = cda.DataAvailabilityHeaderFromShares(s)
	require.Error(t, err)
}

// waitForFree runs garbage collections until a freed slab is back in the pool (finalizers run asynchronously after
// the cycle that finds the slab unreachable), at most ~2 s.
func waitForFree(t *testing.T, recycledBefore uint64) {
	for i := 0; i < 200; i++ {
		runtime.GC()
		runtime.Gosched()
		if cda.Stats().Recycled > recycledBefore {
			return
		}
		time.Sleep(10 * time.Millisecond)
	}
	t.Fatalf("no slab came back through the finalizer")
}

// TestEDSPoolRecycles: ExtendShares' squares live in pooled page-locked slabs; after the squares (and every slice of
// their cells) are unreachable, a garbage collection returns the slabs, later squares reuse them, and every square
// stays bit-exact however its slab came to it.  Slabs are tracked by address only (uintptr): a map of *byte would
// itself keep every slab reachable (ADVICE r05).
func TestEDSPoolRecycles(t *testing.T) {
	r := rand.New(rand.NewSource(7))
	k := 64 // 8 MiB EDS: pooled
	s := sortedShares(r, k*k)
	ref, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
	require.NoError(t, err)
	want := ref.Flattened()
	seen := map[uintptr]int{}
	for i := 0; i < 12; i++ {
		before := cda.Stats().Recycled
		eds, err := cda.ExtendShares(s)
		require.NoError(t, err)
		flat := eds.Flattened()
		require.Equal(t, want, flat, "call %d", i)
		seen[uintptr(unsafe.Pointer(&flat[0][0]))]++
		eds, flat = nil, nil
		waitForFree(t, before)
	}
	require.Less(t, len(seen), 12, "no slab was reused")
	require.Greater(t, cda.Stats().Hits, uint64(0))
	// a square whose cells are still referenced keeps its slab: the next squares get other slabs
	keep, err := cda.ExtendShares(s)
	require.NoError(t, err)
	cell := keep.GetCell(0, 0)
	row0 := keep.Flattened()[0]
	keep = nil
	runtime.GC()
	runtime.GC()
	for i := 0; i < 4; i++ {
		eds, err := cda.ExtendShares(sortedShares(r, k*k))
		require.NoError(t, err)
		_ = eds
	}
	require.Equal(t, cell, row0)
	require.Equal(t, want[0], row0)
}

// TestReleaseReturnsSlabAtOnce: Release hands a square's slab back without a garbage collection; the next square
// reuses it (same address, a pool hit) and is bit-exact; a square not on a pooled slab is ignored.
func TestReleaseReturnsSlabAtOnce(t *testing.T) {
	r := rand.New(rand.NewSource(8))
	k := 64
	s := sortedShares(r, k*k)
	a, err := cda.ExtendShares(s)
	require.NoError(t, err)
	want := a.Flattened()
	wantCopy := make([][]byte, len(want))
	for i := range want {
		wantCopy[i] = append([]byte(nil), want[i]...)
	}
	base := uintptr(unsafe.Pointer(&want[0][0]))
	want = nil
	st := cda.Stats()
	require.True(t, cda.Release(a))
	require.Equal(t, st.Released+1, cda.Stats().Released)
	b, err := cda.ExtendShares(s)
	require.NoError(t, err)
	fb := b.Flattened()
	require.Equal(t, base, uintptr(unsafe.Pointer(&fb[0][0])), "the released slab is reused")
	require.Equal(t, wantCopy, fb)
	ref, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
	require.NoError(t, err)
	require.False(t, cda.Release(ref))
}

// TestRepairPooledAndInPlace: Repair of an imported square copies into a pooled slab; Repair of a square from
// ExtendShares whose cells were erased runs in place on its own slab (no copy); both restore the square.
func TestRepairPooledAndInPlace(t *testing.T) {
	r := rand.New(rand.NewSource(9))
	k := 64
	w := 2 * k
	s := sortedShares(r, k*k)
	full, err := cda.ExtendShares(s)
	require.NoError(t, err)
	rows, _ := full.RowRoots()
	cols, _ := full.ColRoots()
	want := make([][]byte, w*w)
	for i, c := range full.Flattened() {
		want[i] = append([]byte(nil), c...)
	}
	damaged := func(cells [][]byte) [][]byte {
		out := make([][]byte, len(cells))
		for i, c := range cells {
			if r.Intn(2) == 0 {
				out[i] = c
			}
		}
		return out
	}
	copied := make([][]byte, w*w)
	for i := range want {
		copied[i] = append([]byte(nil), want[i]...)
	}
	imp := damaged(copied)
	require.NoError(t, cda.Repair(mustCtx(t), imp, rows, cols))
	require.Equal(t, want, imp)
	inPlace := damaged(full.Flattened())
	base := uintptr(unsafe.Pointer(&full.Flattened()[0][0]))
	require.NoError(t, cda.Repair(mustCtx(t), inPlace, rows, cols))
	require.Equal(t, want, inPlace)
	for i, c := range inPlace {
		require.Equal(t, base+uintptr(i*cda.ShareSize), uintptr(unsafe.Pointer(&c[0])), "cell %d repaired in place", i)
	}
}

func mustCtx(t *testing.T) *cda.Context {
	x, err := cda.Default()
	require.NoError(t, err)
	return x
}

func TestExtendSquareSplitMatchesCPUPath(t *testing.T) {
	m, err := cda.NewMulti(0)
	require.NoError(t, err)
	defer m.Close()
	r := rand.New(rand.NewSource(5))
	for _, k := range []int{1, 4, 32, 128} {
		s := sortedShares(r, k*k)
		want, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
		require.NoError(t, err)
		got, err := m.ExtendSquareSplit(s, true)
		require.NoError(t, err)
		require.Equal(t, want.Flattened(), got.EDS.Flattened(), "k=%d", k)
		wr, _ := want.RowRoots()
		wc, _ := want.ColRoots()
		require.Equal(t, wr, got.RowRoots, "k=%d", k)
		require.Equal(t, wc, got.ColRoots, "k=%d", k)
		dah, err := da.NewDataAvailabilityHeader(want)
		require.NoError(t, err)
		require.Equal(t, dah.Hash(), got.DataHash, "k=%d", k)
	}
}

func TestTreeConstructorMatchesWrapper(t *testing.T) {
	r := rand.New(rand.NewSource(3))
	k := 16
	s := sortedShares(r, k*k)
	want, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
	require.NoError(t, err)
	got, err := rsmt2d.ComputeExtendedDataSquare(s, cda.NewCodec(), cda.NewConstructor(uint64(k)))
	require.NoError(t, err)
	wr, _ := want.RowRoots()
	gr, _ := got.RowRoots()
	require.Equal(t, wr, gr)
}

func TestRepairMatchesRsmt2d(t *testing.T) {
	r := rand.New(rand.NewSource(4))
	k := 64
	s := sortedShares(r, k*k)
	full, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
	require.NoError(t, err)
	rows, _ := full.RowRoots()
	cols, _ := full.ColRoots()
	flat := full.Flattened()
	damaged := make([][]byte, len(flat))
	for i := range flat {
		if r.Float64() < 0.55 {
			damaged[i] = append([]byte{}, flat[i]...)
		}
	}
	ctx, err := cda.Default()
	require.NoError(t, err)
	require.NoError(t, cda.Repair(ctx, damaged, rows, cols))
	require.Equal(t, flat, damaged)
}

func BenchmarkExtendShares(b *testing.B) {
	s := sortedShares(rand.New(rand.NewSource(5)), 128*128)
	b.Run("gpu", func(b *testing.B) {
		for i := 0; i < b.N; i++ {
			eds, _ := cda.ExtendShares(s)
			_, _ = eds.RowRoots()
		}
	})
	b.Run("cpu-reference", func(b *testing.B) {
		for i := 0; i < b.N; i++ {
			eds, _ := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(128))
			_, _ = eds.RowRoots()
		}
	})
}

// TestCreateCommitmentsMatchGoSquare: one batched GPU call against go-square's inclusion.CreateCommitment per blob
// (x/blob/types/blob_tx.go:98), over blob sizes that give 1 share up to multi-row mountains, at the default
// subtree root threshold and a small one.
func TestCreateCommitmentsMatchGoSquare(t *testing.T) {
	ctx, err := cda.Default()
	require.NoError(t, err)
	r := rand.New(rand.NewSource(11))
	sizes := []int{1, 478, 479, 1000, 4096, 65536, 200000, 1 << 20}
	for _, threshold := range []int{64, 8} {
		blobs := make([]*blob.Blob, len(sizes))
		for i, n := range sizes {
			id := make([]byte, appns.NamespaceVersionZeroIDSize)
			r.Read(id)
			data := make([]byte, n)
			r.Read(data)
			blobs[i] = blob.New(appns.MustNewV0(id), data, 0)
		}
		got, err := cda.CreateBlobCommitments(ctx, blobs, threshold)
		require.NoError(t, err)
		for i, b := range blobs {
			want, err := inclusion.CreateCommitment(b, merkle.HashFromByteSlices, threshold)
			require.NoError(t, err)
			require.Equal(t, want, got[i], "blob %d (%d bytes), threshold %d", i, sizes[i], threshold)
		}
	}
}

// TestConstructExtendCommitMatchesCPUPath: a square built by go-square's square.Construct (the step before
// da.ExtendShares in PrepareProposal / ProcessProposal), read back into its layout plan (SegmentsFromShares) and
// assembled + extended + committed on the GPU from the payload bytes alone, gives the same shares and DAH as the CPU
// path over shares.ToBytes(square).
func TestConstructExtendCommitMatchesCPUPath(t *testing.T) {
	ctx, err := cda.Default()
	require.NoError(t, err)
	r := rand.New(rand.NewSource(12))
	var txs [][]byte
	for i := 0; i < 150; i++ {
		tx := make([]byte, 100+r.Intn(800))
		r.Read(tx)
		txs = append(txs, tx)
	}
	sq, err := square.Construct(txs, 128, 64)
	require.NoError(t, err)
	raw := shares.ToBytes(sq)
	segs, err := cda.SegmentsFromShares(raw)
	require.NoError(t, err)
	got, err := cda.ConstructExtendCommit(ctx, sq.Size(), segs, true, false)
	require.NoError(t, err)
	require.Equal(t, bytes.Join(raw, nil), got.ODS)
	eds, err := rsmt2d.ComputeExtendedDataSquare(raw, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(sq.Size())))
	require.NoError(t, err)
	want, err := da.NewDataAvailabilityHeader(eds)
	require.NoError(t, err)
	require.Equal(t, want.Hash(), got.DataHash)
}

// TestShareInclusionProofParts: the proof parts of cda.ShareInclusionProof verify against the data root
// (merkle.Proof.Verify for the row roots; the NMT range proofs are checked field by field against the CPU
// reference in pkg/proof's TestShareInclusionProofMatchesCPUPath).
func TestShareInclusionProofParts(t *testing.T) {
	ctx, err := cda.Default()
	require.NoError(t, err)
	r := rand.New(rand.NewSource(13))
	k := 16
	s := sortedShares(r, k*k)
	eds, err := rsmt2d.ComputeExtendedDataSquare(s, rsmt2d.NewLeoRSCodec(), wrapper.NewConstructor(uint64(k)))
	require.NoError(t, err)
	dah, err := da.NewDataAvailabilityHeader(eds)
	require.NoError(t, err)
	parts, err := cda.ShareInclusionProof(ctx, s, 5, 40)
	require.NoError(t, err)
	require.Equal(t, dah.Hash(), parts.DataRoot)
	for _, p := range parts.Rows {
		mp := merkle.Proof{Total: p.Total, Index: int64(p.Row), LeafHash: p.LeafHash, Aunts: p.Aunts}
		require.NoError(t, mp.Verify(dah.Hash(), p.RowRoot))
	}
}
