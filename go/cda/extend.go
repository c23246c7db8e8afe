//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"fmt"
	"math"

	"github.com/celestiaorg/rsmt2d"
)

func isPowerOfTwo(n int) bool { return n > 0 && n&(n-1) == 0 }

// squareSize is da.SquareSize (data_availability_header.go:205-216): next power of two >= ceil(sqrt(len)).
func squareSize(n int) int {
	k := int(math.Ceil(math.Sqrt(float64(n))))
	p := 1
	for p < k {
		p <<= 1
	}
	return p
}

// ExtendShares is da.ExtendShares (pkg/da/data_availability_header.go:65-75) in one GPU call: the 2-D Leopard
// extension, every row and column NMT root (and the DAH) are computed by cda_extend_commit; the EDS comes back as
// an *rsmt2d.ExtendedDataSquare built by rsmt2d.ImportExtendedDataSquare, whose tree constructor returns the GPU
// roots on the first RowRoots / ColRoots pass, so da.NewDataAvailabilityHeader needs no hashing.
func ExtendShares(s [][]byte) (*rsmt2d.ExtendedDataSquare, error) {
	return ExtendSharesOn(mustDefault(), s)
}

// ExtendSharesOn is ExtendShares on a given context.  A square of 512-byte shares is flattened straight into Q0 of a
// pooled page-locked EDS slab (pool.go) and extended in place by cda_extend_commit_eds: no separate share buffer, no
// host copy of Q0, the input and output copies are direct DMAs, and the returned square's cells live in the slab.
// Anything else (another share size, a count that is not a square) takes cda_extend_commit, which reports the
// reference's errors in the reference's order.
func ExtendSharesOn(ctx *Context, s [][]byte) (*rsmt2d.ExtendedDataSquare, error) {
	if !isPowerOfTwo(len(s)) {
		return nil, fmt.Errorf("number of shares is not a power of 2: got %d", len(s))
	}
	n := len(s[0])
	k := squareSize(len(s))
	w := 2 * k
	if n == ShareSize && k*k == len(s) {
		eds := takeEDS(ctx, w*w*n)
		if err := flattenQ0(eds, s, k); err != nil {
			return nil, err
		}
		rows := make([]byte, w*NodeSize)
		cols := make([]byte, w*NodeSize)
		dah := make([]byte, 32)
		var info C.cda_err_info
		rc := C.cda_extend_commit_eds(ctx.c, C.uint32_t(k), ptr(eds), ptr(rows), ptr(cols), ptr(dah), &info)
		if rc != 0 {
			return nil, toErr(rc, &info)
		}
		return importWithRoots(ctx, eds, w, n, rows, cols)
	}
	flat, arr := takeShares(ctx, len(s)*n)
	defer giveShares(ctx, len(s)*n, arr)
	if err := flattenInto(flat, s, n); err != nil {
		return nil, err
	}
	eds := takeEDS(ctx, w*w*n)
	rows := make([]byte, w*NodeSize)
	cols := make([]byte, w*NodeSize)
	dah := make([]byte, 32)
	var info C.cda_err_info
	rc := C.cda_extend_commit(ctx.c, C.uint32_t(len(s)), C.uint32_t(n), ptr(flat), ptr(eds), ptr(rows), ptr(cols),
		ptr(dah), &info)
	if rc != 0 {
		return nil, toErr(rc, &info)
	}
	return importWithRoots(ctx, eds, w, n, rows, cols)
}

// DataAvailabilityHeaderFromShares is da.NewDataAvailabilityHeader(da.ExtendShares(s)) for callers that read only
// the header -- PrepareProposal and ProcessProposal use nothing of the square but dah.Hash()
// (app/prepare_proposal.go:65-93, app/process_proposal.go:137-151): the same row roots, column roots and data hash
// (and the same errors: not a power of two, not a square, namespace push order) from one cda_extend_commit with no
// EDS copied back.  pkg/da wraps it as da.NewDataAvailabilityHeaderFromShares (../patches/0004).
func DataAvailabilityHeaderFromShares(s [][]byte) (rowRoots, colRoots [][]byte, dataHash []byte, err error) {
	return DataAvailabilityHeaderFromSharesOn(mustDefault(), s)
}

// DataAvailabilityHeaderFromSharesOn is DataAvailabilityHeaderFromShares on a given context.
func DataAvailabilityHeaderFromSharesOn(ctx *Context, s [][]byte) (rowRoots, colRoots [][]byte, dataHash []byte,
	err error) {
	if !isPowerOfTwo(len(s)) {
		return nil, nil, nil, fmt.Errorf("number of shares is not a power of 2: got %d", len(s))
	}
	n := len(s[0])
	flat, arr := takeShares(ctx, len(s)*n)
	defer giveShares(ctx, len(s)*n, arr)
	if err := flattenInto(flat, s, n); err != nil {
		return nil, nil, nil, err
	}
	w := 2 * squareSize(len(s))
	rows := make([]byte, w*NodeSize)
	cols := make([]byte, w*NodeSize)
	dah := make([]byte, 32)
	var info C.cda_err_info
	rc := C.cda_extend_commit(ctx.c, C.uint32_t(len(s)), C.uint32_t(n), ptr(flat), nil, ptr(rows), ptr(cols),
		ptr(dah), &info)
	if rc != 0 {
		return nil, nil, nil, toErr(rc, &info)
	}
	return split(rows, w), split(cols, w), dah, nil
}

// importWithRoots wraps the GPU's EDS as an *rsmt2d.ExtendedDataSquare whose row and column roots are already
// set: RowRoots / ColRoots run here, before the square is handed out, so the root cache's trees only ever see the
// imported, unmodified cells.  Any later tree (Repair, or re-rooting after SetCell) is a full Tree that hashes what
// is pushed to it.
func importWithRoots(ctx *Context, eds []byte, w, n int, rows, cols []byte) (*rsmt2d.ExtendedDataSquare, error) {
	cache := &rootCache{}
	cache.roots[0] = split(rows, w)
	cache.roots[1] = split(cols, w)
	cache.used[0] = make([]bool, w)
	cache.used[1] = make([]bool, w)
	// The square carries the reference's CPU codec for whatever rsmt2d does with it later axis by axis (Repair after
	// cells are erased, re-extension): per axis through host buffers the CPU codec is not slower than the GPU's
	// (DESIGN.md §12.1).  cda.Repair repairs a whole square on the GPU in one call.
	sq, err := rsmt2d.ImportExtendedDataSquare(split(eds, w*w), rsmt2d.NewLeoRSCodec(), cache.constructor(ctx, uint64(w/2)))
	if err != nil {
		return nil, err
	}
	if _, err := sq.RowRoots(); err != nil {
		return nil, err
	}
	if _, err := sq.ColRoots(); err != nil {
		return nil, err
	}
	return sq, nil
}

// Block is one extended block of a batch: the EDS and the DAH inputs.
type Block struct {
	EDS      *rsmt2d.ExtendedDataSquare
	RowRoots [][]byte
	ColRoots [][]byte
	DataHash []byte // DataAvailabilityHeader.Hash (pkg/da/data_availability_header.go:92-108)
}

// Multi is cda_multi: one handle over the GPUs of this process (device mask bit d = HIP device d, 0 = all).
type Multi struct {
	m *C.cda_multi
}

// NewMulti opens every device in mask.
func NewMulti(mask uint32) (*Multi, error) {
	var m *C.cda_multi
	if rc := C.cda_multi_init(C.uint32_t(mask), &m); rc != 0 {
		return nil, toErr(rc, nil)
	}
	return &Multi{m: m}, nil
}

// Close releases the handle's device contexts.  Blocks returned by ExtendBlocks do not depend on them: their
// squares use the process-wide DefaultOn contexts, so they stay valid after Close.
func (m *Multi) Close() {
	if m.m != nil {
		C.cda_multi_free(m.m)
		m.m = nil
	}
}

// ExtendBlocks extends and commits many independent blocks (k*k shares each, same k), sharded over the devices;
// with withEDS false only the roots and data hashes come back (ProcessProposal needs nothing else).
func (m *Multi) ExtendBlocks(blocks [][][]byte, withEDS bool) ([]Block, error) {
	nb := len(blocks)
	if nb == 0 {
		return nil, nil
	}
	count := len(blocks[0])
	if !isPowerOfTwo(count) {
		return nil, fmt.Errorf("number of shares is not a power of 2: got %d", count)
	}
	k := squareSize(count)
	if k*k != count {
		return nil, &Error{Code: ErrCodeNotSquare, Axis: -1, Index: -1, Leaf: -1, Block: 0}
	}
	w := 2 * k
	ods := make([]byte, nb*count*ShareSize)
	for b, s := range blocks {
		if len(s) != count {
			return nil, fmt.Errorf("block %d has %d shares, want %d", b, len(s), count)
		}
		for i, sh := range s {
			if len(sh) != ShareSize {
				return nil, fmt.Errorf("block %d share %d is %d bytes", b, i, len(sh))
			}
			copy(ods[(b*count+i)*ShareSize:], sh)
		}
	}
	var eds []byte
	if withEDS {
		eds = make([]byte, nb*w*w*ShareSize)
	}
	rows := make([]byte, nb*w*NodeSize)
	cols := make([]byte, nb*w*NodeSize)
	dah := make([]byte, nb*32)
	var info C.cda_err_info
	rc := C.cda_multi_extend_commit_batch(m.m, C.uint32_t(k), C.uint32_t(nb), ptr(ods), ptr(eds), ptr(rows), ptr(cols),
		ptr(dah), &info)
	if rc != 0 {
		return nil, toErr(rc, &info)
	}
	var ctx *Context
	if withEDS { // the squares outlive m: their codec / trees run on the process-wide context of m's first device
		var err error
		if ctx, err = DefaultOn(int(C.cda_multi_device(m.m, 0))); err != nil {
			return nil, err
		}
	}
	out := make([]Block, nb)
	for b := range out {
		r := rows[b*w*NodeSize : (b+1)*w*NodeSize]
		c := cols[b*w*NodeSize : (b+1)*w*NodeSize]
		out[b].RowRoots, out[b].ColRoots, out[b].DataHash = split(r, w), split(c, w), dah[b*32:(b+1)*32]
		if withEDS {
			sq, err := importWithRoots(ctx, eds[b*w*w*ShareSize:(b+1)*w*w*ShareSize], w, ShareSize, r, c)
			if err != nil {
				return nil, err
			}
			out[b].EDS = sq
		}
	}
	return out, nil
}

// ExtendSquareSplit extends and commits ONE square with its work split over the handle's devices
// (cda_multi_extend_commit_split, SURVEY.md §8e config C5): the row pass, the exchange of row-encoded shares and
// leaf records over RCCL, the column pass and the tree folds run on every device, the DAH on the first.  The
// result equals ExtendShares on the same shares; with withEDS false only the roots and the data hash come back.
func (m *Multi) ExtendSquareSplit(s [][]byte, withEDS bool) (Block, error) {
	count := len(s)
	if !isPowerOfTwo(count) {
		return Block{}, fmt.Errorf("number of shares is not a power of 2: got %d", count)
	}
	k := squareSize(count)
	if k*k != count {
		return Block{}, &Error{Code: ErrCodeNotSquare, Axis: -1, Index: -1, Leaf: -1, Block: 0}
	}
	flat, n, err := flatten(s)
	if err != nil {
		return Block{}, err
	}
	if n != ShareSize {
		return Block{}, fmt.Errorf("shares are %d bytes, the split path takes %d", n, ShareSize)
	}
	w := 2 * k
	var eds []byte
	if withEDS {
		eds = make([]byte, w*w*ShareSize)
	}
	rows := make([]byte, w*NodeSize)
	cols := make([]byte, w*NodeSize)
	dah := make([]byte, 32)
	var info C.cda_err_info
	rc := C.cda_multi_extend_commit_split(m.m, C.uint32_t(k), ptr(flat), ptr(eds), ptr(rows), ptr(cols), ptr(dah), &info)
	if rc != 0 {
		return Block{}, toErr(rc, &info)
	}
	out := Block{RowRoots: split(rows, w), ColRoots: split(cols, w), DataHash: dah}
	if withEDS {
		ctx, err := DefaultOn(int(C.cda_multi_device(m.m, 0)))
		if err != nil {
			return Block{}, err
		}
		if out.EDS, err = importWithRoots(ctx, eds, w, ShareSize, rows, cols); err != nil {
			return Block{}, err
		}
	}
	return out, nil
}
