//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"fmt"

	"github.com/celestiaorg/rsmt2d"
)

// Repair is (*rsmt2d.ExtendedDataSquare).Repair(rowRoots, colRoots) on the GPU (cda_repair) in one call: the same
// prerepairSanityCheck + solveCrossword order, the same ErrUnrepairableDataSquare / ErrByzantineData{Axis, Index}
// outcomes, and on a Byzantine error the square left as repaired as rsmt2d leaves it.  eds is flattened
// row-major with nil for missing cells; the repaired cells are returned in place of the nils.
//
// libcda repairs 512-byte shares (appconsts.ShareSize) and reads and writes exactly w*w*512 bytes, so the shape is
// checked here before the cgo call: len(eds) == w*w with w = len(rowRoots) == len(colRoots), every non-nil cell
// ShareSize bytes and every root NodeSize bytes.  A mismatch returns an error (as Codec.Decode returns
// reedsolomon.ErrShardSize) instead of letting the library write past a Go buffer.
func Repair(ctx *Context, eds [][]byte, rowRoots, colRoots [][]byte) error {
	w := len(rowRoots)
	if w == 0 || w%2 != 0 || len(colRoots) != w || len(eds) != w*w {
		return fmt.Errorf("cda: Repair needs a %dx%d square and %d roots per axis: got %d cells, %d row and %d column roots",
			w, w, w, len(eds), len(rowRoots), len(colRoots))
	}
	for i, r := range rowRoots {
		if len(r) != NodeSize || len(colRoots[i]) != NodeSize {
			return fmt.Errorf("cda: Repair roots must be %d bytes (axis index %d)", NodeSize, i)
		}
	}
	const n = ShareSize
	for i, c := range eds {
		if c != nil && len(c) != n {
			return fmt.Errorf("cda: Repair cell %d is %d bytes, want %d (shard sizes must be equal)", i, len(c), n)
		}
	}
	// The square to repair in page-locked memory: in place when its present cells already sit in one pooled slab (a
	// square from ExtendShares or an earlier Repair whose cells the caller erased), else the present cells copied
	// into a pooled EDS slab on up to 8 goroutines (a fresh 32 MiB Go buffer per call cost the driver 3.18 / 3.40 ms
	// min / median per C4 repair, BENCH_r05 repair_c4.random).  The repaired cells are slices of the slab, which
	// returns to the pool with the square (Release, or the garbage collector).
	buf := slabOf(eds, n)
	present := make([]byte, w*w)
	for i, c := range eds {
		if len(c) > 0 {
			present[i] = 1
		}
	}
	if buf == nil {
		buf = takeEDS(ctx, w*w*n)
		inParts(w*w, w*w*n, func(i0, i1 int) {
			for i := i0; i < i1; i++ {
				if c := eds[i]; len(c) > 0 {
					copy(buf[i*n:(i+1)*n], c)
				}
			}
		})
	}
	rr, _, _ := flatten(rowRoots)
	cr, _, _ := flatten(colRoots)
	var info C.cda_err_info
	rc := C.cda_repair(ctx.c, C.uint32_t(w/2), ptr(buf), ptr(present), ptr(rr), ptr(cr), &info)
	for i := range eds { // cells repaired so far (also on error)
		if eds[i] == nil && present[i] != 0 {
			eds[i] = buf[i*n : (i+1)*n : (i+1)*n]
		}
	}
	switch int(rc) {
	case 0:
		return nil
	case ErrCodeUnrepairable:
		return rsmt2d.ErrUnrepairableDataSquare
	case ErrCodeByzantine:
		axis := rsmt2d.Row
		if int(info.axis) == 1 {
			axis = rsmt2d.Col
		}
		shares := make([][]byte, w) // the axis as it stood, like rsmt2d's ErrByzantineData.Shares
		for j := 0; j < w; j++ {
			cell := int(info.index)*w + j
			if axis == rsmt2d.Col {
				cell = j*w + int(info.index)
			}
			shares[j] = eds[cell]
		}
		return &rsmt2d.ErrByzantineData{Axis: axis, Index: uint(info.index), Shares: shares}
	default:
		return toErr(rc, &info)
	}
}
