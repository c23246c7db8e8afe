//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"github.com/celestiaorg/rsmt2d"
)

// Repair is (*rsmt2d.ExtendedDataSquare).Repair(rowRoots, colRoots) on the GPU (cda_repair): the same
// prerepairSanityCheck + solveCrossword order, the same ErrUnrepairableDataSquare / ErrByzantineData{Axis, Index}
// outcomes, and on a Byzantine error the square left as repaired as rsmt2d leaves it.  eds is flattened
// row-major with nil for missing cells; the repaired cells are returned in place of the nils.
func Repair(ctx *Context, eds [][]byte, rowRoots, colRoots [][]byte) error {
	w := len(rowRoots)
	n := 0
	for _, c := range eds {
		if len(c) > 0 {
			n = len(c)
			break
		}
	}
	if n == 0 {
		n = ShareSize
	}
	buf := make([]byte, w*w*n)
	present := make([]byte, w*w)
	for i, c := range eds {
		if len(c) > 0 {
			copy(buf[i*n:], c)
			present[i] = 1
		}
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
