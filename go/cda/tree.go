//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"bytes"
	"fmt"
	"sync"

	"github.com/celestiaorg/rsmt2d"

	"github.com/celestiaorg/celestia-app/v2/pkg/wrapper"
)

var parityNamespace = bytes.Repeat([]byte{0xFF}, NamespaceSize) // appns.ParitySharesNamespace

// Tree is wrapper.ErasuredNamespacedMerkleTree (pkg/wrapper/nmt_wrapper.go:26-140) with the hashing on the GPU:
// Push keeps the reference's checks and error order, Root hashes every pushed leaf in one cda_nmt_axis_root.
type Tree struct {
	ctx        *Context
	squareSize uint64
	axisIndex  uint64
	shareIndex uint64
	leaves     []byte
	leafLen    int
	lastNs     []byte
}

var _ rsmt2d.Tree = (*Tree)(nil)

// NewConstructor is wrapper.NewConstructor(squareSize) (nmt_wrapper.go:73-86) on the GPU.
func NewConstructor(squareSize uint64) rsmt2d.TreeConstructorFn {
	ctx := mustDefault()
	return func(_ rsmt2d.Axis, axisIndex uint) rsmt2d.Tree {
		return newTree(ctx, squareSize, uint64(axisIndex))
	}
}

func newTree(ctx *Context, squareSize, axisIndex uint64) *Tree {
	if squareSize == 0 {
		panic("cannot create a ErasuredNamespacedMerkleTree of squareSize == 0")
	}
	return &Tree{ctx: ctx, squareSize: squareSize, axisIndex: axisIndex}
}

func (t *Tree) isQuadrantZero() bool { return t.shareIndex < t.squareSize && t.axisIndex < t.squareSize }

// Push (nmt_wrapper.go:93-114 + nmt's namespace-order check).
func (t *Tree) Push(data []byte) error {
	if t.axisIndex+1 > 2*t.squareSize || t.shareIndex+1 > 2*t.squareSize {
		return fmt.Errorf("pushed past predetermined square size: boundary at %d index at %d %d",
			2*t.squareSize, t.axisIndex, t.shareIndex)
	}
	if len(data) < NamespaceSize {
		return fmt.Errorf("data is too short to contain namespace ID")
	}
	if t.leafLen == 0 {
		t.leafLen = len(data)
	} else if len(data) != t.leafLen {
		return fmt.Errorf("cda: leaves of unequal length (%d vs %d)", len(data), t.leafLen)
	}
	ns := parityNamespace
	if t.isQuadrantZero() {
		ns = data[:NamespaceSize]
	}
	if t.lastNs != nil && bytes.Compare(ns, t.lastNs) < 0 {
		return fmt.Errorf("pushed data has smaller namespace than previous: last %x, pushed %x", t.lastNs, ns)
	}
	t.lastNs = ns
	t.leaves = append(t.leaves, data...)
	t.shareIndex++
	return nil
}

// Root (nmt_wrapper.go:118-124): the 90-byte NMT root of the pushed leaves.
func (t *Tree) Root() ([]byte, error) {
	root := make([]byte, NodeSize)
	var info C.cda_err_info
	rc := C.cda_nmt_axis_root(t.ctx.c, C.uint64_t(t.squareSize), C.uint64_t(t.axisIndex), C.uint32_t(t.shareIndex),
		C.uint32_t(t.leafLen), ptr(t.leaves), ptr(root), &info)
	if rc != 0 {
		return nil, toErr(rc, &info)
	}
	return root, nil
}

// rootCache hands out the roots the GPU computed for a whole square, once per axis: the computeRoots pass that
// importWithRoots runs on the freshly imported square (before any caller can change a cell) reads them instead of
// re-hashing (cda_extend_commit already checked every push order).  Every later tree of the square -- rsmt2d builds
// one only after cells changed, e.g. in Repair -- is the reference's wrapper tree (pkg/wrapper, hashing on the CPU):
// one axis root through host memory is not faster on the GPU (DESIGN.md §12.1).
type rootCache struct {
	mu    sync.Mutex
	roots [2][][]byte // [rsmt2d.Row / rsmt2d.Col][index]
	used  [2][]bool
}

// cachedTree is the first tree of an axis: it counts pushes and returns the GPU root.
type cachedTree struct {
	root       []byte
	squareSize uint64
	axisIndex  uint64
	pushed     uint64
}

func (t *cachedTree) Push(data []byte) error {
	if t.axisIndex+1 > 2*t.squareSize || t.pushed+1 > 2*t.squareSize {
		return fmt.Errorf("pushed past predetermined square size: boundary at %d index at %d %d",
			2*t.squareSize, t.axisIndex, t.pushed)
	}
	if len(data) < NamespaceSize {
		return fmt.Errorf("data is too short to contain namespace ID")
	}
	t.pushed++
	return nil
}

func (t *cachedTree) Root() ([]byte, error) {
	if t.pushed != 2*t.squareSize { // only a whole-axis computeRoots pass may read the precomputed root
		return nil, fmt.Errorf("cda: cached root of axis %d requested after %d of %d pushes", t.axisIndex, t.pushed,
			2*t.squareSize)
	}
	return append([]byte(nil), t.root...), nil
}

func (c *rootCache) constructor(ctx *Context, squareSize uint64) rsmt2d.TreeConstructorFn {
	return func(axis rsmt2d.Axis, axisIndex uint) rsmt2d.Tree {
		a := 0
		if axis == rsmt2d.Col {
			a = 1
		}
		idx := int(axisIndex)
		c.mu.Lock()
		first := idx < len(c.used[a]) && !c.used[a][idx]
		if first {
			c.used[a][idx] = true
		}
		c.mu.Unlock()
		if first {
			return &cachedTree{root: c.roots[a][idx], squareSize: squareSize, axisIndex: uint64(axisIndex)}
		}
		return wrapper.NewConstructor(squareSize)(axis, axisIndex)
	}
}
