//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

// Nodes is every node of the trees the block path builds for one square (cda_extend_commit_nodes): what
// pkg/inclusion's EDSSubTreeRootCacher records through nmt's NodeVisitor (pkg/inclusion/nmt_caching.go:76-124) and
// what pkg/proof recomputes for proofs (pkg/proof/proof.go:82-153).
type Nodes struct {
	K        int
	RowRoots [][]byte
	ColRoots [][]byte
	DataHash []byte
	// RowNodes[t] / ColNodes[t]: tree t's 4k-1 nodes of 90 bytes, the 2k leaves first, then each level, the root last
	RowNodes [][][]byte
	ColNodes [][][]byte
	// DAHNodes: the RFC-6962 tree over rowRoots ‖ colRoots (8k-1 nodes of 32 bytes), leaf hashes first, the data
	// root last
	DAHNodes [][]byte
}

// Node returns node `pos` of level `level` (0 = leaves) of a tree's flattened node list (w leaves).
func Node(tree [][]byte, w, level, pos int) []byte {
	off := 0
	for l := 0; l < level; l++ {
		off += w >> l
	}
	return tree[off+pos]
}

// ExtendCommitNodes extends the k*k shares and returns every row tree node (and, with cols / dahTree, the column
// trees' and the DAH tree's) from one GPU call.
func ExtendCommitNodes(ctx *Context, s [][]byte, cols, dahTree bool) (*Nodes, error) {
	if !isPowerOfTwo(len(s)) {
		return nil, fmt.Errorf("number of shares is not a power of 2: got %d", len(s))
	}
	flat, n, err := flatten(s)
	if err != nil {
		return nil, err
	}
	k := squareSize(len(s))
	w := 2 * k
	per := (2*w - 1) * NodeSize
	rows := make([]byte, w*NodeSize)
	colr := make([]byte, w*NodeSize)
	dah := make([]byte, 32)
	rn := make([]byte, w*per)
	var cn, dn []byte
	if cols {
		cn = make([]byte, w*per)
	}
	if dahTree {
		dn = make([]byte, (4*w-1)*32)
	}
	var info C.cda_err_info
	rc := C.cda_extend_commit_nodes(ctx.c, C.uint32_t(len(s)), C.uint32_t(n), ptr(flat), nil, ptr(rows), ptr(colr),
		ptr(dah), ptr(rn), ptr(cn), ptr(dn), &info)
	if rc != 0 {
		return nil, toErr(rc, &info)
	}
	out := &Nodes{K: k, RowRoots: split(rows, w), ColRoots: split(colr, w), DataHash: dah}
	out.RowNodes = make([][][]byte, w)
	for t := range out.RowNodes {
		out.RowNodes[t] = split(rn[t*per:(t+1)*per], 2*w-1)
	}
	if cols {
		out.ColNodes = make([][][]byte, w)
		for t := range out.ColNodes {
			out.ColNodes[t] = split(cn[t*per:(t+1)*per], 2*w-1)
		}
	}
	if dahTree {
		out.DAHNodes = split(dn, 4*w-1)
	}
	return out, nil
}

// RowProofPart is one proven row of a share inclusion proof: the row root, its RFC-6962 proof in the data root
// (merkle.ProofsFromByteSlices over rowRoots ‖ colRoots, proof.go:82-93) and the NMT range proof of the row's part
// of the range (tree.ProveRange, proof.go:129-152).
type RowProofPart struct {
	Row      int
	RowRoot  []byte
	Total    int64
	LeafHash []byte
	Aunts    [][]byte // bottom-up
	Start    int32
	End      int32
	Nodes    [][]byte // left to right
}

// ShareProofParts is pkg/proof NewShareInclusionProof's content for ODS shares [start, end): one GPU call extends the
// square, exports the nodes and assembles every proof (cda_share_inclusion_proof); no host hashing.
type ShareProofParts struct {
	StartRow, EndRow int
	Rows             []RowProofPart
	DataRoot         []byte
}

// ShareInclusionProof returns the proof parts of shares [start, end) of the square `s` (k*k shares).
func ShareInclusionProof(ctx *Context, s [][]byte, start, end int) (*ShareProofParts, error) {
	if !isPowerOfTwo(len(s)) {
		return nil, fmt.Errorf("number of shares is not a power of 2: got %d", len(s))
	}
	flat, n, err := flatten(s)
	if err != nil {
		return nil, err
	}
	k := squareSize(len(s))
	lg := 0
	for 1<<lg < 2*k {
		lg++
	}
	var info C.cda_share_proof_info
	rr := make([]byte, k*NodeSize)
	lh := make([]byte, k*32)
	au := make([]byte, k*(lg+1)*32)
	ns := make([]int32, 3*k)
	nodes := make([]byte, k*2*lg*NodeSize+1)
	root := make([]byte, 32)
	var e C.cda_err_info
	rc := C.cda_share_inclusion_proof(ctx.c, C.uint32_t(len(s)), C.uint32_t(n), ptr(flat), C.uint32_t(start),
		C.uint32_t(end), &info, ptr(rr), ptr(lh), ptr(au), (*C.int32_t)(unsafe.Pointer(&ns[0])),
		(*C.int32_t)(unsafe.Pointer(&ns[k])), (*C.int32_t)(unsafe.Pointer(&ns[2*k])), ptr(nodes), ptr(root), &e)
	if rc != 0 {
		return nil, toErr(rc, &e)
	}
	out := &ShareProofParts{StartRow: int(info.start_row), EndRow: int(info.end_row), DataRoot: root}
	maxNodes := int(info.max_nodes)
	for i := 0; i < int(info.nrows); i++ {
		p := RowProofPart{
			Row:      int(info.start_row) + i,
			RowRoot:  rr[i*NodeSize : (i+1)*NodeSize : (i+1)*NodeSize],
			Total:    int64(info.total),
			LeafHash: lh[i*32 : (i+1)*32 : (i+1)*32],
			Start:    ns[i],
			End:      ns[k+i],
		}
		for a := 0; a < int(info.naunts); a++ {
			o := (i*(lg+1) + a) * 32
			p.Aunts = append(p.Aunts, au[o:o+32:o+32])
		}
		for j := 0; j < int(ns[2*k+i]); j++ {
			o := (i*maxNodes + j) * NodeSize
			p.Nodes = append(p.Nodes, nodes[o:o+NodeSize:o+NodeSize])
		}
		out.Rows = append(out.Rows, p)
	}
	return out, nil
}
