//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"bytes"
	"encoding/binary"
	"fmt"
	"unsafe"

	"github.com/celestiaorg/rsmt2d"
)

// Segment kinds of a square layout plan (include/cda.h cda_share_segment).
const (
	SegCompact = C.CDA_SEG_COMPACT
	SegSparse  = C.CDA_SEG_SPARSE
	SegPadding = C.CDA_SEG_PADDING
)

// Segment is one run of shares of a square layout plan: a compact sequence (the TRANSACTION or PAY_FOR_BLOB
// namespace's varint-delimited units), a blob's sparse shares, or a run of identical padding shares
// (specs/src/specs/shares.md:31-122).  Data is the sequence's payload, Reserved the compact shares' reserved bytes.
type Segment struct {
	Kind         uint32
	FirstShare   uint32
	NShares      uint32
	ShareVersion uint32
	Namespace    []byte // 29 bytes
	Data         []byte // COMPACT: the varint-delimited sequence; SPARSE: the blob data; PADDING: empty
	Reserved     []uint32
}

var (
	txNamespace  = append(make([]byte, 28), 0x01) // appns.TxNamespace
	pfbNamespace = append(make([]byte, 28), 0x04) // appns.PayForBlobNamespace
)

// SegmentsFromShares reads the layout plan back from a constructed square's shares (go-square square.Construct /
// Build, app/process_proposal.go:121, app/prepare_proposal.go:54): only the payload bytes, not the k*k shares, then
// cross PCIe in ConstructExtendCommit, and the GPU writes the shares itself.  Share headers: namespace ‖ info byte
// (share version << 1 | sequence start) ‖ sequence length (first share) ‖ reserved bytes (compact shares) ‖ payload.
func SegmentsFromShares(s [][]byte) ([]Segment, error) {
	var segs []Segment
	for i := 0; i < len(s); i++ {
		sh := s[i]
		if len(sh) != ShareSize {
			return nil, fmt.Errorf("share %d is %d bytes", i, len(sh))
		}
		ns, info := sh[:NamespaceSize], sh[NamespaceSize]
		start := info&1 == 1
		compact := bytes.Equal(ns, txNamespace) || bytes.Equal(ns, pfbNamespace)
		if !start {
			return nil, fmt.Errorf("share %d continues no sequence", i)
		}
		seqLen := binary.BigEndian.Uint32(sh[NamespaceSize+1:])
		if !compact && seqLen == 0 { // padding: a run of identical shares, each one a sequence start of length 0
			j := i + 1
			for j < len(s) && bytes.Equal(s[j], sh) {
				j++
			}
			segs = append(segs, Segment{Kind: SegPadding, FirstShare: uint32(i), NShares: uint32(j - i),
				ShareVersion: uint32(info >> 1), Namespace: ns})
			i = j - 1
			continue
		}
		seg := Segment{Kind: SegSparse, FirstShare: uint32(i), ShareVersion: uint32(info >> 1), Namespace: ns}
		hdr0, hdrN := NamespaceSize+1+4, NamespaceSize+1
		if compact {
			seg.Kind = SegCompact
			hdr0, hdrN = hdr0+4, hdrN+4
		}
		data := make([]byte, 0, seqLen)
		for j := i; ; j++ {
			if j >= len(s) || (j > i && (!bytes.Equal(s[j][:NamespaceSize], ns) || s[j][NamespaceSize]&1 == 1)) {
				seg.NShares = uint32(j - i)
				i = j - 1
				break
			}
			hdr := hdrN
			if j == i {
				hdr = hdr0
			}
			if compact {
				seg.Reserved = append(seg.Reserved, binary.BigEndian.Uint32(s[j][hdr-4:]))
			}
			data = append(data, s[j][hdr:]...)
		}
		if uint32(len(data)) < seqLen {
			return nil, fmt.Errorf("sequence at share %d is shorter than its length %d", seg.FirstShare, seqLen)
		}
		seg.Data = data[:seqLen]
		segs = append(segs, seg)
	}
	return segs, nil
}

// Square is the result of ConstructExtendCommit.
type Square struct {
	ODS      []byte // k*k*512 row-major, when asked for
	EDS      *rsmt2d.ExtendedDataSquare
	RowRoots [][]byte
	ColRoots [][]byte
	DataHash []byte
}

// ConstructExtendCommit is square.Construct + shares.ToBytes + da.ExtendShares + NewDataAvailabilityHeader of a
// k x k square from its layout plan in one call (cda_construct_extend_commit): the payload bytes go up, the shares
// are assembled in device memory and extended and committed there.
func ConstructExtendCommit(ctx *Context, k int, segs []Segment, wantODS, wantEDS bool) (*Square, error) {
	if len(segs) == 0 {
		return nil, fmt.Errorf("cda: empty layout plan")
	}
	recs := make([]C.cda_share_segment, len(segs))
	var data []byte
	var reserved []uint32
	for i, sg := range segs {
		if len(sg.Namespace) != NamespaceSize {
			return nil, fmt.Errorf("segment %d: namespace of %d bytes", i, len(sg.Namespace))
		}
		r := &recs[i]
		r.kind, r.first_share, r.nshares, r.share_version = C.uint32_t(sg.Kind), C.uint32_t(sg.FirstShare),
			C.uint32_t(sg.NShares), C.uint32_t(sg.ShareVersion)
		r.data_off, r.data_len = C.uint64_t(len(data)), C.uint64_t(len(sg.Data))
		if sg.Kind == SegCompact {
			r.reserved_off = C.uint32_t(len(reserved))
		}
		for j := 0; j < NamespaceSize; j++ {
			r.ns[j] = C.uint8_t(sg.Namespace[j])
		}
		data = append(data, sg.Data...)
		reserved = append(reserved, sg.Reserved...)
	}
	if len(data) == 0 {
		data = []byte{0}
	}
	if len(reserved) == 0 {
		reserved = []uint32{0}
	}
	w := 2 * k
	out := &Square{}
	var ods, eds []byte
	if wantODS {
		ods = make([]byte, k*k*ShareSize)
	}
	if wantEDS {
		eds = takeEDS(ctx, w*w*ShareSize)
	}
	rows := make([]byte, w*NodeSize)
	cols := make([]byte, w*NodeSize)
	dah := make([]byte, 32)
	var info C.cda_err_info
	rc := C.cda_construct_extend_commit(ctx.c, C.uint32_t(k), C.uint32_t(len(recs)), &recs[0], ptr(data),
		C.uint64_t(len(data)), (*C.uint32_t)(unsafe.Pointer(&reserved[0])), C.uint32_t(len(reserved)), ptr(ods),
		ptr(eds), ptr(rows), ptr(cols), ptr(dah), &info)
	if rc != 0 {
		return nil, toErr(rc, &info)
	}
	out.ODS, out.RowRoots, out.ColRoots, out.DataHash = ods, split(rows, w), split(cols, w), dah
	if wantEDS {
		sq, err := importWithRoots(ctx, eds, w, ShareSize, rows, cols)
		if err != nil {
			return nil, err
		}
		out.EDS = sq
	}
	return out, nil
}
