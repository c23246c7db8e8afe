//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"errors"
	"unsafe"

	"github.com/celestiaorg/go-square/blob"
	appns "github.com/celestiaorg/go-square/namespace"
)

// Error codes of the blob path (include/cda.h).
const (
	ErrCodeShareVersion = int(C.CDA_E_SHARE_VERSION)
	ErrCodeBlobSize     = int(C.CDA_E_BLOB_SIZE)
)

// BlobRef is what a share commitment reads from a blob: its 29-byte namespace (version byte then the 28-byte
// ID, go-square share.Namespace.Bytes()), its data and its share version.
type BlobRef struct {
	Namespace    []byte
	Data         []byte
	ShareVersion uint8
}

// CreateCommitments is go-square inclusion.CreateCommitments(blobs, merkle.HashFromByteSlices, threshold) for a
// whole batch in one cda_blob_commitments call: x/blob/types/payforblob.go:53 (MsgPayForBlobs) and the per-blob
// CreateCommitment of ValidateBlobTx (x/blob/types/blob_tx.go:97-105), or every blob of a proposal at once in
// ProcessProposal.  An empty blob returns an *Error with Code ErrCodeBlobSize and an unsupported share version
// ErrCodeShareVersion, Index naming the first offending blob in ValidateBlobs' order (payforblob.go:230-236);
// the caller maps them to types.ErrZeroBlobSize / ErrUnsupportedShareVersion as the reference returns them.
func CreateCommitments(ctx *Context, blobs []BlobRef, subtreeRootThreshold int) ([][]byte, error) {
	n := len(blobs)
	if n == 0 {
		return nil, nil
	}
	if subtreeRootThreshold <= 0 {
		return nil, errors.New("cda: subtree root threshold must be positive")
	}
	ns := make([]byte, n*NamespaceSize)
	versions := make([]byte, n)
	offsets := make([]uint64, n+1)
	total := 0
	for i, b := range blobs {
		if len(b.Namespace) != NamespaceSize {
			return nil, errors.New("cda: blob namespace must be 29 bytes")
		}
		copy(ns[i*NamespaceSize:], b.Namespace)
		versions[i] = b.ShareVersion
		total += len(b.Data)
		offsets[i+1] = uint64(total)
	}
	data := make([]byte, total+1) // +1: a valid pointer even when every blob is empty
	for i, b := range blobs {
		copy(data[offsets[i]:], b.Data)
	}
	out := make([]byte, n*32)
	var info C.cda_err_info
	rc := C.cda_blob_commitments(ctx.c, C.uint32_t(n), ptr(ns), ptr(data), (*C.uint64_t)(unsafe.Pointer(&offsets[0])),
		ptr(versions), C.uint32_t(subtreeRootThreshold), ptr(out), &info)
	if err := toErr(rc, &info); err != nil {
		return nil, err
	}
	return split(out, n), nil
}

// RefOf reads a go-square blob (x/blob/types/payforblob.go:221 builds its namespace the same way).
func RefOf(b *blob.Blob) (BlobRef, error) {
	ns, err := appns.New(uint8(b.NamespaceVersion), b.NamespaceId)
	if err != nil {
		return BlobRef{}, err
	}
	return BlobRef{Namespace: ns.Bytes(), Data: b.Data, ShareVersion: uint8(b.ShareVersion)}, nil
}

// CreateBlobCommitments is CreateCommitments over go-square blobs (the []*blob.Blob of a BlobTx or a proposal).
func CreateBlobCommitments(ctx *Context, blobs []*blob.Blob, subtreeRootThreshold int) ([][]byte, error) {
	refs := make([]BlobRef, len(blobs))
	for i, b := range blobs {
		r, err := RefOf(b)
		if err != nil {
			return nil, err
		}
		refs[i] = r
	}
	return CreateCommitments(ctx, refs, subtreeRootThreshold)
}

// CreateCommitment is go-square inclusion.CreateCommitment for one blob.
func CreateCommitment(ctx *Context, b BlobRef, subtreeRootThreshold int) ([]byte, error) {
	c, err := CreateCommitments(ctx, []BlobRef{b}, subtreeRootThreshold)
	if err != nil {
		return nil, err
	}
	return c[0], nil
}

// MerkleRoots is merkle.HashFromByteSlices over each set of 90-byte NMT nodes, one cda_merkle_roots call for all
// sets: the subtree-root fold of pkg/inclusion/get_commit.go:29 (GetCommitment) when many commitments are
// recomputed from one square.  An empty set hashes to SHA256("").
func MerkleRoots(ctx *Context, sets [][][]byte) ([][]byte, error) {
	n := len(sets)
	if n == 0 {
		return nil, nil
	}
	offsets := make([]uint32, n+1)
	total := 0
	for i, s := range sets {
		total += len(s)
		offsets[i+1] = uint32(total)
	}
	items := make([]byte, total*NodeSize+1)
	k := 0
	for _, s := range sets {
		for _, node := range s {
			if len(node) != NodeSize {
				return nil, errors.New("cda: merkle set items must be 90-byte NMT nodes")
			}
			copy(items[k*NodeSize:], node)
			k++
		}
	}
	out := make([]byte, n*32)
	rc := C.cda_merkle_roots(ctx.c, C.uint32_t(n), (*C.uint32_t)(unsafe.Pointer(&offsets[0])), ptr(items),
		C.uint32_t(NodeSize), ptr(out))
	if err := toErr(rc, nil); err != nil {
		return nil, err
	}
	return split(out, n), nil
}
