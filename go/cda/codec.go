//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"fmt"

	"github.com/celestiaorg/rsmt2d"
	"github.com/klauspost/reedsolomon"
)

// Codec is rsmt2d.Codec on the GPU: klauspost/reedsolomon v1.12.1 Leopard (GF(2^8) for 2k <= 256, GF(2^16)
// above), bit-exact with rsmt2d.LeoRSCodec.  Name() is "Leopard", so rsmt2d's codec registry and every
// consumer that records the codec name see the same codec.
type Codec struct {
	ctx *Context
}

// NewCodec returns the GPU codec on the process-wide context; it has NewLeoRSCodec's shape so it can be
// assigned to appconsts.DefaultCodec once that variable is typed func() rsmt2d.Codec.
func NewCodec() rsmt2d.Codec { return &Codec{ctx: mustDefault()} }

// NewCodecOn returns the GPU codec on a given context.
func NewCodecOn(ctx *Context) *Codec { return &Codec{ctx: ctx} }

// Encode returns the k parity shards of k data shards (LeoRSCodec.Encode).
func (c *Codec) Encode(data [][]byte) ([][]byte, error) {
	flat, n, err := flatten(data)
	if err != nil {
		return nil, err
	}
	if len(data) == 0 {
		return nil, reedsolomon.ErrShortData
	}
	parity := make([]byte, len(flat))
	if rc := C.cda_rs_encode(c.ctx.c, C.uint32_t(len(data)), C.uint32_t(n), ptr(flat), ptr(parity)); rc != 0 {
		return nil, toErr(rc, nil)
	}
	return split(parity, len(data)), nil
}

// Decode fills the nil (missing) shards of data ‖ parity and returns all 2k shards (LeoRSCodec.Decode).
func (c *Codec) Decode(shards [][]byte) ([][]byte, error) {
	total, n := len(shards), 0
	for _, s := range shards {
		if len(s) > 0 {
			n = len(s)
			break
		}
	}
	if total == 0 || total%2 != 0 || n == 0 {
		return nil, reedsolomon.ErrTooFewShards
	}
	buf := make([]byte, total*n)
	present := make([]byte, total)
	for i, s := range shards {
		if len(s) > 0 {
			if len(s) != n {
				return nil, reedsolomon.ErrShardSize
			}
			copy(buf[i*n:], s)
			present[i] = 1
		}
	}
	rc := C.cda_rs_decode(c.ctx.c, C.uint32_t(total/2), C.uint32_t(n), ptr(buf), ptr(present))
	if int(rc) == ErrCodeTooFew {
		return nil, reedsolomon.ErrTooFewShards
	}
	if rc != 0 {
		return nil, toErr(rc, nil)
	}
	out := split(buf, total)
	for i, s := range shards { // present shards are returned as given, like klauspost's Reconstruct
		if len(s) > 0 {
			out[i] = s
		}
	}
	return out, nil
}

// MaxChunks is LeoRSCodec.MaxChunks (32768 * 32768).
func (c *Codec) MaxChunks() int { return int(C.cda_rs_max_chunks()) }

// Name is rsmt2d.Leopard.
func (c *Codec) Name() string { return C.GoString(C.cda_rs_name()) }

// ValidateChunkSize is LeoRSCodec.ValidateChunkSize: Leopard needs multiples of 64 bytes.
func (c *Codec) ValidateChunkSize(chunkSize int) error {
	if C.cda_rs_validate_chunk_size(C.int64_t(chunkSize)) != 0 {
		return fmt.Errorf("chunkSize %d must be a multiple of 64 bytes", chunkSize)
	}
	return nil
}
