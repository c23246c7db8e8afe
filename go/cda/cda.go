//go:build rocm

// Package cda binds libcda.so (include/cda.h), the MI355X data-availability engine, into celestia-app.
//
// It keeps the reference's call surface:
//   - Codec implements rsmt2d.Codec (Encode / Decode / MaxChunks / Name / ValidateChunkSize); a caller may opt in to
//     it behind appconsts.DefaultCodec (pkg/appconsts/global_consts.go:92, after the one-line retype in
//     ../patches/0001-appconsts-DefaultCodec-codec-interface.patch).  The rocm build does not: per axis the GPU
//     does not beat the CPU codec (INTEGRATION.md §2), so only the whole-square operations below go to the GPU;
//   - NewConstructor is an rsmt2d.TreeConstructorFn with wrapper.NewConstructor's semantics
//     (pkg/wrapper/nmt_wrapper.go:73-140) whose Root() hashes on the GPU;
//   - ExtendShares has da.ExtendShares' signature (pkg/da/data_availability_header.go:65-75) and returns an
//     *rsmt2d.ExtendedDataSquare, so da.NewDataAvailabilityHeader, Hash and every caller stay unchanged
//     (../patches/0002-da-ExtendShares-rocm-fast-path.patch routes da.ExtendShares here under -tags rocm).
//
// Build (go/README.md): copy this directory to pkg/cda, then
//   CGO_ENABLED=1 CGO_CFLAGS=-I<engine>/include \
//   CGO_LDFLAGS="-L<engine>/celestia-app_amd/cda -Wl,-rpath,<engine>/celestia-app_amd/cda" go build -tags rocm ./...
// (the reference Dockerfile sets CGO_ENABLED=0, Dockerfile:17).
// The cgo rules hold: only byte buffers without Go pointers cross the boundary and libcda keeps no pointer
// after a call returns.
package cda

/*
#cgo LDFLAGS: -lcda
#include <stdlib.h>
#include "cda.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"sync"
	"unsafe"

	"github.com/celestiaorg/rsmt2d"
)

// ShareSize and NodeSize mirror appconsts.ShareSize (global_consts.go:29) and the 90-byte NMT node.
const (
	ShareSize     = C.CDA_SHARE_SIZE
	NamespaceSize = C.CDA_NAMESPACE_SIZE
	NodeSize      = C.CDA_NODE_SIZE
)

// Error is a libcda error code with the detail cda_err_info carries.
type Error struct {
	Code  int
	Axis  int
	Index int
	Leaf  int
	Block int
}

func (e *Error) Error() string {
	return fmt.Sprintf("%s (axis %d index %d leaf %d block %d)", C.GoString(C.cda_strerror(C.int(e.Code))),
		e.Axis, e.Index, e.Leaf, e.Block)
}

// Error codes (include/cda.h).
const (
	ErrCodeNotPow2      = int(C.CDA_E_NOT_POW2)
	ErrCodeNotSquare    = int(C.CDA_E_NOT_SQUARE)
	ErrCodeShardSize    = int(C.CDA_E_SHARD_SIZE)
	ErrCodeNsShort      = int(C.CDA_E_NS_SHORT)
	ErrCodeNsOrder      = int(C.CDA_E_NS_ORDER)
	ErrCodeTooFew       = int(C.CDA_E_TOO_FEW)
	ErrCodeUnrepairable = int(C.CDA_E_UNREPAIRABLE)
	ErrCodeByzantine    = int(C.CDA_E_BYZANTINE)
	ErrCodePushPast     = int(C.CDA_E_PUSH_PAST)
	ErrCodeNoMem        = int(C.CDA_E_NOMEM)    // std::bad_alloc caught inside libcda
	ErrCodeInternal     = int(C.CDA_E_INTERNAL) // any other C++ exception caught at the C ABI
)

func toErr(rc C.int, info *C.cda_err_info) error {
	if rc == 0 {
		return nil
	}
	e := &Error{Code: int(rc), Axis: -1, Index: -1, Leaf: -1, Block: -1}
	if info != nil {
		e.Axis, e.Index, e.Leaf, e.Block = int(info.axis), int(info.index), int(info.leaf), int(info.block)
	}
	return e
}

// Context is one cda_ctx (one GPU).  Its calls are serialised by libcda, so one Context may be shared by the
// goroutines rsmt2d fans out per axis.
type Context struct {
	c      *C.cda_ctx
	closed bool // set by Close under the pools' locks: slabs of a closed context are never pooled again
}

// NewContext binds HIP device `device`.
func NewContext(device int) (*Context, error) {
	var c *C.cda_ctx
	if rc := C.cda_init(C.int(device), &c); rc != 0 {
		return nil, toErr(rc, nil)
	}
	return &Context{c: c}, nil
}

// Close releases the context: its free pooled slabs are unregistered and dropped, the slabs squares still hold are
// unregistered (they stay valid Go memory and are dropped when they come back), then the context is freed.
func (x *Context) Close() {
	if x.c == nil {
		return
	}
	edsPool.mu.Lock()
	sharePool.mu.Lock()
	x.closed = true
	sharePool.mu.Unlock()
	edsPool.mu.Unlock()
	x.Trim()
	x.unregisterInUse()
	C.cda_free(x.c)
	x.c = nil
}

var (
	deviceMu   sync.Mutex
	deviceCtxs = map[int]*Context{}
)

// Default returns the process-wide context on device 0 (one process per GPU).
func Default() (*Context, error) { return DefaultOn(0) }

// DefaultOn returns the process-wide context of HIP device `device`, created on first use and never closed.  The
// squares ExtendShares / Multi.ExtendBlocks return keep their codec and tree constructor on these contexts, so a
// returned *rsmt2d.ExtendedDataSquare stays usable (Repair, re-rooting after SetCell) whatever is closed later.
func DefaultOn(device int) (*Context, error) {
	deviceMu.Lock()
	defer deviceMu.Unlock()
	if x, ok := deviceCtxs[device]; ok {
		return x, nil
	}
	x, err := NewContext(device)
	if err != nil {
		return nil, err
	}
	deviceCtxs[device] = x
	return x, nil
}

func mustDefault() *Context {
	x, err := Default()
	if err != nil {
		panic(fmt.Sprintf("cda: no GPU context: %v", err))
	}
	return x
}

func ptr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

var errUnequal = errors.New("shares must all be the same length")

// flatten copies equal-length shares into one contiguous buffer (what the C ABI takes).
func flatten(shares [][]byte) ([]byte, int, error) {
	if len(shares) == 0 {
		return nil, 0, nil
	}
	n := len(shares[0])
	out := make([]byte, len(shares)*n)
	if err := flattenInto(out, shares, n); err != nil {
		return nil, 0, err
	}
	return out, n, nil
}

// split views a contiguous buffer as n equal shares (no copy).
func split(buf []byte, n int) [][]byte {
	if n == 0 {
		return nil
	}
	sz := len(buf) / n
	out := make([][]byte, n)
	for i := range out {
		out[i] = buf[i*sz : (i+1)*sz : (i+1)*sz]
	}
	return out
}

var _ rsmt2d.Codec = (*Codec)(nil)
