//go:build rocm

package cda

/*
#include "cda.h"
*/
import "C"

import (
	"reflect"
	"runtime"
	"sync"
	"unsafe"
)

// Page-locked host slabs for the one-block consensus path (csrc/consensus.cpp).
//
// PrepareProposal, ProcessProposal and ExtendBlock extend one square per call (app/prepare_proposal.go:65,
// app/process_proposal.go:137, app/extend_block.go:25).  libcda moves a page-locked buffer by direct DMA, while a
// fresh Go slice is pinned by the HIP runtime page by page on every call, and a never-touched one is first faulted in
// by the kernel: the driver measured 1.05 ms per k=128 block with a fresh 32 MiB EDS slice per call against 0.66 ms
// with page-locked buffers (BENCH_r04 host_buffers.one_block_fresh).  So the binding keeps two pools:
//
//   - share slabs: the flatten every call does anyway (the C ABI takes one contiguous ODS) goes into a registered
//     slab that returns to its pool as soon as the call is over;
//   - EDS slabs: the square ExtendShares returns is an *rsmt2d.ExtendedDataSquare whose cells are slices of the slab,
//     so the slab may be reused only once nothing references any cell.  The slab is a Go heap object (an array from
//     reflect.New) watched by a finalizer: the garbage collector runs it when the square and every slice of its
//     cells are unreachable -- a caller that keeps eds.Flattened()'s cells keeps the slab alive -- and the finalizer
//     puts the (still registered) slab back into the pool.
//
// The slabs are registered once with cda_host_register (hipHostRegister) and never freed while registered: the Go
// heap does not move objects, and a pooled slab is referenced by the pool, so the pages the driver locked stay the
// object's.  A pool that is full falls back to plain Go memory (the slower fresh-buffer path, same results).
// Squares smaller than minPooled bytes are allocated plainly: their copies are short either way.
const (
	minPooled      = 1 << 20
	maxLivePerSize = 4 // registered slabs per size (in use + free), per context
)

type slabKey struct {
	ctx *Context
	n   int
}

type bufferPool struct {
	mu   sync.Mutex
	free map[slabKey][]interface{} // each entry a *[n]byte from reflect.New, registered with ctx
	live map[slabKey]int
}

var (
	edsPool   = &bufferPool{free: map[slabKey][]interface{}{}, live: map[slabKey]int{}}
	sharePool = &bufferPool{free: map[slabKey][]interface{}{}, live: map[slabKey]int{}}
)

func slabBytes(arr interface{}, n int) []byte {
	return unsafe.Slice((*byte)(reflect.ValueOf(arr).UnsafePointer()), n)
}

// take returns a registered slab of n bytes (or plain memory when the pool is full / registration fails) and the
// array object behind it (nil for plain memory).
func (p *bufferPool) take(ctx *Context, n int) ([]byte, interface{}) {
	if n < minPooled {
		return make([]byte, n), nil
	}
	key := slabKey{ctx, n}
	p.mu.Lock()
	if l := p.free[key]; len(l) > 0 {
		arr := l[len(l)-1]
		p.free[key] = l[:len(l)-1]
		p.mu.Unlock()
		return slabBytes(arr, n), arr
	}
	if p.live[key] >= maxLivePerSize {
		p.mu.Unlock()
		return make([]byte, n), nil
	}
	p.live[key]++
	p.mu.Unlock()
	arr := reflect.New(reflect.ArrayOf(n, reflect.TypeOf(byte(0)))).Interface()
	b := slabBytes(arr, n)
	if rc := C.cda_host_register(ctx.c, unsafe.Pointer(&b[0]), C.size_t(n)); rc != 0 {
		p.mu.Lock()
		p.live[key]--
		p.mu.Unlock()
		return b, nil // plain (unregistered) memory: still correct, the slower path
	}
	return b, arr
}

// give puts a registered slab back (no-op for plain memory).
func (p *bufferPool) give(ctx *Context, n int, arr interface{}) {
	if arr == nil {
		return
	}
	key := slabKey{ctx, n}
	p.mu.Lock()
	p.free[key] = append(p.free[key], arr)
	p.mu.Unlock()
}

// takeEDS returns an EDS slab that goes back to the pool when the garbage collector finds it unreferenced.
func takeEDS(ctx *Context, n int) []byte {
	b, arr := edsPool.take(ctx, n)
	if arr != nil {
		runtime.SetFinalizer(arr, func(a interface{}) { edsPool.give(ctx, n, a) })
	}
	return b
}

// takeShares / giveShares bracket one call: the flattened ODS is dead once the C call has returned.
func takeShares(ctx *Context, n int) ([]byte, interface{}) { return sharePool.take(ctx, n) }
func giveShares(ctx *Context, n int, arr interface{})      { sharePool.give(ctx, n, arr) }

// flattenInto copies equal-length shares into dst (len(shares) * share length bytes).
func flattenInto(dst []byte, shares [][]byte, n int) error {
	for _, s := range shares {
		if len(s) != n {
			return errUnequal
		}
	}
	inParts(len(shares), len(shares)*n, func(i0, i1 int) {
		for i := i0; i < i1; i++ {
			copy(dst[i*n:(i+1)*n], shares[i])
		}
	})
	return nil
}

// inParts runs fn over [0, count) in one piece, or -- when the copy it stands for is 1 MiB or more -- in up to 8
// contiguous pieces on their own goroutines: the flatten is the caller's only host work before the GPU call, and one
// thread copies 8 MiB in ~0.1 ms (profiles/r05_bench_v1.log: roots_only_pooled_in vs roots_only).
func inParts(count, bytes int, fn func(i0, i1 int)) {
	parts := 1
	if bytes >= 1<<20 {
		parts = 8
	}
	if parts > count {
		parts = count
	}
	if parts <= 1 {
		fn(0, count)
		return
	}
	var wg sync.WaitGroup
	for p := 0; p < parts; p++ {
		wg.Add(1)
		go func(i0, i1 int) {
			defer wg.Done()
			fn(i0, i1)
		}(count*p/parts, count*(p+1)/parts)
	}
	wg.Wait()
}

// flattenQ0 copies the k*k shares (ShareSize bytes each) into the top-left quadrant of a 2k x 2k EDS buffer: share i
// to row i/k, column i%k (in row bands on up to 8 goroutines, inParts).
func flattenQ0(eds []byte, shares [][]byte, k int) error {
	for _, sh := range shares {
		if len(sh) != ShareSize {
			return errUnequal
		}
	}
	inParts(k, k*k*ShareSize, func(r0, r1 int) {
		for r := r0; r < r1; r++ {
			dst := eds[r*2*k*ShareSize:]
			for c := 0; c < k; c++ {
				copy(dst[c*ShareSize:(c+1)*ShareSize], shares[r*k+c])
			}
		}
	})
	return nil
}

// Trim unregisters and drops every free slab of ctx (e.g. before closing a non-default context).  Slabs still
// referenced by squares stay registered until they come back and are trimmed in a later call.
func (x *Context) Trim() {
	for _, p := range []*bufferPool{edsPool, sharePool} {
		p.mu.Lock()
		for key, l := range p.free {
			if key.ctx != x {
				continue
			}
			for _, arr := range l {
				b := slabBytes(arr, key.n)
				C.cda_host_unregister(x.c, unsafe.Pointer(&b[0]))
				runtime.SetFinalizer(arr, nil)
				p.live[key]--
			}
			delete(p.free, key)
		}
		p.mu.Unlock()
	}
}
