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
	"sync/atomic"
	"unsafe"

	"github.com/celestiaorg/rsmt2d"
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
// The slabs are registered once with cda_host_register (hipHostRegister) and stay registered for their pooled life.
// Squares smaller than minPooled bytes are allocated plainly: their copies are short either way.  A pool that is full
// falls back to plain Go memory (the slower fresh-buffer path, same results).
//
// Invariant (ADVICE r05): HIP keeps the address of a registered slab after cda_host_register returns, which the cgo
// rules allow only for memory that cannot move.  The gc toolchain's heap does not move objects (every release to
// date, including go 1.22.2 of go.mod:3), so a slab stays at its address while the pool or a square references it;
// the slab is unregistered before the pool drops it (Trim, Context.Close) and never freed while registered.
// runtime.Pinner would make the rule explicit, but a pinned object stays reachable through its Pinner and so would
// never reach the finalizer that recycles it; a toolchain with a moving collector needs Release-only slabs instead.
//
// Squares the caller knows are dead go back at once with Release(eds); PoolStats counts hits, misses and recycling.
const (
	minPooled      = 1 << 20
	maxLivePerSize = 4 // registered slabs per size (in use + free), per context
)

type slabKey struct {
	ctx *Context
	n   int
}

// PoolStats are the EDS / share slab pools' counters since the process started.
type PoolStats struct {
	Hits      uint64 // a free registered slab was reused
	Misses    uint64 // a new slab was allocated and registered
	Fallbacks uint64 // pool full (or registration failed): plain Go memory, the fresh-buffer path
	Released  uint64 // EDS slabs returned by Release
	Recycled  uint64 // EDS slabs returned by the garbage collector (finalizer)
	Dropped   uint64 // slabs unregistered and dropped (Trim, Close, or returned after their context closed)
}

var stats struct{ hits, misses, fallbacks, released, recycled, dropped atomic.Uint64 }

// Stats returns the pools' counters.
func Stats() PoolStats {
	return PoolStats{stats.hits.Load(), stats.misses.Load(), stats.fallbacks.Load(), stats.released.Load(),
		stats.recycled.Load(), stats.dropped.Load()}
}

type bufferPool struct {
	mu    sync.Mutex
	free  map[slabKey][]interface{} // each entry a *[n]byte from reflect.New, registered with ctx
	live  map[slabKey]int
	inUse map[uintptr]slabKey // EDS slabs handed to squares, by base address (no reference: the GC still sees them)
}

var (
	edsPool   = newPool()
	sharePool = newPool()
)

func newPool() *bufferPool {
	return &bufferPool{free: map[slabKey][]interface{}{}, live: map[slabKey]int{}, inUse: map[uintptr]slabKey{}}
}

func slabBytes(arr interface{}, n int) []byte {
	return unsafe.Slice((*byte)(reflect.ValueOf(arr).UnsafePointer()), n)
}

func slabArray(base unsafe.Pointer, n int) interface{} {
	return reflect.NewAt(reflect.ArrayOf(n, reflect.TypeOf(byte(0))), base).Interface()
}

// take returns a registered slab of n bytes (or plain memory when the pool is full / registration fails) and the
// array object behind it (nil for plain memory).
func (p *bufferPool) take(ctx *Context, n int) ([]byte, interface{}) {
	if n < minPooled {
		return make([]byte, n), nil
	}
	key := slabKey{ctx, n}
	p.mu.Lock()
	if ctx.closed {
		p.mu.Unlock()
		return make([]byte, n), nil
	}
	if l := p.free[key]; len(l) > 0 {
		arr := l[len(l)-1]
		p.free[key] = l[:len(l)-1]
		p.mu.Unlock()
		stats.hits.Add(1)
		return slabBytes(arr, n), arr
	}
	if p.live[key] >= maxLivePerSize {
		p.mu.Unlock()
		stats.fallbacks.Add(1)
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
		stats.fallbacks.Add(1)
		return b, nil // plain (unregistered) memory: still correct, the slower path
	}
	stats.misses.Add(1)
	return b, arr
}

// give puts a registered slab back (no-op for plain memory); a slab of a closed context was unregistered by Close
// and is dropped.
func (p *bufferPool) give(ctx *Context, n int, arr interface{}) {
	if arr == nil {
		return
	}
	key := slabKey{ctx, n}
	p.mu.Lock()
	defer p.mu.Unlock()
	if ctx.closed {
		p.live[key]--
		stats.dropped.Add(1)
		return
	}
	p.free[key] = append(p.free[key], arr)
}

// takeEDS returns an EDS slab that goes back to the pool when the garbage collector finds it unreferenced, or when
// the square built on it is passed to Release.
func takeEDS(ctx *Context, n int) []byte {
	b, arr := edsPool.take(ctx, n)
	if arr != nil {
		base := uintptr(unsafe.Pointer(&b[0]))
		edsPool.mu.Lock()
		edsPool.inUse[base] = slabKey{ctx, n}
		edsPool.mu.Unlock()
		runtime.SetFinalizer(arr, func(a interface{}) {
			edsPool.mu.Lock()
			delete(edsPool.inUse, base)
			edsPool.mu.Unlock()
			stats.recycled.Add(1)
			edsPool.give(ctx, n, a)
		})
	}
	return b
}

// Release returns the page-locked slab behind a square from ExtendShares / Repair to the pool at once, instead of
// when the garbage collector next finds it unreferenced.  The caller promises that neither eds nor any slice of its
// cells (Flattened returns the cells themselves; GetCell and Row return copies) is used afterwards: the next square is written
// into the same memory.  Squares not built on a pooled slab are ignored.  Reports whether a slab was returned.
func Release(eds *rsmt2d.ExtendedDataSquare) bool {
	if eds == nil {
		return false
	}
	flat := eds.Flattened()
	if len(flat) == 0 || len(flat[0]) == 0 {
		return false
	}
	base := unsafe.Pointer(&flat[0][0])
	edsPool.mu.Lock()
	key, ok := edsPool.inUse[uintptr(base)]
	if ok {
		delete(edsPool.inUse, uintptr(base))
	}
	edsPool.mu.Unlock()
	if !ok {
		return false
	}
	arr := slabArray(base, key.n)
	runtime.SetFinalizer(arr, nil)
	stats.released.Add(1)
	edsPool.give(key.ctx, key.n, arr)
	return true
}

// slabOf returns the pooled slab whose cells a flattened square still is, if every present cell sits at its place in
// one in-use slab of w*w*n bytes (a square from ExtendShares or Repair, cells erased by the caller).
func slabOf(eds [][]byte, n int) []byte {
	var base uintptr
	for i, c := range eds {
		if c == nil {
			continue
		}
		p := uintptr(unsafe.Pointer(&c[0]))
		if base == 0 {
			base = p - uintptr(i*n)
		}
		if p != base+uintptr(i*n) || cap(c) < n {
			return nil
		}
	}
	if base == 0 {
		return nil
	}
	edsPool.mu.Lock()
	key, ok := edsPool.inUse[base]
	edsPool.mu.Unlock()
	if !ok || key.n != len(eds)*n {
		return nil
	}
	return unsafe.Slice((*byte)(unsafe.Pointer(base)), key.n)
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

// Trim unregisters and drops every free slab of ctx.  Slabs still referenced by squares stay registered until they
// come back (and are trimmed by a later call), or until Close.
func (x *Context) Trim() {
	for _, p := range []*bufferPool{edsPool, sharePool} {
		p.mu.Lock()
		for key, l := range p.free {
			if key.ctx != x {
				continue
			}
			var kept []interface{}
			for _, arr := range l {
				b := slabBytes(arr, key.n)
				if x.c != nil {
					if rc := C.cda_host_unregister(x.c, unsafe.Pointer(&b[0])); rc != 0 {
						// still registered: keep the slab in the pool (and its count) rather than drop locked pages
						kept = append(kept, arr)
						continue
					}
				}
				runtime.SetFinalizer(arr, nil)
				p.live[key]--
				stats.dropped.Add(1)
			}
			if len(kept) > 0 {
				p.free[key] = kept
			} else {
				delete(p.free, key)
			}
		}
		p.mu.Unlock()
	}
}

// unregisterInUse unregisters the EDS slabs of x that squares still hold (Close): they become plain Go memory, and
// their finalizers drop them instead of pooling them (give sees x.closed).
func (x *Context) unregisterInUse() {
	edsPool.mu.Lock()
	defer edsPool.mu.Unlock()
	for base, key := range edsPool.inUse {
		if key.ctx == x && x.c != nil {
			_ = C.cda_host_unregister(x.c, unsafe.Pointer(base))
		}
	}
}
