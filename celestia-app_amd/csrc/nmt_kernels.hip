// nmt_kernels.hip — erasured-NMT leaf/inner hashing and the DAH RFC-6962 tree.
//
// Reference semantics (celestia-app @ 2025-02-13):
//   leaf:  ns ‖ ns ‖ SHA256(0x00 ‖ ns ‖ share), ns = share[0:29] in Q0 else 0xFF×29
//          pkg/wrapper/nmt_wrapper.go:93-114,138-140; test/util/malicious/hasher.go:186-209
//   node:  L.min ‖ (R.min == 0xFF×29 ? L.max : R.max) ‖ SHA256(0x01 ‖ L ‖ R)
//          hasher.go:271-310 (IgnoreMaxNamespace=true, nmt_wrapper.go:60)
//   DAH:   RFC-6962 over row roots ‖ col roots, pkg/da/data_availability_header.go:92-108
//
// Design (MI355X): the leaf data of cell (r,c) is identical in row tree r and
// column tree c (both use the share's namespace iff the cell is in Q0), so each
// of the 4k² cells is hashed ONCE (the reference hashes it twice) and both trees
// read the same 96-byte leaf record.  Records are 96 B (90-B node + 6 zero bytes)
// so a node is six 16-B loads/stores.  Inner levels are one launch per level over
// every tree of every block in the batch (4k trees/block, lanes stay full until
// the last few levels).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>

#include "cda_internal.h"
#include "nmt_dev.h"
#include "sha256_dev.h"

namespace cda {

__global__ void __launch_bounds__(256) leaf_hash_kernel(const uint8_t* __restrict__ eds, uint4* __restrict__ nodes,
                                                        unsigned long long* __restrict__ status, int k, int log2w,
                                                        uint32_t total_cells) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total_cells) return;
  leaf_cell(eds, nodes, status, k, log2w, gid);
}

// ---------------------------------------------------------------------------
// Inner NMT node.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_node(const uint4* p, uint32_t* n) {
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint4 v = p[i];
    n[4 * i + 0] = v.x;
    n[4 * i + 1] = v.y;
    n[4 * i + 2] = v.z;
    n[4 * i + 3] = v.w;
  }
}

// One thread per output node. Level 1 reads leaf records in cell-major layout
// ([blk][r][c]); later levels read [blk][tree][n_in].  Trees 0..w-1 are rows,
// w..2w-1 columns.
template <bool FROM_LEAVES>
__global__ void __launch_bounds__(256) nmt_level_kernel(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                        int log2w, int log2n_out, uint32_t total_out) {
  uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total_out) return;
  const int w = 1 << log2w;
  const uint32_t j = gid & ((1u << log2n_out) - 1);
  const uint32_t tree_g = gid >> log2n_out;  // blk * 2w + tree
  const uint32_t blk = tree_g >> (log2w + 1);
  const uint32_t tree = tree_g & (2 * w - 1);
  size_t ia, ib;
  if (FROM_LEAVES) {
    const size_t base = (size_t)blk << (2 * log2w);
    if (tree < (uint32_t)w) {  // row tree: cells (tree, 2j), (tree, 2j+1)
      ia = base + ((size_t)tree << log2w) + 2 * j;
      ib = ia + 1;
    } else {  // column tree: cells (2j, col), (2j+1, col)
      const uint32_t col = tree - w;
      ia = base + ((size_t)(2 * j) << log2w) + col;
      ib = ia + w;
    }
  } else {
    ia = ((size_t)tree_g << (log2n_out + 1)) + 2 * j;
    ib = ia + 1;
  }
  hash_node_mem(in + ia * 6, in + ib * 6, out + (size_t)gid * 6);
}

// ---------------------------------------------------------------------------
// Row and column trees of a batch of blocks, M levels per launch.
//
// Layout of level l (n_l = w >> l nodes per tree) for block b, in 96-B records:
//   row tree r, node i :  base + b*blk + row0 + r*row_t + i*row_i
//   col tree c, node i :  base + b*blk + col0 + c*col_t + i*col_i
// Leaves (l = 0) are the cell-major leaf records (row_t = w, row_i = 1, col_t = 1, col_i = w); inner
// levels keep row trees tree-major ([r][i]) and column trees node-major ([i][c]), so that for both
// kinds the 64 lanes of a wave read 64 adjacent records (row trees: lanes = consecutive i, two
// children each, 192 contiguous bytes per lane; column trees: lanes = consecutive c) and write 64
// adjacent records.  The roots land in d_roots[b][0..w) (rows) and [w..2w) (columns).
//
// A thread owns one output node at level l_in + M and computes its whole subtree level by level
// (2^M - 1 nodes, the intermediate levels written to their level buffers and read back by the same
// thread), so a launch covers M levels: the levels of one block's 4k trees take ceil(log2(2k) / M)
// launches instead of log2(2k).
// ---------------------------------------------------------------------------
struct LevelDesc {
  uint4* p;
  unsigned long long blk;  // records per block
  unsigned row0, row_t, row_i, col0, col_t, col_i;
};
struct LevelSet {
  LevelDesc lv[4];  // levels l_in .. l_in + M (M <= 3)
};

__device__ __forceinline__ uint4* level_rec(const LevelDesc& d, unsigned b, bool col, unsigned tree, unsigned i) {
  const unsigned long long off =
      (unsigned long long)b * d.blk + (col ? d.col0 + tree * d.col_t + i * d.col_i : d.row0 + tree * d.row_t + i * d.row_i);
  return d.p + off * 6;
}

__global__ void __launch_bounds__(256) nmt_levels_kernel(LevelSet ls, int log2w, int log2n_out, int M, uint32_t total) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const unsigned w = 1u << log2w;
  const unsigned per_kind = w << log2n_out;  // output nodes of the row (or column) trees of one block
  const unsigned b = gid / (2 * per_kind);
  const unsigned rem = gid - b * 2 * per_kind;
  const bool col = rem >= per_kind;
  const unsigned r2 = col ? rem - per_kind : rem;
  // row trees: node index fastest; column trees: column fastest
  const unsigned tree = col ? (r2 & (w - 1)) : (r2 >> log2n_out);
  const unsigned j = col ? (r2 >> log2w) : (r2 & ((1u << log2n_out) - 1));
  __shared__ uint4 s_ns[256 * 8];  // per thread: the first 64 B of both children of the node being hashed
  const unsigned k = w >> 1;
  const int l_in = log2w - log2n_out - M;
  for (int q = 1; q <= M; q++) {
    const unsigned cnt = 1u << (M - q);  // nodes of this subtree at level l_in + q
    for (unsigned t = 0; t < cnt; t++) {
      const unsigned i = j * cnt + t;
      // every leaf under node i is a parity leaf (axis >= k, or leaves i << level onward all >= k): nmt_dev.h
#if CDA_NO_PARITY_MID  // diagnostic A/B: every node through the full 64 rounds of block 0
      const bool parity = false;
#else
      const bool parity = tree >= k || (i << (l_in + q)) >= k;
#endif
      hash_node_mem(level_rec(ls.lv[q - 1], b, col, tree, 2 * i), level_rec(ls.lv[q - 1], b, col, tree, 2 * i + 1),
                    level_rec(ls.lv[q], b, col, tree, i), true, s_ns + threadIdx.x * 8, parity);
    }
    // the next level reads what this thread just stored
    if (q < M) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// Leaf records -> roots of all 4k trees of nblocks blocks.  d_levels holds the inner levels
// (2w x (w - 2) records per block at most); M = 2 levels per launch (the last launch may take 1 or 3).
int launch_nmt_trees(const void* d_leaves, void* d_levels, void* d_roots, int k, int nblocks, hipStream_t s,
                     void* prof_ctx) {
  const int w = 2 * k;
  int L = 0;
  while ((1 << L) < w) L++;
  if ((1 << L) != w || L < 1) return -2;
  auto desc = [&](int l) {
    LevelDesc d{};
    const unsigned n = (unsigned)(w >> l);
    if (l == 0) {
      d.p = (uint4*)d_leaves;
      d.blk = (unsigned long long)w * w;
      d.row0 = 0, d.row_t = w, d.row_i = 1, d.col0 = 0, d.col_t = 1, d.col_i = w;
    } else if (l == L) {
      d.p = (uint4*)d_roots;
      d.blk = 2ull * w;
      d.row0 = 0, d.row_t = 1, d.row_i = 0, d.col0 = w, d.col_t = 1, d.col_i = 0;
    } else {
      unsigned long long off = 0;  // levels 1 .. l-1 before this one
      for (int q = 1; q < l; q++) off += 2ull * w * (w >> q);
      d.p = (uint4*)d_levels + off * (unsigned long long)nblocks * 6;
      d.blk = 2ull * w * n;
      d.row0 = 0, d.row_t = n, d.row_i = 1, d.col0 = w * n, d.col_t = 1, d.col_i = w;
    }
    return d;
  };
  for (int l_in = 0; l_in < L;) {
    int M = std::min(2, L - l_in);
    if (L - l_in == 3) M = 3;  // finish with one 3-level launch rather than 2 + 1
    LevelSet ls{};
    for (int q = 0; q <= M; q++) ls.lv[q] = desc(l_in + q);
    const int log2n_out = L - (l_in + M);
    const uint32_t total = (uint32_t)nblocks * 2u * ((uint32_t)w << log2n_out);
    {
      ProfScope ps(prof_ctx, l_in == 0 ? "nmt_levels_1" : "nmt_levels", s);
      hipLaunchKernelGGL(nmt_levels_kernel, dim3((total + 255) / 256), dim3(256), 0, s, ls, L, log2n_out, M, total);
    }
    if (hipGetLastError() != hipSuccess) return -1;
    l_in += M;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// DAH: RFC-6962 over the n = 2w roots (rows then cols), one workgroup per block.
// Levels pair (2i, 2i+1) and promote an odd last node, which is the same tree as
// HashFromByteSlices' "split at the largest power of two below n" recursion.
// ---------------------------------------------------------------------------
// DAH leaf digest: SHA256(0x00 || root record[0..90)) as 8 big-endian words; message block B of it
template <int B>
__device__ __forceinline__ void dah_leaf_block(const uint32_t (&L)[24], uint32_t (&m)[16]) {
  // 0x00 ‖ root[0..90) ‖ 0x80 ‖ ... ‖ len(91*8)
#pragma unroll
  for (int t = 0; t < 16; t++) {
    const int wi = 16 * B + t;
    if (wi == 0) m[t] = be_window(0u, L[0], 3);
    else if (wi <= 21) m[t] = be_window(L[wi - 1], L[wi], 3);
    else if (wi == 22) m[t] = be_window(L[21], L[22], 3) | 0x80u;
    else if (wi < 31) m[t] = 0;
    else m[t] = 91u * 8u;
  }
}
__device__ __forceinline__ void dah_leaf_digest(const uint32_t (&L)[24], uint32_t (&st)[8]) {
  uint32_t m[16];
  sha256_init(st);
  dah_leaf_block<0>(L, m);
  sha256_compress(st, m);
  dah_leaf_block<1>(L, m);
  sha256_compress(st, m);
}
// RFC-6962 inner node message block B of digests Ld, Rd (8 big-endian words each): 0x01 ‖ Ld ‖ Rd ‖ pad, 65 bytes
template <int B>
__device__ __forceinline__ void rfc_node_block(const uint32_t* Ld, const uint32_t* Rd, uint32_t (&m)[16]) {
  if (B == 0) {
    m[0] = 0x01000000u | (Ld[0] >> 8);
#pragma unroll
    for (int t = 1; t < 8; t++) m[t] = (Ld[t - 1] << 24) | (Ld[t] >> 8);
    m[8] = (Ld[7] << 24) | (Rd[0] >> 8);
#pragma unroll
    for (int t = 9; t < 16; t++) m[t] = (Rd[t - 9] << 24) | (Rd[t - 8] >> 8);
  } else {
    m[0] = (Rd[7] << 24) | 0x00800000u;
#pragma unroll
    for (int t = 1; t < 15; t++) m[t] = 0;
    m[15] = 65u * 8u;
  }
}

// RFC-6962 levels over the n leaf digests at sdig ([n + (n+1)/2][8] words of LDS, the first n filled), by the
// calling workgroup (>= 128 threads); the 32-B hash goes to out.  Levels pair (2i, 2i+1) and promote an odd last
// node, which is the same tree as HashFromByteSlices' "split at the largest power of two below n" recursion.  Once
// a level has at most 64 nodes (its chain of dependent compressions is the latency), wave 0 hashes block 0 of each
// node while wave 1 expands the node's second message block into kw (64 x kKwStride words of LDS), and the second
// compression then runs its rounds alone.
__device__ __forceinline__ void dah_fold_kw(uint32_t* sdig, int n, uint32_t* out, uint32_t* kw) {
  uint32_t* src = sdig;
  uint32_t* dst = sdig + n * 8;
  for (int cnt = n; cnt > 1;) {
    const int out_cnt = (cnt + 1) >> 1;
    if (out_cnt > 64) {
      for (int i = threadIdx.x; i < out_cnt; i += blockDim.x) {
        uint32_t* o = dst + i * 8;
        const uint32_t* Ld = src + (2 * i) * 8;
        if (2 * i + 1 >= cnt) {
#pragma unroll
          for (int t = 0; t < 8; t++) o[t] = Ld[t];
          continue;
        }
        const uint32_t* Rd = src + (2 * i + 1) * 8;
        uint32_t st[8], m[16];
        sha256_init(st);
        rfc_node_block<0>(Ld, Rd, m);
        sha256_compress(st, m);
        rfc_node_block<1>(Ld, Rd, m);
        sha256_compress(st, m);
#pragma unroll
        for (int t = 0; t < 8; t++) o[t] = st[t];
      }
    } else {
      // every lane of waves 0 and 1 computes, with full exec masks (lanes past the level's pairs hash stale,
      // in-bounds LDS words and store nothing), as in trees_lds_kernel
      const int i = threadIdx.x & 63;
      const bool pair = i < out_cnt && 2 * i + 1 < cnt;
      uint32_t st[8];
      if (threadIdx.x < 64) {
        const uint32_t* Ld = src + (2 * i) * 8;
        if (i < out_cnt && !pair)
#pragma unroll
          for (int t = 0; t < 8; t++) dst[i * 8 + t] = Ld[t];
        uint32_t m[16];
        sha256_init(st);
        rfc_node_block<0>(Ld, src + (2 * i + 1) * 8, m);
        sha256_compress(st, m);
      } else if (threadIdx.x < 128) {
        uint32_t m[16];
        rfc_node_block<1>(src + (2 * i) * 8, src + (2 * i + 1) * 8, m);
        sha256_kw_store(m, kw + i * kKwStride);
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        sha256_rounds_kw(st, kw + i * kKwStride);
        if (pair)
#pragma unroll
          for (int t = 0; t < 8; t++) dst[i * 8 + t] = st[t];
      }
    }
    __syncthreads();
    uint32_t* tmp = src;
    src = dst;
    dst = tmp;
    cnt = out_cnt;
  }
  if (threadIdx.x < 8) out[threadIdx.x] = bswap(src[threadIdx.x]);
}

// DAH: RFC-6962 over the n = 2w roots (rows then cols), one workgroup per block.
__global__ void __launch_bounds__(256) dah_kernel(const uint4* __restrict__ roots, uint32_t* __restrict__ dah,
                                                  int n) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sdig[];  // [n + (n+1)/2][8] big-endian digests
  const uint4* rb = roots + (size_t)blockIdx.x * n * 6;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t L[24], st[8];
    load_node(rb + (size_t)i * 6, L);
    dah_leaf_digest(L, st);
#pragma unroll
    for (int t = 0; t < 8; t++) sdig[i * 8 + t] = st[t];
  }
  __syncthreads();
  dah_fold_kw(sdig, n, dah + blockIdx.x * 8, sdig + (n + (n + 1) / 2) * 8);
}

// DAH of a batch, wide form: the root digests by P = ceil(n / 256) workgroups per block, one root per thread, and
// the fold by the workgroup that finishes a block's digests last (agent-scope acq_rel counter, put back to 0).  The
// one-workgroup-per-block dah_kernel hashed n / 256 roots per thread first (8 at k = 512) before its fold.
__global__ void __launch_bounds__(256) dah_wide_kernel(const uint4* __restrict__ roots, uint32_t* __restrict__ dah,
                                                       unsigned* __restrict__ done, uint32_t* __restrict__ digests,
                                                       int n, int P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sdig[];  // [n + (n+1)/2][8] digests, then kw rows
  __shared__ unsigned last;
  const unsigned b = blockIdx.x / P, part = blockIdx.x % P;
  if (threadIdx.x == 0) last = 0;
  const int i = part * 256 + threadIdx.x;
  if (i < n) {
    uint32_t L[24], st[8];
    load_node(roots + ((size_t)b * n + i) * 6, L);
    dah_leaf_digest(L, st);
    uint4* dg = reinterpret_cast<uint4*>(digests + ((size_t)b * n + i) * 8);
    dg[0] = make_uint4(st[0], st[1], st[2], st[3]);
    dg[1] = make_uint4(st[4], st[5], st[6], st[7]);
  }
  __threadfence();  // this thread's digest, released at agent scope before the block's counter moves
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(done + b, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)P - 1) last = 1;
  }
  __syncthreads();
  if (!last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the other workgroups' digests
  const uint4* src = reinterpret_cast<const uint4*>(digests + (size_t)b * n * 8);
  for (int x = threadIdx.x; x < n * 2; x += blockDim.x) reinterpret_cast<uint4*>(sdig)[x] = src[x];
  __syncthreads();
  dah_fold_kw(sdig, n, dah + b * 8, sdig + (n + (n + 1) / 2) * 8);
  if (threadIdx.x == 0) __hip_atomic_store(done + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Small batches (the single block of ProcessProposal, config C2): every tree of the batch in ONE launch.  A
// 256-thread workgroup takes two trees (waves 0-1 the first, waves 2-3 the second; one workgroup per CU at k = 128).
// A tree's w leaf records go to LDS
// (112-B stride: the 16-B reads of records two apart are bank-conflict free) and each level is computed into the
// other half of a ping-pong pair, a thread holding both children in registers (hash_node_regs): a level costs its
// 3 dependent compressions and a barrier, not a launch or a memory round trip per compression.  Each tree's root
// then gets its DAH leaf digest; the workgroup that finishes a block's last tree pair (agent-scope acq_rel counter,
// put back to 0 for the next call) folds the block's digests into the DAH, so the step needs no DAH launch.  The
// batched form (nmt_levels_kernel + dah_kernel) keeps every lane on a useful node and stays the throughput path.
constexpr int kLdsRec = 7;  // uint4 per LDS record
#ifndef CDA_TREES_TRACE
#define CDA_TREES_TRACE 0  // diagnostic builds: per-workgroup phase timestamps of trees_lds_kernel
#endif
#if CDA_TREES_TRACE
__device__ unsigned long long* g_trees_trace;  // [workgroup][32 slots][realtime, shader clock]
#endif
// the stamps go to LDS (thread 0) and to memory at the end, so no global store sits between the phases
struct TreesStamps {
  unsigned long long* v;  // LDS: [32][rt, clock]
};
__device__ __forceinline__ void trees_mark(TreesStamps& ts, int slot) {
#if CDA_TREES_TRACE
  if (threadIdx.x == 0) {
    ts.v[2 * slot] = __builtin_amdgcn_s_memrealtime();
    ts.v[2 * slot + 1] = __builtin_amdgcn_s_memtime();
  }
#else
  (void)ts, (void)slot;
#endif
}
__device__ __forceinline__ void trees_flush(const TreesStamps& ts, int lo, int hi) {
#if CDA_TREES_TRACE
  if (threadIdx.x == 0 && g_trees_trace)
    for (int s = lo; s < hi; s++) {
      g_trees_trace[((size_t)blockIdx.x * 32 + s) * 2] = ts.v[2 * s];
      g_trees_trace[((size_t)blockIdx.x * 32 + s) * 2 + 1] = ts.v[2 * s + 1];
    }
#else
  (void)ts, (void)lo, (void)hi;
#endif
}
__device__ __forceinline__ void load_pair(const uint4* in, int i, uint32_t (&L)[24], uint32_t (&R)[24]) {
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const uint4 u = in[(2 * i) * kLdsRec + q], v = in[(2 * i + 1) * kLdsRec + q];
    L[4 * q] = u.x, L[4 * q + 1] = u.y, L[4 * q + 2] = u.z, L[4 * q + 3] = u.w;
    R[4 * q] = v.x, R[4 * q + 1] = v.y, R[4 * q + 2] = v.z, R[4 * q + 3] = v.w;
  }
}
__global__ void __launch_bounds__(256) trees_lds_kernel(const uint4* __restrict__ leaves, uint4* __restrict__ roots,
                                                        uint32_t* __restrict__ dah, unsigned* __restrict__ done,
                                                        uint32_t* __restrict__ digests, int log2w) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // per half: A (w records) | B (w / 2); DAH reuses
  __shared__ unsigned last;
  const int w = 1 << log2w, n = 2 * w;
  const int half = threadIdx.x >> 7, ht = threadIdx.x & 127;  // tree of this half, thread within it
  const unsigned gtree = blockIdx.x * 2 + half;
  const unsigned b = gtree >> (log2w + 1), tree = gtree & (n - 1);
  const bool col = tree >= (unsigned)w;
  const unsigned t = tree & (w - 1);
  const uint4* lb = leaves + (size_t)b * w * w * 6;
#if CDA_TREES_TRACE
  __shared__ unsigned long long tstamp[64];
  TreesStamps tst{tstamp};
#else
  TreesStamps tst{nullptr};
#endif
  trees_mark(tst, 0);
  if (threadIdx.x == 0) last = 0;  // published by the barrier after the leaf copy
  uint4* A = lds + (size_t)half * (w + w / 2) * kLdsRec;
  uint4* B = A + (size_t)w * kLdsRec;
  // K+W schedules of blocks 1 and 2 of up to 64 nodes per tree, after both halves' records
  uint32_t* kw = reinterpret_cast<uint32_t*>(lds + (size_t)2 * (w + w / 2 + 1) * kLdsRec) + half * 2 * 64 * kKwStride;
  for (int x = ht; x < w * 6; x += 128) {  // 16-B words of the w records, adjacent lanes adjacent
    const int i = x / 6, q = x - i * 6;
    const size_t rec = col ? ((size_t)i << log2w) + t : ((size_t)t << log2w) + i;
    A[i * kLdsRec + q] = lb[rec * 6 + q];
  }
  __syncthreads();
  trees_mark(tst, 1);
  for (int l = 1; l <= log2w; l++) {
    const uint4* in = (l & 1) ? A : B;
    uint4* out = (l & 1) ? B : A;
    const int nodes = w >> l;
    if (nodes > 64) {
      for (int i = ht; i < nodes; i += 128) {
        uint32_t L[24], R[24], o[24];
        load_pair(in, i, L, R);
        hash_node_regs(L, R, o);
#pragma unroll
        for (int q = 0; q < 6; q++) out[i * kLdsRec + q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
      }
    } else {
      // wave 0 of the half hashes block 0 of node ht while wave 1 expands blocks 1 and 2 of node ht - 64; after
      // the barrier wave 0 runs the last two compressions from the precomputed schedules.  Every lane computes, also
      // past the level's last node (on stale, in-bounds records; only lanes < nodes write): with the waves' exec
      // masks partly off, levels of <= 16 nodes took 9.4-10.8 us instead of 6.8 (r04_trees_trace.log)
      const int i = ht & 63;
      uint32_t L[24], R[24], st[8];
      load_pair(in, i, L, R);
      if (ht < 64) {
        uint32_t m[16];
        sha256_init(st);
        node_block<0>(L, R, m);
        sha256_compress(st, m);
        trees_mark(tst, 2 + 3 * (l - 1));
      } else {
        uint32_t m[16];
        node_block<1>(L, R, m);
        sha256_kw_store(m, kw + i * kKwStride);
        node_block<2>(L, R, m);
        sha256_kw_store(m, kw + (64 + i) * kKwStride);
      }
      __syncthreads();
      trees_mark(tst, 3 + 3 * (l - 1));
      if (ht < 64) {
        sha256_rounds_kw(st, kw + i * kKwStride);
        sha256_rounds_kw(st, kw + (64 + i) * kKwStride);
        uint32_t o[24];
        node_record(L, R, st, o);
        if (i < nodes)
#pragma unroll
          for (int q = 0; q < 6; q++)
            out[i * kLdsRec + q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
      }
    }
    __syncthreads();
    trees_mark(tst, 4 + 3 * (l - 1));
  }
  const uint4* root = (log2w & 1) ? B : A;
  uint4* rout = roots + ((size_t)b * n + tree) * 6;
  if (ht < 6) rout[ht] = root[ht];
  {  // this root's DAH leaf digest: block 0 by wave 0, block 1's schedule by wave 1 meanwhile (every lane of both
     // waves computes the same digest into its own schedule row, with full exec masks; lane 0 stores it)
    uint32_t L[24], st[8], m[16];
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const uint4 u = root[q];
      L[4 * q] = u.x, L[4 * q + 1] = u.y, L[4 * q + 2] = u.z, L[4 * q + 3] = u.w;
    }
    uint32_t* kwl = kw + (ht & 63) * kKwStride;
    if (ht < 64) {
      sha256_init(st);
      dah_leaf_block<0>(L, m);
      sha256_compress(st, m);
    } else {
      dah_leaf_block<1>(L, m);
      sha256_kw_store(m, kwl);
    }
    __syncthreads();
    if (ht < 64) sha256_rounds_kw(st, kwl);
    if (ht == 0) {
      uint4* dg = reinterpret_cast<uint4*>(digests + ((size_t)b * n + tree) * 8);
      dg[0] = make_uint4(st[0], st[1], st[2], st[3]);
      dg[1] = make_uint4(st[4], st[5], st[6], st[7]);
    }
  }
  __syncthreads();  // both halves' roots and digests are stored (each by lanes of the wave that increments below)
  trees_mark(tst, 26);
  if (threadIdx.x == 0 || threadIdx.x == 128) {  // one increment per tree, from the wave that stored it
    const unsigned prev = __hip_atomic_fetch_add(done + b, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)n - 1) last = 1;  // at most one tree of a block is its last
  }
  __syncthreads();
  trees_mark(tst, 27);
  trees_flush(tst, 0, 28);
  if (!last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the other workgroups' digests (released before their increments)
  uint32_t* sdig = reinterpret_cast<uint32_t*>(lds);
  const uint4* src = reinterpret_cast<const uint4*>(digests + (size_t)b * n * 8);
  for (int x = threadIdx.x; x < n * 2; x += blockDim.x) reinterpret_cast<uint4*>(sdig)[x] = src[x];
  __syncthreads();
  trees_mark(tst, 28);
  dah_fold_kw(sdig, n, dah + b * 8, sdig + (n + (n + 1) / 2) * 8);
  trees_mark(tst, 29);
  trees_flush(tst, 28, 30);
  if (threadIdx.x == 0) __hip_atomic_store(done + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// Single-axis tree (wrapper.NewConstructor(k)(axis, index) with n Pushes).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) axis_leaf_kernel(const uint8_t* __restrict__ leaves, int n,
                                                        unsigned long long square_size,
                                                        unsigned long long axis_index, uint4* __restrict__ nodes,
                                                        unsigned long long* __restrict__ status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool q0 = ((unsigned long long)i < square_size) && (axis_index < square_size);
  const uint4* sh = reinterpret_cast<const uint4*>(leaves + (size_t)i * CDA_SHARE);
  uint32_t A[16];
  load16(sh, A);
  // Push order: leaf i+1 (if also in Q0) must not have a smaller namespace
  if (q0 && (unsigned long long)(i + 1) < square_size && i + 1 < n) {
    uint32_t nb[8];
    const uint4* p = sh + CDA_SHARE / 16;
    uint4 v0 = p[0], v1 = p[1];
    nb[0] = v0.x; nb[1] = v0.y; nb[2] = v0.z; nb[3] = v0.w;
    nb[4] = v1.x; nb[5] = v1.y; nb[6] = v1.z; nb[7] = v1.w;
    if (ns_cmp(nb, A) < 0) atomicMin(status, (unsigned long long)(i + 1));
  }
  leaf_record(sh, A, q0, nodes + (size_t)i * 6);
}

__global__ void __launch_bounds__(256) level_generic_kernel(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                            int n_in) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int n_out = (n_in + 1) >> 1;
  if (j >= n_out) return;
  uint4* po = out + (size_t)j * 6;
  if (2 * j + 1 >= n_in) {  // odd node is promoted unchanged
#pragma unroll
    for (int i = 0; i < 6; i++) po[i] = in[(size_t)(2 * j) * 6 + i];
    return;
  }
  hash_node_mem(in + (size_t)(2 * j) * 6, in + (size_t)(2 * j + 1) * 6, po);
}

// ---------------------------------------------------------------------------
// Roots of a list of EDS axes (Repair verification, split-square path): tree t
// covers axis code a_t = axes ? axes[t] : axis0 + t  ((axis << 24) | index),
// leaves [leaf_off, leaf_off + 2^log2n) of that row / column.  With the full
// range this is the axis root; with an aligned power-of-two sub-range it is the
// root of that subtree (the NMT splits at powers of two, nmt_wrapper.go:118).
// status[t] gets the first leaf index whose Push order check fails.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) axes_leaf_kernel(const uint8_t* __restrict__ eds, int k, int log2w,
                                                        const int* __restrict__ axes, int axis0, int ntrees,
                                                        int leaf_off, int log2n, uint4* __restrict__ nodes,
                                                        unsigned long long* __restrict__ status) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int w = 1 << log2w;
  if (gid >= ((uint32_t)ntrees << log2n)) return;
  const int t = gid >> log2n, i = leaf_off + (int)(gid & ((1u << log2n) - 1));
  const int code = axes ? axes[t] : axis0 + t;
  const int ax = code >> 24, idx = code & 0xFFFFFF;
  const size_t cell = ax == CDA_AXIS_ROW ? ((size_t)idx << log2w) + i : ((size_t)i << log2w) + idx;
  const bool q0 = (i < k) && (idx < k);
  const uint4* sh = reinterpret_cast<const uint4*>(eds + cell * CDA_SHARE);
  uint32_t A[16];
  load16(sh, A);
  if (q0 && i + 1 < k) {
    const size_t nxt = ax == CDA_AXIS_ROW ? cell + 1 : cell + w;
    const uint4* p = reinterpret_cast<const uint4*>(eds + nxt * CDA_SHARE);
    uint4 v0 = p[0], v1 = p[1];
    uint32_t nb[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    if (ns_cmp(nb, A) < 0) atomicMin(status + t, (unsigned long long)(i + 1));
  }
  leaf_record(sh, A, q0, nodes + (size_t)gid * 6);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int launch_leaf_hash(const uint8_t* d_eds, void* d_leaf_nodes, unsigned long long* d_status, int k, int nblocks,
                     hipStream_t s) {
  const int w = 2 * k;
  int log2w = 0;
  while ((1 << log2w) < w) log2w++;
  const uint32_t total = (uint32_t)nblocks * (uint32_t)w * (uint32_t)w;
  const uint32_t grid = (total + 255) / 256;
  hipLaunchKernelGGL(leaf_hash_kernel, dim3(grid), dim3(256), 0, s, d_eds, (uint4*)d_leaf_nodes, d_status, k,
                     log2w, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_nmt_level(const void* d_in, void* d_out, bool from_leaves, int k, int nblocks, int level,
                     hipStream_t s) {
  const int w = 2 * k;
  int log2w = 0;
  while ((1 << log2w) < w) log2w++;
  const int log2n_out = log2w - level;
  const uint32_t total = (uint32_t)nblocks * (uint32_t)(2 * w) * (1u << log2n_out);
  const uint32_t grid = (total + 255) / 256;
  if (from_leaves)
    hipLaunchKernelGGL(nmt_level_kernel<true>, dim3(grid), dim3(256), 0, s, (const uint4*)d_in, (uint4*)d_out, log2w,
                       log2n_out, total);
  else
    hipLaunchKernelGGL(nmt_level_kernel<false>, dim3(grid), dim3(256), 0, s, (const uint4*)d_in, (uint4*)d_out,
                       log2w, log2n_out, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_trees_lds(const void* d_leaves, void* d_roots, void* d_dah, unsigned* d_done, void* d_digests, int k,
                     int nblocks, hipStream_t s) {
  const int w = 2 * k;
  int log2w = 0;
  while ((1 << log2w) < w) log2w++;
  if ((1 << log2w) != w || log2w < 1) return -2;
  if (w > 256) return -2;  // a thread per node of level 1 within a 128-thread half
  // two trees x (w + w / 2) records of 112 B, then 2 x 2 x 64 schedule rows of kKwStride words; the DAH fold
  // reuses it: (2w + w) x 32 B of digests + 64 schedule rows
  const size_t lds = 2 * ((size_t)w + w / 2 + 1) * kLdsRec * 16 + (size_t)4 * 64 * kKwStride * 4;
  if ((size_t)(2 * w + w) * 32 + (size_t)64 * kKwStride * 4 > lds) return -2;
  // the dynamic-LDS limit is raised to what the launch needs: 160 KiB would exceed the CU's LDS by the kernel's
  // static __shared__ word and the call would fail (and with it the launch)
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)trees_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return -1;
#if CDA_TREES_TRACE
  {
    unsigned long long* tp = nullptr;
    if (const char* e = getenv("CDA_TREES_TRACE_PTR")) tp = (unsigned long long*)(uintptr_t)strtoull(e, nullptr, 0);
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_trees_trace), &tp, sizeof tp, 0, hipMemcpyHostToDevice, s) != hipSuccess)
      return -1;
  }
#endif
  hipLaunchKernelGGL(trees_lds_kernel, dim3((unsigned)nblocks * w), dim3(256), lds, s,
                     (const uint4*)d_leaves, (uint4*)d_roots, (uint32_t*)d_dah, d_done, (uint32_t*)d_digests, log2w);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dah_wide(const void* d_roots, void* d_dah, unsigned* d_done, void* d_digests, int n, int nblocks,
                    hipStream_t s) {
  if (n < 1 || nblocks < 1) return -2;
  const size_t lds = ((size_t)n + (n + 1) / 2) * 32 + (size_t)64 * kKwStride * 4;
  if (lds > 160 * 1024 - 64) return -2;
  // the dynamic-LDS limit is a per-device attribute: raised on the current device for each launch that needs it
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)dah_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return -1;
  const int P = (n + 255) / 256;
  hipLaunchKernelGGL(dah_wide_kernel, dim3((unsigned)nblocks * P), dim3(256), lds, s, (const uint4*)d_roots,
                     (uint32_t*)d_dah, d_done, (uint32_t*)d_digests, n, P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dah(const void* d_roots, void* d_dah, int n_roots_total, int nblocks, hipStream_t s) {
  if (n_roots_total < 1) return -2;
  // digests, then 64 K+W schedule rows for dah_fold_kw
  const size_t lds = ((size_t)n_roots_total + (n_roots_total + 1) / 2) * 32 + (size_t)64 * kKwStride * 4;
  if (lds > 160 * 1024) return -2;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)dah_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(dah_kernel, dim3(nblocks), dim3(256), lds, s, (const uint4*)d_roots, (uint32_t*)d_dah,
                     n_roots_total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_axis_leaf(const uint8_t* d_leaves, int n, uint64_t square_size, uint64_t axis_index, void* d_nodes,
                     unsigned long long* d_status, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(axis_leaf_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d_leaves, n,
                     (unsigned long long)square_size, (unsigned long long)axis_index, (uint4*)d_nodes, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_axes_roots(const uint8_t* d_eds, int k, const int* d_axes, int axis0, int ntrees, int leaf_off, int nleaves,
                      void* d_nodes, void* d_scratch, void* d_roots, unsigned long long* d_status, hipStream_t s) {
  if (ntrees <= 0) return 0;
  int log2w = 0, log2n = 0;
  while ((1 << log2w) < 2 * k) log2w++;
  while ((1 << log2n) < nleaves) log2n++;
  if ((1 << log2n) != nleaves || leaf_off < 0 || leaf_off % nleaves || leaf_off + nleaves > 2 * k) return -2;
  const uint32_t total = (uint32_t)ntrees << log2n;
  hipLaunchKernelGGL(axes_leaf_kernel, dim3((total + 255) / 256), dim3(256), 0, s, d_eds, k, log2w, d_axes, axis0,
                     ntrees, leaf_off, log2n, (uint4*)(log2n == 0 ? d_roots : d_nodes), d_status);
  if (hipGetLastError() != hipSuccess) return -1;
  return launch_nmt_fold(d_nodes, d_scratch, d_roots, ntrees, log2n, s);
}

// ntrees x 2^log2n contiguous node records -> ntrees roots (levels ping-pong
// between `nodes` and `scratch`; the last level writes `roots`).
int launch_nmt_fold(void* d_nodes, void* d_scratch, void* d_roots, int ntrees, int log2n, hipStream_t s) {
  void* bufs[2] = {d_nodes, d_scratch};
  for (int level = 1; level <= log2n; level++) {
    const int log2n_out = log2n - level;
    const uint32_t tot = (uint32_t)ntrees << log2n_out;
    void* out = level == log2n ? d_roots : bufs[level & 1];
    // nmt_level_kernel<false>'s log2w argument only sizes the tree: trees of 2^log2n leaves
    hipLaunchKernelGGL(nmt_level_kernel<false>, dim3((tot + 255) / 256), dim3(256), 0, s,
                       (const uint4*)bufs[(level - 1) & 1], (uint4*)out, log2n, log2n_out, tot);
    if (hipGetLastError() != hipSuccess) return -1;
  }
  return 0;
}

// flags[a] |= 1 if the k parity cells of axis axes[a] differ from par[a][0..k)
__global__ void __launch_bounds__(256) parity_compare_kernel(const uint8_t* __restrict__ eds, int k, int log2w,
                                                             const int* __restrict__ axes, int naxes,
                                                             const uint8_t* __restrict__ par,
                                                             unsigned* __restrict__ flags) {
  const size_t per_axis = (size_t)k * (CDA_SHARE / 16);
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= per_axis * naxes) return;
  const int a = (int)(gid / per_axis);
  const size_t r = gid % per_axis;
  const int j = (int)(r / (CDA_SHARE / 16)), q = (int)(r % (CDA_SHARE / 16));
  const int ax = axes[a] >> 24, idx = axes[a] & 0xFFFFFF;
  const int i = k + j;
  const size_t cell = ax == CDA_AXIS_ROW ? ((size_t)idx << log2w) + i : ((size_t)i << log2w) + idx;
  const uint4 x = reinterpret_cast<const uint4*>(eds + cell * CDA_SHARE)[q];
  const uint4 y = reinterpret_cast<const uint4*>(par + ((size_t)a * k + j) * CDA_SHARE)[q];
  if ((x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w)) atomicOr(flags + a, 1u);
}

int launch_parity_compare(const uint8_t* d_eds, int k, const int* d_axes, int naxes, const uint8_t* d_par,
                          unsigned* d_flags, hipStream_t s) {
  if (naxes <= 0) return 0;
  int log2w = 0;
  while ((1 << log2w) < 2 * k) log2w++;
  const size_t total = (size_t)naxes * k * (CDA_SHARE / 16);
  hipLaunchKernelGGL(parity_compare_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, d_eds, k, log2w,
                     d_axes, naxes, d_par, d_flags);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Repair's root check on the device: tree t (axis code axes[t]) passes iff its status word is clean
// and its 90-B root equals want[axis][index]; *flag = min(flag, base + t) over failing trees, so
// the flag holds the first failure in verification order.
__global__ void __launch_bounds__(256) roots_check_kernel(const uint8_t* __restrict__ recs,
                                                          const unsigned long long* __restrict__ st,
                                                          const int* __restrict__ axes, int n,
                                                          const uint8_t* __restrict__ want_rows,
                                                          const uint8_t* __restrict__ want_cols,
                                                          unsigned* __restrict__ flag, unsigned base) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int ax = axes[t] >> 24, idx = axes[t] & 0xFFFFFF;
  const uint8_t* w = (ax == CDA_AXIS_ROW ? want_rows : want_cols) + (size_t)idx * CDA_NODE_SIZE;
  const uint8_t* r = recs + (size_t)t * CDA_REC_BYTES;
  unsigned diff = st[t] != ~0ull ? 1u : 0u;
  for (int i = 0; i < CDA_NODE_SIZE; i++) diff |= (unsigned)(r[i] ^ w[i]);
  if (diff) atomicMin(flag, base + (unsigned)t);
}

// Repair verification in one launch: one workgroup per axis tree.  The w leaf records are built
// in LDS, the levels fold in place there (level l node i at slot i << l, a barrier between
// levels), and the root is compared with want[axis][index]; a push-order violation (Q0 namespace
// decreasing) or a differing root sets *flag = min(*flag, base + tree) (per_tree: flag[tree] = 1).  Replaces the leaf
// kernel + log2(w) level launches + check of the generic path with one launch whose serial depth
// is the same log2(w) node hashes.
__global__ void __launch_bounds__(256) axes_verify_kernel(const uint8_t* __restrict__ eds, int k, int log2w,
                                                          const int* __restrict__ axes,
                                                          const uint8_t* __restrict__ want_rows,
                                                          const uint8_t* __restrict__ want_cols,
                                                          unsigned* __restrict__ flag, unsigned base,
                                                          int per_tree) {
  extern __shared__ __attribute__((aligned(16))) uint4 lnodes[];  // [w][6]
  __shared__ unsigned bad;
  const int w = 1 << log2w;
  const int t = blockIdx.x;
  const int code = axes[t];
  const int ax = code >> 24, idx = code & 0xFFFFFF;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < w; i += blockDim.x) {
    const size_t cell = ax == CDA_AXIS_ROW ? ((size_t)idx << log2w) + i : ((size_t)i << log2w) + idx;
    const bool q0 = (i < k) && (idx < k);
    const uint4* sh = reinterpret_cast<const uint4*>(eds + cell * CDA_SHARE);
    uint32_t A[16];
    load16(sh, A);
    if (q0 && i + 1 < k) {
      const size_t nxt = ax == CDA_AXIS_ROW ? cell + 1 : cell + w;
      const uint4* p = reinterpret_cast<const uint4*>(eds + nxt * CDA_SHARE);
      uint4 v0 = p[0], v1 = p[1];
      uint32_t nb[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      if (ns_cmp(nb, A) < 0) bad = 1;
    }
    leaf_record<false>(sh, A, q0, lnodes + (size_t)i * 6);
  }
  __syncthreads();
  for (int l = 1; l <= log2w; l++) {
    const int nodes = w >> l;
    if (nodes >= 64) {
      for (int i = threadIdx.x; i < nodes; i += blockDim.x)
        hash_node_mem(lnodes + ((size_t)(2 * i) << (l - 1)) * 6, lnodes + ((size_t)(2 * i + 1) << (l - 1)) * 6,
                      lnodes + ((size_t)i << l) * 6);
    } else if (threadIdx.x < 64) {
      // a level of < 64 nodes: the whole wave computes with a full exec mask (lanes past the last node hash node 0
      // again and store nothing; reads precede the stores within the wave) -- partly masked waves ran the tree
      // kernels' small levels ~40 % slower (r04_trees_trace.log)
      const int i = (int)threadIdx.x < nodes ? (int)threadIdx.x : 0;
      hash_node_mem(lnodes + ((size_t)(2 * i) << (l - 1)) * 6, lnodes + ((size_t)(2 * i + 1) << (l - 1)) * 6,
                    lnodes + ((size_t)i << l) * 6, (int)threadIdx.x < nodes);
    }
    __syncthreads();
  }
  if (threadIdx.x < 64) {  // root (slot 0) against the committed root: one 90-B compare, a wave's lanes
    const uint8_t* r = reinterpret_cast<const uint8_t*>(lnodes);
    const uint8_t* wr = (ax == CDA_AXIS_ROW ? want_rows : want_cols) + (size_t)idx * CDA_NODE_SIZE;
    unsigned d = 0;
    for (int i = threadIdx.x; i < CDA_NODE_SIZE; i += 64) d |= (unsigned)(r[i] ^ wr[i]);
    if (threadIdx.x == 0) d |= bad;
    if (__any(d != 0) && threadIdx.x == 0) {
      if (per_tree) flag[t] = 1u;
      else atomicMin(flag, base + (unsigned)t);
    }
  }
}

int launch_axes_verify(const uint8_t* d_eds, int k, const int* d_axes, int ntrees, const uint8_t* d_want_rows,
                       const uint8_t* d_want_cols, unsigned* d_flag, unsigned base, bool per_tree, hipStream_t s) {
  if (ntrees <= 0) return 0;
  int log2w = 0;
  while ((1 << log2w) < 2 * k) log2w++;
  const size_t lds = ((size_t)2 * k) * CDA_REC_BYTES;
  if (lds > 160 * 1024) return -2;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)axes_verify_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return -1;
  hipLaunchKernelGGL(axes_verify_kernel, dim3(ntrees), dim3(256), lds, s, d_eds, k, log2w, d_axes, d_want_rows,
                     d_want_cols, d_flag, base, per_tree ? 1 : 0);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// trees of at most this many leaves also run a level of 65..128 nodes through the latency path (LDS for 2 x 128 rows)
constexpr int kAxisRootsKw128MaxLeaves = 512;
// trees of at most this many leaves hash their leaves in the pipelined form (512 threads, below)
constexpr int kAxisRootsPipeLeaves = 256;

// Message block j (1..8) of a leaf: 0x00 ‖ ns ‖ share, so block j >= 1 holds share bytes 64j - 30 .. 64j + 33
// (windows of share words 16j - 8 .. 16j + 8); block 8 ends the 542-byte message (leaf_record's blocks 1..8).
__device__ __forceinline__ void leaf_block_words(const uint4* sh, int j, uint32_t (&m)[16]) {
  uint32_t H[8];
  {
    const uint4 a = sh[4 * j - 2], b = sh[4 * j - 1];  // share words 16j - 8 .. 16j - 1
    H[0] = a.x, H[1] = a.y, H[2] = a.z, H[3] = a.w, H[4] = b.x, H[5] = b.y, H[6] = b.z, H[7] = b.w;
  }
#pragma unroll
  for (int i = 0; i < 7; i++) m[i] = be_window(H[i], H[i + 1], 2);
  if (j < 8) {
    uint32_t C[16];
    load16(sh + 4 * j, C);
    m[7] = be_window(H[7], C[0], 2);
#pragma unroll
    for (int i = 8; i < 16; i++) m[i] = be_window(C[i - 8], C[i - 7], 2);
  } else {
    m[7] = be_window(H[7], 0x80u, 2);
#pragma unroll
    for (int i = 8; i < 15; i++) m[i] = 0;
    m[15] = 542u * 8u;
  }
}

// Block 0 of a leaf from its first 64 share bytes A (leaf_record's block 0; ns = share[0:29] if q0, else 0xFF x 29)
__device__ __forceinline__ void leaf_block0_words(const uint32_t (&A)[16], bool q0, uint32_t (&m)[16]) {
  if (q0) {
    m[0] = be_window(0u, A[0], 3);
#pragma unroll
    for (int i = 1; i < 7; i++) m[i] = be_window(A[i - 1], A[i], 3);
    m[7] = (be_window(A[6], A[7], 3) & 0xFFFF0000u) | (bswap(A[0]) >> 16);
  } else {
    m[0] = 0x00FFFFFFu;
#pragma unroll
    for (int i = 1; i < 7; i++) m[i] = 0xFFFFFFFFu;
    m[7] = 0xFFFF0000u | (bswap(A[0]) >> 16);
  }
#pragma unroll
  for (int i = 8; i < 16; i++) m[i] = be_window(A[i - 8], A[i - 7], 2);
}

// The 96-B leaf record ns ‖ ns ‖ digest ‖ 6 zero bytes from the final state (leaf_record's tail)
__device__ __forceinline__ void leaf_record_out(const uint32_t (&A)[16], bool q0, const uint32_t (&st)[8], uint4* out) {
  uint32_t ns[8], d[8], o[24];
#pragma unroll
  for (int i = 0; i < 8; i++) ns[i] = q0 ? A[i] : 0xFFFFFFFFu;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = bswap(st[i]);
#pragma unroll
  for (int i = 0; i < 7; i++) o[i] = ns[i];
  o[7] = (ns[7] & 0xFFu) | (ns[0] << 8);
#pragma unroll
  for (int i = 8; i < 14; i++) o[i] = le_window(ns[i - 8], ns[i - 7], 3);
  o[14] = (le_window(ns[6], ns[7], 3) & 0xFFFFu) | (d[0] << 16);
#pragma unroll
  for (int i = 15; i < 22; i++) o[i] = le_window(d[i - 15], d[i - 14], 2);
  o[22] = d[7] >> 16;
  o[23] = 0;
#pragma unroll
  for (int i = 0; i < 6; i++) out[i] = make_uint4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

// Roots of independent wrapper trees handed over through the per-axis seam (ErasuredNamespacedMerkleTree Push x n +
// Root, pkg/wrapper/nmt_wrapper.go:93-124; axisq.cpp coalesces concurrent calls into one launch).  Tree t's n leaves
// are contiguous 512-B shares at leaves + t * tree_stride; its axis index axis_idx[t] and the square size give the
// quadrant rule (leaf i hashes its own namespace iff i < square_size and axis index < square_size, else 0xFF x 29,
// :138-140).  One workgroup per tree: leaf records in LDS, levels folded in place (level l node i at slot i << l; a
// last odd node keeps its slot, which is the nmt split at the largest power of two below n), the root record to
// roots[t] and the first leaf whose Push order check fails (nmt ErrInvalidPushOrder) to status[t] (~0 when none).
// Replaces the leaf launch + ceil(log2 n) level launches of the generic single-tree path.
// PIPE (n <= kAxisRootsPipeLeaves, 512 threads): the leaves' 9 compressions are the other half of the tree's latency
// chain, so waves 4-7 expand each leaf's next block's K+W schedule into LDS while waves 0-3 run the current block's
// rounds alone (block 0 in full, then 8 x the 64 rounds: ~8,600 instead of ~13,000 instructions per leaf, double-
// buffered schedule rows, a barrier per block).  LDS: schedule rows A | B (2 x 256 x kKwStride words); the records
// go to region B after the last block (block 8's rows are in A), and the levels' schedule rows reuse A.
template <bool PIPE>
__global__ void __launch_bounds__(PIPE ? 512 : 256) axis_roots_kernel(const uint8_t* __restrict__ leaves,
                                                                      long long tree_stride, int n,
                                                                      unsigned long long square_size,
                                                                      const unsigned long long* __restrict__ axis_idx,
                                                                      uint4* __restrict__ roots,
                                                                      unsigned long long* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds_axis[];
  __shared__ unsigned bad;
  constexpr int kRows = kAxisRootsPipeLeaves * kKwStride;  // words of one schedule buffer (PIPE)
  uint32_t* const kwA = reinterpret_cast<uint32_t*>(lds_axis);
  // records: [n][6] (after the schedule buffer A and inside B when PIPE); then the levels' 2 x 64 (or 128) rows
  uint4* const lnodes = PIPE ? reinterpret_cast<uint4*>(kwA + kRows) : lds_axis;
  uint32_t* kw = PIPE ? kwA : reinterpret_cast<uint32_t*>(lnodes + (size_t)n * 6);
  const int t = blockIdx.x;
  const unsigned long long axis = axis_idx[t];
  const uint8_t* base = leaves + (size_t)t * tree_stride;
  if (threadIdx.x == 0) bad = 0xFFFFFFFFu;
  __syncthreads();
  if (PIPE) {
    const bool rounds = threadIdx.x < kAxisRootsPipeLeaves;
    const int i = (int)threadIdx.x & (kAxisRootsPipeLeaves - 1);
    const int li = i < n ? i : 0;  // lanes past the last leaf hash leaf 0 again and store nothing
    const bool q0 = (unsigned long long)li < square_size && axis < square_size;
    const uint4* sh = reinterpret_cast<const uint4*>(base + (size_t)li * CDA_SHARE);
    uint32_t A[16], st[8];
    uint32_t* const kwB = kwA + kRows;
    if (rounds) {
      load16(sh, A);
      if (i < n && q0 && (unsigned long long)(i + 1) < square_size && i + 1 < n) {
        const uint4* p = sh + CDA_SHARE / 16;
        const uint4 v0 = p[0], v1 = p[1];
        uint32_t nb[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        if (ns_cmp(nb, A) < 0) atomicMin(&bad, (unsigned)(i + 1));
      }
      uint32_t m[16];
      leaf_block0_words(A, q0, m);
      sha256_init(st);
      sha256_compress(st, m);
    } else {
      uint32_t m[16];
      leaf_block_words(sh, 1, m);
      sha256_kw_store(m, kwB + i * kKwStride);
    }
    __syncthreads();
    for (int j = 1; j <= 8; j++) {
      uint32_t* cur = (j & 1) ? kwB : kwA;
      uint32_t* nxt = (j & 1) ? kwA : kwB;
      if (rounds) {
        sha256_rounds_kw(st, cur + i * kKwStride);
      } else if (j < 8) {
        uint32_t m[16];
        leaf_block_words(sh, j + 1, m);
        sha256_kw_store(m, nxt + i * kKwStride);
      }
      __syncthreads();
    }
    if (rounds && i < n) leaf_record_out(A, q0, st, lnodes + (size_t)i * 6);
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const bool q0 = (unsigned long long)i < square_size && axis < square_size;
      const uint4* sh = reinterpret_cast<const uint4*>(base + (size_t)i * CDA_SHARE);
      uint32_t A[16];
      load16(sh, A);
      if (q0 && (unsigned long long)(i + 1) < square_size && i + 1 < n) {
        const uint4* p = sh + CDA_SHARE / 16;
        const uint4 v0 = p[0], v1 = p[1];
        uint32_t nb[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        if (ns_cmp(nb, A) < 0) atomicMin(&bad, (unsigned)(i + 1));
      }
      leaf_record<false>(sh, A, q0, lnodes + (size_t)i * 6);
    }
  }
  __syncthreads();
  int l = 0;
  for (int c = n; c > 1; c = (c + 1) >> 1) {
    l++;
    const int pairs = c >> 1;
    // round lanes of the latency path: 64 (one wave), or 128 for a level of 65..128 nodes when LDS holds the rows
    const int nr = pairs <= 64 ? 64 : 128;
    if (pairs > 128 || (nr == 128 && n > kAxisRootsKw128MaxLeaves)) {
      for (int i = threadIdx.x; i < pairs; i += blockDim.x)
        hash_node_mem(lnodes + ((size_t)(2 * i) << (l - 1)) * 6, lnodes + ((size_t)(2 * i + 1) << (l - 1)) * 6,
                      lnodes + ((size_t)i << l) * 6);
    } else {
      // a level of <= 64 nodes is the tree's latency chain (one wave per node set, ~5.4 cycles per instruction):
      // wave 0 hashes block 0 of its node while wave 1 expands the K+W schedules of blocks 1 and 2, and after the
      // barrier wave 0 runs only those two blocks' rounds (as trees_lds_kernel; lanes past the last pair hash node 0
      // again and store nothing, with full exec masks)
      const int i = (int)threadIdx.x & (nr - 1);
      const int p = i < pairs ? i : 0;
      uint32_t L[24], R[24], st[8];
      if ((int)threadIdx.x < 2 * nr) {
        const uint4* pl = lnodes + ((size_t)(2 * p) << (l - 1)) * 6;
        const uint4* pr = lnodes + ((size_t)(2 * p + 1) << (l - 1)) * 6;
#pragma unroll
        for (int q = 0; q < 6; q++) {
          const uint4 u = pl[q], v = pr[q];
          L[4 * q] = u.x, L[4 * q + 1] = u.y, L[4 * q + 2] = u.z, L[4 * q + 3] = u.w;
          R[4 * q] = v.x, R[4 * q + 1] = v.y, R[4 * q + 2] = v.z, R[4 * q + 3] = v.w;
        }
        uint32_t m[16];
        if ((int)threadIdx.x < nr) {
          sha256_init(st);
          node_block<0>(L, R, m);
          sha256_compress(st, m);
        } else {
          node_block<1>(L, R, m);
          sha256_kw_store(m, kw + i * kKwStride);
          node_block<2>(L, R, m);
          sha256_kw_store(m, kw + (nr + i) * kKwStride);
        }
      }
      __syncthreads();
      if ((int)threadIdx.x < nr) {
        sha256_rounds_kw(st, kw + i * kKwStride);
        sha256_rounds_kw(st, kw + (nr + i) * kKwStride);
        uint32_t o[24];
        node_record(L, R, st, o);
        if (i < pairs) {
          uint4* po = lnodes + ((size_t)i << l) * 6;
#pragma unroll
          for (int q = 0; q < 6; q++) po[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        }
      }
    }
    __syncthreads();
  }
  if (threadIdx.x < 6) roots[(size_t)t * 6 + threadIdx.x] = lnodes[threadIdx.x];
  if (threadIdx.x == 0) status[t] = bad == 0xFFFFFFFFu ? ~0ull : (unsigned long long)bad;
}

// The dynamic-LDS limits of both forms, raised once per device to the most any launch asks for: the axis queue
// launches from several threads at once (csrc/axisq.cpp), and a per-launch limit set by one thread could otherwise
// lower the limit another thread's larger launch relies on.
static int axis_roots_limits() {
  static std::mutex mu;
  static std::set<int> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  std::lock_guard<std::mutex> g(mu);
  if (done.count(dev)) return 0;
  const size_t pipe = (size_t)2 * kAxisRootsPipeLeaves * kKwStride * 4;
  const size_t wide = std::max((size_t)kAxisRootsMaxLeaves * CDA_REC_BYTES + (size_t)2 * 64 * kKwStride * 4,
                               (size_t)kAxisRootsKw128MaxLeaves * CDA_REC_BYTES + (size_t)2 * 128 * kKwStride * 4);
  if (hipFuncSetAttribute((const void*)axis_roots_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)pipe) != hipSuccess ||
      hipFuncSetAttribute((const void*)axis_roots_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)wide) != hipSuccess)
    return -1;
  done.insert(dev);
  return 0;
}

int launch_axis_roots(const uint8_t* d_leaves, long long tree_stride, int n, uint64_t square_size,
                      const unsigned long long* d_axis_idx, int ntrees, void* d_roots, unsigned long long* d_status,
                      hipStream_t s) {
  if (ntrees <= 0) return 0;
  if (n < 1 || n > kAxisRootsMaxLeaves) return -2;
  if (axis_roots_limits()) return -1;
  if (n <= kAxisRootsPipeLeaves) {  // the schedule buffers hold the levels' rows and the records (B) as well
    const size_t lds = (size_t)2 * kAxisRootsPipeLeaves * kKwStride * 4;
    hipLaunchKernelGGL(axis_roots_kernel<true>, dim3(ntrees), dim3(512), lds, s, d_leaves, tree_stride, n,
                       (unsigned long long)square_size, d_axis_idx, (uint4*)d_roots, d_status);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const size_t lds = (size_t)n * CDA_REC_BYTES + (size_t)2 * (n <= kAxisRootsKw128MaxLeaves ? 128 : 64) * kKwStride * 4;
  hipLaunchKernelGGL(axis_roots_kernel<false>, dim3(ntrees), dim3(256), lds, s, d_leaves, tree_stride, n,
                     (unsigned long long)square_size, d_axis_idx, (uint4*)d_roots, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_roots_check(const void* d_recs, const unsigned long long* d_status, const int* d_axes, int n,
                       const uint8_t* d_want_rows, const uint8_t* d_want_cols, unsigned* d_flag, unsigned base,
                       hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(roots_check_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)d_recs, d_status,
                     d_axes, n, d_want_rows, d_want_cols, d_flag, base);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_level_generic(const void* d_in, void* d_out, int n_in, hipStream_t s) {
  const int n_out = (n_in + 1) / 2;
  hipLaunchKernelGGL(level_generic_kernel, dim3((n_out + 255) / 256), dim3(256), 0, s, (const uint4*)d_in,
                     (uint4*)d_out, n_in);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cda
