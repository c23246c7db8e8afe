// split_kernels.hip — the NMT pieces of one square split over devices (host side in
// split.cpp): leaf records of a rectangle of EDS cells, push-order checks on leaf records, and roots of a set of
// trees whose leaves sit at any (tree, leaf) strides.
//
// Reference semantics as nmt_kernels.hip: leaf = ns ‖ ns ‖ SHA256(0x00 ‖ ns ‖ share), ns = share[0:29] iff the
// cell is in Q0 (pkg/wrapper/nmt_wrapper.go:93-114,138-140); node = HashNode with the IgnoreMaxNamespace range rule
// (test/util/malicious/hasher.go:271-310); push order = nmt's non-decreasing namespace check.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "cda_internal.h"
#include "nmt_dev.h"
#include "sha256_dev.h"

namespace cda {

// One thread per cell (r, c) of the rectangle [r0, r0 + nr) x [c0, c0 + 2^log2nc) of a 2k x 2k EDS whose cell
// (r0 + i, c0 + j) is at cells + i * cell_pitch + j * 512 and whose record goes to recs[i * rec_pitch + j].  With
// row_order, horizontal Q0 pairs inside the rectangle get nmt's push-order check (key axis << 40 | index << 20 |
// leaf, atomicMin into *status -- the block path's encoding).
__global__ void __launch_bounds__(256) region_leaf_kernel(const uint8_t* __restrict__ cells, long long cell_pitch,
                                                          int r0, int c0, int log2nc, uint32_t total, int k,
                                                          uint4* __restrict__ recs, long long rec_pitch,
                                                          unsigned long long* __restrict__ status, int row_order) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int i = (int)(gid >> log2nc), j = (int)(gid & ((1u << log2nc) - 1));
  const int r = r0 + i, c = c0 + j;
  const bool q0 = r < k && c < k;
  const uint4* sh = reinterpret_cast<const uint4*>(cells + i * cell_pitch + (long long)j * CDA_SHARE);
  uint32_t A[16];
  load16(sh, A);
  if (row_order && q0 && c + 1 < k && j + 1 < (1 << log2nc)) {
    const uint4* p = sh + CDA_SHARE / 16;
    const uint4 v0 = p[0], v1 = p[1];
    const uint32_t nb[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    if (ns_cmp(nb, A) < 0)
      atomicMin(status, ((unsigned long long)CDA_AXIS_ROW << 40) | ((unsigned long long)r << 20) | (unsigned)(c + 1));
  }
  leaf_record(sh, A, q0, recs + (i * rec_pitch + j) * 6);
}

// Column push order from leaf records (a leaf record starts with its namespace): records of rows 0..nr-1 of
// columns c0 .. c0 + nc - 1 at recs[r * rec_pitch + j]; pair (r, r + 1) of a Q0 column is checked.
__global__ void __launch_bounds__(256) records_col_order_kernel(const uint4* __restrict__ recs, long long rec_pitch,
                                                                int nr, int c0, int nc, int k,
                                                                unsigned long long* __restrict__ status) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (uint32_t)(nr - 1) * (uint32_t)nc) return;
  const int r = (int)(gid / (uint32_t)nc), j = (int)(gid % (uint32_t)nc);
  const int c = c0 + j;
  if (c >= k || r + 1 >= k) return;
  const uint4* a = recs + (r * rec_pitch + j) * 6;
  const uint4* b = recs + ((r + 1) * rec_pitch + j) * 6;
  const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
  const uint32_t na[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const uint32_t nb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  if (ns_cmp(nb, na) < 0)
    atomicMin(status, ((unsigned long long)CDA_AXIS_COL << 40) | ((unsigned long long)c << 20) | (unsigned)(r + 1));
}

// Levels of up to two sets of trees with the same depth, M levels per launch (the nmt_levels_kernel scheme with
// free strides): node i of tree t at level l is record lv[l].p[t * t_stride + i * i_stride].  A thread owns one
// output node and computes its subtree; tree_fastest puts consecutive trees on consecutive lanes (node-major
// layouts).  Both sets share a launch so the thin top levels of one set are not launched alone.
struct TreeLevel {
  uint4* p;
  unsigned long long t_stride, i_stride;
};
struct TreeSets {
  TreeLevel lv[2][4];
  uint32_t ntrees[2];
  int tree_fastest[2];
};

__device__ __forceinline__ uint4* tree_rec(const TreeLevel& d, unsigned t, unsigned i) {
  return d.p + (t * d.t_stride + i * d.i_stride) * 6;
}

__global__ void __launch_bounds__(256) tree_levels_kernel(TreeSets ts, int log2n_out, int M, uint32_t total0,
                                                          uint32_t total) {
  uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int set = gid >= total0;
  if (set) gid -= total0;
  const uint32_t ntrees = ts.ntrees[set];
  const unsigned t = ts.tree_fastest[set] ? gid % ntrees : gid >> log2n_out;
  const unsigned j = ts.tree_fastest[set] ? gid / ntrees : gid & ((1u << log2n_out) - 1);
  const TreeLevel* lv = ts.lv[set];
  for (int q = 1; q <= M; q++) {
    const unsigned cnt = 1u << (M - q);
    for (unsigned u = 0; u < cnt; u++) {
      const unsigned i = j * cnt + u;
      hash_node_mem(tree_rec(lv[q - 1], t, 2 * i), tree_rec(lv[q - 1], t, 2 * i + 1), tree_rec(lv[q], t, i));
    }
    if (q < M) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// ---------------------------------------------------------------------------
int launch_region_leaf(const uint8_t* d_cells, long long cell_pitch, int r0, int c0, int nr, int nc, int k,
                       void* d_recs, long long rec_pitch, unsigned long long* d_status, bool row_order, hipStream_t s) {
  int log2nc = 0;
  while ((1 << log2nc) < nc) log2nc++;
  if ((1 << log2nc) != nc || nr <= 0) return -2;
  const uint32_t total = (uint32_t)nr << log2nc;
  hipLaunchKernelGGL(region_leaf_kernel, dim3((total + 255) / 256), dim3(256), 0, s, d_cells, cell_pitch, r0, c0,
                     log2nc, total, k, (uint4*)d_recs, rec_pitch, d_status, row_order ? 1 : 0);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_records_col_order(const void* d_recs, long long rec_pitch, int nr, int c0, int nc, int k,
                             unsigned long long* d_status, hipStream_t s) {
  if (nr < 2 || nc < 1) return 0;
  const uint32_t total = (uint32_t)(nr - 1) * (uint32_t)nc;
  hipLaunchKernelGGL(records_col_order_kernel, dim3((total + 255) / 256), dim3(256), 0, s, (const uint4*)d_recs,
                     rec_pitch, nr, c0, nc, k, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Up to two sets of trees of n = 2^log2n leaves each: set q has spec[q].ntrees trees, leaf i of tree t at
// leaves[t * t_stride + i * i_stride], root to roots[t * r_stride]; inner levels in its own scratch (ntrees * n
// records suffice), tree-major unless tree_fastest (then node-major).
int launch_tree_roots(const TreeSpec* spec, int nsets, int log2n, hipStream_t s) {
  if (nsets < 1 || nsets > 2) return -2;
  if (log2n == 0) return -2;  // a one-leaf tree's root is the leaf record: the caller copies it
  const int L = log2n;
  auto desc = [&](const TreeSpec& sp, int l) {
    TreeLevel d{};
    const unsigned long long n = 1ull << (L - l);
    if (l == 0) {
      d.p = (uint4*)sp.leaves;
      d.t_stride = sp.t_stride;
      d.i_stride = sp.i_stride;
    } else if (l == L) {
      d.p = (uint4*)sp.roots;
      d.t_stride = sp.r_stride;
      d.i_stride = 0;
    } else {
      unsigned long long off = 0;
      for (int q = 1; q < l; q++) off += (unsigned long long)sp.ntrees << (L - q);
      d.p = (uint4*)sp.scratch + off * 6;
      d.t_stride = sp.tree_fastest ? 1 : n;
      d.i_stride = sp.tree_fastest ? sp.ntrees : 1;
    }
    return d;
  };
  for (int l_in = 0; l_in < L;) {
    int M = std::min(2, L - l_in);
    if (L - l_in == 3) M = 3;
    TreeSets ts{};
    for (int q = 0; q < nsets; q++) {
      for (int u = 0; u <= M; u++) ts.lv[q][u] = desc(spec[q], l_in + u);
      ts.ntrees[q] = spec[q].ntrees;
      ts.tree_fastest[q] = spec[q].tree_fastest ? 1 : 0;
    }
    const int log2n_out = L - (l_in + M);
    const uint32_t total0 = spec[0].ntrees << log2n_out;
    const uint32_t total = total0 + (nsets > 1 ? spec[1].ntrees << log2n_out : 0);
    if (total) {
      hipLaunchKernelGGL(tree_levels_kernel, dim3((total + 255) / 256), dim3(256), 0, s, ts, log2n_out, M, total0,
                         total);
      if (hipGetLastError() != hipSuccess) return -1;
    }
    l_in += M;
  }
  return 0;
}

}  // namespace cda
