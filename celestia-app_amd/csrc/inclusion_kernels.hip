// inclusion_kernels.hip — blob share commitments and RFC-6962 roots over NMT nodes (gfx950).
//
// Reference semantics (celestia-app @ 2025-02-13):
//   go-square v1.0.1 inclusion.CreateCommitment (go.mod:9, not vendored), called by
//   x/blob/types/payforblob.go:53 and blob_tx.go:98:
//     shares = sparse shares of the blob (specs/src/specs/shares.md:31-81)
//     W      = SubTreeWidth(len(shares), SubtreeRootThreshold)   (data_square_layout.md:53)
//     trees  = MerkleMountainRangeSizes(len(shares), W): W, W, .., then decreasing powers of two
//     roots  = NMT root of every tree over leaves ns ‖ share (IgnoreMaxNamespace)
//     commit = merkle.HashFromByteSlices(roots)
//   merkle.HashFromByteSlices over NMT nodes: the DAH (pkg/da/data_availability_header.go:92-108)
//   and GetCommitment (pkg/inclusion/get_commit.go:29).
//
// Design: the host only plans (share counts, mountain boundaries).  The shares of
// every blob of a call are materialised contiguously in HBM (one 16-B store per
// lane), hashed one thread per share into 96-B leaf records (the erasured-NMT Q0
// leaf of nmt_dev.h: a blob share's namespace is its own), then all mountains of
// all blobs are folded in place, one launch per level: the node over leaves
// [p, p + 2^l) of a mountain overwrites record p.  The commitments are RFC-6962
// roots over the mountain roots, one workgroup per blob, levels in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cda_internal.h"
#include "nmt_dev.h"
#include "sha256_dev.h"

namespace cda {

__constant__ uint32_t c_sha_empty[8] = {0xe3b0c442u, 0x98fc1c14u, 0x9afbf4c8u, 0x996fb924u,
                                        0x27ae41e4u, 0x649b934cu, 0xa495991bu, 0x7852b855u};

// Blob holding share g: the last blob whose first share is <= g.
__device__ __forceinline__ int find_blob(const BlobDesc* __restrict__ d, int n, uint32_t g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].share_off <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Mountain of blob-local share j (n shares, full mountains of width w): its size and j's position in it.
__device__ __forceinline__ void mountain_of(uint32_t j, uint32_t n, uint32_t w, uint32_t& size, uint32_t& pos) {
  const uint32_t full = n / w * w;
  if (j < full) {
    size = w;
    pos = j & (w - 1);
    return;
  }
  const uint32_t r = n - full;
  uint32_t jj = j - full, cum = 0;
  size = 1;
  pos = 0;
  for (int b = 31; b >= 0; b--) {
    const uint32_t s = 1u << b;
    if (!(r & s)) continue;
    if (jj < cum + s) {
      size = s;
      pos = jj - cum;
      return;
    }
    cum += s;
  }
}

// Sparse shares (SparseShareSplitter.Write): ns ‖ info ‖ [sequence length] ‖ data ‖ zeros.
// One thread per 16-byte word of the output, 32 threads per share.
__global__ void __launch_bounds__(256) blob_shares_kernel(const BlobDesc* __restrict__ d, int nblobs,
                                                          const uint8_t* __restrict__ data, uint32_t total,
                                                          uint4* __restrict__ shares) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = (uint32_t)(gid >> 5), q = (uint32_t)(gid & 31);
  if (g >= total) return;
  const BlobDesc& b = d[find_blob(d, nblobs, g)];
  const uint32_t j = g - b.share_off;
  const uint8_t* src = data + b.data_off;
  constexpr uint32_t NS = CDA_NAMESPACE_SIZE;
  uint32_t w[4];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const uint32_t pos = 16 * q + 4 * t + e;
      uint32_t byte;
      if (pos < NS) byte = b.ns[pos];
      else if (pos == NS) byte = ((uint32_t)b.ns[NS] << 1) | (j == 0 ? 1u : 0u);  // info byte
      else if (j == 0 && pos < NS + 5) byte = (b.len >> (8 * (NS + 4 - pos))) & 0xFFu;  // sequence length
      else {
        const uint32_t idx = j == 0 ? pos - (NS + 5) : 478u + (j - 1) * 482u + (pos - (NS + 1));
        byte = idx < b.len ? src[idx] : 0u;
      }
      v |= byte << (8 * e);
    }
    w[t] = v;
  }
  shares[(size_t)g * 32 + q] = make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void __launch_bounds__(256) blob_leaf_kernel(const uint8_t* __restrict__ shares, uint32_t total,
                                                        uint4* __restrict__ recs) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  const uint4* sh = reinterpret_cast<const uint4*>(shares + (size_t)g * CDA_SHARE);
  uint32_t A[16];
  load16(sh, A);
  leaf_record(sh, A, true, recs + (size_t)g * 6);
}

// Level `level` of every mountain: the node over leaves [p, p + 2^level) replaces record p.
__global__ void __launch_bounds__(256) blob_mountain_level_kernel(const BlobDesc* __restrict__ d, int nblobs,
                                                                  uint4* recs, uint32_t total, int level) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  const BlobDesc& b = d[find_blob(d, nblobs, g)];
  uint32_t size, pos;
  mountain_of(g - b.share_off, b.nshares, b.width, size, pos);
  const uint32_t span = 1u << level;
  if (size < span || (pos & (span - 1))) return;
  hash_node_mem(recs + (size_t)g * 6, recs + (size_t)(g + span / 2) * 6, recs + (size_t)g * 6);
}

// SHA256(0x00 ‖ node[0..90)) of a 96-B record: the RFC-6962 leaf hash of an NMT node.
__device__ __forceinline__ void leaf90_digest(const uint4* rec, uint32_t* st) {
  uint32_t L[24];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint4 v = rec[i];
    L[4 * i] = v.x;
    L[4 * i + 1] = v.y;
    L[4 * i + 2] = v.z;
    L[4 * i + 3] = v.w;
  }
  uint32_t m[16];
  sha256_init(st);
  m[0] = be_window(0u, L[0], 3);
#pragma unroll
  for (int t = 1; t < 16; t++) m[t] = be_window(L[t - 1], L[t], 3);
  sha256_compress(st, m);
#pragma unroll
  for (int t = 0; t < 16; t++) {
    const int wi = 16 + t;
    if (wi <= 21) m[t] = be_window(L[wi - 1], L[wi], 3);
    else if (wi == 22) m[t] = be_window(L[21], L[22], 3) | 0x80u;
    else if (wi < 31) m[t] = 0;
    else m[t] = 91u * 8u;
  }
  sha256_compress(st, m);
}

// SHA256(0x01 ‖ L ‖ R) of two digests held as big-endian words.
__device__ __forceinline__ void inner_digest(const uint32_t* Ld, const uint32_t* Rd, uint32_t* o) {
  uint32_t st[8], m[16];
  sha256_init(st);
  m[0] = 0x01000000u | (Ld[0] >> 8);
#pragma unroll
  for (int t = 1; t < 8; t++) m[t] = (Ld[t - 1] << 24) | (Ld[t] >> 8);
  m[8] = (Ld[7] << 24) | (Rd[0] >> 8);
#pragma unroll
  for (int t = 9; t < 16; t++) m[t] = (Rd[t - 9] << 24) | (Rd[t - 8] >> 8);
  sha256_compress(st, m);
  m[0] = (Rd[7] << 24) | 0x00800000u;
#pragma unroll
  for (int t = 1; t < 15; t++) m[t] = 0;
  m[15] = 65u * 8u;
  sha256_compress(st, m);
#pragma unroll
  for (int t = 0; t < 8; t++) o[t] = st[t];
}

// One workgroup per set.  Levels pair (2i, 2i+1) and promote an odd last node,
// the same tree as HashFromByteSlices' split at the largest power of two below n.
__global__ void __launch_bounds__(256) merkle_sets_kernel(const uint4* __restrict__ recs,
                                                          const uint32_t* __restrict__ idx,
                                                          const uint32_t* __restrict__ off, uint32_t* __restrict__ out,
                                                          uint32_t* __restrict__ nodes_out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sdig[];
  const uint32_t s = blockIdx.x, b0 = off[s];
  const int n = (int)(off[s + 1] - b0);
  if (n == 0) {  // HashFromByteSlices of no items = SHA256("")
    if (threadIdx.x < 8) out[s * 8 + threadIdx.x] = bswap(c_sha_empty[threadIdx.x]);
    return;
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t r = idx ? idx[b0 + i] : b0 + (uint32_t)i;
    uint32_t st[8];
    leaf90_digest(recs + (size_t)r * 6, st);
#pragma unroll
    for (int t = 0; t < 8; t++) sdig[i * 8 + t] = st[t];
    if (nodes_out) {
#pragma unroll
      for (int t = 0; t < 8; t++) nodes_out[(size_t)i * 8 + t] = bswap(st[t]);
    }
  }
  __syncthreads();
  uint32_t* src = sdig;
  uint32_t* dst = sdig + n * 8;
  size_t base = (size_t)n;
  for (int cnt = n; cnt > 1;) {
    const int oc = (cnt + 1) >> 1;
    for (int i = threadIdx.x; i < oc; i += blockDim.x) {
      uint32_t* o = dst + i * 8;
      if (2 * i + 1 < cnt) {
        inner_digest(src + 2 * i * 8, src + (2 * i + 1) * 8, o);
      } else {
#pragma unroll
        for (int t = 0; t < 8; t++) o[t] = src[2 * i * 8 + t];
      }
      if (nodes_out) {
#pragma unroll
        for (int t = 0; t < 8; t++) nodes_out[(base + i) * 8 + t] = bswap(o[t]);
      }
    }
    __syncthreads();
    uint32_t* tmp = src;
    src = dst;
    dst = tmp;
    base += oc;
    cnt = oc;
  }
  if (threadIdx.x < 8) out[s * 8 + threadIdx.x] = bswap(src[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int launch_blob_shares(const BlobDesc* d_desc, int nblobs, const uint8_t* d_data, uint32_t total, uint8_t* d_shares,
                       hipStream_t s) {
  if (total == 0 || nblobs <= 0) return 0;
  const uint64_t grid = ((uint64_t)total * 32 + 255) / 256;
  if (grid > 0x7FFFFFFFull) return -2;
  hipLaunchKernelGGL(blob_shares_kernel, dim3((unsigned)grid), dim3(256), 0, s, d_desc, nblobs, d_data, total,
                     (uint4*)d_shares);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_blob_leaves(const uint8_t* d_shares, uint32_t total, void* d_recs, hipStream_t s) {
  if (total == 0) return 0;
  hipLaunchKernelGGL(blob_leaf_kernel, dim3((total + 255) / 256), dim3(256), 0, s, d_shares, total, (uint4*)d_recs);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_blob_mountain_level(const BlobDesc* d_desc, int nblobs, void* d_recs, uint32_t total, int level,
                               hipStream_t s) {
  if (total == 0 || nblobs <= 0) return 0;
  hipLaunchKernelGGL(blob_mountain_level_kernel, dim3((total + 255) / 256), dim3(256), 0, s, d_desc, nblobs,
                     (uint4*)d_recs, total, level);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Node export, one level at a time: the 90-byte nodes of level h of trees [t0, t0 + nt) of one kind (rows: trees
// 0..w-1 of the level buffer, columns: w..2w-1; leaves: the cell-major records) into the per-tree node lists
// out[t - t0][off_h + p] (2w - 1 nodes of 90 B per tree, leaves first, root last) -- the layout the export hands back,
// built on the device so that one copy moves it (no host repacking of 96-byte records).  One thread per node, 45
// two-byte words (a 90-byte node is 2-byte aligned).
__global__ void __launch_bounds__(256) pack_tree_level_kernel(const uint8_t* __restrict__ recs, uint8_t* __restrict__ out,
                                                              int log2w, int h, int col, uint32_t t0, uint32_t nt,
                                                              uint32_t off_h) {
  const uint32_t w = 1u << log2w, nh = w >> h;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nt * nh) return;
  const uint32_t t = t0 + g / nh, p = g % nh;
  size_t rec;
  if (h == 0) rec = col ? (size_t)p * w + t : (size_t)t * w + p;  // leaves: cell (row t, col p) / (row p, col t)
  else rec = ((size_t)(col ? w + t : t)) * nh + p;                // levels: [tree][n], rows then columns
  const uint16_t* src = reinterpret_cast<const uint16_t*>(recs + rec * CDA_REC_BYTES);
  uint16_t* dst = reinterpret_cast<uint16_t*>(out + ((size_t)(t - t0) * (2 * w - 1) + off_h + p) * CDA_NODE_SIZE);
#pragma unroll
  for (int q = 0; q < CDA_NODE_SIZE / 2; q++) dst[q] = src[q];
}

int launch_pack_tree_level(const void* d_recs, void* d_out, int log2w, int h, bool col, uint32_t t0, uint32_t nt,
                           uint32_t off_h, hipStream_t s) {
  const uint32_t n = nt * ((1u << log2w) >> h);
  if (n == 0) return 0;
  hipLaunchKernelGGL(pack_tree_level_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)d_recs,
                     (uint8_t*)d_out, log2w, h, col ? 1 : 0, t0, nt, off_h);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_merkle_sets(const void* d_recs, const uint32_t* d_idx, const uint32_t* d_off, int nsets, int max_set,
                       void* d_out, void* d_nodes_out, hipStream_t s) {
  if (nsets <= 0) return 0;
  const size_t lds = ((size_t)max_set + (max_set + 1) / 2) * 32;
  if (lds > 160 * 1024) return -2;
  if (lds > 64 * 1024 && hipFuncSetAttribute((const void*)merkle_sets_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(merkle_sets_kernel, dim3(nsets), dim3(256), lds ? lds : 32, s, (const uint4*)d_recs, d_idx, d_off,
                     (uint32_t*)d_out, (uint32_t*)d_nodes_out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cda
