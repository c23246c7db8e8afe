// nmt_dev.h — erasured-NMT leaf hashing device code (leaf_hash_kernel and the
// single-tree / axis-list leaf kernels in nmt_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cda_internal.h"
#include "sha256_dev.h"

namespace cda {

// ---------------------------------------------------------------------------
// Leaf hashing: one thread per EDS cell.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load16(const uint4* p, uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint4 v = p[i];
    w[4 * i + 0] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}

// Big-endian namespace words of a 29-byte namespace held little-endian in n[0..7]
// (n[7] byte 0 = ns[28]) compared lexicographically: returns -1/0/1.
__device__ __forceinline__ int ns_cmp(const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t x = bswap(a[i]), y = bswap(b[i]);
    if (i == 7) {
      x >>= 24;
      y >>= 24;
    }
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

// A parity leaf's first block starts 0x00 ‖ 0xFF x 29 (message words 0..6 constant): its working state after rounds
// 0..6 is a constant, so those rounds are skipped (3 in 4 cells of a square are parity leaves).
constexpr uint32_t kParityLeafMid7[8] = {0x1ca5c518, 0x33e5c969, 0xbd2d00ce, 0xa4502bae,
                                         0xce23fa11, 0x90a5b516, 0x5df56d75, 0xf3f677da};
#ifndef CDA_NO_PARITY_MID
#define CDA_NO_PARITY_MID 0  // diagnostic A/B: every leaf and inner node through all 64 rounds of its first block
#endif

// Leaf record of one 512-B share whose first 64 bytes are already in A[0..16):
// ns ‖ ns ‖ SHA256(0x00 ‖ ns ‖ share) ‖ 6 zero bytes, ns = share[0:29] if q0 else 0xFF×29.
// Blocks 1..7 stay a loop (one copy of the compression code: measured as fast as
// the unrolled form on MI355X, with half the instruction footprint).
// The share is read one 128-B line at a time (two 64-B chunks loaded together, the odd chunk held in N until its
// block): loaded a compression apart, the line's second half missed in L2 often enough that the leaf kernel fetched
// 1.31x its bytes (all 128-B requests, profiles/r04_rdreq_sizes.json).  PAIRS = false: one chunk per block (16
// fewer VGPRs; repair's root check, whose kernel would otherwise pass 128).
template <bool PAIRS = true>
__device__ __forceinline__ void leaf_record(const uint4* sh, uint32_t* A, bool q0, uint4* out) {
  uint32_t N[16];
  if (PAIRS) load16(sh + 4, N);  // chunk 1, the rest of the line A came from
  uint32_t ns[8];
#pragma unroll
  for (int i = 0; i < 8; i++) ns[i] = q0 ? A[i] : 0xFFFFFFFFu;
  uint32_t st[8];
  sha256_init(st);
  uint32_t m[16];
  // block 0: 0x00 ‖ ns[0..29) ‖ share[0..34)
  if (q0) {
    m[0] = be_window(0u, A[0], 3);
#pragma unroll
    for (int i = 1; i < 7; i++) m[i] = be_window(A[i - 1], A[i], 3);
    // bytes 28..31 = ns[27], ns[28], share[0], share[1]
    m[7] = (be_window(A[6], A[7], 3) & 0xFFFF0000u) | (bswap(A[0]) >> 16);
  } else {
    m[0] = 0x00FFFFFFu;
#pragma unroll
    for (int i = 1; i < 7; i++) m[i] = 0xFFFFFFFFu;
    m[7] = 0xFFFF0000u | (bswap(A[0]) >> 16);
  }
#pragma unroll
  for (int i = 8; i < 16; i++) m[i] = be_window(A[i - 8], A[i - 7], 2);
  // wave-uniform only (a wave of parity and Q0 cells runs the general path: both paths in one wave cost more than the
  // 7 rounds saved)
  if (!CDA_NO_PARITY_MID && __all(!q0)) {
    uint32_t mw[16], mid[8];
    mw[0] = 0x00FFFFFFu;
#pragma unroll
    for (int i = 1; i < 7; i++) mw[i] = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 7; i < 16; i++) mw[i] = m[i];
#pragma unroll
    for (int i = 0; i < 8; i++) mid[i] = kParityLeafMid7[i];
    sha256_compress_fenced_from<7, false>(st, mid, mw);
  } else {
    sha256_compress(st, m);
  }
  // blocks 1..7: message words 16j..16j+15 = share bytes 64j-30.. : windows of S[16j-8 .. 16j+8].
  // H carries the upper half of the previous 16-word chunk.
  uint32_t H[8];
#pragma unroll
  for (int i = 0; i < 8; i++) H[i] = A[8 + i];
#pragma unroll 1
  for (int j = 1; j < 8; j++) {
    uint32_t C[16];
    if (!PAIRS) {
      load16(sh + 4 * j, C);
    } else if (j & 1) {  // odd chunk: loaded with the even one before it
#pragma unroll
      for (int i = 0; i < 16; i++) C[i] = N[i];
    } else {
      load16(sh + 4 * j, C);
      load16(sh + 4 * (j + 1), N);
    }
#pragma unroll
    for (int i = 0; i < 7; i++) m[i] = be_window(H[i], H[i + 1], 2);
    m[7] = be_window(H[7], C[0], 2);
#pragma unroll
    for (int i = 8; i < 16; i++) m[i] = be_window(C[i - 8], C[i - 7], 2);
    sha256_compress(st, m);
#pragma unroll
    for (int i = 0; i < 8; i++) H[i] = C[8 + i];
  }
  // block 8: share bytes 482..511, 0x80, zeros, bit length 542*8
#pragma unroll
  for (int i = 0; i < 7; i++) m[i] = be_window(H[i], H[i + 1], 2);
  m[7] = be_window(H[7], 0x80u, 2);
#pragma unroll
  for (int i = 8; i < 15; i++) m[i] = 0;
  m[15] = 542u * 8u;
  sha256_compress(st, m);
  // record: ns ‖ ns ‖ digest ‖ 6 zero bytes
  uint32_t d[8];
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = bswap(st[i]);
  uint32_t o[24];
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

// One EDS cell `gid` (= blk * w^2 + r * w + c) of a batch: push-order check against
// its Q0 right / lower neighbours, then its 96-B leaf record.
__device__ __forceinline__ void leaf_cell(const uint8_t* __restrict__ eds, uint4* __restrict__ nodes,
                                          unsigned long long* __restrict__ status, int k, int log2w, uint32_t gid) {
  const int w = 1 << log2w;
  const uint32_t cell = gid & ((1u << (2 * log2w)) - 1);
  const uint32_t blk = gid >> (2 * log2w);
  const int r = (int)(cell >> log2w), c = (int)(cell & (w - 1));
  const bool q0 = (r < k) && (c < k);
  const uint4* sh = reinterpret_cast<const uint4*>(eds + (size_t)gid * CDA_SHARE);

  uint32_t A[16];
  load16(sh, A);
  uint32_t ns[8];
#pragma unroll
  for (int i = 0; i < 8; i++) ns[i] = A[i];

  // Namespace order (nmt Push ErrInvalidPushOrder) — checked for Q0 neighbours;
  // parity leaves carry 0xFF×29, the maximum, so only Q0 pairs can violate it.
  if (q0) {
    if (c + 1 < k) {
      uint32_t nb[8];
      const uint4* p = reinterpret_cast<const uint4*>(eds + ((size_t)gid + 1) * CDA_SHARE);
      uint4 v0 = p[0], v1 = p[1];
      nb[0] = v0.x; nb[1] = v0.y; nb[2] = v0.z; nb[3] = v0.w;
      nb[4] = v1.x; nb[5] = v1.y; nb[6] = v1.z; nb[7] = v1.w;
      if (ns_cmp(nb, ns) < 0) {
        unsigned long long key = ((unsigned long long)CDA_AXIS_ROW << 40) | ((unsigned long long)r << 20) | (c + 1);
        atomicMin(status + blk, key);
      }
    }
    if (r + 1 < k) {
      uint32_t nb[8];
      const uint4* p = reinterpret_cast<const uint4*>(eds + ((size_t)gid + w) * CDA_SHARE);
      uint4 v0 = p[0], v1 = p[1];
      nb[0] = v0.x; nb[1] = v0.y; nb[2] = v0.z; nb[3] = v0.w;
      nb[4] = v1.x; nb[5] = v1.y; nb[6] = v1.z; nb[7] = v1.w;
      if (ns_cmp(nb, ns) < 0) {
        unsigned long long key = ((unsigned long long)CDA_AXIS_COL << 40) | ((unsigned long long)c << 20) | (r + 1);
        atomicMin(status + blk, key);
      }
    }
  }

  leaf_record(sh, A, q0, nodes + (size_t)gid * 6);
}

// ---------------------------------------------------------------------------
// Inner NMT node (also the in-place mountain fold of inclusion_kernels.hip).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ld4(const uint4* p, uint32_t* w) {  // 4 x 16 B -> 16 words
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint4 v = p[i];
    w[4 * i + 0] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}

// Inner node from the two child records at pl / pr, written to po (po may equal
// pl: every read precedes the stores).  The children are read block by block
// through laundered pointers ordered after the previous compression, so the
// reads are neither merged nor hoisted and kept live, and each compression is
// fenced: 89 VGPRs (5 waves/SIMD) instead of 205 when both children stayed in
// registers.
// ns_lds (optional): this thread's 128-B LDS slot; the first 64 B of both children are parked there when loaded for
// blocks 0 / 1 and the namespace range is read back from it instead of from global memory.  With the slots 128 B
// apart, lane i's piece j shares banks with every other lane's piece j (8-way conflicts on ds_write_b128 /
// ds_read_b128).  Swizzling the pieces (piece ^ ((lane ^ lane >> 3) & 7)) removed every conflict of the levels 1-2
// launch (SQ_LDS_BANK_CONFLICT 132 M -> 0) but moved blocks/s by +0.3 / +0.9 % on two boxes (the kernel is
// VALU-bound): below the 1 % bar, not kept.
// parity: both children lie in the parity part of the square (every leaf below them has the parity namespace, so each
// child's first 58 bytes are 0xFF): block 0 is 0x01 ‖ 0xFF x 58 ‖ 5 digest bytes, and its first 14 rounds run on
// constant words from a constant state -- they are skipped (kParityMid14), 14 of the node's 192 rounds.  About 3 in 4
// inner nodes of a square are such (rows / columns >= k entirely, the right half of the others).
constexpr uint32_t kParityMid14[8] = {0xa8abd42b, 0x092979bd, 0x8d5926ca, 0x8df58526,
                                      0xa812caa9, 0x7cc8da5d, 0x33a85111, 0x7d669380};
__device__ __forceinline__ void hash_node_mem(const uint4* pl, const uint4* pr, uint4* po, bool store = true,
                                              uint4* ns_lds = nullptr, bool parity = false) {
  uint32_t st[8], m[16];
  sha256_init(st);
  // message = 0x01 ‖ L[0..90) ‖ R[0..90) ‖ 0x80 ‖ 0.. ‖ len(1448 bits); 48 words
  {  // block 0: words 0..15 <- L words 0..15
    uint32_t L[16];
    ld4(launder(pl), L);
    m[0] = be_window(0x01000000u, L[0], 3);
#pragma unroll
    for (int i = 1; i < 16; i++) m[i] = be_window(L[i - 1], L[i], 3);
    if (ns_lds)
#pragma unroll
      for (int i = 0; i < 4; i++) ns_lds[i] = make_uint4(L[4 * i], L[4 * i + 1], L[4 * i + 2], L[4 * i + 3]);
  }
  // wave-uniform only: a wave whose nodes are partly parity takes the general path (in a divergent wave both paths
  // would run, 114 rounds instead of 64; measured 3 % slower on the step, profiles/r06_ab_parity_mid.jsonl)
  if (__all(parity)) {
    uint32_t mw[16];
    mw[0] = 0x01FFFFFFu;
#pragma unroll
    for (int i = 1; i < 14; i++) mw[i] = 0xFFFFFFFFu;
    mw[14] = m[14];
    mw[15] = m[15];
    uint32_t mid[8];
#pragma unroll
    for (int i = 0; i < 8; i++) mid[i] = kParityMid14[i];
    sha256_compress_fenced_from<14>(st, mid, mw);
  } else {
    sha256_compress_fenced(st, m);
  }
  {  // block 1: words 16..31 <- L words 15..22, R words 0..8
    uint32_t L[16], R[16];  // L words 12..27, R words 0..15
    ld4(launder_after(pl, st[0]) + 3, L);  // words 12..27: only 12..23 are read
    ld4(launder_after(pr, st[0]), R);      // words 0..15: only 0..11 are read
    if (ns_lds)
#pragma unroll
      for (int i = 0; i < 4; i++) ns_lds[4 + i] = make_uint4(R[4 * i], R[4 * i + 1], R[4 * i + 2], R[4 * i + 3]);
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int wi = 16 + i;
      if (wi <= 21) m[i] = be_window(L[wi - 13], L[wi - 12], 3);
      else if (wi == 22) m[i] = be_window(L[9], L[10], 3) | (R[0] & 0xFFu);
      else m[i] = be_window(R[wi - 23], R[wi - 22], 1);
    }
  }
  sha256_compress_fenced(st, m);
  {  // block 2: words 32..47 <- R words 8..23
    uint32_t R[16];
    ld4(launder_after(pr, st[0]) + 2, R);
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int wi = 32 + i;
      if (wi <= 44) m[i] = be_window(R[wi - 31], R[wi - 30], 1);
      else if (wi == 45) m[i] = be_window(R[14], R[15], 1) | 0x00800000u;
      else if (wi == 46) m[i] = 0;
      else m[i] = 181u * 8u;
    }
  }
  sha256_compress_fenced(st, m);

  // namespace range: min = L.min; max = R.min == parity ns ? L.max : R.max
  uint32_t L[16], R[16];
  if (ns_lds) {
    uint32_t z = 0;  // an offset tied to the last compression keeps the LDS reads below it (pointer stays in LDS)
    asm volatile("" : "+v"(z) : "v"(st[0]));
    ld4(ns_lds + z, L);
    ld4(ns_lds + z + 4, R);
#pragma unroll
    for (int i = 0; i < 16; i++) asm volatile("" : "+v"(L[i]), "+v"(R[i]));  // values, not a select of addresses
  } else {
    ld4(launder_after(pl, st[0]), L);
    ld4(launder_after(pr, st[0]), R);
  }
  bool rmin_max = true;
#pragma unroll
  for (int i = 0; i < 7; i++) rmin_max &= (R[i] == 0xFFFFFFFFu);
  rmin_max &= ((R[7] & 0xFFu) == 0xFFu);
  uint32_t S[16];
#pragma unroll
  for (int i = 7; i < 15; i++) S[i] = rmin_max ? L[i] : R[i];
  uint32_t d[8];
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = bswap(st[i]);
  uint32_t o[24];
#pragma unroll
  for (int i = 0; i < 7; i++) o[i] = L[i];
  o[7] = (L[7] & 0xFFu) | (S[7] & 0xFFFFFF00u);
#pragma unroll
  for (int i = 8; i < 14; i++) o[i] = S[i];
  o[14] = (S[14] & 0xFFFFu) | (d[0] << 16);
#pragma unroll
  for (int i = 15; i < 22; i++) o[i] = le_window(d[i - 15], d[i - 14], 2);
  o[22] = d[7] >> 16;
  o[23] = 0;
  if (store)
#pragma unroll
    for (int i = 0; i < 6; i++) po[i] = make_uint4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

// Message block B (0..2) of an inner node: 0x01 ‖ L[0..90) ‖ R[0..90) ‖ 0x80 ‖ 0.. ‖ len(1448 bits), children in
// record layout (24 words each).
template <int B>
__device__ __forceinline__ void node_block(const uint32_t (&L)[24], const uint32_t (&R)[24], uint32_t (&m)[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int wi = 16 * B + i;
    if (wi == 0) m[i] = be_window(0x01000000u, L[0], 3);
    else if (wi <= 21) m[i] = be_window(L[wi - 1], L[wi], 3);
    else if (wi == 22) m[i] = be_window(L[21], L[22], 3) | (R[0] & 0xFFu);
    else if (wi <= 44) m[i] = be_window(R[wi - 23], R[wi - 22], 1);
    else if (wi == 45) m[i] = be_window(R[22], R[23], 1) | 0x00800000u;
    else if (wi == 46) m[i] = 0;
    else m[i] = 181u * 8u;
  }
}
// The node record from its children and the digest state: min = L.min; max = R.min == parity ns ? L.max : R.max.
__device__ __forceinline__ void node_record(const uint32_t (&L)[24], const uint32_t (&R)[24], const uint32_t (&st)[8],
                                            uint32_t (&o)[24]);

// hash_node_mem with both children already in registers (24 words each, record layout): the form for latency
// kernels that run one wave per SIMD, where registers are free and a memory round trip per compression is not.
__device__ __forceinline__ void hash_node_regs(const uint32_t (&L)[24], const uint32_t (&R)[24], uint32_t (&o)[24]) {
  uint32_t st[8], m[16];
  sha256_init(st);
  node_block<0>(L, R, m);
  sha256_compress(st, m);
  node_block<1>(L, R, m);
  sha256_compress(st, m);
  node_block<2>(L, R, m);
  sha256_compress(st, m);
  node_record(L, R, st, o);
}
__device__ __forceinline__ void node_record(const uint32_t (&L)[24], const uint32_t (&R)[24], const uint32_t (&st)[8],
                                            uint32_t (&o)[24]) {
  bool rmin_max = true;
#pragma unroll
  for (int i = 0; i < 7; i++) rmin_max &= (R[i] == 0xFFFFFFFFu);
  rmin_max &= ((R[7] & 0xFFu) == 0xFFu);
  uint32_t S[16];
#pragma unroll
  for (int i = 7; i < 15; i++) S[i] = rmin_max ? L[i] : R[i];
  uint32_t d[8];
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = bswap(st[i]);
#pragma unroll
  for (int i = 0; i < 7; i++) o[i] = L[i];
  o[7] = (L[7] & 0xFFu) | (S[7] & 0xFFFFFF00u);
#pragma unroll
  for (int i = 8; i < 14; i++) o[i] = S[i];
  o[14] = (S[14] & 0xFFFFu) | (d[0] << 16);
#pragma unroll
  for (int i = 15; i < 22; i++) o[i] = le_window(d[i - 15], d[i - 14], 2);
  o[22] = d[7] >> 16;
  o[23] = 0;
}

}  // namespace cda
