// rs_kernels.hip — Leopard Reed-Solomon encode on gfx950, bit-sliced.
//
// Reference: klauspost/reedsolomon v1.12.1 leopardFF8.encode as called by rsmt2d
// LeoRSCodec.Encode (upstream, pinned go.mod:153/13; selected by
// pkg/appconsts/global_consts.go:92).  Algorithm: work =
// data ‖ zero pad to m = ceilPow2(k); IFFT-DIT with skew[m-1+·]; FFT-DIT with
// skew[·-1]; parity = work[0..k).  The radix-4 passes of the reference are
// re-expressed as radix-2 layers (identical arithmetic, same order of layers):
//   IFFT layer D = 1,2,..,m/2 : group s (multiple of 2D): y ^= x; x ^= y*exp(skew[m-1+s+D])
//   FFT  layer D = m/2,..,2,1 : group s               : x ^= y*exp(skew[s+D-1]); y ^= x
// with log == modulus meaning "no multiply" (XOR only), exactly as the reference.
//
// MI355X design: GF(2^8) multiplication by a constant is GF(2)-linear, so the
// 32 bytes a lane owns are bit-sliced into 8 plane words (bit j of 32 bytes per
// word) and butterflies are whole-register XORs.  Two kernels:
//  * rs_encode8_g2_kernel (batched EDS path): 2 codewords per workgroup held in
//    registers, lane bit 0 = element index bit 0 (d = 0 butterflies over DPP lane
//    pairs), every other index bit a register or wave bit.  One body per wave
//    index, so every layer constant is a compile-time value and each multiply is a
//    fixed XOR3 program on the planes in Leopard's own (Cantor) coordinates
//    (gf8_const.h) -- full-rate v_xor / v_bitop3 only, no scalar branches.
//  * rs_encode8_kernel (single codewords / small k / odd shard lengths): state
//    in LDS, radix-2 layers, constant matrix applied with v_bitop3 masks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <vector>

#include "cda_internal.h"
#include "gf8_const.h"
#include "gf_slice.h"

namespace cda {

__constant__ uint16_t c_skew8[256];
__constant__ unsigned long long c_col8[256];

// LDS bank swizzle of the plane-major state of the LDS encoders ([plane][m*U] words, element e = x*U + u).  In a
// layer D the 32 lanes of a half-wave touch e with one bit fixed (bit log2(D*U)) and bits 0..5 otherwise free, so for
// D*U < 32 two lanes whose e differ in bit 5 only land in the same bank (2-way conflicts in every low layer).
// Flipping bits 0..4 when bit 5 is set separates them for any fixed bit, and keeps contiguous runs conflict-free.
__device__ __forceinline__ int lds_sw(int e) { return e ^ (((e >> 5) & 1) * 31); }

// x ^= M * y, M(j,b) = bit (8b+j) of cb
__device__ __forceinline__ void gf8_muladd(uint32_t x[8], const uint32_t y[8], unsigned long long cb) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t acc = x[j];
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint32_t mask = 0u - (uint32_t)((cb >> (8 * b + j)) & 1ull);
      acc = __builtin_amdgcn_bitop3_b32(acc, y[b], mask, 0x78);  // acc ^ (y & mask)
    }
    x[j] = acc;
  }
}

template <bool INVERSE>
__device__ __forceinline__ void butterfly8(uint32_t* st, int mU, int U, int x, int y, int u, unsigned log_m,
                                           unsigned long long cb) {
  uint32_t X[8], Y[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    X[j] = st[j * mU + lds_sw(x * U + u)];
    Y[j] = st[j * mU + lds_sw(y * U + u)];
  }
  if (INVERSE) {  // IFFT2
#pragma unroll
    for (int j = 0; j < 8; j++) Y[j] ^= X[j];
    if (log_m != 255u) gf8_muladd(X, Y, cb);
  } else {  // FFT2
    if (log_m != 255u) gf8_muladd(X, Y, cb);
#pragma unroll
    for (int j = 0; j < 8; j++) Y[j] ^= X[j];
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    st[j * mU + lds_sw(x * U + u)] = X[j];
    st[j * mU + lds_sw(y * U + u)] = Y[j];
  }
}

template <bool INVERSE>
__device__ __forceinline__ void rs_layer8(uint32_t* st, int m, int U, int log2U, int D, int log2D,
                                          const unsigned long long* s_cb) {
  const int nbu = (m >> 1) << log2U;
  for (int bu = threadIdx.x; bu < nbu; bu += blockDim.x) {
    const int p = bu >> log2U, u = bu & (U - 1);
    const int s0 = (p >> log2D) << (log2D + 1);
    const int x = s0 | (p & (D - 1));
    const int y = x + D;
    const int idx = INVERSE ? (m - 1 + s0 + D) : (s0 + D - 1);
    if (s_cb) {  // latency launches: the layer's matrix from the LDS copy (0 = no multiply)
      unsigned long long cb = s_cb[idx];
      if ((D << log2U) >= 64) {
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)cb);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(cb >> 32));
        cb = (unsigned long long)hi << 32 | lo;
      }
      butterfly8<INVERSE>(st, m << log2U, U, x, y, u, cb ? 0u : 255u, cb);
    } else if ((D << log2U) >= 64) {  // constant is wave-uniform: masks in SGPRs
      const int sidx = __builtin_amdgcn_readfirstlane(idx);
      const unsigned lm = c_skew8[sidx];
      butterfly8<INVERSE>(st, m << log2U, U, x, y, u, lm, c_col8[lm]);
    } else {
      const unsigned lm = c_skew8[idx];
      butterfly8<INVERSE>(st, m << log2U, U, x, y, u, lm, c_col8[lm]);
    }
  }
  __syncthreads();
}

struct Rs8Args {
  const uint8_t* src;
  long long src_blk, src_cw, src_sh;
  uint8_t* dst;
  long long dst_blk, dst_cw, dst_sh;
  uint8_t* cpy;
  long long cpy_blk, cpy_cw, cpy_sh;
  int k, m, log2m, cw_per_blk, U, log2U, slices;
  int lat;  // layer matrices staged in LDS at the start (small latency-bound launches; see launch_rs_encode8)
};

__global__ void __launch_bounds__(256) rs_encode8_kernel(Rs8Args a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t st[];  // [8][m][U] plane-major (conflict-free)
  const int U = a.U;
  int wg = blockIdx.x;
  const int slice = wg % a.slices;
  wg /= a.slices;
  const int cw = wg % a.cw_per_blk;
  const int blk = wg / a.cw_per_blk;
  const long long byte_off = (long long)slice * U * 32;
  const uint8_t* src = a.src + blk * a.src_blk + cw * a.src_cw + byte_off;
  uint8_t* dst = a.dst + blk * a.dst_blk + cw * a.dst_cw + byte_off;
  uint8_t* cpy = a.cpy ? a.cpy + blk * a.cpy_blk + cw * a.cpy_cw + byte_off : nullptr;

  // per-index layer matrices c_col8[c_skew8[i]] (0 = no multiply) after the state: a per-lane constant is then one
  // LDS read per layer instead of two dependent constant-memory loads
  unsigned long long* s_cb = nullptr;
  if (a.lat) {
    s_cb = reinterpret_cast<unsigned long long*>(st + 8 * (a.m << a.log2U));
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_cb[i] = c_col8[c_skew8[i]];
  }
  // load + bit-slice: element (s, u), s < m.  At most two elements per thread (the latency launches, whose shards may
  // sit in page-locked host memory read over PCIe): both loads are issued before either is used, one round trip.
  const int items = a.m << a.log2U;
  if (items <= 2 * (int)blockDim.x) {
    uint4 v[2][2];
#pragma unroll
    for (int it = 0; it < 2; it++) {
      const int e = threadIdx.x + it * blockDim.x, s = e >> a.log2U, u = e & (U - 1);
      if (e < items && s < a.k) {
        const uint4* p = reinterpret_cast<const uint4*>(src + s * a.src_sh + u * 32);
        v[it][0] = p[0];
        v[it][1] = p[1];
      }
    }
#pragma unroll
    for (int it = 0; it < 2; it++) {
      const int e = threadIdx.x + it * blockDim.x, s = e >> a.log2U, u = e & (U - 1);
      if (e >= items) continue;
      uint32_t w[8];
      if (s < a.k) {
        if (cpy) {
          uint4* q = reinterpret_cast<uint4*>(cpy + s * a.cpy_sh + u * 32);
          q[0] = v[it][0];
          q[1] = v[it][1];
        }
        w[0] = v[it][0].x; w[1] = v[it][0].y; w[2] = v[it][0].z; w[3] = v[it][0].w;
        w[4] = v[it][1].x; w[5] = v[it][1].y; w[6] = v[it][1].z; w[7] = v[it][1].w;
        bitslice8(w);
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = 0;
      }
#pragma unroll
      for (int j = 0; j < 8; j++) st[j * items + lds_sw(s * U + u)] = w[j];
    }
  }
  for (int e = threadIdx.x; items > 2 * (int)blockDim.x && e < items; e += blockDim.x) {
    const int s = e >> a.log2U, u = e & (U - 1);
    uint32_t w[8];
    if (s < a.k) {
      const uint4* p = reinterpret_cast<const uint4*>(src + s * a.src_sh + u * 32);
      uint4 v0 = p[0], v1 = p[1];
      if (cpy) {
        uint4* q = reinterpret_cast<uint4*>(cpy + s * a.cpy_sh + u * 32);
        q[0] = v0;
        q[1] = v1;
      }
      w[0] = v0.x; w[1] = v0.y; w[2] = v0.z; w[3] = v0.w;
      w[4] = v1.x; w[5] = v1.y; w[6] = v1.z; w[7] = v1.w;
      bitslice8(w);
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) w[j] = 0;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) st[j * (a.m << a.log2U) + lds_sw(s * U + u)] = w[j];
  }
  __syncthreads();
  // IFFT (data at points m..m+k-1), D = 1 .. m/2
  for (int lD = 0; lD < a.log2m; lD++) rs_layer8<true>(st, a.m, U, a.log2U, 1 << lD, lD, s_cb);
  // FFT to points 0..k-1, D = m/2 .. 1
  for (int lD = a.log2m - 1; lD >= 0; lD--) rs_layer8<false>(st, a.m, U, a.log2U, 1 << lD, lD, s_cb);
  // un-slice + store parity
  for (int e = threadIdx.x; e < (a.k << a.log2U); e += blockDim.x) {
    const int s = e >> a.log2U, u = e & (U - 1);
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = st[j * (a.m << a.log2U) + lds_sw(s * U + u)];
    bitslice8(w);
    uint4* q = reinterpret_cast<uint4*>(dst + s * a.dst_sh + u * 32);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

// ---- Leopard's field --------------------------------------------------------
// Leopard's byte e is the Cantor-basis coordinate vector of phi(e) in the standard field
// GF(2)[x]/(x^8+x^4+x^3+x^2+1), and exp(L) maps to alpha^L (alpha = x):
//   mul_leopard(a, b) = phi^-1(phi(a) * phi(b))      (checked in tests/test_oracle.py).
// The g2 encoder multiplies by compile-time constants only, so it works directly on
// Leopard's coordinates with each constant's matrix (gf8_const.h).

struct Rs8RegArgs {
  const uint8_t* src;
  long long src_blk, src_cw, src_sh;
  uint8_t* dst;
  long long dst_blk, dst_cw, dst_sh;
  uint8_t* cpy;
  long long cpy_blk, cpy_cw, cpy_sh;
  int k, groups_per_blk, slices;
  int remap;  // XCD-contiguous workgroup order
};

// ===========================================================================
// Two-codeword register encoder (default): 2 codewords x 16 units per workgroup,
// 8 elements per lane, so a workgroup holds 128 KiB of state and two
// workgroups fit on a CU (one streams HBM while the other computes).
//
// Lane l: index bit 0 of its elements = l&1 ("sw"), unit (l>>1)&15, codeword l>>5.
// Every other index bit
// is a register bit (3 per layout) or a wave bit, so for any layer d >= 1 the
// butterfly partner is in the same lane and the constant (a function of index
// bits > d) is fixed per wave.  Layer d = 0 pairs lanes l and l^1 (d0_w).
//   P1 f=1: IFFT d=0 (cross-lane), d=1..3 | exchange | P2 f=L-3: IFFT d=4..L-1,
//   FFT d=L-1..L-3 | exchange | P3 f=1: FFT d=min(3,L-4)..1, d=0 (cross-lane).
// ===========================================================================
__host__ __device__ constexpr int x2_of(int w, int sw, int r, int f) {
  // bits 1..L-1 of the element index: 3 register bits at (f..f+2), wave bits elsewhere
  const int y = ((w >> (f - 1)) << (f + 2)) | (r << (f - 1)) | (w & ((1 << (f - 1)) - 1));
  return (y << 1) | sw;
}

// P2 layers (register bits F..F+2 = the top three index bits, d >= F): every index bit above d is a register
// bit, so the constant of each butterfly is a compile-time value and the multiply is its GF(2) matrix
// (gf8_const.h) -- no scalar branches, about 18 VALU instead of ~45.
template <bool INVERSE, int M, int F, int D, int R>
__device__ __forceinline__ void bfly_const(uint32_t (&E)[8][8]) {
  static_assert(D >= F && F + 3 == __builtin_ctz(M), "P2 layout: index bits above d are register bits");
  constexpr int rb = D - F;
  if constexpr (!(R & (1 << rb))) {
    constexpr int s0 = ((R << F) >> (D + 1)) << (D + 1);
    constexpr int idx = INVERSE ? (M - 1 + s0 + (1 << D)) : (s0 + (1 << D) - 1);
    constexpr unsigned c = kCpoly8.v[idx];
    uint32_t(&X)[8] = E[R];
    uint32_t(&Y)[8] = E[R | (1 << rb)];
    if (INVERSE) {
#pragma unroll
      for (int j = 0; j < 8; j++) Y[j] ^= X[j];
    }
    if constexpr (c != 0u) gf8_muladd_cantor<c>(X, Y);
    if (!INVERSE) {
#pragma unroll
      for (int j = 0; j < 8; j++) Y[j] ^= X[j];
    }
  }
}

template <bool INVERSE, int M, int F, int D>
__device__ __forceinline__ void layer2_const(uint32_t (&E)[8][8]) {
  bfly_const<INVERSE, M, F, D, 0>(E);
  bfly_const<INVERSE, M, F, D, 1>(E);
  bfly_const<INVERSE, M, F, D, 2>(E);
  bfly_const<INVERSE, M, F, D, 3>(E);
  bfly_const<INVERSE, M, F, D, 4>(E);
  bfly_const<INVERSE, M, F, D, 5>(E);
  bfly_const<INVERSE, M, F, D, 6>(E);
  bfly_const<INVERSE, M, F, D, 7>(E);
}

// P2 of rs_g2_body: IFFT d = 4..L-1, then FFT d = L-1..F (F = L-3, d >= 1)
template <int L, int F, int D, bool INVERSE>
__device__ __forceinline__ void p2_layers(uint32_t (&E)[8][8]) {
  constexpr int M = 1 << L;
  if constexpr (INVERSE) {
    if constexpr (D < L) {
      layer2_const<true, M, F, D>(E);
      p2_layers<L, F, D + 1, true>(E);
    } else {
      p2_layers<L, F, L - 1, false>(E);
    }
  } else if constexpr (D >= F && D >= 1) {
    layer2_const<false, M, F, D>(E);
    p2_layers<L, F, D - 1, false>(E);
  }
}

// ---- P1 / P3 with compile-time constants ------------------------------------
// In the f = 1 layout the constants of layers d = 0..3 are functions of the register bits and of the wave
// index w (bits 4..L-1).  w is wave-uniform, so a scalar branch on it selects a copy of P1 / P3 specialised for
// that wave, where every constant is again a compile-time value (the XOR3 program of gf8_const.h, ~14 VALU,
// instead of ~45 VALU + scalar branches for a runtime constant).  Costs code size: 2^(L-4) kernel bodies.
template <bool INVERSE, unsigned C>
__device__ __forceinline__ void bfly_cc(uint32_t (&X)[8], uint32_t (&Y)[8]) {
  if (INVERSE) {
#pragma unroll
    for (int j = 0; j < 8; j++) Y[j] ^= X[j];
  }
  if constexpr (C != 0u) gf8_muladd_cantor<C>(X, Y);
  if (!INVERSE) {
#pragma unroll
    for (int j = 0; j < 8; j++) Y[j] ^= X[j];
  }
}

// layer d >= 1 of the f = 1 layout (register bit d - 1), wave W
template <bool INVERSE, int M, int W, int D, int R>
__device__ __forceinline__ void bfly_w(uint32_t (&E)[8][8]) {
  constexpr int rb = D - 1;
  if constexpr (!(R & (1 << rb))) {
    constexpr int x = x2_of(W, 0, R, 1);
    constexpr int s0 = (x >> (D + 1)) << (D + 1);
    constexpr int idx = INVERSE ? (M - 1 + s0 + (1 << D)) : (s0 + (1 << D) - 1);
    bfly_cc<INVERSE, kCpoly8.v[idx]>(E[R], E[R | (1 << rb)]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool INVERSE, int M, int W, int D>
__device__ __forceinline__ void layer_w(uint32_t (&E)[8][8]) {
  bfly_w<INVERSE, M, W, D, 0>(E);
  bfly_w<INVERSE, M, W, D, 1>(E);
  bfly_w<INVERSE, M, W, D, 2>(E);
  bfly_w<INVERSE, M, W, D, 3>(E);
  bfly_w<INVERSE, M, W, D, 4>(E);
  bfly_w<INVERSE, M, W, D, 5>(E);
  bfly_w<INVERSE, M, W, D, 6>(E);
  bfly_w<INVERSE, M, W, D, 7>(E);
}

// layer d = 0, wave W.  The element index bit 0 sits on lane bit 0, so a butterfly's two elements are in lanes 2i and 2i+1 and one DPP quad_perm read hands each lane its partner's plane,
// folded into the XOR.  Each lane computes only its own output; `lm` is all-ones in the x (even) lanes:
//   IFFT: T = x ^ y;  x' = x ^ c*T, y' = T                      (c*T computed wave-wide, kept in x lanes)
//   FFT:  S = y (own or partner), T = x ^ y;  x' = x ^ c*S, y' = T ^ c*S = (lm ? x : T) ^ c*S
// (Round 1 kept bit 0 on lane bit 5: two v_permlane32_swap + copies per plane, both halves computing the whole
// butterfly -- about twice the VALU of this form.)
__device__ __forceinline__ uint32_t lane_pair_xor(uint32_t v) {  // v ^ v[lane ^ 1]
  return v ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
}
// T[j] = E[j] ^ E[j][lane ^ 1] for 8 planes as one volatile block: with the intrinsic the compiler hoisted the DPP
// reads of all eight FFT d = 0 butterflies ahead of the first (64 extra live VGPRs, spills).  s_nop 1 covers the
// VALU-write -> DPP-read hazard (2 wait states) for inputs written just before the block.
__device__ __forceinline__ void lane_pair_xor8(uint32_t (&T)[8], const uint32_t (&E)[8]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_xor_b32_dpp %0, %8, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_xor_b32_dpp %1, %9, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_xor_b32_dpp %2, %10, %10 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_xor_b32_dpp %3, %11, %11 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_xor_b32_dpp %4, %12, %12 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_xor_b32_dpp %5, %13, %13 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_xor_b32_dpp %6, %14, %14 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_xor_b32_dpp %7, %15, %15 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
      : "=&v"(T[0]), "=&v"(T[1]), "=&v"(T[2]), "=&v"(T[3]), "=&v"(T[4]), "=&v"(T[5]), "=&v"(T[6]), "=&v"(T[7])
      : "v"(E[0]), "v"(E[1]), "v"(E[2]), "v"(E[3]), "v"(E[4]), "v"(E[5]), "v"(E[6]), "v"(E[7]));
}
template <bool INVERSE, int M, int W, int R>
__device__ __forceinline__ void d0_w(uint32_t (&E)[8][8], uint32_t lm) {
  constexpr int x = x2_of(W, 0, R, 1);
  constexpr unsigned c = kCpoly8.v[INVERSE ? (M - 1 + x + 1) : x];
  {
    uint32_t T[8];
    if constexpr (INVERSE) {
#pragma unroll
      for (int j = 0; j < 8; j++) T[j] = lane_pair_xor(E[R][j]);
    } else {
      lane_pair_xor8(T, E[R]);
    }
    if constexpr (INVERSE) {
      if constexpr (c != 0u) gf8_muladd_cantor<c>(E[R], T);
#pragma unroll
      for (int j = 0; j < 8; j++) E[R][j] = __builtin_amdgcn_bitop3_b32(lm, E[R][j], T[j], 0xCA);  // lm ? E : T
    } else {
      uint32_t S[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        S[j] = __builtin_amdgcn_bitop3_b32(E[R][j], T[j], lm, 0x78);       // E ^ (T & lm) = y
        E[R][j] = __builtin_amdgcn_bitop3_b32(lm, E[R][j], T[j], 0xCA);    // lm ? x : T
      }
      if constexpr (c != 0u) gf8_muladd_cantor<c>(E[R], S);
    }
    // pin the results here: otherwise the compiler sinks this arithmetic into the (conditional) store blocks
    // while the DPP reads stay put, and every butterfly's T / S stays live until the stores
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("" : "+v"(E[R][j]));
  }
  __builtin_amdgcn_sched_barrier(0);  // one butterfly's temporaries live at a time
}

template <bool INVERSE, int M, int W>
__device__ __forceinline__ void layer_d0_w(uint32_t (&E)[8][8], uint32_t lm) {
  d0_w<INVERSE, M, W, 0>(E, lm);
  d0_w<INVERSE, M, W, 1>(E, lm);
  d0_w<INVERSE, M, W, 2>(E, lm);
  d0_w<INVERSE, M, W, 3>(E, lm);
  d0_w<INVERSE, M, W, 4>(E, lm);
  d0_w<INVERSE, M, W, 5>(E, lm);
  d0_w<INVERSE, M, W, 6>(E, lm);
  d0_w<INVERSE, M, W, 7>(E, lm);
}

// P1: IFFT d = 0..min(3, L-1); P3: FFT d = min(F2-1, 3)..1, then d = 0
template <int L, int W>
__device__ __forceinline__ void p1_w(uint32_t (&E)[8][8], uint32_t lm) {
  constexpr int M = 1 << L;
  layer_d0_w<true, M, W>(E, lm);
  layer_w<true, M, W, 1>(E);
  if constexpr (L > 2) layer_w<true, M, W, 2>(E);
  if constexpr (L > 3) layer_w<true, M, W, 3>(E);
}

template <int L, int W>
__device__ __forceinline__ void p3_w(uint32_t (&E)[8][8], uint32_t lm) {
  constexpr int M = 1 << L, F2 = L - 3;
  if constexpr (F2 - 1 >= 3) layer_w<false, M, W, 3>(E);
  if constexpr (F2 - 1 >= 2) layer_w<false, M, W, 2>(E);
  if constexpr (F2 - 1 >= 1) layer_w<false, M, W, 1>(E);
  layer_d0_w<false, M, W>(E, lm);
}

// LDS exchange of the 8 x 8 register state between layouts (two halves of 4 planes).
template <int M>
__device__ __forceinline__ void exchange2(uint32_t (&E)[8][8], uint4* xbuf, int w, int sw, int li, int f_from,
                                          int f_to) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int x = x2_of(w, sw, r, f_from);
      xbuf[x * 32 + li] = make_uint4(E[r][4 * h], E[r][4 * h + 1], E[r][4 * h + 2], E[r][4 * h + 3]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int x = x2_of(w, sw, r, f_to);
      const uint4 v = xbuf[x * 32 + li];
      E[r][4 * h] = v.x;
      E[r][4 * h + 1] = v.y;
      E[r][4 * h + 2] = v.z;
      E[r][4 * h + 3] = v.w;
    }
    __syncthreads();
  }
}

// Work of workgroup `wg` (blockDim = 64 << (L - 4)) for its wave WC (== w); xbuf = [M][32] x 16 B LDS (L > 4).
template <int L, int WC>
__device__ __forceinline__ void rs_g2_impl(const Rs8RegArgs& a, int wg, uint4* xbuf, int w) {
  constexpr int M = 1 << L;
  const int lane = threadIdx.x & 63;
  // lane = (li, sw): sw = element index bit 0 (DPP pairs), li = unit u (16) and codeword cwi (2)
  const int sw = lane & 1, li = lane >> 1;
  const int u = li & 15, cwi = li >> 4;
  uint32_t lm = sw ? 0u : ~0u;  // x lanes of the d = 0 butterflies
  asm volatile("" : "+v"(lm));
  const int slice = wg % a.slices;
  wg /= a.slices;
  const int grp = wg % a.groups_per_blk;
  const int blk = wg / a.groups_per_blk;
  const int cw = grp * 2 + cwi;
  // lane u owns bytes [16u, 16u+16) and [256+16u, 256+16u+16) of each 512-B share: every 16-B load or
  // store instruction of the wave covers whole 256-B runs (the bit-slice is byte-position agnostic, so
  // any fixed byte->lane map works as long as load and store agree)
  const long long off = (long long)slice * 512 + u * 16;
  const uint8_t* src = a.src + blk * a.src_blk + cw * a.src_cw + off;
  uint8_t* dst = a.dst + blk * a.dst_blk + cw * a.dst_cw + off;
  uint8_t* cpy = a.cpy ? a.cpy + blk * a.cpy_blk + cw * a.cpy_cw + off : nullptr;

  uint32_t E[8][8];
  const SliceMasks km = slice_masks();
  constexpr int wv = WC;
#pragma unroll
  for (int r = 0; r < 8; r++) {
    // x0 (the pair's even element) is wave-uniform and, k being even on this path, x < k iff x0 < k: the branch is
    // scalar, so no lane-divergent control flow surrounds the cross-lane butterflies
    const int x = x2_of(wv, sw, r, 1), x0 = x2_of(wv, 0, r, 1);
    if (x0 < a.k) {
      const uint4* p = reinterpret_cast<const uint4*>(src + x * a.src_sh);
      const uint4 v0 = p[0], v1 = p[16];
      if (cpy) {
        uint4* q = reinterpret_cast<uint4*>(cpy + x * a.cpy_sh);
        q[0] = v0;
        q[16] = v1;
      }
      E[r][0] = v0.x; E[r][1] = v0.y; E[r][2] = v0.z; E[r][3] = v0.w;
      E[r][4] = v1.x; E[r][5] = v1.y; E[r][6] = v1.z; E[r][7] = v1.w;
      bitslice8(E[r], km);
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) E[r][j] = 0;
    }
  }
  constexpr int F2 = L - 3;  // P2 register bits F2..F2+2 = L-3..L-1
#ifndef CDA_RS8_DIAG_NOCOMPUTE  // diagnostic build (scripts/rs8_diag.sh): loads and stores only
  // P1 (f=1): IFFT d=0 (cross-lane), d=1..3 (or up to L-1 when L == 4)
  p1_w<L, WC>(E, lm);
  if (L > 4) exchange2<M>(E, xbuf, WC, sw, li, 1, F2);
  // P2: IFFT d=4..L-1, FFT d=L-1..F2 (compile-time constants)
  p2_layers<L, (F2 > 1 ? F2 : 1), 4, true>(E);
  if (L > 4) exchange2<M>(E, xbuf, WC, sw, li, F2, 1);
  // P3 (f=1): FFT d=F2-1..1, then d=0 (cross-lane)
  p3_w<L, WC>(E, lm);
#else
  (void)lm;
  (void)F2;
#endif
  const SliceMasks ko = slice_masks();
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int x = x2_of(wv, sw, r, 1), x0 = x2_of(wv, 0, r, 1);
    if (x0 < a.k) {  // wave-uniform, as at the load
      uint32_t v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = E[r][j];
      bitslice8(v, ko);
      uint4* q = reinterpret_cast<uint4*>(dst + x * a.dst_sh);
      q[0] = make_uint4(v[0], v[1], v[2], v[3]);
      q[16] = make_uint4(v[4], v[5], v[6], v[7]);
    }
  }
}

// scalar dispatch on the wave index (w is an SGPR value): one whole body per wave index, so that no
// control-flow merge with the 64 live state registers follows the specialised phases (a merge after
// P1 or P3 alone made the register allocator spill)
template <int L, int W>
__device__ __forceinline__ void rs_g2_select(const Rs8RegArgs& a, int wg, uint4* xbuf, int w) {
  if constexpr (W < (1 << (L - 4))) {
    if (w == W)
      rs_g2_impl<L, W>(a, wg, xbuf, w);
    else
      rs_g2_select<L, W + 1>(a, wg, xbuf, w);
  }
}

template <int L>
__device__ __forceinline__ void rs_g2_body(const Rs8RegArgs& a, int wg, uint4* xbuf) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & ((1 << (L - 4)) - 1);
  rs_g2_select<L, 0>(a, wg, xbuf, w);
}

template <int L>
__global__ void __launch_bounds__(64 << (L - 4), 4) rs_encode8_g2_kernel(Rs8RegArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 xbuf[];
  // XCD-contiguous work (a.remap): the dispatcher deals workgroups to the 8 XCDs round-robin, so XCD x runs blocks
  // x, x + 8, ...; map them to one contiguous range of codeword pairs per XCD
  const unsigned g = gridDim.x, b = blockIdx.x;
  const int wg = (a.remap && (g % 8u) == 0) ? (int)((b % 8u) * (g / 8u) + b / 8u) : (int)b;
  // (static issue priority, s_setprio 1, for the second half of the waves: columns 0.857 vs 0.839 ms per B = 128
  // step in a rotating same-box A/B, profiles/r05_prio_ab.log; not kept)
  rs_g2_body<L>(a, wg, xbuf);
}

static Rs8RegArgs reg_args(const RsJob& j);

int rs_init_device_tables(int device) {
  (void)device;
  const LeoTables& t = leo_tables(8);
  uint16_t skew[256];
  unsigned long long col[256];
  for (int i = 0; i < 255; i++) skew[i] = t.skew[i];
  skew[255] = 255;
  for (unsigned l = 0; l < 256; l++) col[l] = leo8_colbits(l);
  if (hipMemcpyToSymbol(HIP_SYMBOL(c_skew8), skew, sizeof skew) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(c_col8), col, sizeof col) != hipSuccess) return -1;
  // alpha^L in the standard basis (LFSR of x^8+x^4+x^3+x^2+1), per skew index
  uint8_t apow[255];
  unsigned st = 1;
  for (int i = 0; i < 255; i++) {
    apow[i] = (uint8_t)st;
    st <<= 1;
    if (st & 0x100) st ^= 0x11D;
  }
  uint8_t cpoly[256];
  for (int i = 0; i < 256; i++) cpoly[i] = skew[i] >= 255 ? 0 : apow[skew[i]];
  for (int i = 0; i < 256; i++)
    if (cpoly[i] != kCpoly8.v[i]) return -1;  // the encoder's compile-time constants (gf8_const.h)
  if (hipFuncSetAttribute((const void*)rs_encode8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024) !=
      hipSuccess)
    return -1;
  const void* g2k[4] = {(const void*)rs_encode8_g2_kernel<4>, (const void*)rs_encode8_g2_kernel<5>,
                        (const void*)rs_encode8_g2_kernel<6>, (const void*)rs_encode8_g2_kernel<7>};
  for (auto f : g2k)
    if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) != hipSuccess) return -1;

  return 0;
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) l++;
  return l;
}

static Rs8RegArgs reg_args(const RsJob& j) {
  Rs8RegArgs r{};
  r.src = j.src;
  r.src_blk = j.src_blk;
  r.src_cw = j.src_cw;
  r.src_sh = j.src_sh;
  r.dst = j.dst;
  r.dst_blk = j.dst_blk;
  r.dst_cw = j.dst_cw;
  r.dst_sh = j.dst_sh;
  r.cpy = j.cpy;
  r.cpy_blk = j.cpy_blk;
  r.cpy_cw = j.cpy_cw;
  r.cpy_sh = j.cpy_sh;
  r.k = j.k;
  r.groups_per_blk = j.cw_per_blk / 2;
  r.slices = j.shard_len / 512;
  // XCD-contiguous order for the row pass only (positions contiguous): rows 0.599 -> 0.580 ms per B = 128 step; the
  // column pass got slower with it (0.826 -> 0.877 ms), scripts/env_ab_bench.sh, round 3
  r.remap = j.src_sh == j.shard_len;
  return r;
}

int launch_rs_encode8(const RsJob& j, hipStream_t s) {
  if (j.k < 1 || j.k > 128 || j.shard_len % 64 != 0) return -2;
  const int L = ilog2(j.k);
  // Latency launches: when the register encoder's grid would leave most CUs idle (one block: 64 / 128 workgroups
  // for rows / columns at k = 128, a consensus band 16), the LDS encoder splits each codeword's bytes over
  // workgroups of U units (32 B each) instead, so the pass spreads over the chip.  CDA_RS8_LAT_U picks U
  // (0 = off; default 4); results are identical either way (both encoders are bit-exact).
  static const int lat_u = [] {
    const char* e = CDA_AB_ENV("CDA_RS8_LAT_U");
    const int v = e ? atoi(e) : 4;
    return (v == 1 || v == 2 || v == 4 || v == 8 || v == 16) ? v : 0;
  }();
  const long long g2_grid = (long long)j.nblk * (j.cw_per_blk / 2) * (j.shard_len / 512);
  const bool lat = lat_u && L >= 4 && j.shard_len % (32 * lat_u) == 0 && g2_grid < 32;
  // Batched path: 2 codewords per workgroup, register-resident (k >= 16).
  if (!lat && L >= 4 && j.k % 2 == 0 && j.cw_per_blk % 2 == 0 && j.shard_len % 512 == 0) {
    const Rs8RegArgs r = reg_args(j);
    const long long grid = (long long)j.nblk * r.groups_per_blk * r.slices;
    if (grid <= 0 || grid > 0x7FFFFFFF) return -2;
    const size_t lds = L > 4 ? (size_t)(1 << L) * 32 * 16 : 0;
    const dim3 block(64 << (L - 4));
    switch (L) {
      case 4: hipLaunchKernelGGL(rs_encode8_g2_kernel<4>, dim3((unsigned)grid), block, lds, s, r); break;
      case 5: hipLaunchKernelGGL(rs_encode8_g2_kernel<5>, dim3((unsigned)grid), block, lds, s, r); break;
      case 6: hipLaunchKernelGGL(rs_encode8_g2_kernel<6>, dim3((unsigned)grid), block, lds, s, r); break;
      default: hipLaunchKernelGGL(rs_encode8_g2_kernel<7>, dim3((unsigned)grid), block, lds, s, r); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  // General path (any k <= 128, any shard length, single codewords): LDS-resident.
  Rs8Args a;
  a.src = j.src;
  a.src_blk = j.src_blk;
  a.src_cw = j.src_cw;
  a.src_sh = j.src_sh;
  a.dst = j.dst;
  a.dst_blk = j.dst_blk;
  a.dst_cw = j.dst_cw;
  a.dst_sh = j.dst_sh;
  a.cpy = j.cpy;
  a.cpy_blk = j.cpy_blk;
  a.cpy_cw = j.cpy_cw;
  a.cpy_sh = j.cpy_sh;
  a.k = j.k;
  a.log2m = L;
  a.m = 1 << L;
  a.cw_per_blk = j.cw_per_blk;
  const int units = j.shard_len / 32;  // even
  int U = lat ? lat_u : 16;
  while (units % U) U >>= 1;
  a.U = U;
  a.log2U = ilog2(U);
  a.slices = units / U;
  a.lat = lat ? 1 : 0;
  const size_t lds = (size_t)a.m * 8 * U * 4 + (lat ? 256 * 8 : 0);
  const long long grid = (long long)j.nblk * j.cw_per_blk * a.slices;
  if (grid <= 0 || grid > 0x7FFFFFFF) return -2;
  hipLaunchKernelGGL(rs_encode8_kernel, dim3((unsigned)grid), dim3(256), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ===========================================================================
// GF(2^16) encoder (klauspost leopardFF16 as selected for 2k > 256).
// Element t of every 64-byte block = byte[t] | byte[t+32] << 8; a lane's unit is
// one 64-byte block = 32 elements = 16 bit-planes (lo bytes -> planes 0..7, hi
// bytes -> planes 8..15).  State for one codeword x U units lives in LDS as
// [16][m][U] words (plane-major: the elements a wave touches in one plane are
// contiguous, so LDS accesses are conflict-free); radix-2 layers as in FF8.  Multiplication in the
// standard basis of GF(2)[x]/(x^16+x^5+x^3+x^2+1) (phi16 below), constant per
// lane: masks from the constant's bits, or wave-uniform branches when all lanes
// of the wave share the butterfly group (D*U >= 64).
// ===========================================================================
constexpr uint16_t kPhi16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                 0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
constexpr uint16_t kPhiInv16[16] = {0x0001, 0x4690, 0x65D8, 0x62D0, 0x5734, 0x45F0, 0x53B8, 0x1E38,
                                    0x7CAE, 0x4E38, 0x6708, 0xC25C, 0x7A64, 0x9EAC, 0x1124, 0x523A};

__device__ __forceinline__ void apply16(uint32_t (&v)[16], const uint16_t (&cols)[16]) {
  uint32_t o[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((cols[j] >> i) & 1) acc ^= v[j];
    o[i] = acc;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = o[i];
}

__device__ __forceinline__ void xtime16(uint32_t (&T)[16]) {  // T *= x; x^16 = x^5 + x^3 + x^2 + 1
  const uint32_t t = T[15];
#pragma unroll
  for (int i = 15; i > 0; i--) T[i] = T[i - 1];
  T[0] = t;
  T[2] ^= t;
  T[3] ^= t;
  T[5] ^= t;
}

// X ^= c*Y, c wave-uniform (branches on its bits)
__device__ __forceinline__ void gf16_muladd_uniform(uint32_t (&X)[16], const uint32_t (&Y)[16], unsigned c) {
  uint32_t T[16];
#pragma unroll
  for (int j = 0; j < 16; j++) T[j] = Y[j];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    if (c & (1u << i)) {
#pragma unroll
      for (int j = 0; j < 16; j++) X[j] ^= T[j];
    }
    if (i < 15) xtime16(T);
  }
}

// X ^= c*Y, c per lane (masks)
__device__ __forceinline__ void gf16_muladd_lane(uint32_t (&X)[16], const uint32_t (&Y)[16], unsigned c) {
  uint32_t T[16];
#pragma unroll
  for (int j = 0; j < 16; j++) T[j] = Y[j];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t mk = 0u - ((c >> i) & 1u);
#pragma unroll
    for (int j = 0; j < 16; j++) X[j] = __builtin_amdgcn_bitop3_b32(X[j], T[j], mk, 0x78);
    if (i < 15) xtime16(T);
  }
}

template <bool INVERSE, bool UNIFORM>
__device__ __forceinline__ void butterfly16(uint32_t* st, int mU, int U, int x, int y, int u, unsigned c) {
  uint32_t X[16], Y[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    X[j] = st[j * mU + lds_sw(x * U + u)];
    Y[j] = st[j * mU + lds_sw(y * U + u)];
  }
  if (INVERSE) {
#pragma unroll
    for (int j = 0; j < 16; j++) Y[j] ^= X[j];
  }
  if (UNIFORM) {
    if (c != 0u) gf16_muladd_uniform(X, Y, c);
  } else {
    gf16_muladd_lane(X, Y, c);
  }
  if (!INVERSE) {
#pragma unroll
    for (int j = 0; j < 16; j++) Y[j] ^= X[j];
  }
#pragma unroll
  for (int j = 0; j < 16; j++) {
    st[j * mU + lds_sw(x * U + u)] = X[j];
    st[j * mU + lds_sw(y * U + u)] = Y[j];
  }
}

struct Rs16Args {
  const uint8_t* src;
  long long src_blk, src_cw, src_sh;
  uint8_t* dst;
  long long dst_blk, dst_cw, dst_sh;
  uint8_t* cpy;
  long long cpy_blk, cpy_cw, cpy_sh;
  const uint16_t* cpoly;  // [65536] per skew index: alpha^skew in std basis (0 = no multiply)
  int k, m, log2m, cw_per_blk, U, log2U, slices;
  int lat;  // layer matrices staged in LDS at the start (small latency-bound launches; see launch_rs_encode8)
};

template <bool INVERSE>
__device__ __forceinline__ void rs_layer16(uint32_t* st, const Rs16Args& a, int D, int log2D) {
  const int U = a.U;
  const int nbu = (a.m >> 1) << a.log2U;
  for (int bu = threadIdx.x; bu < nbu; bu += blockDim.x) {
    const int p = bu >> a.log2U, u = bu & (U - 1);
    const int s0 = (p >> log2D) << (log2D + 1);
    const int x = s0 | (p & (D - 1));
    const int y = x + D;
    const int idx = INVERSE ? (a.m - 1 + s0 + D) : (s0 + D - 1);
    if ((D << a.log2U) >= 64) {
      const int sidx = __builtin_amdgcn_readfirstlane(idx);
      butterfly16<INVERSE, true>(st, a.m << a.log2U, U, x, y, u, a.cpoly[sidx]);
    } else {
      butterfly16<INVERSE, false>(st, a.m << a.log2U, U, x, y, u, a.cpoly[idx]);
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) rs_encode16_kernel(Rs16Args a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t st[];  // [16][m][U]
  const int U = a.U, mU = a.m << a.log2U;
  int wg = blockIdx.x;
  const int slice = wg % a.slices;
  wg /= a.slices;
  const int cw = wg % a.cw_per_blk;
  const int blk = wg / a.cw_per_blk;
  const long long byte_off = (long long)slice * U * 64;
  const uint8_t* src = a.src + blk * a.src_blk + cw * a.src_cw + byte_off;
  uint8_t* dst = a.dst + blk * a.dst_blk + cw * a.dst_cw + byte_off;
  uint8_t* cpy = a.cpy ? a.cpy + blk * a.cpy_blk + cw * a.cpy_cw + byte_off : nullptr;
  for (int e = threadIdx.x; e < (a.m << a.log2U); e += blockDim.x) {
    const int s = e >> a.log2U, u = e & (U - 1);
    uint32_t v[16];
    if (s < a.k) {
      const uint4* p = reinterpret_cast<const uint4*>(src + (long long)s * a.src_sh + u * 64);
      uint4 q[4] = {p[0], p[1], p[2], p[3]};
      if (cpy) {
        uint4* o = reinterpret_cast<uint4*>(cpy + (long long)s * a.cpy_sh + u * 64);
#pragma unroll
        for (int i = 0; i < 4; i++) o[i] = q[i];
      }
      uint32_t lo[8] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w};
      uint32_t hi[8] = {q[2].x, q[2].y, q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w};
      bitslice8(lo);
      bitslice8(hi);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        v[j] = lo[j];
        v[8 + j] = hi[j];
      }
      apply16(v, kPhi16);
    } else {
#pragma unroll
      for (int j = 0; j < 16; j++) v[j] = 0;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) st[j * mU + lds_sw(s * U + u)] = v[j];
  }
  __syncthreads();
  for (int lD = 0; lD < a.log2m; lD++) rs_layer16<true>(st, a, 1 << lD, lD);
  for (int lD = a.log2m - 1; lD >= 0; lD--) rs_layer16<false>(st, a, 1 << lD, lD);
  for (int e = threadIdx.x; e < (a.k << a.log2U); e += blockDim.x) {
    const int s = e >> a.log2U, u = e & (U - 1);
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = st[j * mU + lds_sw(s * U + u)];
    apply16(v, kPhiInv16);
    uint32_t lo[8], hi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      lo[j] = v[j];
      hi[j] = v[8 + j];
    }
    bitslice8(lo);
    bitslice8(hi);
    uint4* o = reinterpret_cast<uint4*>(dst + (long long)s * a.dst_sh + u * 64);
    o[0] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    o[1] = make_uint4(lo[4], lo[5], lo[6], lo[7]);
    o[2] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    o[3] = make_uint4(hi[4], hi[5], hi[6], hi[7]);
  }
}

static uint16_t* g_cpoly16[64] = {nullptr};

int rs16_init_device_tables(int device) {
  if (device < 0 || device >= 64) return -1;
  if (g_cpoly16[device]) return 0;
  const LeoTables& t = leo_tables(16);
  std::vector<uint16_t> apow(65535), cpoly(65536);
  unsigned st = 1;
  for (int i = 0; i < 65535; i++) {
    apow[i] = (uint16_t)st;
    st <<= 1;
    if (st & 0x10000) st ^= 0x1002D;
  }
  for (int i = 0; i < 65535; i++) cpoly[i] = t.skew[i] >= 65535 ? 0 : apow[t.skew[i]];
  cpoly[65535] = 0;
  void* d = nullptr;
  if (hipMalloc(&d, 65536 * 2) != hipSuccess) return -1;
  if (hipMemcpy(d, cpoly.data(), 65536 * 2, hipMemcpyHostToDevice) != hipSuccess) return -1;
  if (hipFuncSetAttribute((const void*)rs_encode16_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024) !=
      hipSuccess)
    return -1;
  if (rs16_reg_init(device)) return -1;
  g_cpoly16[device] = (uint16_t*)d;
  return 0;
}

const char* rs8_diag_tag() {
#ifdef CDA_RS8_DIAG_NOCOMPUTE
  return "rs8_nocompute";
#else
  return "";
#endif
}

int launch_rs_encode16(const RsJob& j, hipStream_t s) {
  if (j.k < 1 || j.k > 32768 || j.shard_len % 64 != 0) return -2;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64 || !g_cpoly16[dev]) return -1;
  // k = 512 codewords of whole 512-B shards: the register-resident encoder (rs16_kernels.hip); CDA_RS16=lds forces
  // this LDS encoder (same bytes) for A/B runs
  static const bool force_lds = [] {
    const char* e = CDA_AB_ENV("CDA_RS16");
    return e && e[0] == 'l';
  }();
  if (!force_lds && rs16_reg_eligible(j)) return launch_rs_encode16_reg(j, g_cpoly16[dev], s);
  Rs16Args a;
  a.src = j.src;
  a.src_blk = j.src_blk;
  a.src_cw = j.src_cw;
  a.src_sh = j.src_sh;
  a.dst = j.dst;
  a.dst_blk = j.dst_blk;
  a.dst_cw = j.dst_cw;
  a.dst_sh = j.dst_sh;
  a.cpy = j.cpy;
  a.cpy_blk = j.cpy_blk;
  a.cpy_cw = j.cpy_cw;
  a.cpy_sh = j.cpy_sh;
  a.cpoly = g_cpoly16[dev];
  a.k = j.k;
  a.log2m = ilog2(j.k);
  a.m = 1 << a.log2m;
  a.cw_per_blk = j.cw_per_blk;
  const int units = j.shard_len / 64;
  // LDS per workgroup: m * 64 B per unit column.  The budget sets the occupancy (LDS-bound: 160 KiB per CU)
  // against how many layers have wave-uniform constants (D * U >= 64).  Measured at k = 512 (m = 512):
  // 32 KiB (U = 1, 5 workgroups per CU) rows 0.47 + cols 0.83 ms per 2 squares, 64 KiB (U = 2) 0.56 + 1.03,
  // 128 KiB 0.83 + 1.55 -- occupancy wins over the extra lane-masked layers.
  static const size_t budget = [] {
    const char* e = CDA_AB_ENV("CDA_RS16_LDS_KB");
    return (size_t)(e ? atoi(e) : 32) * 1024;
  }();
  int U = 8;
  while (U > 1 && ((size_t)a.m * 64 * U > budget || units % U)) U >>= 1;
  if ((size_t)a.m * 64 * U > 128 * 1024) return -2;  // m > 2048: not on the device path yet
  a.U = U;
  a.log2U = ilog2(U);
  a.slices = units / U;
  const size_t lds = (size_t)a.m * 16 * U * 4;
  const long long grid = (long long)j.nblk * j.cw_per_blk * a.slices;
  if (grid <= 0 || grid > 0x7FFFFFFF) return -2;
  hipLaunchKernelGGL(rs_encode16_kernel, dim3((unsigned)grid), dim3(256), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cda
