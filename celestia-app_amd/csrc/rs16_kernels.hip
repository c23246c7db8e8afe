// rs16_kernels.hip — register-resident Leopard GF(2^16) encoder for m = 512 (k = 512, config C5: the testground
// square, pkg/appconsts/testground/app_consts.go:8).
//
// Reference: klauspost/reedsolomon v1.12.1 leopardFF16 encode as called by rsmt2d LeoRSCodec for 2k > 256
// (upstream, pinned go.mod:153): work = data at points m..2m-1; IFFT-DIT with
// skew[m - 1 + s0 + D], then FFT-DIT with skew[s0 + D - 1]; radix-2 layers d = log2 D (rs_kernels.hip header).
//
// Design.  One workgroup holds ONE whole codeword in registers: 512 positions x 512-B shards = 256 KiB = 16 waves x
// 64 lanes x 64 VGPRs.  A lane owns one 64-B unit of 4 positions (unit = 32 GF(2^16) elements bit-sliced into 16
// plane words, standard polynomial basis of GF(2)[x]/(x^16+x^5+x^3+x^2+1), as the LDS encoder):
//   lane bits 0..2 = unit u (32 whole elements of every shard: 8 lanes cover a 512-B shard; see pair_in),
//   lane bits 3, 4, 5 = three position bits (A3, A4, A5), register slot bits R0, R1 = two position bits,
//   wave bits W0..W3 = four position bits.
// A layer's butterfly bit is always moved into a register slot, so every butterfly is two register sets of one
// lane.  The layouts (position bit p0..p8 -> slot) and the moves between them:
//   LA  p0:R0 p1:R1 p2:A5 p3:A4 p4:A3 p5..p8:W0..W3   IFFT d = 0, 1          (load)  / FFT d = 1, 0   (store)
//   LB  p2:R0 p3:R1 p0:A5 p1:A4                        IFFT d = 2             / FFT d = 2
//       (LA <-> LB: v_permlane32_swap / v_permlane16_swap, one instruction per register pair and plane)
//   LC  p4:R0 p3:R1 p2:A3                              IFFT d = 3, 4          / FFT d = 4, 3
//       (LB <-> LC: DPP row_ror:8 = lane ^ 8, and two v_bitop3 selects)
//   LD  p5:R0 p6:R1 p4:W0 p3:W1                        IFFT d = 5, 6          / FFT d = 6, 5
//   LE  p7:R0 p8:R1 p5:W2 p6:W3                        IFFT d = 7, 8, FFT d = 8, 7
//       (LC <-> LD <-> LE: register bits <-> wave bits through LDS, 2 rounds of 8 planes, 128 KiB)
// A layer constant depends on the position bits above d.  When they all sit in registers it is a compile-time
// value and the multiply is its 16x16 GF(2) matrix as a straight v_bitop3 XOR3 program (~64 VALU); when several
// sit in lane bits (d <= 1) it is per lane (16 lane masks x 16 planes, v_bitop3).  The old LDS encoder paid the
// per-lane form on 12 of 18 layers and one LDS round trip + barrier per layer; here 4 of 18 layers are per-lane and
// the state crosses LDS 4 times.
//
// Wave bits W1..W3 are made compile-time by running one kernel body per value (8 bodies, scalar branch at entry), so
// layers 5..8 (LD, LE) multiply by compile-time constants.  The other runtime bits above a layer (W0 in LC; lane bit
// 3 at layer 2 in LB) are split off: Leopard's skews are GF(2)-affine in the position bits (FFTSkew[j + 2^(i+1)] =
// FFTSkew[j] ^ temp[i] in FFTInitialize; checked for every layer in tests/test_rs16_affine.py), so such a constant
// is c_ct ^ sum(b_i * t_i) with c_ct, t_i compile-time: one XOR program plus one more per set runtime bit
// (exec-masked for wave bits, lane-masked for the lane bit), no per-bit scalar branches.
//
// Persistent: one workgroup per CU walks codewords blockIdx.x, + gridDim.x, ...; after the last LDS exchange of a
// codeword each wave streams half of its share of the next codeword into the idle exchange buffer (global_load_lds).
// DESIGN.md §6 has the measured steps.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "cda_internal.h"
#include "gf16_const.h"
#include "gf_slice.h"

namespace cda {

namespace r16 {

constexpr int L = 9, M = 1 << L;

// ---- compile-time GF(2^16) matrices -------------------------------------------------------------------------------
constexpr unsigned xtime16c(unsigned v) {
  v <<= 1;
  return (v & 0x10000u) ? (v ^ 0x1002Du) : v;
}
// row i of the matrix of y -> c*y: bit j = bit i of c * x^j
constexpr unsigned mul_row(unsigned c, int i) {
  unsigned row = 0, col = c;
  for (int j = 0; j < 16; j++) {
    row |= ((col >> i) & 1u) << j;
    col = xtime16c(col);
  }
  return row;
}
// row i of a basis-change matrix given by its columns
constexpr uint16_t kPhi[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                               0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
constexpr uint16_t kPhiInv[16] = {0x0001, 0x4690, 0x65D8, 0x62D0, 0x5734, 0x45F0, 0x53B8, 0x1E38,
                                  0x7CAE, 0x4E38, 0x6708, 0xC25C, 0x7A64, 0x9EAC, 0x1124, 0x523A};
template <bool INV>
constexpr unsigned basis_row(int i) {
  unsigned row = 0;
  for (int j = 0; j < 16; j++) row |= (unsigned)(((INV ? kPhiInv[j] : kPhi[j]) >> i) & 1u) << j;
  return row;
}

// acc ^ XOR of Y[j] for the set bits j of ROW, two terms per v_bitop3 (XOR3)
template <unsigned ROW, int J, int PEND>
__device__ __forceinline__ uint32_t fold_row(uint32_t acc, const uint32_t (&Y)[16]) {
  if constexpr (J == 16) {
    if constexpr (PEND >= 0)
      return acc ^ Y[PEND];
    else
      return acc;
  } else if constexpr (((ROW >> J) & 1u) != 0) {
    if constexpr (PEND < 0)
      return fold_row<ROW, J + 1, J>(acc, Y);
    else
      return fold_row<ROW, J + 1, -1>(__builtin_amdgcn_bitop3_b32(acc, Y[PEND], Y[J], 0x96), Y);
  } else {
    return fold_row<ROW, J + 1, PEND>(acc, Y);
  }
}
// X ^= C * Y, C a compile-time constant (0 = nothing)
template <unsigned C, int I = 0>
__device__ __forceinline__ void muladd_const(uint32_t (&X)[16], const uint32_t (&Y)[16]) {
  if constexpr (C != 0 && I < 16) {
    X[I] = fold_row<mul_row(C, I), 0, -1>(X[I], Y);
    muladd_const<C, I + 1>(X, Y);
  }
}
// V = Phi * V (INV = false: Leopard's Cantor coordinates -> standard basis; true: back)
template <bool INV, int I = 0>
__device__ __forceinline__ void basis_rows(uint32_t (&O)[16], const uint32_t (&V)[16]) {
  if constexpr (I < 16) {
    O[I] = fold_row<basis_row<INV>(I), 0, -1>(0u, V);
    basis_rows<INV, I + 1>(O, V);
  }
}
template <bool INV>
__device__ __forceinline__ void change_basis(uint32_t (&V)[16]) {
  uint32_t O[16];
  basis_rows<INV>(O, V);
#pragma unroll
  for (int i = 0; i < 16; i++) V[i] = O[i];
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
// X ^= c * Y, c per lane (16 lane masks)
__device__ __forceinline__ void muladd_lane(uint32_t (&X)[16], const uint32_t (&Y)[16], unsigned c) {
  uint32_t T[16];
#pragma unroll
  for (int j = 0; j < 16; j++) T[j] = Y[j];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t mk = (uint32_t)__builtin_amdgcn_sbfe(c, i, 1);  // -1 if bit i of c, else 0
#pragma unroll
    for (int j = 0; j < 16; j++) X[j] = __builtin_amdgcn_bitop3_b32(X[j], T[j], mk, 0x78);  // X ^ (T & mk)
    if (i < 15) xtime16(T);
  }
}

// ---- layouts -------------------------------------------------------------------------------------------------------
// slot codes: 0, 1 = register bits R0, R1; 3, 4, 5 = lane bits; 8 + i = wave bit i
struct Lay {
  int s[L];
};
constexpr Lay LA{{0, 1, 5, 4, 3, 8, 9, 10, 11}};
constexpr Lay LB{{5, 4, 0, 1, 3, 8, 9, 10, 11}};
constexpr Lay LC{{5, 4, 3, 1, 0, 8, 9, 10, 11}};
constexpr Lay LD{{5, 4, 3, 9, 8, 0, 1, 10, 11}};
constexpr Lay LE{{5, 4, 3, 9, 8, 10, 11, 0, 1}};

// position bits of register slot r under layout Y, and the masks of the lane / wave parts
constexpr int pos_r(const Lay& Y, int r) {
  int p = 0;
  for (int b = 0; b < L; b++)
    if (Y.s[b] < 2 && ((r >> Y.s[b]) & 1)) p |= 1 << b;
  return p;
}
__device__ __forceinline__ int pos_lane(const Lay& Y, int lane) {
  int p = 0;
#pragma unroll
  for (int b = 0; b < L; b++)
    if (Y.s[b] >= 3 && Y.s[b] < 8) p |= ((lane >> Y.s[b]) & 1) << b;
  return p;
}
__device__ __forceinline__ int pos_wave(const Lay& Y, int w) {
  int p = 0;
#pragma unroll
  for (int b = 0; b < L; b++)
    if (Y.s[b] >= 8) p |= ((w >> (Y.s[b] - 8)) & 1) << b;
  return p;
}
constexpr int pos_w_ct(const Lay& Y, int wv) {  // position bits of wave index wv (compile-time)
  int p = 0;
  for (int b = 0; b < L; b++)
    if (Y.s[b] >= 8 && ((wv >> (Y.s[b] - 8)) & 1)) p |= 1 << b;
  return p;
}
constexpr int pos_of_slot(const Lay& Y, int slot) {  // the position bit held by a slot
  for (int b = 0; b < L; b++)
    if (Y.s[b] == slot) return b;
  return -1;
}
constexpr bool bits_above_in(const Lay& Y, int d, int lo, int hi) {  // any position bit > d in slots [lo, hi)
  for (int b = d + 1; b < L; b++)
    if (Y.s[b] >= lo && Y.s[b] < hi) return true;
  return false;
}

// The 8 generic per-lane constants (layers d = 0, 1 of both transforms, two butterflies each) are fetched once at
// the start, together with the data, two 16-bit values per VGPR: fetched at their layer, each would stall its wave on
// a global-load round trip inside the compute phase.
constexpr int lv_slot(bool inv, int d, int r) {  // r = the butterfly's lower register index
  return (inv ? 0 : 4) + (inv ? d : 1 - d) * 2 + ((r & 1) | (r >> 1));
}
struct Ctx {
  const uint16_t* cpoly;  // alpha^skew[i] in the standard basis, 0 = no multiply
  int lane, w;
  uint32_t lv[4];         // packed per-lane constants, slot lv_slot(..)
  uint32_t lm3;           // all-ones in lanes with lane bit 3 set
};

// One butterfly of layer d (bit d in register slot RB of layout Y) between E[R] and E[R | 1 << RB].
// layer constant index for group start s0 (bits above d of the position)
template <bool INVERSE, int D>
constexpr int cidx(int s0) {
  return INVERSE ? (M - 1 + s0 + (1 << D)) : (s0 + (1 << D) - 1);
}
// X ^= t * Y for the runtime wave bit in slot SLOT (position bit P) if that bit of w is set: t = g(2^P) ^ g(0) with
// g the layer's constant as a function of the group start.  The bit test is made to look lane-divergent (opaque
// VGPR copy of w), so the compiler guards the XOR program with the exec mask and updates X in place (a scalar
// branch renamed X and paid copies on the other path).
template <bool INVERSE, int D, int SLOT, int P>
__device__ __forceinline__ void muladd_wbit(uint32_t (&X)[16], const uint32_t (&Yv)[16], uint32_t wv) {
  constexpr unsigned t = kCpoly16[cidx<INVERSE, D>(1 << P)] ^ kCpoly16[cidx<INVERSE, D>(0)];
  if ((wv >> (SLOT - 8)) & 1u) muladd_const<t>(X, Yv);
}
// X ^= (C * Y) & mk, C compile-time
template <unsigned C, int I = 0>
__device__ __forceinline__ void muladd_const_masked(uint32_t (&X)[16], const uint32_t (&Y)[16], uint32_t mk) {
  if constexpr (C != 0 && I < 16) {
    constexpr unsigned ROW = mul_row(C, I);
    if constexpr (ROW != 0) {
      const uint32_t z = fold_row<ROW, 0, -1>(0u, Y);
      X[I] = __builtin_amdgcn_bitop3_b32(X[I], z, mk, 0x78);  // X ^ (z & mk)
    }
    muladd_const_masked<C, I + 1>(X, Y, mk);
  }
}
constexpr int lane_bits_above(const Lay& Y, int d) {
  int n = 0;
  for (int b = d + 1; b < L; b++)
    if (Y.s[b] >= 3 && Y.s[b] < 8) n++;
  return n;
}
template <const Lay& Y, bool INVERSE, int D, int R, int OM>
__device__ __forceinline__ void butterfly(uint32_t (&E)[4][16], const Ctx& cx) {
  constexpr int RB = Y.s[D];
  static_assert(RB == 0 || RB == 1, "butterfly bit must sit in a register slot");
  if constexpr (!((R >> RB) & 1)) {
    uint32_t(&X)[16] = E[R];
    uint32_t(&Yv)[16] = E[R | (1 << RB)];
    constexpr int hi = ~((2 << D) - 1);
    if (INVERSE) {
#pragma unroll
      for (int j = 0; j < 16; j++) Yv[j] ^= X[j];
    }
    if constexpr (lane_bits_above(Y, D) > 1) {  // per-lane constant (preloaded), generic multiply
      constexpr int slot = lv_slot(INVERSE, D, R);
      muladd_lane(X, Yv, (cx.lv[slot >> 1] >> (16 * (slot & 1))) & 0xFFFFu);
    } else {  // compile-time, plus one term per runtime wave bit (W0) and lane bit 3 above d
      constexpr int sct = (pos_r(Y, R) + pos_w_ct(Y, OM * 2)) & hi;
      static_assert(cidx<INVERSE, D>(sct) < kCpoly16N, "constant table too short");
      muladd_const<kCpoly16[cidx<INVERSE, D>(sct)]>(X, Yv);
      constexpr int p8 = pos_of_slot(Y, 8), p9 = -1;
      if constexpr (p8 > D) {
        uint32_t wv = cx.w;
        asm volatile("" : "+v"(wv));
        if constexpr (p8 > D) muladd_wbit<INVERSE, D, 8, p8>(X, Yv, wv);
        if constexpr (p9 > D) muladd_wbit<INVERSE, D, 9, p9>(X, Yv, wv);
      }
      if constexpr (lane_bits_above(Y, D) == 1) {  // a single lane bit (layer 2 in LB: p4 on lane bit 3)
        constexpr int pl = pos_of_slot(Y, 3);
        static_assert(pl > D, "the one lane bit above d is lane bit 3");
        constexpr unsigned t = kCpoly16[cidx<INVERSE, D>(1 << pl)] ^ kCpoly16[cidx<INVERSE, D>(0)];
        muladd_const_masked<t>(X, Yv, cx.lm3);
      }
    }
    if (!INVERSE) {
#pragma unroll
      for (int j = 0; j < 16; j++) Yv[j] ^= X[j];
    }
  }
}
template <const Lay& Y, bool INVERSE, int D, int OM>
__device__ __forceinline__ void layer(uint32_t (&E)[4][16], const Ctx& cx) {
  butterfly<Y, INVERSE, D, 0, OM>(E, cx);
  butterfly<Y, INVERSE, D, 1, OM>(E, cx);
  butterfly<Y, INVERSE, D, 2, OM>(E, cx);
  butterfly<Y, INVERSE, D, 3, OM>(E, cx);
}

template <const Lay& Y, bool INVERSE, int D, int R>
__device__ __forceinline__ void lv_fetch(Ctx& cx) {
  constexpr int RB = Y.s[D];
  constexpr int hi = ~((2 << D) - 1);
  constexpr int base = INVERSE ? (M - 1 + (pos_r(Y, R) & hi) + (1 << D)) : ((pos_r(Y, R) & hi) + (1 << D) - 1);
  constexpr int slot = lv_slot(INVERSE, D, R);
  static_assert(!((R >> RB) & 1), "R is the lower register of its butterfly");
  const uint32_t c = cx.cpoly[base + ((pos_lane(Y, cx.lane) + pos_wave(Y, cx.w)) & hi)];
  cx.lv[slot >> 1] |= c << (16 * (slot & 1));
}
__device__ __forceinline__ void lv_fetch_all(Ctx& cx) {
#pragma unroll
  for (int i = 0; i < 4; i++) cx.lv[i] = 0;
  lv_fetch<LA, true, 0, 0>(cx);
  lv_fetch<LA, true, 0, 2>(cx);
  lv_fetch<LA, true, 1, 0>(cx);
  lv_fetch<LA, true, 1, 1>(cx);
  lv_fetch<LA, false, 1, 0>(cx);
  lv_fetch<LA, false, 1, 1>(cx);
  lv_fetch<LA, false, 0, 0>(cx);
  lv_fetch<LA, false, 0, 2>(cx);
}

// ---- moves between layouts ----------------------------------------------------------------------------------------
// R0 <-> lane bit 5 and R1 <-> lane bit 4 (LA <-> LB): v_permlane32_swap(a, b) exchanges lanes 32..63 of a with lanes
// 0..31 of b, i.e. swaps the register bit of the pair (a, b) with lane bit 5; v_permlane16_swap likewise for lane
// bit 4 (per 32-lane half).  Involution.
__device__ __forceinline__ void swap_lane45(uint32_t (&E)[4][16]) {
#pragma unroll
  for (int j = 0; j < 16; j++) {
    auto p0 = __builtin_amdgcn_permlane32_swap(E[0][j], E[1][j], false, false);
    E[0][j] = p0[0];
    E[1][j] = p0[1];
    auto p1 = __builtin_amdgcn_permlane32_swap(E[2][j], E[3][j], false, false);
    E[2][j] = p1[0];
    E[3][j] = p1[1];
  }
#pragma unroll
  for (int j = 0; j < 16; j++) {
    auto p0 = __builtin_amdgcn_permlane16_swap(E[0][j], E[2][j], false, false);
    E[0][j] = p0[0];
    E[2][j] = p0[1];
    auto p1 = __builtin_amdgcn_permlane16_swap(E[1][j], E[3][j], false, false);
    E[1][j] = p1[0];
    E[3][j] = p1[1];
  }
}
// R0 <-> lane bit 3 (LB <-> LC): the partner lane (lane ^ 8) via DPP row_ror:8, selects on lm = all-ones in lanes
// with bit 3 set.  Involution.
__device__ __forceinline__ uint32_t ror8(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
}
__device__ __forceinline__ void swap_lane3(uint32_t (&E)[4][16], uint32_t lm) {
#pragma unroll
  for (int q = 0; q < 4; q += 2) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t a = E[q][j], b = E[q + 1][j];
      const uint32_t send = __builtin_amdgcn_bitop3_b32(lm, a, b, 0xCA);  // lm ? a : b
      const uint32_t recv = ror8(send);
      E[q][j] = __builtin_amdgcn_bitop3_b32(lm, recv, a, 0xCA);
      E[q + 1][j] = __builtin_amdgcn_bitop3_b32(lm, b, recv, 0xCA);
    }
  }
}
// Register bits (R0, R1) <-> wave bits (W_{2H}, W_{2H+1}) through LDS (LC <-> LD: H = 0, LD <-> LE: H = 1).  Slot key
// (other wave bits, wave pair, register): thread (w, r) writes key (w_other, w_pair, r) and reads key
// (w_other, r, w_pair); the register equal to the wave pair stays in place.  Two rounds of 8 planes.
template <int H>
__device__ __forceinline__ void exchange_w(uint32_t (&E)[4][16], uint4* xb, int w, int lane) {
  const int wp = (w >> (2 * H)) & 3;
  const int wo = H == 0 ? (w >> 2) : (w & 3);
#pragma unroll
  for (int half = 0; half < 2; half++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      if (r == wp) continue;
      uint4* p = xb + ((((wo * 4 + wp) * 4 + r) * 2) * 64 + lane);
      p[0] = make_uint4(E[r][8 * half + 0], E[r][8 * half + 1], E[r][8 * half + 2], E[r][8 * half + 3]);
      p[64] = make_uint4(E[r][8 * half + 4], E[r][8 * half + 5], E[r][8 * half + 6], E[r][8 * half + 7]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; r++) {
      if (r == wp) continue;
      const uint4* p = xb + ((((wo * 4 + r) * 4 + wp) * 2) * 64 + lane);
      const uint4 v0 = p[0], v1 = p[64];
      E[r][8 * half + 0] = v0.x;
      E[r][8 * half + 1] = v0.y;
      E[r][8 * half + 2] = v0.z;
      E[r][8 * half + 3] = v0.w;
      E[r][8 * half + 4] = v1.x;
      E[r][8 * half + 5] = v1.y;
      E[r][8 * half + 6] = v1.z;
      E[r][8 * half + 7] = v1.w;
    }
    __syncthreads();
  }
}

struct Args {
  const uint8_t* src;
  long long src_blk, src_cw, src_sh;
  uint8_t* dst;
  long long dst_blk, dst_cw, dst_sh;
  uint8_t* cpy;
  long long cpy_blk, cpy_cw, cpy_sh;
  const uint16_t* cpoly;
  int cw_per_blk, slices, total;  // total = codewords of the launch
#if CDA_RS16_TRACE
  unsigned long long* trace;  // diagnostic builds: s_memrealtime at 4 points of the first 8 codewords of each workgroup
#endif
};

#ifndef CDA_RS16_TRACE
#define CDA_RS16_TRACE 0
#endif
// trace[(blockIdx * 8 + it) * 4 + ph] by lane 0 of wave 0 (vector store); ph 0 = codeword in registers (top part
// done), 1 = last LDS exchange done, 2 = transforms done, 3 = stores (and the next codeword's direct loads) issued
__device__ __forceinline__ void rs16_mark(const Args& a, int w, int it, int ph) {
#if CDA_RS16_TRACE
  if (w == 0 && it < 8) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) a.trace[((size_t)blockIdx.x * 8 + it) * 4 + ph] = t;
  }
#else
  (void)a, (void)w, (void)it, (void)ph;
#endif
}

// Diagnostic builds only (scripts/gpu_rs16_diag.sh compiles a separate library with -DCDA_RS16_DIAG_MODE=N):
// 1 = loads + stores only; 2 = no loads; 3 = no loads, no stores.  A release build is always 0 (encode) -- no
// environment switch can change what the product path computes; cda_build_info() names a diag build.
#ifndef CDA_RS16_DIAG_MODE
#define CDA_RS16_DIAG_MODE 0
#endif
constexpr int kMode = CDA_RS16_DIAG_MODE;

// Coalesced shard access.  Leopard's GF(2^16) shard layout pairs element e of each 64-B block with bytes e (low)
// and 32 + e (high).  Lane u (= lane & 7) of a position moves the 16-B chunks at u*16 + 128q, q = 0..3, so the 8
// lanes of a position cover 128 contiguous bytes per instruction (64-B strided chunks cost 4x the memory requests):
// lanes with lane bit 1 clear hold low halves, their partners (lane ^ 2, one DPP quad_perm) the matching high
// halves.  pair_in trades chunks so that each lane holds low + high bytes of 32 whole elements (blocks 2q + (u>>2)
// for q = 0, 1 on the low lane, q = 2, 3 on the high lane); pair_out is its inverse.  m1 = all-ones iff lane bit 1.
__device__ __forceinline__ uint32_t xq2(uint32_t v) {  // v of lane ^ 2
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
}
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}
__device__ __forceinline__ void pair_in(const uint4& q0, const uint4& q1, const uint4& q2, const uint4& q3, uint32_t m1,
                                        uint32_t (&lo)[8], uint32_t (&hi)[8]) {
  const uint32_t a[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
  const uint32_t b[8] = {q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t rv = xq2(sel(m1, a[i], b[i]));  // low lane sends b, high lane sends a
    lo[i] = sel(m1, rv, a[i]);
    hi[i] = sel(m1, b[i], rv);
  }
}
__device__ __forceinline__ void pair_out(const uint32_t (&lo)[8], const uint32_t (&hi)[8], uint32_t m1, uint4& q0,
                                         uint4& q1, uint4& q2, uint4& q3) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t rv = xq2(sel(m1, lo[i], hi[i]));  // low lane sends hi, high lane sends lo
    a[i] = sel(m1, rv, lo[i]);
    b[i] = sel(m1, hi[i], rv);
  }
  q0 = make_uint4(a[0], a[1], a[2], a[3]);
  q1 = make_uint4(a[4], a[5], a[6], a[7]);
  q2 = make_uint4(b[0], b[1], b[2], b[3]);
  q3 = make_uint4(b[4], b[5], b[6], b[7]);
}

typedef __attribute__((address_space(1))) void* glb_ptr;
typedef __attribute__((address_space(3))) void* lds_ptr;

// Persistent: workgroup blockIdx.x encodes codewords g = blockIdx.x, + gridDim.x, ... (one workgroup per CU: the
// state fills the CU's registers, so a CU never holds a second codeword whose loads could overlap this one's
// compute).  Once the last LDS exchange of codeword g is done, each wave streams positions r = 0, 1 of its share
// of codeword g + gridDim.x into the (then idle) exchange buffer with global_load_lds (its own 8 KiB: 2 positions
// x 4 x 1 KiB, lane-linear), behind the remaining FFT layers and the stores; the next codeword reads them from LDS
// and loads only r = 2, 3 from HBM.
template <int OM>  // the body of the waves with (W3, W2) = OM
__device__ __forceinline__ void body(const Args& a, uint4* xb, int w) {
  const int lane0 = threadIdx.x & 63;
  Ctx cx{a.cpoly, lane0, w, {}, ((lane0 >> 3) & 1) ? ~0u : 0u};
  asm volatile("" : "+v"(cx.lm3));
  lv_fetch_all(cx);
  uint4* xw = xb + w * 512;  // this wave's prefetch slots [r = 0, 1][q = 0..3][lane]
  bool pre = false;          // positions r = 0, 1 of codeword g are in xw
  for (int g = blockIdx.x; g < a.total; g += gridDim.x) {
    // opaque per iteration: otherwise LICM hoists the per-lane multiplies' 16 masks per constant (all derived from
    // loop-invariant values) out of the loop and the register allocator spills
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" : "+v"(cx.lv[i]));
    asm volatile("" : "+v"(cx.lm3));
    int lane = lane0;  // likewise for the lane-derived LDS exchange addresses
    asm volatile("" : "+v"(lane));
    const int u = lane & 7;
    const int pl = pos_lane(LA, lane) + pos_wave(LA, w);
    const SliceMasks km = slice_masks();
    uint32_t m1 = (lane & 2) ? ~0u : 0u;
    asm volatile("" : "+v"(m1));
    const int slice = g % a.slices;
    const int cw = (g / a.slices) % a.cw_per_blk, blk = (g / a.slices) / a.cw_per_blk;
    const long long off = (long long)slice * 512 + u * 16;
    const uint8_t* src = a.src + blk * a.src_blk + cw * a.src_cw + off;
    uint8_t* dst = a.dst + blk * a.dst_blk + cw * a.dst_cw + off;
    uint8_t* cpy = a.cpy ? a.cpy + blk * a.cpy_blk + cw * a.cpy_cw + off : nullptr;

    uint32_t E[4][16];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int s = pl + pos_r(LA, r);  // data shard s sits at point m + s (all k = m shards present)
      const uint4* p = reinterpret_cast<const uint4*>(src + s * a.src_sh);
      uint4 q0, q1, q2, q3;
      if (r < 2 && pre) {
        q0 = xw[(r * 4 + 0) * 64 + lane], q1 = xw[(r * 4 + 1) * 64 + lane];
        q2 = xw[(r * 4 + 2) * 64 + lane], q3 = xw[(r * 4 + 3) * 64 + lane];
      } else if (kMode < 2) {  // modes >= 2: synthetic data, no loads
        q0 = p[0], q1 = p[8], q2 = p[16], q3 = p[24];
      } else {
        q0 = make_uint4(s, lane, w, r), q1 = make_uint4(lane * 3, s ^ 5, 7, w), q2 = q0, q3 = q1;
      }
      if (cpy) {
        uint4* o = reinterpret_cast<uint4*>(cpy + s * a.cpy_sh);
        o[0] = q0;
        o[8] = q1;
        o[16] = q2;
        o[24] = q3;
      }
      uint32_t lo[8], hi[8];
      pair_in(q0, q1, q2, q3, m1, lo, hi);
      bitslice8(lo, km);
      bitslice8(hi, km);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        E[r][j] = lo[j];
        E[r][8 + j] = hi[j];
      }
      change_basis<false>(E[r]);
    }
    const int gn = g + (int)gridDim.x;
    pre = false;
    if (kMode != 1) {
      // IFFT, D = 1 .. m/2
      layer<LA, true, 0, OM>(E, cx);
      layer<LA, true, 1, OM>(E, cx);
      swap_lane45(E);
      layer<LB, true, 2, OM>(E, cx);
      swap_lane3(E, cx.lm3);
      layer<LC, true, 3, OM>(E, cx);
      layer<LC, true, 4, OM>(E, cx);
      __syncthreads();  // every wave has read its prefetch slots before the exchange overwrites them
      exchange_w<0>(E, xb, w, lane);
      layer<LD, true, 5, OM>(E, cx);
      layer<LD, true, 6, OM>(E, cx);
      exchange_w<1>(E, xb, w, lane);
      layer<LE, true, 7, OM>(E, cx);
      layer<LE, true, 8, OM>(E, cx);
      // FFT, D = m/2 .. 1
      layer<LE, false, 8, OM>(E, cx);
      layer<LE, false, 7, OM>(E, cx);
      exchange_w<1>(E, xb, w, lane);
      layer<LD, false, 6, OM>(E, cx);
      layer<LD, false, 5, OM>(E, cx);
      exchange_w<0>(E, xb, w, lane);  // ends with a barrier: the exchange buffer is free until the next codeword
      {  // issued unconditionally (no branch with the state live): without a next codeword, re-read this one
        const int gp = gn < a.total ? gn : g;
        const int sl = gp % a.slices;
        const int cwn = (gp / a.slices) % a.cw_per_blk, bn = (gp / a.slices) / a.cw_per_blk;
        const uint8_t* srcn = a.src + bn * a.src_blk + cwn * a.src_cw + (long long)sl * 512 + u * 16;
#pragma unroll
        for (int r = 0; r < 2; r++) {
          const uint8_t* sp = srcn + (pl + pos_r(LA, r)) * a.src_sh;
#pragma unroll
          for (int q = 0; q < 4; q++)
            __builtin_amdgcn_global_load_lds((glb_ptr)(sp + 128 * q), (lds_ptr)(xw + (r * 4 + q) * 64), 16, 0, 0);
        }
        pre = kMode == 0;
      }
      layer<LC, false, 4, OM>(E, cx);
      layer<LC, false, 3, OM>(E, cx);
      swap_lane3(E, cx.lm3);
      layer<LB, false, 2, OM>(E, cx);
      swap_lane45(E);
      layer<LA, false, 1, OM>(E, cx);
      layer<LA, false, 0, OM>(E, cx);
    }
    if (kMode == 3) continue;
    // parity shard s = point s
    const SliceMasks ko = slice_masks();
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int s = pl + pos_r(LA, r);
      uint32_t v[16];
#pragma unroll
      for (int j = 0; j < 16; j++) v[j] = E[r][j];
      change_basis<true>(v);
      uint32_t lo[8], hi[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        lo[j] = v[j];
        hi[j] = v[8 + j];
      }
      bitslice8(lo, ko);
      bitslice8(hi, ko);
      uint4* o = reinterpret_cast<uint4*>(dst + s * a.dst_sh);
      uint4 q0, q1, q2, q3;
      pair_out(lo, hi, m1, q0, q1, q2, q3);
      o[0] = q0;
      o[8] = q1;
      o[16] = q2;
      o[24] = q3;
    }
  }
}

#ifndef CDA_RS16_PIPE
#define CDA_RS16_PIPE 1  // 0: the round-3 loop (body), for same-box A/B builds
#endif

// 64-B unit of one position: raw 16-B chunks <-> the 16 plane words of the state
__device__ __forceinline__ void to_state(const uint4& q0, const uint4& q1, const uint4& q2, const uint4& q3, uint32_t m1,
                                         const SliceMasks& km, uint32_t (&Er)[16]) {
  uint32_t lo[8], hi[8];
  pair_in(q0, q1, q2, q3, m1, lo, hi);
  bitslice8(lo, km);
  bitslice8(hi, km);
#pragma unroll
  for (int j = 0; j < 8; j++) {
    Er[j] = lo[j];
    Er[8 + j] = hi[j];
  }
  change_basis<false>(Er);
}
__device__ __forceinline__ void from_state(const uint32_t (&Er)[16], uint32_t m1, const SliceMasks& ko, uint4& q0,
                                           uint4& q1, uint4& q2, uint4& q3) {
  uint32_t v[16];
#pragma unroll
  for (int j = 0; j < 16; j++) v[j] = Er[j];
  change_basis<true>(v);
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    lo[j] = v[j];
    hi[j] = v[8 + j];
  }
  bitslice8(lo, ko);
  bitslice8(hi, ko);
  pair_out(lo, hi, m1, q0, q1, q2, q3);
}

// The LDS prefetch of positions r = 0, 1, all in inline asm.  hipcc waits vmcnt(0) -- the whole store drain -- at
// the first use of any load result and before any barrier while it knows of an LDS-DMA in flight, and treats an
// LDS read after one the same way; loads, stores and LDS-DMA in fact retire from vmcnt in issue order
// (MI355X_MICROARCH.md, s_waitcnt).  So the DMA is issued by asm (the compiler sees no LDS-DMA) and read back by asm
// behind a counted wait: exactly kAfterPrefetch vector-memory instructions of this wave follow the 8 DMA loads in
// program order (the 16 parity stores and the 8 loads of r = 2, 3 of the store phase), so vmcnt(24) is the wait
// for the prefetch alone.  The compiler's own waits for the r = 2, 3 loads then stay partial.
// The counts are checked on the built code object, over every control-flow path from each prefetch to its wait
// (tools/vmcnt_check.py, tests/test_rs16_vmcnt.py): a store or spill the compiler moved across would fail the build
// check instead of racing.
constexpr int kAfterPrefetch = 24;  // in the loop; 8 (the R loads) after the prologue's prefetch
// M0 is reserved by the compiler; nothing else in this kernel uses it (the only M0 writes in its ISA are these), and
// the clobber still tells the compiler it changes.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const uint8_t* g, uint32_t lds_uniform) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g), "s"(lds_uniform) : "memory", "m0");
}
#pragma clang diagnostic pop
// 8 DMA loads: position r (0, 1), chunk q (0..3) of this wave's share -> slot (r * 4 + q) of xw (lane-linear)
__device__ __forceinline__ void prefetch01(const uint8_t* src, long long sh, int pl, const uint4* xw) {
  const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr)xw);
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const uint8_t* sp = src + (pl + r) * sh;  // pos_r(LA, r) = r for r < 2 (LA: p0 -> R0)
#pragma unroll
    for (int q = 0; q < 4; q++) glds16(sp + 128 * q, base + (uint32_t)(r * 4 + q) * 1024u);
  }
}

// Parity stores of the persistent loop, non-temporal: nothing in this kernel reads them again (the leaf hashing does,
// a launch later), and the store drain at each codeword's end is the part of the memory phase the next codeword waits
// behind.  Same-box rotating A/B, 3 rounds (profiles/r05_rs16_ab.log, ms per square): columns 0.252-0.254 vs
// 0.259-0.267, rows 0.129-0.131 vs 0.131-0.134.  CDA_RS16_NT_STORES=0 builds the plain stores (A/B).
//
// Measured and not kept (same log): a round-ahead cache prefetch -- each workgroup pulling 1/G of the next persistent
// round's input (two 128-KiB row segments of the column pass, its own next row of the row pass) into L2 / the
// Infinity Cache through LDS-DMA "touch" loads at the top of each codeword, so that the strided column reads would hit
// the cache: columns 0.272-0.287 vs 0.259-0.267 ms per square without it, rows unchanged, memory-only builds
// unchanged (0.117 / 0.052 ms).  The column pass's memory phase is not made shorter by moving its DRAM reads earlier.
#ifndef CDA_RS16_NT_STORES
#define CDA_RS16_NT_STORES 1
#endif
__device__ __forceinline__ void store_parity(uint4* o, const uint4& q0, const uint4& q1, const uint4& q2,
                                             const uint4& q3) {
#if CDA_RS16_NT_STORES
  typedef unsigned v4 __attribute__((ext_vector_type(4)));
  v4* p = reinterpret_cast<v4*>(o);
  __builtin_nontemporal_store(v4{q0.x, q0.y, q0.z, q0.w}, p);
  __builtin_nontemporal_store(v4{q1.x, q1.y, q1.z, q1.w}, p + 8);
  __builtin_nontemporal_store(v4{q2.x, q2.y, q2.z, q2.w}, p + 16);
  __builtin_nontemporal_store(v4{q3.x, q3.y, q3.z, q3.w}, p + 24);
#else
  o[0] = q0, o[8] = q1, o[16] = q2, o[24] = q3;
#endif
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 u4(v4u v) { return make_uint4(v.x, v.y, v.z, v.w); }
template <int N>
__device__ __forceinline__ void read_prefetch(const uint4* xl, uint4 (&q)[2][4]) {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx9");
  const uint32_t addr = (uint32_t)(uintptr_t)(lds_ptr)xl;
  v4u a0, a1, a2, a3, a4, a5, a6, a7;
  asm volatile(
      "s_waitcnt vmcnt(%9)\n\t"
      "ds_read_b128 %0, %8\n\t"
      "ds_read_b128 %1, %8 offset:1024\n\t"
      "ds_read_b128 %2, %8 offset:2048\n\t"
      "ds_read_b128 %3, %8 offset:3072\n\t"
      "ds_read_b128 %4, %8 offset:4096\n\t"
      "ds_read_b128 %5, %8 offset:5120\n\t"
      "ds_read_b128 %6, %8 offset:6144\n\t"
      "ds_read_b128 %7, %8 offset:7168\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(a4), "=&v"(a5), "=&v"(a6), "=&v"(a7)
      : "v"(addr), "i"(N)
      : "memory");
  q[0][0] = u4(a0), q[0][1] = u4(a1), q[0][2] = u4(a2), q[0][3] = u4(a3);
  q[1][0] = u4(a4), q[1][1] = u4(a5), q[1][2] = u4(a6), q[1][3] = u4(a7);
}

__device__ __forceinline__ int lane_id() {  // recomputed where needed: a loop-carried copy was spilled to scratch,
                                             // and the reload's vmcnt(0) waited for the whole store drain
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Top of codeword g: r = 0, 1 from the LDS prefetch (N = the vector-memory instructions issued after it), layer 0's
// (0, 1) butterfly, then r = 2, 3 from R and layer 0's (2, 3) butterfly.  (The Q0 copy of the rows pass stores the
// raw chunks on the way.)  Instantiated twice -- after the prologue and at the end of the loop body -- so that the
// compiler's wait for R in each copy is computed from one straight-line history, not merged at a loop header.
template <int OM, int N>
__device__ __forceinline__ void top_part(const Args& a, uint4* xw, int w, int g, const Ctx& cx, uint4 (&R)[2][4],
                                         uint32_t (&E)[4][16]) {
  const int lane = lane_id();
  const int u = lane & 7;
  const int pl = pos_lane(LA, lane) + pos_wave(LA, w);
  const SliceMasks km = slice_masks();
  uint32_t m1 = (lane & 2) ? ~0u : 0u;
  asm volatile("" : "+v"(m1));
  const int slice = g % a.slices;
  const int cw = (g / a.slices) % a.cw_per_blk, blk = (g / a.slices) / a.cw_per_blk;
  uint8_t* cpy = a.cpy ? a.cpy + blk * a.cpy_blk + cw * a.cpy_cw + (long long)slice * 512 + u * 16 : nullptr;
  {
    uint4 q[2][4];
    read_prefetch<N>(xw + lane, q);
#pragma unroll
    for (int r = 0; r < 2; r++) {
      if (cpy) {
        uint4* o = reinterpret_cast<uint4*>(cpy + (pl + pos_r(LA, r)) * a.cpy_sh);
        o[0] = q[r][0], o[8] = q[r][1], o[16] = q[r][2], o[24] = q[r][3];
      }
      to_state(q[r][0], q[r][1], q[r][2], q[r][3], m1, km, E[r]);
    }
  }
  butterfly<LA, true, 0, 0, OM>(E, cx);  // layer 0, pair (0, 1): before r = 2, 3 are needed
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 2; r < 4; r++) {
    if (cpy) {
      uint4* o = reinterpret_cast<uint4*>(cpy + (pl + pos_r(LA, r)) * a.cpy_sh);
      o[0] = R[r - 2][0], o[8] = R[r - 2][1], o[16] = R[r - 2][2], o[24] = R[r - 2][3];
    }
    to_state(R[r - 2][0], R[r - 2][1], R[r - 2][2], R[r - 2][3], m1, km, E[r]);
  }
  butterfly<LA, true, 0, 2, OM>(E, cx);
}

// Software-pipelined persistent loop (round 4).  Per codeword g of this workgroup:
//   top      (top_part) r = 0, 1 from the LDS prefetch; layer 0's (0, 1) butterfly; r = 2, 3 from the registers R
//            that the previous store phase loaded; layer 0's (2, 3) butterfly.
//   middle   the transforms as in body(); after the last exchange, global_load_lds of r = 0, 1 of codeword g + grid.
//   bottom   r = 2: parity stores, then the NEXT codeword's r = 2 loads into R[0] (the registers E[2] just freed);
//            r = 3 likewise into R[1]; then the r = 0, 1 stores.
// On gfx950 vmcnt counts loads and stores in one in-order counter, so in body() the next codeword's direct loads,
// issued after all 16 stores, could not be waited for without draining every store first.  Here the waits are
// (a) vmcnt(24) for the LDS prefetch: nothing of the store phase; (b) the compiler's wait before R[0] is first read:
// the r = 2, 3 stores and loads only, while the r = 0, 1 stores still drain -- and that wait comes after the
// conversion of r = 0, 1 and a per-lane butterfly.  No extra registers: each load lands in the 16 VGPRs its
// position's state just left.  Without a next codeword the loads read the first 512 B of the source (cache hits)
// instead of re-reading a whole codeword.
template <int OM>
__device__ __forceinline__ void body2(const Args& a, uint4* xb, int w) {
  const int lane0 = threadIdx.x & 63;
  Ctx cx{a.cpoly, lane0, w, {}, ((lane0 >> 3) & 1) ? ~0u : 0u};
  asm volatile("" : "+v"(cx.lm3));
  lv_fetch_all(cx);
  uint4* xw = xb + w * 512;  // this wave's prefetch slots [r = 0, 1][q = 0..3][lane]
  uint4 R[2][4];             // positions r = 2, 3 of the next codeword, raw
  int g = blockIdx.x;
  {  // prologue: the first codeword's r = 0, 1 into the LDS slots, r = 2, 3 into R (the loop's own order)
    const int u = lane0 & 7;
    const int pl = pos_lane(LA, lane0) + pos_wave(LA, w);
    const int slice = g % a.slices;
    const int cw = (g / a.slices) % a.cw_per_blk, blk = (g / a.slices) / a.cw_per_blk;
    const uint8_t* src = a.src + blk * a.src_blk + cw * a.src_cw + (long long)slice * 512 + u * 16;
    prefetch01(src, a.src_sh, pl, xw);
#pragma unroll
    for (int r = 2; r < 4; r++) {
      const uint4* p = reinterpret_cast<const uint4*>(src + (pl + pos_r(LA, r)) * a.src_sh);
      R[r - 2][0] = p[0], R[r - 2][1] = p[8], R[r - 2][2] = p[16], R[r - 2][3] = p[24];
    }
  }
  uint32_t E[4][16];
  top_part<OM, 8>(a, xw, w, g, cx, R, E);  // after the prologue only its 8 R loads follow the prefetch
  for (int it = 0;; it++) {
    rs16_mark(a, w, it, 0);
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" : "+v"(cx.lv[i]));
    asm volatile("" : "+v"(cx.lm3));
    const int lane = lane_id();
    const int u = lane & 7;
    const int pl = pos_lane(LA, lane) + pos_wave(LA, w);
    const int gn = g + (int)gridDim.x;
    const bool more = gn < a.total;
    // the next codeword's source (a dummy 512-B window of the source when there is none)
    const int gq = more ? gn : 0;
    const int sln = gq % a.slices;
    const int cwn = (gq / a.slices) % a.cw_per_blk, bn = (gq / a.slices) / a.cw_per_blk;
    const uint8_t* srcn = a.src + bn * a.src_blk + cwn * a.src_cw + (long long)sln * 512 + u * 16;
    const long long shn = more ? a.src_sh : 0;
    // IFFT, D = 1 .. m/2
    layer<LA, true, 1, OM>(E, cx);
    swap_lane45(E);
    layer<LB, true, 2, OM>(E, cx);
    swap_lane3(E, cx.lm3);
    layer<LC, true, 3, OM>(E, cx);
    layer<LC, true, 4, OM>(E, cx);
    __syncthreads();  // every wave has read its prefetch slots before the exchange overwrites them
    exchange_w<0>(E, xb, w, lane);
    layer<LD, true, 5, OM>(E, cx);
    layer<LD, true, 6, OM>(E, cx);
    exchange_w<1>(E, xb, w, lane);
    layer<LE, true, 7, OM>(E, cx);
    layer<LE, true, 8, OM>(E, cx);
    // FFT, D = m/2 .. 1
    layer<LE, false, 8, OM>(E, cx);
    layer<LE, false, 7, OM>(E, cx);
    exchange_w<1>(E, xb, w, lane);
    layer<LD, false, 6, OM>(E, cx);
    layer<LD, false, 5, OM>(E, cx);
    exchange_w<0>(E, xb, w, lane);  // ends with a barrier: the exchange buffer is free until the next codeword
    rs16_mark(a, w, it, 1);
    prefetch01(srcn, shn, pl, xw);
    layer<LC, false, 4, OM>(E, cx);
    layer<LC, false, 3, OM>(E, cx);
    swap_lane3(E, cx.lm3);
    layer<LB, false, 2, OM>(E, cx);
    swap_lane45(E);
    layer<LA, false, 1, OM>(E, cx);
    layer<LA, false, 0, OM>(E, cx);
    rs16_mark(a, w, it, 2);
    {  // parity shard s = point s; r = 2, 3 first, each followed by the next codeword's loads of that position
      uint32_t m1 = (lane & 2) ? ~0u : 0u;
      asm volatile("" : "+v"(m1));
      const int slice = g % a.slices;
      const int cw = (g / a.slices) % a.cw_per_blk, blk = (g / a.slices) / a.cw_per_blk;
      uint8_t* dst = a.dst + blk * a.dst_blk + cw * a.dst_cw + (long long)slice * 512 + u * 16;
      const SliceMasks ko = slice_masks();
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int r = (i + 2) & 3;
        uint4 q0, q1, q2, q3;
        from_state(E[r], m1, ko, q0, q1, q2, q3);
        uint4* o = reinterpret_cast<uint4*>(dst + (pl + pos_r(LA, r)) * a.dst_sh);
        store_parity(o, q0, q1, q2, q3);
        if (r >= 2) {
          const uint4* p = reinterpret_cast<const uint4*>(srcn + (pl + pos_r(LA, r)) * shn);
          R[r - 2][0] = p[0], R[r - 2][1] = p[8], R[r - 2][2] = p[16], R[r - 2][3] = p[24];
        }
      }
    }
    rs16_mark(a, w, it, 3);
    if (!more) break;
    g = gn;
    top_part<OM, kAfterPrefetch>(a, xw, w, g, cx, R, E);
  }
}

// one whole body per value of W1..W3 (scalar branch at entry; each runs to the end, so no control-flow merge with
// the 64 live state registers follows the specialised layers -- such a merge made the register allocator spill)
__global__ void __launch_bounds__(1024, 1) rs_encode16_reg_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 xb[];  // 64 keys x 2 quads x 64 lanes x 16 B = 128 KiB
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // (s_setprio 1 for waves 8-15, so that the second-dispatched half does not lose every issue arbitration before the
  // exchange barriers: columns 0.250-0.260 vs 0.252-0.258 ms per square, profiles/r05_prio_ab.log; not kept)
#if CDA_RS16_PIPE && CDA_RS16_DIAG_MODE == 0
#define CDA_RS16_BODY body2
#else
#define CDA_RS16_BODY body
#endif
  switch (w >> 1) {
    case 0: CDA_RS16_BODY<0>(a, xb, w); break;
    case 1: CDA_RS16_BODY<1>(a, xb, w); break;
    case 2: CDA_RS16_BODY<2>(a, xb, w); break;
    case 3: CDA_RS16_BODY<3>(a, xb, w); break;
    case 4: CDA_RS16_BODY<4>(a, xb, w); break;
    case 5: CDA_RS16_BODY<5>(a, xb, w); break;
    case 6: CDA_RS16_BODY<6>(a, xb, w); break;
    default: CDA_RS16_BODY<7>(a, xb, w); break;
  }
}

}  // namespace r16

const char* rs16_diag_tag() {
#if CDA_RS16_DIAG_MODE != 0
#define CDA_STR2(x) #x
#define CDA_STR(x) CDA_STR2(x)
  return "rs16_mode=" CDA_STR(CDA_RS16_DIAG_MODE);
#else
  return "";
#endif
}

bool rs16_reg_eligible(const RsJob& j) { return j.k == r16::M && j.shard_len % 512 == 0; }

int rs16_reg_init(int device) {
  (void)device;
  // the compile-time constants must equal the host-built table (leopard_tables.cpp)
  const LeoTables& t = leo_tables(16);
  unsigned st = 1;
  static uint16_t apow[65535];
  for (int i = 0; i < 65535; i++) {
    apow[i] = (uint16_t)st;
    st <<= 1;
    if (st & 0x10000) st ^= 0x1002D;
  }
  for (int i = 0; i < kCpoly16N; i++) {
    const uint16_t want = t.skew[i] >= 65535 ? 0 : apow[t.skew[i]];
    if (want != kCpoly16[i]) return -1;
  }
  return hipFuncSetAttribute((const void*)r16::rs_encode16_reg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             128 * 1024) == hipSuccess
             ? 0
             : -1;
}

int launch_rs_encode16_reg(const RsJob& j, const uint16_t* d_cpoly, hipStream_t s) {
  if (!rs16_reg_eligible(j)) return -2;
  r16::Args a;
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
  a.cpoly = d_cpoly;
  a.cw_per_blk = j.cw_per_blk;
#if CDA_RS16_TRACE
  a.trace = nullptr;
  if (const char* e = getenv("CDA_RS16_TRACE_PTR")) a.trace = (unsigned long long*)(uintptr_t)strtoull(e, nullptr, 0);
  if (!a.trace) return -2;
#endif
  a.slices = j.shard_len / 512;
  const long long total = (long long)j.nblk * j.cw_per_blk * a.slices;
  if (total <= 0 || total > 0x7FFFFFFF) return -2;
  a.total = (int)total;
  static const int ncu = [] {  // one persistent workgroup per CU
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const int grid = (int)(total < ncu ? total : ncu);
  hipLaunchKernelGGL(r16::rs_encode16_reg_kernel, dim3((unsigned)grid), dim3(1024), 128 * 1024, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cda
