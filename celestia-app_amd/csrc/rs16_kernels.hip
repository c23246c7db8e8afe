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

#include <map>
#include <mutex>
#include <utility>

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
  unsigned long long* trace;      // diagnostic builds (CDA_RS16_H2_TRACE): per-workgroup phase timestamps
  int* queue;                     // half-slice kernel: per-partition item counters + a done counter (zero at launch)
};

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
  for (;;) {
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
    prefetch01(srcn, shn, pl, xw);
    layer<LC, false, 4, OM>(E, cx);
    layer<LC, false, 3, OM>(E, cx);
    swap_lane3(E, cx.lm3);
    layer<LB, false, 2, OM>(E, cx);
    swap_lane45(E);
    layer<LA, false, 1, OM>(E, cx);
    layer<LA, false, 0, OM>(E, cx);
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
        o[0] = q0, o[8] = q1, o[16] = q2, o[24] = q3;
        if (r >= 2) {
          const uint4* p = reinterpret_cast<const uint4*>(srcn + (pl + pos_r(LA, r)) * shn);
          R[r - 2][0] = p[0], R[r - 2][1] = p[8], R[r - 2][2] = p[16], R[r - 2][3] = p[24];
        }
      }
    }
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


// ---- half-slice form: two workgroups per CU (round 4) --------------------------------------------------------------
// The whole-codeword kernel above fills a CU's registers with one codeword, so its loads and stores never overlap
// another workgroup's compute: memory-only 0.116 ms and compute-only 0.138 ms per column square add up to the
// product's 0.27 (profiles/r04_rs16_diag.log).  Here a work item is HALF of every shard's 512-B slice (the FFT is
// over positions, element by element, so the two 256-B halves are independent codewords of the same transform):
// 512 positions x 256 B = 128 KiB = 8 waves x 64 lanes x 64 VGPRs, and a CU holds two such workgroups, one
// computing while the other loads or stores (the FF8 encoder's arrangement).
//   lane bits 0..1 = unit u (four lanes cover the 256-B half of a shard: pair_in's chunks at u*16 + 64q),
//   lane bits 2..5 = four position bits, register bits R0, R1 = two, wave bits W0..W2 = three.
//   LA  p0:R0 p1:R1 p2:L5 p3:L4 p4:L3 p5:L2 p6..p8:W0..W2   IFFT d = 0, 1 (load)  / FFT d = 1, 0 (store)
//   LB  p2:R0 p3:R1 p0:L5 p1:L4                           IFFT d = 2, 3         / FFT d = 3, 2   (swap_lane45)
//   LC  p4:R0 p5:R1 p2:L3 p3:L2                           IFFT d = 4, 5         / FFT d = 5, 4   (lane ^ 8, ^ 4)
//   LD  p6:R0 p7:R1 p4:W0 p5:W1                           IFFT d = 6, 7         / FFT d = 7, 6   (LDS, 2 bits)
//   LE  p8:R0 p6:W2                                       IFFT d = 8, FFT d = 8                  (LDS, 1 bit)
// Every wave bit is compile-time (one body per wave), so layers 4..8 multiply by compile-time constants; layers 2, 3
// have two lane bits above them (p4, p5): the affine split, two lane-masked XOR programs; layers 0, 1 (four lane bits
// above) use the generic per-lane multiply with preloaded constants, as the whole-codeword kernel.
namespace h2 {

#ifndef CDA_RS16_H2_STAGGER
#define CDA_RS16_H2_STAGGER 0
#endif
#ifndef CDA_RS16_H2_SPLIT
#define CDA_RS16_H2_SPLIT 0  // A/B builds: static split of the items by dispatch age (numerator over 8), no queue
#endif
#ifndef CDA_RS16_H2_TRACE
#define CDA_RS16_H2_TRACE 0  // diagnostic builds: s_memrealtime at 4 phases of the first 8 items of each workgroup
#endif
// trace[(bid * 8 + item) * 4 + phase], phase 0 = loop top, 1 = state built (loads consumed), 2 = transforms done,
// 3 = stores issued; written by lane 0 of wave 0 with a vector store
__device__ __forceinline__ void h2_mark(const Args& a, int w, int it, int ph) {
#if CDA_RS16_H2_TRACE
  if (w == 0 && it < 8) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) a.trace[((size_t)blockIdx.x * 8 + it) * 4 + ph] = t;
    if (it == 0 && ph == 0 && (threadIdx.x & 63) == 0) {  // where the workgroup runs: XCC_ID << 32 | HW_ID
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
      a.trace[(size_t)gridDim.x * 32 + blockIdx.x] = ((unsigned long long)xcc << 32) | hw;
    }
  }
#else
  (void)a, (void)w, (void)it, (void)ph;
#endif
}

struct Lay {
  int s[L];  // slot of position bit b: 0, 1 = R0, R1; 2..5 = lane bit; 8, 9, 10 = W0..W2
};
constexpr Lay LA{{0, 1, 5, 4, 3, 2, 8, 9, 10}};
constexpr Lay LB{{5, 4, 0, 1, 3, 2, 8, 9, 10}};
constexpr Lay LC{{5, 4, 3, 2, 0, 1, 8, 9, 10}};
constexpr Lay LD{{5, 4, 3, 2, 8, 9, 0, 1, 10}};
constexpr Lay LE{{5, 4, 3, 2, 8, 9, 10, 1, 0}};

constexpr bool is_lane(int s) { return s >= 2 && s < 8; }
constexpr int pos_r(const Lay& Y, int r) {
  int p = 0;
  for (int b = 0; b < L; b++)
    if (Y.s[b] < 2 && ((r >> Y.s[b]) & 1)) p |= 1 << b;
  return p;
}
constexpr int pos_w(const Lay& Y, int w) {
  int p = 0;
  for (int b = 0; b < L; b++)
    if (Y.s[b] >= 8 && ((w >> (Y.s[b] - 8)) & 1)) p |= 1 << b;
  return p;
}
__device__ __forceinline__ int pos_lane(const Lay& Y, int lane) {
  int p = 0;
#pragma unroll
  for (int b = 0; b < L; b++)
    if (is_lane(Y.s[b])) p |= ((lane >> Y.s[b]) & 1) << b;
  return p;
}
constexpr int lane_bits_above(const Lay& Y, int d) {
  int n = 0;
  for (int b = d + 1; b < L; b++)
    if (is_lane(Y.s[b])) n++;
  return n;
}
constexpr int pos_of_slot(const Lay& Y, int slot) {
  for (int b = 0; b < L; b++)
    if (Y.s[b] == slot) return b;
  return -1;
}

struct Ctx {
  const uint16_t* cpoly;
  uint32_t lv[4];  // generic per-lane constants of layers 0, 1 (r16::lv_slot)
  uint32_t lm[4];  // all-ones in lanes with lane bit 2 + i set
};

// X ^= t * Y in the lanes whose lane bit SLOT is set, t = g(2^P) ^ g(0) (the affine term of position bit P)
template <bool INVERSE, int D, const Lay& Y, int SLOT>
__device__ __forceinline__ void lane_term(uint32_t (&X)[16], const uint32_t (&Yv)[16], const Ctx& cx) {
  constexpr int P = pos_of_slot(Y, SLOT);
  if constexpr (P > D) {
    constexpr unsigned t = kCpoly16[cidx<INVERSE, D>(1 << P)] ^ kCpoly16[cidx<INVERSE, D>(0)];
    muladd_const_masked<t>(X, Yv, cx.lm[SLOT - 2]);
  }
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
    if constexpr (lane_bits_above(Y, D) > 2) {  // layers 0, 1: per-lane constant (preloaded), generic multiply
      constexpr int slot = lv_slot(INVERSE, D, R);
      muladd_lane(X, Yv, (cx.lv[slot >> 1] >> (16 * (slot & 1))) & 0xFFFFu);
    } else {  // compile-time (register and wave bits), plus one lane-masked term per lane bit above d
      constexpr int sct = (pos_r(Y, R) + pos_w(Y, OM)) & hi;
      static_assert(cidx<INVERSE, D>(sct) < kCpoly16N, "constant table too short");
      muladd_const<kCpoly16[cidx<INVERSE, D>(sct)]>(X, Yv);
      lane_term<INVERSE, D, Y, 2>(X, Yv, cx);
      lane_term<INVERSE, D, Y, 3>(X, Yv, cx);
      lane_term<INVERSE, D, Y, 4>(X, Yv, cx);
      lane_term<INVERSE, D, Y, 5>(X, Yv, cx);
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

template <bool INVERSE, int D, int R, int OM>
__device__ __forceinline__ void lv_fetch(Ctx& cx, int lane) {
  constexpr int hi = ~((2 << D) - 1);
  constexpr int base = INVERSE ? (M - 1 + (pos_r(LA, R) & hi) + (1 << D)) : ((pos_r(LA, R) & hi) + (1 << D) - 1);
  constexpr int slot = lv_slot(INVERSE, D, R);
  const uint32_t c = cx.cpoly[base + ((pos_lane(LA, lane) + pos_w(LA, OM)) & hi)];
  cx.lv[slot >> 1] |= c << (16 * (slot & 1));
}
template <int OM>
__device__ __forceinline__ void lv_fetch_all(Ctx& cx, int lane) {
#pragma unroll
  for (int i = 0; i < 4; i++) cx.lv[i] = 0;
  lv_fetch<true, 0, 0, OM>(cx, lane);
  lv_fetch<true, 0, 2, OM>(cx, lane);
  lv_fetch<true, 1, 0, OM>(cx, lane);
  lv_fetch<true, 1, 1, OM>(cx, lane);
  lv_fetch<false, 1, 0, OM>(cx, lane);
  lv_fetch<false, 1, 1, OM>(cx, lane);
  lv_fetch<false, 0, 0, OM>(cx, lane);
  lv_fetch<false, 0, 2, OM>(cx, lane);
}

// R1 <-> lane bit 2 (with swap_lane3: LB <-> LC): the partner lane ^ 4 by DPP row_ror:12 (lanes with bit 2 clear,
// partner l + 4) or row_ror:4 (bit 2 set, partner l - 4), selects on lm = all-ones in lanes with bit 2 set.
__device__ __forceinline__ uint32_t x4(uint32_t v, uint32_t lm) {
  const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12C, 0xF, 0xF, false);  // row_ror:12
  const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  return sel(lm, dn, up);
}
__device__ __forceinline__ void swap_lane2(uint32_t (&E)[4][16], uint32_t lm) {
#pragma unroll
  for (int q = 0; q < 2; q++) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t a = E[q][j], b = E[q + 2][j];
      const uint32_t recv = x4(sel(lm, a, b), lm);
      E[q][j] = sel(lm, recv, a);
      E[q + 2][j] = sel(lm, b, recv);
    }
  }
}

// (R0, R1) <-> (W0, W1) through LDS (LC <-> LD), as r16::exchange_w<0> with one other wave bit (W2): thread (w, r)
// writes key (W2, wp, r), reads key (W2, r, wp); two rounds of 8 planes, 64 KiB.
__device__ __forceinline__ void exchange2(uint32_t (&E)[4][16], uint4* xb, int w, int lane) {
  const int wp = w & 3, wo = w >> 2;
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
      E[r][8 * half + 0] = v0.x, E[r][8 * half + 1] = v0.y, E[r][8 * half + 2] = v0.z, E[r][8 * half + 3] = v0.w;
      E[r][8 * half + 4] = v1.x, E[r][8 * half + 5] = v1.y, E[r][8 * half + 6] = v1.z, E[r][8 * half + 7] = v1.w;
    }
    __syncthreads();
  }
}
// R0 <-> W2 through LDS (LD <-> LE): register r = (r1, r0) of wave w = (b = W2, wl = W1 W0) moves iff r0 != b; it
// writes key (wl, r1, r0) and reads key (wl, r1, b) -- all 16 planes in one round, 16 keys x 4 KiB = 64 KiB.
__device__ __forceinline__ void exchange1(uint32_t (&E)[4][16], uint4* xb, int w, int lane) {
  const int b = w >> 2, wl = w & 3;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    if ((r & 1) == b) continue;
    uint4* p = xb + ((((wl * 2 + (r >> 1)) * 2 + (r & 1)) * 4) * 64 + lane);
#pragma unroll
    for (int c = 0; c < 4; c++) p[c * 64] = make_uint4(E[r][4 * c], E[r][4 * c + 1], E[r][4 * c + 2], E[r][4 * c + 3]);
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; r++) {
    if ((r & 1) == b) continue;
    const uint4* p = xb + ((((wl * 2 + (r >> 1)) * 2 + b) * 4) * 64 + lane);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint4 v = p[c * 64];
      E[r][4 * c] = v.x, E[r][4 * c + 1] = v.y, E[r][4 * c + 2] = v.z, E[r][4 * c + 3] = v.w;
    }
  }
  __syncthreads();
}

// 64-B unit of one position of the half slice: chunks q = 0..3 at u*16 + 64q
template <int OM>
__device__ __forceinline__ void body(const Args& a, uint4* xb, int* s_item) {
  constexpr int w = OM;
  const int lane0 = threadIdx.x & 63;
  Ctx cx{a.cpoly, {}, {}};
#pragma unroll
  for (int i = 0; i < 4; i++) cx.lm[i] = ((lane0 >> (2 + i)) & 1) ? ~0u : 0u;
  lv_fetch_all<OM>(cx, lane0);
  // Dynamic item queue.  With a static stride the older workgroup of a CU wins the SIMDs' issue arbitration (it
  // computed an item in ~27 us, its partner in ~53 us) and finishes first; the other then runs alone on half the
  // waves (r04 phase trace, scripts/h2_trace_probe.py).  Each workgroup instead takes the next item of its
  // partition (one per XCD under round-robin dispatch: consecutive items -- the two halves of a shard slice -- are
  // read through one L2) until the partition is empty, so both workgroups of a CU stay busy to the end.
  const int G = (int)gridDim.x, bid = (int)blockIdx.x;
  const int nparts = G < 8 ? G : 8, part = bid % nparts;
  const int lo = (int)((long long)a.total * part / nparts), hi_item = (int)((long long)a.total * (part + 1) / nparts);
#if CDA_RS16_H2_STAGGER > 0
  // A/B builds: start the workgroups of the second half of the grid (the second workgroup of each CU) later, so
  // that the two workgroups of a CU begin out of phase
  if (bid >= G / 2)
    for (int i = 0; i < CDA_RS16_H2_STAGGER; i++) __builtin_amdgcn_s_sleep(127);
#endif
#if CDA_RS16_H2_SPLIT > 0
  // static split by dispatch age: the first G/2 workgroups (one per CU) take SPLIT/8 of the items
  (void)s_item, (void)lo, (void)hi_item;
  const int nf = G / 2, fast = bid < nf;
  const int nF = (int)((long long)a.total * CDA_RS16_H2_SPLIT / 8);
  const int pool_lo = fast ? 0 : nF, pool_n = fast ? nF : a.total - nF, nw = fast ? nf : G - nf;
  const int me = fast ? bid : bid - nf;
  for (int it = 0, t = me; t < pool_n; t += nw, it++) {
    const int g = pool_lo + t;
#else
  for (int it = 0;; it++) {
    if (threadIdx.x == 0) *s_item = lo + atomicAdd(&a.queue[part], 1);
    __syncthreads();  // (the previous item's reads of *s_item all precede its exchanges' barriers)
    const int g = *s_item;
    if constexpr (kMode == 1) __syncthreads();  // no exchange barriers follow in the memory-only diagnostic
    if (g >= hi_item) break;
#endif
    h2_mark(a, w, it, 0);
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" : "+v"(cx.lv[i]), "+v"(cx.lm[i]));
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int u = lane & 3;
    const int pl = pos_lane(LA, lane) + pos_w(LA, w);
    const SliceMasks km = slice_masks();
    uint32_t m1 = (lane & 2) ? ~0u : 0u;
    asm volatile("" : "+v"(m1));
    const int slice = g % a.slices;
    const int cw = (g / a.slices) % a.cw_per_blk, blk = (g / a.slices) / a.cw_per_blk;
    const long long off = (long long)slice * 256 + u * 16;
    const uint8_t* src = a.src + blk * a.src_blk + cw * a.src_cw + off;
    uint8_t* dst = a.dst + blk * a.dst_blk + cw * a.dst_cw + off;
    uint8_t* cpy = a.cpy ? a.cpy + blk * a.cpy_blk + cw * a.cpy_cw + off : nullptr;

    uint32_t E[4][16];
    uint4 q[4][4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int sh = pl + pos_r(LA, r);
      if (kMode < 2) {
        const uint4* p = reinterpret_cast<const uint4*>(src + sh * a.src_sh);
        q[r][0] = p[0], q[r][1] = p[4], q[r][2] = p[8], q[r][3] = p[12];
      } else {  // diagnostic modes >= 2: synthetic data, no loads
        q[r][0] = make_uint4(sh, lane, w, r), q[r][1] = make_uint4(lane * 3, sh ^ 5, 7, w), q[r][2] = q[r][0];
        q[r][3] = q[r][1];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      if (cpy) {
        uint4* o = reinterpret_cast<uint4*>(cpy + (pl + pos_r(LA, r)) * a.cpy_sh);
        o[0] = q[r][0], o[4] = q[r][1], o[8] = q[r][2], o[12] = q[r][3];
      }
      to_state(q[r][0], q[r][1], q[r][2], q[r][3], m1, km, E[r]);
    }
    h2_mark(a, w, it, 1);
    if (kMode != 1) {
    // IFFT, D = 1 .. m/2
    layer<LA, true, 0, OM>(E, cx);
    layer<LA, true, 1, OM>(E, cx);
    swap_lane45(E);
    layer<LB, true, 2, OM>(E, cx);
    layer<LB, true, 3, OM>(E, cx);
    swap_lane3(E, cx.lm[1]);
    swap_lane2(E, cx.lm[0]);
    layer<LC, true, 4, OM>(E, cx);
    layer<LC, true, 5, OM>(E, cx);
    exchange2(E, xb, w, lane);
    layer<LD, true, 6, OM>(E, cx);
    layer<LD, true, 7, OM>(E, cx);
    exchange1(E, xb, w, lane);
    layer<LE, true, 8, OM>(E, cx);
    // FFT, D = m/2 .. 1
    layer<LE, false, 8, OM>(E, cx);
    exchange1(E, xb, w, lane);
    layer<LD, false, 7, OM>(E, cx);
    layer<LD, false, 6, OM>(E, cx);
    exchange2(E, xb, w, lane);
    layer<LC, false, 5, OM>(E, cx);
    layer<LC, false, 4, OM>(E, cx);
    swap_lane2(E, cx.lm[0]);
    swap_lane3(E, cx.lm[1]);
    layer<LB, false, 3, OM>(E, cx);
    layer<LB, false, 2, OM>(E, cx);
    swap_lane45(E);
    layer<LA, false, 1, OM>(E, cx);
    layer<LA, false, 0, OM>(E, cx);
    }
    h2_mark(a, w, it, 2);
    if (kMode == 3) continue;
    const SliceMasks ko = slice_masks();
#pragma unroll
    for (int r = 0; r < 4; r++) {  // parity shard s = point s
      uint4 q0, q1, q2, q3;
      from_state(E[r], m1, ko, q0, q1, q2, q3);
      uint4* o = reinterpret_cast<uint4*>(dst + (pl + pos_r(LA, r)) * a.dst_sh);
      o[0] = q0, o[4] = q1, o[8] = q2, o[12] = q3;
    }
    h2_mark(a, w, it, 3);
  }
  // the last workgroup out leaves the counters zero for the next launch on this stream
  if (CDA_RS16_H2_SPLIT == 0 && threadIdx.x == 0 && atomicAdd(&a.queue[8], 1) == G - 1) {
    __threadfence();
#pragma unroll
    for (int i = 0; i < 9; i++) __hip_atomic_store(&a.queue[i], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(512, 2) rs_encode16_h2_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 xb[];  // 64 KiB: the larger exchange (32 keys x 2 KiB)
  __shared__ int s_item;
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: body<0>(a, xb, &s_item); break;
    case 1: body<1>(a, xb, &s_item); break;
    case 2: body<2>(a, xb, &s_item); break;
    case 3: body<3>(a, xb, &s_item); break;
    case 4: body<4>(a, xb, &s_item); break;
    case 5: body<5>(a, xb, &s_item); break;
    case 6: body<6>(a, xb, &s_item); break;
    default: body<7>(a, xb, &s_item); break;
  }
}

}  // namespace h2

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
                             128 * 1024) == hipSuccess &&
                 hipFuncSetAttribute((const void*)r16::h2::rs_encode16_h2_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess
             ? 0
             : -1;
}

#ifndef CDA_RS16_H2
#define CDA_RS16_H2 0  // 1: the half-slice kernel (A/B builds; measured slower)
#endif

// The half-slice kernel's item counters, one set per (device, stream): launches on one stream run in order and the
// kernel's last workgroup zeroes them, so they are zero at every launch; launches on other streams have their own.
static int* h2_queue(hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, int*> m;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  int*& p = m[{dev, s}];
  if (!p) {
    if (hipMalloc((void**)&p, 16 * sizeof(int)) != hipSuccess) return p = nullptr;
    if (hipMemsetAsync(p, 0, 16 * sizeof(int), s) != hipSuccess) {
      (void)hipFree(p);
      return p = nullptr;
    }
  }
  return p;
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
  a.trace = nullptr;
  a.queue = nullptr;
#if CDA_RS16_H2_TRACE
  if (const char* e = getenv("CDA_H2_TRACE_PTR")) a.trace = (unsigned long long*)(uintptr_t)strtoull(e, nullptr, 0);
  if (!a.trace) return -2;
#endif
  a.cw_per_blk = j.cw_per_blk;
  const bool half = CDA_RS16_H2 != 0;  // items = 256-B halves of each 512-B slice, two workgroups per CU
  a.slices = j.shard_len / (half ? 256 : 512);
  const long long total = (long long)j.nblk * j.cw_per_blk * a.slices;
  if (total <= 0 || total > 0x7FFFFFFF) return -2;
  a.total = (int)total;
  static const int ncu = [] {  // persistent workgroups: one (whole codeword) or two (half slices) per CU
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  if (half) {
    if (!(a.queue = h2_queue(s))) return -1;
    const int grid = (int)(total < 2 * ncu ? total : 2 * ncu);
    hipLaunchKernelGGL(r16::h2::rs_encode16_h2_kernel, dim3((unsigned)grid), dim3(512), 64 * 1024, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const int grid = (int)(total < ncu ? total : ncu);
  hipLaunchKernelGGL(r16::rs_encode16_reg_kernel, dim3((unsigned)grid), dim3(1024), 128 * 1024, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cda
