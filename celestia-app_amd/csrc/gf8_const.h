// gf8_const.h — the Leopard GF(2^8) FFT constants as compile-time values, and X ^= C*Y on bit-planes for a
// compile-time C.
//
// The g2 encoder's P2 phase (rs_kernels.hip) keeps the top three index bits in registers, so every constant of its
// layers is a function of template parameters only.  With the constant known to the compiler the multiply is the
// 8x8 GF(2) matrix of C applied row by row (X[i] ^= XOR of the Y[j] with bit i of C*alpha^j set, two Y terms per
// v_bitop3), about 18 VALU per butterfly instead of the ~45 of the branchy runtime-constant form (gf8_mul_asm.h).
//
// The table is built by the same steps as leopard_tables.cpp (klauspost/reedsolomon v1.12.1 initConstants8 and
// initFFT8), evaluated by the compiler; rs_init_device_tables checks it entry by entry against
// the host-built table and refuses to initialise on any difference.
#pragma once
#include <stdint.h>

namespace cda {

struct Cpoly8 {
  uint8_t v[256];
};

constexpr Cpoly8 make_cpoly8() {
  constexpr unsigned kBits = 8, kOrder = 256, kMod = 255, kPoly = 0x11D;
  constexpr uint16_t kBasis[8] = {1, 214, 152, 146, 86, 200, 88, 230};
  uint16_t exp_t[256] = {}, log_t[256] = {}, skew[255] = {};
  unsigned state = 1;
  for (unsigned i = 0; i < kMod; i++) {
    exp_t[state] = (uint16_t)i;
    state <<= 1;
    if (state >= kOrder) state ^= kPoly;
  }
  exp_t[0] = kMod;
  log_t[0] = 0;
  for (unsigned i = 0; i < kBits; i++) {
    const unsigned width = 1u << i;
    for (unsigned j = 0; j < width; j++) log_t[j + width] = log_t[j] ^ kBasis[i];
  }
  for (unsigned i = 0; i < kOrder; i++) log_t[i] = exp_t[log_t[i]];
  for (unsigned i = 0; i < kOrder; i++) exp_t[log_t[i]] = (uint16_t)i;
  exp_t[kMod] = exp_t[0];
  auto add_mod = [](unsigned a, unsigned b) {
    const unsigned s = a + b;
    return (s + (s >> 8)) & 255u;
  };
  auto mul_log = [&](unsigned a, unsigned lb) -> unsigned { return a == 0 ? 0 : exp_t[add_mod(log_t[a], lb)]; };
  unsigned temp[7] = {};
  for (unsigned i = 1; i < kBits; i++) temp[i - 1] = 1u << i;
  for (unsigned m = 0; m < kBits - 1; m++) {
    const unsigned step = 1u << (m + 1);
    skew[(1u << m) - 1] = 0;
    for (unsigned i = m; i < kBits - 1; i++) {
      const unsigned s = 1u << (i + 1);
      for (unsigned j = (1u << m) - 1; j < s; j += step) skew[j + s] = skew[j] ^ (uint16_t)temp[i];
    }
    temp[m] = kMod - log_t[mul_log(temp[m], log_t[temp[m] ^ 1])];
    for (unsigned i = m + 1; i < kBits - 1; i++) temp[i] = mul_log(temp[i], add_mod(log_t[temp[i] ^ 1], temp[m]));
  }
  for (unsigned i = 0; i < kMod; i++) skew[i] = log_t[skew[i]];
  // alpha^L in the standard basis, per skew index (0 = no multiply)
  uint8_t apow[255] = {};
  unsigned st = 1;
  for (unsigned i = 0; i < kMod; i++) {
    apow[i] = (uint8_t)st;
    st <<= 1;
    if (st & 0x100) st ^= kPoly;
  }
  Cpoly8 r = {};
  for (unsigned i = 0; i < kMod; i++) r.v[i] = skew[i] >= kMod ? 0 : apow[skew[i]];
  r.v[255] = 0;
  return r;
}

inline constexpr Cpoly8 kCpoly8 = make_cpoly8();

// Row i of the multiply-by-C matrix in the standard basis: bit j set when bit i of C * alpha^j is set.
constexpr unsigned gf8_row(unsigned c, int i) {
  unsigned row = 0, v = c;
  for (int j = 0; j < 8; j++) {
    row |= ((v >> i) & 1u) << j;
    v <<= 1;
    if (v & 0x100) v ^= 0x11D;
  }
  return row;
}

constexpr int ctz8(unsigned v) {
  int n = 0;
  while (!(v & 1u)) {
    v >>= 1;
    n++;
  }
  return n;
}

__device__ __forceinline__ uint32_t xor3c(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// x ^= XOR of Y[j] over the set bits j of ROW, two terms per v_bitop3
template <unsigned ROW>
__device__ __forceinline__ void gf8_row_add(uint32_t& x, const uint32_t (&Y)[8]) {
  if constexpr (ROW != 0) {
    constexpr int j0 = ctz8(ROW);
    constexpr unsigned rest = ROW & (ROW - 1);
    if constexpr (rest == 0) {
      x ^= Y[j0];
    } else {
      x = xor3c(x, Y[j0], Y[ctz8(rest)]);
      gf8_row_add<rest & (rest - 1)>(x, Y);
    }
  }
}

// X ^= C * Y on 8 bit-planes (standard basis), C a compile-time constant
template <unsigned C>
__device__ __forceinline__ void gf8_muladd_const(uint32_t (&X)[8], const uint32_t (&Y)[8]) {
  gf8_row_add<gf8_row(C, 0)>(X[0], Y);
  gf8_row_add<gf8_row(C, 1)>(X[1], Y);
  gf8_row_add<gf8_row(C, 2)>(X[2], Y);
  gf8_row_add<gf8_row(C, 3)>(X[3], Y);
  gf8_row_add<gf8_row(C, 4)>(X[4], Y);
  gf8_row_add<gf8_row(C, 5)>(X[5], Y);
  gf8_row_add<gf8_row(C, 6)>(X[6], Y);
  gf8_row_add<gf8_row(C, 7)>(X[7], Y);
}

}  // namespace cda
