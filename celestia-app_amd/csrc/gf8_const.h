// gf8_const.h — the Leopard GF(2^8) FFT constants as compile-time values, and X ^= C*Y on bit-planes for a
// compile-time C.
//
// The g2 encoder (rs_kernels.hip) keeps every index bit that a layer constant depends on in registers or in the
// wave index, and instantiates one kernel body per wave index, so every constant of every layer is a compile-time
// value.  A multiply by such a constant is its 8x8 GF(2) matrix in Leopard's own (Cantor) coordinates, emitted as a
// straight program of 3-input XORs with shared terms factored out (gf8_prog): about 14 VALU per butterfly, against
// ~45 VALU plus scalar branches for a runtime constant.
//
// The table is built by the same steps as leopard_tables.cpp (klauspost/reedsolomon v1.12.1 initConstants8 and
// initFFT8), evaluated by the compiler; rs_init_device_tables checks it entry by entry against
// the host-built table and refuses to initialise on any difference, and tests/test_gf8_prog.py checks every program
// against the oracle's Leopard multiply.
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

// ---- multiply in Leopard's own (Cantor) coordinates, with shared XOR terms ------------------------------------
// With every constant known at compile time the basis only matters through the density of the constants' matrices;
// the Cantor basis (the byte bits themselves) is within 2 % of the standard one for the FF8 constants, so the planes
// stay in Leopard's coordinates and no basis change is needed at load or store.  Leopard's x*exp(L) is
// phi^-1(alpha^L * phi(x)); column j of its matrix is phi^-1(c * phi(e_j)) with c = alpha^L in the standard basis
// (the kCpoly8 entry).
constexpr unsigned gf8_mulstd(unsigned a, unsigned b) {
  unsigned r = 0;
  while (b) {
    if (b & 1u) r ^= a;
    a <<= 1;
    if (a & 0x100u) a ^= 0x11Du;
    b >>= 1;
  }
  return r;
}
constexpr unsigned kPhi8[8] = {1, 214, 152, 146, 86, 200, 88, 230};
constexpr unsigned kPhiInv8[8] = {1, 104, 92, 100, 114, 240, 86, 18};
constexpr unsigned gf8_apply(const unsigned (&cols)[8], unsigned v) {
  unsigned r = 0;
  for (int j = 0; j < 8; j++)
    if ((v >> j) & 1u) r ^= cols[j];
  return r;
}
// row i of x -> phi^-1(c * phi(x)): bit j set when bit i of column j is set
constexpr unsigned gf8_row_cantor(unsigned c, int i) {
  unsigned row = 0;
  for (int j = 0; j < 8; j++) {
    const unsigned col = gf8_apply(kPhiInv8, gf8_mulstd(c, kPhi8[j]));
    row |= ((col >> i) & 1u) << j;
  }
  return row;
}

// X[i] ^= XOR of Y[j] over row i, as a straight-line program of 3-input XORs.  Greedy common-subexpression pass:
// while some triple of terms appears in >= 2 rows (or a pair in >= 3), one v_bitop3 makes it a temporary that those
// rows use instead (~17 % fewer VALU than row by row over the constants of a k = 128 encode).
struct Gf8Prog {
  int n;            // number of ops
  int dst[48];      // >= 0: X[dst] ^= ...; < 0: temporary value index -dst (>= 8)
  int s[48][3];     // source value indices (0..7 = Y planes, >= 8 temporaries), -1 = unused
};
constexpr Gf8Prog gf8_prog(unsigned c) {
  Gf8Prog p{};
  unsigned rows[8] = {};
  for (int i = 0; i < 8; i++) rows[i] = gf8_row_cantor(c, i);
  int nv = 8;
  for (;;) {
    int best_g = 0, bs[3] = {-1, -1, -1};
    for (int a = 0; a < nv; a++)
      for (int b = a + 1; b < nv; b++) {
        const unsigned mab = (1u << a) | (1u << b);
        int n2 = 0;
        for (int i = 0; i < 8; i++) n2 += (rows[i] & mab) == mab;
        if (n2 - 2 > best_g) {  // doubled gains: pair n*0.5-1, triple n-1
          best_g = n2 - 2;
          bs[0] = a, bs[1] = b, bs[2] = -1;
        }
        for (int d = b + 1; d < nv; d++) {
          const unsigned m3 = mab | (1u << d);
          int n3 = 0;
          for (int i = 0; i < 8; i++) n3 += (rows[i] & m3) == m3;
          if (2 * n3 - 2 > best_g) {
            best_g = 2 * n3 - 2;
            bs[0] = a, bs[1] = b, bs[2] = d;
          }
        }
      }
    if (best_g <= 0 || nv >= 24) break;
    unsigned m = (1u << bs[0]) | (1u << bs[1]) | (bs[2] >= 0 ? 1u << bs[2] : 0u);
    p.dst[p.n] = -nv;
    p.s[p.n][0] = bs[0], p.s[p.n][1] = bs[1], p.s[p.n][2] = bs[2];
    p.n++;
    for (int i = 0; i < 8; i++)
      if ((rows[i] & m) == m) rows[i] = (rows[i] & ~m) | (1u << nv);
    nv++;
  }
  for (int i = 0; i < 8; i++) {
    unsigned r = rows[i];
    while (r) {
      const int a = ctz8(r);
      r &= r - 1;
      int b = -1;
      if (r) {
        b = ctz8(r);
        r &= r - 1;
      }
      p.dst[p.n] = i;
      p.s[p.n][0] = a, p.s[p.n][1] = b, p.s[p.n][2] = -1;
      p.n++;
    }
  }
  return p;
}

template <unsigned C>
struct Gf8ProgOf {
  static constexpr Gf8Prog p = gf8_prog(C);
};

template <unsigned C, int I>
__device__ __forceinline__ void gf8_prog_run(uint32_t (&X)[8], uint32_t (&V)[24]) {
  if constexpr (I < Gf8ProgOf<C>::p.n) {
    constexpr int d = Gf8ProgOf<C>::p.dst[I];
    constexpr int a = Gf8ProgOf<C>::p.s[I][0], b = Gf8ProgOf<C>::p.s[I][1], e = Gf8ProgOf<C>::p.s[I][2];
    if constexpr (d < 0) {
      if constexpr (e >= 0)
        V[-d] = xor3c(V[a], V[b], V[e]);
      else
        V[-d] = V[a] ^ V[b];
    } else {
      if constexpr (b >= 0)
        X[d] = xor3c(X[d], V[a], V[b]);
      else
        X[d] ^= V[a];
    }
    gf8_prog_run<C, I + 1>(X, V);
  }
}

// X ^= c * Y on 8 bit-planes in Leopard's coordinates, c = alpha^L (standard basis) a compile-time constant
template <unsigned C>
__device__ __forceinline__ void gf8_muladd_cantor(uint32_t (&X)[8], const uint32_t (&Y)[8]) {
  uint32_t V[24];
#pragma unroll
  for (int j = 0; j < 8; j++) V[j] = Y[j];
  gf8_prog_run<C, 0>(X, V);
}

}  // namespace cda
