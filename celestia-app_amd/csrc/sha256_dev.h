// sha256_dev.h — SHA-256 compression for gfx950 (CDNA4).
//
// The DA path spends ~75% of its instructions here.  gfx950
// has a 3-input arbitrary bitwise op (v_bitop3_b32) and a funnel shift
// (v_alignbit_b32), so one round is 14 VALU ops:
//   Σ1 = 3 alignbit + 1 bitop3(0x96), Ch = bitop3(0xCA), Σ0 = 4, Maj = bitop3(0xE8),
//   T1/T2/e/a = 2 add3 + 2 add.
// Message-schedule word: σ0/σ1 = 2 alignbit + shift + bitop3 each, 2 adds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cda {

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// Big-endian word made of bytes [off, off+4) of the little-endian 8-byte
// concatenation lo ‖ hi (lo holds bytes 0..3).  v_alignbyte_b32 computes
// ({hi,lo} >> 8*off)[31:0]; using the builtin (not a 64-bit shift) keeps
// InstCombine from turning neighbouring windows into unaligned scratch loads.
__device__ __forceinline__ uint32_t le_window(uint32_t lo, uint32_t hi, int off) {
  return off == 0 ? lo : __builtin_amdgcn_alignbyte(hi, lo, off);
}
// One v_perm_b32 picks bytes off+3, off+2, off+1, off of {hi, lo} (selector byte i = source byte of
// result byte i; 0-3 = lo, 4-7 = hi): the window and the byte swap in a single 4-cycle instruction
// instead of v_alignbyte + v_perm (profiles/r02_valu_ubench.txt).
__device__ __forceinline__ uint32_t be_window(uint32_t lo, uint32_t hi, int off) {
  const uint32_t sel = (uint32_t)(off + 3) | (uint32_t)(off + 2) << 8 | (uint32_t)(off + 1) << 16 | (uint32_t)off << 24;
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// Round constants; the unrolled rounds index this constexpr table so each K
// folds into an s_mov literal.
struct K256 {
  static constexpr uint32_t v[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
};

__device__ __forceinline__ void sha256_init(uint32_t s[8]) {
  s[0] = 0x6a09e667;
  s[1] = 0xbb67ae85;
  s[2] = 0x3c6ef372;
  s[3] = 0xa54ff53a;
  s[4] = 0x510e527f;
  s[5] = 0x9b05688c;
  s[6] = 0x1f83d9ab;
  s[7] = 0x5be0cd19;
}

// One compression of a 16-word big-endian block (w is clobbered: used as the
// rolling message schedule).
__device__ __forceinline__ void sha256_compress(uint32_t s[8], uint32_t w[16]) {
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int t = 0; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ch(e, f, g) + K256::v[t] + wt;
    uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  s[0] += a;
  s[1] += b;
  s[2] += c;
  s[3] += d;
  s[4] += e;
  s[5] += f;
  s[6] += g;
  s[7] += h;
}

// Latency path (one wave per SIMD, where a lone wave issues about one instruction per 5.4 cycles whatever its
// ILP, so a compression costs its instruction count): a block's message schedule does not depend on the chaining
// state, so an otherwise idle wave can expand it beforehand.  sha256_kw_store writes kw[t] = K[t] + W[t] for the
// 64 rounds (one LDS row of kKwStride words: node-major, 4-word writes / reads are bank-conflict free over 16
// lanes); sha256_rounds_kw then runs the 64 rounds alone: about 900 instructions instead of 1,440.
constexpr int kKwStride = 68;
__device__ __forceinline__ void sha256_kw_store(uint32_t (&w)[16], uint32_t* kw) {
#pragma unroll
  for (int t4 = 0; t4 < 16; t4++) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int t = 4 * t4 + j;
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
        const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
        wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        w[t & 15] = wt;
      }
      v[j] = wt + K256::v[t];
    }
    reinterpret_cast<uint4*>(kw)[t4] = make_uint4(v[0], v[1], v[2], v[3]);
  }
}
__device__ __forceinline__ void sha256_rounds_kw(uint32_t s[8], const uint32_t* kw) {
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int t4 = 0; t4 < 16; t4++) {
    const uint4 q = reinterpret_cast<const uint4*>(kw)[t4];
    const uint32_t kv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ch(e, f, g) + kv[j];
      const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c);
      h = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
  }
  s[0] += a;
  s[1] += b;
  s[2] += c;
  s[3] += d;
  s[4] += e;
  s[5] += f;
  s[6] += g;
  s[7] += h;
}

// N independent compressions advanced in lockstep (round-interleaved), giving
// the scheduler N independent dependency chains per wave.
template <int N, int SB = 0>
__device__ __forceinline__ void sha256_compress_n(uint32_t (&s)[N][8], uint32_t (&w)[N][16]) {
  uint32_t a[N], b[N], c[N], d[N], e[N], f[N], g[N], h[N];
#pragma unroll
  for (int n = 0; n < N; n++) {
    a[n] = s[n][0]; b[n] = s[n][1]; c[n] = s[n][2]; d[n] = s[n][3];
    e[n] = s[n][4]; f[n] = s[n][5]; g[n] = s[n][6]; h[n] = s[n][7];
  }
#pragma unroll
  for (int t = 0; t < 64; t++) {
#pragma unroll
    for (int n = 0; n < N; n++) {
      uint32_t wt;
      if (t < 16) {
        wt = w[n][t];
      } else {
        uint32_t w15 = w[n][(t - 15) & 15], w2 = w[n][(t - 2) & 15];
        uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
        uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
        wt = w[n][t & 15] + s0 + w[n][(t - 7) & 15] + s1;
        w[n][t & 15] = wt;
      }
      uint32_t t1 = h[n] + xor3(rotr(e[n], 6), rotr(e[n], 11), rotr(e[n], 25)) + ch(e[n], f[n], g[n]) + K256::v[t] + wt;
      uint32_t t2 = xor3(rotr(a[n], 2), rotr(a[n], 13), rotr(a[n], 22)) + maj(a[n], b[n], c[n]);
      h[n] = g[n];
      g[n] = f[n];
      f[n] = e[n];
      e[n] = d[n] + t1;
      d[n] = c[n];
      c[n] = b[n];
      b[n] = a[n];
      a[n] = t1 + t2;
    }
    // Optional scheduling fence every SB rounds: keeps the machine scheduler
    // from hoisting message-schedule words far ahead (register pressure).
    if (SB > 0 && (t % SB) == SB - 1) __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int n = 0; n < N; n++) {
    s[n][0] += a[n]; s[n][1] += b[n]; s[n][2] += c[n]; s[n][3] += d[n];
    s[n][4] += e[n]; s[n][5] += f[n]; s[n][6] += g[n]; s[n][7] += h[n];
  }
}

// One compression with scheduling fences every 8 rounds and after the block.
// Straight-line code with several compressions (NMT inner nodes: 3 blocks)
// otherwise lets the machine scheduler hoist later message-schedule words far
// ahead.  The fences alone do not stop IR-level passes from hoisting the child
// loads of later blocks to the top (150 VGPRs, 3 waves/SIMD); launder_after()
// below ties each load to the previous compression: 89 VGPRs, 5 waves/SIMD.
__device__ __forceinline__ void sha256_compress_fenced(uint32_t s[8], const uint32_t w[16]) {
  uint32_t S[1][8], W[1][16];
#pragma unroll
  for (int i = 0; i < 8; i++) S[0][i] = s[i];
#pragma unroll
  for (int i = 0; i < 16; i++) W[0][i] = w[i];
  sha256_compress_n<1, 8>(S, W);
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = S[0][i];
  __builtin_amdgcn_sched_barrier(0);
}

// A block whose first START message words are the constants w[0..START) and whose chaining input is s: the 64-round
// compression started from `mid`, the working state after rounds 0..START-1 (precomputed on the host for the fixed
// prefix).  The schedule still reads w[0..16) (the constant words fold into it).  s += the final working state.
template <int START, bool FENCED = true>
__device__ __forceinline__ void sha256_compress_fenced_from(uint32_t s[8], const uint32_t (&mid)[8],
                                                            uint32_t (&w)[16]) {
  uint32_t a = mid[0], b = mid[1], c = mid[2], d = mid[3], e = mid[4], f = mid[5], g = mid[6], h = mid[7];
#pragma unroll
  for (int t = START; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    const uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ch(e, f, g) + K256::v[t] + wt;
    const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
    if (FENCED && (t % 8) == 7) __builtin_amdgcn_sched_barrier(0);
  }
  s[0] += a;
  s[1] += b;
  s[2] += c;
  s[3] += d;
  s[4] += e;
  s[5] += f;
  s[6] += g;
  s[7] += h;
  if (FENCED) __builtin_amdgcn_sched_barrier(0);
}

// Opaque copy of a pointer: loads through it are neither merged with earlier
// loads of the same address (CSE) nor kept live from them.
template <typename T>
__device__ __forceinline__ const T* launder(const T* p) {
  asm volatile("" : "+v"(p));
  return p;
}
// launder(p) that also depends on `after`: loads through the result cannot be
// hoisted above the computation of `after` (e.g. the previous compression).
template <typename T>
__device__ __forceinline__ const T* launder_after(const T* p, uint32_t after) {
  asm volatile("" : "+v"(p) : "v"(after));
  return p;
}

}  // namespace cda
