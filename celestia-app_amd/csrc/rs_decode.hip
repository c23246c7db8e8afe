// rs_decode.hip — Leopard erasure decoding on gfx950 (rsmt2d LeoRSCodec.Decode
// -> klauspost/reedsolomon v1.12.1 leopardFF8/FF16 reconstruct; upstream,
// pinned go.mod:153).  Used by cda_rs_decode and by the Repair driver.
//
// Per codeword (k data, k parity, m = ceilPow2(k), n = 2m), as in the reference:
//   E = erased positions of the n-space: parity i missing -> i, i in [k, m) -> i,
//       data i missing -> m + i
//   errLocs[p] = sum_{j in E, j != p} log(p ^ j)   (mod 2^bits - 1)
//     (the reference gets the same values via two Walsh-Hadamard transforms)
//   work[p] = shard(p) * exp(errLocs[p]) for present p, 0 otherwise
//   work = FFT_DIT( FormalDerivative( IFFT_DIT(work) ) )   (skew[s + D - 1], size n)
//   missing shard(p) = work[p] * exp(-errLocs[p])
// FormalDerivative: new[x] = old[x] ^ XOR_{b: bit b of x is 0} old[x + 2^b]
// (closed form of the reference's "work[i-w..i) ^= work[i..i+w)" loop).
// The code is MDS, so the output equals any other correct decoder's; the tests
// compare it with the oracle's Lagrange decoder.
//
// Layout: one workgroup per (codeword, unit slice); state [n][PL planes][U] in LDS,
// bit-sliced and in the standard polynomial basis (see rs_kernels.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "cda_internal.h"
#include "gf_slice.h"

namespace cda {
namespace dec {

template <int PL>
struct Field;
template <>
struct Field<8> {
  static constexpr unsigned kMod = 255;
  static constexpr uint16_t phi[8] = {1, 214, 152, 146, 86, 200, 88, 230};
  static constexpr uint16_t phi_inv[8] = {1, 104, 92, 100, 114, 240, 86, 18};
  __device__ static void xtime(uint32_t (&T)[8]) {  // x^8 = x^4+x^3+x^2+1
    const uint32_t t = T[7];
#pragma unroll
    for (int i = 7; i > 0; i--) T[i] = T[i - 1];
    T[0] = t;
    T[2] ^= t;
    T[3] ^= t;
    T[4] ^= t;
  }
};
template <>
struct Field<16> {
  static constexpr unsigned kMod = 65535;
  static constexpr uint16_t phi[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                       0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
  static constexpr uint16_t phi_inv[16] = {0x0001, 0x4690, 0x65D8, 0x62D0, 0x5734, 0x45F0, 0x53B8, 0x1E38,
                                           0x7CAE, 0x4E38, 0x6708, 0xC25C, 0x7A64, 0x9EAC, 0x1124, 0x523A};
  __device__ static void xtime(uint32_t (&T)[16]) {  // x^16 = x^5+x^3+x^2+1
    const uint32_t t = T[15];
#pragma unroll
    for (int i = 15; i > 0; i--) T[i] = T[i - 1];
    T[0] = t;
    T[2] ^= t;
    T[3] ^= t;
    T[5] ^= t;
  }
};

template <int PL>
__device__ __forceinline__ void apply(uint32_t (&v)[PL], const uint16_t (&cols)[PL]) {
  uint32_t o[PL];
#pragma unroll
  for (int i = 0; i < PL; i++) {
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < PL; j++)
      if ((cols[j] >> i) & 1) acc ^= v[j];
    o[i] = acc;
  }
#pragma unroll
  for (int i = 0; i < PL; i++) v[i] = o[i];
}

// X ^= c*Y (std basis), c per lane
template <int PL>
__device__ __forceinline__ void muladd_lane(uint32_t (&X)[PL], const uint32_t (&Y)[PL], unsigned c) {
  uint32_t T[PL];
#pragma unroll
  for (int j = 0; j < PL; j++) T[j] = Y[j];
#pragma unroll
  for (int i = 0; i < PL; i++) {
    const uint32_t mk = 0u - ((c >> i) & 1u);
#pragma unroll
    for (int j = 0; j < PL; j++) X[j] = __builtin_amdgcn_bitop3_b32(X[j], T[j], mk, 0x78);
    if (i < PL - 1) Field<PL>::xtime(T);
  }
}
// X = c*Y
template <int PL>
__device__ __forceinline__ void mul_lane(uint32_t (&X)[PL], const uint32_t (&Y)[PL], unsigned c) {
#pragma unroll
  for (int j = 0; j < PL; j++) X[j] = 0;
  muladd_lane<PL>(X, Y, c);
}

// raw bytes (unit, already loaded as PL / 4 16-byte words) -> planes
template <int PL>
__device__ __forceinline__ void planes_of_raw(const uint4 (&q)[PL / 4], uint32_t (&v)[PL]) {
  if constexpr (PL == 8) {
    const uint4 a = q[0], b = q[1];
    uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    bitslice8(w);
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = w[j];
  } else {
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    uint32_t lo[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t hi[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
    bitslice8(lo);
    bitslice8(hi);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      v[j] = lo[j];
      v[(8 + j) % PL] = hi[j];
    }
  }
  apply<PL>(v, Field<PL>::phi);
}

// planes -> raw bytes (unit)
template <int PL>
__device__ __forceinline__ void store_unit(uint8_t* p, uint32_t (&v)[PL]) {
  apply<PL>(v, Field<PL>::phi_inv);
  uint4* q = reinterpret_cast<uint4*>(p);
  if (PL == 8) {
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = v[j];
    bitslice8(w);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
  } else {
    uint32_t lo[8], hi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      lo[j] = v[j];
      hi[j] = v[(8 + j) % PL];
    }
    bitslice8(lo);
    bitslice8(hi);
    q[0] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    q[1] = make_uint4(lo[4], lo[5], lo[6], lo[7]);
    q[2] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    q[3] = make_uint4(hi[4], hi[5], hi[6], hi[7]);
  }
}

struct DecArgs {
  uint8_t* base;                // shard i of codeword c at base + off[c] + i * stride[c] (+ slice/unit offset)
  const long long* off;         // [ncw]
  const long long* stride;      // [ncw]
  const uint8_t* present;       // [ncw][2k]
  const uint16_t* log_t;        // field log table (Leopard representation)
  const uint16_t* apow;         // alpha^i in the standard basis, i in [0, mod)
  const uint16_t* skew;         // FFT skew table (log values)
  int k, m, log2m, n, log2n, U, log2U, slices;
};

template <int PL>
__device__ __forceinline__ unsigned cpoly_of_log(const DecArgs& a, unsigned l) {
  return a.apow[l % Field<PL>::kMod];
}

template <int PL, bool INVERSE>
__device__ __forceinline__ void layer(uint32_t* st, const uint16_t* ctab, const DecArgs& a, int D, int log2D) {
  const int U = a.U, nU = a.n << a.log2U;
  const int nbu = (a.n >> 1) << a.log2U;
  for (int bu = threadIdx.x; bu < nbu; bu += blockDim.x) {
    const int p = bu >> a.log2U, u = bu & (U - 1);
    const int s0 = (p >> log2D) << (log2D + 1);
    const int x = s0 | (p & (D - 1));
    const int y = x + D;
    const unsigned cm = ctab[s0 + D - 1];  // alpha^skew in the standard basis, 0 = skip
    uint32_t X[PL], Y[PL];
#pragma unroll
    for (int j = 0; j < PL; j++) {
      X[j] = st[j * nU + x * U + u];
      Y[j] = st[j * nU + y * U + u];
    }
    if (INVERSE) {
#pragma unroll
      for (int j = 0; j < PL; j++) Y[j] ^= X[j];
      if (cm) muladd_lane<PL>(X, Y, cm);
    } else {
      if (cm) muladd_lane<PL>(X, Y, cm);
#pragma unroll
      for (int j = 0; j < PL; j++) Y[j] ^= X[j];
    }
#pragma unroll
    for (int j = 0; j < PL; j++) {
      st[j * nU + x * U + u] = X[j];
      st[j * nU + y * U + u] = Y[j];
    }
  }
  __syncthreads();
}

// Two consecutive layers (D and 2D) per LDS round trip: a thread holds the quad x0, x0+D, x0+2D, x0+3D of one
// unit (x0 with bits log2D and log2D+1 clear).  IFFT order: layer D then 2D; FFT order: 2D then D.  Constants as in
// layer(): group s0 + D - 1 for layer D (two groups in the quad), s0 + 2D - 1 for layer 2D (one group).
template <int PL, bool INVERSE>
__device__ __forceinline__ void bfly_lane(uint32_t (&X)[PL], uint32_t (&Y)[PL], unsigned c) {
  if (INVERSE) {
#pragma unroll
    for (int j = 0; j < PL; j++) Y[j] ^= X[j];
    if (c) muladd_lane<PL>(X, Y, c);
  } else {
    if (c) muladd_lane<PL>(X, Y, c);
#pragma unroll
    for (int j = 0; j < PL; j++) Y[j] ^= X[j];
  }
}

template <int PL, bool INVERSE>
__device__ __forceinline__ void layer4(uint32_t* st, const uint16_t* ctab, const DecArgs& a, int log2D) {
  const int U = a.U, nU = a.n << a.log2U, D = 1 << log2D;
  const int nq = (a.n >> 2) << a.log2U;
  for (int q = threadIdx.x; q < nq; q += blockDim.x) {
    const int p4 = q >> a.log2U, u = q & (U - 1);
    const int s0 = (p4 >> log2D) << (log2D + 2);
    const int x0 = s0 | (p4 & (D - 1));
    uint32_t E0[PL], E1[PL], E2[PL], E3[PL];
#pragma unroll
    for (int j = 0; j < PL; j++) {
      uint32_t* b = st + j * nU + u;
      E0[j] = b[x0 * U];
      E1[j] = b[(x0 + D) * U];
      E2[j] = b[(x0 + 2 * D) * U];
      E3[j] = b[(x0 + 3 * D) * U];
    }
    const unsigned cA = ctab[s0 + D - 1], cB = ctab[s0 + 3 * D - 1], cC = ctab[s0 + 2 * D - 1];
    if (INVERSE) {
      bfly_lane<PL, true>(E0, E1, cA);
      bfly_lane<PL, true>(E2, E3, cB);
      bfly_lane<PL, true>(E0, E2, cC);
      bfly_lane<PL, true>(E1, E3, cC);
    } else {
      bfly_lane<PL, false>(E0, E2, cC);
      bfly_lane<PL, false>(E1, E3, cC);
      bfly_lane<PL, false>(E0, E1, cA);
      bfly_lane<PL, false>(E2, E3, cB);
    }
#pragma unroll
    for (int j = 0; j < PL; j++) {
      uint32_t* b = st + j * nU + u;
      b[x0 * U] = E0[j];
      b[(x0 + D) * U] = E1[j];
      b[(x0 + 2 * D) * U] = E2[j];
      b[(x0 + 3 * D) * U] = E3[j];
    }
  }
  __syncthreads();
}

template <int PL>
__global__ void __launch_bounds__(256) rs_decode_kernel(DecArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* st = smem;  // [PL][n][U] plane-major: a wave's accesses within a plane are contiguous
  uint16_t* errl = reinterpret_cast<uint16_t*>(smem + (size_t)a.n * PL * a.U);  // [n]
  uint16_t* elist = errl + a.n;                                                // [n]
  uint16_t* ltab = elist + a.n;  // [n] log table for p ^ j < n
  uint16_t* ctab = ltab + a.n;   // [n] FFT layer constants: apow[skew[i]], 0 where skew[i] = mod (no multiply)
  __shared__ int ecount;
  const int U = a.U, nU = a.n << a.log2U;
  int wg = blockIdx.x;
  const int slice = wg % a.slices;
  const int cw = wg / a.slices;
  const uint8_t* pres = a.present + (size_t)cw * 2 * a.k;
  uint8_t* base = a.base + a.off[cw] + (long long)slice * U * (PL * 4);
  const long long sstride = a.stride[cw];

  // erasure set in n-space, gathered in parallel (its order is irrelevant: errLocs sums over it)
  if (threadIdx.x == 0) ecount = 0;
  for (int i = threadIdx.x; i < a.n; i += blockDim.x) {
    ltab[i] = a.log_t[i];
    const unsigned sk = i + 1 < a.n ? a.skew[i] : Field<PL>::kMod;  // layers read indices <= n - 2
    ctab[i] = sk == Field<PL>::kMod ? 0 : a.apow[sk];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < a.m + a.k; i += blockDim.x) {
    const bool erased = i < a.m ? (i >= a.k || !pres[a.k + i]) : !pres[i - a.m];
    if (erased) elist[atomicAdd(&ecount, 1)] = (uint16_t)i;
  }
  __syncthreads();
  const int ne = ecount;
  for (int p = threadIdx.x; p < a.m + a.k; p += blockDim.x) {
    unsigned acc = 0;  // ne < 2^11 terms below 2^16: no overflow
    int t = 0;
    // eight erasures per step: their indices and log entries are independent LDS reads issued together, not a chain
    // of dependent round trips (the sum was ~128 serial elist -> ltab pairs per thread at 50 % loss)
    for (; t + 8 <= ne; t += 8) {
      int j[8];
#pragma unroll
      for (int u = 0; u < 8; u++) j[u] = elist[t + u];
#pragma unroll
      for (int u = 0; u < 8; u++) acc += j[u] != p ? ltab[p ^ j[u]] : 0u;
    }
    for (; t < ne; t++) {
      const int j = elist[t];
      acc += j != p ? ltab[p ^ j] : 0u;
    }
    errl[p] = (uint16_t)(acc % Field<PL>::kMod);
  }
  __syncthreads();
  // work[p] = shard(p) * exp(errLocs[p]) (present), else 0.  A thread owns at most 4 items (n * U <= 1024 at the
  // launch); all of its loads are issued before the first is used, so the phase waits on memory once.
  {
    const int items = a.n << a.log2U;
    uint4 raw[4][PL / 4];
    int shard[4];
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int e = threadIdx.x + it * blockDim.x;
      shard[it] = -1;
      if (e < items) {
        const int p = e >> a.log2U, u = e & (U - 1);
        if (p < a.k) shard[it] = pres[a.k + p] ? a.k + p : -1;
        else if (p >= a.m && p < a.m + a.k) shard[it] = pres[p - a.m] ? p - a.m : -1;
        if (shard[it] >= 0) {
          const uint4* q = reinterpret_cast<const uint4*>(base + shard[it] * sstride + u * (PL * 4));
#pragma unroll
          for (int h = 0; h < PL / 4; h++) raw[it][h] = q[h];
        }
      }
    }
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int e = threadIdx.x + it * blockDim.x;
      if (e >= items) continue;
      const int p = e >> a.log2U, u = e & (U - 1);
      uint32_t v[PL];
      if (shard[it] >= 0) {
        uint32_t w[PL];
        planes_of_raw<PL>(raw[it], w);
        mul_lane<PL>(v, w, cpoly_of_log<PL>(a, errl[p]));
      } else {
#pragma unroll
        for (int j = 0; j < PL; j++) v[j] = 0;
      }
#pragma unroll
      for (int j = 0; j < PL; j++) st[j * nU + p * U + u] = v[j];
    }
  }
  __syncthreads();
  {  // IFFT: layers D = 1, 2, 4, ... (GF(2^8): two per LDS round trip; GF(2^16) keeps one, its quad
     // state would cost 180 VGPRs)
    int lD = 0;
    if (PL == 8)
      for (; lD + 1 < a.log2n; lD += 2) layer4<PL, true>(st, ctab, a, lD);
    for (; lD < a.log2n; lD++) layer<PL, true>(st, ctab, a, 1 << lD, lD);
  }
  // formal derivative (out of place through registers; <= 4 items per thread)
  {
    uint32_t nv[4][PL];
    const int items = a.n << a.log2U;
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int e = threadIdx.x + it * blockDim.x;
      if (e < items) {
        const int x = e >> a.log2U, u = e & (U - 1);
#pragma unroll
        for (int j = 0; j < PL; j++) nv[it][j] = st[j * nU + x * U + u];
        for (int b = 0; b < a.log2n; b++) {
          if ((x >> b) & 1) continue;
          const int y = x + (1 << b);
#pragma unroll
          for (int j = 0; j < PL; j++) nv[it][j] ^= st[j * nU + y * U + u];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int e = threadIdx.x + it * blockDim.x;
      if (e < items) {
        const int x = e >> a.log2U, u = e & (U - 1);
#pragma unroll
        for (int j = 0; j < PL; j++) st[j * nU + x * U + u] = nv[it][j];
      }
    }
    __syncthreads();
  }
  {  // FFT: layers D = n/2, ..., 2, 1 (GF(2^8): an odd top layer alone, then pairs (2D, D))
    int top = a.log2n - 1;
    if (PL == 8) {
      if (a.log2n & 1) {
        layer<PL, false>(st, ctab, a, 1 << top, top);
        top--;
      }
      for (; top >= 1; top -= 2) layer4<PL, false>(st, ctab, a, top - 1);
    }
    for (; top >= 0; top--) layer<PL, false>(st, ctab, a, 1 << top, top);
  }
  // reveal erasures: missing shard(p) = work[p] * exp(-errLocs[p])
  for (int e = threadIdx.x; e < (a.n << a.log2U); e += blockDim.x) {
    const int p = e >> a.log2U, u = e & (U - 1);
    int shard = -1;
    if (p < a.k) shard = pres[a.k + p] ? -1 : a.k + p;
    else if (p >= a.m && p < a.m + a.k) shard = pres[p - a.m] ? -1 : p - a.m;
    if (shard < 0) continue;
    uint32_t w[PL], v[PL];
#pragma unroll
    for (int j = 0; j < PL; j++) w[j] = st[j * nU + p * U + u];
    const unsigned l = (Field<PL>::kMod - errl[p]) % Field<PL>::kMod;
    mul_lane<PL>(v, w, cpoly_of_log<PL>(a, l));
    store_unit<PL>(base + shard * sstride + u * (PL * 4), v);
  }
}

struct Tables {
  uint16_t* log_t = nullptr;
  uint16_t* apow = nullptr;
  uint16_t* skew = nullptr;
};
static Tables g_tab[2][64];

static int upload(int device, int bits) {
  Tables& t = g_tab[bits == 16][device];
  if (t.log_t) return 0;
  const LeoTables& lt = leo_tables(bits);
  const unsigned order = lt.order, mod = lt.modulus;
  const unsigned poly = bits == 8 ? 0x11D : 0x1002D;
  std::vector<uint16_t> apow(order, 0), skew(order, (uint16_t)mod);
  unsigned s = 1;
  for (unsigned i = 0; i < mod; i++) {
    apow[i] = (uint16_t)s;
    s <<= 1;
    if (s & order) s ^= poly;
  }
  for (unsigned i = 0; i < mod; i++) skew[i] = lt.skew[i];
  void *a = nullptr, *b = nullptr, *c = nullptr;
  if (hipMalloc(&a, order * 2) != hipSuccess || hipMalloc(&b, order * 2) != hipSuccess ||
      hipMalloc(&c, order * 2) != hipSuccess)
    return -1;
  if (hipMemcpy(a, lt.log_t, order * 2, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(b, apow.data(), order * 2, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c, skew.data(), order * 2, hipMemcpyHostToDevice) != hipSuccess)
    return -1;
  t.log_t = (uint16_t*)a;
  t.apow = (uint16_t*)b;
  t.skew = (uint16_t*)c;
  return 0;
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) l++;
  return l;
}

}  // namespace dec

constexpr int kDecMaxLds = 144 * 1024;

int rs_decode_init_device_tables(int device) {
  if (device < 0 || device >= 64) return -1;
  if (dec::upload(device, 8) || dec::upload(device, 16)) return -1;
  if (hipFuncSetAttribute((const void*)dec::rs_decode_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kDecMaxLds) != hipSuccess ||
      hipFuncSetAttribute((const void*)dec::rs_decode_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kDecMaxLds) != hipSuccess)
    return -1;
  return 0;
}

int launch_rs_decode(uint8_t* d_base, const long long* d_off, const long long* d_stride, const uint8_t* d_present,
                     int ncw, int k, int shard_len, hipStream_t s) {
  if (k < 1 || k > 32768 || shard_len % 64 != 0 || ncw <= 0) return -2;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return -1;
  const bool ff16 = 2 * k > 256;
  const dec::Tables& t = dec::g_tab[ff16][dev];
  if (!t.log_t) return -1;
  dec::DecArgs a;
  a.base = d_base;
  a.off = d_off;
  a.stride = d_stride;
  a.present = d_present;
  a.log_t = t.log_t;
  a.apow = t.apow;
  a.skew = t.skew;
  a.k = k;
  a.log2m = dec::ilog2(k);
  a.m = 1 << a.log2m;
  a.n = 2 * a.m;
  a.log2n = a.log2m + 1;
  const int PL = ff16 ? 16 : 8;
  const int unit = PL * 4;  // bytes per lane unit
  const int units = shard_len / unit;
  int U = 16;
  while (U > 1 && (units % U || a.n * U > 1024)) U >>= 1;  // <= 4 derivative items per thread
  if (a.n * U > 1024) return -2;                          // n > 1024 (k > 512): not on the device path yet
  // A few codewords (the per-axis Decode, a short crossword batch) leave most CUs idle: split each codeword's bytes
  // over more workgroups (fewer units each) until the launch has 512 of them -- a workgroup's latency falls with its
  // items per thread, and the error locator it recomputes is cheap next to that.
  while (U > 1 && (long long)ncw * (units / U) < 512) U >>= 1;
  a.U = U;
  a.log2U = dec::ilog2(U);
  a.slices = units / U;
  const size_t lds = (size_t)a.n * PL * U * 4 + (size_t)a.n * 8;
  if (lds > (size_t)kDecMaxLds) return -2;
  const long long grid = (long long)ncw * a.slices;
  if (grid > 0x7FFFFFFF) return -2;
  if (ff16)
    hipLaunchKernelGGL(dec::rs_decode_kernel<16>, dim3((unsigned)grid), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(dec::rs_decode_kernel<8>, dim3((unsigned)grid), dim3(256), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cda
