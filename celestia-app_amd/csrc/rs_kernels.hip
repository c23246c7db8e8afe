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
// word) and x ^= c*y becomes 64 v_bitop3 (acc ^ (y_b & mask_jb)) per 32 bytes,
// no tables in the inner loop.  The mask matrix of each butterfly constant comes
// from an 8-byte column table in constant memory; when all lanes of a wave share
// the constant (D*U >= 64) it is read through readfirstlane so the masks live in
// SGPRs (SALU), otherwise per lane.  One workgroup owns one codeword x 16 units
// (the whole 512-B shard); the m x 512-B state stays in LDS for all 2*log2(m) layers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cda_internal.h"

namespace cda {

__constant__ uint16_t c_skew8[256];
__constant__ unsigned long long c_col8[256];

// --- bit slicing -----------------------------------------------------------
// 8 words (32 bytes, little-endian) <-> 8 planes; plane j bit (8b+i) = bit j of
// byte 4i+b.  Three SWAPMOVE stages transpose the 8x8 bit blocks of each byte
// lane; the transform is an involution.
__device__ __forceinline__ void swapmove(uint32_t& a, uint32_t& b, uint32_t mask, int n) {
  uint32_t t = __builtin_amdgcn_bitop3_b32(a >> n, b, mask, 0x28);  // ((a>>n) ^ b) & mask
  b ^= t;
  a ^= t << n;
}
__device__ __forceinline__ void bitslice8(uint32_t w[8]) {
  swapmove(w[0], w[1], 0x55555555u, 1);
  swapmove(w[2], w[3], 0x55555555u, 1);
  swapmove(w[4], w[5], 0x55555555u, 1);
  swapmove(w[6], w[7], 0x55555555u, 1);
  swapmove(w[0], w[2], 0x33333333u, 2);
  swapmove(w[1], w[3], 0x33333333u, 2);
  swapmove(w[4], w[6], 0x33333333u, 2);
  swapmove(w[5], w[7], 0x33333333u, 2);
  swapmove(w[0], w[4], 0x0F0F0F0Fu, 4);
  swapmove(w[1], w[5], 0x0F0F0F0Fu, 4);
  swapmove(w[2], w[6], 0x0F0F0F0Fu, 4);
  swapmove(w[3], w[7], 0x0F0F0F0Fu, 4);
}

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
__device__ __forceinline__ void butterfly8(uint32_t* st, int U, int x, int y, int u, unsigned log_m,
                                           unsigned long long cb) {
  uint32_t X[8], Y[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    X[j] = st[(x * 8 + j) * U + u];
    Y[j] = st[(y * 8 + j) * U + u];
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
    st[(x * 8 + j) * U + u] = X[j];
    st[(y * 8 + j) * U + u] = Y[j];
  }
}

template <bool INVERSE>
__device__ __forceinline__ void rs_layer8(uint32_t* st, int m, int U, int log2U, int D, int log2D) {
  const int nbu = (m >> 1) << log2U;
  for (int bu = threadIdx.x; bu < nbu; bu += blockDim.x) {
    const int p = bu >> log2U, u = bu & (U - 1);
    const int s0 = (p >> log2D) << (log2D + 1);
    const int x = s0 | (p & (D - 1));
    const int y = x + D;
    const int idx = INVERSE ? (m - 1 + s0 + D) : (s0 + D - 1);
    if ((D << log2U) >= 64) {  // constant is wave-uniform: masks in SGPRs
      const int sidx = __builtin_amdgcn_readfirstlane(idx);
      const unsigned lm = c_skew8[sidx];
      butterfly8<INVERSE>(st, U, x, y, u, lm, c_col8[lm]);
    } else {
      const unsigned lm = c_skew8[idx];
      butterfly8<INVERSE>(st, U, x, y, u, lm, c_col8[lm]);
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
};

__global__ void __launch_bounds__(256) rs_encode8_kernel(Rs8Args a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t st[];  // [m][8][U]
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

  // load + bit-slice: element (s, u), s < m
  for (int e = threadIdx.x; e < (a.m << a.log2U); e += blockDim.x) {
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
    for (int j = 0; j < 8; j++) st[(s * 8 + j) * U + u] = w[j];
  }
  __syncthreads();
  // IFFT (data at points m..m+k-1), D = 1 .. m/2
  for (int lD = 0; lD < a.log2m; lD++) rs_layer8<true>(st, a.m, U, a.log2U, 1 << lD, lD);
  // FFT to points 0..k-1, D = m/2 .. 1
  for (int lD = a.log2m - 1; lD >= 0; lD--) rs_layer8<false>(st, a.m, U, a.log2U, 1 << lD, lD);
  // un-slice + store parity
  for (int e = threadIdx.x; e < (a.k << a.log2U); e += blockDim.x) {
    const int s = e >> a.log2U, u = e & (U - 1);
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = st[(s * 8 + j) * U + u];
    bitslice8(w);
    uint4* q = reinterpret_cast<uint4*>(dst + s * a.dst_sh + u * 32);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

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
  if (hipFuncSetAttribute((const void*)rs_encode8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024) !=
      hipSuccess)
    return -1;
  return 0;
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) l++;
  return l;
}

int launch_rs_encode8(const RsJob& j, hipStream_t s) {
  if (j.k < 1 || j.k > 128 || j.shard_len % 64 != 0) return -2;
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
  a.log2m = ilog2(j.k);
  a.m = 1 << a.log2m;
  a.cw_per_blk = j.cw_per_blk;
  const int units = j.shard_len / 32;  // even
  int U = 16;
  while (units % U) U >>= 1;
  a.U = U;
  a.log2U = ilog2(U);
  a.slices = units / U;
  const size_t lds = (size_t)a.m * 8 * U * 4;
  const long long grid = (long long)j.nblk * j.cw_per_blk * a.slices;
  if (grid <= 0 || grid > 0x7FFFFFFF) return -2;
  hipLaunchKernelGGL(rs_encode8_kernel, dim3((unsigned)grid), dim3(256), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_rs_encode16(const RsJob& j, hipStream_t s) {
  (void)j;
  (void)s;
  return -2;  // GF(2^16) path: not yet on device
}

}  // namespace cda
