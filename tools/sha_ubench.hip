// Micro-benchmark: SHA-256 compression throughput on gfx950 (registers only).
// Variants: N independent chains per lane (1,2,4), occupancy via launch bounds, and
// alternative instruction selections for the rotates and the additions:
//   ROT 0: v_alignbit_b32 (the product's sha256_dev.h)
//   ROT 1: rotr = v_lshl_or_b32(x, 32-n, x >> n)
//   ROT 2: Sigma = XOR of six shifts (two v_bitop3 + one v_xor)
//   ADD 0: compiler's choice (v_add3_u32 where it can)
//   ADD 1: two-input v_add_u32 only (inline asm keeps the compiler from forming add3)
// Results committed as profiles/r02_sha_ubench.txt.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../celestia-app_amd/csrc/sha256_dev.h"
using namespace cda;

template <int ROT>
__device__ __forceinline__ uint32_t S3(uint32_t x, int a, int b, int c) {  // rotr a ^ rotr b ^ rotr c
  if (ROT == 0) return xor3(rotr(x, a), rotr(x, b), rotr(x, c));
  if (ROT == 1) {
    auto r = [](uint32_t v, int n) {
      uint32_t o;
      asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(o) : "v"(v), "i"(32 - n), "v"(v >> n));
      return o;
    };
    return xor3(r(x, a), r(x, b), r(x, c));
  }
  const uint32_t lo = xor3(x >> a, x >> b, x >> c);
  return xor3(lo, x << (32 - a), x << (32 - b)) ^ (x << (32 - c));
}
template <int ROT>
__device__ __forceinline__ uint32_t s2sh(uint32_t x, int a, int b, int sh) {  // rotr a ^ rotr b ^ x >> sh
  if (ROT == 0) return xor3(rotr(x, a), rotr(x, b), x >> sh);
  if (ROT == 1) {
    auto r = [](uint32_t v, int n) {
      uint32_t o;
      asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(o) : "v"(v), "i"(32 - n), "v"(v >> n));
      return o;
    };
    return xor3(r(x, a), r(x, b), x >> sh);
  }
  const uint32_t lo = xor3(x >> a, x >> b, x >> sh);
  return xor3(lo, x << (32 - a), x << (32 - b));
}
template <int ADD>
__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  if (ADD == 0) return a + b;
  uint32_t o;
  asm("v_add_u32 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b));
  return o;
}

template <int ROT, int ADD>
__device__ __forceinline__ void compress_v(uint32_t s[8], uint32_t w[16]) {
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int t = 0; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t s0 = s2sh<ROT>(w[(t - 15) & 15], 7, 18, 3);
      const uint32_t s1 = s2sh<ROT>(w[(t - 2) & 15], 17, 19, 10);
      wt = add2<ADD>(add2<ADD>(w[t & 15], s0), add2<ADD>(w[(t - 7) & 15], s1));
      w[t & 15] = wt;
    }
    const uint32_t t1 = add2<ADD>(add2<ADD>(add2<ADD>(h, S3<ROT>(e, 6, 11, 25)), add2<ADD>(ch(e, f, g), K256::v[t])), wt);
    const uint32_t t2 = add2<ADD>(S3<ROT>(a, 2, 13, 22), maj(a, b, c));
    h = g;
    g = f;
    f = e;
    e = add2<ADD>(d, t1);
    d = c;
    c = b;
    b = a;
    a = add2<ADD>(t1, t2);
  }
  s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

template <int N, int MINW, int SB>
__global__ void __launch_bounds__(256, MINW) k_sha(uint32_t* out, int iters, uint32_t seed) {
  uint32_t st[N][8], w[N][16];
  for (int n = 0; n < N; n++) {
    sha256_init(st[n]);
    for (int i = 0; i < 16; i++) w[n][i] = seed ^ (threadIdx.x * 16 + i + n * 977);
  }
  for (int it = 0; it < iters; it++) {
    sha256_compress_n<N, SB>(st, w);
    for (int n = 0; n < N; n++)
      for (int i = 0; i < 8; i++) w[n][i] ^= st[n][i];
  }
  uint32_t acc = 0;
  for (int n = 0; n < N; n++)
    for (int i = 0; i < 8; i++) acc ^= st[n][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int ROT, int ADD>
__global__ void __launch_bounds__(256, 4) k_sha_v(uint32_t* out, int iters, uint32_t seed) {
  uint32_t st[8], w[16];
  sha256_init(st);
  for (int i = 0; i < 16; i++) w[i] = seed ^ (threadIdx.x * 16 + i);
  for (int it = 0; it < iters; it++) {
    compress_v<ROT, ADD>(st, w);
    for (int i = 0; i < 8; i++) w[i] ^= st[i];
  }
  uint32_t acc = 0;
  for (int i = 0; i < 8; i++) acc ^= st[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t*, int, uint32_t);
static uint32_t g_ref = 0;
void time_it(const char* label, kfn f, uint32_t* d, int blocks, int iters, int n_per_lane) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 2, 1u);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  uint32_t first = 0;
  (void)hipMemcpy(&first, d, 4, hipMemcpyDeviceToHost);
  const double comps = (double)blocks * 256 * n_per_lane * iters;
  printf("%-28s blocks=%5d: %8.3f ms  %6.2f Gcomp/s  out[0]=%08x\n", label, blocks, best, comps / best / 1e6, first);
  (void)g_ref;
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 1 << 26);
  const int iters = 200;
  for (int blocks : {2048, 8192}) {
    time_it("N=1 minw=1 (product)", k_sha<1, 1, 0>, d, blocks, iters, 1);
    time_it("N=1 minw=4", k_sha<1, 4, 0>, d, blocks, iters, 1);
    time_it("N=1 minw=8", k_sha<1, 8, 0>, d, blocks, iters, 1);
    time_it("N=2 minw=4", k_sha<2, 4, 0>, d, blocks / 2, iters, 2);
    time_it("N=1 minw=8 SB=8", k_sha<1, 8, 8>, d, blocks, iters, 1);
    time_it("ROT0 ADD0 (alignbit,add3)", k_sha_v<0, 0>, d, blocks, iters, 1);
    time_it("ROT0 ADD1 (alignbit,add)", k_sha_v<0, 1>, d, blocks, iters, 1);
    time_it("ROT1 ADD0 (lshl_or,add3)", k_sha_v<1, 0>, d, blocks, iters, 1);
    time_it("ROT1 ADD1 (lshl_or,add)", k_sha_v<1, 1>, d, blocks, iters, 1);
    time_it("ROT2 ADD0 (shifts,add3)", k_sha_v<2, 0>, d, blocks, iters, 1);
    time_it("ROT2 ADD1 (shifts,add)", k_sha_v<2, 1>, d, blocks, iters, 1);
  }
  return 0;
}
