// SALU vs VALU co-issue on gfx950: the GF(2^8) bit-matrix multiply pattern.
#include <hip/hip_runtime.h>
#include <cstdio>

// variant 0: masks from s_bfe (SALU) feeding v_bitop3 with SGPR operand
// variant 1: masks precomputed in SGPRs (no SALU work per multiply)
// variant 2: only SALU (s_bfe chain), no VALU
template <int V>
__global__ void __launch_bounds__(256) k(unsigned* out, int iters, unsigned long long cb0) {
  unsigned x[8], y[8];
  for (int j = 0; j < 8; j++) { x[j] = threadIdx.x * 8 + j; y[j] = threadIdx.x ^ (j * 77); }
  unsigned long long cb = __builtin_amdgcn_readfirstlane((unsigned)cb0) | ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(cb0 >> 32)) << 32);
  unsigned sacc = 0;
  for (int it = 0; it < iters; it++) {
    const unsigned lo = (unsigned)cb, hi = (unsigned)(cb >> 32);
    if (V == 3) {  // polynomial basis: x ^= sum_{i: c_i} alpha^i y, uniform branches on c's bits
      unsigned Y[8];
#pragma unroll
      for (int j = 0; j < 8; j++) Y[j] = y[j];
      const unsigned c = __builtin_amdgcn_readfirstlane(lo & 0xFF);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (c & (1u << i)) {
#pragma unroll
          for (int j = 0; j < 8; j++) x[j] ^= Y[j];
        }
        if (i < 7) {  // Y *= alpha (poly 0x11D): taps 0,2,3,4
          const unsigned t = Y[7];
          Y[7] = Y[6]; Y[6] = Y[5]; Y[5] = Y[4]; Y[4] = Y[3] ^ t; Y[3] = Y[2] ^ t; Y[2] = Y[1] ^ t; Y[1] = Y[0]; Y[0] = t;
        }
      }
      cb = cb * 6364136223846793005ull + 1442695040888963407ull;
#pragma unroll
      for (int j = 0; j < 8; j++) y[j] ^= x[(j + 1) & 7];
      continue;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      unsigned acc = x[j];
#pragma unroll
      for (int b = 0; b < 8; b++) {
        unsigned m;
        if (V == 1) m = (b & 1) ? lo : hi;
        else m = (unsigned)(((int)((b < 4 ? lo : hi) << (31 - (8 * (b & 3) + j)))) >> 31);
        if (V == 2) sacc += m; else acc = __builtin_amdgcn_bitop3_b32(acc, y[b], m, 0x78);
      }
      x[j] = acc;
    }
    cb = cb * 6364136223846793005ull + 1442695040888963407ull;  // keep masks loop-variant
#pragma unroll
    for (int j = 0; j < 8; j++) y[j] ^= x[(j + 1) & 7];
  }
  unsigned r = sacc;
  for (int j = 0; j < 8; j++) r ^= x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int V>
void run(unsigned* d, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  int iters = 2000;
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, d, 10, 0x123456789abcdefull);
  hipDeviceSynchronize();
  hipEventRecord(a);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, d, iters, 0x123456789abcdefull);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double mults = (double)blocks * 4 * iters;  // wave-level multiplies
  printf("variant %d blocks %d: %.3f ms, %.1f ns per wave-multiply per SIMD\n", V, blocks, ms, ms * 1e6 / (mults / 1024));
}
int main() {
  unsigned* d; hipMalloc(&d, 1 << 26);
  for (int blocks : {1024, 2048, 4096}) { run<0>(d, blocks); run<1>(d, blocks); run<2>(d, blocks); run<3>(d, blocks); }
}
