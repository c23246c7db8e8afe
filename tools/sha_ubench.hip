// Micro-benchmark: SHA-256 compression throughput on gfx950 (registers only).
// Variants: N independent chains per lane (1,2,4), occupancy via launch bounds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../celestia-app_amd/csrc/sha256_dev.h"
using namespace cda;

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

template <int N, int MINW, int SB = 0>
void run(uint32_t* d, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k_sha<N, MINW, SB>), dim3(blocks), dim3(256), 0, 0, d, 2, 1u);
  hipDeviceSynchronize();
  hipEventRecord(a);
  hipLaunchKernelGGL((k_sha<N, MINW, SB>), dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double comps = (double)blocks * 256 * N * iters;
  printf("N=%d minwaves=%d SB=%d blocks=%d: %.3f ms  %.2f Gcomp/s\n", N, MINW, SB, blocks, ms, comps / ms / 1e6);
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 1 << 26);
  int iters = 200;
  for (int blocks : {1024, 2048, 4096, 8192}) {
    run<1, 1>(d, blocks, iters);
    run<1, 4>(d, blocks, iters);
    run<1, 8>(d, blocks, iters);
    run<2, 1>(d, blocks / 2, iters);
    run<2, 4>(d, blocks / 2, iters);
    run<4, 1>(d, blocks / 4, iters);
    run<4, 2>(d, blocks / 4, iters);
    run<1, 1, 1>(d, blocks, iters);
    run<1, 8, 1>(d, blocks, iters);
    run<1, 8, 2>(d, blocks, iters);
    run<1, 8, 4>(d, blocks, iters);
    run<2, 4, 1>(d, blocks / 2, iters);
    run<2, 4, 2>(d, blocks / 2, iters);
  }
  return 0;
}
