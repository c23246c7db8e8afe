// Calibrates rocprofv3 FETCH_SIZE on gfx950 for this engine's read patterns (MI355X_MICROARCH.md §HBM: only the
// 16-B-per-lane streaming read is calibrated, at 1/2).  Each kernel reads 1 GiB once (4x the Infinity Cache) and
// writes one dword per 64 threads:
//   stream16 : lane i reads 16 B at 16*i (the calibrated pattern)
//   rec96    : lane i reads its own 96-B record (6 x 16 B), records contiguous across lanes (tree levels)
//   cell512  : lane i reads its own 512-B share (32 x 16 B) (leaf hashing)
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace`; FETCH_SIZE (KB) x 1024 / 2^30 is the reported fraction.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void stream16(const uint4* __restrict__ p, unsigned* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 v = p[i];
  const unsigned x = v.x ^ v.y ^ v.z ^ v.w;
  if ((threadIdx.x & 63) == 0 && x == 0x12345678u) out[blockIdx.x] = x;
}
__global__ void rec96(const uint4* __restrict__ p, unsigned* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = 0;
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const uint4 v = p[i * 6 + q];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if ((threadIdx.x & 63) == 0 && x == 0x12345678u) out[blockIdx.x] = x;
}
__global__ void cell512(const uint4* __restrict__ p, unsigned* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = 0;
  for (int q = 0; q < 32; q++) {
    const uint4 v = p[i * 32 + q];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if ((threadIdx.x & 63) == 0 && x == 0x12345678u) out[blockIdx.x] = x;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  uint4* p;
  unsigned* out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  (void)hipMemset(p, 1, bytes);
  for (int rep = 0; rep < 2; rep++) {
    size_t n = bytes / 16;
    hipLaunchKernelGGL(stream16, dim3((unsigned)(n / 256)), dim3(256), 0, 0, p, out, n);
    n = bytes / 96;
    hipLaunchKernelGGL(rec96, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, p, out, n);
    n = bytes / 512;
    hipLaunchKernelGGL(cell512, dim3((unsigned)(n / 256)), dim3(256), 0, 0, p, out, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("fetch_calib: 3 kernels x 2 reps, each reading %zu bytes\n", bytes);
  return 0;
}
