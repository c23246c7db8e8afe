// copy_bw.hip — the HBM ceilings the memory-bound kernels are measured against (bench.py "hbm_ceilings").
//
// Hand-written streaming kernels, 16 B per lane per access (global_load_dwordx4 / global_store_dwordx4), U
// independent accesses in flight per thread, over buffers 4x the 256 MB Infinity Cache:
//   copy  : dst[i] = src[i]                       (read + write: the shape of the RS encoder's traffic)
//   read  : XOR-reduce src (one dword written per wave only if it equals a magic value)
//   write : dst[i] = constant
// Each kernel is swept over U in {1, 2, 4, 8} and workgroup sizes {256, 512, 1024}; the best rate of each
// kind is reported (bytes moved = read + written bytes).  Built as tools/libcopybw.so (bench.py, ctypes) and
// tools/copy_bw (standalone, for rocprofv3).  Not part of libcda.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

template <int U>
__global__ void copy_k(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int j = 0; j < U; j++) {
    const size_t i = base + (size_t)j * blockDim.x;
    if (i < n) v[j] = src[i];
  }
#pragma unroll
  for (int j = 0; j < U; j++) {
    const size_t i = base + (size_t)j * blockDim.x;
    if (i < n) dst[i] = v[j];
  }
}

template <int U>
__global__ void read_k(const uint4* __restrict__ src, unsigned* out, size_t n) {
  const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  unsigned x = 0;
#pragma unroll
  for (int j = 0; j < U; j++) {
    const size_t i = base + (size_t)j * blockDim.x;
    if (i < n) {
      const uint4 v = src[i];
      x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (x == 0x9E3779B9u) out[blockIdx.x & 1023] = x;
}

template <int U>
__global__ void write_k(uint4* __restrict__ dst, size_t n) {
  const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  const uint4 c = make_uint4(0x01234567u, 0x89ABCDEFu, 0xFEDCBA98u, (unsigned)blockIdx.x);
#pragma unroll
  for (int j = 0; j < U; j++) {
    const size_t i = base + (size_t)j * blockDim.x;
    if (i < n) dst[i] = c;
  }
}

namespace {
#define CK(x)                          \
  do {                                 \
    if ((x) != hipSuccess) return -1;  \
  } while (0)

template <int U>
int launch(int kind, const uint4* s, uint4* d, unsigned* o, size_t n, int wg, hipStream_t st) {
  const size_t per = (size_t)wg * U;
  const unsigned grid = (unsigned)((n + per - 1) / per);
  if (kind == 0) hipLaunchKernelGGL(copy_k<U>, dim3(grid), dim3(wg), 0, st, s, d, n);
  else if (kind == 1) hipLaunchKernelGGL(read_k<U>, dim3(grid), dim3(wg), 0, st, s, o, n);
  else hipLaunchKernelGGL(write_k<U>, dim3(grid), dim3(wg), 0, st, d, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_u(int u, int kind, const uint4* s, uint4* d, unsigned* o, size_t n, int wg, hipStream_t st) {
  switch (u) {
    case 1: return launch<1>(kind, s, d, o, n, wg, st);
    case 2: return launch<2>(kind, s, d, o, n, wg, st);
    case 4: return launch<4>(kind, s, d, o, n, wg, st);
    default: return launch<8>(kind, s, d, o, n, wg, st);
  }
}
}  // namespace

extern "C" {
// out[0..2] = best copy / read / write GB/s (bytes read + written per second); cfg[0..2] = U * 10000 + workgroup
// size of each best.  bytes: buffer size (each of src, dst).  Returns 0 or -1.
int copybw_measure(int device, size_t bytes, int reps, double* out, int* cfg) {
  CK(hipSetDevice(device));
  const size_t n = bytes / 16;
  uint4 *s = nullptr, *d = nullptr;
  unsigned* o = nullptr;
  hipStream_t st;
  hipEvent_t a, b;
  CK(hipMalloc(&s, n * 16));
  CK(hipMalloc(&d, n * 16));
  CK(hipMalloc(&o, 4096));
  CK(hipMemset(s, 0x5A, n * 16));
  CK(hipMemset(d, 0, n * 16));
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int us[4] = {1, 2, 4, 8}, wgs[3] = {256, 512, 1024};
  int rc = 0;
  for (int kind = 0; kind < 3 && rc == 0; kind++) {
    out[kind] = 0;
    cfg[kind] = 0;
    const double moved = (kind == 0 ? 2.0 : 1.0) * (double)(n * 16);
    for (int ui = 0; ui < 4 && rc == 0; ui++)
      for (int wi = 0; wi < 3 && rc == 0; wi++) {
        rc = launch_u(us[ui], kind, s, d, o, n, wgs[wi], st);  // warm-up
        if (rc == 0 && hipEventRecord(a, st) != hipSuccess) rc = -1;
        for (int r = 0; r < reps && rc == 0; r++) rc = launch_u(us[ui], kind, s, d, o, n, wgs[wi], st);
        float ms = 0.f;
        if (rc == 0 && (hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
                        hipEventElapsedTime(&ms, a, b) != hipSuccess))
          rc = -1;
        if (rc == 0 && ms > 0) {
          const double gbs = moved * reps / (ms * 1e-3) / 1e9;
          if (gbs > out[kind]) {
            out[kind] = gbs;
            cfg[kind] = us[ui] * 10000 + wgs[wi];
          }
        }
      }
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipStreamDestroy(st);
  (void)hipFree(s);
  (void)hipFree(d);
  (void)hipFree(o);
  return rc;
}
}

#ifdef COPYBW_MAIN
int main(int argc, char** argv) {
  const size_t bytes = (size_t)(argc > 1 ? atoi(argv[1]) : 1024) << 20;
  double out[3];
  int cfg[3];
  if (copybw_measure(0, bytes, 10, out, cfg)) {
    fprintf(stderr, "copy_bw: HIP error\n");
    return 1;
  }
  const char* names[3] = {"copy (read+write)", "read", "write"};
  for (int i = 0; i < 3; i++)
    printf("%-18s %8.1f GB/s  (U=%d, workgroup %d)\n", names[i], out[i], cfg[i] / 10000, cfg[i] % 10000);
  return 0;
}
#endif
