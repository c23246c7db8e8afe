// rccl_self_probe.cpp — the RCCL calls of csrc/split.cpp on the one GPU a 1-GPU box has.
//
// The k = 512 split (cda_multi_extend_commit_split) drives G communicators from ONE thread: ncclCommInitAll over the
// handle's devices, then per step one ncclGroupStart / ncclGroupEnd holding, for every device g, hipSetDevice(g) and
// an ncclSend + ncclRecv pair per peer h on device g's stream (split.cpp exchange / gather).  RCCL refuses two ranks
// on one device ("Duplicate GPU detected", profiles/r03_rccl_same_gpu_probe.txt), so on one GPU the closest run is
// G = 1 with the peer loop covering the device itself: a grouped send / recv to self through the same calls, sizes
// and streams the split uses (the top-half block of one device at k = 512, G = 1: 256 MiB, plus the leaf-record
// block), checked byte for byte.  Prints one line; exit status 0 = every byte arrived.
//
// build: hipcc -O2 --offload-arch=gfx950 tools/rccl_self_probe.cpp -o tools/rccl_self_probe -L/opt/rocm/lib -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIPX(x)                                                                   \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 2;                                                                   \
    }                                                                             \
  } while (0)
#define NCCLX(x)                                                                  \
  do {                                                                            \
    ncclResult_t r_ = (x);                                                        \
    if (r_ != ncclSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, ncclGetErrorString(r_));                    \
      return 3;                                                                   \
    }                                                                             \
  } while (0)

__global__ void fill(uint8_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint8_t)((i * 2654435761u) ^ seed);
}
__global__ void check(const uint8_t* p, size_t n, uint32_t seed, unsigned long long* bad) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != (uint8_t)((i * 2654435761u) ^ seed)) atomicAdd(bad, 1ull);
}

int main() {
  int ver = 0;
  NCCLX(ncclGetVersion(&ver));
  int ndev = 0;
  HIPX(hipGetDeviceCount(&ndev));
  if (ndev < 1) return 4;
  std::vector<int> devs = {0};
  std::vector<ncclComm_t> comms(1);
  NCCLX(ncclCommInitAll(comms.data(), 1, devs.data()));
  HIPX(hipSetDevice(0));
  hipStream_t s;
  HIPX(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // the split's per-peer blocks at k = 512, G = 1: shares 512 x 512 x 512 B (rows x columns x share) = 128 MiB and
  // leaf records 512 x 512 x 96 B = 24 MiB; sent as two messages like split.cpp's ncclSend pair
  const size_t bsh = (size_t)512 * 512 * 512, brec = (size_t)512 * 512 * 96;
  uint8_t *sh_s, *sh_r, *rc_s, *rc_r;
  unsigned long long* bad;
  HIPX(hipMalloc(&sh_s, bsh));
  HIPX(hipMalloc(&sh_r, bsh));
  HIPX(hipMalloc(&rc_s, brec));
  HIPX(hipMalloc(&rc_r, brec));
  HIPX(hipMalloc(&bad, sizeof *bad));
  HIPX(hipMemsetAsync(bad, 0, sizeof *bad, s));
  HIPX(hipMemsetAsync(sh_r, 0, bsh, s));
  HIPX(hipMemsetAsync(rc_r, 0, brec, s));
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, sh_s, bsh, 0x51u);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, rc_s, brec, 0x77u);
  HIPX(hipGetLastError());
  float ms = 0;
  hipEvent_t a, b;
  HIPX(hipEventCreate(&a));
  HIPX(hipEventCreate(&b));
  for (int rep = 0; rep < 3; rep++) {
    HIPX(hipEventRecord(a, s));
    NCCLX(ncclGroupStart());
    for (int g = 0; g < 1; g++) {  // every device of the handle (one here), every peer h (itself)
      HIPX(hipSetDevice(devs[g]));
      for (int h = 0; h < 1; h++) {
        NCCLX(ncclSend(sh_s, bsh, ncclUint8, h, comms[g], s));
        NCCLX(ncclSend(rc_s, brec, ncclUint8, h, comms[g], s));
        NCCLX(ncclRecv(sh_r, bsh, ncclUint8, h, comms[g], s));
        NCCLX(ncclRecv(rc_r, brec, ncclUint8, h, comms[g], s));
      }
    }
    NCCLX(ncclGroupEnd());
    HIPX(hipEventRecord(b, s));
    HIPX(hipStreamSynchronize(s));
    HIPX(hipEventElapsedTime(&ms, a, b));
  }
  hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, s, sh_r, bsh, 0x51u, bad);
  hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, s, rc_r, brec, 0x77u, bad);
  unsigned long long nbad = 0;
  HIPX(hipMemcpyAsync(&nbad, bad, sizeof nbad, hipMemcpyDeviceToHost, s));
  HIPX(hipStreamSynchronize(s));
  printf("{\"rccl_version\": %d, \"devices\": %d, \"bytes\": %zu, \"self_exchange_ms\": %.3f, \"bad_bytes\": %llu}\n",
         ver, ndev, bsh + brec, ms, nbad);
  NCCLX(ncclCommDestroy(comms[0]));
  HIPX(hipFree(sh_s));
  HIPX(hipFree(sh_r));
  HIPX(hipFree(rc_s));
  HIPX(hipFree(rc_r));
  HIPX(hipFree(bad));
  return nbad == 0 ? 0 : 1;
}
