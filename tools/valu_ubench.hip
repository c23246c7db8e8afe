// Per-instruction VALU issue cost on gfx950 (MI355X): 8 independent chains per lane,
// inline asm, 32 x 8 instructions per loop iteration.  Two occupancies: 1 wave per
// SIMD (blocks = 256 x 256 threads -> 4 waves/CU) and 8 waves per SIMD (2048 blocks).
// Output: ns per wave-instruction per SIMD and cycles at the measured clock-free
// reference (2 cyc = full rate for a wave64 on a SIMD-32 at 2.4 GHz = 0.833 ns).
// The results are committed as profiles/r02_valu_ubench.txt (backs DESIGN.md §4).
#include <hip/hip_runtime.h>
#include <cstdio>

#define BODY8(INS)                                                                                       \
  asm volatile(INS : "+v"(a0) : "v"(k0), "v"(k1)); asm volatile(INS : "+v"(a1) : "v"(k0), "v"(k1));        \
  asm volatile(INS : "+v"(a2) : "v"(k0), "v"(k1)); asm volatile(INS : "+v"(a3) : "v"(k0), "v"(k1));        \
  asm volatile(INS : "+v"(a4) : "v"(k0), "v"(k1)); asm volatile(INS : "+v"(a5) : "v"(k0), "v"(k1));        \
  asm volatile(INS : "+v"(a6) : "v"(k0), "v"(k1)); asm volatile(INS : "+v"(a7) : "v"(k0), "v"(k1));

#define KERNEL(NAME, INS)                                                                                \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, int iters) {                                \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, \
             a7 = a0 + 7;                                                                                \
    unsigned k0 = blockIdx.x, k1 = blockIdx.x * 3 + 1;                                                  \
    for (int i = 0; i < iters; i++) {                                                                    \
      BODY8(INS) BODY8(INS) BODY8(INS) BODY8(INS)                                                        \
    }                                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                  \
  }

KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_add3_same, "v_add3_u32 %0, %0, %1, %1")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")
KERNEL(k_alignbit_self, "v_alignbit_b32 %0, %0, %0, 7")
KERNEL(k_alignbit_2, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL(k_alignbit_v, "v_alignbit_b32 %0, %0, %0, %1")
KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 3")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 3, %0")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 7, %1")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 7, %1")
KERNEL(k_add_lshl, "v_add_lshl_u32 %0, %0, %1, 7")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, 3, 17")
KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL(k_fma, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_pk_add16, "v_pk_add_u16 %0, %0, %1")

// 64-bit shift of a (x, x) register pair: low word = rotr(x, n)
#define BODY8D(INS)                                                                                      \
  asm volatile(INS : "+v"(a0)); asm volatile(INS : "+v"(a1)); asm volatile(INS : "+v"(a2));            \
  asm volatile(INS : "+v"(a3)); asm volatile(INS : "+v"(a4)); asm volatile(INS : "+v"(a5));            \
  asm volatile(INS : "+v"(a6)); asm volatile(INS : "+v"(a7));
#define KERNELD(NAME, INS)                                                                               \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, int iters) {                                \
    unsigned long long a0 = threadIdx.x * 0x100000001ull, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,          \
                       a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                \
    for (int i = 0; i < iters; i++) {                                                                    \
      BODY8D(INS) BODY8D(INS) BODY8D(INS) BODY8D(INS)                                                    \
    }                                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);      \
  }
KERNELD(k_lshr64, "v_lshrrev_b64 %0, 7, %0")

#define BODY8S(INS)                                                                                      \
  asm volatile(INS : "+v"(a0) : "v"(k0), "s"(s1)); asm volatile(INS : "+v"(a1) : "v"(k0), "s"(s1));        \
  asm volatile(INS : "+v"(a2) : "v"(k0), "s"(s1)); asm volatile(INS : "+v"(a3) : "v"(k0), "s"(s1));        \
  asm volatile(INS : "+v"(a4) : "v"(k0), "s"(s1)); asm volatile(INS : "+v"(a5) : "v"(k0), "s"(s1));        \
  asm volatile(INS : "+v"(a6) : "v"(k0), "s"(s1)); asm volatile(INS : "+v"(a7) : "v"(k0), "s"(s1));
#define KERNELS(NAME, INS)                                                                               \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, int iters) {                                \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, \
             a7 = a0 + 7;                                                                                \
    unsigned k0 = blockIdx.x;                                                                            \
    unsigned s1 = __builtin_amdgcn_readfirstlane(blockIdx.x * 3 + 1);                                    \
    for (int i = 0; i < iters; i++) {                                                                    \
      BODY8S(INS) BODY8S(INS) BODY8S(INS) BODY8S(INS)                                                    \
    }                                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                  \
  }
KERNELS(k_bitop3_s, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x78")
KERNELS(k_xor_s, "v_xor_b32 %0, %2, %0")
KERNELS(k_add_s, "v_add_u32 %0, %2, %0")
KERNELS(k_add3_s, "v_add3_u32 %0, %0, %1, %2")
KERNELS(k_and_or_s, "v_and_or_b32 %0, %0, %1, %2")

typedef void (*kfn)(unsigned*, int);
void run(const char* name, kfn f, unsigned* d, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4000;
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 10);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    hipEventRecord(a);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  const double winstr = (double)blocks * 4 * iters * 32;  // wave-instructions
  const double per_simd = winstr / 1024.0;
  const double ns = best * 1e6 / per_simd;
  printf("%-18s waves/SIMD=%d  %8.3f ms  %7.1f G wave-instr/s  %.3f ns/wave-instr/SIMD  (%.2f cyc @2.4GHz)\n", name,
         blocks >= 2048 ? 8 : blocks / 256, best, winstr / best / 1e6, ns, ns * 2.4);
}

int main() {
  unsigned* d;
  hipMalloc(&d, 1 << 26);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("device %s  CUs %d  clockRate %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  struct {
    const char* n;
    kfn f;
  } ks[] = {{"v_add_u32", k_add},           {"v_add_u32_e64", k_add_e64},   {"v_xor_b32", k_xor},
            {"v_add3_u32", k_add3},         {"v_add3 (x,y,y)", k_add3_same}, {"v_bitop3_b32", k_bitop3},
            {"v_or3_b32", k_or3},           {"v_alignbit self", k_alignbit_self},
            {"v_alignbit 2src", k_alignbit_2}, {"v_alignbit vshift", k_alignbit_v}, {"v_alignbyte_b32", k_alignbyte},
            {"v_perm_b32", k_perm},         {"v_lshrrev_b32", k_lshr},      {"v_lshl_or_b32", k_lshl_or},
            {"v_lshl_add_u32", k_lshl_add}, {"v_add_lshl_u32", k_add_lshl}, {"v_xad_u32", k_xad},
            {"v_and_or_b32", k_and_or},     {"v_bfi_b32", k_bfi},           {"v_bfe_u32", k_bfe},
            {"v_mad_u32_u24", k_mad24},     {"v_fma_f32", k_fma},           {"v_pk_add_u16", k_pk_add16},
            {"v_lshrrev_b64", k_lshr64},    {"v_bitop3 +sgpr", k_bitop3_s}, {"v_xor +sgpr", k_xor_s},
            {"v_add_u32 +sgpr", k_add_s},   {"v_add3 +sgpr", k_add3_s},     {"v_and_or +sgpr", k_and_or_s}};
  for (int blocks : {256, 8192})
    for (auto& k : ks) run(k.n, k.f, d, blocks);
  return 0;
}
