// Per-instruction VALU throughput on gfx950: 8 independent chains per lane, inline asm.
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
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_alignbit_self, "v_alignbit_b32 %0, %0, %0, 7")
KERNEL(k_alignbit_2, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 3, %0")
KERNEL(k_fma, "v_fma_f32 %0, %0, %1, %2")

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
KERNELS(k_and_or_s, "v_and_or_b32 %0, %0, %1, %2")

typedef void (*kfn)(unsigned*, int);
void run(const char* name, kfn f, unsigned* d, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int iters = 4000;
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 10);
  hipDeviceSynchronize();
  hipEventRecord(a);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double winstr = (double)blocks * 4 * iters * 32;  // wave-instructions
  double per_simd = winstr / 1024.0;
  printf("%-16s blocks=%5d  %.3f ms  %.1f G wave-instr/s  %.2f ns per wave-instr per SIMD\n", name, blocks, ms,
         winstr / ms / 1e6, ms * 1e6 / per_simd);
}

int main() {
  unsigned* d;
  hipMalloc(&d, 1 << 26);
  for (int blocks : {1024, 4096}) {
    run("v_add_u32", k_add, d, blocks);
    run("v_xor_b32", k_xor, d, blocks);
    run("v_add3_u32", k_add3, d, blocks);
    run("v_bitop3_b32", k_bitop3, d, blocks);
    run("v_alignbit self", k_alignbit_self, d, blocks);
    run("v_alignbit 2src", k_alignbit_2, d, blocks);
    run("v_lshrrev_b32", k_lshr, d, blocks);
    run("v_fma_f32", k_fma, d, blocks);
    run("v_bitop3 sgpr", k_bitop3_s, d, blocks);
    run("v_xor sgpr", k_xor_s, d, blocks);
    run("v_and_or sgpr", k_and_or_s, d, blocks);
  }
}
