// gf_slice.h — byte <-> bit-plane transposition shared by the RS encode and
// decode kernels (rs_kernels.hip, rs_decode.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cda {

// --- bit slicing -----------------------------------------------------------
// 8 words (32 bytes, little-endian) <-> 8 planes; plane j bit (8b+i) = bit j of
// byte 4i+b.  Three SWAPMOVE stages transpose the 8x8 bit blocks of each byte
// lane; the transform is an involution.
//
// Each SWAPMOVE is two shifts and two v_bitop3 selects (b' = m ? a>>n : b,
// a' = m<<n ? b<<n : a).  The six masks are held in VGPRs (SliceMasks): a VALU op
// reading an SGPR or literal issues at half rate on gfx950 (tools/valu_ubench.hip),
// and the compiler otherwise keeps the mask constants in SGPRs.
struct SliceMasks {
  uint32_t m1, m1h, m2, m2h, m4, m4h;
};
__device__ __forceinline__ SliceMasks slice_masks() {
  SliceMasks k{0x55555555u, 0xAAAAAAAAu, 0x33333333u, 0xCCCCCCCCu, 0x0F0F0F0Fu, 0xF0F0F0F0u};
  asm volatile("" : "+v"(k.m1), "+v"(k.m1h), "+v"(k.m2), "+v"(k.m2h), "+v"(k.m4), "+v"(k.m4h));
  return k;
}
__device__ __forceinline__ void swapmove(uint32_t& a, uint32_t& b, uint32_t m, uint32_t mh, int n) {
  const uint32_t nb = __builtin_amdgcn_bitop3_b32(m, a >> n, b, 0xCA);
  a = __builtin_amdgcn_bitop3_b32(mh, b << n, a, 0xCA);
  b = nb;
}
__device__ __forceinline__ void bitslice8(uint32_t w[8], const SliceMasks& k) {
  swapmove(w[0], w[1], k.m1, k.m1h, 1);
  swapmove(w[2], w[3], k.m1, k.m1h, 1);
  swapmove(w[4], w[5], k.m1, k.m1h, 1);
  swapmove(w[6], w[7], k.m1, k.m1h, 1);
  swapmove(w[0], w[2], k.m2, k.m2h, 2);
  swapmove(w[1], w[3], k.m2, k.m2h, 2);
  swapmove(w[4], w[6], k.m2, k.m2h, 2);
  swapmove(w[5], w[7], k.m2, k.m2h, 2);
  swapmove(w[0], w[4], k.m4, k.m4h, 4);
  swapmove(w[1], w[5], k.m4, k.m4h, 4);
  swapmove(w[2], w[6], k.m4, k.m4h, 4);
  swapmove(w[3], w[7], k.m4, k.m4h, 4);
}
__device__ __forceinline__ void bitslice8(uint32_t w[8]) { bitslice8(w, slice_masks()); }

}  // namespace cda
