// square_kernels.hip — the original data square built on the device from a share plan.
//
// go-square v1.0.1 square.Construct + shares.ToBytes (called at app/prepare_proposal.go:54,65 and
// app/process_proposal.go:121,137; go.mod:9, not vendored), restated from specs/src/specs/shares.md:
//   compact share  (TRANSACTION / PAY_FOR_BLOB namespaces):  ns ‖ info ‖ [sequence length, first share]
//                  ‖ reserved bytes (4, big-endian: offset of the first unit starting in the share, or 0)
//                  ‖ sequence bytes ‖ zeros                                               (:61-80)
//   sparse share   (blobs):  ns ‖ info ‖ [sequence length, first share] ‖ blob bytes ‖ zeros  (:31-60)
//   padding share  (namespace / reserved / tail padding):  ns ‖ 0x01 ‖ 00000000 ‖ zeros   (:82-122)
//   info byte = share_version << 1 | sequence start.
// The host only plans the layout (which tx / blob goes where, the PFB share indexes, the compact
// reserved offsets); the bytes are assembled here, one thread per 16-byte word of the square, straight
// into the ODS buffer that the extension reads next.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cda_internal.h"

namespace cda {

// segment holding share g: the last segment whose first share is <= g
__device__ __forceinline__ int find_segment(const cda_share_segment* __restrict__ s, int n, uint32_t g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s[mid].first_share <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(256) build_ods_kernel(const cda_share_segment* __restrict__ segs, int nseg,
                                                        const uint8_t* __restrict__ data,
                                                        const uint32_t* __restrict__ reserved, uint32_t nshares,
                                                        uint4* __restrict__ ods) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = (uint32_t)(gid >> 5), q = (uint32_t)(gid & 31);
  if (g >= nshares) return;
  const cda_share_segment& sg = segs[find_segment(segs, nseg, g)];
  constexpr uint32_t NS = CDA_NAMESPACE_SIZE;
  const uint32_t j = g - sg.first_share;  // share index within the segment's sequence
  const bool first = j == 0;
  const bool compact = sg.kind == CDA_SEG_COMPACT, padding = sg.kind == CDA_SEG_PADDING;
  // payload start and capacity of this share
  const uint32_t hdr = NS + 1 + (first || padding ? 4 : 0) + (compact ? 4 : 0);
  const uint32_t cap0 = CDA_SHARE - (NS + 1 + 4 + (compact ? 4 : 0));  // first share
  const uint32_t capn = CDA_SHARE - (NS + 1 + (compact ? 4 : 0));      // continuation shares
  const uint64_t pay0 = first ? 0 : cap0 + (uint64_t)(j - 1) * capn;  // sequence offset of this share's payload
  const uint32_t seqlen = padding ? 0u : (uint32_t)sg.data_len;
  const uint32_t resv = compact ? reserved[sg.reserved_off + j] : 0u;
  const uint8_t* src = data + sg.data_off;
  uint32_t w[4];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const uint32_t pos = 16 * q + 4 * t + e;
      uint32_t byte = 0;
      if (pos < NS) {
        byte = sg.ns[pos];
      } else if (pos == NS) {
        byte = (sg.share_version << 1) | (first || padding ? 1u : 0u);
      } else if ((first || padding) && pos < NS + 5) {
        byte = (seqlen >> (8 * (NS + 4 - pos))) & 0xFFu;  // sequence length, big-endian
      } else if (compact && pos < hdr) {
        byte = (resv >> (8 * (hdr - 1 - pos))) & 0xFFu;  // reserved bytes, big-endian
      } else if (!padding) {
        const uint64_t idx = pay0 + (pos - hdr);
        byte = idx < sg.data_len ? src[idx] : 0u;
      }
      v |= byte << (8 * e);
    }
    w[t] = v;
  }
  ods[(size_t)g * 32 + q] = make_uint4(w[0], w[1], w[2], w[3]);
}

int launch_build_ods(const cda_share_segment* d_segs, int nseg, const uint8_t* d_data, const uint32_t* d_reserved,
                     uint32_t nshares, void* d_ods, hipStream_t s) {
  if (nseg <= 0 || nshares == 0) return -2;
  const uint64_t threads = (uint64_t)nshares * 32;
  hipLaunchKernelGGL(build_ods_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, d_segs, nseg, d_data,
                     d_reserved, nshares, (uint4*)d_ods);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Runs of 512-B cells packed back to back in `compact` (run i = cells [pre[i], pre[i+1]) of the packed stream)
// go to cell dst_cell[i] onward of `dst`: cda_repair's upload of only the present cells.  One thread per 16-B
// word, the run found by binary search over pre (nruns + 1 entries).  SAME: `compact` is the caller's whole square
// in page-locked host memory (its device alias), laid out like `dst`; the runs are read straight from it over PCIe.
template <bool SAME>
__global__ void __launch_bounds__(256) scatter_cell_runs_kernel(const uint4* __restrict__ compact,
                                                                uint4* __restrict__ dst,
                                                                const uint32_t* __restrict__ dst_cell,
                                                                const uint32_t* __restrict__ pre, int nruns,
                                                                uint32_t nwords) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nwords) return;
  const uint32_t cell = t >> 5;
  int lo = 0, hi = nruns - 1;  // the last run with pre[i] <= cell
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= cell) lo = mid;
    else hi = mid - 1;
  }
  const size_t w = ((size_t)dst_cell[lo] + (cell - pre[lo])) * 32 + (t & 31);
  dst[w] = compact[SAME ? w : t];
}

int launch_scatter_cell_runs(const void* d_compact, void* d_dst, const uint32_t* d_dst_cell, const uint32_t* d_pre,
                             int nruns, uint32_t ncells, hipStream_t s, bool same_layout) {
  if (nruns <= 0 || ncells == 0) return 0;
  if (ncells > (1u << 26)) return -2;
  const uint32_t nwords = ncells * 32;
  if (same_layout)
    hipLaunchKernelGGL(scatter_cell_runs_kernel<true>, dim3((nwords + 255) / 256), dim3(256), 0, s,
                       (const uint4*)d_compact, (uint4*)d_dst, d_dst_cell, d_pre, nruns, nwords);
  else
    hipLaunchKernelGGL(scatter_cell_runs_kernel<false>, dim3((nwords + 255) / 256), dim3(256), 0, s,
                       (const uint4*)d_compact, (uint4*)d_dst, d_dst_cell, d_pre, nruns, nwords);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cda
