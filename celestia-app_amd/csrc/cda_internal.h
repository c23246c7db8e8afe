// cda_internal.h — internal declarations shared by the HIP kernels and the host engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/cda.h"

#define CDA_SHARE 512
#define CDA_REC_WORDS 24 /* 96-byte node record: 90-byte NMT node + 6 zero bytes */
#define CDA_REC_BYTES 96

// Test / diagnostic builds (-DCDA_TEST_HOOKS=1: `make hooks` -> cda/libcda_hooks.so) read the A/B switches of the
// measured experiments from the environment at cda_init / first use.  A release library contains none of
// their names and reads none of them: its only environment inputs are the deployment options
// CDA_NUMA_BIND and CDA_COPY_THREADS (cda_build_info() names them).
#ifndef CDA_TEST_HOOKS
#define CDA_TEST_HOOKS 0
#endif
#if CDA_TEST_HOOKS
#define CDA_AB_ENV(name) getenv(name)
#else
#define CDA_AB_ENV(name) ((const char*)nullptr)
#endif

namespace cda {

// Leopard field tables (product-side; built in leopard_tables.cpp).
struct LeoTables {
  int bits;
  unsigned order, modulus;
  const uint16_t* exp_t;  // [order]
  const uint16_t* log_t;  // [order]
  const uint16_t* skew;   // [modulus]
};
const LeoTables& leo_tables(int bits);
// 64-bit bit-matrix of "multiply by exp(log_m)" in GF(2^8) (Leopard representation):
// byte b = (1 << b) * exp(log_m).  log_m == 255 -> all zero (multiplier 0).
uint64_t leo8_colbits(unsigned log_m);
// 16 x 16 bit-matrix for GF(2^16): word b (uint16) = (1 << b) * exp(log_m).
void leo16_colbits(unsigned log_m, uint16_t out[16]);

// Description of one batched codeword encode launch (byte strides).
struct RsJob {
  const uint8_t* src;
  long long src_blk, src_cw, src_sh;
  uint8_t* dst;
  long long dst_blk, dst_cw, dst_sh;
  uint8_t* cpy;  // optional copy of the data shards (may be null)
  long long cpy_blk, cpy_cw, cpy_sh;
  int k;           // data shards per codeword
  int cw_per_blk;  // codewords per block
  int nblk;        // blocks
  int shard_len;   // bytes, multiple of 64
};

// launchers (return 0 on success, -1 on launch error)
int rs_init_device_tables(int device);
int rs16_init_device_tables(int device);
int rs_decode_init_device_tables(int device);
// Batched erasure decode of ncw codewords of 2k shards each (data then parity);
// shard i of codeword c at d_base + d_off[c] + i * d_stride[c]; present[c][2k].
// Missing shards are written in place.
int launch_rs_decode(uint8_t* d_base, const long long* d_off, const long long* d_stride, const uint8_t* d_present,
                     int ncw, int k, int shard_len, hipStream_t s);
int launch_rs_encode8(const RsJob& job, hipStream_t s);
int launch_rs_encode16(const RsJob& job, hipStream_t s);
// register-resident GF(2^16) encoder for k = 512 (rs16_kernels.hip)
bool rs16_reg_eligible(const RsJob& j);
// diagnostic-build tags ("" in a release build; cda_build_info)
const char* rs16_diag_tag();
const char* rs8_diag_tag();
int rs16_reg_init(int device);
int launch_rs_encode16_reg(const RsJob& j, const uint16_t* d_cpoly, hipStream_t s);
int launch_leaf_hash(const uint8_t* d_eds, void* d_leaf_nodes, unsigned long long* d_status, int k, int nblocks,
                     hipStream_t s);
int launch_nmt_level(const void* d_in, void* d_out, bool from_leaves, int k, int nblocks, int level, hipStream_t s);
// Leaf records -> all 4k roots of nblocks blocks, several levels per launch; d_levels: nblocks x 2w x w
// records of scratch for the inner levels.  prof_ctx: the cda_ctx for ProfScope (or null).
int launch_nmt_trees(const void* d_leaves, void* d_levels, void* d_roots, int k, int nblocks, hipStream_t s,
                     void* prof_ctx);
int launch_dah(const void* d_roots, void* d_dah, int n_roots_total, int nblocks, hipStream_t s);
// the batched path's DAH: digests by ceil(n / 256) workgroups per block, fold by the last (counters in d_done)
int launch_dah_wide(const void* d_roots, void* d_dah, unsigned* d_done, void* d_digests, int n, int nblocks,
                    hipStream_t s);
// every tree of nblocks blocks in one launch (LDS-resident), the DAH by the last workgroup of each block;
// d_done: nblocks zeroed counters (left zeroed); d_digests: nblocks x 4k x 32 B scratch
int launch_trees_lds(const void* d_leaves, void* d_roots, void* d_dah, unsigned* d_done, void* d_digests, int k,
                     int nblocks, hipStream_t s);
// single-axis tree (wrapper.NewConstructor tree of n leaves of 512 B)
int launch_axis_leaf(const uint8_t* d_leaves, int n, uint64_t square_size, uint64_t axis_index, void* d_nodes,
                     unsigned long long* d_status, hipStream_t s);
int launch_level_generic(const void* d_in, void* d_out, int n_in, hipStream_t s);
// Roots of ntrees independent wrapper trees of n leaves each (per-axis seam, axisq.cpp): tree t's leaves at
// d_leaves + t * tree_stride, its axis index d_axis_idx[t]; 96-B root records and status words (first bad leaf or ~0).
// One workgroup per tree with the tree in LDS: n <= kAxisRootsMaxLeaves (-2 otherwise).
constexpr int kAxisRootsMaxLeaves = 1024;
int launch_axis_roots(const uint8_t* d_leaves, long long tree_stride, int n, uint64_t square_size,
                      const unsigned long long* d_axis_idx, int ntrees, void* d_roots, unsigned long long* d_status,
                      hipStream_t s);
// roots of ntrees EDS axes (code_t = d_axes ? d_axes[t] : axis0 + t, code = axis << 24 | index) over
// leaves [leaf_off, leaf_off + nleaves) (nleaves a power of two, leaf_off a multiple of it), 96-B
// records into d_roots; d_nodes / d_scratch hold ntrees * nleaves records each.  -2: bad range.
int launch_axes_roots(const uint8_t* d_eds, int k, const int* d_axes, int axis0, int ntrees, int leaf_off, int nleaves,
                      void* d_nodes, void* d_scratch, void* d_roots, unsigned long long* d_status, hipStream_t s);
// ntrees x 2^log2n contiguous 96-B node records -> ntrees roots (d_nodes is overwritten)
int launch_nmt_fold(void* d_nodes, void* d_scratch, void* d_roots, int ntrees, int log2n, hipStream_t s);
int launch_parity_compare(const uint8_t* d_eds, int k, const int* d_axes, int naxes, const uint8_t* d_par,
                          unsigned* d_flags, hipStream_t s);
// repair verification fused: leaves, levels and root check of ntrees axis trees (one workgroup each);
// failing tree t: *d_flag = min(*d_flag, base + t), or d_flag[t] = 1 when per_tree
int launch_axes_verify(const uint8_t* d_eds, int k, const int* d_axes, int ntrees, const uint8_t* d_want_rows,
                       const uint8_t* d_want_cols, unsigned* d_flag, unsigned base, bool per_tree, hipStream_t s);
// *d_flag = min(*d_flag, base + t) for every tree t whose status is dirty or whose root differs from
// want_{rows,cols}[index] (repair's root verification without a host round trip)
int launch_roots_check(const void* d_recs, const unsigned long long* d_status, const int* d_axes, int n,
                       const uint8_t* d_want_rows, const uint8_t* d_want_cols, unsigned* d_flag, unsigned base,
                       hipStream_t s);

// Blob of a share-commitment batch (go-square inclusion.CreateCommitment), built by the host.
struct BlobDesc {
  unsigned long long data_off;  // first data byte in the call's data buffer
  uint32_t len;                 // data bytes (> 0)
  uint32_t share_off;           // first share of the blob in the call's share buffer
  uint32_t nshares;             // shares.SparseSharesNeeded(len)
  uint32_t width;               // SubTreeWidth(nshares, threshold), a power of two
  uint8_t ns[32];               // namespace (29 B); share version at [29]
};
// sparse shares of every blob, contiguous (total shares x 512 B)
int launch_blob_shares(const BlobDesc* d_desc, int nblobs, const uint8_t* d_data, uint32_t total, uint8_t* d_shares,
                       hipStream_t s);
// 96-B leaf records of shares whose namespace is their own (ns ‖ share leaves)
int launch_blob_leaves(const uint8_t* d_shares, uint32_t total, void* d_recs, hipStream_t s);
// one level of every mountain of every blob, folded in place
int launch_blob_mountain_level(const BlobDesc* d_desc, int nblobs, void* d_recs, uint32_t total, int level,
                               hipStream_t s);
// RFC-6962 root (merkle.HashFromByteSlices) of each set of 90-B node records: set s =
// records idx[off[s] .. off[s+1]) (idx == null: records off[s] ..).  out: nsets x 32 B.
// nodes_out (nsets == 1 only): every level's 32-B digests, leaves first.  -2: set too large.
// node export: level h's 90-byte nodes of trees [t0, t0 + nt) (col: column trees) into per-tree node lists
int launch_pack_tree_level(const void* d_recs, void* d_out, int log2w, int h, bool col, uint32_t t0, uint32_t nt,
                           uint32_t off_h, hipStream_t s);
int launch_merkle_sets(const void* d_recs, const uint32_t* d_idx, const uint32_t* d_off, int nsets, int max_set,
                       void* d_out, void* d_nodes_out, hipStream_t s);

// ODS of a share plan (square_kernels.hip), one thread per 16-B word; -2: empty plan
int launch_scatter_cell_runs(const void* d_compact, void* d_dst, const uint32_t* d_dst_cell, const uint32_t* d_pre,
                             int nruns, uint32_t ncells, hipStream_t s, bool same_layout = false);
int launch_build_ods(const cda_share_segment* d_segs, int nseg, const uint8_t* d_data, const uint32_t* d_reserved,
                     uint32_t nshares, void* d_ods, hipStream_t s);

struct TreeSpec {  // a set of trees for launch_tree_roots
  const void* leaves;
  unsigned long long t_stride, i_stride;  // leaf i of tree t = leaves[t * t_stride + i * i_stride] (96-B records)
  uint32_t ntrees;
  bool tree_fastest;  // node-major inner levels (consecutive trees on consecutive lanes)
  void* scratch;      // ntrees * n records
  void* roots;
  unsigned long long r_stride;
};

// profiling hook implemented by the engine
struct ProfScope {
  void* ctx;
  const char* name;
  hipStream_t stream;
  hipEvent_t a, b;
  ProfScope(void* ctx, const char* name, hipStream_t s);
  ~ProfScope();
};

}  // namespace cda
