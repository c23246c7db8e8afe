/*
 * cda.h — C ABI of the MI355X data-availability engine (libcda.so).
 *
 * Drop-in boundary for celestia-app's DA hot path.  Every entry
 * point takes plain pointers and sizes, returns 0 on success or a negative
 * CDA_E_* code, never aborts, and never retains a caller pointer after it
 * returns (cgo rule).  Each function cites the reference interface it replaces
 * (paths relative to the celestia-app reference tree).
 *
 * Threading: a cda_ctx serialises its own calls with an internal mutex, so the
 * entry points are re-entrant from concurrent goroutines (rsmt2d calls
 * Codec.Encode / Decode / NewTree concurrently per axis); use one ctx per OS
 * thread for parallel submission.  The device-resident entry points (..._device)
 * enqueue on the caller's stream but share the ctx's workspace: the ctx orders
 * them after its earlier work and every later call after them (events), so
 * mixing them with the synchronous calls is safe.
 */
#ifndef CDA_H
#define CDA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CDA_SHARE_SIZE 512    /* appconsts.ShareSize, pkg/appconsts/global_consts.go:29 */
#define CDA_NAMESPACE_SIZE 29 /* appconsts.NamespaceSize, global_consts.go:26 */
#define CDA_NODE_SIZE 90      /* NMT node = min ns ‖ max ns ‖ sha256 (test/util/malicious/app_test.go:58) */
#define CDA_HASH_SIZE 32

enum {
  CDA_OK = 0,
  CDA_E_NOT_POW2 = -1,     /* da.ExtendShares "number of shares is not a power of 2" (data_availability_header.go:67-69) */
  CDA_E_NOT_SQUARE = -2,   /* rsmt2d newDataSquare "number of chunks must be a square number" */
  CDA_E_SHARD_SIZE = -3,   /* LeoRSCodec.ValidateChunkSize: chunk size % 64 != 0 / uneven chunks */
  CDA_E_NS_SHORT = -4,     /* wrapper Push "data is too short to contain namespace ID" (nmt_wrapper.go:97-99) */
  CDA_E_NS_ORDER = -5,     /* nmt ErrInvalidPushOrder (leaf namespaces must be non-decreasing) */
  CDA_E_TOO_FEW = -6,      /* reedsolomon ErrTooFewShards (Decode with < k shards) */
  CDA_E_UNREPAIRABLE = -7, /* rsmt2d ErrUnrepairableDataSquare */
  CDA_E_BYZANTINE = -8,    /* rsmt2d ErrByzantineData{Axis, Index} */
  CDA_E_ARG = -9,          /* invalid argument (null pointer, k out of range, ...) */
  CDA_E_DEVICE = -10,      /* HIP runtime / device failure */
  CDA_E_PUSH_PAST = -11,   /* wrapper Push "pushed past predetermined square size" (nmt_wrapper.go:94-96) */
  CDA_E_UNSUPPORTED = -12, /* configuration not implemented on the device path */
  CDA_E_SHARE_VERSION = -13, /* x/blob ErrUnsupportedShareVersion (appconsts.SupportedShareVersions = {0}) */
  CDA_E_BLOB_SIZE = -14,     /* x/blob ErrZeroBlobSize: empty blob data (x/blob/types/payforblob.go:230-232) */
  CDA_E_NOMEM = -15,         /* host allocation failed inside the library (std::bad_alloc caught at the C ABI) */
  CDA_E_INTERNAL = -16,      /* any other C++ exception caught at the C ABI (e.g. a helper thread failed to start);
                                no exception ever crosses an entry point (app/process_proposal.go:28-34 recovers
                                Go panics only) */
};

enum { CDA_AXIS_ROW = 0, CDA_AXIS_COL = 1 }; /* rsmt2d.Row / rsmt2d.Col */

typedef struct cda_ctx cda_ctx;

/* Detail for NS_ORDER / BYZANTINE / NS_SHORT errors (mirrors rsmt2d.ErrByzantineData
 * and nmt's push-order error: which axis/index and which leaf). */
typedef struct {
  int32_t code;
  int32_t axis;  /* CDA_AXIS_ROW / CDA_AXIS_COL, or -1 */
  int32_t index; /* axis index, or -1 */
  int32_t leaf;  /* leaf (share) index within the axis, or -1 */
  int32_t block; /* block index within a batch, or -1 */
} cda_err_info;

/* ---- context ---------------------------------------------------------- */
/* Creates a context bound to HIP device `device` (one process per GPU). */
int cda_init(int device, cda_ctx** out);
void cda_free(cda_ctx* ctx);
const char* cda_strerror(int code);
/* Last HIP error string recorded by the context (for CDA_E_DEVICE). */
const char* cda_last_device_error(cda_ctx* ctx);
/* "release gfx950", or "diagnostic gfx950 <tags>" for a library built with a diagnostic define that changes what
 * the kernels compute (timing experiments only; no environment variable can do that to a release build). */
const char* cda_build_info(void);
/* Per-context options (default 0).  CDA_OPT_HUGE_PAGES = 1: when the one-block path gets a fresh, never-touched
 * pageable EDS buffer, madvise(MADV_HUGEPAGE) its 2 MiB-aligned interior before faulting it in (faster first touch,
 * but it changes the page policy of caller memory -- under cgo, Go heap; off unless asked for).  CDA_E_ARG for an
 * unknown option. */
enum { CDA_OPT_HUGE_PAGES = 1 };
int cda_set_option(cda_ctx* ctx, int option, int64_t value);

/* ---- rsmt2d.Codec (LeoRSCodec replacement) ---------------------------- */
/* Replaces rsmt2d.LeoRSCodec selected by appconsts.DefaultCodec
 * (pkg/appconsts/global_consts.go:92).  Leopard GF(2^8) for 2k <= 256, GF(2^16) above. */
/* Codec.Encode(data [][]byte) ([][]byte, error): k data shards (contiguous,
 * k*shard_len bytes) -> k parity shards (k*shard_len). */
int cda_rs_encode(cda_ctx* ctx, uint32_t k, uint32_t shard_len, const uint8_t* data, uint8_t* parity);
/* Codec.Decode(shards [][]byte) ([][]byte, error): shards = 2k*shard_len bytes
 * (data then parity), present[i] != 0 marks available shards; missing shards are
 * reconstructed in place.  CDA_E_TOO_FEW if fewer than k are present. */
int cda_rs_decode(cda_ctx* ctx, uint32_t k, uint32_t shard_len, uint8_t* shards, const uint8_t* present);
/* Codec.MaxChunks() */
int64_t cda_rs_max_chunks(void);
/* Codec.Name() -> "Leopard" */
const char* cda_rs_name(void);
/* Codec.ValidateChunkSize(int) error */
int cda_rs_validate_chunk_size(int64_t chunk_size);

/* ---- block path: da.ExtendShares + da.NewDataAvailabilityHeader -------- */
/* Replaces da.ExtendShares (pkg/da/data_availability_header.go:65-75) followed by
 * da.NewDataAvailabilityHeader (:44-63) and DataAvailabilityHeader.Hash (:92-108).
 * shares: `count` shares of share_len bytes, row-major ODS (count must be a
 * power of two and a perfect square, k = sqrt(count)).
 * eds_or_null: 4k^2*share_len bytes row-major EDS, or NULL to skip the copy-out.
 * row_roots / col_roots: 2k*90 bytes each.  dah: 32 bytes. */
int cda_extend_commit(cda_ctx* ctx, uint32_t count, uint32_t share_len, const uint8_t* shares,
                      uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                      cda_err_info* err);

/* Batched form: nblocks independent ODS of k*k shares each, stride k*k*share_len;
 * outputs strided the same way (eds: 4k^2*share_len per block, roots 2k*90, dah 32). */
int cda_extend_commit_batch(cda_ctx* ctx, uint32_t k, uint32_t nblocks, const uint8_t* ods,
                            uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                            cda_err_info* err);

/* In-place form of cda_extend_commit for one k x k square: `eds` (4k^2*512 bytes, row-major) holds the ODS in its
 * top-left quadrant Q0 (row r of the ODS at eds + r*2k*512); the call writes Q1..Q3 around it and returns the roots
 * and DAH as cda_extend_commit.  rsmt2d's ComputeExtendedDataSquare builds the same square from the shares
 * (pkg/da/data_availability_header.go:74); go/cda's ExtendShares flattens the shares straight into Q0 of a pooled
 * page-locked EDS slab and calls this, so there is no separate share buffer and no host copy of Q0. */
int cda_extend_commit_eds(cda_ctx* ctx, uint32_t k, uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots,
                          uint8_t* dah, cda_err_info* err);

/* Host buffers are streamed through the GPU in chunks: H2D of chunk i+1, the extension and trees
 * of chunk i and D2H of chunk i-1 overlap on three streams (PCIe full duplex).  Pageable memory
 * works; memory from cda_host_alloc (pinned) avoids the runtime's staging copies. */

/* Pinned host memory for share / EDS buffers (hipHostMalloc); free with cda_host_free. */
int cda_host_alloc(cda_ctx* ctx, size_t bytes, void** out);
int cda_host_free(cda_ctx* ctx, void* p);
/* Page-lock caller memory for reuse as share / EDS buffers (hipHostRegister): go/cda's buffer pools register Go-heap
 * slabs once and recycle them through the garbage collector, so the consensus path's copies are direct DMAs
 * (app/prepare_proposal.go:65, app/process_proposal.go:137, app/extend_block.go:25 through da.ExtendShares).
 * The runtime keeps the registered address after this call returns.  For Go memory that stretches cgo's rule that C
 * keeps no Go pointer: it is sound only because the gc toolchain's heap never moves an object (go/cda/pool.go states
 * the invariant; a slab is unregistered before the pool drops it and never freed while registered).  Unregister only
 * after the last call that used the range has returned (unregister first drains this context's compute, H2D, D2H
 * and auxiliary streams). */
int cda_host_register(cda_ctx* ctx, void* p, size_t bytes);
int cda_host_unregister(cda_ctx* ctx, void* p);

/* ---- multi-device batch (SURVEY.md §8b "batch ... plus a device mask", §8e) ----
 * One handle over the GPUs in `device_mask` (bit d = HIP device d; 0 = all visible devices), one
 * cda_ctx per device.  cda_multi_extend_commit_batch shards the nblocks independent blocks into
 * contiguous ranges, one per device, each streamed by its own host thread (no collective: blocks are
 * independent).  Buffers and errors as cda_extend_commit_batch; err->block is the global block index
 * of the lowest failing block. */
typedef struct cda_multi cda_multi;
int cda_multi_init(uint32_t device_mask, cda_multi** out);
void cda_multi_free(cda_multi* m);
int cda_multi_device_count(const cda_multi* m);
/* The per-device context i (0-based, in device order) for the single-device entry points. */
cda_ctx* cda_multi_context(cda_multi* m, int i);
/* HIP device id of the handle's device i (0-based, in device order), or -1. */
int cda_multi_device(const cda_multi* m, int i);
int cda_multi_extend_commit_batch(cda_multi* m, uint32_t k, uint32_t nblocks, const uint8_t* ods,
                                  uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                                  cda_err_info* err);

/* ---- one square split over the handle's devices ----
 * da.ExtendShares + NewDataAvailabilityHeader (pkg/da/data_availability_header.go:44-75) of ONE k x k square
 * (k up to 512: appconsts/testground SquareSizeUpperBound, pkg/appconsts/testground/app_consts.go:8) over the G
 * devices of `m` (G a power of two dividing k): device g row-encodes ODS rows [g k/G, (g+1) k/G), one RCCL exchange
 * (ncclSend / ncclRecv pairs in one group, communicators from ncclCommInitAll) hands every device the top half of
 * its 2k/G columns with their leaf records, each device column-encodes and roots its columns and the bottom rows'
 * subtrees over them, and device 0 folds those and hashes the DAH.  Outputs and errors as cda_extend_commit
 * (ods: k*k*512 bytes row-major; eds_or_null: 4k^2*512, gathered from the devices). */
int cda_multi_extend_commit_split(cda_multi* m, uint32_t k, const uint8_t* ods, uint8_t* eds_or_null,
                                  uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, cda_err_info* err);
/* The same with the ODS already on the devices: d_ods_slabs[g] = device memory of device g holding ODS rows
 * [g k/G, (g+1) k/G) (k/G * k * 512 bytes).  The EDS stays on the devices (in the handle's workspace). */
int cda_multi_extend_commit_split_device(cda_multi* m, uint32_t k, const void* const* d_ods_slabs, uint8_t* row_roots,
                                         uint8_t* col_roots, uint8_t* dah, cda_err_info* err);
/* A handle of `count` contexts on ONE device whose split exchanges are device-to-device copies instead of RCCL:
 * the same plan and kernels for G = 2, 4, 8 on a single GPU (tests, rehearsal).  Free with cda_multi_free. */
int cda_multi_init_replicas(int device, uint32_t count, cda_multi** out);

/* Device-resident form (pointers are device memory of this ctx's GPU; `stream`
 * is a hipStream_t or NULL for the null stream).  Asynchronous: returns after
 * enqueueing; namespace-order errors are reported into the device word
 * `d_status` (uint64 per block: all-ones = ok, else the first namespace-order
 * violation packed as axis << 40 | axis_index << 20 | leaf) for the caller to read.
 * d_roots: nblocks * 4k * 96 bytes (row roots then col roots, 90-B node + 6 zero
 * bytes per record).  d_dah: nblocks * 32. */
int cda_extend_commit_device(cda_ctx* ctx, uint32_t k, uint32_t nblocks, const void* d_ods, void* d_eds,
                             void* d_roots, void* d_dah, void* d_status, void* stream);

/* ---- device-resident building blocks (one square split over GPUs) ----
 * All pointers are device memory of this ctx's GPU; asynchronous on `stream`
 * (hipStream_t or NULL).  They share the ctx's scratch workspace, so calls on
 * different streams of one ctx must be ordered by the caller. */

/* Batched strided Codec.Encode: for codeword c < ncw, data shard i at
 * d_src + c*src_cw + i*src_sh, parity shard i written to d_dst + c*dst_cw + i*dst_sh
 * (byte strides).  The rows of rsmt2d erasureExtendSquare are (src_cw = row
 * pitch, src_sh = shard_len), its columns (src_cw = shard_len, src_sh = row pitch). */
int cda_rs_encode_device(cda_ctx* ctx, uint32_t k, uint32_t shard_len, uint32_t ncw, const void* d_src, int64_t src_cw,
                         int64_t src_sh, void* d_dst, int64_t dst_cw, int64_t dst_sh, void* stream);

/* Erasured-NMT roots of `naxes` consecutive axes (axis = CDA_AXIS_ROW/COL,
 * indices first_index ..) of a 2k x 2k row-major EDS `d_eds` (512-B shares; only
 * the cells read are needed), over leaves [leaf_off, leaf_off + nleaves):
 * nleaves = 2k gives the axis root (eds.RowRoots / ColRoots, nmt_wrapper.go:118-124);
 * an aligned power-of-two sub-range gives the root of that subtree, which the
 * split-square path folds across GPUs.  d_roots: naxes 96-B records (90-B node +
 * 6 zero bytes).  d_status: naxes uint64, all-ones or the first leaf index whose
 * Push order check failed (nmt ErrInvalidPushOrder). */
int cda_nmt_roots_device(cda_ctx* ctx, uint32_t k, const void* d_eds, uint32_t axis, uint32_t first_index,
                         uint32_t naxes, uint32_t leaf_off, uint32_t nleaves, void* d_roots, void* d_status,
                         void* stream);

/* ntrees x n (power of two) contiguous 96-B node records -> ntrees root records
 * (NmtHasher.HashNode levels, test/util/malicious/hasher.go:271-310). */
int cda_nmt_fold_device(cda_ctx* ctx, uint32_t ntrees, uint32_t n, const void* d_nodes, void* d_roots, void* stream);

/* DataAvailabilityHeader.Hash over n_total 96-B root records (row roots then
 * column roots) -> 32 B (pkg/da/data_availability_header.go:92-108). */
int cda_dah_device(cda_ctx* ctx, uint32_t n_total, const void* d_roots, void* d_dah, void* stream);

/* Roots + DAH of an existing EDS (rsmt2d eds.RowRoots/ColRoots + DAH hash). */
int cda_commit_eds(cda_ctx* ctx, uint32_t k, const uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots,
                   uint8_t* dah, cda_err_info* err);

/* DataAvailabilityHeader.Hash() over given roots (RFC-6962, go-square/merkle
 * HashFromByteSlices over rowRoots ‖ colRoots; n roots per axis, 90 B each). */
int cda_dah_hash(cda_ctx* ctx, uint32_t n, const uint8_t* row_roots, const uint8_t* col_roots, uint8_t* dah);

/* ---- wrapper.NewConstructor tree (rsmt2d.TreeConstructorFn) ------------ */
/* Root of one erasured NMT axis: replaces ErasuredNamespacedMerkleTree
 * Push x n + Root (pkg/wrapper/nmt_wrapper.go:93-124) for square size k and
 * axis index `axis_index`.  leaves: n * leaf_len bytes. */
int cda_nmt_axis_root(cda_ctx* ctx, uint64_t square_size, uint64_t axis_index, uint32_t n, uint32_t leaf_len,
                      const uint8_t* leaves, uint8_t* root, cda_err_info* err);

/* ---- rsmt2d Repair ------------------------------------------------------ */
/* Replaces (*rsmt2d.ExtendedDataSquare).Repair(rowRoots, colRoots): eds is the
 * 4k^2*share_len square with missing cells marked by present[r*2k+c] == 0;
 * repaired in place (present updated).  Returns CDA_OK, CDA_E_UNREPAIRABLE or
 * CDA_E_BYZANTINE (err->axis/index). */
int cda_repair(cda_ctx* ctx, uint32_t k, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
               const uint8_t* col_roots, cda_err_info* err);
/* The same on a square already in device memory of this ctx's GPU (d_eds, 4k^2*512 bytes, repaired
 * in place; e.g. assembled there by a sampling / reconstruction pipeline, or the output of
 * cda_extend_commit_device).  present / roots / err are host memory.  Ordered after prior work on
 * `stream` (0 = the null stream); returns when the repair is complete. */
int cda_repair_device(cda_ctx* ctx, uint32_t k, void* d_eds, uint8_t* present, const uint8_t* row_roots,
                      const uint8_t* col_roots, cda_err_info* err, void* stream);

/* ---- blob share commitments (x/blob, go-square inclusion) -------------- */
/* inclusion.CreateCommitments(blobs, merkle.HashFromByteSlices, threshold)
 * (x/blob/types/payforblob.go:53; CreateCommitment per blob in ValidateBlobTx,
 * blob_tx.go:97-105).  Blob b = namespace namespaces[29b, 29b+29) and data
 * data[offsets[b], offsets[b+1]); share_versions may be NULL (all 0).
 * commitments: nblobs x 32 B.  Errors name the blob in err->index, checked in
 * ValidateBlobs' order (payforblob.go:230-236): CDA_E_BLOB_SIZE, CDA_E_SHARE_VERSION. */
int cda_blob_commitments(cda_ctx* ctx, uint32_t nblobs, const uint8_t* namespaces, const uint8_t* data,
                         const uint64_t* offsets, const uint8_t* share_versions, uint32_t subtree_root_threshold,
                         uint8_t* commitments, cda_err_info* err);

/* merkle.HashFromByteSlices over sets of 90-B NMT nodes (the subtree-root fold of
 * pkg/inclusion/get_commit.go:29): set s = items[off[s]-off[0], off[s+1]-off[0]);
 * roots: nsets x 32 B; an empty set hashes to SHA256("").  item_len must be 90. */
int cda_merkle_roots(cda_ctx* ctx, uint32_t nsets, const uint32_t* set_offsets, const uint8_t* items,
                     uint32_t item_len, uint8_t* roots);

/* ---- NMT node export and share inclusion proofs (pkg/inclusion, pkg/proof) ---- */
/* cda_extend_commit plus every node of the trees the block path builds: what the
 * inner-node cache of pkg/inclusion/nmt_caching.go:76-124 records through nmt's
 * NodeVisitor, and what pkg/proof/proof.go:82-153 recomputes for proofs.
 * row_nodes / col_nodes (optional): 2k trees x (4k-1) nodes x 90 B; per tree the
 * 2k leaves first, then each level, the root last.  dah_nodes (optional):
 * (8k-1) x 32 B, the RFC-6962 tree over rowRoots ‖ colRoots, leaf hashes first,
 * the data root last. */
int cda_extend_commit_nodes(cda_ctx* ctx, uint32_t count, uint32_t share_len, const uint8_t* shares,
                            uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                            uint8_t* row_nodes, uint8_t* col_nodes, uint8_t* dah_nodes, cda_err_info* err);

typedef struct {
  uint32_t start_row, end_row; /* RowProof.StartRow / EndRow */
  uint32_t nrows;              /* end_row - start_row + 1 */
  uint32_t total;              /* Proof.Total = 4k (rowRoots ‖ colRoots) */
  uint32_t naunts;             /* aunts per row proof = log2(4k) */
  uint32_t max_nodes;          /* node slots per row in nmt_nodes = 2 log2(2k) */
} cda_share_proof_info;

/* pkg/proof NewShareInclusionProof (proof.go:55-167) for the ODS shares
 * [start, end) of the k x k square `shares` (count = k*k).  Per proven row i
 * (capacity k rows): row_roots 90 B; the row root's RFC-6962 proof in the data
 * root (merkle.ProofsFromByteSlices, :82-93): leaf_hashes 32 B, aunts naunts x 32 B
 * bottom-up; the NMT range proof (ProveRange, :129-152): nmt_start / nmt_end /
 * nmt_count and nmt_nodes (max_nodes x 90-B slots, left to right).  data_root
 * (optional): the DAH hash.  ShareProof.Data is the caller's input range. */
int cda_share_inclusion_proof(cda_ctx* ctx, uint32_t count, uint32_t share_len, const uint8_t* shares, uint32_t start,
                              uint32_t end, cda_share_proof_info* info, uint8_t* row_roots, uint8_t* leaf_hashes,
                              uint8_t* aunts, int32_t* nmt_start, int32_t* nmt_end, int32_t* nmt_count,
                              uint8_t* nmt_nodes, uint8_t* data_root, cda_err_info* err);

/* ---- square construction on the device (go-square square.Construct + shares.ToBytes) ---- */
/* The step before the DA path (app/prepare_proposal.go:54,65, app/process_proposal.go:121,137): the
 * host plans the layout -- which sequence or blob goes where, the PFB share indexes, the compact
 * reserved offsets -- as share segments; libcda writes the k*k shares straight into device memory
 * (specs/src/specs/shares.md) and, in cda_construct_extend_commit, extends and commits them.  Segments
 * are sorted by first_share and tile [0, k*k) exactly. */
enum { CDA_SEG_COMPACT = 0, CDA_SEG_SPARSE = 1, CDA_SEG_PADDING = 2 };
typedef struct {
  uint32_t kind;          /* CDA_SEG_* */
  uint32_t first_share;   /* row-major ODS index of the segment's first share */
  uint32_t nshares;
  uint32_t share_version; /* info byte = share_version << 1 | sequence start */
  uint64_t data_off;      /* COMPACT: varint-delimited sequence, SPARSE: blob data, in `data` */
  uint64_t data_len;      /* sequence length written in the first share (0 for padding) */
  uint32_t reserved_off;  /* COMPACT: index in `reserved` of the segment's first share */
  uint8_t ns[29];         /* namespace (version byte ‖ 28-byte ID) */
  uint8_t pad_[3];
} cda_share_segment;
/* Builds the ODS (k*k*512 bytes) of the plan into device memory d_ods on `stream` (asynchronous). */
int cda_build_ods_device(cda_ctx* ctx, uint32_t k, uint32_t nseg, const cda_share_segment* segs, const uint8_t* data,
                         uint64_t data_len, const uint32_t* reserved, uint32_t nreserved, void* d_ods, void* stream);
/* square.Construct + shares.ToBytes + da.ExtendShares + NewDataAvailabilityHeader in one call from a
 * host plan: only the payload bytes (sequences and blobs) cross PCIe.  Outputs as cda_extend_commit
 * (ods_or_null additionally receives the k*k shares). */
int cda_construct_extend_commit(cda_ctx* ctx, uint32_t k, uint32_t nseg, const cda_share_segment* segs,
                                const uint8_t* data, uint64_t data_len, const uint32_t* reserved, uint32_t nreserved,
                                uint8_t* ods_or_null, uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots,
                                uint8_t* dah, cda_err_info* err);

/* ---- instrumentation ----------------------------------------------------- */
/* When enabled, every kernel launch is bracketed by HIP events on its own
 * stream and per-kernel total time / launch counts are accumulated. */
int cda_profile_enable(cda_ctx* ctx, int enable);
/* Copies up to `cap` entries: names (NUL-separated into names_buf), total ms, launches. */
int cda_profile_read(cda_ctx* ctx, char* names_buf, size_t names_cap, double* total_ms, int64_t* launches,
                     int cap);
int cda_profile_reset(cda_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
