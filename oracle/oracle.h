/*
 * oracle.h — CPU restatement of celestia-app's DA hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libcda) links, loads or
 * calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / baseline.
 *
 * What it restates (reference = /root/reference, celestia-app @ 2025-02-13):
 *   - da.ExtendShares / NewDataAvailabilityHeader / DAH.Hash
 *       pkg/da/data_availability_header.go:44-108
 *   - wrapper.ErasuredNamespacedMerkleTree Push/Root
 *       pkg/wrapper/nmt_wrapper.go:93-140
 *   - NMT hasher (leaf, node, ns-range with IgnoreMaxNamespace, empty root)
 *       test/util/malicious/hasher.go:161-168,186-209,271-310 (copy of nmt v0.20.0)
 *   - RFC-6962 merkle.HashFromByteSlices (go-square/merkle, pinned go.mod:10)
 *       specs/src/specs/data_structures.md:174-204
 *   - rsmt2d v0.12.0 ComputeExtendedDataSquare / Repair (go.mod:13; not vendored,
 *     restated from the upstream algorithm; call site data_availability_header.go:74)
 *   - klauspost/reedsolomon v1.12.1 Leopard FF8/FF16 encode (go.mod:153; not vendored,
 *     restated from the upstream algorithm)
 *
 * Pinning: SHA-256, NMT, quadrant namespace rule, root order and RFC-6962 are
 * pinned by the reference's own known-answer DAH hashes
 * (pkg/da/data_availability_header_test.go:15-68).  The Leopard parity bytes
 * for non-constant data are pinned by the mainnet block fixture (see
 * tests/golden/README.md) when that test is present; otherwise they are
 * "parity unpinned" and rest on the FFT == Lagrange interpolation identity.
 */
#ifndef CDA_ORACLE_H
#define CDA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_SHARE 512
#define ORA_NS 29
#define ORA_NODE 90 /* min ns ‖ max ns ‖ sha256 */

enum {
  ORA_OK = 0,
  ORA_E_NOT_POW2 = -1,
  ORA_E_NOT_SQUARE = -2,
  ORA_E_SHARD_SIZE = -3,
  ORA_E_NS_SHORT = -4,
  ORA_E_NS_ORDER = -5,
  ORA_E_TOO_FEW = -6,
  ORA_E_UNREPAIRABLE = -7,
  ORA_E_BYZANTINE = -8,
  ORA_E_ARG = -9,
  ORA_E_PUSH_PAST = -11,
  ORA_E_SHARE_VERSION = -13, /* appconsts.SupportedShareVersions / ErrUnsupportedShareVersion */
  ORA_E_BLOB_SIZE = -14,     /* x/blob ErrZeroBlobSize */
};

/* ---- primitives ---- */
void ora_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);

/* ---- Leopard (klauspost/reedsolomon v1.12.1, WithLeopardGF(true)) ---- */
/* bits = 8 if 2k <= 256 else 16 (rsmt2d LeoRSCodec field selection). */
int ora_leo_bits_for(int k);
/* Systematic encode: k data shards -> k parity shards (rsmt2d LeoRSCodec.Encode). */
int ora_leo_encode(int k, size_t shard_len, const uint8_t* const* data, uint8_t* const* parity);
/* Erasure decode of a 2k-shard codeword (rsmt2d LeoRSCodec.Decode): present[i]
 * != 0 marks an available shard.  Missing shards are written in place.
 * Uses Lagrange interpolation over Leopard's field, a decoder independent from
 * the FFT path (MDS => any correct decoder returns identical bytes). */
int ora_leo_decode(int k, size_t shard_len, uint8_t* const* shards, const uint8_t* present);
/* The same erasure decode through klauspost's own Leopard reconstruct (error locators, IFFT, formal derivative,
 * FFT): O(k log k) per shard byte, the CPU baseline's decoder (bench.py).  Checked against ora_leo_decode. */
int ora_leo_decode_fft(int k, size_t shard_len, uint8_t* const* shards, const uint8_t* present);
/* Field helpers (Leopard representation) exposed for property tests. */
unsigned ora_leo_mul(int bits, unsigned a, unsigned b);
int ora_leo_skew(int bits, int i);      /* FFT skew log table entry */
int ora_leo_log(int bits, unsigned a);
int ora_leo_exp(int bits, unsigned l);

/* ---- NMT / merkle ---- */
/* Erasured NMT root of one axis: leaves[0..n) are shares of length share_len.
 * square_size = k, axis_index = row/col index.  Returns ORA_OK or an error
 * code; *err_leaf gets the offending leaf for ORA_E_NS_ORDER / NS_SHORT. */
int ora_nmt_axis_root(uint64_t square_size, uint64_t axis_index, const uint8_t* const* leaves,
                      const size_t* lens, int n, uint8_t root[ORA_NODE], int* err_leaf);
/* RFC-6962 root (go-square/merkle HashFromByteSlices). */
void ora_merkle_root(const uint8_t* const* items, const size_t* lens, int n, uint8_t out[32]);

/* ---- 2-D pipeline ---- */
/* ODS (k*k*share_len, row-major) -> EDS (2k*2k*share_len, row-major). */
int ora_extend(int k, size_t share_len, const uint8_t* ods, uint8_t* eds, int nthreads);
/* Row/col roots of an EDS (2k roots each, 90 B).  err_axis: 0 row / 1 col. */
int ora_roots(int k, size_t share_len, const uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots,
              int nthreads, int* err_axis, int* err_index);
/* DAH hash = RFC-6962 over row roots ‖ col roots (n roots per axis). */
void ora_dah_hash(int n, const uint8_t* row_roots, const uint8_t* col_roots, uint8_t out[32]);
/* da.ExtendShares + NewDataAvailabilityHeader on `count` shares. */
/* Throughput sample (bench cpu_baseline): nthreads workers each run whole single-threaded
 * ora_extend_commit calls on `shares` until `seconds` pass; returns blocks completed
 * (negative ORA_E_* if any call failed or its DAH differed). */
long ora_extend_commit_throughput(int count, size_t share_len, const uint8_t* shares, int nthreads, double seconds,
                                  double* elapsed);
int ora_extend_commit(int count, size_t share_len, const uint8_t* shares, uint8_t* eds_or_null,
                      uint8_t* row_roots, uint8_t* col_roots, uint8_t dah[32], int nthreads);

/* rsmt2d Repair: eds (2k*2k*share_len) with present map (4k^2 bytes).
 * Returns ORA_OK, ORA_E_UNREPAIRABLE or ORA_E_BYZANTINE (with axis/index). */
int ora_repair(int k, size_t share_len, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
               const uint8_t* col_roots, int* err_axis, int* err_index);
/* ora_repair with the decoder chosen: fft_decoder = 0 Lagrange (ora_repair), 1 Leopard reconstruct. */
int ora_repair_ex(int k, size_t share_len, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
                  const uint8_t* col_roots, int* err_axis, int* err_index, int fft_decoder);

/* ---- NMT building blocks (da.c) ---- */
void ora_nmt_hash_node_ns(int ns_len, const uint8_t* l, const uint8_t* r, uint8_t* out);
void ora_nmt_leaf_node(const uint8_t* ns, const uint8_t* data, size_t len, uint8_t* out);
void ora_nmt_root_of_nodes(const uint8_t* leaf_nodes, int n, uint8_t* out);

/* ---- blob share commitments, subtree roots and proofs (inclusion.c) ---- */
int ora_sparse_shares_needed(uint32_t len);
int ora_blob_to_shares(const uint8_t* ns, const uint8_t* data, uint32_t len, int share_version, uint8_t* out);
int ora_blob_min_square_size(int share_count);
int ora_subtree_width(int share_count, int threshold);
int ora_mmr_sizes(int total, int max_tree, int* sizes);
int ora_blob_commitment(const uint8_t* ns, const uint8_t* data, uint32_t len, int share_version, int threshold,
                        uint8_t out[32]);
int ora_subtree_root_coords(int max_depth, int min_depth, int start, int end, int* coords);
void ora_axis_leaf_nodes(int k, const uint8_t* eds, int axis, int idx, uint8_t* out);
void ora_nmt_tree_levels(const uint8_t* leaf_nodes, int n, uint8_t* out);
int ora_get_commitment(int k, const uint8_t* eds, int start, int blob_share_len, int threshold, uint8_t out[32]);
int ora_nmt_prove_range(const uint8_t* leaf_nodes, int n, int start, int end, uint8_t* out_nodes);
int ora_nmt_verify_inclusion(int ns_len, const uint8_t* nid, const uint8_t* leaves, size_t leaf_len, int nleaves,
                             int start, int end, const uint8_t* nodes, int nnodes, const uint8_t* root);
int ora_merkle_proof(const uint8_t* items, size_t item_len, int n, int index, uint8_t leaf[32], uint8_t* aunts,
                     uint8_t root[32]);
int ora_merkle_verify(int64_t total, int64_t index, const uint8_t* proof_leaf_hash, const uint8_t* aunts, int na,
                      const uint8_t* root, const uint8_t* item, size_t item_len);

/* Deterministic generator used by tests and bench:
 * v0 namespaces (0x00 x19 ‖ 10 random bytes) ‖ 483 random bytes, sorted. */
void ora_gen_ods(int k, uint64_t seed, uint8_t* ods);

#ifdef __cplusplus
}
#endif
#endif
