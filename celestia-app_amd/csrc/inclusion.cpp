// inclusion.cpp — C ABI for blob share commitments, RFC-6962 roots of node lists,
// NMT node export and share inclusion proofs (include/cda.h).
//
//   cda_blob_commitments       go-square inclusion.CreateCommitments (x/blob/types/payforblob.go:53,
//                              blob_tx.go:98)
//   cda_merkle_roots           merkle.HashFromByteSlices over lists of NMT nodes (pkg/inclusion/get_commit.go:29)
//   cda_extend_commit_nodes    ExtendShares + NewDataAvailabilityHeader returning every node of the row /
//                              column trees and of the DAH tree (what pkg/inclusion/nmt_caching.go:33-45 and
//                              pkg/proof/proof.go:82,105-153 recompute on the CPU)
//   cda_share_inclusion_proof  pkg/proof NewShareInclusionProof (proof.go:55-167)
// The host plans (share counts, mountain boundaries, proof node positions) and
// copies; every hash runs in inclusion_kernels.hip / nmt_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "ctx.h"
#include "plan.h"

using namespace cda;

namespace {

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Square-shape checks of da.ExtendShares / rsmt2d for the node-export entry points.
int square_k(uint32_t count, uint32_t share_len, uint32_t* k, cda_err_info* err) {
  if (!is_pow2(count)) return set_err(err, CDA_E_NOT_POW2, -1, -1, -1, -1), CDA_E_NOT_POW2;
  const uint32_t kk = (uint32_t)std::ceil(std::sqrt((double)count));
  if (kk * kk != count) return set_err(err, CDA_E_NOT_SQUARE, -1, -1, -1, -1), CDA_E_NOT_SQUARE;
  if (cda_rs_validate_chunk_size(share_len)) return CDA_E_SHARD_SIZE;
  if (share_len != CDA_SHARE || kk > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  *k = kk;
  return CDA_OK;
}

// node (h, p) of a perfect tree of w leaves exported as levels (leaves first, root last), 90 B per node
const uint8_t* tree_node(const uint8_t* base, uint32_t w, int h, uint32_t p) {
  size_t off = 0;
  for (int i = 0; i < h; i++) off += w >> i;
  return base + (off + p) * CDA_NODE_SIZE;
}

}  // namespace

extern "C" {

int cda_blob_commitments(cda_ctx* c, uint32_t nblobs, const uint8_t* namespaces, const uint8_t* data,
                         const uint64_t* offsets, const uint8_t* share_versions, uint32_t subtree_root_threshold,
                         uint8_t* commitments, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || subtree_root_threshold == 0) return CDA_E_ARG;
  if (nblobs == 0) return CDA_OK;
  if (!namespaces || !offsets || !commitments || !data) return CDA_E_ARG;
  std::vector<BlobDesc> desc(nblobs);
  std::vector<uint32_t> tree_rec, set_off(nblobs + 1);
  uint64_t total = 0;
  uint32_t max_w = 1, max_trees = 0;
  for (uint32_t b = 0; b < nblobs; b++) {
    if (offsets[b + 1] < offsets[b]) return set_err(err, CDA_E_ARG, -1, (int)b, -1, -1), CDA_E_ARG;
    const uint64_t len = offsets[b + 1] - offsets[b];
    const unsigned ver = share_versions ? share_versions[b] : 0u;
    // x/blob ValidateBlobs order (payforblob.go:230-236): empty data, then share version
    if (len == 0) return set_err(err, CDA_E_BLOB_SIZE, -1, (int)b, -1, -1), CDA_E_BLOB_SIZE;
    if (ver != 0) return set_err(err, CDA_E_SHARE_VERSION, -1, (int)b, -1, -1), CDA_E_SHARE_VERSION;
    if (len > 0xFFFFFFFFull) return set_err(err, CDA_E_UNSUPPORTED, -1, (int)b, -1, -1), CDA_E_UNSUPPORTED;
    BlobDesc& d = desc[b];
    memset(&d, 0, sizeof d);
    d.data_off = offsets[b] - offsets[0];
    d.len = (uint32_t)len;
    d.share_off = (uint32_t)total;
    d.nshares = plan::sparse_shares_needed(len);
    d.width = plan::subtree_width(d.nshares, subtree_root_threshold);
    memcpy(d.ns, namespaces + (size_t)b * CDA_NAMESPACE_SIZE, CDA_NAMESPACE_SIZE);
    d.ns[CDA_NAMESPACE_SIZE] = (uint8_t)ver;
    set_off[b] = (uint32_t)tree_rec.size();
    plan::mountains(d.nshares, d.width, (uint32_t)total, tree_rec);  // first share of each mountain
    max_trees = std::max<uint32_t>(max_trees, (uint32_t)tree_rec.size() - set_off[b]);
    max_w = std::max(max_w, d.width);
    total += d.nshares;
    if (total > (1u << 24)) return CDA_E_UNSUPPORTED;  // 8 GiB of shares per call
  }
  set_off[nblobs] = (uint32_t)tree_rec.size();
  const uint64_t data_b = offsets[nblobs] - offsets[0];
  Lock l(c);
  hipStream_t s = c->stream;
  const size_t desc_b = align256((size_t)nblobs * sizeof(BlobDesc)), idx_b = align256(tree_rec.size() * 4),
               off_b = align256(set_off.size() * 4);
  int rc;
  if ((rc = ensure(c, c->ods, data_b)) || (rc = ensure(c, c->eds, (size_t)total * CDA_SHARE)) ||
      (rc = ensure(c, c->leaf, (size_t)total * CDA_REC_BYTES)) ||
      (rc = ensure(c, c->dah, desc_b + idx_b + off_b + (size_t)nblobs * 32)))
    return rc;
  uint8_t* meta = (uint8_t*)c->dah.p;
  BlobDesc* d_desc = (BlobDesc*)meta;
  uint32_t* d_idx = (uint32_t*)(meta + desc_b);
  uint32_t* d_off = (uint32_t*)(meta + desc_b + idx_b);
  uint8_t* d_out = meta + desc_b + idx_b + off_b;
  if (!dev_ok(c, hipMemcpyAsync(c->ods.p, data + offsets[0], data_b, hipMemcpyHostToDevice, s), "H2D") ||
      !dev_ok(c, hipMemcpyAsync(d_desc, desc.data(), (size_t)nblobs * sizeof(BlobDesc), hipMemcpyHostToDevice, s),
              "H2D") ||
      !dev_ok(c, hipMemcpyAsync(d_idx, tree_rec.data(), tree_rec.size() * 4, hipMemcpyHostToDevice, s), "H2D") ||
      !dev_ok(c, hipMemcpyAsync(d_off, set_off.data(), set_off.size() * 4, hipMemcpyHostToDevice, s), "H2D"))
    return CDA_E_DEVICE;
  const uint32_t tot = (uint32_t)total;
  {
    ProfScope ps(c, "blob_shares", s);
    if (launch_blob_shares(d_desc, (int)nblobs, (const uint8_t*)c->ods.p, tot, (uint8_t*)c->eds.p, s))
      return CDA_E_DEVICE;
  }
  {
    ProfScope ps(c, "blob_leaf", s);
    if (launch_blob_leaves((const uint8_t*)c->eds.p, tot, c->leaf.p, s)) return CDA_E_DEVICE;
  }
  for (int level = 1; (1u << level) <= max_w; level++) {
    ProfScope ps(c, "blob_mountain_level", s);
    if (launch_blob_mountain_level(d_desc, (int)nblobs, c->leaf.p, tot, level, s)) return CDA_E_DEVICE;
  }
  {
    ProfScope ps(c, "blob_commit", s);
    const int lr = launch_merkle_sets(c->leaf.p, d_idx, d_off, (int)nblobs, (int)max_trees, d_out, nullptr, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  if (!dev_ok(c, hipMemcpyAsync(commitments, d_out, (size_t)nblobs * 32, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipStreamSynchronize(s), "sync"))
    return CDA_E_DEVICE;
  flush_profile(c);
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_merkle_roots(cda_ctx* c, uint32_t nsets, const uint32_t* set_offsets, const uint8_t* items, uint32_t item_len,
                     uint8_t* roots) {
  CDA_API_TRY
  if (!c) return CDA_E_ARG;
  if (item_len != CDA_NODE_SIZE) return CDA_E_UNSUPPORTED;
  if (nsets == 0) return CDA_OK;
  if (!set_offsets || !roots) return CDA_E_ARG;
  uint32_t max_set = 0;
  for (uint32_t i = 0; i < nsets; i++) {
    if (set_offsets[i + 1] < set_offsets[i]) return CDA_E_ARG;
    max_set = std::max(max_set, set_offsets[i + 1] - set_offsets[i]);
  }
  const uint32_t n = set_offsets[nsets] - set_offsets[0];
  if (n && !items) return CDA_E_ARG;
  std::vector<uint8_t> recs((size_t)n * CDA_REC_BYTES, 0);
  for (uint32_t i = 0; i < n; i++)
    memcpy(recs.data() + (size_t)i * CDA_REC_BYTES, items + (size_t)i * CDA_NODE_SIZE, CDA_NODE_SIZE);
  std::vector<uint32_t> off(nsets + 1);
  for (uint32_t i = 0; i <= nsets; i++) off[i] = set_offsets[i] - set_offsets[0];
  Lock l(c);
  hipStream_t s = c->stream;
  const size_t off_b = align256(off.size() * 4);
  int rc;
  if ((rc = ensure(c, c->roots, recs.size())) || (rc = ensure(c, c->dah, off_b + (size_t)nsets * 32))) return rc;
  uint32_t* d_off = (uint32_t*)c->dah.p;
  uint8_t* d_out = (uint8_t*)c->dah.p + off_b;
  if ((n && !dev_ok(c, hipMemcpyAsync(c->roots.p, recs.data(), recs.size(), hipMemcpyHostToDevice, s), "H2D")) ||
      !dev_ok(c, hipMemcpyAsync(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice, s), "H2D"))
    return CDA_E_DEVICE;
  {
    ProfScope ps(c, "merkle_roots", s);
    const int lr = launch_merkle_sets(c->roots.p, nullptr, d_off, (int)nsets, (int)max_set, d_out, nullptr, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  if (!dev_ok(c, hipMemcpyAsync(roots, d_out, (size_t)nsets * 32, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipStreamSynchronize(s), "sync"))
    return CDA_E_DEVICE;
  flush_profile(c);
  return CDA_OK;
  CDA_API_CATCH(c)
}

}  // extern "C"

namespace {

// cda_extend_commit_nodes with the row trees' nodes exported for rows [row_lo, row_hi) only (row_nodes then holds
// row_hi - row_lo trees): a share proof needs the trees of its own rows, not all 2k of them.
int extend_commit_nodes_rows(cda_ctx* c, uint32_t count, uint32_t share_len, const uint8_t* shares,
                             uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                             uint8_t* row_nodes, uint32_t row_lo, uint32_t row_hi, uint8_t* col_nodes,
                             uint8_t* dah_nodes, cda_err_info* err) {
  uint32_t k = 0;
  if (int rc = square_k(count, share_len, &k, err)) return rc;
  Lock l(c);
  const uint32_t w = 2 * k;
  const int L = ilog2i(w);
  const size_t cells = (size_t)w * w, ods_b = (size_t)k * k * CDA_SHARE, eds_b = cells * CDA_SHARE;
  const size_t roots_b = (size_t)2 * w * CDA_REC_BYTES, dn = 2 * (size_t)(2 * w) - 1;
  int rc;
  // meta: status [0, 256) | set offsets [256, 512) | dah [512, 544) | merkle out [544, 576) | dah nodes
  if ((rc = ensure(c, c->ods, ods_b)) || (rc = ensure(c, c->eds, eds_b)) ||
      (rc = ensure(c, c->leaf, cells * CDA_REC_BYTES)) || (rc = ensure(c, c->scratch, cells * CDA_REC_BYTES)) ||
      (rc = ensure(c, c->roots, roots_b)) || (rc = ensure(c, c->dah, 576 + dn * 32)))
    return rc;
  uint8_t* meta = (uint8_t*)c->dah.p;
  unsigned long long* d_status = (unsigned long long*)meta;
  uint32_t* d_off = (uint32_t*)(meta + 256);
  uint8_t* d_dah = meta + 512;
  uint8_t* d_mout = meta + 544;
  uint8_t* d_dnodes = meta + 576;
  hipStream_t s = c->stream;
  const uint32_t off[2] = {0, 2 * w};
  if (!dev_ok(c, hipMemcpyAsync(c->ods.p, shares, ods_b, hipMemcpyHostToDevice, s), "H2D") ||
      !dev_ok(c, hipMemsetAsync(d_status, 0xFF, 8, s), "memset") ||
      !dev_ok(c, hipMemcpyAsync(d_off, off, sizeof off, hipMemcpyHostToDevice, s), "H2D"))
    return CDA_E_DEVICE;
  if ((rc = enqueue_rs(c, k, 1, (const uint8_t*)c->ods.p, (uint8_t*)c->eds.p, s))) return rc;
  {
    ProfScope ps(c, "leaf_hash", s);
    if (launch_leaf_hash((const uint8_t*)c->eds.p, c->leaf.p, d_status, (int)k, 1, s)) return CDA_E_DEVICE;
  }
  // The exported trees' nodes are packed on the device into the per-tree lists the caller gets (rows [row_lo, row_hi),
  // every column tree when asked), level by level before the next level overwrites its ping-pong buffer, and come
  // back in one copy per kind.
  if (row_hi > w || row_lo >= row_hi) row_lo = 0, row_hi = w;
  const size_t per_tree = 2 * (size_t)w - 1;
  const size_t rows_b = row_nodes ? (size_t)(row_hi - row_lo) * per_tree * CDA_NODE_SIZE : 0;
  const size_t cols_b = col_nodes ? (size_t)w * per_tree * CDA_NODE_SIZE : 0;
  if (rows_b + cols_b && (rc = ensure(c, c->nodes, rows_b + cols_b))) return rc;
  uint8_t* d_rn = (uint8_t*)c->nodes.p;
  uint8_t* d_cn = d_rn + rows_b;
  auto pack = [&](const void* recs, int h, uint32_t off_h) {
    return (row_nodes && launch_pack_tree_level(recs, d_rn, L, h, false, row_lo, row_hi - row_lo, off_h, s)) ||
           (col_nodes && launch_pack_tree_level(recs, d_cn, L, h, true, 0, w, off_h, s));
  };
  uint32_t off_h = 0;
  if (pack(c->leaf.p, 0, off_h)) return CDA_E_DEVICE;
  off_h += w;
  void* bufs[2] = {c->leaf.p, c->scratch.p};
  for (int level = 1; level <= L; level++) {
    void* out = level == L ? c->roots.p : bufs[level & 1];
    {
      ProfScope ps(c, level == 1 ? "nmt_level1" : "nmt_level", s);
      if (launch_nmt_level(bufs[(level - 1) & 1], out, level == 1, (int)k, 1, level, s)) return CDA_E_DEVICE;
    }
    if (pack(out, level, off_h)) return CDA_E_DEVICE;
    off_h += w >> level;
  }
  {
    ProfScope ps(c, "dah", s);
    const int lr = launch_dah(c->roots.p, d_dah, (int)(2 * w), 1, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  if (dah_nodes) {
    {
      ProfScope ps(c, "dah_nodes", s);
      const int lr = launch_merkle_sets(c->roots.p, nullptr, d_off, 1, (int)(2 * w), d_mout, d_dnodes, s);
      if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
    }
    if (!dev_ok(c, hipMemcpyAsync(dah_nodes, d_dnodes, dn * 32, hipMemcpyDeviceToHost, s), "D2H")) return CDA_E_DEVICE;
  }
  std::vector<uint8_t> recs(roots_b);
  uint64_t st = 0;
  if ((eds_or_null && !dev_ok(c, hipMemcpyAsync(eds_or_null, c->eds.p, eds_b, hipMemcpyDeviceToHost, s), "D2H")) ||
      (rows_b && !dev_ok(c, hipMemcpyAsync(row_nodes, d_rn, rows_b, hipMemcpyDeviceToHost, s), "D2H")) ||
      (cols_b && !dev_ok(c, hipMemcpyAsync(col_nodes, d_cn, cols_b, hipMemcpyDeviceToHost, s), "D2H")) ||
      !dev_ok(c, hipMemcpyAsync(recs.data(), c->roots.p, roots_b, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipMemcpyAsync(dah, d_dah, 32, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipMemcpyAsync(&st, d_status, 8, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipStreamSynchronize(s), "sync"))
    return CDA_E_DEVICE;
  flush_profile(c);
  pack_roots(recs.data(), w, row_roots);
  pack_roots(recs.data() + (size_t)w * CDA_REC_BYTES, w, col_roots);
  return map_status(st, 0, err);
}

}  // namespace

extern "C" {

int cda_extend_commit_nodes(cda_ctx* c, uint32_t count, uint32_t share_len, const uint8_t* shares, uint8_t* eds_or_null,
                            uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, uint8_t* row_nodes,
                            uint8_t* col_nodes, uint8_t* dah_nodes, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !shares || !row_roots || !col_roots || !dah) return CDA_E_ARG;
  return extend_commit_nodes_rows(c, count, share_len, shares, eds_or_null, row_roots, col_roots, dah, row_nodes, 0,
                                  ~0u, col_nodes, dah_nodes, err);
  CDA_API_CATCH(c)
}

int cda_share_inclusion_proof(cda_ctx* c, uint32_t count, uint32_t share_len, const uint8_t* shares, uint32_t start,
                              uint32_t end, cda_share_proof_info* info, uint8_t* row_roots, uint8_t* leaf_hashes,
                              uint8_t* aunts, int32_t* nmt_start, int32_t* nmt_end, int32_t* nmt_count,
                              uint8_t* nmt_nodes, uint8_t* data_root, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !shares || !info || !row_roots || !leaf_hashes || !aunts || !nmt_start || !nmt_end || !nmt_count ||
      !nmt_nodes)
    return CDA_E_ARG;
  uint32_t k = 0;
  if (int rc = square_k(count, share_len, &k, err)) return rc;
  if (start >= end || end > count) return CDA_E_ARG;  // the range ParseNamespace validates (querier.go:126-141)
  const uint32_t w = 2 * k;
  const int L = ilog2i(w);
  const size_t per_tree = 2 * (size_t)w - 1;
  const uint32_t start_row = start / k, end_row = (end - 1) / k;
  // only the proof's own row trees come back (rn: rows start_row..end_row)
  std::vector<uint8_t> rr((size_t)w * CDA_NODE_SIZE), cr((size_t)w * CDA_NODE_SIZE),
      rn((size_t)(end_row - start_row + 1) * per_tree * CDA_NODE_SIZE), dn((2 * (size_t)(2 * w) - 1) * 32);
  uint8_t root[32];
  if (int rc = extend_commit_nodes_rows(c, count, share_len, shares, nullptr, rr.data(), cr.data(), root, rn.data(),
                                        start_row, end_row + 1, nullptr, dn.data(), err))
    return rc;
  info->start_row = start_row;
  info->end_row = end_row;
  info->nrows = end_row - start_row + 1;
  info->total = 2 * w;
  info->naunts = (uint32_t)L + 1;
  info->max_nodes = 2 * (uint32_t)L;
  for (uint32_t i = 0; i < info->nrows; i++) {
    const uint32_t r = start_row + i;
    memcpy(row_roots + (size_t)i * CDA_NODE_SIZE, rr.data() + (size_t)r * CDA_NODE_SIZE, CDA_NODE_SIZE);
    // RFC-6962 proof of row root r among rowRoots ‖ colRoots: leaf hash, then siblings bottom-up
    memcpy(leaf_hashes + (size_t)i * 32, dn.data() + (size_t)r * 32, 32);
    size_t base = 0, n = 2 * (size_t)w;
    uint32_t idx = r;
    for (uint32_t h = 0; h < info->naunts; h++) {
      memcpy(aunts + ((size_t)i * info->naunts + h) * 32, dn.data() + (base + (idx ^ 1u)) * 32, 32);
      base += n;
      n >>= 1;
      idx >>= 1;
    }
    // NMT range proof inside the row: [startLeaf, k) on the first row, [0, k) between, [0, endLeaf] on the last
    const uint32_t s = i == 0 ? start % k : 0, e = i + 1 == info->nrows ? (end - 1) % k + 1 : k;
    std::vector<std::pair<int, uint32_t>> nodes;
    plan::prove_range(L, s, e, nodes);
    nmt_start[i] = (int32_t)s;
    nmt_end[i] = (int32_t)e;
    nmt_count[i] = (int32_t)nodes.size();
    const uint8_t* tree = rn.data() + (size_t)i * per_tree * CDA_NODE_SIZE;
    for (size_t q = 0; q < nodes.size(); q++)
      memcpy(nmt_nodes + ((size_t)i * info->max_nodes + q) * CDA_NODE_SIZE,
             tree_node(tree, w, nodes[q].first, nodes[q].second), CDA_NODE_SIZE);
  }
  if (data_root) memcpy(data_root, root, 32);
  return CDA_OK;
  CDA_API_CATCH(c)
}

}  // extern "C"
