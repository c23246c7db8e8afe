/*
 * inclusion.c — CPU restatement of blob share commitments, NMT range proofs and
 * RFC-6962 proofs (TEST INFRASTRUCTURE ONLY: the checker for the GPU path).
 *
 *   inclusion.CreateCommitment   go-square v1.0.1 (go.mod:9, not vendored), called from
 *                                x/blob/types/payforblob.go:53 and blob_tx.go:98; rules in
 *                                specs/src/specs/data_square_layout.md:38-58 (SubtreeWidth,
 *                                Merkle mountain range) and shares.md:31-81 (sparse shares)
 *   pkg/inclusion GetCommitment  pkg/inclusion/get_commit.go:12-30, paths.go:16-173
 *   nmt ProveRange / VerifyInclusion  nmt v0.20.0 (go.mod:12, not vendored); proofs are
 *                                built by pkg/proof/proof.go:105-153 and checked by
 *                                pkg/proof/share_proof.go:54-82
 *   merkle.ProofsFromByteSlices / Proof.Verify  go-square/merkle (RFC-6962 proofs),
 *                                pkg/proof/proof.go:82-93, row_proof.go:30-48
 *
 * Pinning: the commitment restatement is pinned by the real share commitments of
 * every PayForBlobs message in the reference's mainnet block fixture
 * (x/blob/test/testdata/block_response.json, tests/golden/make_blob_commitments.py);
 * the proof verifiers by the reference's own valid ShareProof / RowProof
 * (pkg/proof/share_proof_test.go:77-93, row_proof_test.go:68-89).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MAXNODE (2 * 64 + 32)

/* ---- go-square shares / inclusion arithmetic ---- */
static int round_up_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}
static int round_down_pow2(int v) {
  int p = 1;
  while (p * 2 <= v) p <<= 1;
  return p;
}
static int isqrt_ceil(int n) {
  int r = 0;
  while (r * r < n) r++;
  return r;
}

/* shares.SparseSharesNeeded: the first share holds 478 data bytes, continuation shares 482 */
int ora_sparse_shares_needed(uint32_t len) {
  const uint32_t first = ORA_SHARE - ORA_NS - 1 - 4, cont = ORA_SHARE - ORA_NS - 1;
  if (len == 0) return 0;
  if (len <= first) return 1;
  return 1 + (int)((len - first + cont - 1) / cont);
}

/* SparseShareSplitter.Write: ns ‖ info ‖ [sequence length, first share] ‖ data ‖ zero padding */
int ora_blob_to_shares(const uint8_t* ns, const uint8_t* data, uint32_t len, int share_version, uint8_t* out) {
  int n = ora_sparse_shares_needed(len);
  uint32_t pos = 0;
  for (int s = 0; s < n; s++) {
    uint8_t* sh = out + (size_t)s * ORA_SHARE;
    memset(sh, 0, ORA_SHARE);
    memcpy(sh, ns, ORA_NS);
    sh[ORA_NS] = (uint8_t)((share_version << 1) | (s == 0 ? 1 : 0));
    int h = ORA_NS + 1;
    if (s == 0) {
      sh[h + 0] = (uint8_t)(len >> 24);
      sh[h + 1] = (uint8_t)(len >> 16);
      sh[h + 2] = (uint8_t)(len >> 8);
      sh[h + 3] = (uint8_t)len;
      h += 4;
    }
    uint32_t take = (uint32_t)(ORA_SHARE - h);
    if (take > len - pos) take = len - pos;
    memcpy(sh + h, data + pos, take);
    pos += take;
  }
  return n;
}

/* inclusion.BlobMinSquareSize / SubTreeWidth (data_square_layout.md:53) */
int ora_blob_min_square_size(int share_count) { return round_up_pow2(isqrt_ceil(share_count)); }
int ora_subtree_width(int share_count, int threshold) {
  int s = share_count / threshold + (share_count % threshold ? 1 : 0);
  s = round_up_pow2(s);
  int m = ora_blob_min_square_size(share_count);
  return s < m ? s : m;
}

/* inclusion.MerkleMountainRangeSizes: max-size trees first, then decreasing powers of two */
int ora_mmr_sizes(int total, int max_tree, int* sizes) {
  int n = 0;
  while (total > 0) {
    int t = total >= max_tree ? max_tree : round_down_pow2(total);
    if (sizes) sizes[n] = t;
    n++;
    total -= t;
  }
  return n;
}

/* RFC-6962 root over n items of item_len bytes (merkle.HashFromByteSlices) */
static void merkle_flat(const uint8_t* items, int n, size_t item_len, uint8_t out[32]) {
  const uint8_t** p = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)(n ? n : 1));
  size_t* l = (size_t*)malloc(sizeof(size_t) * (size_t)(n ? n : 1));
  for (int i = 0; i < n; i++) {
    p[i] = items + (size_t)i * item_len;
    l[i] = item_len;
  }
  ora_merkle_root(p, l, n, out);
  free(p);
  free(l);
}

/* inclusion.CreateCommitment: NMT root of each mountain (leaves ns ‖ share), RFC-6962 over them.
 * Argument checks in the order of x/blob ValidateBlobs (payforblob.go:230-236). */
int ora_blob_commitment(const uint8_t* ns, const uint8_t* data, uint32_t len, int share_version, int threshold,
                        uint8_t out[32]) {
  if (len == 0) return ORA_E_BLOB_SIZE;               /* ErrZeroBlobSize */
  if (share_version != 0) return ORA_E_SHARE_VERSION; /* appconsts.SupportedShareVersions = {0} */
  if (threshold <= 0) return ORA_E_ARG;
  int n = ora_sparse_shares_needed(len);
  uint8_t* shares = (uint8_t*)malloc((size_t)n * ORA_SHARE);
  ora_blob_to_shares(ns, data, len, share_version, shares);
  int w = ora_subtree_width(n, threshold);
  int ntrees = ora_mmr_sizes(n, w, NULL);
  int* sizes = (int*)malloc(sizeof(int) * (size_t)ntrees);
  ora_mmr_sizes(n, w, sizes);
  uint8_t* leaves = (uint8_t*)malloc((size_t)n * ORA_NODE);
  for (int i = 0; i < n; i++) ora_nmt_leaf_node(ns, shares + (size_t)i * ORA_SHARE, ORA_SHARE, leaves + (size_t)i * ORA_NODE);
  uint8_t* roots = (uint8_t*)malloc((size_t)ntrees * ORA_NODE);
  int cur = 0;
  for (int t = 0; t < ntrees; t++) {
    ora_nmt_root_of_nodes(leaves + (size_t)cur * ORA_NODE, sizes[t], roots + (size_t)t * ORA_NODE);
    cur += sizes[t];
  }
  merkle_flat(roots, ntrees, ORA_NODE, out);
  free(roots);
  free(leaves);
  free(sizes);
  free(shares);
  return ORA_OK;
}

/* ---- pkg/inclusion GetCommitment over an EDS ---- */
/* calculateSubTreeRootCoordinates (paths.go:108-173): (depth, position) pairs into coords */
int ora_subtree_root_coords(int max_depth, int min_depth, int start, int end, int* coords) {
  int n = 0;
  int leaf = start, nd = max_depth, np = start, lnd = nd, lnp = np, lleaf = leaf, range = 1;
  for (;;) {
    int pd, pp;
    if (leaf + 1 == end) {
      if (coords) coords[2 * n] = nd, coords[2 * n + 1] = np;
      return n + 1;
    } else if (leaf + 1 > end) { /* climbed too high: keep the last node */
      pd = lnd, pp = lnp;
      leaf = lleaf + 1;
    } else if (!(np % 2 == 0 && nd > min_depth)) { /* cannot climb right */
      pd = nd, pp = np;
      leaf++;
    } else { /* climb */
      lleaf = leaf;
      lnd = nd, lnp = np;
      leaf += range;
      range *= 2;
      nd -= 1;
      np /= 2;
      continue;
    }
    if (coords) coords[2 * n] = pd, coords[2 * n + 1] = pp;
    n++;
    /* reset(): lastNode = node, lastLeaf = leaf, node = the leaf's coordinate */
    lnd = nd, lnp = np, lleaf = leaf;
    nd = max_depth, np = leaf, range = 1;
  }
}

static int ilog2_exact(int v) {
  int l = 0;
  while ((1 << l) < v) l++;
  return l;
}

/* Erasured leaf nodes of one EDS axis (0 row / 1 col): quadrant rule of nmt_wrapper.go:100-107 */
void ora_axis_leaf_nodes(int k, const uint8_t* eds, int axis, int idx, uint8_t* out) {
  static const uint8_t parity[ORA_NS] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                        0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                        0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};
  const int w = 2 * k;
  for (int i = 0; i < w; i++) {
    const int r = axis == 0 ? idx : i, c = axis == 0 ? i : idx;
    const uint8_t* sh = eds + ((size_t)r * w + c) * ORA_SHARE;
    ora_nmt_leaf_node((i < k && idx < k) ? sh : parity, sh, ORA_SHARE, out + (size_t)i * ORA_NODE);
  }
}

/* Every level of the perfect tree over n (a power of two) leaf nodes: leaves first, root last. */
void ora_nmt_tree_levels(const uint8_t* leaf_nodes, int n, uint8_t* out) {
  memcpy(out, leaf_nodes, (size_t)n * ORA_NODE);
  size_t in = 0, o = (size_t)n;
  for (int cnt = n; cnt > 1; cnt >>= 1) {
    for (int i = 0; i < cnt / 2; i++)
      ora_nmt_hash_node_ns(ORA_NS, out + (in + 2 * (size_t)i) * ORA_NODE, out + (in + 2 * (size_t)i + 1) * ORA_NODE,
                           out + (o + (size_t)i) * ORA_NODE);
    in = o;
    o += (size_t)cnt / 2;
  }
}

/* GetCommitment (get_commit.go:12-30): subtree roots of the ODS half of the row
 * trees at calculateCommitmentPaths (paths.go:16-47), RFC-6962 over them.
 * eds: 2k x 2k shares.  The path "WalkLeft ‖ genSubTreeRootPath(depth, pos)" of
 * row r is the node over row leaves [pos << (log2k - depth), (pos+1) << (log2k - depth)). */
int ora_get_commitment(int k, const uint8_t* eds, int start, int blob_share_len, int threshold, uint8_t out[32]) {
  if (blob_share_len <= 0 || start < 0 || start + blob_share_len > k * k) return ORA_E_ARG;
  int w = ora_subtree_width(blob_share_len, threshold);
  start = (start + w - 1) / w * w; /* inclusion.NextShareIndex */
  int start_row = start / k, end_row = (start + blob_share_len - 1) / k;
  int nstart = start % k, nend = (start + blob_share_len) - end_row * k;
  int max_depth = ilog2_exact(k), min_depth = max_depth - ilog2_exact(w);
  int cap = 0;
  for (int r = start_row; r <= end_row; r++) {
    int s = r == start_row ? nstart : 0, e = r == end_row ? nend : k;
    cap += ora_subtree_root_coords(max_depth, min_depth, s, e, NULL);
  }
  uint8_t* roots = (uint8_t*)malloc((size_t)(cap ? cap : 1) * ORA_NODE);
  uint8_t* leaves = (uint8_t*)malloc((size_t)2 * k * ORA_NODE);
  int* coords = (int*)malloc(sizeof(int) * 2 * (size_t)(k + 1));
  int nr = 0;
  for (int r = start_row; r <= end_row; r++) {
    int s = r == start_row ? nstart : 0, e = r == end_row ? nend : k;
    int nc = ora_subtree_root_coords(max_depth, min_depth, s, e, coords);
    ora_axis_leaf_nodes(k, eds, 0, r, leaves);
    for (int i = 0; i < nc; i++) {
      int span = 1 << (max_depth - coords[2 * i]);
      ora_nmt_root_of_nodes(leaves + (size_t)coords[2 * i + 1] * span * ORA_NODE, span, roots + (size_t)nr * ORA_NODE);
      nr++;
    }
  }
  merkle_flat(roots, nr, ORA_NODE, out);
  free(coords);
  free(leaves);
  free(roots);
  return ORA_OK;
}

/* ---- NMT range proofs (nmt v0.20.0 buildRangeProof / VerifyLeafHashes) ---- */
static int split_point(int n) { /* getSplitPoint: largest power of two < n (0 for n = 1) */
  int k = 1;
  while (k * 2 <= n) k *= 2;
  if (k == n) k >>= 1;
  return k;
}

typedef struct {
  const uint8_t* leaves; /* n leaf nodes */
  int n, ps, pe;
  uint8_t* out;
  int nout;
} prove_t;

static void prove_emit(prove_t* P, const uint8_t* h) {
  if (P->out) memcpy(P->out + (size_t)P->nout * ORA_NODE, h, ORA_NODE);
  P->nout++;
}

/* recurse(start, end, includeNode): 1 and the subtree hash in h if the subtree exists */
static int prove_rec(prove_t* P, int start, int end, int include, uint8_t* h) {
  if (start >= P->n) return 0;
  if (end - start == 1) {
    memcpy(h, P->leaves + (size_t)start * ORA_NODE, ORA_NODE);
    if ((start < P->ps || start >= P->pe) && include) prove_emit(P, h);
    return 1;
  }
  int newinc = include;
  if ((end <= P->ps || start >= P->pe) && include) newinc = 0;
  int k = split_point(end - start);
  uint8_t L[ORA_NODE], R[ORA_NODE];
  prove_rec(P, start, start + k, newinc, L);
  if (!prove_rec(P, start + k, end, newinc, R))
    memcpy(h, L, ORA_NODE);
  else
    ora_nmt_hash_node_ns(ORA_NS, L, R, h);
  if (include && !newinc) prove_emit(P, h);
  return 1;
}

/* ProveRange(start, end) over n leaf nodes (90 B): proof nodes left to right; returns their count */
int ora_nmt_prove_range(const uint8_t* leaf_nodes, int n, int start, int end, uint8_t* out_nodes) {
  if (start < 0 || start >= end || end > n) return -1;
  prove_t P = {leaf_nodes, n, start, end, out_nodes, 0};
  int full = split_point(n) * 2;
  if (full < 1) full = 1;
  uint8_t h[ORA_NODE];
  prove_rec(&P, 0, full, 1, h);
  return P.nout;
}

typedef struct {
  const uint8_t* hashes;
  int nh;
  const uint8_t* nodes;
  int nn;
  int ps, pe, ns_len, node_len, bad;
} verify_t;

/* HashNode with the sibling-order validation of nmt's ValidateNodes (left.max <= right.min) */
static void verify_hash(verify_t* V, const uint8_t* L, const uint8_t* R, uint8_t* h) {
  if (memcmp(L + V->ns_len, R, (size_t)V->ns_len) > 0) V->bad = 1;
  ora_nmt_hash_node_ns(V->ns_len, L, R, h);
}

static int pop_node(verify_t* V, uint8_t* h) {
  if (V->nn <= 0) return 0;
  memcpy(h, V->nodes, (size_t)V->node_len);
  V->nodes += V->node_len;
  V->nn--;
  return 1;
}

static int verify_rec(verify_t* V, int start, int end, uint8_t* h) {
  if (end - start == 1) {
    if (V->ps <= start && start < V->pe) {
      if (V->nh <= 0) return (V->bad = 1), 0;
      memcpy(h, V->hashes, (size_t)V->node_len);
      V->hashes += V->node_len;
      V->nh--;
      return 1;
    }
    return pop_node(V, h);
  }
  if (end <= V->ps || start >= V->pe) return pop_node(V, h);
  int k = split_point(end - start);
  uint8_t L[MAXNODE], R[MAXNODE];
  int hl = verify_rec(V, start, start + k, L);
  int hr = verify_rec(V, start + k, end, R);
  if (!hr) {
    if (hl) memcpy(h, L, (size_t)V->node_len);
    return hl;
  }
  if (!hl) return (V->bad = 1), 0;
  verify_hash(V, L, R, h);
  return 1;
}

/* Proof.VerifyInclusion(sha256, nid, leaves without namespace, root) for an
 * inclusion proof [start, end) with `nodes`: 1 = valid.  ns_len generalises the
 * namespace size so the reference's own (33-byte namespace) fixture in
 * pkg/proof/share_proof_test.go can pin this verifier. */
int ora_nmt_verify_inclusion(int ns_len, const uint8_t* nid, const uint8_t* leaves, size_t leaf_len, int nleaves,
                             int start, int end, const uint8_t* nodes, int nnodes, const uint8_t* root) {
  const int node_len = 2 * ns_len + 32;
  if (ns_len <= 0 || ns_len > 64 || start < 0 || start >= end || end - start != nleaves) return 0;
  uint8_t* hashes = (uint8_t*)malloc((size_t)nleaves * node_len);
  uint8_t* msg = (uint8_t*)malloc(1 + (size_t)ns_len + leaf_len);
  for (int i = 0; i < nleaves; i++) { /* HashLeaf(nid ‖ leaf) = nid ‖ nid ‖ SHA256(0x00 ‖ nid ‖ leaf) */
    msg[0] = 0x00;
    memcpy(msg + 1, nid, (size_t)ns_len);
    memcpy(msg + 1 + ns_len, leaves + (size_t)i * leaf_len, leaf_len);
    uint8_t* o = hashes + (size_t)i * node_len;
    memcpy(o, nid, (size_t)ns_len);
    memcpy(o + ns_len, nid, (size_t)ns_len);
    ora_sha256(msg, 1 + (size_t)ns_len + leaf_len, o + 2 * ns_len);
  }
  free(msg);
  verify_t V = {hashes, nleaves, nodes, nnodes, start, end, ns_len, node_len, 0};
  int est = split_point(end) * 2;
  if (est < 1) est = 1;
  uint8_t h[MAXNODE];
  int ok = verify_rec(&V, 0, est, h) == 1 && V.nh == 0;
  while (ok && V.nn > 0) { /* remaining nodes are right siblings up to the root */
    uint8_t r[MAXNODE], t[MAXNODE];
    pop_node(&V, r);
    verify_hash(&V, h, r, t);
    memcpy(h, t, (size_t)node_len);
  }
  ok = ok && !V.bad && memcmp(h, root, (size_t)node_len) == 0;
  free(hashes);
  return ok;
}

/* ---- RFC-6962 proofs (merkle.ProofsFromByteSlices / Proof.Verify) ---- */
static void leaf_hash(const uint8_t* item, size_t len, uint8_t out[32]) {
  uint8_t* b = (uint8_t*)malloc(1 + len);
  b[0] = 0x00;
  memcpy(b + 1, item, len);
  ora_sha256(b, 1 + len, out);
  free(b);
}
static void inner_hash(const uint8_t* l, const uint8_t* r, uint8_t out[32]) {
  uint8_t b[65];
  b[0] = 0x01;
  memcpy(b + 1, l, 32);
  memcpy(b + 33, r, 32);
  ora_sha256(b, 65, out);
}

/* trailsFromByteSlices: root of items[lo, hi) into h; the aunts of `index` are appended bottom-up */
static void trail_rec(const uint8_t* items, size_t item_len, int lo, int hi, int index, uint8_t* aunts, int* na,
                      uint8_t h[32]) {
  int n = hi - lo;
  if (n == 1) {
    leaf_hash(items + (size_t)lo * item_len, item_len, h);
    return;
  }
  int k = split_point(n);
  uint8_t L[32], R[32];
  trail_rec(items, item_len, lo, lo + k, index, aunts, na, L);
  trail_rec(items, item_len, lo + k, hi, index, aunts, na, R);
  if (index >= lo && index < lo + k) memcpy(aunts + 32 * (size_t)(*na)++, R, 32);
  else if (index >= lo + k && index < hi) memcpy(aunts + 32 * (size_t)(*na)++, L, 32);
  inner_hash(L, R, h);
}

/* Proof of item `index` of n items: leaf hash, aunts (bottom-up), root; returns the aunt count */
int ora_merkle_proof(const uint8_t* items, size_t item_len, int n, int index, uint8_t leaf[32], uint8_t* aunts,
                     uint8_t root[32]) {
  if (n <= 0 || index < 0 || index >= n) return -1;
  int na = 0;
  trail_rec(items, item_len, 0, n, index, aunts, &na, root);
  leaf_hash(items + (size_t)index * item_len, item_len, leaf);
  return na;
}

static int hash_from_aunts(int64_t index, int64_t total, const uint8_t* leaf, const uint8_t* aunts, int na,
                           uint8_t out[32]) {
  if (index >= total || index < 0 || total <= 0) return 0;
  if (total == 1) {
    if (na != 0) return 0;
    memcpy(out, leaf, 32);
    return 1;
  }
  if (na == 0) return 0;
  int64_t left = split_point((int)total);
  uint8_t sub[32];
  if (index < left) {
    if (!hash_from_aunts(index, left, leaf, aunts, na - 1, sub)) return 0;
    inner_hash(sub, aunts + 32 * (size_t)(na - 1), out);
  } else {
    if (!hash_from_aunts(index - left, total - left, leaf, aunts, na - 1, sub)) return 0;
    inner_hash(aunts + 32 * (size_t)(na - 1), sub, out);
  }
  return 1;
}

/* merkle.Proof.Verify(rootHash, leaf): 1 = valid */
int ora_merkle_verify(int64_t total, int64_t index, const uint8_t* proof_leaf_hash, const uint8_t* aunts, int na,
                      const uint8_t* root, const uint8_t* item, size_t item_len) {
  if (total < 0 || index < 0 || na > 100) return 0;
  uint8_t lh[32], h[32];
  leaf_hash(item, item_len, lh);
  if (memcmp(lh, proof_leaf_hash, 32) != 0) return 0;
  if (!hash_from_aunts(index, total, lh, aunts, na, h)) return 0;
  return memcmp(h, root, 32) == 0;
}
