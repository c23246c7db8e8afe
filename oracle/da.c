/*
 * da.c — CPU restatement of the celestia-app DA path (TEST INFRASTRUCTURE ONLY).
 *
 *   ExtendShares            pkg/da/data_availability_header.go:65-75
 *   NewDataAvailabilityHeader / Hash   :44-63, :92-108
 *   ErasuredNamespacedMerkleTree.Push  pkg/wrapper/nmt_wrapper.go:93-114 (+ isQuadrantZero :138-140)
 *   NMT HashLeaf / HashNode / computeNsRange / EmptyRoot
 *                           test/util/malicious/hasher.go:161-168,186-209,271-310
 *   RFC-6962 HashFromByteSlices  specs/src/specs/data_structures.md:174-204
 *   rsmt2d v0.12.0 erasureExtendSquare / computeRoots / Repair (upstream, not vendored;
 *     orchestration restated: Q1,Q2 from Q0 then Q3 from Q2 rows; Repair =
 *     prerepairSanityCheck + solveCrossword row-then-col sweep)
 *
 * SHA-256 is OpenSSL's (SHA-NI on x86 hosts) — the same primitive as Go's
 * crypto/sha256 used through consts.NewBaseHashFunc (global_consts.go:86).
 */
#define _POSIX_C_SOURCE 200809L
#include <math.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

static const uint8_t kParityNs[ORA_NS] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                          0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                          0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};

/* Low-level SHA256_* (SHA-NI block function, no per-call EVP algorithm fetch):
 * OpenSSL 3's one-shot SHA256() fetches the digest under a global lock on every
 * call, which made the threaded oracle slower than one thread. */
void ora_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  SHA256_CTX c;
  SHA256_Init(&c);
  if (len) SHA256_Update(&c, msg, len);
  SHA256_Final(out, &c);
}

/* ------------------------------------------------------------------ */
/* tiny parallel-for (rsmt2d fans out one goroutine per axis)          */
/* ------------------------------------------------------------------ */
typedef void (*task_fn)(void* ctx, int i);
typedef struct {
  task_fn fn;
  void* ctx;
  int n;
  atomic_int next;
} pfor_t;

static void* pfor_worker(void* p) {
  pfor_t* t = (pfor_t*)p;
  for (;;) {
    int i = atomic_fetch_add(&t->next, 1);
    if (i >= t->n) break;
    t->fn(t->ctx, i);
  }
  return NULL;
}

static void parallel_for(int n, int nthreads, task_fn fn, void* ctx) {
  if (nthreads <= 1 || n <= 1) {
    for (int i = 0; i < n; i++) fn(ctx, i);
    return;
  }
  if (nthreads > n) nthreads = n;
  pfor_t t;
  t.fn = fn;
  t.ctx = ctx;
  t.n = n;
  atomic_init(&t.next, 0);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, pfor_worker, &t);
  pfor_worker(&t);
  for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
  free(th);
}

/* ------------------------------------------------------------------ */
/* NMT                                                                 */
/* ------------------------------------------------------------------ */

/* HashNode (hasher.go:271-301) with computeNsRange (:303-310), IgnoreMaxNamespace=true */
static void nmt_hash_node(const uint8_t* l, const uint8_t* r, uint8_t* out) {
  uint8_t buf[1 + 2 * ORA_NODE];
  buf[0] = 0x01;
  memcpy(buf + 1, l, ORA_NODE);
  memcpy(buf + 1 + ORA_NODE, r, ORA_NODE);
  uint8_t res[ORA_NODE];
  memcpy(res, l, ORA_NS); /* min = left.min */
  if (memcmp(r, kParityNs, ORA_NS) == 0)
    memcpy(res + ORA_NS, l + ORA_NS, ORA_NS); /* right.min == MAX => left.max */
  else
    memcpy(res + ORA_NS, r + ORA_NS, ORA_NS);
  ora_sha256(buf, sizeof buf, res + 2 * ORA_NS);
  memcpy(out, res, ORA_NODE);
}

static void nmt_empty_root(uint8_t* out) { /* hasher.go:161-168 */
  memset(out, 0, 2 * ORA_NS);
  ora_sha256(NULL, 0, out + 2 * ORA_NS);
}

static int largest_pow2_below(int n) { /* getSplitPoint: largest power of 2 < n */
  int k = 1;
  while (k * 2 < n) k *= 2;
  return k;
}

static void nmt_compute_root(const uint8_t* leaf_nodes, int lo, int hi, uint8_t* out) {
  int n = hi - lo;
  if (n == 0) {
    nmt_empty_root(out);
    return;
  }
  if (n == 1) {
    memcpy(out, leaf_nodes + (size_t)lo * ORA_NODE, ORA_NODE);
    return;
  }
  int k = largest_pow2_below(n);
  uint8_t L[ORA_NODE], R[ORA_NODE];
  nmt_compute_root(leaf_nodes, lo, lo + k, L);
  nmt_compute_root(leaf_nodes, lo + k, hi, R);
  nmt_hash_node(L, R, out);
}

int ora_nmt_axis_root(uint64_t square_size, uint64_t axis_index, const uint8_t* const* leaves,
                      const size_t* lens, int n, uint8_t root[ORA_NODE], int* err_leaf) {
  uint8_t* nodes = (uint8_t*)malloc((size_t)(n > 0 ? n : 1) * ORA_NODE);
  const uint8_t* prev_ns = NULL;
  uint8_t* msg = NULL;
  size_t msg_cap = 0;
  int rc = ORA_OK;
  for (int i = 0; i < n; i++) {
    /* Push bounds check (nmt_wrapper.go:94-96) */
    if (axis_index + 1 > 2 * square_size || (uint64_t)i + 1 > 2 * square_size) {
      rc = ORA_E_PUSH_PAST;
      if (err_leaf) *err_leaf = i;
      break;
    }
    if (lens[i] < ORA_NS) { /* :97-99 */
      rc = ORA_E_NS_SHORT;
      if (err_leaf) *err_leaf = i;
      break;
    }
    const uint8_t* ns = ((uint64_t)i < square_size && axis_index < square_size) ? leaves[i] : kParityNs;
    if (prev_ns && memcmp(ns, prev_ns, ORA_NS) < 0) { /* nmt ErrInvalidPushOrder */
      rc = ORA_E_NS_ORDER;
      if (err_leaf) *err_leaf = i;
      break;
    }
    prev_ns = ns;
    size_t mlen = 1 + ORA_NS + lens[i];
    if (mlen > msg_cap) {
      free(msg);
      msg_cap = mlen;
      msg = (uint8_t*)malloc(msg_cap);
    }
    msg[0] = 0x00; /* LeafPrefix */
    memcpy(msg + 1, ns, ORA_NS);
    memcpy(msg + 1 + ORA_NS, leaves[i], lens[i]);
    uint8_t* node = nodes + (size_t)i * ORA_NODE;
    memcpy(node, ns, ORA_NS);
    memcpy(node + ORA_NS, ns, ORA_NS);
    ora_sha256(msg, mlen, node + 2 * ORA_NS);
  }
  if (rc == ORA_OK) nmt_compute_root(nodes, 0, n, root);
  free(msg);
  free(nodes);
  return rc;
}

/* ------------------------------------------------------------------ */
/* RFC-6962                                                            */
/* ------------------------------------------------------------------ */
static void merkle_rec(const uint8_t* const* items, const size_t* lens, int n, uint8_t out[32]) {
  if (n == 0) {
    ora_sha256(NULL, 0, out);
    return;
  }
  if (n == 1) {
    uint8_t* buf = (uint8_t*)malloc(1 + lens[0]);
    buf[0] = 0x00;
    memcpy(buf + 1, items[0], lens[0]);
    ora_sha256(buf, 1 + lens[0], out);
    free(buf);
    return;
  }
  int k = largest_pow2_below(n);
  uint8_t buf[65];
  buf[0] = 0x01;
  merkle_rec(items, lens, k, buf + 1);
  merkle_rec(items + k, lens + k, n - k, buf + 33);
  ora_sha256(buf, 65, out);
}

void ora_merkle_root(const uint8_t* const* items, const size_t* lens, int n, uint8_t out[32]) {
  merkle_rec(items, lens, n, out);
}

void ora_dah_hash(int n, const uint8_t* row_roots, const uint8_t* col_roots, uint8_t out[32]) {
  int total = 2 * n;
  const uint8_t** items = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)(total > 0 ? total : 1));
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)(total > 0 ? total : 1));
  for (int i = 0; i < n; i++) {
    items[i] = row_roots + (size_t)i * ORA_NODE;
    items[n + i] = col_roots + (size_t)i * ORA_NODE;
    lens[i] = lens[n + i] = ORA_NODE;
  }
  merkle_rec(items, lens, total, out);
  free(items);
  free(lens);
}

/* ------------------------------------------------------------------ */
/* 2-D extension (rsmt2d erasureExtendSquare)                          */
/* ------------------------------------------------------------------ */
typedef struct {
  int k;
  size_t L;
  uint8_t* eds;
  int phase; /* 0: rows 0..k-1 and cols 0..k-1 ; 1: rows k..2k-1 */
} ext_ctx;

static uint8_t* cell(uint8_t* eds, int w, size_t L, int r, int c) { return eds + ((size_t)r * w + c) * L; }

static void ext_task(void* p, int t) {
  ext_ctx* x = (ext_ctx*)p;
  int k = x->k, w = 2 * k;
  const uint8_t** data = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)k);
  uint8_t** par = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)k);
  if (x->phase == 0) {
    int i = t >> 1;
    if ((t & 1) == 0) { /* erasureExtendRow(i) */
      for (int j = 0; j < k; j++) {
        data[j] = cell(x->eds, w, x->L, i, j);
        par[j] = cell(x->eds, w, x->L, i, k + j);
      }
    } else { /* erasureExtendCol(i) */
      for (int j = 0; j < k; j++) {
        data[j] = cell(x->eds, w, x->L, j, i);
        par[j] = cell(x->eds, w, x->L, k + j, i);
      }
    }
  } else { /* erasureExtendRow(k + t) from Q2 */
    int i = k + t;
    for (int j = 0; j < k; j++) {
      data[j] = cell(x->eds, w, x->L, i, j);
      par[j] = cell(x->eds, w, x->L, i, k + j);
    }
  }
  ora_leo_encode(k, x->L, data, par);
  free(data);
  free(par);
}

int ora_extend(int k, size_t share_len, const uint8_t* ods, uint8_t* eds, int nthreads) {
  int w = 2 * k;
  for (int r = 0; r < k; r++)
    for (int c = 0; c < k; c++) memcpy(cell(eds, w, share_len, r, c), ods + ((size_t)r * k + c) * share_len, share_len);
  ext_ctx x = {k, share_len, eds, 0};
  parallel_for(2 * k, nthreads, ext_task, &x);
  x.phase = 1;
  parallel_for(k, nthreads, ext_task, &x);
  return ORA_OK;
}

/* ------------------------------------------------------------------ */
/* Roots (rsmt2d computeRoots with wrapper.NewConstructor(k))          */
/* ------------------------------------------------------------------ */
typedef struct {
  int k;
  size_t L;
  const uint8_t* eds;
  uint8_t* row_roots;
  uint8_t* col_roots;
  int* rcs;
} roots_ctx;

static void roots_task(void* p, int t) {
  roots_ctx* x = (roots_ctx*)p;
  int k = x->k, w = 2 * k;
  int axis = t / w, idx = t % w; /* 0 row, 1 col */
  const uint8_t** leaves = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)w);
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)w);
  for (int i = 0; i < w; i++) {
    size_t off = axis == 0 ? ((size_t)idx * w + i) : ((size_t)i * w + idx);
    leaves[i] = x->eds + off * x->L;
    lens[i] = x->L;
  }
  uint8_t* out = (axis == 0 ? x->row_roots : x->col_roots) + (size_t)idx * ORA_NODE;
  x->rcs[t] = ora_nmt_axis_root((uint64_t)k, (uint64_t)idx, leaves, lens, w, out, NULL);
  free(leaves);
  free(lens);
}

int ora_roots(int k, size_t share_len, const uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots,
              int nthreads, int* err_axis, int* err_index) {
  int w = 2 * k;
  int* rcs = (int*)calloc((size_t)2 * w, sizeof(int));
  roots_ctx x = {k, share_len, eds, row_roots, col_roots, rcs};
  parallel_for(2 * w, nthreads, roots_task, &x);
  int rc = ORA_OK;
  for (int t = 0; t < 2 * w; t++)
    if (rcs[t] != ORA_OK) {
      rc = rcs[t];
      if (err_axis) *err_axis = t / w;
      if (err_index) *err_index = t % w;
      break;
    }
  free(rcs);
  return rc;
}

/* ------------------------------------------------------------------ */
/* ExtendShares + NewDataAvailabilityHeader                            */
/* ------------------------------------------------------------------ */
int ora_extend_commit(int count, size_t share_len, const uint8_t* shares, uint8_t* eds_or_null,
                      uint8_t* row_roots, uint8_t* col_roots, uint8_t dah[32], int nthreads) {
  if (count <= 0 || (count & (count - 1)) != 0) return ORA_E_NOT_POW2; /* :67-69 */
  int width = (int)ceil(sqrt((double)count));
  if (width * width != count) return ORA_E_NOT_SQUARE; /* rsmt2d newDataSquare */
  if (share_len % 64 != 0) return ORA_E_SHARD_SIZE;   /* LeoRSCodec.ValidateChunkSize */
  int k = width;
  size_t eds_bytes = (size_t)4 * k * k * share_len;
  uint8_t* eds = eds_or_null ? eds_or_null : (uint8_t*)malloc(eds_bytes);
  ora_extend(k, share_len, shares, eds, nthreads);
  int rc = ora_roots(k, share_len, eds, row_roots, col_roots, nthreads, NULL, NULL);
  if (rc == ORA_OK) ora_dah_hash(2 * k, row_roots, col_roots, dah);
  if (!eds_or_null) free(eds);
  return rc;
}

/* ------------------------------------------------------------------ */
/* Throughput sample for the bench's cpu_baseline: `nthreads` workers  */
/* each run whole ExtendShares+NewDataAvailabilityHeader calls (one    */
/* block per call, single-threaded inside) on the same ODS until       */
/* `seconds` have passed — independent blocks spread over every core,  */
/* the CPU analogue of the GPU batch.  Returns blocks completed; the   */
/* wall time until the last worker finished goes to *elapsed.          */
/* ------------------------------------------------------------------ */
typedef struct {
  int count;
  size_t L;
  const uint8_t* ods;
  double deadline;
  atomic_long done;
  atomic_int rc;
  uint8_t dah0[32];
} tput_t;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* tput_worker(void* p) {
  tput_t* t = (tput_t*)p;
  const int k = (int)lround(sqrt((double)t->count));
  uint8_t* eds = (uint8_t*)malloc((size_t)4 * t->count * t->L);
  uint8_t* rr = (uint8_t*)malloc((size_t)2 * k * ORA_NODE);
  uint8_t* cr = (uint8_t*)malloc((size_t)2 * k * ORA_NODE);
  uint8_t dah[32];
  do {
    int rc = ora_extend_commit(t->count, t->L, t->ods, eds, rr, cr, dah, 1);
    if (rc != ORA_OK || memcmp(dah, t->dah0, 32) != 0) atomic_store(&t->rc, rc != ORA_OK ? rc : ORA_E_ARG);
    atomic_fetch_add(&t->done, 1);
  } while (now_s() < t->deadline);
  free(eds);
  free(rr);
  free(cr);
  return NULL;
}

long ora_extend_commit_throughput(int count, size_t share_len, const uint8_t* shares, int nthreads, double seconds,
                                  double* elapsed) {
  if (nthreads < 1) nthreads = 1;
  tput_t t;
  t.count = count;
  t.L = share_len;
  t.ods = shares;
  atomic_init(&t.done, 0);
  atomic_init(&t.rc, ORA_OK);
  { /* expected DAH (every call must reproduce it) */
    const int k = (int)lround(sqrt((double)count));
    uint8_t* rr = (uint8_t*)malloc((size_t)2 * k * ORA_NODE);
    uint8_t* cr = (uint8_t*)malloc((size_t)2 * k * ORA_NODE);
    int rc = ora_extend_commit(count, share_len, shares, NULL, rr, cr, t.dah0, 1);
    free(rr);
    free(cr);
    if (rc != ORA_OK) return rc;
  }
  const double t0 = now_s();
  t.deadline = t0 + seconds;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, tput_worker, &t);
  for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  free(th);
  if (elapsed) *elapsed = now_s() - t0;
  if (atomic_load(&t.rc) != ORA_OK) return atomic_load(&t.rc);
  return atomic_load(&t.done);
}

/* ------------------------------------------------------------------ */
/* Repair (rsmt2d v0.12.0 Repair)                                      */
/* ------------------------------------------------------------------ */
typedef struct {
  int k, w;
  size_t L;
  uint8_t* eds;
  uint8_t* present;
  const uint8_t* row_roots;
  const uint8_t* col_roots;
  int fft_decoder; /* 1: klauspost's Leopard reconstruct, 0: Lagrange (independent check) */
} rep_t;

static uint8_t* rcell(rep_t* R, int axis, int idx, int i) {
  int r = axis == 0 ? idx : i, c = axis == 0 ? i : idx;
  return R->eds + ((size_t)r * R->w + c) * R->L;
}
static int rpresent(rep_t* R, int axis, int idx, int i) {
  int r = axis == 0 ? idx : i, c = axis == 0 ? i : idx;
  return R->present[(size_t)r * R->w + c];
}
static void rset_present(rep_t* R, int axis, int idx, int i) {
  int r = axis == 0 ? idx : i, c = axis == 0 ? i : idx;
  R->present[(size_t)r * R->w + c] = 1;
}

/* noMissingData(vector, skip) */
static int axis_complete(rep_t* R, int axis, int idx, int skip) {
  for (int i = 0; i < R->w; i++)
    if (i != skip && !rpresent(R, axis, idx, i)) return 0;
  return 1;
}

/* computeSharesRoot via the tree constructor; returns 1 if root matches. */
static int verify_root(rep_t* R, int axis, int idx, const uint8_t* const* shares) {
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)R->w);
  for (int i = 0; i < R->w; i++) lens[i] = R->L;
  uint8_t root[ORA_NODE];
  int rc = ora_nmt_axis_root((uint64_t)R->k, (uint64_t)idx, shares, lens, R->w, root, NULL);
  free(lens);
  if (rc != ORA_OK) return 0; /* any error computing the root is byzantine */
  const uint8_t* want = (axis == 0 ? R->row_roots : R->col_roots) + (size_t)idx * ORA_NODE;
  return memcmp(root, want, ORA_NODE) == 0;
}

static int verify_parity(rep_t* R, int axis, int idx) {
  int k = R->k;
  const uint8_t** data = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)k);
  uint8_t** par = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)k);
  uint8_t* buf = (uint8_t*)malloc((size_t)k * R->L);
  for (int i = 0; i < k; i++) {
    data[i] = rcell(R, axis, idx, i);
    par[i] = buf + (size_t)i * R->L;
  }
  ora_leo_encode(k, R->L, data, par);
  int ok = 1;
  for (int i = 0; i < k && ok; i++) ok = memcmp(par[i], rcell(R, axis, idx, k + i), R->L) == 0;
  free(data);
  free(par);
  free(buf);
  return ok;
}

/* solveCrosswordRow / solveCrosswordCol. returns <0 error, else sets *solved,*progress */
static int solve_axis(rep_t* R, int axis, int idx, int* solved, int* progress, int* bad_axis, int* bad_idx) {
  int w = R->w, k = R->k;
  *solved = 0;
  *progress = 0;
  if (axis_complete(R, axis, idx, -1)) {
    *solved = 1;
    return ORA_OK;
  }
  /* rebuildShares -> codec.Decode */
  uint8_t* buf = (uint8_t*)malloc((size_t)w * R->L);
  uint8_t** sh = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)w);
  uint8_t* pres = (uint8_t*)malloc((size_t)w);
  for (int i = 0; i < w; i++) {
    sh[i] = buf + (size_t)i * R->L;
    pres[i] = (uint8_t)rpresent(R, axis, idx, i);
    if (pres[i]) memcpy(sh[i], rcell(R, axis, idx, i), R->L);
  }
  int rc = R->fft_decoder ? ora_leo_decode_fft(k, R->L, sh, pres) : ora_leo_decode(k, R->L, sh, pres);
  if (rc != ORA_OK) { /* not decodable yet: no progress, no error */
    free(buf);
    free(sh);
    free(pres);
    return ORA_OK;
  }
  int result = ORA_OK;
  if (!verify_root(R, axis, idx, (const uint8_t* const*)sh)) {
    result = ORA_E_BYZANTINE;
    *bad_axis = axis;
    *bad_idx = idx;
    goto out;
  }
  /* newly completed orthogonal vectors */
  for (int j = 0; j < w; j++) {
    int oaxis = 1 - axis;
    if (rpresent(R, oaxis, j, idx)) continue;
    if (axis_complete(R, oaxis, j, idx)) {
      const uint8_t** ov = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)w);
      for (int i = 0; i < w; i++) ov[i] = (i == idx) ? sh[j] : rcell(R, oaxis, j, i);
      int ok = verify_root(R, oaxis, j, ov);
      free(ov);
      if (!ok) {
        result = ORA_E_BYZANTINE;
        *bad_axis = oaxis;
        *bad_idx = j;
        goto out;
      }
    }
  }
  for (int i = 0; i < w; i++)
    if (!rpresent(R, axis, idx, i)) {
      memcpy(rcell(R, axis, idx, i), sh[i], R->L);
      rset_present(R, axis, idx, i);
    }
  *solved = 1;
  *progress = 1;
out:
  free(buf);
  free(sh);
  free(pres);
  return result;
}

int ora_repair(int k, size_t share_len, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
               const uint8_t* col_roots, int* err_axis, int* err_index) {
  return ora_repair_ex(k, share_len, eds, present, row_roots, col_roots, err_axis, err_index, 0);
}

int ora_repair_ex(int k, size_t share_len, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
                  const uint8_t* col_roots, int* err_axis, int* err_index, int fft_decoder) {
  rep_t R = {k, 2 * k, share_len, eds, present, row_roots, col_roots, fft_decoder};
  int w = 2 * k;
  /* prerepairSanityCheck */
  for (int i = 0; i < w; i++) {
    int rowc = axis_complete(&R, 0, i, -1), colc = axis_complete(&R, 1, i, -1);
    for (int step = 0; step < 4; step++) {
      int axis = step & 1;
      int complete = axis == 0 ? rowc : colc;
      if (!complete) continue;
      int ok;
      if (step < 2) {
        const uint8_t** v = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)w);
        for (int j = 0; j < w; j++) v[j] = rcell(&R, axis, i, j);
        ok = verify_root(&R, axis, i, v);
        free(v);
      } else {
        ok = verify_parity(&R, axis, i);
      }
      if (!ok) {
        if (err_axis) *err_axis = axis;
        if (err_index) *err_index = i;
        return ORA_E_BYZANTINE;
      }
    }
  }
  /* solveCrossword */
  for (;;) {
    int solved = 1, progress = 0;
    for (int i = 0; i < w; i++) {
      for (int axis = 0; axis < 2; axis++) {
        int s, p, ba = 0, bi = 0;
        int rc = solve_axis(&R, axis, i, &s, &p, &ba, &bi);
        if (rc != ORA_OK) {
          if (err_axis) *err_axis = ba;
          if (err_index) *err_index = bi;
          return rc;
        }
        solved = solved && s;
        progress = progress || p;
      }
    }
    if (solved) break;
    if (!progress) return ORA_E_UNREPAIRABLE;
  }
  return ORA_OK;
}

/* ------------------------------------------------------------------ */
/* Input generator                                        */
/* ------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static int share_cmp(const void* a, const void* b) { return memcmp(a, b, ORA_SHARE); }

void ora_gen_ods(int k, uint64_t seed, uint8_t* ods) {
  uint64_t s = seed;
  size_t n = (size_t)k * k;
  for (size_t i = 0; i < n; i++) {
    uint8_t* sh = ods + i * ORA_SHARE;
    uint8_t rnd[496];
    for (int w = 0; w < 62; w++) {
      uint64_t v = splitmix64(&s);
      memcpy(rnd + 8 * w, &v, 8);
    }
    memset(sh, 0, 19);
    memcpy(sh + 19, rnd, 10);
    memcpy(sh + 29, rnd + 10, ORA_SHARE - 29);
  }
  qsort(ods, n, ORA_SHARE, share_cmp);
}

/* ------------------------------------------------------------------ */
/* NMT building blocks for inclusion.c                                 */
/* ------------------------------------------------------------------ */
/* HashNode (hasher.go:271-310) for a namespace of ns_len bytes; ns_len = 29 is nmt_hash_node. */
void ora_nmt_hash_node_ns(int ns_len, const uint8_t* l, const uint8_t* r, uint8_t* out) {
  const int node = 2 * ns_len + 32;
  uint8_t buf[1 + 2 * (2 * 64 + 32)], res[2 * 64 + 32];
  int rmax = 1;
  for (int i = 0; i < ns_len; i++) rmax &= r[i] == 0xFF;
  buf[0] = 0x01;
  memcpy(buf + 1, l, (size_t)node);
  memcpy(buf + 1 + node, r, (size_t)node);
  memcpy(res, l, (size_t)ns_len);
  memcpy(res + ns_len, rmax ? l + ns_len : r + ns_len, (size_t)ns_len);
  ora_sha256(buf, 1 + 2 * (size_t)node, res + 2 * ns_len);
  memcpy(out, res, (size_t)node);
}

/* HashLeaf (hasher.go:186-209) of ns ‖ data: ns ‖ ns ‖ SHA256(0x00 ‖ ns ‖ data) */
void ora_nmt_leaf_node(const uint8_t* ns, const uint8_t* data, size_t len, uint8_t* out) {
  uint8_t* msg = (uint8_t*)malloc(1 + ORA_NS + len);
  msg[0] = 0x00;
  memcpy(msg + 1, ns, ORA_NS);
  memcpy(msg + 1 + ORA_NS, data, len);
  uint8_t node[ORA_NODE];
  memcpy(node, ns, ORA_NS);
  memcpy(node + ORA_NS, ns, ORA_NS);
  ora_sha256(msg, 1 + ORA_NS + len, node + 2 * ORA_NS);
  memcpy(out, node, ORA_NODE);
  free(msg);
}

/* nmt computeRoot over n leaf nodes */
void ora_nmt_root_of_nodes(const uint8_t* leaf_nodes, int n, uint8_t* out) { nmt_compute_root(leaf_nodes, 0, n, out); }
