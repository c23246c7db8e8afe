/*
 * rsmt2d_axes.c — rsmt2d v0.12.0's own call pattern over the per-axis seams, as a plain C caller.
 *
 * Under -tags rocm, appconsts.DefaultCodec is the GPU codec (go/pkg_da/extend_rocm.go) and squares returned by
 * cda.ExtendShares carry it, so every unpatched rsmt2d caller -- ComputeExtendedDataSquare with
 * appconsts.DefaultCodec() (test/util/malicious/tree.go:70, pkg/inclusion/nmt_caching_test.go:122, celestia-node),
 * and (*ExtendedDataSquare).Repair on a returned square -- reaches libcda one axis at a time through
 * Codec.Encode / Codec.Decode (cda_rs_encode / cda_rs_decode) and the wrapper tree's Root (cda_nmt_axis_root,
 * pkg/wrapper/nmt_wrapper.go:118-124).  This program makes exactly those calls, in rsmt2d's order and with its
 * fan-out (one goroutine per axis in erasureExtendSquare / computeRoots / prerepairSanityCheck, the crossword
 * sequential), from pageable malloc'd buffers standing in for Go slices, so that bench.py (`per_axis`) can time
 * the seams and tests/test_per_axis_gpu.py can check their bytes.
 *
 * The same driver runs over the CPU restatement (oracle/liboracle.so: ora_leo_encode, ora_leo_decode_fft,
 * ora_nmt_axis_root) as bench.py's CPU baseline of those shapes.  The backend library is dlopen'ed by path, so the
 * GPU run never loads the oracle and the CPU run never loads libcda.
 *
 *   rsmt2d_axes cda|oracle <lib.so> single <k> <reps> <ods.bin>
 *       one Encode (k x 512 B), one Decode (2k shards, every other one present), one axis Root (2k leaves), each
 *       `reps` times; prints {"encode_us": [min, median], "decode_us": [...], "root_us": [...]}
 *   rsmt2d_axes cda|oracle <lib.so> extend <k> <threads> <reps> <ods.bin> <out_dir>
 *       ComputeExtendedDataSquare(ods, codec, wrapper.NewConstructor(k)) + RowRoots/ColRoots: erasureExtendSquare
 *       (k goroutines: row i then column i; then k goroutines: row k+i) and computeRoots (2k goroutines: row root i,
 *       column root i) on `threads` worker threads; writes eds.bin, row_roots.bin, col_roots.bin of the last rep
 *   rsmt2d_axes cda|oracle <lib.so> repair <k> <threads> <reps> <eds.bin> <present.bin> <roots.bin> <out_dir>
 *       Repair(rowRoots, colRoots): prerepairSanityCheck (parallel) + solveCrossword (sequential, row then column
 *       per index, until solved or no progress); roots.bin = row roots ‖ column roots (90 B each); writes
 *       repaired.bin of the last rep and prints rc, byzantine axis / index and the call counts
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>
#include <unistd.h>

#define SHARE 512
#define NS 29
#define NODE 90

/* ---- backends ------------------------------------------------------------------------------------------------ */
typedef struct {
  int32_t code, axis, index, leaf, block;
} err_info; /* cda_err_info */

static int use_cda;
/* libcda */
static void* g_ctx;
static int (*p_cda_init)(int, void**);
static void (*p_cda_free)(void*);
static int (*p_cda_rs_encode)(void*, uint32_t, uint32_t, const uint8_t*, uint8_t*);
static int (*p_cda_rs_decode)(void*, uint32_t, uint32_t, uint8_t*, const uint8_t*);
static int (*p_cda_nmt_axis_root)(void*, uint64_t, uint64_t, uint32_t, uint32_t, const uint8_t*, uint8_t*, err_info*);
static int (*p_cda_profile_enable)(void*, int);
static int (*p_cda_profile_read)(void*, char*, size_t, double*, int64_t*, int);
/* oracle */
static int (*p_ora_encode)(int, size_t, const uint8_t* const*, uint8_t* const*);
static int (*p_ora_decode)(int, size_t, uint8_t* const*, const uint8_t*);
static int (*p_ora_root)(uint64_t, uint64_t, const uint8_t* const*, const size_t*, int, uint8_t*, int*);

static atomic_long n_enc, n_dec, n_root;

static void* sym(void* h, const char* name) {
  void* p = dlsym(h, name);
  if (!p) {
    fprintf(stderr, "missing symbol %s\n", name);
    exit(2);
  }
  return p;
}

static void load_backend(const char* kind, const char* path) {
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "dlopen %s: %s\n", path, dlerror());
    exit(2);
  }
  use_cda = strcmp(kind, "cda") == 0;
  if (use_cda) {
    *(void**)&p_cda_init = sym(h, "cda_init");
    *(void**)&p_cda_free = sym(h, "cda_free");
    *(void**)&p_cda_rs_encode = sym(h, "cda_rs_encode");
    *(void**)&p_cda_rs_decode = sym(h, "cda_rs_decode");
    *(void**)&p_cda_nmt_axis_root = sym(h, "cda_nmt_axis_root");
    *(void**)&p_cda_profile_enable = sym(h, "cda_profile_enable");
    *(void**)&p_cda_profile_read = sym(h, "cda_profile_read");
    if (p_cda_init(0, &g_ctx) != 0) {
      fprintf(stderr, "cda_init failed\n");
      exit(2);
    }
  } else {
    *(void**)&p_ora_encode = sym(h, "ora_leo_encode");
    *(void**)&p_ora_decode = sym(h, "ora_leo_decode_fft");
    *(void**)&p_ora_root = sym(h, "ora_nmt_axis_root");
  }
}

/* Codec.Encode: k contiguous data shards -> k contiguous parity shards */
static int enc(int k, const uint8_t* data, uint8_t* parity) {
  atomic_fetch_add(&n_enc, 1);
  if (use_cda) return p_cda_rs_encode(g_ctx, (uint32_t)k, SHARE, data, parity);
  const uint8_t* d[512];
  uint8_t* p[512];
  for (int i = 0; i < k; i++) {
    d[i] = data + (size_t)i * SHARE;
    p[i] = parity + (size_t)i * SHARE;
  }
  return p_ora_encode(k, SHARE, d, p);
}

/* Codec.Decode: 2k contiguous shards, present[i]; missing shards filled in place; 0 or an error */
static int dec(int k, uint8_t* shards, const uint8_t* present) {
  atomic_fetch_add(&n_dec, 1);
  if (use_cda) return p_cda_rs_decode(g_ctx, (uint32_t)k, SHARE, shards, present);
  uint8_t* s[1024];
  for (int i = 0; i < 2 * k; i++) s[i] = shards + (size_t)i * SHARE;
  return p_ora_decode(k, SHARE, s, present);
}

/* wrapper tree: Push the 2k contiguous leaves, Root */
static int root(int k, int axis_index, const uint8_t* leaves, uint8_t out[NODE]) {
  atomic_fetch_add(&n_root, 1);
  const int n = 2 * k;
  if (use_cda) {
    err_info e;
    return p_cda_nmt_axis_root(g_ctx, (uint64_t)k, (uint64_t)axis_index, (uint32_t)n, SHARE, leaves, out, &e);
  }
  const uint8_t* l[1024];
  size_t lens[1024];
  for (int i = 0; i < n; i++) {
    l[i] = leaves + (size_t)i * SHARE;
    lens[i] = SHARE;
  }
  int el = 0;
  return p_ora_root((uint64_t)k, (uint64_t)axis_index, l, lens, n, out, &el);
}

/* ---- helpers ------------------------------------------------------------------------------------------------- */
static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint8_t* read_all(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f || fseek(f, 0, SEEK_END) != 0) {
    fprintf(stderr, "cannot read %s\n", path);
    exit(2);
  }
  const long sz = ftell(f);
  uint8_t* b = malloc((size_t)sz + 1);
  rewind(f);
  if (sz < 0 || fread(b, 1, (size_t)sz, f) != (size_t)sz) exit(2);
  fclose(f);
  *n = (size_t)sz;
  return b;
}

static void write_file(const char* dir, const char* name, const void* p, size_t n) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(p, 1, n, f) != n) {
    fprintf(stderr, "cannot write %s\n", path);
    exit(2);
  }
  fclose(f);
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}
static void min_med(double* t, int n, double* mn, double* med) {
  qsort(t, (size_t)n, sizeof *t, cmp_d);
  *mn = t[0];
  *med = n % 2 ? t[n / 2] : 0.5 * (t[n / 2 - 1] + t[n / 2]);
}

/* ---- worker pool: one task per "goroutine", pulled by `threads` OS threads ---------------------------------- */
typedef void (*task_fn)(int i, void* arg);
typedef struct {
  pthread_t* th;
  int n;
  pthread_barrier_t start, end;
  task_fn fn;
  void* arg;
  int ntasks;
  atomic_int next;
  atomic_int rc;
  int quit;
} pool_t;
static pool_t P;

static void* worker(void* unused) {
  (void)unused;
  for (;;) {
    pthread_barrier_wait(&P.start);
    if (P.quit) return NULL;
    for (;;) {
      const int i = atomic_fetch_add(&P.next, 1);
      if (i >= P.ntasks) break;
      P.fn(i, P.arg);
    }
    pthread_barrier_wait(&P.end);
  }
}
static void pool_init(int n) {
  P.n = n;
  P.th = calloc((size_t)n, sizeof(pthread_t));
  pthread_barrier_init(&P.start, NULL, (unsigned)n + 1);
  pthread_barrier_init(&P.end, NULL, (unsigned)n + 1);
  for (int i = 0; i < n; i++) pthread_create(&P.th[i], NULL, worker, NULL);
}
/* errgroup.Go for each i < ntasks, then Wait */
static void pool_run(task_fn fn, void* arg, int ntasks) {
  P.fn = fn;
  P.arg = arg;
  P.ntasks = ntasks;
  atomic_store(&P.next, 0);
  pthread_barrier_wait(&P.start);
  pthread_barrier_wait(&P.end);
}
static void pool_quit(void) {
  P.quit = 1;
  pthread_barrier_wait(&P.start);
  for (int i = 0; i < P.n; i++) pthread_join(P.th[i], NULL);
}
static void set_rc(int rc) {
  if (rc) {
    int z = 0;
    atomic_compare_exchange_strong(&P.rc, &z, rc);
  }
}

/* ---- the square -------------------------------------------------------------------------------------------- */
typedef struct {
  int k, w;
  uint8_t* eds;      /* w*w*512, row-major */
  uint8_t* present;  /* w*w (repair) */
  uint8_t* rr;       /* w*90 */
  uint8_t* cr;       /* w*90 */
  const uint8_t* want_rr;
  const uint8_t* want_cr;
} sq_t;

static uint8_t* cell(sq_t* s, int r, int c) { return s->eds + ((size_t)r * s->w + c) * SHARE; }

/* rsmt2d erasureExtendRow(i): Encode(rowSlice(i, 0, k)) -> setRowSlice(i, k, parity) */
static int extend_row(sq_t* s, int i) {
  const int k = s->k;
  uint8_t* par = malloc((size_t)k * SHARE);
  /* Codec.Encode flattens the row's k cells (go/cda/codec.go flatten): one copy */
  uint8_t* flat = malloc((size_t)k * SHARE);
  memcpy(flat, cell(s, i, 0), (size_t)k * SHARE);
  const int rc = enc(k, flat, par);
  if (!rc) memcpy(cell(s, i, k), par, (size_t)k * SHARE);
  free(flat);
  free(par);
  return rc;
}
/* rsmt2d erasureExtendCol(i): Encode(colSlice(0, i, k)) -> setColSlice(k, i, parity) */
static int extend_col(sq_t* s, int i) {
  const int k = s->k;
  uint8_t* flat = malloc((size_t)k * SHARE);
  uint8_t* par = malloc((size_t)k * SHARE);
  for (int r = 0; r < k; r++) memcpy(flat + (size_t)r * SHARE, cell(s, r, i), SHARE);
  const int rc = enc(k, flat, par);
  if (!rc)
    for (int r = 0; r < k; r++) memcpy(cell(s, k + r, i), par + (size_t)r * SHARE, SHARE);
  free(flat);
  free(par);
  return rc;
}
/* one axis pushed into a fresh wrapper tree (Push appends each share: the tree holds a copy), then Root */
static int axis_root(sq_t* s, int axis, int idx, uint8_t out[NODE]) {
  const int w = s->w;
  uint8_t* leaves = malloc((size_t)w * SHARE);
  for (int j = 0; j < w; j++) memcpy(leaves + (size_t)j * SHARE, axis == 0 ? cell(s, idx, j) : cell(s, j, idx), SHARE);
  const int rc = root(s->k, idx, leaves, out);
  free(leaves);
  return rc;
}

static void t_phase1(int i, void* a) {  /* erasureExtendSquare, first loop: row i then column i */
  sq_t* s = a;
  set_rc(extend_row(s, i));
  set_rc(extend_col(s, i));
}
static void t_phase2(int i, void* a) {  /* second loop: rows k..2k-1 (Q2 -> Q3) */
  sq_t* s = a;
  set_rc(extend_row(s, s->k + i));
}
static void t_roots(int i, void* a) {  /* computeRoots: row root i, column root i */
  sq_t* s = a;
  set_rc(axis_root(s, 0, i, s->rr + (size_t)i * NODE));
  set_rc(axis_root(s, 1, i, s->cr + (size_t)i * NODE));
}

/* ---- Repair (rsmt2d v0.12.0 extendeddatasquare.go / repair.go) --------------------------------------------- */
static int present_at(sq_t* s, int axis, int idx, int j) {
  return s->present[axis == 0 ? (size_t)idx * s->w + j : (size_t)j * s->w + idx];
}
static int complete(sq_t* s, int axis, int idx, int skip) { /* noMissingData(vector, skip) */
  for (int j = 0; j < s->w; j++)
    if (j != skip && !present_at(s, axis, idx, j)) return 0;
  return 1;
}
static int root_matches(sq_t* s, int axis, int idx, const uint8_t* leaves) {
  uint8_t r[NODE];
  if (root(s->k, idx, leaves, r)) return 0;  /* any error computing the root is a mismatch */
  return memcmp(r, (axis == 0 ? s->want_rr : s->want_cr) + (size_t)idx * NODE, NODE) == 0;
}
static uint8_t* gather(sq_t* s, int axis, int idx) {
  uint8_t* v = malloc((size_t)s->w * SHARE);
  for (int j = 0; j < s->w; j++)
    memcpy(v + (size_t)j * SHARE, axis == 0 ? cell(s, idx, j) : cell(s, j, idx), SHARE);
  return v;
}

static atomic_int sanity_bad;  /* lowest (index * 4 + step) that failed, or INT32_MAX */
static void t_sanity(int i, void* a) {
  sq_t* s = a;
  const int k = s->k;
  const int rowc = complete(s, 0, i, -1), colc = complete(s, 1, i, -1);
  for (int step = 0; step < 4; step++) {
    const int axis = step & 1;
    if (!(axis == 0 ? rowc : colc)) continue;
    uint8_t* v = gather(s, axis, i);
    int ok;
    if (step < 2) {
      ok = root_matches(s, axis, i, v);
    } else {  /* codec.Encode(data half) == parity half */
      uint8_t* par = malloc((size_t)k * SHARE);
      ok = enc(k, v, par) == 0 && memcmp(par, v + (size_t)k * SHARE, (size_t)k * SHARE) == 0;
      free(par);
    }
    free(v);
    if (!ok) {
      int cur = atomic_load(&sanity_bad), me = i * 4 + step;
      while (me < cur && !atomic_compare_exchange_weak(&sanity_bad, &cur, me)) {
      }
      return;
    }
  }
}

/* solveCrosswordRow / Col: 1 solved+progress, 0 not decodable yet (or complete: *solved), <0 Byzantine */
static int solve_axis(sq_t* s, int axis, int idx, int* solved, int* progress, int* bad_axis, int* bad_idx) {
  const int w = s->w, k = s->k;
  *solved = *progress = 0;
  if (complete(s, axis, idx, -1)) {
    *solved = 1;
    return 0;
  }
  uint8_t* sh = gather(s, axis, idx);
  uint8_t* pres = malloc((size_t)w);
  for (int j = 0; j < w; j++) pres[j] = (uint8_t)present_at(s, axis, idx, j);
  int rc = 0;
  if (dec(k, sh, pres) != 0) goto out; /* too few shares: no progress, no error */
  if (!root_matches(s, axis, idx, sh)) {
    *bad_axis = axis;
    *bad_idx = idx;
    rc = -1;
    goto out;
  }
  for (int j = 0; j < w; j++) { /* newly completed orthogonal vectors */
    const int oaxis = 1 - axis;
    if (present_at(s, oaxis, j, idx)) continue;
    if (!complete(s, oaxis, j, idx)) continue;
    uint8_t* ov = gather(s, oaxis, j);
    memcpy(ov + (size_t)idx * SHARE, sh + (size_t)j * SHARE, SHARE);
    const int ok = root_matches(s, oaxis, j, ov);
    free(ov);
    if (!ok) {
      *bad_axis = oaxis;
      *bad_idx = j;
      rc = -1;
      goto out;
    }
  }
  for (int j = 0; j < w; j++)
    if (!present_at(s, axis, idx, j)) {
      memcpy(axis == 0 ? cell(s, idx, j) : cell(s, j, idx), sh + (size_t)j * SHARE, SHARE);
      s->present[axis == 0 ? (size_t)idx * w + j : (size_t)j * w + idx] = 1;
    }
  *solved = *progress = 1;
out:
  free(sh);
  free(pres);
  return rc;
}

/* 0 ok, 1 unrepairable, 2 byzantine */
static int repair(sq_t* s, int* bad_axis, int* bad_idx) {
  atomic_store(&sanity_bad, INT32_MAX);
  pool_run(t_sanity, s, s->w);
  const int sb = atomic_load(&sanity_bad);
  if (sb != INT32_MAX) {
    *bad_axis = (sb % 4) & 1;
    *bad_idx = sb / 4;
    return 2;
  }
  for (;;) {
    int all = 1, prog = 0;
    for (int i = 0; i < s->w; i++)
      for (int axis = 0; axis < 2; axis++) {
        int sv, pg;
        if (solve_axis(s, axis, i, &sv, &pg, bad_axis, bad_idx) < 0) return 2;
        all = all && sv;
        prog = prog || pg;
      }
    if (all) return 0;
    if (!prog) return 1;
  }
}

/* ---- modes ------------------------------------------------------------------------------------------------- */
static void mode_single(int k, int reps, const uint8_t* ods) {
  const int w = 2 * k;
  uint8_t* data = malloc((size_t)k * SHARE);
  uint8_t* par = malloc((size_t)k * SHARE);
  memcpy(data, ods, (size_t)k * SHARE);  /* ODS row 0 */
  uint8_t* sh = malloc((size_t)w * SHARE);
  uint8_t* pres = malloc((size_t)w);
  uint8_t rt[NODE];
  double* t = malloc(sizeof(double) * (size_t)reps);
  double r[3][2];
  if (enc(k, data, par)) exit(3);
  for (int i = 0; i < reps; i++) {
    const double a = now_s();
    if (enc(k, data, par)) exit(3);
    t[i] = now_s() - a;
  }
  min_med(t, reps, &r[0][0], &r[0][1]);
  memcpy(sh, data, (size_t)k * SHARE);
  memcpy(sh + (size_t)k * SHARE, par, (size_t)k * SHARE);
  for (int j = 0; j < w; j++) pres[j] = (uint8_t)(j % 2 == 0);
  for (int i = 0; i < reps; i++) {
    const double a = now_s();
    if (dec(k, sh, pres)) exit(3);
    t[i] = now_s() - a;
  }
  min_med(t, reps, &r[1][0], &r[1][1]);
  if (memcmp(sh, data, (size_t)k * SHARE) || memcmp(sh + (size_t)k * SHARE, par, (size_t)k * SHARE)) {
    fprintf(stderr, "decode differs from the encoded codeword\n");
    exit(3);
  }
  for (int i = 0; i < reps; i++) {
    const double a = now_s();
    if (root(k, 0, sh, rt)) exit(3);
    t[i] = now_s() - a;
  }
  min_med(t, reps, &r[2][0], &r[2][1]);
  printf("{\"encode_us\": [%.1f, %.1f], \"decode_us\": [%.1f, %.1f], \"root_us\": [%.1f, %.1f], \"reps\": %d, "
         "\"root0\": \"",
         1e6 * r[0][0], 1e6 * r[0][1], 1e6 * r[1][0], 1e6 * r[1][1], 1e6 * r[2][0], 1e6 * r[2][1], reps);
  for (int i = 0; i < NODE; i++) printf("%02x", rt[i]);
  printf("\"");
  if (use_cda) {  /* the device share of each call: the same calls again with libcda's per-launch HIP events */
    p_cda_profile_enable(g_ctx, 1);
    for (int i = 0; i < 50; i++) {
      if (enc(k, data, par) || dec(k, sh, pres) || root(k, 0, sh, rt)) exit(3);
    }
    char names[1024];
    double ms[16];
    int64_t cnt[16];
    const int nk = p_cda_profile_read(g_ctx, names, sizeof names, ms, cnt, 16);
    p_cda_profile_enable(g_ctx, 0);
    printf(", \"kernel_us\": {");
    const char* nm = names;
    for (int i = 0; i < nk; i++) {
      printf("%s\"%s\": %.1f", i ? ", " : "", nm, 1e3 * ms[i] / (double)(cnt[i] ? cnt[i] : 1));
      nm += strlen(nm) + 1;
    }
    printf("}");
  }
  printf("}\n");
}

static void mode_extend(int k, int threads, int reps, const uint8_t* ods, const char* out) {
  const int w = 2 * k;
  sq_t s = {k, w, malloc((size_t)w * w * SHARE), NULL, malloc((size_t)w * NODE), malloc((size_t)w * NODE), NULL, NULL};
  double* te = malloc(sizeof(double) * (size_t)reps);
  double* tr = malloc(sizeof(double) * (size_t)reps);
  double* tt = malloc(sizeof(double) * (size_t)reps);
  pool_init(threads);
  for (int it = -1; it < reps; it++) { /* it = -1: untimed warm-up */
    memset(s.eds, 0, (size_t)w * w * SHARE);
    for (int r = 0; r < k; r++) memcpy(cell(&s, r, 0), ods + (size_t)r * k * SHARE, (size_t)k * SHARE);
    atomic_store(&P.rc, 0);
    struct rusage u0, u1;
    getrusage(RUSAGE_SELF, &u0);
    const double a = now_s();
    pool_run(t_phase1, &s, k);
    pool_run(t_phase2, &s, k);
    const double b = now_s();
    pool_run(t_roots, &s, w);
    const double c = now_s();
    getrusage(RUSAGE_SELF, &u1);
    if (getenv("RSMT2D_AXES_VERBOSE")) /* per-rep phases and the process's CPU time over the rep (diagnosis) */
      fprintf(stderr, "rep %d extend %.3f roots %.3f ms cpu user %.1f sys %.1f ms ctxsw %ld/%ld\n", it, 1e3 * (b - a),
              1e3 * (c - b),
              1e3 * (u1.ru_utime.tv_sec - u0.ru_utime.tv_sec) + 1e-3 * (u1.ru_utime.tv_usec - u0.ru_utime.tv_usec),
              1e3 * (u1.ru_stime.tv_sec - u0.ru_stime.tv_sec) + 1e-3 * (u1.ru_stime.tv_usec - u0.ru_stime.tv_usec),
              u1.ru_nvcsw - u0.ru_nvcsw, u1.ru_nivcsw - u0.ru_nivcsw);
    if (atomic_load(&P.rc)) {
      fprintf(stderr, "call failed rc=%d\n", atomic_load(&P.rc));
      exit(3);
    }
    if (it >= 0) {
      te[it] = b - a;
      tr[it] = c - b;
      tt[it] = c - a;
    }
  }
  pool_quit();
  write_file(out, "eds.bin", s.eds, (size_t)w * w * SHARE);
  write_file(out, "row_roots.bin", s.rr, (size_t)w * NODE);
  write_file(out, "col_roots.bin", s.cr, (size_t)w * NODE);
  double e0, e1, r0, r1, t0, t1;
  min_med(te, reps, &e0, &e1);
  min_med(tr, reps, &r0, &r1);
  min_med(tt, reps, &t0, &t1);
  printf("{\"extend_ms\": [%.3f, %.3f], \"roots_ms\": [%.3f, %.3f], \"total_ms\": [%.3f, %.3f], \"threads\": %d, "
         "\"reps\": %d, \"encodes\": %ld, \"roots\": %ld}\n",
         1e3 * e0, 1e3 * e1, 1e3 * r0, 1e3 * r1, 1e3 * t0, 1e3 * t1, threads, reps, atomic_load(&n_enc) / (reps + 1),
         atomic_load(&n_root) / (reps + 1));
}

static void mode_repair(int k, int threads, int reps, const uint8_t* eds0, const uint8_t* pres0, const uint8_t* roots,
                        const char* out) {
  const int w = 2 * k;
  sq_t s = {k, w, malloc((size_t)w * w * SHARE), malloc((size_t)w * w), NULL, NULL, roots, roots + (size_t)w * NODE};
  double* t = malloc(sizeof(double) * (size_t)reps);
  int rc = 0, ba = -1, bi = -1;
  long calls[3] = {0, 0, 0};
  pool_init(threads);
  for (int it = -1; it < reps; it++) {
    memcpy(s.present, pres0, (size_t)w * w);
    for (size_t i = 0; i < (size_t)w * w; i++) /* missing cells hold nothing (nil in rsmt2d) */
      if (pres0[i]) memcpy(s.eds + i * SHARE, eds0 + i * SHARE, SHARE);
      else memset(s.eds + i * SHARE, 0, SHARE);
    const long e0 = atomic_load(&n_enc), d0 = atomic_load(&n_dec), r0 = atomic_load(&n_root);
    ba = bi = -1;
    const double a = now_s();
    rc = repair(&s, &ba, &bi);
    const double b = now_s();
    calls[0] = atomic_load(&n_enc) - e0;
    calls[1] = atomic_load(&n_dec) - d0;
    calls[2] = atomic_load(&n_root) - r0;
    if (it >= 0) t[it] = b - a;
  }
  pool_quit();
  write_file(out, "repaired.bin", s.eds, (size_t)w * w * SHARE);
  write_file(out, "repaired_present.bin", s.present, (size_t)w * w);
  double m0, m1;
  min_med(t, reps, &m0, &m1);
  printf("{\"rc\": %d, \"axis\": %d, \"index\": %d, \"repair_ms\": [%.3f, %.3f], \"reps\": %d, \"encodes\": %ld, "
         "\"decodes\": %ld, \"roots\": %ld}\n",
         rc, ba, bi, 1e3 * m0, 1e3 * m1, reps, calls[0], calls[1], calls[2]);
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: see the header of rsmt2d_axes.c\n");
    return 2;
  }
  load_backend(argv[1], argv[2]);
  const char* mode = argv[3];
  const int k = atoi(argv[4]);
  if (k < 1 || k > 512) return 2;
  size_t n = 0;
  if (!strcmp(mode, "single") && argc == 7) {
    const uint8_t* ods = read_all(argv[6], &n);
    if (n < (size_t)k * k * SHARE) return 2;
    mode_single(k, atoi(argv[5]), ods);
  } else if (!strcmp(mode, "extend") && argc == 9) {
    const uint8_t* ods = read_all(argv[7], &n);
    if (n != (size_t)k * k * SHARE) return 2;
    mode_extend(k, atoi(argv[5]), atoi(argv[6]), ods, argv[8]);
  } else if (!strcmp(mode, "repair") && argc == 11) {
    size_t ne, np, nr;
    const uint8_t* eds = read_all(argv[7], &ne);
    const uint8_t* pres = read_all(argv[8], &np);
    const uint8_t* roots = read_all(argv[9], &nr);
    const size_t w = 2 * (size_t)k;
    if (ne != w * w * SHARE || np != w * w || nr != 2 * w * NODE) return 2;
    mode_repair(k, atoi(argv[5]), atoi(argv[6]), eds, pres, roots, argv[10]);
  } else {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  if (use_cda) p_cda_free(g_ctx);
  /* The host-ASan build leaves without the exit-time destructors of the HIP runtime (the ASan runtime's own checks
     fire inside them, after every libcda call has returned; tests/abi_client/abi_host_client.c does the same).  The
     plain build exits normally, so that a profiler's exit-time output (rocprofv3) is written. */
  fflush(stdout);
  fflush(stderr);
#if defined(__has_feature)
#if __has_feature(address_sanitizer)
  _exit(0);
#endif
#endif
  return 0;
}
