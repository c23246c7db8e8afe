// engine.cpp — host side of libcda: context, device workspace, launch
// orchestration and the C ABI declared in include/cda.h.
//
// The block pipeline (da.ExtendShares + da.NewDataAvailabilityHeader,
// pkg/da/data_availability_header.go:44-75) on one HIP stream:
//   1. rs_encode8  rows     : ODS row r -> EDS Q0 copy + Q1 row r          (k codewords / block)
//   2. rs_encode8  columns  : EDS column c of [Q0|Q1] -> [Q2|Q3] column c  (2k codewords / block)
//      (Q3 = Enc(Q2 rows) in rsmt2d; by linearity Enc_col(Q1) is the same bytes)
//   3. leaf_hash            : every EDS cell once -> 96-B leaf records + namespace-order status
//   4. nmt_levels           : row and column trees of every block, 2 (or 3) levels per launch
//   5. dah                  : RFC-6962 over row roots ‖ col roots
// rsmt2d Repair lives in repair.cpp, the host-buffer batch pipeline in host_pipeline.cpp.
// Nothing here computes on the CPU: the host only validates arguments, moves
// buffers and maps device status words to error codes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "ctx.h"


namespace cda {

ProfScope::ProfScope(void* c, const char* n, hipStream_t s) : ctx(c), name(n), stream(s), a(nullptr), b(nullptr) {
  cda_ctx* x = static_cast<cda_ctx*>(ctx);
  if (!x || !x->prof) return;
  auto get = [&]() {
    hipEvent_t e;
    if (!x->event_pool.empty()) {
      e = x->event_pool.back();
      x->event_pool.pop_back();
    } else {
      (void)hipEventCreate(&e);
    }
    return e;
  };
  a = get();
  b = get();
  (void)hipEventRecord(a, stream);
}

ProfScope::~ProfScope() {
  cda_ctx* x = static_cast<cda_ctx*>(ctx);
  if (!x || !x->prof || !a) return;
  (void)hipEventRecord(b, stream);
  x->pending.push_back({name, a, b});
}

}  // namespace cda

using namespace cda;

namespace cda {

bool dev_ok(cda_ctx* c, hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  c->last_err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

int api_exception(cda_ctx* c) noexcept {
  int code = CDA_E_INTERNAL;
  const char* what = "unknown exception";
  try {
    throw;
  } catch (const std::bad_alloc&) {
    code = CDA_E_NOMEM;
    what = "out of host memory (std::bad_alloc)";
  } catch (const std::exception& ex) {
    what = ex.what();
  } catch (...) {
  }
  if (c) {
    try {
      c->last_err = what;
    } catch (...) {
    }
  }
  return code;
}

#if CDA_TEST_HOOKS
void fault_point(const char* site) {
  const char* e = getenv("CDA_FAULT_INJECT");
  if (!e || strcmp(e, site) != 0) return;
  if (strcmp(site, "thread") == 0)
    throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again), "injected thread failure");
  throw std::bad_alloc();
}
#endif

int ensure(cda_ctx* c, cda_ctx::Buf& b, size_t bytes) {
  if (b.cap >= bytes) return CDA_OK;
  fault_point("alloc");
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  if (!dev_ok(c, hipMalloc(&b.p, bytes ? bytes : 16), "hipMalloc")) return CDA_E_DEVICE;
  b.cap = bytes;
  return CDA_OK;
}

void flush_profile(cda_ctx* c) {
  for (auto& p : c->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      auto& acc = c->prof_acc[p.name];
      acc.first += ms;
      acc.second += 1;
    }
    c->event_pool.push_back(p.a);
    c->event_pool.push_back(p.b);
  }
  c->pending.clear();
}

void* bufs0(cda_ctx* c, size_t rec_off) { return (uint8_t*)c->leaf.p + rec_off * CDA_REC_BYTES; }

int ilog2i(uint32_t v) {
  int l = 0;
  while ((1u << l) < v) l++;
  return l;
}
bool is_pow2(uint64_t v) { return v && !(v & (v - 1)); }


void set_err(cda_err_info* e, int code, int axis, int index, int leaf, int block) {
  if (!e) return;
  e->code = code;
  e->axis = axis;
  e->index = index;
  e->leaf = leaf;
  e->block = block;
}

// Enqueue the whole block pipeline for blocks [0, nblocks) of the given buffers,
// using leaf/scratch records starting at record offset `rec_off`.
// RS phase: rows (Q0 copy + Q1) then columns (Q2|Q3) of nblocks blocks.
RsJob rows_job(uint32_t k, uint32_t nblocks, const uint8_t* d_ods, uint8_t* d_eds) {
  const uint32_t w = 2 * k;
  const long long S = CDA_SHARE;
  RsJob j{};
  j.src = d_ods;
  j.src_blk = (long long)k * k * S;
  j.src_cw = (long long)k * S;
  j.src_sh = S;
  j.dst = d_eds + (size_t)k * S;
  j.dst_blk = (long long)w * w * S;
  j.dst_cw = (long long)w * S;
  j.dst_sh = S;
  j.cpy = d_eds;
  j.cpy_blk = j.dst_blk;
  j.cpy_cw = j.dst_cw;
  j.cpy_sh = S;
  j.k = (int)k;
  j.cw_per_blk = (int)k;
  j.nblk = (int)nblocks;
  j.shard_len = CDA_SHARE;
  return j;
}

RsJob cols_job(uint32_t k, uint32_t nblocks, uint8_t* d_eds) {
  const uint32_t w = 2 * k;
  const long long S = CDA_SHARE;
  RsJob j{};
  j.src = d_eds;
  j.src_blk = (long long)w * w * S;
  j.src_cw = S;
  j.src_sh = (long long)w * S;
  j.dst = d_eds + (size_t)k * w * S;
  j.dst_blk = j.src_blk;
  j.dst_cw = S;
  j.dst_sh = (long long)w * S;
  j.cpy = nullptr;
  j.k = (int)k;
  j.cw_per_blk = (int)w;
  j.nblk = (int)nblocks;
  j.shard_len = CDA_SHARE;
  return j;
}

int enqueue_rs(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* d_ods, uint8_t* d_eds, hipStream_t s) {
  {
    const RsJob j = rows_job(k, nblocks, d_ods, d_eds);
    ProfScope ps(c, 2 * k <= 256 ? "rs_encode8_rows" : "rs_encode16_rows", s);
    const int lr = 2 * k <= 256 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  {
    const RsJob j = cols_job(k, nblocks, d_eds);
    ProfScope ps(c, 2 * k <= 256 ? "rs_encode8_cols" : "rs_encode16_cols", s);
    const int lr = 2 * k <= 256 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  return CDA_OK;
}

// Commitment phase: leaf hashing, NMT levels, DAH of nblocks extended blocks.
// NMT levels + DAH of nblocks blocks whose leaf records are at record offset rec_off.
// small batches (latency: the consensus path extends one block): all trees + the DAH in one LDS-resident launch
static bool lds_trees_path(uint32_t k, uint32_t nblocks) {
  static const int lds_trees = CDA_AB_ENV("CDA_TREES_LDS") ? atoi(CDA_AB_ENV("CDA_TREES_LDS")) : kLdsTreesMax;  // once
  return (size_t)nblocks * 4 * k <= (size_t)lds_trees && 2 * k <= 256;
}

// The tree phase's per-block counters (zeroed once; the kernels leave them at 0) and digest scratch, grown before
// any work that must not be interrupted is started (the one-block path's copy pool, consensus.cpp).
int prepare_trees(cda_ctx* c, uint32_t k, uint32_t nblocks, hipStream_t s) {
  if (!lds_trees_path(k, nblocks) && 2 * k < 1024) return CDA_OK;  // level kernels + dah_kernel: no scratch
  const size_t cnt_b = ((size_t)nblocks * 4 + 255) & ~(size_t)255, need = cnt_b + (size_t)nblocks * 4 * k * 32;
  if (c->done.cap >= need) return CDA_OK;
  int rc = ensure(c, c->done, std::max<size_t>(need, 64 * 1024));
  if (rc) return rc;
  return dev_ok(c, hipMemsetAsync(c->done.p, 0, c->done.cap, s), "hipMemsetAsync") ? CDA_OK : CDA_E_DEVICE;
}

int enqueue_trees(cda_ctx* c, uint32_t k, uint32_t nblocks, void* d_roots, void* d_dah, hipStream_t s, size_t rec_off) {
  const uint32_t w = 2 * k;
  if (lds_trees_path(k, nblocks)) {
    const size_t cnt_b = ((size_t)nblocks * 4 + 255) & ~(size_t)255;
    if (int rc = prepare_trees(c, k, nblocks, s)) return rc;
    ProfScope ps(c, "trees_lds", s);
    const int lr = launch_trees_lds((uint8_t*)c->leaf.p + rec_off * CDA_REC_BYTES, d_roots, d_dah,
                                    (unsigned*)c->done.p, (uint8_t*)c->done.p + cnt_b, (int)k, (int)nblocks, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
    return CDA_OK;
  }
  // inner levels in c->scratch: 2 records per leaf record of the chunk (2w x (w - 2) per block)
  const int lr0 = launch_nmt_trees((uint8_t*)c->leaf.p + rec_off * CDA_REC_BYTES,
                                   (uint8_t*)c->scratch.p + 2 * rec_off * CDA_REC_BYTES, d_roots, (int)k, (int)nblocks, s,
                                   c);
  if (lr0) return lr0 == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  if (w < 1024) {  // k <= 256: one workgroup per block (the wide form's agent-scope release of the digests cost
                   // more than its 4 -> 2 digest compressions saved: 0.077 -> 0.112 ms per B = 128 step at k = 128)
    ProfScope ps(c, "dah", s);
    const int lr = launch_dah(d_roots, d_dah, (int)(2 * w), (int)nblocks, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  } else {  // k = 512: 2,048 roots, 8 digest compressions per thread in one workgroup -> 2 over eight (0.147 ->
            // 0.112 ms per two squares)
    // per-block counters (zeroed once; the kernel leaves them at 0), then n digests of 32 B per block
    const size_t cnt_b = ((size_t)nblocks * 4 + 255) & ~(size_t)255;
    if (int rc = prepare_trees(c, k, nblocks, s)) return rc;
    ProfScope ps(c, "dah", s);
    const int lr = launch_dah_wide(d_roots, d_dah, (unsigned*)c->done.p, (uint8_t*)c->done.p + cnt_b, (int)(2 * w),
                                   (int)nblocks, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  return CDA_OK;
}

int enqueue_commit(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* d_eds, void* d_roots, void* d_dah,
                   unsigned long long* d_status, hipStream_t s, size_t rec_off, bool init_status) {
  if (init_status && !dev_ok(c, hipMemsetAsync(d_status, 0xFF, (size_t)nblocks * 8, s), "hipMemsetAsync"))
    return CDA_E_DEVICE;
  {
    ProfScope ps(c, "leaf_hash", s);
    if (launch_leaf_hash(d_eds, bufs0(c, rec_off), d_status, (int)k, (int)nblocks, s)) return CDA_E_DEVICE;
  }
  return enqueue_trees(c, k, nblocks, d_roots, d_dah, s, rec_off);
}

int enqueue_pipeline(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* d_ods, uint8_t* d_eds, void* d_roots,
                     void* d_dah, unsigned long long* d_status, hipStream_t s) {
  // One stream, one kernel per stage: each stage already fills the GPU.  Measured slower and removed
  // (DESIGN.md §4 "Scheduling experiments"): sub-streams over independent chunks, a two-stream RS/SHA
  // software pipeline, sequential Infinity-Cache-sized chunks, CU-masked streams, RS fused with leaf hashing.
  const uint32_t w = 2 * k;
  const size_t cells = (size_t)nblocks * w * w;
  int rc = ensure(c, c->leaf, cells * CDA_REC_BYTES);
  if (rc) return rc;
  rc = ensure(c, c->scratch, 2 * cells * CDA_REC_BYTES);  // inner tree levels
  if (rc) return rc;
  // the order-status words are set before the extension, so no fill sits between the column pass and the leaf
  // hashing on the dependent chain of a one-block call
  if (!dev_ok(c, hipMemsetAsync(d_status, 0xFF, (size_t)nblocks * 8, s), "hipMemsetAsync")) return CDA_E_DEVICE;
  if ((rc = enqueue_rs(c, k, nblocks, d_ods, d_eds, s))) return rc;
  return enqueue_commit(c, k, nblocks, d_eds, d_roots, d_dah, d_status, s, 0, false);
}

// 96-B records -> packed 90-B nodes
void pack_roots(const uint8_t* recs, uint32_t n, uint8_t* out) {
  for (uint32_t i = 0; i < n; i++) memcpy(out + (size_t)i * CDA_NODE_SIZE, recs + (size_t)i * CDA_REC_BYTES, CDA_NODE_SIZE);
}

int map_status(uint64_t st, int block, cda_err_info* err) {
  if (st == ~0ull) return CDA_OK;
  set_err(err, CDA_E_NS_ORDER, (int)(st >> 40), (int)((st >> 20) & 0xFFFFF), (int)(st & 0xFFFFF), block);
  return CDA_E_NS_ORDER;
}


}  // namespace cda

extern "C" {

int cda_init(int device, cda_ctx** out) {
  CDA_API_TRY
  if (!out) return CDA_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return CDA_E_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return CDA_E_DEVICE;
  cda_ctx* c = new cda_ctx();
  struct Owner {  // releases a half-built context on every failure path (including an exception)
    cda_ctx* c;
    ~Owner() {
      if (c) cda_free(c);
    }
  } own{c};
  c->device = device;
  const char* fail = nullptr;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) fail = "stream";
  else if (rs_init_device_tables(device)) fail = "rs8 tables";
  else if (rs16_init_device_tables(device)) fail = "rs16 tables";
  else if (rs_decode_init_device_tables(device)) fail = "decode tables";
  if (fail) {
    fprintf(stderr, "cda_init: %s initialisation failed: %s\n", fail, hipGetErrorString(hipGetLastError()));
    return CDA_E_DEVICE;
  }
  if (const char* e = CDA_AB_ENV("CDA_REPAIR_OVERLAP")) c->repair_overlap = atoi(e) != 0;
  if (const char* e = CDA_AB_ENV("CDA_REPAIR_FUSED")) c->repair_fused_verify = atoi(e) != 0;
  if (const char* e = CDA_AB_ENV("CDA_REPAIR_EARLY")) c->repair_early = atoi(e) != 0;
  if (const char* e = CDA_AB_ENV("CDA_STAGING")) c->staging = atoi(e) & 3;
  if (const char* e = CDA_AB_ENV("CDA_CONSENSUS")) c->consensus = atoi(e) != 0;
  // the one-block path's A/B forms and the huge-page opt-in (test builds only, CDA_AB_ENV): read here once, never per
  // call (ctx.h); CDA_COPY_THREADS is a deployment option of every build
  if (const char* e = CDA_AB_ENV("CDA_CONS_IN")) c->cons_in = std::max(0, std::min(2, atoi(e)));
  if (const char* e = CDA_AB_ENV("CDA_CONS_OUT")) c->cons_out = atoi(e) == 2 ? 2 : 0;
  if (const char* e = CDA_AB_ENV("CDA_CONS_STG")) c->cons_stg_mib = std::max(0, atoi(e));
  if (const char* e = getenv("CDA_COPY_THREADS")) c->copy_threads = std::max(1, std::min(64, atoi(e)));
  if (const char* e = CDA_AB_ENV("CDA_HUGE_PAGES")) c->huge_pages = atoi(e) != 0;
  c->cons_trace = CDA_AB_ENV("CDA_CONS_TRACE") != nullptr;
  find_local_cpus(c);
  // the streams that overlap each other, created right after `stream` so that they land on distinct hardware
  // queues (HIP assigns streams to its GPU_MAX_HW_QUEUES = 4 queues round-robin)
  bool ok = ensure_pipeline(c) == CDA_OK &&
            hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ws_event, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->sync_ev, hipEventDisableTiming) == hipSuccess;
  for (int i = 0; i < cda_ctx::kJoin && ok; i++)
    ok = hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming) == hipSuccess;
  if (!ok) return CDA_E_DEVICE;
  own.c = nullptr;
  *out = c;
  return CDA_OK;
  CDA_API_CATCH(nullptr)
}

void cda_free(cda_ctx* c) {
  if (!c) return;
  try {
    Lock l(c);
    (void)hipStreamSynchronize(c->stream);
    flush_profile(c);
    for (auto* b : {&c->ods, &c->eds, &c->leaf, &c->scratch, &c->roots, &c->dah, &c->status, &c->plan, &c->payload,
                    &c->rdesc, &c->rcompact, &c->rruns, &c->done, &c->nodes, &c->sp_ods, &c->sp_R, &c->sp_LR, &c->sp_S, &c->sp_C, &c->sp_LC, &c->sp_scratch,
                    &c->sp_meta, &c->sp_gather})
      if (b->p) (void)hipFree(b->p);
    for (auto e : c->sp_ev)
      if (e) (void)hipEventDestroy(e);
    if (c->rstage.p) (void)hipHostFree(c->rstage.p);
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < cda_ctx::kJoin; i++)
      if (c->join_ev[i]) (void)hipEventDestroy(c->join_ev[i]);
    free_consensus(c);  // joins its copy threads first
    free_axisq(c);
    free_pipeline(c);
    free_staging(c);
    if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->ws_event) (void)hipEventDestroy(c->ws_event);
    if (c->sync_ev) (void)hipEventDestroy(c->sync_ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  } catch (...) {  // nothing may escape the C ABI; the context is released regardless
  }
  delete c;
}

const char* cda_strerror(int code) {
  switch (code) {
    case CDA_OK: return "ok";
    case CDA_E_NOT_POW2: return "number of shares is not a power of 2";
    case CDA_E_NOT_SQUARE: return "number of chunks must be a square number";
    case CDA_E_SHARD_SIZE: return "chunk size must be a multiple of 64 bytes";
    case CDA_E_NS_SHORT: return "data is too short to contain namespace ID";
    case CDA_E_NS_ORDER: return "pushed data has smaller namespace than previous (invalid push order)";
    case CDA_E_TOO_FEW: return "too few shards given";
    case CDA_E_UNREPAIRABLE: return "failed to solve data square";
    case CDA_E_BYZANTINE: return "byzantine data";
    case CDA_E_ARG: return "invalid argument";
    case CDA_E_DEVICE: return "device error";
    case CDA_E_PUSH_PAST: return "pushed past predetermined square size";
    case CDA_E_UNSUPPORTED: return "unsupported configuration";
    case CDA_E_SHARE_VERSION: return "unsupported share version";
    case CDA_E_BLOB_SIZE: return "cannot use zero blob size";
    case CDA_E_NOMEM: return "out of host memory";
    case CDA_E_INTERNAL: return "internal error (exception caught at the C ABI)";
    default: return "unknown error";
  }
}

const char* cda_last_device_error(cda_ctx* c) { return c ? c->last_err.c_str() : ""; }

const char* cda_build_info(void) {
  static const std::string info = [] {
    std::string d;
    for (const char* t : {rs8_diag_tag(), rs16_diag_tag(), CDA_TEST_HOOKS ? "test_hooks" : ""})
      if (*t) d += (d.empty() ? "" : ",") + std::string(t);
    // a release library reads only the deployment options named here (cda_internal.h CDA_AB_ENV)
    return d.empty() ? std::string("release gfx950; env: CDA_NUMA_BIND, CDA_COPY_THREADS") : "diagnostic gfx950 " + d;
  }();
  return info.c_str();
}

int cda_set_option(cda_ctx* c, int option, int64_t value) {
  CDA_API_TRY
  if (!c) return CDA_E_ARG;
  Lock l(c);
  switch (option) {
    case CDA_OPT_HUGE_PAGES: c->huge_pages = value != 0; return CDA_OK;
    default: return CDA_E_ARG;
  }
  CDA_API_CATCH(c)
}

int64_t cda_rs_max_chunks(void) { return (int64_t)32768 * 32768; }
const char* cda_rs_name(void) { return "Leopard"; }
int cda_rs_validate_chunk_size(int64_t chunk_size) {
  return (chunk_size > 0 && chunk_size % 64 == 0) ? CDA_OK : CDA_E_SHARD_SIZE;
}

// cda_rs_encode, cda_rs_decode, cda_nmt_axis_root: the per-axis seams, axisq.cpp

int cda_extend_commit_device(cda_ctx* c, uint32_t k, uint32_t nblocks, const void* d_ods, void* d_eds, void* d_roots,
                             void* d_dah, void* d_status, void* stream) {
  CDA_API_TRY
  if (!c || !d_ods || !d_eds || !d_roots || !d_dah || !d_status || nblocks == 0) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  hipStream_t s = stream ? (hipStream_t)stream : nullptr;
  DevLock l(c, s);
  return enqueue_pipeline(c, k, nblocks, (const uint8_t*)d_ods, (uint8_t*)d_eds, d_roots, d_dah,
                          (unsigned long long*)d_status, s);
  CDA_API_CATCH(c)
}

int cda_rs_encode_device(cda_ctx* c, uint32_t k, uint32_t shard_len, uint32_t ncw, const void* d_src, int64_t src_cw,
                         int64_t src_sh, void* d_dst, int64_t dst_cw, int64_t dst_sh, void* stream) {
  CDA_API_TRY
  if (!c || !d_src || !d_dst || k == 0 || k > 32768) return CDA_E_ARG;
  if (cda_rs_validate_chunk_size(shard_len)) return CDA_E_SHARD_SIZE;
  if (ncw == 0) return CDA_OK;
  hipStream_t s = stream ? (hipStream_t)stream : nullptr;
  DevLock l(c, s);
  RsJob j{};
  j.src = (const uint8_t*)d_src;
  j.src_cw = src_cw;
  j.src_sh = src_sh;
  j.dst = (uint8_t*)d_dst;
  j.dst_cw = dst_cw;
  j.dst_sh = dst_sh;
  j.k = (int)k;
  j.cw_per_blk = (int)ncw;
  j.nblk = 1;
  j.shard_len = (int)shard_len;
  ProfScope ps(c, 2 * k <= 256 ? "rs_encode8" : "rs_encode16", s);
  const int lr = 2 * k <= 256 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s);
  if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_nmt_roots_device(cda_ctx* c, uint32_t k, const void* d_eds, uint32_t axis, uint32_t first_index,
                         uint32_t naxes, uint32_t leaf_off, uint32_t nleaves, void* d_roots, void* d_status,
                         void* stream) {
  CDA_API_TRY
  if (!c || !d_eds || !d_roots || !d_status || (axis != CDA_AXIS_ROW && axis != CDA_AXIS_COL)) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  const uint32_t w = 2 * k;
  if (k > kMaxDeviceK || first_index + naxes > w || !is_pow2(nleaves) || leaf_off % nleaves || leaf_off + nleaves > w)
    return CDA_E_ARG;
  if (naxes == 0) return CDA_OK;
  hipStream_t s = stream ? (hipStream_t)stream : nullptr;
  DevLock l(c, s);
  const size_t recs = (size_t)naxes * nleaves * CDA_REC_BYTES;
  int rc;
  if ((rc = ensure(c, c->leaf, recs)) || (rc = ensure(c, c->scratch, recs))) return rc;
  if (!dev_ok(c, hipMemsetAsync(d_status, 0xFF, (size_t)naxes * 8, s), "hipMemsetAsync")) return CDA_E_DEVICE;
  ProfScope ps(c, "nmt_roots", s);
  const int lr = launch_axes_roots((const uint8_t*)d_eds, (int)k, nullptr, (int)((axis << 24) | first_index),
                                   (int)naxes, (int)leaf_off, (int)nleaves, c->leaf.p, c->scratch.p, d_roots,
                                   (unsigned long long*)d_status, s);
  if (lr) return lr == -2 ? CDA_E_ARG : CDA_E_DEVICE;
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_nmt_fold_device(cda_ctx* c, uint32_t ntrees, uint32_t n, const void* d_nodes, void* d_roots, void* stream) {
  CDA_API_TRY
  if (!c || !d_nodes || !d_roots || !is_pow2(n)) return CDA_E_ARG;
  if (ntrees == 0) return CDA_OK;
  hipStream_t s = stream ? (hipStream_t)stream : nullptr;
  DevLock l(c, s);
  const size_t bytes = (size_t)ntrees * n * CDA_REC_BYTES;
  if (n == 1) return dev_ok(c, hipMemcpyAsync(d_roots, d_nodes, bytes, hipMemcpyDeviceToDevice, s), "D2D") ? CDA_OK
                                                                                                          : CDA_E_DEVICE;
  int rc;
  if ((rc = ensure(c, c->leaf, bytes)) || (rc = ensure(c, c->scratch, bytes))) return rc;
  if (!dev_ok(c, hipMemcpyAsync(c->leaf.p, d_nodes, bytes, hipMemcpyDeviceToDevice, s), "D2D")) return CDA_E_DEVICE;
  ProfScope ps(c, "nmt_fold", s);
  return launch_nmt_fold(c->leaf.p, c->scratch.p, d_roots, (int)ntrees, ilog2i(n), s) ? CDA_E_DEVICE : CDA_OK;
  CDA_API_CATCH(c)
}

int cda_dah_device(cda_ctx* c, uint32_t n_total, const void* d_roots, void* d_dah, void* stream) {
  CDA_API_TRY
  if (!c || !d_roots || !d_dah || n_total == 0) return CDA_E_ARG;
  hipStream_t s = stream ? (hipStream_t)stream : nullptr;
  DevLock l(c, s);
  ProfScope ps(c, "dah", s);
  const int lr = launch_dah(d_roots, d_dah, (int)n_total, 1, s);
  if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_extend_commit_batch(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* ods, uint8_t* eds_or_null,
                            uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !ods || !row_roots || !col_roots || !dah || nblocks == 0) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  Lock l(c);
  if (nblocks > 1 && !c->prof) return batch_pipelined(c, k, nblocks, ods, eds_or_null, row_roots, col_roots, dah, err, 0);
  // one block: the consensus path's call (PrepareProposal / ProcessProposal), copies overlapped with the device work
  if (nblocks == 1 && consensus_eligible(c, k)) return extend_one_host(c, k, ods, eds_or_null, row_roots, col_roots, dah, err);
  // profiling (kernels must not overlap the event brackets) or k = 512: serial on c->stream
  const uint32_t w = 2 * k;
  const size_t ods_b = (size_t)nblocks * k * k * CDA_SHARE, eds_b = (size_t)nblocks * w * w * CDA_SHARE;
  const size_t roots_b = (size_t)nblocks * 2 * w * CDA_REC_BYTES;
  int rc;
  if ((rc = ensure(c, c->ods, ods_b)) || (rc = ensure(c, c->eds, eds_b)) || (rc = ensure(c, c->roots, roots_b)) ||
      (rc = ensure(c, c->dah, (size_t)nblocks * 32)) || (rc = ensure(c, c->status, (size_t)nblocks * 8)))
    return rc;
  if (!dev_ok(c, hipMemcpyAsync(c->ods.p, ods, ods_b, hipMemcpyHostToDevice, c->stream), "H2D")) return CDA_E_DEVICE;
  // With the EDS wanted (da.ExtendShares returns it): the EDS is final once the extension has run, so its copy-out
  // runs on the D2H stream beside the tree hashing instead of after it.  The hashing is enqueued first: the
  // pageable copy holds this thread until it is done.
  const bool overlap = eds_or_null && !c->prof;
  if (overlap) {
    const size_t cells = (size_t)nblocks * w * w;
    if ((rc = ensure_pipeline(c)) || (rc = ensure(c, c->leaf, cells * CDA_REC_BYTES)) ||
        (rc = ensure(c, c->scratch, 2 * cells * CDA_REC_BYTES)) ||
        (rc = enqueue_rs(c, k, nblocks, (const uint8_t*)c->ods.p, (uint8_t*)c->eds.p, c->stream)))
      return rc;
    if (!dev_ok(c, hipEventRecord(c->ev_comp[0], c->stream), "hipEventRecord")) return CDA_E_DEVICE;
    if ((rc = enqueue_commit(c, k, nblocks, (const uint8_t*)c->eds.p, c->roots.p, c->dah.p,
                             (unsigned long long*)c->status.p, c->stream, 0)))
      return rc;
    if (!dev_ok(c, hipStreamWaitEvent(c->d2h_stream, c->ev_comp[0], 0), "hipStreamWaitEvent") ||
        !dev_ok(c, hipMemcpyAsync(eds_or_null, c->eds.p, eds_b, hipMemcpyDeviceToHost, c->d2h_stream), "D2H") ||
        !dev_ok(c, hipStreamSynchronize(c->d2h_stream), "sync"))
      return CDA_E_DEVICE;
  } else {
    rc = enqueue_pipeline(c, k, nblocks, (const uint8_t*)c->ods.p, (uint8_t*)c->eds.p, c->roots.p, c->dah.p,
                          (unsigned long long*)c->status.p, c->stream);
    if (rc) return rc;
    if (eds_or_null &&
        !dev_ok(c, hipMemcpyAsync(eds_or_null, c->eds.p, eds_b, hipMemcpyDeviceToHost, c->stream), "D2H"))
      return CDA_E_DEVICE;
  }
  std::vector<uint8_t> recs(roots_b);
  std::vector<uint64_t> st(nblocks);
  if (!dev_ok(c, hipMemcpyAsync(recs.data(), c->roots.p, roots_b, hipMemcpyDeviceToHost, c->stream), "D2H") ||
      !dev_ok(c, hipMemcpyAsync(dah, c->dah.p, (size_t)nblocks * 32, hipMemcpyDeviceToHost, c->stream), "D2H") ||
      !dev_ok(c, hipMemcpyAsync(st.data(), c->status.p, (size_t)nblocks * 8, hipMemcpyDeviceToHost, c->stream), "D2H") ||
      !dev_ok(c, hipStreamSynchronize(c->stream), "sync"))
    return CDA_E_DEVICE;
  flush_profile(c);
  for (uint32_t b = 0; b < nblocks; b++) {
    const uint8_t* r = recs.data() + (size_t)b * 2 * w * CDA_REC_BYTES;
    pack_roots(r, w, row_roots + (size_t)b * w * CDA_NODE_SIZE);
    pack_roots(r + (size_t)w * CDA_REC_BYTES, w, col_roots + (size_t)b * w * CDA_NODE_SIZE);
  }
  for (uint32_t b = 0; b < nblocks; b++)
    if ((rc = map_status(st[b], (int)b, err))) return rc;
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_extend_commit(cda_ctx* c, uint32_t count, uint32_t share_len, const uint8_t* shares, uint8_t* eds_or_null,
                      uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !shares || !row_roots || !col_roots || !dah) return CDA_E_ARG;
  // da.ExtendShares: power-of-two check (data_availability_header.go:67-69)
  if (!is_pow2(count)) return set_err(err, CDA_E_NOT_POW2, -1, -1, -1, -1), CDA_E_NOT_POW2;
  // rsmt2d ComputeExtendedDataSquare: square count, chunk size
  const uint32_t k = (uint32_t)std::ceil(std::sqrt((double)count));
  if (k * k != count) return set_err(err, CDA_E_NOT_SQUARE, -1, -1, -1, -1), CDA_E_NOT_SQUARE;
  if (cda_rs_validate_chunk_size(share_len)) return CDA_E_SHARD_SIZE;
  if (share_len != CDA_SHARE) return CDA_E_UNSUPPORTED;
  return cda_extend_commit_batch(c, k, 1, shares, eds_or_null, row_roots, col_roots, dah, err);
  CDA_API_CATCH(c)
}

// In place: the ODS is Q0 of the caller's EDS buffer.  One block of k <= 256 takes the consensus path without its Q0
// copy (the input bands are 2-D DMAs from the caller's rows); anything else (k = 512, profiling, a context without the
// consensus path) gathers Q0 into a contiguous host copy and runs cda_extend_commit_batch, which writes Q0 back
// unchanged.
int cda_extend_commit_eds(cda_ctx* c, uint32_t k, uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                          cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !eds || !row_roots || !col_roots || !dah) return CDA_E_ARG;
  if (!is_pow2(k)) return set_err(err, CDA_E_NOT_POW2, -1, -1, -1, -1), CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  const size_t rowS = (size_t)k * CDA_SHARE, erowS = 2 * rowS;
  {
    Lock l(c);
    if (consensus_eligible(c, k)) return extend_one_host(c, k, eds, eds, row_roots, col_roots, dah, err, erowS);
  }
  std::vector<uint8_t> ods((size_t)k * rowS);
  for (uint32_t r = 0; r < k; r++) memcpy(ods.data() + r * rowS, eds + r * erowS, rowS);
  return cda_extend_commit_batch(c, k, 1, ods.data(), eds, row_roots, col_roots, dah, err);
  CDA_API_CATCH(c)
}

int cda_commit_eds(cda_ctx* c, uint32_t k, const uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                   cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !eds || !row_roots || !col_roots || !dah) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  Lock l(c);
  const uint32_t w = 2 * k;
  const size_t eds_b = (size_t)w * w * CDA_SHARE, roots_b = (size_t)2 * w * CDA_REC_BYTES;
  int rc;
  if ((rc = ensure(c, c->eds, eds_b)) || (rc = ensure(c, c->roots, roots_b)) || (rc = ensure(c, c->dah, 32)) ||
      (rc = ensure(c, c->status, 8)) || (rc = ensure(c, c->leaf, (size_t)w * w * CDA_REC_BYTES)) ||
      (rc = ensure(c, c->scratch, (size_t)2 * w * w * CDA_REC_BYTES)))
    return rc;
  hipStream_t s = c->stream;
  if (!dev_ok(c, hipMemcpyAsync(c->eds.p, eds, eds_b, hipMemcpyHostToDevice, s), "H2D") ||
      !dev_ok(c, hipMemsetAsync(c->status.p, 0xFF, 8, s), "memset"))
    return CDA_E_DEVICE;
  {
    ProfScope ps(c, "leaf_hash", s);
    if (launch_leaf_hash((const uint8_t*)c->eds.p, c->leaf.p, (unsigned long long*)c->status.p, (int)k, 1, s))
      return CDA_E_DEVICE;
  }
  // trees + DAH as the block path runs one block (the one-launch LDS tree kernel for k <= 128)
  if ((rc = enqueue_trees(c, k, 1, c->roots.p, c->dah.p, s, 0))) return rc;
  std::vector<uint8_t> recs(roots_b);
  uint64_t st = 0;
  if (!dev_ok(c, hipMemcpyAsync(recs.data(), c->roots.p, roots_b, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipMemcpyAsync(dah, c->dah.p, 32, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipMemcpyAsync(&st, c->status.p, 8, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipStreamSynchronize(s), "sync"))
    return CDA_E_DEVICE;
  flush_profile(c);
  pack_roots(recs.data(), w, row_roots);
  pack_roots(recs.data() + (size_t)w * CDA_REC_BYTES, w, col_roots);
  return map_status(st, 0, err);
  CDA_API_CATCH(c)
}

int cda_dah_hash(cda_ctx* c, uint32_t n, const uint8_t* row_roots, const uint8_t* col_roots, uint8_t* dah) {
  CDA_API_TRY
  if (!c || !dah) return CDA_E_ARG;
  if (n == 0) {  // merkle.HashFromByteSlices(nil) = SHA256("")
    static const uint8_t kEmpty[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                       0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                       0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};
    memcpy(dah, kEmpty, 32);
    return CDA_OK;
  }
  if (!row_roots || !col_roots) return CDA_E_ARG;
  Lock l(c);
  const size_t roots_b = (size_t)2 * n * CDA_REC_BYTES;
  int rc;
  if ((rc = ensure(c, c->roots, roots_b)) || (rc = ensure(c, c->dah, 32))) return rc;
  std::vector<uint8_t> recs(roots_b, 0);
  for (uint32_t i = 0; i < n; i++) {
    memcpy(recs.data() + (size_t)i * CDA_REC_BYTES, row_roots + (size_t)i * CDA_NODE_SIZE, CDA_NODE_SIZE);
    memcpy(recs.data() + (size_t)(n + i) * CDA_REC_BYTES, col_roots + (size_t)i * CDA_NODE_SIZE, CDA_NODE_SIZE);
  }
  hipStream_t s = c->stream;
  if (!dev_ok(c, hipMemcpyAsync(c->roots.p, recs.data(), roots_b, hipMemcpyHostToDevice, s), "H2D"))
    return CDA_E_DEVICE;
  {
    ProfScope ps(c, "dah", s);
    int lr = launch_dah(c->roots.p, c->dah.p, (int)(2 * n), 1, s);
    if (lr == -2) return CDA_E_UNSUPPORTED;
    if (lr) return CDA_E_DEVICE;
  }
  if (!dev_ok(c, hipMemcpyAsync(dah, c->dah.p, 32, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipStreamSynchronize(s), "sync"))
    return CDA_E_DEVICE;
  flush_profile(c);
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_profile_enable(cda_ctx* c, int enable) {
  CDA_API_TRY
  if (!c) return CDA_E_ARG;
  Lock l(c);
  c->prof = enable != 0;
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_profile_reset(cda_ctx* c) {
  CDA_API_TRY
  if (!c) return CDA_E_ARG;
  Lock l(c);
  flush_profile(c);
  c->prof_acc.clear();
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_profile_read(cda_ctx* c, char* names_buf, size_t names_cap, double* total_ms, int64_t* launches, int cap) {
  CDA_API_TRY
  if (!c) return CDA_E_ARG;
  Lock l(c);
  flush_profile(c);
  int i = 0;
  size_t off = 0;
  for (auto& kv : c->prof_acc) {
    if (i >= cap) break;
    const size_t len = kv.first.size() + 1;
    if (names_buf && off + len <= names_cap) {
      memcpy(names_buf + off, kv.first.c_str(), len);
      off += len;
    }
    if (total_ms) total_ms[i] = kv.second.first;
    if (launches) launches[i] = kv.second.second;
    i++;
  }
  return i;
  CDA_API_CATCH(c)
}

}  // extern "C"
