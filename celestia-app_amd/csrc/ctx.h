// ctx.h — libcda host context and helpers shared by engine.cpp (block path,
// codec, repair) and inclusion.cpp (blob commitments, node export, proofs).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cda_internal.h"

namespace cda {
struct AxisQueue;  // axisq.cpp
struct Stager;     // staging.cpp
struct Consensus;  // consensus.cpp
}

struct cda_ctx {
  int device = 0;
  // the CPUs of the GPU's NUMA node that this process may run on (sysfs local_cpulist of its PCI function
  // intersected with the affinity at cda_init); libcda's copy helper threads run there, so the pinned staging
  // rings they allocate and fill sit next to the GPU.  Empty: no binding (CDA_NUMA_BIND=0, or unknown).
  std::vector<int> local_cpus;
  std::recursive_mutex mu;
  hipStream_t stream = nullptr;
  // CDA_REPAIR_OVERLAP=0: repair verifies each batch on the decode stream instead of a second stream
  bool repair_overlap = true;
  // CDA_REPAIR_FUSED=0: verify with the generic leaf + per-level launches instead of one fused launch
  bool repair_fused_verify = true;
  // CDA_REPAIR_EARLY=0: repair copies the square back only at the end (no early row return)
  bool repair_early = true;
  // HIP maps streams round-robin onto GPU_MAX_HW_QUEUES (4) hardware queues, so the streams that must run
  // concurrently are created first, together: stream, h2d_stream, d2h_stream, aux_stream.
  hipStream_t aux_stream = nullptr;
  // Workspace ordering across streams: the device-resident entry points enqueue on the caller's
  // stream but use this ctx's workspace (leaf/scratch records).  ws_event marks the end of the
  // last such enqueue; synchronous entry points make `stream` wait on it, and device entry points
  // wait on it and on `stream` (sync_ev), so no two uses of the workspace overlap.
  hipEvent_t ws_event = nullptr, sync_ev = nullptr;
  bool ws_pending = false;
  // host-buffer batch pipeline (host_pipeline.cpp): copy streams and per-slot events
  static constexpr int kSlots = 3;
  hipStream_t h2d_stream = nullptr, d2h_stream = nullptr;
  hipEvent_t ev_h2d[kSlots] = {}, ev_comp[kSlots] = {}, ev_d2h[kSlots] = {};
  // fork / join of repair's verification streams
  static constexpr int kJoin = 2;
  hipEvent_t fork_ev = nullptr, join_ev[kJoin] = {};
  std::string last_err;
  // workspace
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
  };
  Buf ods, eds, leaf, scratch, roots, dah, status, plan, payload;
  Buf done;  // per-block tree counters of the small-batch tree launch (trees_lds_kernel), kept at zero
  Buf nodes;  // node export (inclusion.cpp): the exported trees' per-tree node lists, packed on the device
  // one square split over devices (split.cpp): this device's slab, row / column slabs, leaf records, send blocks,
  // tree scratch, per-device results (meta) and, on the first device, the gathered results
  Buf sp_ods, sp_R, sp_LR, sp_S, sp_C, sp_LC, sp_scratch, sp_meta, sp_gather;
  hipEvent_t sp_ev[2] = {};  // replicas transport: sender-side "ready" events
  // repair: device root table + per-sweep descriptors, and their pinned host staging
  Buf rdesc, rstage;
  // repair: the present cells of a sparse caller square packed (upload) and their run table
  Buf rcompact, rruns;
  // pinned staging rings for cda_repair's large copies of caller (pageable) memory, one per direction
  // (staging.cpp); CDA_STAGING: bit 0 stages uploads, bit 1 downloads (0 = plain hipMemcpyAsync)
  cda::Stager* st_in = nullptr;
  cda::Stager* st_out = nullptr;
  int staging = 3;
  // the one-block host-buffer path (consensus.cpp): copy-thread pool, pinned slabs, events.  CDA_CONSENSUS=0 sends
  // one-block calls down the serial form instead (A/B runs)
  cda::Consensus* cons = nullptr;
  bool consensus = true;
  // A/B forms of the one-block path, read ONCE at cda_init (never per call: glibc getenv is not safe against a Go
  // runtime's concurrent setenv, and the environment must not steer a running node's path).  cons_in: 0 = default,
  // 1 = four input bands, 2 = one copy (CDA_CONS_IN); cons_out: 2 = the resident-buffer form on any pageable output
  // (CDA_CONS_OUT); cons_stg_mib: MiB of the bottom half staged through the pinned slab, -1 = default (CDA_CONS_STG);
  // cons_trace: phase timestamps to stderr (CDA_CONS_TRACE); copy_threads: pool size (CDA_COPY_THREADS).
  int cons_in = 0, cons_out = 0, cons_stg_mib = -1, copy_threads = 7;
  bool cons_trace = false;
  // Transparent huge pages for a fresh (never-touched) caller output buffer: madvise(MADV_HUGEPAGE) on its 2 MiB-aligned
  // interior before the copy pool touches it.  OFF by default: the hint changes the page policy of memory
  // the library does not own -- under cgo, Go heap.  Opt in per context with cda_set_option(CDA_OPT_HUGE_PAGES, 1) or
  // CDA_HUGE_PAGES=1 at cda_init.  A caller that recycles pinned buffers (go/cda's EDS pool) never takes this path.
  bool huge_pages = false;
  // the per-axis seams (axisq.cpp): queue of concurrent Encode / Decode / Root calls, its batch slots
  cda::AxisQueue* axq = nullptr;
  // profiling
  bool prof = false;
  struct Pending {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;
  std::map<std::string, std::pair<double, long long>> prof_acc;
};

namespace cda {

// Largest ODS width on the device block path: FF16 codewords up to m = 2048 in
// LDS, DAH tree of 4k roots in one workgroup's LDS (k <= 512).
constexpr uint32_t kMaxDeviceK = 512;
// batches of at most this many trees (B x 2w) take the one-launch LDS tree path (enqueue_trees; CDA_TREES_LDS)
constexpr int kLdsTreesMax = 512;

bool dev_ok(cda_ctx* c, hipError_t e, const char* what);
int ensure(cda_ctx* c, cda_ctx::Buf& b, size_t bytes);
void flush_profile(cda_ctx* c);
int ilog2i(uint32_t v);
bool is_pow2(uint64_t v);
void set_err(cda_err_info* e, int code, int axis, int index, int leaf, int block);
// 96-B records -> packed 90-B nodes
void pack_roots(const uint8_t* recs, uint32_t n, uint8_t* out);
// device status word -> CDA_OK / CDA_E_NS_ORDER (+ err detail)
int map_status(uint64_t st, int block, cda_err_info* err);
// whole block pipeline of nblocks device-resident blocks on stream s (engine.cpp)
int enqueue_pipeline(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* d_ods, uint8_t* d_eds, void* d_roots,
                     void* d_dah, unsigned long long* d_status, hipStream_t s);
// host-buffer batch as an H2D / compute / D2H pipeline (host_pipeline.cpp); caller holds the lock
int batch_pipelined(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* ods, uint8_t* eds_or_null,
                    uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, cda_err_info* err, int block0);
int ensure_pipeline(cda_ctx* c);  // copy streams + per-slot events (host_pipeline.cpp)
void free_pipeline(cda_ctx* c);
// Caller-memory copies (staging.cpp): large pageable buffers through the pinned rings, pinned / small ones
// directly.  staged_h2d returns once the source may be released (DMA enqueued on s); staged_d2h once the
// bytes are in h_dst (it waits for s).
int staged_h2d(cda_ctx* c, void* d_dst, const void* h_src, size_t n, hipStream_t s);
int staged_d2h(cda_ctx* c, void* h_dst, const void* d_src, size_t n, hipStream_t s);
// all of [p, p + n) inside one page-locked range (staging.cpp); its device address (or nullptr)
bool pinned_range(const void* p, size_t n);
const void* pinned_device_alias(const void* p, size_t n);
void free_staging(cda_ctx* c);
// byte range [off, off + len) of a host buffer
struct HostRun {
  size_t off, len;
};
// the runs of h_base, concatenated, to d_dst (through the pinned ring; no pinned fast path)
int staged_h2d_runs(cda_ctx* c, void* d_dst, const uint8_t* h_base, const HostRun* runs, size_t nruns,
                    hipStream_t s);
void bind_helper_thread(const cda_ctx* c);  // the calling helper thread -> c->local_cpus (no-op if empty)
void find_local_cpus(cda_ctx* c);
// one block through host buffers, overlapped with pinned staging and a copy pool (consensus.cpp; lock held)
bool consensus_eligible(const cda_ctx* c, uint32_t k);
// ods_pitch: bytes between ODS rows (0 = k * 512, contiguous); ods == eds_or_null with pitch 2k * 512 is the in-place
// form (cda_extend_commit_eds: the caller's EDS buffer holds the ODS in Q0)
int extend_one_host(cda_ctx* c, uint32_t k, const uint8_t* ods, uint8_t* eds_or_null, uint8_t* row_roots,
                    uint8_t* col_roots, uint8_t* dah, cda_err_info* err, size_t ods_pitch = 0);
void free_consensus(cda_ctx* c);
void free_axisq(cda_ctx* c);  // axisq.cpp: the per-axis queue's staging and streams
// RS jobs of the block path: rows (ODS row r -> Q0 copy + Q1 row r) and columns (top half -> bottom half)
RsJob rows_job(uint32_t k, uint32_t nblocks, const uint8_t* d_ods, uint8_t* d_eds);
RsJob cols_job(uint32_t k, uint32_t nblocks, uint8_t* d_eds);
// commitment phase (leaf hashing, NMT levels, DAH) of nblocks extended blocks in d_eds on stream s; the order-status
// words are set to "no error" first unless the caller already did (init_status = false)
int enqueue_commit(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* d_eds, void* d_roots, void* d_dah,
                   unsigned long long* d_status, hipStream_t s, size_t rec_off, bool init_status = true);
// grow the tree phase's counters / digest scratch for (k, nblocks) before its launch (engine.cpp)
int prepare_trees(cda_ctx* c, uint32_t k, uint32_t nblocks, hipStream_t s);
// RS phase of the block pipeline: rows (Q0 copy + Q1) then columns (Q2|Q3) of nblocks blocks.
int enqueue_rs(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* d_ods, uint8_t* d_eds, hipStream_t s);
// split_kernels.hip
int launch_region_leaf(const uint8_t* d_cells, long long cell_pitch, int r0, int c0, int nr, int nc, int k,
                       void* d_recs, long long rec_pitch, unsigned long long* d_status, bool row_order, hipStream_t s);
int launch_records_col_order(const void* d_recs, long long rec_pitch, int nr, int c0, int nc, int k,
                             unsigned long long* d_status, hipStream_t s);
void free_split_comm(cda_multi* m);  // split.cpp
int launch_tree_roots(const TreeSpec* spec, int nsets, int log2n, hipStream_t s);

// ---- exception barrier of the C ABI ----
// No C++ exception may cross an extern "C" entry point: under cgo it reaches std::terminate inside the Go node,
// where neither ProcessProposal's recover() (app/process_proposal.go:28-34) nor any caller can handle it.  Every
// entry point wraps its body in CDA_API_TRY / CDA_API_CATCH(ctx): std::bad_alloc -> CDA_E_NOMEM, anything else
// (std::system_error from a thread start, ...) -> CDA_E_INTERNAL, with what() in cda_last_device_error.
int api_exception(cda_ctx* c) noexcept;  // call from a catch block: classifies the exception in flight
// Failure injection, TEST BUILDS ONLY (-DCDA_TEST_HOOKS=1: `make hooks` -> cda/libcda_hooks.so, loaded by the fault
// tests through CDA_LIB): CDA_FAULT_INJECT=<site> throws at that site -- "entry" (every entry point, before its
// body), "alloc" (device workspace growth, as std::bad_alloc), "thread" (a helper-thread start, as
// std::system_error).  In a release library fault_point is an empty inline function: no environment variable can
// make a release build fail; cda_build_info() names a hooks build.
#if CDA_TEST_HOOKS
void fault_point(const char* site);
#else
inline void fault_point(const char*) {}
#endif
#define CDA_API_TRY try { ::cda::fault_point("entry");
#define CDA_API_CATCH(ctx) \
  }                        \
  catch (...) { return ::cda::api_exception(ctx); }

// Joins helper threads on every exit path (an exception between two thread starts would otherwise destroy a
// joinable std::thread, i.e. std::terminate); `stop` runs first so that blocked helpers can leave.
template <class Stop>
struct ThreadJoiner {
  std::vector<std::thread*> ts;
  Stop stop;
  explicit ThreadJoiner(Stop s) : stop(s) {}
  ~ThreadJoiner() {
    bool any = false;
    for (auto* t : ts) any = any || t->joinable();
    if (!any) return;
    stop();
    for (auto* t : ts)
      if (t->joinable()) t->join();
  }
};

// One handle over several contexts (host_pipeline.cpp: block batches; split.cpp: one square split over them).
struct SplitComm;  // split.cpp: RCCL communicators of the handle

// Synchronous entry points (work on c->stream): ordered after any device-resident enqueue.
struct Lock {
  cda_ctx* c;
  std::lock_guard<std::recursive_mutex> g;
  explicit Lock(cda_ctx* x) : c(x), g(x->mu) {
    (void)hipSetDevice(x->device);
    if (x->ws_pending) {
      (void)hipStreamWaitEvent(x->stream, x->ws_event, 0);
      x->ws_pending = false;
    }
  }
};

// Device-resident entry points enqueueing on the caller's stream `s`: ordered after the previous
// users of the workspace (device enqueues on other streams, synchronous calls on c->stream), and
// marking their own end for the next user.
struct DevLock {
  cda_ctx* c;
  hipStream_t s;
  std::lock_guard<std::recursive_mutex> g;
  DevLock(cda_ctx* x, hipStream_t st) : c(x), s(st), g(x->mu) {
    (void)hipSetDevice(x->device);
    (void)hipEventRecord(x->sync_ev, x->stream);
    (void)hipStreamWaitEvent(s, x->sync_ev, 0);
    if (x->ws_pending) (void)hipStreamWaitEvent(s, x->ws_event, 0);
  }
  ~DevLock() {
    (void)hipEventRecord(c->ws_event, s);
    c->ws_pending = true;
  }
};

}  // namespace cda

struct cda_multi {
  std::vector<cda_ctx*> ctx;
  std::vector<int> devices;
  bool replicas = false;              // every context on one device (cda_multi_init_replicas): split exchanges are
                                      // device copies instead of RCCL (tests, rehearsal of G > 1 on one GPU)
  std::mutex split_mu;                // one split at a time per handle
  cda::SplitComm* comm = nullptr;     // RCCL communicators (created by the first split with G > 1)
  uint8_t* pin_res = nullptr;         // pinned: a split's roots, DAH and status words (one D2H per call)
  size_t pin_cap = 0;
};
