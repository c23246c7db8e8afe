// consensus.cpp — ONE block through host buffers, shaped for the consensus path.
//
// PrepareProposal and ProcessProposal extend one block per call (app/prepare_proposal.go:65-93,
// app/process_proposal.go:137-151 -> da.ExtendShares + da.NewDataAvailabilityHeader,
// pkg/da/data_availability_header.go:44-75), and go/cda.ExtendSharesOn hands libcda a freshly copied share buffer
// and a NEW 4k^2 x 512 B EDS slice per call (go/cda/extend.go:42-48).  The serial form -- H2D, the whole pipeline,
// one pageable D2H -- took 0.91 ms with a written output buffer but 3.6 ms with a fresh one: the runtime pins a
// never-touched buffer page by page, faulting 8,192 pages in one thread (profiles/r04_pass1.log).  Here the copies
// overlap the device work and the output's first touch is spread over a pool of copy threads (extend_one_host):
//
//   ODS    : up band by band, each band's RS row pass launched as soon as its copy lands.
//   Q0     : the EDS's top-left quadrant IS the ODS (rsmt2d copies the shares in): the pool copies it host to host
//            from the caller's ODS into the caller's EDS -- it never crosses PCIe.
//   Q1     : each band's right halves come back into a pinned slab (one DMA per band) right after that band's row pass,
//            and the pool copies them into the caller's rows.
//   Q2|Q3  : the bottom half comes back right after the column pass, while the leaf hashing, the trees and the DAH
//            run on the compute stream.
//   pages  : a fresh output gets transparent huge pages and is touched by the pool while the device works.
// k <= 256 (pinned slabs of up to 32 + 96 MiB per context); larger squares and profiling runs use the serial form.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"

namespace cda {

// Copy workers of one context.  A job is an ordered list of tasks; workers (and, once it has issued the device
// work, the calling thread) take them in order.  Tasks that need a DMA to land wait for it themselves.  Each job is
// its own object: a worker that wakes late only ever draws from the job it picked up, whose counter is spent.
class CopyPool {
 public:
  CopyPool(const cda_ctx* c, int n) {
    th_.reserve(n);
    try {
      for (int i = 0; i < n; i++)
        th_.emplace_back([this, c] {
          bind_helper_thread(c);
          loop();
        });
    } catch (...) {
      shutdown();
      throw;
    }
  }
  ~CopyPool() { shutdown(); }
  void start(std::vector<std::function<void()>>* tasks) {
    auto j = std::make_shared<Job>();
    j->tasks = tasks;
    j->n = tasks->size();
    {
      std::lock_guard<std::mutex> g(m_);
      cur_ = j;
      ++gen_;
    }
    cv_.notify_all();
  }
  // the calling thread takes tasks too, then waits until every task of the job has finished
  void help_and_wait() {
    std::shared_ptr<Job> j;
    {
      std::lock_guard<std::mutex> g(m_);
      j = cur_;
      cur_.reset();
    }
    if (!j) return;
    run(*j);
    while (j->done.load(std::memory_order_acquire) < j->n) std::this_thread::yield();
  }

 private:
  struct Job {
    std::vector<std::function<void()>>* tasks = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0}, done{0};
  };
  static void run(Job& j) {
    for (;;) {
      const size_t i = j.next.fetch_add(1);
      if (i >= j.n) return;
      (*j.tasks)[i]();
      j.done.fetch_add(1, std::memory_order_release);
    }
  }
  void loop() {
    unsigned seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        j = cur_;
      }
      if (j) run(*j);
    }
  }
  void shutdown() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_)
      if (t.joinable()) t.join();
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::shared_ptr<Job> cur_;
  unsigned gen_ = 0;
  bool stop_ = false;
};

struct Consensus {
  static constexpr int kMaxBands = 4, kMaxPieces = 16;
  CopyPool* pool = nullptr;
  uint8_t* pin_out = nullptr;  // Q1 (k x k shares) of a pageable output
  uint8_t* pin_res = nullptr;  // 4k root records | DAH | status
  uint8_t* d_res = nullptr;    // the same on the device: one D2H of the results
  size_t cap_out = 0, cap_res = 0, cap_dres = 0;
  hipEvent_t ev_in[kMaxBands] = {}, ev_rows[kMaxBands] = {}, ev_q1[kMaxBands] = {}, ev_cols = nullptr,
             ev_done = nullptr, ev_h2d_end = nullptr, ev_d2h_end = nullptr, ev_stg[kMaxPieces] = {};
  ~Consensus() {
    delete pool;
    for (uint8_t* p : {pin_out, pin_res})
      if (p) (void)hipHostFree(p);
    if (d_res) (void)hipFree(d_res);
    for (int i = 0; i < kMaxBands; i++)
      for (hipEvent_t e : {ev_in[i], ev_rows[i], ev_q1[i]})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ev_cols, ev_done, ev_h2d_end, ev_d2h_end})
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_stg)
      if (e) (void)hipEventDestroy(e);
  }
};

void free_consensus(cda_ctx* c) {
  delete c->cons;
  c->cons = nullptr;
}

bool consensus_eligible(const cda_ctx* c, uint32_t k) { return c->consensus && !c->prof && k <= 256; }

namespace {


int grow_pinned(cda_ctx* c, uint8_t*& p, size_t& cap, size_t need) {
  if (cap >= need) return CDA_OK;
  fault_point("alloc");
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  if (!dev_ok(c, hipHostMalloc((void**)&p, need, hipHostMallocDefault), "hipHostMalloc")) return CDA_E_DEVICE;
  cap = need;
  return CDA_OK;
}
int grow_device(cda_ctx* c, uint8_t*& p, size_t& cap, size_t need) {
  if (cap >= need) return CDA_OK;
  fault_point("alloc");
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  if (!dev_ok(c, hipMalloc((void**)&p, need), "hipMalloc")) return CDA_E_DEVICE;
  cap = need;
  return CDA_OK;
}

int get_consensus(cda_ctx* c, Consensus*& out) {
  if (!c->cons) {
    auto* s = new Consensus();
    bool ok = true;
    for (int i = 0; i < Consensus::kMaxBands && ok; i++)
      ok = hipEventCreateWithFlags(&s->ev_in[i], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&s->ev_rows[i], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&s->ev_q1[i], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&s->ev_cols, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&s->ev_h2d_end, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&s->ev_d2h_end, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; i < Consensus::kMaxPieces && ok; i++)
      ok = hipEventCreateWithFlags(&s->ev_stg[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      delete s;
      c->last_err = "consensus path: event creation failed";
      return CDA_E_DEVICE;
    }
    c->cons = s;
  }
  if (!c->cons->pool) {
    fault_point("thread");
    // 7 + the calling thread by default (measured: scripts/consensus_probe.py); CDA_COPY_THREADS read at cda_init
    c->cons->pool = new CopyPool(c, c->copy_threads);
  }
  out = c->cons;
  return CDA_OK;
}

// spin until a host-side counter reaches `need` (a DMA's event has been recorded), or the call aborts
bool wait_count(const std::atomic<int>& cnt, int need, const std::atomic<bool>& abort) {
  while (cnt.load(std::memory_order_acquire) < need) {
    if (abort.load(std::memory_order_relaxed)) return false;
    std::this_thread::yield();
  }
  return true;
}

bool wait_event(hipEvent_t e, std::atomic<bool>& abort) {
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return true;
    if (r != hipErrorNotReady) {
      abort.store(true);
      return false;
    }
    if (abort.load(std::memory_order_relaxed)) return false;
    std::this_thread::yield();
  }
}

// First touch of a range of the caller's output while the device works.  A locked OR with 0 per page: it takes the
// page fault with write intent (the kernel maps a fresh page once, no zero-page / copy-on-write detour) and leaves
// whatever is there -- a copy task of the same page may already have written it on another thread.
// (asm: the compiler lowers an idempotent atomic RMW to a plain load, which only maps the shared zero page.)
inline void touch_byte(uint8_t* b) { asm volatile("lock orb $0, %0" : "+m"(*b) : : "memory"); }
void touch_pages(uint8_t* p, size_t n) {
  for (size_t o = 0; o < n; o += 4096) touch_byte(p + o);
  if (n) touch_byte(p + n - 1);
}

// The caller's output pages: resident (a buffer the caller has written before) or not (a fresh allocation, first
// touched by this call)?  mincore over four 64 KiB windows spread over the range (a whole-range mincore walks 8 K
// page-table entries per call); a failure counts as "not resident".  Either answer is correct for any buffer -- a
// partly resident one only takes the slower form.
bool pages_resident(const uint8_t* p, size_t n) {
  unsigned char vec[16];
  for (int i = 0; i < 4; i++) {
    const uintptr_t at = ((uintptr_t)p + (n - std::min<size_t>(n, 65536)) * i / 3) & ~(uintptr_t)4095;
    const size_t len = std::min<size_t>(65536, (uintptr_t)p + n - at) & ~(size_t)4095;
    if (!len) continue;
    if (mincore((void*)at, len, vec) != 0) return false;
    for (size_t j = 0; j < len / 4096; j++)
      if (!(vec[j] & 1)) return false;
  }
  return true;
}

// Fresh output, opt-in only (cda_set_option(CDA_OPT_HUGE_PAGES)): ask for transparent huge pages on its 2 MiB-aligned
// interior before anything touches it.  The GPU box runs THP in "madvise" mode; with 4 KiB pages the first-touch
// faults of 32 MiB did not scale past ~14 GB/s over any number of threads, with huge pages 8 threads wrote fresh memory
// at ~58 GB/s (tools/fault_probe.cpp, profiles/r04_pass1.log).  It changes page size, never contents -- but it is a
// page policy on memory the library does not own (a Go heap span under cgo), so it is not the default.
void want_huge_pages(uint8_t* p, size_t n) {
  const uintptr_t lo = ((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
  const uintptr_t hi = ((uintptr_t)p + n) & ~(uintptr_t)((2u << 20) - 1);
  if (hi > lo) (void)madvise((void*)lo, hi - lo, MADV_HUGEPAGE);
}

}  // namespace

// The caller holds the context lock.  One block of width k (k <= 256): ods host (k^2 x 512), eds_or_null host
// (4k^2 x 512), roots / dah / err as cda_extend_commit_batch.
//
// Input: pageable hipMemcpyAsync (the runtime pins the caller's written pages on the fly).  Roots only: one copy,
// 0.467 ms per block, against 0.553 ms in four bands (each pageable copy pays its own set-up) and 0.59 ms staged
// through a pinned slab by the copy pool (profiles/r04_pass2.log).  With the EDS: four bands, so that the first
// band's Q1 goes down while the rest comes up (reused output 0.73 vs 0.76-0.78 ms, r04_pass5.log).  Pinning the
// caller's shares for the call (hipHostRegister: an asynchronous H2D with the kernels queued behind it at once) gave
// 0.447 vs 0.452 ms roots only and was slower with the EDS (r04_pass8.log): the rows pass of one block is
// latency-bound (~20 us whatever its size), so the device chain after the input is the same either way.
// Output, by what the caller's EDS buffer is:
//   (every form: Q1 through the pinned slab, copied into the caller's rows by the pool -- a strided D2H runs at half
//   the link rate)
//   pinned      the bottom half straight to it by one DMA;
//   resident    the bottom half split between a pageable DMA (the written pages pin cheaply) and the pinned slab
//               (below);
//   fresh       huge pages asked for (only if the caller opted in) and every page first touched by the pool (one 2 MiB
//               range per task) while the
//               device works, then the resident form, the pageable part of the bottom half in pieces, each sent once
//               its pages are touched.  A pageable DMA into never-touched memory faults it page by page in one thread (3.6 ms
//               per block, r04_pass1); sending the bottom half through the pinned slab in 1 MiB chunks copied out by
//               the pool took 1.02-1.23 ms against 0.80-0.88 ms for this form (r04_pass4.log); registering it
//               (hipHostRegister, async DMA, unregister) was no faster.
// Q0 is always the host copy of the caller's shares.  A/B forms (ctx fields read once at cda_init, ctx.h):
// cons_in = 1 (bands) / 2 (one copy), cons_out = 2 (the resident form on any pageable buffer), cons_trace (phase
// timestamps), cons_stg_mib.  A fresh output gets the huge-page hint only when the caller opted in (huge_pages).
//
// In place (cda_extend_commit_eds): the ODS is Q0 of the caller's EDS buffer (pitch 2k x 512), so there is no Q0 copy
// and each input band is one 2-D DMA from the caller's rows (as fast as a contiguous one from page-locked memory:
// 0.154 vs 0.155 ms per 8 MiB, scripts/h2d_2d_probe.py, profiles/r05_h2d_2d.log).
int extend_one_host(cda_ctx* c, uint32_t k, const uint8_t* ods, uint8_t* eds_or_null, uint8_t* row_roots,
                    uint8_t* col_roots, uint8_t* dah, cda_err_info* err, size_t ods_pitch) {
  const int in_mode_env = c->cons_in, out_mode = c->cons_out;
  const bool trace = c->cons_trace;
  double tr[8] = {0};
  const auto t_start = std::chrono::steady_clock::now();
  auto mark = [&](int i) {
    if (trace) tr[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_start).count();
  };
  const uint32_t w = 2 * k;
  const size_t S = CDA_SHARE, rowS = (size_t)k * S, erowS = (size_t)w * S;
  const size_t ods_b = (size_t)k * rowS, eds_b = (size_t)w * erowS, q1_b = ods_b, bot_b = (size_t)k * erowS;
  const size_t roots_b = (size_t)2 * w * CDA_REC_BYTES, res_b = roots_b + 32 + 8;
  const size_t cells = (size_t)w * w;
  if (!ods_pitch) ods_pitch = rowS;
  const bool inplace = ods == eds_or_null;
  if ((inplace && ods_pitch != erowS) || (!inplace && ods_pitch != rowS)) return CDA_E_ARG;
  Consensus* X = nullptr;
  int rc;
  if ((rc = ensure_pipeline(c)) || (rc = get_consensus(c, X)) || (rc = ensure(c, c->ods, ods_b)) ||
      (rc = ensure(c, c->eds, eds_b)) || (rc = ensure(c, c->leaf, cells * CDA_REC_BYTES)) ||
      (rc = ensure(c, c->scratch, 2 * cells * CDA_REC_BYTES)) || (rc = prepare_trees(c, k, 1, c->stream)))
    return rc;
  const bool want = eds_or_null != nullptr;
  const bool out_pinned = want && pinned_range(eds_or_null, eds_b);
  const bool resident = want && !out_pinned && (out_mode == 2 || pages_resident(eds_or_null, eds_b));
  const bool fresh = want && !out_pinned && !resident;
  const bool banded = in_mode_env ? in_mode_env == 1 : want;

  // A pageable output's bottom half comes down in two concurrent parts: the front by pageable DMA on the D2H stream,
  // the back through the pinned slab on the second stream, copied out by the pool chunk by chunk as it lands.  The
  // pageable DMA alone ran at 36-46 GB/s; side by side the two fill the link.  Staged share, same box
  // (r04_pass12..14.log, k = 128, 16 MiB bottom half): fresh output 0 / 6 / 8 / 10 / 12 MiB -> 0.86 / 0.77 / 0.755
  // / 0.84 / 0.86-0.97 ms, written output 0 / 6 / 8 MiB -> 0.73 / 0.71 / 0.77 ms; so half for a fresh buffer,
  // 3/8 for a written one.  cons_stg_mib (CDA_CONS_STG) = MiB to stage instead (0: all pageable; A/B runs).
  const size_t stg_want = c->cons_stg_mib >= 0 ? ((size_t)c->cons_stg_mib << 20) : (fresh ? bot_b / 2 : bot_b / 8 * 3);
  const size_t stg_b = (want && !out_pinned) ? std::min(bot_b / 4 * 3, stg_want / (2 * erowS) * (2 * erowS)) : 0;
  const size_t dir_b = bot_b - stg_b;  // the pageable part, at the front of the bottom half
  const int n_stg = stg_b ? std::min(Consensus::kMaxPieces, std::max(1, (int)(stg_b >> 20))) : 0;
  if ((want && (rc = grow_pinned(c, X->pin_out, X->cap_out, q1_b + stg_b))) ||
      (rc = grow_pinned(c, X->pin_res, X->cap_res, res_b)) || (rc = grow_device(c, X->d_res, X->cap_dres, res_b)))
    return rc;
  if (fresh && c->huge_pages) want_huge_pages(eds_or_null, eds_b);  // opt-in only (cda_set_option)
  uint8_t* d_ods = (uint8_t*)c->ods.p;
  uint8_t* d_eds = (uint8_t*)c->eds.p;
  uint8_t* d_roots = X->d_res;
  uint8_t* d_dah = X->d_res + roots_b;
  auto* d_status = (unsigned long long*)(X->d_res + roots_b + 32);

  // row-pass bands (an even number of rows each: the FF8 encoder takes codeword pairs); bottom-half pieces of a fresh
  // output (two huge pages each), each sent once the pool has touched its pages
  const uint32_t nband = (banded && k >= 16) ? Consensus::kMaxBands : 1, kb = k / nband;
  const int n_touch = fresh ? (int)std::max<size_t>(1, bot_b >> 21) : 0;
  const int n_piece = fresh ? std::min(Consensus::kMaxPieces, std::max(1, n_touch / 2)) : 1;
  std::atomic<bool> abort{false};
  std::atomic<int> q1_rec{0}, stg_rec{0};
  std::atomic<int> touched[Consensus::kMaxPieces];
  for (int p = 0; p < Consensus::kMaxPieces; p++) touched[p].store(0);

  std::vector<std::function<void()>> tasks;
  tasks.reserve(64);
  if (want) {
    for (int j = 0; j < n_touch; j++) {  // first touch of a fresh bottom half, one 2 MiB range per task
      const size_t lo = bot_b * j / n_touch, hi = bot_b * (j + 1) / n_touch;
      const int piece = j * n_piece / n_touch;
      tasks.emplace_back([=, &touched] {
        touch_pages(eds_or_null + k * erowS + lo, hi - lo);
        touched[piece].fetch_add(1, std::memory_order_acq_rel);
      });
    }
    // Q0 = the shares, host to host (and the first touch of each row's Q1 half); a task covers 1 MiB of EDS rows at
    // k = 128, the even tasks first so that the first faults land on distinct huge pages.  In place: Q0 is there.
    const uint32_t rows_per_task = std::max<uint32_t>(1, (uint32_t)(((size_t)512 << 10) / rowS));
    const uint32_t n_q0 = (k + rows_per_task - 1) / rows_per_task;
    for (uint32_t half = 0; half < 2 && (fresh || !inplace); half++)
      for (uint32_t t = half; t < n_q0; t += 2) {
        const uint32_t r0 = t * rows_per_task;
        tasks.emplace_back([=] {
          for (uint32_t r = r0; r < std::min(k, r0 + rows_per_task); r++) {
            if (fresh) touch_pages(eds_or_null + r * erowS + rowS, rowS);
            if (!inplace) memcpy(eds_or_null + r * erowS, ods + r * rowS, rowS);
          }
        });
      }
    for (uint32_t b = 0; b < nband; b++)  // Q1 rows of band b, once its DMA into the slab has landed
        for (uint32_t r0 = b * kb; r0 < (b + 1) * kb; r0 += rows_per_task)
          tasks.emplace_back([=, &q1_rec, &abort] {
            if (!wait_count(q1_rec, (int)b + 1, abort) || !wait_event(X->ev_q1[b], abort)) return;
            for (uint32_t r = r0; r < std::min((b + 1) * kb, r0 + rows_per_task); r++)
              memcpy(eds_or_null + r * erowS + rowS, X->pin_out + r * rowS, rowS);
          });
    for (int j = 0; j < n_stg; j++) {  // staged chunk j of the bottom half's tail, four copy tasks each
      const size_t lo = stg_b * j / n_stg, hi = stg_b * (j + 1) / n_stg;
      for (int h = 0; h < 4; h++) {
        const size_t a0 = lo + (hi - lo) * h / 4, a1 = lo + (hi - lo) * (h + 1) / 4;
        tasks.emplace_back([=, &stg_rec, &abort] {
          if (!wait_count(stg_rec, j + 1, abort) || !wait_event(X->ev_stg[j], abort)) return;
          memcpy(eds_or_null + k * erowS + dir_b + a0, X->pin_out + q1_b + a0, a1 - a0);
        });
      }
    }
  }
  X->pool->start(&tasks);
  // From here the pool's tasks reference this frame (tasks, touched, the counters, abort) and the caller's buffers:
  // on ANY exit before the orderly join below -- an error return or an exception -- the guard stops them, joins the
  // job and drains the three streams before those locals (declared above it) are destroyed.
  struct JoinGuard {
    cda_ctx* c;
    Consensus* X;
    std::atomic<bool>& abort;
    bool armed = true;
    ~JoinGuard() {
      if (!armed) return;
      abort.store(true);
      X->pool->help_and_wait();
      (void)hipStreamSynchronize(c->h2d_stream);
      (void)hipStreamSynchronize(c->stream);
      (void)hipStreamSynchronize(c->d2h_stream);
    }
  } guard{c, X, abort};
  mark(1);

  hipStream_t s = c->stream;
  const char* fail = nullptr;
  int frc = CDA_OK;
  // the order-status word is set on the compute stream while the input is still coming up (off the chain)
  if (hipMemsetAsync(d_status, 0xFF, 8, s) != hipSuccess) fail = "status";
  // Q1 of band b back to the host once its row pass has run (D2H stream).  It lands contiguously in the pinned slab
  // and the pool moves the rows into the caller's buffer: a DMA into the strided right halves of the caller's rows ran
  // at about half the link rate (8 MiB: 0.31-0.40 ms against 0.16 ms contiguous, pinned caller memory too; a strided
  // DEVICE source costs nothing: 0.17 ms; scripts/pcie_duplex_probe.py, profiles/r05_pcie_duplex.log).
  auto issue_q1 = [&](uint32_t b) -> bool {
    const size_t r0 = (size_t)b * kb;
    if (hipStreamWaitEvent(c->d2h_stream, X->ev_rows[b], 0) != hipSuccess ||
        hipMemcpy2DAsync(X->pin_out + r0 * rowS, rowS, d_eds + r0 * erowS + rowS, erowS, rowS, kb,
                         hipMemcpyDeviceToHost, c->d2h_stream) != hipSuccess ||
        hipEventRecord(X->ev_q1[b], c->d2h_stream) != hipSuccess)
      return false;
    q1_rec.store((int)b + 1, std::memory_order_release);
    return true;
  };
  for (uint32_t b = 0; b < nband && !fail; b++) {  // device work, band by band as the input lands
    const size_t r0 = (size_t)b * kb;
    // (a page-locked input read by the row pass itself across PCIe, no DMA: 66 us per 2 MiB band against 44 us by
    // DMA, 0.84 vs 0.74 ms per call; measured and removed, profiles/r05_consensus_timeline.log)
    const hipError_t in_rc =
        ods_pitch == rowS ? hipMemcpyAsync(d_ods + r0 * rowS, ods + r0 * rowS, (size_t)kb * rowS,
                                           hipMemcpyHostToDevice, c->h2d_stream)
                          : hipMemcpy2DAsync(d_ods + r0 * rowS, rowS, ods + r0 * ods_pitch, ods_pitch, rowS, kb,
                                             hipMemcpyHostToDevice, c->h2d_stream);
    if (in_rc != hipSuccess || hipEventRecord(X->ev_in[b], c->h2d_stream) != hipSuccess ||
        hipStreamWaitEvent(s, X->ev_in[b], 0) != hipSuccess) {
      fail = "H2D";
      break;
    }
    RsJob j = rows_job(k, 1, d_ods, d_eds);
    j.src += r0 * rowS;
    j.dst += r0 * erowS;
    j.cpy += r0 * erowS;
    j.cw_per_blk = (int)kb;
    if (const int lr = 2 * k <= 256 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s)) {
      frc = lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
      fail = "rows";
      break;
    }
    if (want && (hipEventRecord(X->ev_rows[b], s) != hipSuccess || !issue_q1(b))) {
      fail = "Q1 D2H";
      break;
    }
  }
  mark(2);
  if (!fail) {
    const RsJob j = cols_job(k, 1, d_eds);
    if (const int lr = 2 * k <= 256 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s)) {
      frc = lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
      fail = "cols";
    }
  }
  if (!fail && want &&
      (hipEventRecord(X->ev_cols, s) != hipSuccess || hipStreamWaitEvent(c->d2h_stream, X->ev_cols, 0) != hipSuccess))
    fail = "event";
  // pinned output: the bottom half straight to it, one DMA behind the Q1 bands.  Device-to-host copies run one at a
  // time whatever stream they are on (a second stream's copy started ~9 us after the first ended), so moving it to
  // the idle input stream, whole or half, changed nothing (profiles/r05_consensus_timeline.log)
  if (!fail && out_pinned &&
      hipMemcpyAsync(eds_or_null + k * erowS, d_eds + k * erowS, bot_b, hipMemcpyDeviceToHost, c->d2h_stream) !=
          hipSuccess)
    fail = "bottom D2H";
  if (!fail && n_stg && hipStreamWaitEvent(c->h2d_stream, X->ev_cols, 0) != hipSuccess) fail = "event";
  for (int j = 0; j < n_stg && !fail; j++) {
    const size_t lo = stg_b * j / n_stg, hi = stg_b * (j + 1) / n_stg;
    if (hipMemcpyAsync(X->pin_out + q1_b + lo, d_eds + k * erowS + dir_b + lo, hi - lo, hipMemcpyDeviceToHost,
                       c->h2d_stream) != hipSuccess ||
        hipEventRecord(X->ev_stg[j], c->h2d_stream) != hipSuccess) {
      fail = "staged D2H";
      break;
    }
    stg_rec.store(j + 1, std::memory_order_release);
  }
  if (!fail) {
    if ((rc = enqueue_commit(c, k, 1, d_eds, d_roots, d_dah, d_status, s, 0, false))) {
      frc = rc;
      fail = "commit";
    } else if (hipMemcpyAsync(X->pin_res, X->d_res, res_b, hipMemcpyDeviceToHost, s) != hipSuccess ||
               hipEventRecord(X->ev_done, s) != hipSuccess) {
      fail = "results D2H";
    }
  }
  mark(3);
  // pageable output: the bottom half by pageable DMA from this thread (it waits in each call while the pool copies
  // Q0 / Q1); a fresh output piece by piece as the pool finishes touching it
  for (int p = 0; p < n_piece && !fail && want && !out_pinned; p++) {
    if (fresh) {  // the touch tasks of piece p: j with j * n_piece / n_touch == p
      const int need = (int)(((int64_t)(p + 1) * n_touch + n_piece - 1) / n_piece -
                             ((int64_t)p * n_touch + n_piece - 1) / n_piece);
      while (touched[p].load(std::memory_order_acquire) < need && !abort.load(std::memory_order_relaxed))
        std::this_thread::yield();
    }
    const size_t lo = std::min(dir_b, bot_b * p / n_piece), hi = std::min(dir_b, bot_b * (p + 1) / n_piece);
    if (hi > lo && hipMemcpyAsync(eds_or_null + k * erowS + lo, d_eds + k * erowS + lo, hi - lo,
                                  hipMemcpyDeviceToHost, c->d2h_stream) != hipSuccess)
      fail = "bottom D2H";
  }
  if (!fail && (hipEventRecord(X->ev_h2d_end, c->h2d_stream) != hipSuccess ||
                hipEventRecord(X->ev_d2h_end, c->d2h_stream) != hipSuccess))
    fail = "event";
  mark(4);
  if (fail) abort.store(true);
  X->pool->help_and_wait();
  guard.armed = false;  // joined here; the streams are waited for below on every path
  mark(5);
  if (!fail) wait_event(X->ev_done, abort);
  mark(6);
  // every DMA of this call has finished before the caller's buffers (or the staging) can be touched again: the
  // streams' end events (a stream sync costs ~6 us per stream here), or whole-stream syncs after a failure
  bool synced;
  if (!fail && !abort.load())
    synced = wait_event(X->ev_h2d_end, abort) && wait_event(X->ev_d2h_end, abort);
  else
    synced = hipStreamSynchronize(c->h2d_stream) == hipSuccess && hipStreamSynchronize(s) == hipSuccess &&
             hipStreamSynchronize(c->d2h_stream) == hipSuccess;
  mark(7);
  if (trace)
    fprintf(stderr, "cons_trace fresh=%d resident=%d pool_started=%.1f rows_issued=%.1f commit_issued=%.1f "
            "bottom_dma_issued=%.1f pool_done=%.1f done_event=%.1f synced=%.1f\n",
            (int)fresh, (int)resident, tr[1], tr[2], tr[3], tr[4], tr[5], tr[6], tr[7]);
  if (fail) {
    if (frc == CDA_OK) {
      c->last_err = std::string("consensus path: ") + fail + ": " + hipGetErrorString(hipGetLastError());
      frc = CDA_E_DEVICE;
    }
    return frc;
  }
  if (abort.load() || !synced) {
    c->last_err = std::string("consensus path: ") + hipGetErrorString(hipGetLastError());
    return CDA_E_DEVICE;
  }
  pack_roots(X->pin_res, w, row_roots);
  pack_roots(X->pin_res + (size_t)w * CDA_REC_BYTES, w, col_roots);
  memcpy(dah, X->pin_res + roots_b, 32);
  uint64_t st;
  memcpy(&st, X->pin_res + roots_b + 32, 8);
  return map_status(st, 0, err);
}

}  // namespace cda
