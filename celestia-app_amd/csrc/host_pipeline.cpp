// host_pipeline.cpp — the drop-in boundary with HOST buffers (what a cgo caller hands over):
// cda_extend_commit_batch as a three-stage pipeline, and the multi-device batch.
//
// da.ExtendShares + da.NewDataAvailabilityHeader (pkg/da/data_availability_header.go:44-75) over
// many independent blocks whose shares live in host memory.  PCIe, not the GPU, bounds this path
// (8 MiB of ODS in and 32 MiB of EDS out per k=128 block against ~50 GB/s per direction), so the
// batch is cut into chunks and three streams overlap
//     H2D(chunk i+1)  ‖  extension + trees(chunk i)  ‖  D2H(chunk i-1)
// through a ring of kSlots device slots.  The two copy stages run on their own host threads: a copy
// from / to pageable memory blocks its calling thread, and PCIe is full duplex, so the H2D and D2H
// streams must be fed independently for the two directions to overlap.
//
// Ordering (slot j = i % kSlots, events per slot):
//   H2D(i)  waits ev_comp[j] of chunk i-kSlots (its ODS slot was read)   -> records ev_h2d[j]
//   comp(i) waits ev_h2d[j] and ev_d2h[j] of chunk i-kSlots (EDS slot drained) -> records ev_comp[j]
//   D2H(i)  waits ev_comp[j]                                              -> records ev_d2h[j]
// A stage waits on an event only after the stage that records it has issued that chunk (host-side
// counters), so every hipStreamWaitEvent sees the intended record.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"

using namespace cda;

namespace {

// Blocks per chunk: ~32 MiB of ODS (4 blocks at k = 128) keeps the kernels of a chunk efficient
// while leaving several chunks to overlap.
uint32_t chunk_blocks(uint32_t k, uint32_t nblocks) {
  const size_t ods_b = (size_t)k * k * CDA_SHARE;
  uint32_t c = (uint32_t)std::max<size_t>(1, ((size_t)32 << 20) / ods_b);
  // at least 3 chunks when the batch allows it, so all three stages are busy
  while (c > 1 && (nblocks + c - 1) / c < 3) c = (c + 1) / 2;
  return std::min(c, nblocks);
}

struct Progress {  // chunks issued by each stage; waits are bounded by `abort`
  std::mutex m;
  std::condition_variable cv;
  uint32_t h2d = 0, comp = 0, d2h = 0;
  bool abort = false;
  void bump(uint32_t Progress::*f) {
    {
      std::lock_guard<std::mutex> g(m);
      ++(this->*f);
    }
    cv.notify_all();
  }
  bool wait_for(uint32_t Progress::*f, uint32_t at_least) {  // false if aborted
    std::unique_lock<std::mutex> g(m);
    cv.wait(g, [&] { return abort || this->*f >= at_least; });
    return !abort;
  }
  void fail() {
    {
      std::lock_guard<std::mutex> g(m);
      abort = true;
    }
    cv.notify_all();
  }
};

}  // namespace

namespace cda {

int ensure_pipeline(cda_ctx* c) {
  if (c->h2d_stream) return CDA_OK;
  bool ok = hipStreamCreateWithFlags(&c->h2d_stream, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking) == hipSuccess;
  for (int j = 0; j < cda_ctx::kSlots && ok; j++)
    ok = hipEventCreateWithFlags(&c->ev_h2d[j], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_comp[j], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_d2h[j], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    c->last_err = "pipeline stream/event creation failed";
    return CDA_E_DEVICE;
  }
  return CDA_OK;
}

void free_pipeline(cda_ctx* c) {
  if (c->h2d_stream) (void)hipStreamDestroy(c->h2d_stream);
  if (c->d2h_stream) (void)hipStreamDestroy(c->d2h_stream);
  for (int j = 0; j < cda_ctx::kSlots; j++) {
    if (c->ev_h2d[j]) (void)hipEventDestroy(c->ev_h2d[j]);
    if (c->ev_comp[j]) (void)hipEventDestroy(c->ev_comp[j]);
    if (c->ev_d2h[j]) (void)hipEventDestroy(c->ev_d2h[j]);
  }
}

// The pipelined batch (caller holds the ctx lock).  `block0` offsets error reports (multi-device).
int batch_pipelined(cda_ctx* c, uint32_t k, uint32_t nblocks, const uint8_t* ods, uint8_t* eds_or_null,
                    uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, cda_err_info* err, int block0) {
  const uint32_t w = 2 * k;
  const size_t ods_blk = (size_t)k * k * CDA_SHARE, eds_blk = (size_t)w * w * CDA_SHARE;
  const size_t rec_blk = (size_t)2 * w * CDA_REC_BYTES;
  const uint32_t C = chunk_blocks(k, nblocks);
  const uint32_t nchunks = (nblocks + C - 1) / C;
  const int S = cda_ctx::kSlots;
  int rc;
  if ((rc = ensure_pipeline(c))) return rc;
  // slot layout: S x [ODS C blocks] in c->ods, S x [EDS C blocks] in c->eds, S x roots/dah/status
  if ((rc = ensure(c, c->ods, S * C * ods_blk)) || (rc = ensure(c, c->eds, S * C * eds_blk)) ||
      (rc = ensure(c, c->roots, S * C * rec_blk)) || (rc = ensure(c, c->dah, (size_t)S * C * 32)) ||
      (rc = ensure(c, c->status, (size_t)S * C * 8)) || (rc = ensure(c, c->leaf, (size_t)C * w * w * CDA_REC_BYTES)) ||
      (rc = ensure(c, c->scratch, (size_t)2 * C * w * w * CDA_REC_BYTES)))
    return rc;
  std::vector<uint8_t> recs((size_t)nblocks * rec_blk);
  std::vector<uint64_t> st(nblocks);
  Progress pr;
  std::atomic<int> first_rc{CDA_OK};
  auto fail = [&](int code, const char* what) {
    int expect = CDA_OK;
    if (first_rc.compare_exchange_strong(expect, code) && what) c->last_err = what;
    pr.fail();
  };
  auto nb_of = [&](uint32_t i) { return std::min(C, nblocks - i * C); };
  auto slot_ods = [&](uint32_t i) { return (uint8_t*)c->ods.p + (size_t)(i % S) * C * ods_blk; };
  auto slot_eds = [&](uint32_t i) { return (uint8_t*)c->eds.p + (size_t)(i % S) * C * eds_blk; };
  auto slot_rec = [&](uint32_t i) { return (uint8_t*)c->roots.p + (size_t)(i % S) * C * rec_blk; };
  auto slot_dah = [&](uint32_t i) { return (uint8_t*)c->dah.p + (size_t)(i % S) * C * 32; };
  auto slot_st = [&](uint32_t i) { return (uint8_t*)c->status.p + (size_t)(i % S) * C * 8; };
  const int dev = c->device;
  // helpers: a failed start of the second (or an exception below) aborts the first and joins it, then the
  // streams drain before the caller's buffers are released
  std::thread h2d, d2h;
  auto stop = [&] {
    pr.fail();
    if (h2d.joinable()) h2d.join();
    if (d2h.joinable()) d2h.join();
    (void)hipStreamSynchronize(c->h2d_stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->d2h_stream);
  };
  ThreadJoiner<decltype(stop)> joiner(stop);
  joiner.ts = {&h2d, &d2h};
  // a helper's own exception (e.g. std::system_error from its mutex) becomes this call's error code
  auto guarded = [&](auto body) {
    return [&, body] {
      try {
        body();
      } catch (...) {
        fail(api_exception(c), nullptr);
      }
    };
  };

  h2d = std::thread(guarded([&] {
    (void)hipSetDevice(dev);
    for (uint32_t i = 0; i < nchunks; i++) {
      const int j = (int)(i % S);
      if (i >= (uint32_t)S) {
        if (!pr.wait_for(&Progress::comp, i - S + 1)) return;
        if (hipStreamWaitEvent(c->h2d_stream, c->ev_comp[j], 0) != hipSuccess) return fail(CDA_E_DEVICE, "wait");
      }
      if (hipMemcpyAsync(slot_ods(i), ods + (size_t)i * C * ods_blk, nb_of(i) * ods_blk, hipMemcpyHostToDevice,
                         c->h2d_stream) != hipSuccess ||
          hipEventRecord(c->ev_h2d[j], c->h2d_stream) != hipSuccess)
        return fail(CDA_E_DEVICE, "H2D");
      pr.bump(&Progress::h2d);
    }
  }));
  fault_point("thread");
  d2h = std::thread(guarded([&] {
    (void)hipSetDevice(dev);
    for (uint32_t i = 0; i < nchunks; i++) {
      const int j = (int)(i % S);
      if (!pr.wait_for(&Progress::comp, i + 1)) return;
      const uint32_t nb = nb_of(i);
      if (hipStreamWaitEvent(c->d2h_stream, c->ev_comp[j], 0) != hipSuccess) return fail(CDA_E_DEVICE, "wait");
      if ((eds_or_null && hipMemcpyAsync(eds_or_null + (size_t)i * C * eds_blk, slot_eds(i), nb * eds_blk,
                                         hipMemcpyDeviceToHost, c->d2h_stream) != hipSuccess) ||
          hipMemcpyAsync(recs.data() + (size_t)i * C * rec_blk, slot_rec(i), nb * rec_blk, hipMemcpyDeviceToHost,
                         c->d2h_stream) != hipSuccess ||
          hipMemcpyAsync(dah + (size_t)i * C * 32, slot_dah(i), (size_t)nb * 32, hipMemcpyDeviceToHost,
                         c->d2h_stream) != hipSuccess ||
          hipMemcpyAsync(st.data() + (size_t)i * C, slot_st(i), (size_t)nb * 8, hipMemcpyDeviceToHost,
                         c->d2h_stream) != hipSuccess ||
          hipEventRecord(c->ev_d2h[j], c->d2h_stream) != hipSuccess)
        return fail(CDA_E_DEVICE, "D2H");
      pr.bump(&Progress::d2h);
    }
  }));
  for (uint32_t i = 0; i < nchunks; i++) {
    const int j = (int)(i % S);
    if (!pr.wait_for(&Progress::h2d, i + 1)) break;
    if (hipStreamWaitEvent(c->stream, c->ev_h2d[j], 0) != hipSuccess) {
      fail(CDA_E_DEVICE, "wait");
      break;
    }
    if (i >= (uint32_t)S) {
      if (!pr.wait_for(&Progress::d2h, i - S + 1)) break;
      if (hipStreamWaitEvent(c->stream, c->ev_d2h[j], 0) != hipSuccess) {
        fail(CDA_E_DEVICE, "wait");
        break;
      }
    }
    const int r = enqueue_pipeline(c, k, nb_of(i), slot_ods(i), slot_eds(i), slot_rec(i), slot_dah(i),
                                   (unsigned long long*)slot_st(i), c->stream);
    if (r) {
      fail(r, nullptr);
      break;
    }
    if (hipEventRecord(c->ev_comp[j], c->stream) != hipSuccess) {
      fail(CDA_E_DEVICE, "record");
      break;
    }
    pr.bump(&Progress::comp);
  }
  h2d.join();
  d2h.join();
  // drain every stream before the workspace can be reused or the caller's buffers released
  const bool synced = hipStreamSynchronize(c->h2d_stream) == hipSuccess &&
                      hipStreamSynchronize(c->stream) == hipSuccess &&
                      hipStreamSynchronize(c->d2h_stream) == hipSuccess;
  if (first_rc.load() != CDA_OK) return first_rc.load();
  if (!synced) return dev_ok(c, hipGetLastError(), "sync"), CDA_E_DEVICE;
  flush_profile(c);
  for (uint32_t b = 0; b < nblocks; b++) {
    const uint8_t* r = recs.data() + (size_t)b * rec_blk;
    pack_roots(r, w, row_roots + (size_t)b * w * CDA_NODE_SIZE);
    pack_roots(r + (size_t)w * CDA_REC_BYTES, w, col_roots + (size_t)b * w * CDA_NODE_SIZE);
  }
  for (uint32_t b = 0; b < nblocks; b++)
    if ((rc = map_status(st[b], block0 + (int)b, err))) return rc;
  return CDA_OK;
}

}  // namespace cda

extern "C" {

int cda_host_alloc(cda_ctx* c, size_t bytes, void** out) {
  CDA_API_TRY
  if (!c || !out) return CDA_E_ARG;
  *out = nullptr;
  Lock l(c);
  if (!dev_ok(c, hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault), "hipHostMalloc")) return CDA_E_DEVICE;
  return CDA_OK;
  CDA_API_CATCH(c)
}

int cda_host_free(cda_ctx* c, void* p) {
  CDA_API_TRY
  if (!c) return CDA_E_ARG;
  if (!p) return CDA_OK;
  Lock l(c);
  return dev_ok(c, hipHostFree(p), "hipHostFree") ? CDA_OK : CDA_E_DEVICE;
  CDA_API_CATCH(c)
}

int cda_host_register(cda_ctx* c, void* p, size_t bytes) {
  CDA_API_TRY
  if (!c || !p || !bytes) return CDA_E_ARG;
  Lock l(c);
  return dev_ok(c, hipHostRegister(p, bytes, hipHostRegisterDefault), "hipHostRegister") ? CDA_OK : CDA_E_DEVICE;
  CDA_API_CATCH(c)
}

int cda_host_unregister(cda_ctx* c, void* p) {
  CDA_API_TRY
  if (!c || !p) return CDA_E_ARG;
  Lock l(c);
  // Every DMA this context enqueued into or out of the range has finished before the pages are released: the
  // synchronous entry points return only after their copies completed, and the copy streams (h2d / d2h: the batch
  // pipeline, the one-block path, repair; aux: repair's verification) and the main stream are drained here as well,
  // so this holds whatever a future entry point leaves in flight.
  for (hipStream_t s : {c->stream, c->h2d_stream, c->d2h_stream, c->aux_stream})
    if (s && !dev_ok(c, hipStreamSynchronize(s), "sync")) return CDA_E_DEVICE;
  return dev_ok(c, hipHostUnregister(p), "hipHostUnregister") ? CDA_OK : CDA_E_DEVICE;
  CDA_API_CATCH(c)
}

// ---- multi-device batch ----------------------------------------------------------------------
// (struct cda_multi: ctx.h)

int cda_multi_init(uint32_t device_mask, cda_multi** out) {
  CDA_API_TRY
  if (!out) return CDA_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CDA_E_DEVICE;
  if (device_mask == 0) device_mask = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1);
  cda_multi* m = new cda_multi();
  struct Owner {
    cda_multi* m;
    ~Owner() {
      if (m) cda_multi_free(m);
    }
  } own{m};
  for (int d = 0; d < 32; d++) {
    if (!(device_mask & (1u << d))) continue;
    cda_ctx* c = nullptr;
    if (d >= n || cda_init(d, &c) != CDA_OK) return CDA_E_DEVICE;
    m->ctx.reserve(m->ctx.size() + 1);
    m->ctx.push_back(c);
    m->devices.push_back(d);
  }
  own.m = nullptr;
  *out = m;
  return CDA_OK;
  CDA_API_CATCH(nullptr)
}

void cda_multi_free(cda_multi* m) {
  if (!m) return;
  free_split_comm(m);
  if (m->pin_res) (void)hipHostFree(m->pin_res);
  for (auto* c : m->ctx) cda_free(c);
  delete m;
}

int cda_multi_device_count(const cda_multi* m) { return m ? (int)m->ctx.size() : 0; }

int cda_multi_device(const cda_multi* m, int i) {
  return (m && i >= 0 && i < (int)m->devices.size()) ? m->devices[i] : -1;
}

cda_ctx* cda_multi_context(cda_multi* m, int i) {
  return (m && i >= 0 && i < (int)m->ctx.size()) ? m->ctx[i] : nullptr;
}

int cda_multi_extend_commit_batch(cda_multi* m, uint32_t k, uint32_t nblocks, const uint8_t* ods,
                                  uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                                  cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!m || m->ctx.empty() || !ods || !row_roots || !col_roots || !dah || nblocks == 0) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  const uint32_t w = 2 * k;
  const size_t ods_blk = (size_t)k * k * CDA_SHARE, eds_blk = (size_t)w * w * CDA_SHARE;
  const size_t root_blk = (size_t)w * CDA_NODE_SIZE;
  const uint32_t G = (uint32_t)m->ctx.size();
  std::vector<int> rcs(G, CDA_OK);
  std::vector<cda_err_info> errs(G);
  std::vector<std::thread> th;
  th.reserve(G);
  struct JoinAll {
    std::vector<std::thread>& v;
    ~JoinAll() {
      for (auto& t : v)
        if (t.joinable()) t.join();
    }
  } join_all{th};
  uint32_t done = 0;
  for (uint32_t g = 0; g < G; g++) {  // contiguous block ranges, no collective
    const uint32_t nb = (nblocks - done) / (G - g);
    const uint32_t b0 = done;
    done += nb;
    if (nb == 0) continue;
    th.emplace_back([&, g, nb, b0] {
      cda_ctx* c = m->ctx[g];
      try {
        Lock l(c);
        rcs[g] = batch_pipelined(c, k, nb, ods + (size_t)b0 * ods_blk,
                                 eds_or_null ? eds_or_null + (size_t)b0 * eds_blk : nullptr,
                                 row_roots + (size_t)b0 * root_blk, col_roots + (size_t)b0 * root_blk,
                                 dah + (size_t)b0 * 32, &errs[g], (int)b0);
      } catch (...) {
        rcs[g] = api_exception(c);
      }
    });
  }
  for (auto& t : th) t.join();
  // report the lowest failing block (device order = block order)
  for (uint32_t g = 0; g < G; g++)
    if (rcs[g] != CDA_OK) {
      if (err) *err = errs[g];
      if (err) err->code = rcs[g];
      return rcs[g];
    }
  return CDA_OK;
  CDA_API_CATCH(nullptr)
}

}  // extern "C"
