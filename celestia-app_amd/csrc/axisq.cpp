// axisq.cpp — the per-axis seams of the drop-in: rsmt2d.Codec Encode / Decode (cda_rs_encode, cda_rs_decode) and the
// wrapper tree's Root (cda_nmt_axis_root), as rsmt2d calls them when appconsts.DefaultCodec is the GPU codec
// (pkg/appconsts/global_consts.go:92, go/pkg_da/extend_rocm.go) and the tree constructor is go/cda's
// (pkg/wrapper/nmt_wrapper.go:73-124).
//
// rsmt2d issues these one axis at a time -- erasureExtendSquare and computeRoots from one goroutine per axis,
// prerepairSanityCheck likewise, the Repair crossword sequentially -- through pageable Go slices.  A call that went
// to the device on its own paid a pageable H2D, one or more launches, a pageable D2H and a synchronisation, and
// concurrent calls queued behind the context mutex one round trip at a time.  Here every call is a request on the
// context's axis queue (group commit):
//   * a caller that finds a free batch slot becomes a leader and takes every request queued so far (up to the
//     slot's share of kBatchBytes of staging); requests that arrive while every slot is busy form the next batch, so
//     a lone caller pays no wait and concurrent callers share launches.  Up to kSlots batches are in flight at once,
//     each on its own stream and staging: a batch of axis trees or codewords is a latency-bound launch on a few CUs,
//     so batches run side by side instead of one after another;
//   * each caller copies its own input into its batch's page-locked staging and its own output back (the copies run
//     on the callers' threads in parallel), and the kernels read and write that staging directly (zero-copy);
//   * requests of one shape run as one launch: the encoder over n codewords (RsJob with cw stride = slot size), the
//     decoder over n codewords (per-codeword descriptors), and axis_roots_kernel over n trees (one workgroup each,
//     the tree in LDS: one launch instead of a leaf launch plus a launch per level).
// The outputs are the bytes the single-call path produced (same kernels, same arithmetic); the leader synchronises
// before any caller reads its result, and no caller pointer is kept after its call returns (cgo rule).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "ctx.h"

namespace cda {

namespace {

enum : int { kEnc = 0, kRoot = 1, kDec = 2 };  // group order in a batch: inputs-only kinds first, in+out (decode) last
// kTaken: in a batch whose leader is still preparing its slot (its owner waits)
enum : int { kQueued = 0, kTaken = 1, kCopyIn = 2, kCopied = 3, kResult = 4, kDone = 5 };

// staging of all batches in flight: at most this many bytes, split evenly over the slots (a larger single request
// runs alone)
constexpr size_t kBatchBytes = 64ull << 20;
constexpr size_t kAlign = 512;
// batches in flight at once (CDA_AXIS_SLOTS in the test-hooks build, 1..kMaxSlots)
constexpr int kSlots = 4, kMaxSlots = 8;

size_t up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

}  // namespace

// One batch in flight: its page-locked staging (host address and the device's alias of it) and its stream.
struct AxisSlot {
  uint8_t* h = nullptr;
  uint8_t* hd = nullptr;
  size_t cap = 0;
  hipStream_t s = nullptr;
  bool busy = false;
  size_t copy_left = 0, out_left = 0;
  std::condition_variable lead_cv;  // the batch's leader waits here for its members' copies
};

struct AxisReq {
  int kind = kEnc;
  uint32_t k = 0, len = 0, n = 0;  // enc / dec: k data shards of len bytes; root: n leaves of 512 bytes
  uint64_t square_size = 0, axis_index = 0;
  const uint8_t* in = nullptr;       // enc: k*len data; dec: 2k*len shards; root: n*512 leaves
  uint8_t* out = nullptr;            // enc: k*len parity; dec: the shards (missing ones written)
  const uint8_t* present = nullptr;  // dec: 2k flags
  size_t off = 0, out_off = 0, st_off = 0;  // offsets in the batch's staging
  AxisSlot* slot = nullptr;                 // the batch's slot, once taken into one
  int state = kQueued;
  int rc = CDA_OK;
  uint8_t rec[CDA_REC_BYTES];  // root: the root record
  uint64_t st = ~0ull;         // root: first leaf failing the push-order check, or ~0
  std::condition_variable cv;  // its owner waits here: one wake-up per state change, no thundering herd

  size_t in_bytes() const { return kind == kEnc ? (size_t)k * len : kind == kDec ? (size_t)2 * k * len : (size_t)n * len; }
  size_t bytes() const { return in_bytes() + (kind == kEnc ? (size_t)k * len : kind == kRoot ? 128 : 2 * (size_t)k + 16); }
};

struct AxisQueue {
  std::mutex mu;
  std::vector<AxisReq*> pending;
  AxisSlot slot[kMaxSlots];
  int nslots = kSlots;
  size_t batch_bytes = kBatchBytes / kSlots;  // staging per slot (kBatchBytes / nslots)
  size_t largest = 0;  // the largest staging any slot has needed: a slot that grows grows to at least this
};

namespace {

struct Group {
  int kind;
  uint32_t k, len, n;
  uint64_t ss;
  std::vector<AxisReq*> reqs;
  size_t item_in = 0, item_out = 0;  // slot sizes (the codeword / tree stride of the launch)
  size_t in0 = 0, out0 = 0, st0 = 0, desc0 = 0;
};

struct Layout {
  std::vector<Group> groups;
  size_t total = 0;
};

// Staging layout of a batch: inputs of encodes and roots | descriptors | decode codewords (in place) | parity, root
// records and status words.
void plan(std::vector<AxisReq*>& batch, Layout& L) {
  std::map<std::tuple<int, uint32_t, uint32_t, uint64_t>, size_t> idx;
  for (AxisReq* r : batch) {
    const auto key = r->kind == kRoot ? std::make_tuple(r->kind, r->n, r->len, r->square_size)
                                      : std::make_tuple(r->kind, r->k, r->len, (uint64_t)0);
    auto it = idx.find(key);
    if (it == idx.end()) {
      it = idx.emplace(key, L.groups.size()).first;
      L.groups.push_back(Group{r->kind, r->k, r->len, r->n, r->square_size, {}});
    }
    L.groups[it->second].reqs.push_back(r);
  }
  std::stable_sort(L.groups.begin(), L.groups.end(), [](const Group& a, const Group& b) { return a.kind < b.kind; });
  size_t cur = 0;
  for (Group& g : L.groups) {  // inputs of encodes and roots
    if (g.kind == kDec) continue;
    g.item_in = up(g.kind == kEnc ? (size_t)g.k * g.len : (size_t)g.n * g.len);
    g.in0 = cur;
    for (AxisReq* r : g.reqs) r->off = cur, cur += g.item_in;
  }
  for (Group& g : L.groups) {  // descriptors: axis indices of the trees; offsets, strides and presence of codewords
    if (g.kind == kEnc) continue;
    g.desc0 = cur;
    cur += up(g.kind == kRoot ? 8 * g.reqs.size() : g.reqs.size() * (16 + 2 * (size_t)g.k));
  }
  for (Group& g : L.groups) {  // decode codewords (in and out)
    if (g.kind != kDec) continue;
    g.item_in = up((size_t)2 * g.k * g.len);
    g.in0 = cur;
    for (AxisReq* r : g.reqs) r->off = r->out_off = cur, cur += g.item_in;
  }
  for (Group& g : L.groups) {  // parity, root records, status words
    if (g.kind == kEnc) {
      g.item_out = up((size_t)g.k * g.len);
      g.out0 = cur;
      for (AxisReq* r : g.reqs) r->out_off = cur, cur += g.item_out;
    } else if (g.kind == kRoot) {
      g.out0 = cur;
      cur += up(CDA_REC_BYTES * g.reqs.size());
      g.st0 = cur;
      cur += up(8 * g.reqs.size());
      for (size_t t = 0; t < g.reqs.size(); t++) {
        g.reqs[t]->out_off = g.out0 + t * CDA_REC_BYTES;
        g.reqs[t]->st_off = g.st0 + t * 8;
      }
    }
  }
  L.total = cur;
}

// descriptors of the batch, written by the leader while the callers copy their inputs
void fill_desc(const Layout& L, uint8_t* h) {
  for (const Group& g : L.groups) {
    const size_t n = g.reqs.size();
    if (g.kind == kRoot) {
      for (size_t t = 0; t < n; t++) memcpy(h + g.desc0 + 8 * t, &g.reqs[t]->axis_index, 8);
    } else if (g.kind == kDec) {
      for (size_t t = 0; t < n; t++) {
        const long long off = (long long)g.reqs[t]->off, stride = g.len;
        memcpy(h + g.desc0 + 8 * t, &off, 8);
        memcpy(h + g.desc0 + 8 * (n + t), &stride, 8);
        uint8_t* p = h + g.desc0 + 16 * n + 2 * (size_t)g.k * t;
        for (uint32_t i = 0; i < 2 * g.k; i++) p[i] = g.reqs[t]->present[i] ? 1 : 0;
      }
    }
  }
}

void copy_in(const AxisReq* r, uint8_t* h) {
  if (r->kind == kDec) {  // the present shards only: the decoder overwrites the rest
    for (uint32_t i = 0; i < 2 * r->k; i++)
      if (r->present[i]) memcpy(h + r->off + (size_t)i * r->len, r->in + (size_t)i * r->len, r->len);
  } else {
    memcpy(h + r->off, r->in, r->in_bytes());
  }
}

void copy_out(AxisReq* r, const uint8_t* h) {
  if (r->kind == kEnc) {
    memcpy(r->out, h + r->out_off, (size_t)r->k * r->len);
  } else if (r->kind == kDec) {
    for (uint32_t i = 0; i < 2 * r->k; i++)
      if (!r->present[i]) memcpy(r->out + (size_t)i * r->len, h + r->off + (size_t)i * r->len, r->len);
  } else {
    memcpy(r->rec, h + r->out_off, CDA_REC_BYTES);
    memcpy(&r->st, h + r->st_off, 8);
  }
}

int code_of(int lr) { return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE; }

// The batch on the device: one launch per group on the slot's stream, reading and writing the page-locked staging
// itself (zero-copy: a batch's bytes cross the link once each way, with no DMA submissions), then one
// synchronisation of that stream.  The context lock is held only while launching (profiling events, error text),
// not while the kernels run, so other slots' batches and the block path proceed meanwhile.  A group the kernels do
// not support (-2) fails alone with CDA_E_UNSUPPORTED; a runtime failure fails the batch with CDA_E_DEVICE.
int run_device(cda_ctx* c, const Layout& L, AxisSlot* sl) {
  (void)hipSetDevice(c->device);
  hipStream_t s = sl->s;
  uint8_t* D = sl->hd;
  int rc = CDA_OK;
  {
    Lock l(c);
    for (const Group& g : L.groups) {
      const int n = (int)g.reqs.size();
      int lr = 0;
      if (g.kind == kEnc) {
        RsJob j{};
        j.src = D + g.in0;
        j.src_cw = (long long)g.item_in;
        j.src_sh = g.len;
        j.dst = D + g.out0;
        j.dst_cw = (long long)g.item_out;
        j.dst_sh = g.len;
        j.k = (int)g.k;
        j.cw_per_blk = n;
        j.nblk = 1;
        j.shard_len = (int)g.len;
        const bool ff8 = 2 * g.k <= 256;
        ProfScope ps(c, ff8 ? "axis_rs_encode8" : "axis_rs_encode16", s);
        lr = ff8 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s);
      } else if (g.kind == kRoot) {
        ProfScope ps(c, "axis_roots", s);
        lr = launch_axis_roots(D + g.in0, (long long)g.item_in, (int)g.n, g.ss,
                               (const unsigned long long*)(D + g.desc0), n, D + g.out0,
                               (unsigned long long*)(D + g.st0), s);
      } else {
        ProfScope ps(c, "axis_rs_decode", s);
        const uint8_t* d = D + g.desc0;
        lr = launch_rs_decode(D, (const long long*)d, (const long long*)(d + 8 * (size_t)n), d + 16 * (size_t)n, n,
                              (int)g.k, (int)g.len, s);
      }
      if (lr == -2) {
        for (AxisReq* r : g.reqs) r->rc = CDA_E_UNSUPPORTED;
      } else if (lr) {
        c->last_err = std::string("axis launch: ") + hipGetErrorString(hipGetLastError());
        rc = code_of(lr);
        break;
      }
    }
  }
  // always drained, also after a failed launch: earlier launches of the batch may still read the staging
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess || c->prof) {
    Lock l(c);
    if (e != hipSuccess) {
      dev_ok(c, e, "sync");
      rc = CDA_E_DEVICE;
    }
    flush_profile(c);
  }
  return rc;
}

void free_host(AxisSlot* sl) {
  if (!sl->h) return;
  (void)hipHostUnregister(sl->h);
  free(sl->h);
  sl->h = sl->hd = nullptr;
  sl->cap = 0;
}

// The slot's stream (created on first use) and at least `bytes` of staging (`hint`: the size to grow to at least).
bool ensure_slot(cda_ctx* c, AxisSlot* sl, size_t bytes, size_t hint, size_t limit) {
  (void)hipSetDevice(c->device);
  if (!sl->s && hipStreamCreateWithFlags(&sl->s, hipStreamNonBlocking) != hipSuccess) {
    sl->s = nullptr;
    (void)hipGetLastError();
    return false;
  }
  if (sl->cap >= bytes) return true;
  const size_t cap =
      (std::max({bytes, hint, std::min((size_t)4 << 20, limit), std::min(2 * sl->cap, limit)}) + 4095) & ~(size_t)4095;
  free_host(sl);
  void* p = nullptr;
  void* d = nullptr;
  // page-aligned host memory page-locked by registration (coarse-grained): coherent at the points this queue uses it
  // -- the callers write a batch's inputs before its kernels are launched and read its results after the stream is
  // synchronised.  (Registered rather than fine-grained hipHostMalloc memory: one Encode 31.0 -> 29-30 us, DESIGN
  // §12.7.)
  if (posix_memalign(&p, 4096, cap) != 0) return false;
  if (hipHostRegister(p, cap, hipHostRegisterDefault) != hipSuccess) {
    free(p);
    (void)hipGetLastError();
    return false;
  }
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
    (void)hipHostUnregister(p);
    free(p);
    (void)hipGetLastError();
    return false;
  }
  sl->h = (uint8_t*)p;
  sl->hd = (uint8_t*)d;
  sl->cap = cap;
  return true;
}

AxisSlot* free_slot(AxisQueue* q) {
  for (int i = 0; i < q->nslots; i++)
    if (!q->slot[i].busy) return &q->slot[i];
  return nullptr;
}

// A slot is free again (or a leader gave up): the owner of the oldest queued request, if any, leads the next batch.
void hand_over(AxisQueue* q) {
  if (!q->pending.empty()) q->pending.front()->cv.notify_one();
}

// Runs one batch as its leader on slot `sl`: `self` (queued, in q->pending) and whatever else is queued.  lk is held
// on entry and on return.  Every request of the batch is kDone when it returns, and the slot is free again.
void lead(cda_ctx* c, AxisQueue* q, std::unique_lock<std::mutex>& lk, AxisReq* self, AxisSlot* sl) {
  sl->busy = true;
  std::vector<AxisReq*> batch, rest;
  Layout L;
  int fail = CDA_OK;
  try {  // nothing below changes the queue until it has succeeded (an allocation failure leaves it as it was)
    batch.reserve(q->pending.size());
    rest.reserve(q->pending.size());
    size_t bytes = 0;
    for (AxisReq* r : q->pending) {
      if (batch.empty() || bytes + r->bytes() <= q->batch_bytes || r == self) {
        batch.push_back(r);
        bytes += r->bytes();
      } else {
        rest.push_back(r);
      }
    }
    plan(batch, L);
  } catch (...) {
    fail = CDA_E_NOMEM;
  }
  if (!fail && (!sl->s || sl->cap < L.total)) {
    // The slot's stream or staging is set up without the queue lock (registering tens of MiB takes milliseconds,
    // and every other caller needs the lock to move on); the batch's requests leave the queue meanwhile (kTaken).
    q->pending.swap(rest);
    for (AxisReq* r : batch) r->state = kTaken;
    q->largest = std::max(q->largest, L.total);
    const size_t hint = std::min(q->largest, q->batch_bytes);
    lk.unlock();
    bool ok = false;
    try {
      ok = ensure_slot(c, sl, L.total, hint, q->batch_bytes);
    } catch (...) {
    }
    lk.lock();
    if (!ok) {  // only this caller's request fails; the others go back to the head of the queue, in order
      fail = CDA_E_NOMEM;
      std::vector<AxisReq*> back;
      for (AxisReq* r : batch)
        if (r != self) r->state = kQueued, back.push_back(r);
      q->pending.insert(q->pending.begin(), back.begin(), back.end());
    }
    rest = q->pending;  // requests queued meanwhile stay queued
  }
  if (fail) {
    q->pending.erase(std::remove(q->pending.begin(), q->pending.end(), self), q->pending.end());
    self->rc = fail;
    self->state = kDone;
    sl->busy = false;
    hand_over(q);
    return;
  }
  q->pending.swap(rest);
  sl->copy_left = batch.size();
  for (AxisReq* r : batch) {
    r->slot = sl;
    r->state = kCopyIn;
    if (r != self) r->cv.notify_one();
  }
  if (!q->pending.empty() && free_slot(q)) hand_over(q);  // requests this batch could not take may lead another
  lk.unlock();
  fill_desc(L, sl->h);
  copy_in(self, sl->h);
  lk.lock();
  self->state = kCopied;
  sl->copy_left--;
  while (sl->copy_left > 0) sl->lead_cv.wait(lk);
  lk.unlock();
  int rc;
  try {
    rc = run_device(c, L, sl);
  } catch (...) {
    rc = api_exception(c);
  }
  lk.lock();
  sl->out_left = batch.size();
  for (AxisReq* r : batch) {
    if (r->rc == CDA_OK) r->rc = rc;
    r->state = kResult;
    if (r != self) r->cv.notify_one();
  }
  lk.unlock();
  if (self->rc == CDA_OK) copy_out(self, sl->h);
  lk.lock();
  self->state = kDone;
  sl->out_left--;
  while (sl->out_left > 0) sl->lead_cv.wait(lk);
  sl->busy = false;
  hand_over(q);
}

AxisQueue* queue_of(cda_ctx* c) {
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (!c->axq) {
    c->axq = new AxisQueue();
    if (const char* e = CDA_AB_ENV("CDA_AXIS_SLOTS")) c->axq->nslots = std::max(1, std::min(kMaxSlots, atoi(e)));
    c->axq->batch_bytes = kBatchBytes / c->axq->nslots;
  }
  return c->axq;
}

// Queues r and returns its rc once its batch has run (this thread may lead that batch itself).
int submit(cda_ctx* c, AxisReq* r) {
  AxisQueue* q = queue_of(c);
  std::unique_lock<std::mutex> lk(q->mu);
  q->pending.push_back(r);
  for (;;) {
    if (r->state == kDone) return r->rc;
    if (r->state == kCopyIn) {
      AxisSlot* sl = r->slot;
      lk.unlock();
      copy_in(r, sl->h);
      lk.lock();
      r->state = kCopied;
      if (--sl->copy_left == 0) sl->lead_cv.notify_one();
      continue;
    }
    if (r->state == kResult) {
      AxisSlot* sl = r->slot;
      lk.unlock();
      if (r->rc == CDA_OK) copy_out(r, sl->h);
      lk.lock();
      r->state = kDone;
      if (--sl->out_left == 0) sl->lead_cv.notify_one();
      return r->rc;
    }
    if (r->state == kQueued) {
      if (AxisSlot* sl = free_slot(q)) {
        lead(c, q, lk, r, sl);
        continue;
      }
    }
    r->cv.wait(lk);
  }
}

constexpr uint8_t kEmptySha[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                   0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                   0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

// Trees wider than one workgroup's LDS (n > kAxisRootsMaxLeaves, squares beyond the device block path): leaf launch
// plus one launch per level, on the caller's thread.
int axis_root_wide(cda_ctx* c, uint64_t square_size, uint64_t axis_index, uint32_t n, const uint8_t* leaves,
                   uint8_t* rec, uint64_t* st) {
  Lock l(c);
  const size_t in_b = (size_t)n * CDA_SHARE, rec_b = (size_t)n * CDA_REC_BYTES;
  int rc;
  if ((rc = ensure(c, c->ods, in_b)) || (rc = ensure(c, c->leaf, rec_b)) || (rc = ensure(c, c->scratch, rec_b)) ||
      (rc = ensure(c, c->status, 8)))
    return rc;
  hipStream_t s = c->stream;
  if (!dev_ok(c, hipMemcpyAsync(c->ods.p, leaves, in_b, hipMemcpyHostToDevice, s), "H2D") ||
      !dev_ok(c, hipMemsetAsync(c->status.p, 0xFF, 8, s), "memset"))
    return CDA_E_DEVICE;
  {
    ProfScope ps(c, "axis_leaf", s);
    if (launch_axis_leaf((const uint8_t*)c->ods.p, (int)n, square_size, axis_index, c->leaf.p,
                         (unsigned long long*)c->status.p, s))
      return CDA_E_DEVICE;
  }
  void* bufs[2] = {c->leaf.p, c->scratch.p};
  int cur = 0;
  for (uint32_t cnt = n; cnt > 1; cnt = (cnt + 1) / 2) {
    ProfScope ps(c, "nmt_level_generic", s);
    if (launch_level_generic(bufs[cur], bufs[cur ^ 1], (int)cnt, s)) return CDA_E_DEVICE;
    cur ^= 1;
  }
  if (!dev_ok(c, hipMemcpyAsync(rec, bufs[cur], CDA_REC_BYTES, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipMemcpyAsync(st, c->status.p, 8, hipMemcpyDeviceToHost, s), "D2H") ||
      !dev_ok(c, hipStreamSynchronize(s), "sync"))
    return CDA_E_DEVICE;
  flush_profile(c);
  return CDA_OK;
}

}  // namespace

void free_axisq(cda_ctx* c) {
  if (!c->axq) return;
  for (AxisSlot& sl : c->axq->slot) {
    if (sl.s) {
      (void)hipStreamSynchronize(sl.s);
      (void)hipStreamDestroy(sl.s);
    }
    free_host(&sl);
  }
  delete c->axq;
  c->axq = nullptr;
}

}  // namespace cda

using namespace cda;

extern "C" {

int cda_rs_encode(cda_ctx* c, uint32_t k, uint32_t shard_len, const uint8_t* data, uint8_t* parity) {
  CDA_API_TRY
  if (!c || !data || !parity || k == 0 || k > 32768) return CDA_E_ARG;
  if (cda_rs_validate_chunk_size(shard_len)) return CDA_E_SHARD_SIZE;
  AxisReq r;
  r.kind = kEnc;
  r.k = k;
  r.len = shard_len;
  r.in = data;
  r.out = parity;
  return submit(c, &r);
  CDA_API_CATCH(c)
}

int cda_rs_decode(cda_ctx* c, uint32_t k, uint32_t shard_len, uint8_t* shards, const uint8_t* present) {
  CDA_API_TRY
  if (!c || !shards || !present || k == 0 || k > 32768) return CDA_E_ARG;
  if (cda_rs_validate_chunk_size(shard_len)) return CDA_E_SHARD_SIZE;
  uint32_t np = 0;
  for (uint32_t i = 0; i < 2 * k; i++) np += present[i] ? 1 : 0;
  if (np < k) return CDA_E_TOO_FEW;
  if (np == 2 * k) return CDA_OK;
  AxisReq r;
  r.kind = kDec;
  r.k = k;
  r.len = shard_len;
  r.in = shards;
  r.out = shards;
  r.present = present;
  return submit(c, &r);
  CDA_API_CATCH(c)
}

int cda_nmt_axis_root(cda_ctx* c, uint64_t square_size, uint64_t axis_index, uint32_t n, uint32_t leaf_len,
                      const uint8_t* leaves, uint8_t* root, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !root || (n && !leaves) || square_size == 0) return CDA_E_ARG;
  // ErasuredNamespacedMerkleTree.Push checks (nmt_wrapper.go:94-99) happen leaf by leaf in the
  // reference, before nmt's order check of the same leaf: the bounds check fails first at leaf 0
  // (axis index out of range) or at leaf 2k (pushed past the square), the namespace-length check at
  // leaf 0.  An order violation at a leaf j < 2k therefore wins over a push past the square; the
  // device pass below only looks at the leaves the reference would have accepted.
  if (n > 0 && axis_index + 1 > 2 * square_size)
    return set_err(err, CDA_E_PUSH_PAST, -1, (int)axis_index, 0, -1), CDA_E_PUSH_PAST;
  if (n > 0 && leaf_len < CDA_NAMESPACE_SIZE)
    return set_err(err, CDA_E_NS_SHORT, -1, (int)axis_index, 0, -1), CDA_E_NS_SHORT;
  const uint64_t push_limit = 2 * square_size;
  const bool past = (uint64_t)n > push_limit;
  if (past) n = (uint32_t)push_limit;
  if (n == 0) {  // EmptyRoot: 0x00*58 ‖ SHA256("")
    memset(root, 0, 58);
    memcpy(root + 58, kEmptySha, 32);
    return CDA_OK;
  }
  if (leaf_len != CDA_SHARE) return CDA_E_UNSUPPORTED;
  uint8_t rec[CDA_REC_BYTES];
  uint64_t st = ~0ull;
  int rc;
  if (n <= (uint32_t)kAxisRootsMaxLeaves) {
    AxisReq r;
    r.kind = kRoot;
    r.n = n;
    r.len = leaf_len;
    r.square_size = square_size;
    r.axis_index = axis_index;
    r.in = leaves;
    rc = submit(c, &r);
    memcpy(rec, r.rec, CDA_REC_BYTES);
    st = r.st;
  } else {
    rc = axis_root_wide(c, square_size, axis_index, n, leaves, rec, &st);
  }
  if (rc) return rc;
  if (st != ~0ull) return set_err(err, CDA_E_NS_ORDER, -1, (int)axis_index, (int)st, -1), CDA_E_NS_ORDER;
  if (past) return set_err(err, CDA_E_PUSH_PAST, -1, (int)axis_index, (int)push_limit, -1), CDA_E_PUSH_PAST;
  memcpy(root, rec, CDA_NODE_SIZE);
  return CDA_OK;
  CDA_API_CATCH(c)
}

}  // extern "C"
