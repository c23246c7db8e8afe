// repair.cpp — rsmt2d (*ExtendedDataSquare).Repair on the GPU: cda_repair (caller square in host memory)
// and cda_repair_device (square already in HBM).  The decodes are rs_decode.hip's, the root checks
// nmt_kernels.hip's axes_verify_kernel, the copies of caller memory staging.cpp's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ctx.h"
#include "plan.h"

using namespace cda;

// pinned host buffer (hipHostMalloc), grown like ensure()
static int ensure_host(cda_ctx* c, cda_ctx::Buf& b, size_t bytes) {
  if (b.cap >= bytes) return CDA_OK;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  if (!dev_ok(c, hipHostMalloc(&b.p, bytes ? bytes : 16, hipHostMallocDefault), "hipHostMalloc")) return CDA_E_DEVICE;
  b.cap = bytes;
  return CDA_OK;
}

// rsmt2d (*ExtendedDataSquare).Repair (v0.12.0, upstream):
//   prerepairSanityCheck: every complete row/col must match its root and
//     re-encode to its parity (ErrByzantineData otherwise);
//   solveCrossword: sweeps of "row i, then col i" for i = 0..w-1; an incomplete
//     axis with >= k shares is decoded, its root and the roots of orthogonal
//     axes it completes are verified, then its cells are inserted; a sweep
//     without progress is ErrUnrepairableDataSquare.
// The host replays exactly that order on presence bitsets (control only), for
// every sweep up front as if all checks pass, and the GPU runs every decode /
// root / re-encode: consecutive operations already decodable at the batch start
// form a batch, all batches are enqueued at once (decodes in order on one
// stream, each batch's root check on another), and the host waits once.  The
// first batch with a failing root check is replayed one operation at a time
// (see below), so a Byzantine report and the square left "most repaired prior
// to the Byzantine axis" are exactly the sequential reference's.
using plan::enc_axis;
using plan::Presence;

// Repair of the square in host memory `eds` (uploaded, repaired, copied back) or, when eds is null,
// of the square already in device memory d_eds_in; the caller holds the lock for stream s.
// CDA_REPAIR_TRACE=1: host-side phase times of each repair on stderr (where a slow host-buffer repair spends it)
struct RepairTrace {
  bool on = false;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
  std::string line;
  RepairTrace() {
    static const bool env = CDA_AB_ENV("CDA_REPAIR_TRACE") && atoi(CDA_AB_ENV("CDA_REPAIR_TRACE")) != 0;
    on = env;
  }
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    char b[64];
    snprintf(b, sizeof b, " %s=%.0f", what, std::chrono::duration<double, std::micro>(now - last).count());
    line += b;
    last = now;
  }
  ~RepairTrace() {
    if (on)
      fprintf(stderr, "cda_repair trace (us):%s total=%.0f\n", line.c_str(),
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
};

static int repair_impl(cda_ctx* c, uint32_t k, uint8_t* eds, uint8_t* d_eds_in, uint8_t* present,
                       const uint8_t* row_roots, const uint8_t* col_roots, cda_err_info* err, hipStream_t s) {
  const int w = (int)(2 * k), K = (int)k;
  const size_t ncell = (size_t)w * w, eds_b = ncell * CDA_SHARE;
  int rc;
  // Generic verification workspace (sequential replay, CDA_REPAIR_FUSED=0): leaf / level records
  // for up to 4w trees.  Repair descriptors (device, staged in pinned host memory at the same
  // offsets): an operation completes an axis, so a repair has at most 2w operations, 4w verified
  // axes (each axis is its own operation's and at most one other operation's orthogonal
  // completion) and 2w batches.
  //   off[2w] | stride[2w] | pres[2w][w] | vaxes[4w] | sanity axes[2w] | all axes[2w]
  //   | batch flags[2w] | sanity root flags[2w] | parity flags[2w]      (after the 2w x 90 B roots)
  const size_t trees_cap = (size_t)4 * w, W = (size_t)w;
  const size_t want_b = (2 * W * CDA_NODE_SIZE + 255) & ~(size_t)255;
  const size_t o_off = 0, o_str = o_off + 2 * W * 8, o_pres = o_str + 2 * W * 8, o_ax = o_pres + 2 * W * W,
               o_sax = o_ax + 4 * W * 4, o_all = o_sax + 2 * W * 4, o_bfl = o_all + 2 * W * 4,
               o_sfl = o_bfl + 2 * W * 4, o_pfl = o_sfl + 2 * W * 4, desc_b = o_pfl + 2 * W * 4;
  if ((eds && (rc = ensure(c, c->eds, eds_b))) || (rc = ensure(c, c->ods, eds_b)) ||
      (rc = ensure(c, c->leaf, trees_cap * w * CDA_REC_BYTES)) ||
      (rc = ensure(c, c->scratch, trees_cap * w * CDA_REC_BYTES)) ||
      (rc = ensure(c, c->roots, trees_cap * CDA_REC_BYTES)) || (rc = ensure(c, c->status, trees_cap * 8 + 64)) ||
      (rc = ensure(c, c->dah, trees_cap * (16 + W) + 64)) || (rc = ensure(c, c->rdesc, want_b + desc_b)) ||
      (rc = ensure_host(c, c->rstage, desc_b)))
    return rc;
  uint8_t* d_eds = eds ? (uint8_t*)c->eds.p : d_eds_in;
  uint8_t* d_par = (uint8_t*)c->ods.p;
  const uint8_t* d_want = (const uint8_t*)c->rdesc.p;
  uint8_t* h = (uint8_t*)c->rstage.p;
  uint8_t* dd = (uint8_t*)c->rdesc.p + want_b;
  unsigned* d_bfl = (unsigned*)(dd + o_bfl);
  const unsigned* bfl = (const unsigned*)(h + o_bfl);
  const unsigned* sfl = (const unsigned*)(h + o_sfl);
  const unsigned* pfl = (const unsigned*)(h + o_pfl);
  Presence P;
  P.init(w, present);
  // The EDS upload (pageable memory: the copy occupies the calling thread) runs on a helper thread while this
  // one plans the whole repair on the presence bitsets.  A sparse square (e.g. Q0 only: 25 % of the bytes) goes
  // up as its runs of present cells only (gaps of < 8 missing cells are sent along), packed through the pinned
  // ring into rcompact and scattered into place on the device; its missing cells are zeroed there first, so a
  // failed repair hands back zeros, not a previous square's bytes, in the cells it could not fill.
  std::vector<HostRun> runs;
  std::vector<uint32_t> run_tab;  // dst cell of each run, then the packed prefix (nruns + 1)
  size_t packed_cells = 0;
  if (eds) {
    constexpr uint32_t kGap = 8;
    const uint32_t ncells = (uint32_t)(W * W);
    std::vector<std::pair<uint32_t, uint32_t>> cr;  // (first cell, cells)
    size_t npresent = 0;
    for (int r = 0; r < w; r++) npresent += P.cnt[CDA_AXIS_ROW][r];
    // runs of present cells in row-major order, word by word; a gap of < kGap cells joins two runs
    for (int r = 0; r < w && npresent * 4 <= (size_t)ncells * 3 && cr.size() <= (1u << 16); r++) {
      const uint64_t* b = P.bits[CDA_AXIS_ROW].data() + (size_t)r * P.words;
      for (int wd = 0; wd < P.words; wd++) {
        uint64_t m = b[wd] & P.full;
        while (m) {
          const int lo = __builtin_ctzll(m);
          const uint64_t above = ~m >> lo;  // the run of set bits starting at lo
          const int len = above ? __builtin_ctzll(above) : 64 - lo;
          const uint32_t g0 = (uint32_t)r * w + wd * 64 + lo;
          if (!cr.empty() && g0 - (cr.back().first + cr.back().second) < kGap)
            cr.back().second = g0 + len - cr.back().first;
          else
            cr.emplace_back(g0, (uint32_t)len);
          m = lo + len >= 64 ? 0 : m & (~0ull << (lo + len));
        }
      }
    }
    for (auto& x : cr) packed_cells += x.second;
    if (npresent * 4 <= (size_t)ncells * 3 && packed_cells * 4 <= (size_t)ncells * 3 && cr.size() <= (1u << 16)) {
      runs.reserve(cr.size());
      run_tab.resize(2 * cr.size() + 1);
      uint32_t pre = 0;
      for (size_t i = 0; i < cr.size(); i++) {
        runs.push_back(HostRun{(size_t)cr[i].first * CDA_SHARE, (size_t)cr[i].second * CDA_SHARE});
        run_tab[i] = cr[i].first;
        run_tab[cr.size() + i] = pre;
        pre += cr[i].second;
      }
      run_tab[2 * cr.size()] = pre;
    } else {
      packed_cells = 0;
    }
  }
  const bool packed = !runs.empty();
  // a sparse square in page-locked memory (go/cda's pooled slab, cda_host_register): the scatter kernel reads its
  // present runs over PCIe itself -- no host copy through the staging ring, no upload ahead of the planning
  const void* zc = packed ? pinned_device_alias(eds, eds_b) : nullptr;
  if (packed) {
    if ((!zc && (rc = ensure(c, c->rcompact, packed_cells * CDA_SHARE))) ||
        (rc = ensure(c, c->rruns, run_tab.size() * 4)))
      return rc;
    if (!dev_ok(c, hipMemcpyAsync(c->rruns.p, run_tab.data(), run_tab.size() * 4, hipMemcpyHostToDevice, s), "H2D") ||
        !dev_ok(c, hipMemsetAsync(d_eds, 0, eds_b, s), "memset"))
      return CDA_E_DEVICE;
  }
  bool h2d_ok = true;
  std::thread h2d;
  if (eds && !zc)
    h2d = std::thread([&] {
      try {
        (void)hipSetDevice(c->device);
        bind_helper_thread(c);
        h2d_ok = (packed ? staged_h2d_runs(c, c->rcompact.p, eds, runs.data(), runs.size(), s)
                         : staged_h2d(c, d_eds, eds, eds_b, s)) == CDA_OK;
      } catch (...) {  // nothing may escape a helper thread (std::terminate)
        (void)api_exception(c);
        h2d_ok = false;
      }
    });
  struct Joiner {  // an early return or exception: the upload finishes before the caller's buffer is released
    std::thread& t;
    hipStream_t s;
    ~Joiner() {
      if (!t.joinable()) return;
      t.join();
      (void)hipStreamSynchronize(s);
    }
  } joiner{h2d, s};
  RepairTrace tr;
  tr.mark("setup");
  const uint8_t* want[2] = {row_roots, col_roots};

  // ---- plan: prerepairSanityCheck axes, then every crossword sweep on the optimistic presence (plan.cpp) ----
  plan::RepairPlan rp;
  if ((rc = plan::plan_repair(P, K, rp, h + o_pres))) return rc;
  const std::vector<int>& sane = rp.sane;
  const std::vector<plan::RepairOp>& ops = rp.ops;
  const std::vector<plan::RepairBatch>& bat = rp.bat;
  const std::vector<int>& vall = rp.vall;
  const std::vector<int>& blast = rp.blast;  // rows go back to the caller once their last writer has run
  const bool solved = rp.solved;
  for (size_t q = 0; q < ops.size(); q++) {
    const plan::RepairOp& op = ops[q];
    ((long long*)(h + o_off))[q] =
        op.axis == CDA_AXIS_ROW ? (long long)op.idx * w * CDA_SHARE : (long long)op.idx * CDA_SHARE;
    ((long long*)(h + o_str))[q] = op.axis == CDA_AXIS_ROW ? CDA_SHARE : (long long)w * CDA_SHARE;
  }
  const size_t nbat = bat.size();
  const bool early = eds && !c->prof && nbat > 0 && c->repair_early;
  std::vector<hipEvent_t> bev(early ? nbat : 0, nullptr);
  struct EventsGuard {
    std::vector<hipEvent_t>& v;
    ~EventsGuard() {
      for (auto e : v)
        if (e) (void)hipEventDestroy(e);
    }
  } events_guard{bev};
  for (int r = 0; r < w && early; r++)
    if (blast[r] >= 0 && !bev[blast[r]] &&
        !dev_ok(c, hipEventCreateWithFlags(&bev[blast[r]], hipEventDisableTiming), "hipEventCreate"))
      return CDA_E_DEVICE;
  memcpy(h + o_ax, vall.data(), vall.size() * 4);
  memcpy(h + o_sax, sane.data(), sane.size() * 4);
  for (int i = 0; i < w; i++) {
    ((int*)(h + o_all))[i] = enc_axis(CDA_AXIS_ROW, i);
    ((int*)(h + o_all))[w + i] = enc_axis(CDA_AXIS_COL, i);
  }
  tr.mark("plan");
  fault_point("thread");
  if (h2d.joinable()) h2d.join();
  tr.mark("h2d_wait");
  if (!h2d_ok) {
    c->last_err = "H2D failed";
    return CDA_E_DEVICE;
  }
  if (packed) {
    const uint32_t* d_tab = (const uint32_t*)c->rruns.p;
    const int nr = (int)runs.size();
    if (launch_scatter_cell_runs(zc ? zc : c->rcompact.p, d_eds, d_tab, d_tab + nr, nr, (uint32_t)packed_cells, s,
                                 zc != nullptr))
      return CDA_E_DEVICE;
  }
  const int* d_ax = (const int*)(dd + o_ax);
  const int* d_sax = (const int*)(dd + o_sax);
  const int* d_all = (const int*)(dd + o_all);
  if (!dev_ok(c, hipMemcpyAsync(c->rdesc.p, row_roots, W * CDA_NODE_SIZE, hipMemcpyHostToDevice, s), "H2D") ||
      !dev_ok(c, hipMemcpyAsync((uint8_t*)c->rdesc.p + W * CDA_NODE_SIZE, col_roots, W * CDA_NODE_SIZE,
                                hipMemcpyHostToDevice, s),
              "H2D") ||
      !dev_ok(c, hipMemcpyAsync(dd, h, o_bfl, hipMemcpyHostToDevice, s), "H2D") ||
      !dev_ok(c, hipMemsetAsync(d_bfl, 0xFF, 2 * W * 4, s), "memset") ||
      !dev_ok(c, hipMemsetAsync(dd + o_sfl, 0, 4 * W * 4, s), "memset"))
    return CDA_E_DEVICE;

  // GPU roots of a list of axes -> host records (sequential replay and the generic sanity path)
  std::vector<uint8_t> recs;
  std::vector<uint64_t> st;
  auto roots_of = [&](const std::vector<int>& axes) -> int {
    if (axes.empty()) return CDA_OK;
    if (axes.size() > trees_cap) return CDA_E_ARG;
    int* d_axes = (int*)c->dah.p;
    if (!dev_ok(c, hipMemcpyAsync(d_axes, axes.data(), axes.size() * 4, hipMemcpyHostToDevice, s), "H2D") ||
        !dev_ok(c, hipMemsetAsync(c->status.p, 0xFF, axes.size() * 8, s), "memset"))
      return CDA_E_DEVICE;
    {
      ProfScope ps(c, "repair_roots", s);
      if (launch_axes_roots(d_eds, K, d_axes, 0, (int)axes.size(), 0, w, c->leaf.p, c->scratch.p, c->roots.p,
                            (unsigned long long*)c->status.p, s))
        return CDA_E_DEVICE;
    }
    recs.resize(axes.size() * CDA_REC_BYTES);
    st.resize(axes.size());
    if (!dev_ok(c, hipMemcpyAsync(recs.data(), c->roots.p, recs.size(), hipMemcpyDeviceToHost, s), "D2H") ||
        !dev_ok(c, hipMemcpyAsync(st.data(), c->status.p, st.size() * 8, hipMemcpyDeviceToHost, s), "D2H") ||
        !dev_ok(c, hipStreamSynchronize(s), "sync"))
      return CDA_E_DEVICE;
    return CDA_OK;
  };
  auto root_ok = [&](size_t t, int axis_code) {
    const int axis = axis_code >> 24, idx = axis_code & 0xFFFFFF;
    if (st[t] != ~0ull) return false;  // push error => byzantine
    return memcmp(recs.data() + t * CDA_REC_BYTES, want[axis] + (size_t)idx * CDA_NODE_SIZE, CDA_NODE_SIZE) == 0;
  };
  std::thread early_d2h;
  bool early_ok = false, early_failed = false;  // the early rows are the answer / the copier hit an error
  struct EarlyJoiner {
    std::thread& t;
    ~EarlyJoiner() {
      if (t.joinable()) t.join();
    }
  } early_joiner{early_d2h};
  auto finish = [&](int code, int axis, int idx) -> int {
    tr.mark("evaluate");
    if (early_d2h.joinable()) early_d2h.join();
    tr.mark("early_join");
    if (eds && !(early_ok && !early_failed)) {
      const int r2 = staged_d2h(c, eds, d_eds, eds_b, s);
      if (r2) return r2;
    }
    for (int r = 0; r < w; r++) P.bytes(CDA_AXIS_ROW, r, present + (size_t)r * w);
    if (!dev_ok(c, hipStreamSynchronize(s), "sync")) return CDA_E_DEVICE;
    tr.mark("final_d2h");
    flush_profile(c);
    if (code != CDA_OK) set_err(err, code, axis, idx, -1, -1);
    return code;
  };
  // Verification streams.  Decodes run in order on `s`; batch b's verification runs after decode b
  // on a second stream, overlapping decode b+1 (which writes only cells missing after batch b, and
  // every axis batch b verifies is complete after it).  The fused kernel keeps its trees in LDS, so
  // batches verify concurrently on 2 streams; the generic path shares the leaf / level workspace.
  // (aux_stream and h2d_stream sit on hardware queues of their own, see ctx.h; the rows going back
  // early use d2h_stream.)
  const int nvs = c->repair_overlap ? (c->repair_fused_verify ? 2 : 1) : 0;
  hipStream_t vs[2] = {c->aux_stream, c->h2d_stream};
  auto vstream = [&](size_t b) { return nvs ? vs[b % nvs] : s; };
  auto fork = [&](hipStream_t v) {
    return v == s || (dev_ok(c, hipEventRecord(c->fork_ev, s), "event") &&
                      dev_ok(c, hipStreamWaitEvent(v, c->fork_ev, 0), "wait"));
  };
  auto join = [&]() {
    for (int i = 0; i < nvs; i++)
      if (!dev_ok(c, hipEventRecord(c->join_ev[i], vs[i]), "event") ||
          !dev_ok(c, hipStreamWaitEvent(s, c->join_ev[i], 0), "wait"))
        return false;
    return true;
  };

  // ---- prerepairSanityCheck, enqueued: every complete row / column must match its root and
  // re-encode to its own parity.  Crossword decodes write only missing cells, never a cell of a
  // complete axis, so the check runs concurrently with them; it is evaluated first afterwards. ----
  std::vector<uint8_t> san_bad(sane.size(), 0);
  if (!sane.empty()) {
    if (!c->repair_fused_verify) {  // generic: roots through the workspace, compared on the host
      if ((rc = roots_of(sane))) return rc;
      for (size_t t = 0; t < sane.size(); t++) san_bad[t] = root_ok(t, sane[t]) ? 0 : 1;
    }
    hipStream_t v = vstream(0);
    if (!fork(v)) return CDA_E_DEVICE;
    if (c->repair_fused_verify) {
      ProfScope ps(c, "repair_roots", v);
      if (launch_axes_verify(d_eds, K, d_sax, (int)sane.size(), d_want, d_want + W * CDA_NODE_SIZE,
                             (unsigned*)(dd + o_sfl), 0, true, v))
        return CDA_E_DEVICE;
    }
    for (int axis = 0; axis < 2; axis++) {  // re-encode every row and column data half
      RsJob j{};
      j.src = d_eds;
      j.src_cw = axis == CDA_AXIS_ROW ? (long long)w * CDA_SHARE : CDA_SHARE;
      j.src_sh = axis == CDA_AXIS_ROW ? CDA_SHARE : (long long)w * CDA_SHARE;
      j.dst = d_par + (size_t)axis * w * K * CDA_SHARE;
      j.dst_cw = (long long)K * CDA_SHARE;
      j.dst_sh = CDA_SHARE;
      j.k = K;
      j.cw_per_blk = w;
      j.nblk = 1;
      j.shard_len = CDA_SHARE;
      ProfScope ps(c, "repair_reencode", v);
      const int lr = 2 * K <= 256 ? launch_rs_encode8(j, v) : launch_rs_encode16(j, v);
      if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
      if (launch_parity_compare(d_eds, K, d_all + axis * w, w, j.dst, (unsigned*)(dd + o_pfl) + axis * w, v))
        return CDA_E_DEVICE;
    }
  }

  // ---- solveCrossword, optimistic: every batch as if all checks pass, one wait at the end ----
  // A batch whose every root check passes equals the sequential rsmt2d run: each checked axis then
  // holds its committed values, so every decode saw only true shares and the sequential decode
  // (with more shares) gives the same bytes.  Presence only grows and a decode writes only cells
  // missing in its own presence, so work enqueued after a failing batch never writes a cell that
  // batch (or an earlier one) reads: the device state at the first failing batch's start is
  // intact, and that batch is replayed one operation at a time with the presence each operation
  // sees in rsmt2d's order, so Byzantine reports (axis, index, the square repaired so far) are
  // exactly the sequential ones even when a row and a column of a batch write the same cell.
  auto enqueue_batches = [&](size_t from) -> int {
    for (size_t b = from; b < nbat; b++) {
      const plan::RepairBatch& bt = bat[b];
      {
        ProfScope ps(c, "repair_decode", s);
        const int lr = launch_rs_decode(d_eds, (const long long*)(dd + o_off) + bt.q0,
                                        (const long long*)(dd + o_str) + bt.q0, dd + o_pres + bt.q0 * W,
                                        (int)(bt.q1 - bt.q0), K, CDA_SHARE, s);
        if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
      }
      if (from == 0 && early && bev[b] && !dev_ok(c, hipEventRecord(bev[b], s), "hipEventRecord")) return CDA_E_DEVICE;
      hipStream_t v = vstream(b);
      if (!fork(v)) return CDA_E_DEVICE;
      const size_t nv = bt.v1 - bt.v0;
      if (c->repair_fused_verify) {
        ProfScope ps(c, "repair_roots", v);
        if (launch_axes_verify(d_eds, K, d_ax + bt.v0, (int)nv, d_want, d_want + W * CDA_NODE_SIZE, d_bfl + b, 0,
                               false, v))
          return CDA_E_DEVICE;
        continue;
      }
      for (size_t v0 = 0; v0 < nv; v0 += trees_cap) {  // chunks of at most trees_cap trees
        const int n = (int)std::min(trees_cap, nv - v0);
        if (!dev_ok(c, hipMemsetAsync(c->status.p, 0xFF, (size_t)n * 8, v), "memset")) return CDA_E_DEVICE;
        ProfScope ps(c, "repair_roots", v);
        if (launch_axes_roots(d_eds, K, d_ax + bt.v0 + v0, 0, n, 0, w, c->leaf.p, c->scratch.p, c->roots.p,
                              (unsigned long long*)c->status.p, v) ||
            launch_roots_check(c->roots.p, (const unsigned long long*)c->status.p, d_ax + bt.v0 + v0, n, d_want,
                               d_want + W * CDA_NODE_SIZE, d_bfl + b, (unsigned)v0, v))
          return CDA_E_DEVICE;
      }
    }
    if (!join() ||
        !dev_ok(c, hipMemcpyAsync(h + o_bfl, dd + o_bfl, o_pfl + 2 * W * 4 - o_bfl, hipMemcpyDeviceToHost, s),
                "D2H"))
      return CDA_E_DEVICE;
    return CDA_OK;
  };
  tr.mark("upload_rest");
  if ((rc = enqueue_batches(0))) return rc;
  tr.mark("enqueue");
  if (early)  // rows whose last writer has run go back on their own stream (pageable: from a helper thread)
    early_d2h = std::thread([&] {
      try {
        (void)hipSetDevice(c->device);
        bind_helper_thread(c);
        hipStream_t d2h = c->d2h_stream;
        const size_t row_b = W * CDA_SHARE;
        for (size_t b = 0; b < nbat && !early_failed; b++) {
          if (!bev[b]) continue;
          if (hipEventSynchronize(bev[b]) != hipSuccess) {
            early_failed = true;
            break;
          }
          for (int r = 0; r < w;) {  // runs of consecutive rows finished by batch b
            if (blast[r] != (int)b) {
              r++;
              continue;
            }
            int r1 = r;
            while (r1 < w && blast[r1] == (int)b) r1++;
            if (staged_d2h(c, eds + r * row_b, d_eds + r * row_b, (size_t)(r1 - r) * row_b, d2h) != CDA_OK)
              early_failed = true;
            r = r1;
          }
        }
        if (hipStreamSynchronize(d2h) != hipSuccess) early_failed = true;
      } catch (...) {
        (void)api_exception(c);
        early_failed = true;
      }
    });
  if (!dev_ok(c, hipStreamSynchronize(s), "sync")) return CDA_E_DEVICE;
  tr.mark("gpu_wait");
  {  // the early rows are the answer when the sanity check and every batch of this first pass passed
    bool all = true;
    for (size_t b = 0; b < nbat; b++) all = all && bfl[b] == ~0u;
    for (size_t t = 0; t < sane.size() && all; t++) all = c->repair_fused_verify ? sfl[t] == 0 : san_bad[t] == 0;
    for (int i = 0; i < 2 * w && all && !sane.empty(); i++)
      all = (i < w ? P.cnt[CDA_AXIS_ROW][i] : P.cnt[CDA_AXIS_COL][i - w]) != w || pfl[i] == 0;
    early_ok = early && all;
  }

  // sanity report in a fixed order: i ascending; row root, col root, row parity, col parity
  if (!sane.empty()) {
    std::vector<uint8_t> rbad(w, 0), cbad(w, 0);
    for (size_t t = 0; t < sane.size(); t++) {
      const bool bad = c->repair_fused_verify ? sfl[t] != 0 : san_bad[t] != 0;
      (sane[t] >> 24 == CDA_AXIS_ROW ? rbad : cbad)[sane[t] & 0xFFFFFF] = bad;
    }
    for (int i = 0; i < w; i++) {
      const bool rowc = P.cnt[CDA_AXIS_ROW][i] == w, colc = P.cnt[CDA_AXIS_COL][i] == w;
      if (rowc && rbad[i]) return finish(CDA_E_BYZANTINE, CDA_AXIS_ROW, i);
      if (colc && cbad[i]) return finish(CDA_E_BYZANTINE, CDA_AXIS_COL, i);
      if (rowc && pfl[i]) return finish(CDA_E_BYZANTINE, CDA_AXIS_ROW, i);
      if (colc && pfl[w + i]) return finish(CDA_E_BYZANTINE, CDA_AXIS_COL, i);
    }
  }
  for (size_t b = 0; b < nbat;) {
    if (bfl[b] == ~0u) {
      for (size_t q = bat[b].q0; q < bat[b].q1; q++) P.fill(ops[q].axis, ops[q].idx);
      b++;
      continue;
    }
    if (bat[b].q1 - bat[b].q0 == 1) {
      const int bad = vall[bat[b].v0 + bfl[b]];
      return finish(CDA_E_BYZANTINE, bad >> 24, bad & 0xFFFFFF);
    }
    for (size_t q = bat[b].q0; q < bat[b].q1; q++) {  // sequential replay of the failed batch
      // decode op q with the presence it sees in order, then verify its own and orthogonal roots
      long long off = ((const long long*)(h + o_off))[q], stride = ((const long long*)(h + o_str))[q];
      std::vector<uint8_t> pres(W);
      P.bytes(ops[q].axis, ops[q].idx, pres.data());
      long long* d_off = (long long*)c->dah.p;
      uint8_t* d_pres = (uint8_t*)(d_off + 2);
      if (!dev_ok(c, hipMemcpyAsync(d_off, &off, 8, hipMemcpyHostToDevice, s), "H2D") ||
          !dev_ok(c, hipMemcpyAsync(d_off + 1, &stride, 8, hipMemcpyHostToDevice, s), "H2D") ||
          !dev_ok(c, hipMemcpyAsync(d_pres, pres.data(), W, hipMemcpyHostToDevice, s), "H2D"))
        return CDA_E_DEVICE;
      {
        ProfScope ps(c, "repair_decode", s);
        const int lr = launch_rs_decode(d_eds, d_off, d_off + 1, d_pres, 1, K, CDA_SHARE, s);
        if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
      }
      std::vector<int> vaxes{enc_axis(ops[q].axis, ops[q].idx)};
      for (int o : ops[q].ortho) vaxes.push_back(o);
      if ((rc = roots_of(vaxes))) return rc;
      for (size_t u = 0; u < vaxes.size(); u++)
        if (!root_ok(u, vaxes[u])) return finish(CDA_E_BYZANTINE, vaxes[u] >> 24, vaxes[u] & 0xFFFFFF);
      P.fill(ops[q].axis, ops[q].idx);
    }
    // the replay passed: P equals the optimistic presence after batch b again, so the remaining
    // batches' descriptors still hold; run them again on the replayed square
    if (b + 1 < nbat) {
      if (!dev_ok(c, hipMemsetAsync(d_bfl + b + 1, 0xFF, (nbat - b - 1) * 4, s), "memset")) return CDA_E_DEVICE;
      if ((rc = enqueue_batches(b + 1))) return rc;
      if (!dev_ok(c, hipStreamSynchronize(s), "sync")) return CDA_E_DEVICE;
    }
    b++;
  }
  return finish(solved ? CDA_OK : CDA_E_UNREPAIRABLE, -1, -1);
}

extern "C" {

int cda_repair(cda_ctx* c, uint32_t k, uint8_t* eds, uint8_t* present, const uint8_t* row_roots,
               const uint8_t* col_roots, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !eds || !present || !row_roots || !col_roots) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  Lock l(c);
  return repair_impl(c, k, eds, nullptr, present, row_roots, col_roots, err, c->stream);
  CDA_API_CATCH(c)
}

int cda_repair_device(cda_ctx* c, uint32_t k, void* d_eds, uint8_t* present, const uint8_t* row_roots,
                      const uint8_t* col_roots, cda_err_info* err, void* stream) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !d_eds || !present || !row_roots || !col_roots) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  DevLock l(c, (hipStream_t)stream);
  return repair_impl(c, k, nullptr, (uint8_t*)d_eds, present, row_roots, col_roots, err, (hipStream_t)stream);
  CDA_API_CATCH(c)
}

}  // extern "C"
