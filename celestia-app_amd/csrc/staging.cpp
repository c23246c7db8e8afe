// staging.cpp — host <-> device copies of caller memory through pinned staging rings (used by cda_repair).
//
// cda_repair moves the whole 32 MiB square up and back from helper threads (the upload overlaps the host's
// planning, rows return while later batches run).  Issued as plain pageable hipMemcpyAsync from those
// threads the copies were erratic on MI355X boxes: C4 with a freshly allocated caller buffer took 2.6 ms at
// best but 15-22 ms at the median (scripts/fresh_buffer_probe.py, CDA_STAGING=0).  Through a ring of pinned
// slots -- worker threads copy chunk i into a slot (host memcpy, ~35 GB/s with three threads) while the DMA
// of chunk i-1 runs -- the same repair takes 2.6-2.9 ms every time.  The block paths keep plain
// hipMemcpyAsync: there the staged copy measured 20-30 % slower (a 48-block batch with its EDS 42 vs 32 ms)
// and the pageable copies were steady.  Pinned caller memory (cda_host_alloc, hipHostRegister) and small
// copies go straight to hipMemcpyAsync.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"

namespace cda {

// NUMA placement of the helper threads (measured, scripts/c4_numa_probe.py: C4 host-buffer repair on threads of
// the GPU's node 2.38 / 2.84 ms min / median, on the other socket 2.97 / 3.37 ms).
void find_local_cpus(cda_ctx* c) {
  c->local_cpus.clear();
  if (const char* e = getenv("CDA_NUMA_BIND"))
    if (atoi(e) == 0) return;
  char bdf[64] = {};
  if (hipDeviceGetPCIBusId(bdf, sizeof bdf, c->device) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  for (char* q = bdf; *q; q++) *q = (char)tolower((unsigned char)*q);
  char path[160];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/local_cpulist", bdf);
  FILE* f = fopen(path, "r");
  if (!f) return;
  char buf[4096] = {};
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
  for (char* q = buf; *q;) {  // "0-63,128-191"
    char* end = nullptr;
    const long a = strtol(q, &end, 10);
    if (end == q) break;
    long b = a;
    if (*end == '-') {
      q = end + 1;
      b = strtol(q, &end, 10);
    }
    for (long x = a; x <= b && x < CPU_SETSIZE; x++)
      if (x >= 0 && CPU_ISSET(x, &allowed)) c->local_cpus.push_back((int)x);
    q = end;
    while (*q == ',' || *q == '\n' || *q == ' ') q++;
  }
}

void bind_helper_thread(const cda_ctx* c) {
  if (c->local_cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int x : c->local_cpus) CPU_SET(x, &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);  // best effort: placement, not correctness
}

struct Piece {
  uint8_t* dst;
  const uint8_t* src;
  size_t n;
};

struct Stager {
  static constexpr int kSlots = 3;
  static constexpr size_t kSlotBytes = (size_t)4 << 20;
  static constexpr int kWorkers = 2;  // + the calling thread
  uint8_t* ring = nullptr;            // kSlots x kSlotBytes pinned
  hipEvent_t ev[kSlots] = {};
  bool used[kSlots] = {};  // ev[j] has been recorded (waits on never-recorded events are skipped)
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv_work, cv_done;
  // the current job: one contiguous copy (jdst, jsrc, jn) or, with jp, the concatenation of jnp pieces
  // (jn = their total bytes); part i of kWorkers + 1 copies bytes [jn * i / parts, jn * (i + 1) / parts)
  uint8_t* jdst = nullptr;
  const uint8_t* jsrc = nullptr;
  const Piece* jp = nullptr;
  size_t jn = 0, jnp = 0;
  unsigned gen = 0;
  int pending = 0;
  bool stop = false;

  void part(int i) {
    const size_t parts = kWorkers + 1, lo = jn * i / parts, hi = jn * (i + 1) / parts;
    if (hi <= lo) return;
    if (!jp) {
      memcpy(jdst + lo, jsrc + lo, hi - lo);
      return;
    }
    size_t pos = 0;
    for (size_t q = 0; q < jnp && pos < hi; pos += jp[q].n, q++) {
      const size_t a = std::max(lo, pos), b = std::min(hi, pos + jp[q].n);
      if (b > a) memcpy(jp[q].dst + (a - pos), jp[q].src + (a - pos), b - a);
    }
  }
  void worker(int i) {
    unsigned seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m);
        cv_work.wait(g, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      part(i);
      {
        std::lock_guard<std::mutex> g(m);
        --pending;
      }
      cv_done.notify_one();
    }
  }
  void run_job() {
    {
      std::lock_guard<std::mutex> g(m);
      pending = kWorkers;
      ++gen;
    }
    cv_work.notify_all();
    part(kWorkers);
    std::unique_lock<std::mutex> g(m);
    cv_done.wait(g, [&] { return pending == 0; });
  }
  // memcpy split over the workers and the calling thread
  void pmemcpy(void* dst, const void* src, size_t n) {
    if (n < ((size_t)256 << 10)) {
      memcpy(dst, src, n);
      return;
    }
    jdst = (uint8_t*)dst;
    jsrc = (const uint8_t*)src;
    jp = nullptr;
    jn = n;
    run_job();
  }
  // the pieces' bytes, split by position over the workers and the calling thread
  void pgather(const Piece* p, size_t np, size_t total) {
    jp = p;
    jnp = np;
    jn = total;
    run_job();
    jp = nullptr;
  }
  ~Stager() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv_work.notify_all();
    for (auto& t : th) t.join();
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
    if (ring) (void)hipHostFree(ring);
  }
};

static int get_stager(cda_ctx* c, Stager*& st) {
  if (st) return CDA_OK;
  auto* s = new Stager();
  bool ok = hipHostMalloc((void**)&s->ring, Stager::kSlots * Stager::kSlotBytes, hipHostMallocDefault) == hipSuccess;
  for (int j = 0; j < Stager::kSlots && ok; j++)
    ok = hipEventCreateWithFlags(&s->ev[j], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    c->last_err = "staging ring allocation failed";
    delete s;
    return CDA_E_DEVICE;
  }
  try {
    s->th.reserve(Stager::kWorkers);
    for (int i = 0; i < Stager::kWorkers; i++)
      s->th.emplace_back([s, i, c] {
        bind_helper_thread(c);
        s->worker(i);
      });
  } catch (...) {
    delete s;  // stops and joins the workers already started
    throw;
  }
  st = s;
  return CDA_OK;
}

// Host memory that the DMA engines can read directly (hipHostMalloc'd or registered).
static bool is_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory is not an error here
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Is all of [p, p + n) inside ONE page-locked range (hipHostMalloc'd or registered)?  A DMA or a kernel may then
// address it directly; a range only partly registered (its start pinned, its end not) fails the DMA engine's
// translation, so it is pageable here.
bool pinned_range(const void* p, size_t n) {
  if (!is_pinned(p)) return false;
  void* start = nullptr;
  size_t size = 0;
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess || !start) {
    (void)hipGetLastError();
    return false;
  }
  const uintptr_t a = (uintptr_t)p, s0 = (uintptr_t)start;
  return a >= s0 && a + n <= s0 + size;
}

// The device address of page-locked host memory [p, p + n) when one range holds all of it (kernels may then read it
// over PCIe directly), else nullptr.
const void* pinned_device_alias(const void* p, size_t n) {
  void* d = nullptr;
  if (!pinned_range(p, n) || hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

static bool direct(const cda_ctx* c, const void* host, size_t n, int dir_bit) {
  return !(c->staging & dir_bit) || n < ((size_t)2 << 20) || pinned_range(host, n);
}

int staged_h2d(cda_ctx* c, void* d_dst, const void* h_src, size_t n, hipStream_t s) {
  if (n == 0) return CDA_OK;
  if (direct(c, h_src, n, 1))
    return dev_ok(c, hipMemcpyAsync(d_dst, h_src, n, hipMemcpyHostToDevice, s), "H2D") ? CDA_OK : CDA_E_DEVICE;
  int rc = get_stager(c, c->st_in);
  if (rc) return rc;
  Stager& st = *c->st_in;
  const size_t B = Stager::kSlotBytes;
  for (size_t off = 0, i = 0; off < n; off += B, i++) {
    const int j = (int)(i % Stager::kSlots);
    const size_t len = std::min(B, n - off);
    uint8_t* slot = st.ring + (size_t)j * B;
    // the slot's previous DMA (chunk i - kSlots, or the last call's) has read it
    if (st.used[j] && !dev_ok(c, hipEventSynchronize(st.ev[j]), "staging wait")) return CDA_E_DEVICE;
    st.pmemcpy(slot, (const uint8_t*)h_src + off, len);
    if (!dev_ok(c, hipMemcpyAsync((uint8_t*)d_dst + off, slot, len, hipMemcpyHostToDevice, s), "H2D") ||
        !dev_ok(c, hipEventRecord(st.ev[j], s), "staging record"))
      return CDA_E_DEVICE;
    st.used[j] = true;
  }
  return CDA_OK;
}

int staged_h2d_runs(cda_ctx* c, void* d_dst, const uint8_t* h_base, const HostRun* runs, size_t nruns,
                    hipStream_t s) {
  size_t total = 0;
  for (size_t i = 0; i < nruns; i++) total += runs[i].len;
  if (total == 0) return CDA_OK;
  int rc = get_stager(c, c->st_in);
  if (rc) return rc;
  Stager& st = *c->st_in;
  const size_t B = Stager::kSlotBytes;
  std::vector<Piece> pieces;
  size_t r = 0, r_used = 0;  // next run, bytes of it already staged
  for (size_t off = 0, i = 0; off < total; off += B, i++) {
    const int j = (int)(i % Stager::kSlots);
    const size_t len = std::min(B, total - off);
    uint8_t* slot = st.ring + (size_t)j * B;
    pieces.clear();
    for (size_t fill = 0; fill < len;) {  // the next `len` bytes of the concatenated runs
      const size_t take = std::min(len - fill, runs[r].len - r_used);
      pieces.push_back(Piece{slot + fill, h_base + runs[r].off + r_used, take});
      fill += take;
      r_used += take;
      if (r_used == runs[r].len) r++, r_used = 0;
    }
    if (st.used[j] && !dev_ok(c, hipEventSynchronize(st.ev[j]), "staging wait")) return CDA_E_DEVICE;
    st.pgather(pieces.data(), pieces.size(), len);
    if (!dev_ok(c, hipMemcpyAsync((uint8_t*)d_dst + off, slot, len, hipMemcpyHostToDevice, s), "H2D") ||
        !dev_ok(c, hipEventRecord(st.ev[j], s), "staging record"))
      return CDA_E_DEVICE;
    st.used[j] = true;
  }
  return CDA_OK;
}

int staged_d2h(cda_ctx* c, void* h_dst, const void* d_src, size_t n, hipStream_t s) {
  if (n == 0) return CDA_OK;
  if (direct(c, h_dst, n, 2))
    return dev_ok(c, hipMemcpyAsync(h_dst, d_src, n, hipMemcpyDeviceToHost, s), "D2H") &&
                   dev_ok(c, hipStreamSynchronize(s), "sync")
               ? CDA_OK
               : CDA_E_DEVICE;
  int rc = get_stager(c, c->st_out);
  if (rc) return rc;
  Stager& st = *c->st_out;
  const size_t B = Stager::kSlotBytes, nchunks = (n + B - 1) / B;
  auto issue = [&](size_t i) {
    const int j = (int)(i % Stager::kSlots);
    const size_t off = i * B, len = std::min(B, n - off);
    st.used[j] = true;
    return dev_ok(c, hipMemcpyAsync(st.ring + (size_t)j * B, (const uint8_t*)d_src + off, len, hipMemcpyDeviceToHost,
                                    s),
                  "D2H") &&
           dev_ok(c, hipEventRecord(st.ev[j], s), "staging record");
  };
  for (size_t i = 0; i < std::min<size_t>(Stager::kSlots, nchunks); i++)
    if (!issue(i)) return CDA_E_DEVICE;
  for (size_t i = 0; i < nchunks; i++) {
    const int j = (int)(i % Stager::kSlots);
    const size_t off = i * B, len = std::min(B, n - off);
    if (!dev_ok(c, hipEventSynchronize(st.ev[j]), "staging wait")) return CDA_E_DEVICE;
    st.pmemcpy((uint8_t*)h_dst + off, st.ring + (size_t)j * B, len);
    if (i + Stager::kSlots < nchunks && !issue(i + Stager::kSlots)) return CDA_E_DEVICE;
  }
  return CDA_OK;
}

void free_staging(cda_ctx* c) {
  delete c->st_in;
  delete c->st_out;
  c->st_in = c->st_out = nullptr;
}

}  // namespace cda
