// split.cpp — ONE k x k square extended and committed across the G devices of a cda_multi handle
// (k = 512, GF(2^16), beyond one block's natural single-GPU size in testground).
//
// Reference: da.ExtendShares + NewDataAvailabilityHeader (pkg/da/data_availability_header.go:44-75) at
// appconsts/testground SquareSizeUpperBound = 512 (pkg/appconsts/testground/app_consts.go:8).  G is a power of two
// dividing k; device g owns ODS rows [g rp, (g+1) rp) (rp = k/G) and EDS columns [g cp, (g+1) cp) (cp = 2k/G):
//
//   1. row pass      : its rows -> Q0 copy + Q1 (row slab R, rp x 2k cells); the leaf record of every cell of
//                      those rows (LR) with the row push-order check; the roots of its top rows.
//   2. one exchange  : the top half changes hands: block (g, h) = rows of g x columns of h, shares AND their leaf
//                      records (so no top cell is hashed twice), one ncclSend / ncclRecv pair per peer inside one
//                      ncclGroupStart / ncclGroupEnd (RCCL over xGMI).  Device h then holds its columns' top half
//                      (column slab C, 2k x cp cells; records LC).
//   3. column pass   : column push order from the records; columns -> Q2|Q3 (bottom half of C; rsmt2d's
//                      Q3 = Enc(Q2 rows) is the same bytes by linearity); leaf records of the bottom half; the roots
//                      of its columns; for each bottom row r the root of the NMT subtree over its cp columns (the tree
//                      splits at powers of two, nmt_wrapper.go:118, so it is a node of row r's tree).
//   4. one gather    : each device's roots, subtree nodes and push-order status word (one contiguous record array)
//                      go to device 0, which folds the G subtree nodes of every bottom row (log2 G levels) and hashes
//                      the DAH over rowRoots ‖ colRoots.
// Every cell is hashed exactly once over all devices and the only inter-device traffic is the exchange (the top
// half: k x 2k shares + records) and the gather (4k + kG records).  At G = 1 the row slab IS the column slab's top
// half, so the split path does the block path's work with no copies.
//
// Transports: RCCL communicators from ncclCommInitAll over the handle's devices (one process, all GPUs -- what a
// Go node can do); or, for a handle made by cda_multi_init_replicas (G contexts on ONE device), device-to-device
// copies ordered by events: the same plan and kernels, testable on one GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"

using namespace cda;

namespace cda {

struct SplitComm {
  std::vector<ncclComm_t> comms;
};

void free_split_comm(cda_multi* m) {
  if (!m || !m->comm) return;
  for (auto cm : m->comm->comms)
    if (cm) (void)ncclCommDestroy(cm);
  delete m->comm;
  m->comm = nullptr;
}

}  // namespace cda

namespace {

struct Plan {
  uint32_t k, w, G, rp, cp;
  size_t S = CDA_SHARE, R = CDA_REC_BYTES;
  size_t meta_recs() const { return (size_t)rp + cp + k + 1; }  // top roots | column roots | subtree roots | status
};

int nccl_ok(cda_ctx* c, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return CDA_OK;
  c->last_err = std::string(what) + ": " + ncclGetErrorString(r);
  return CDA_E_DEVICE;
}

// Per-device buffers for one split (grown like the block path's workspace; kept between calls).
int ensure_split(cda_ctx* c, const Plan& p, int g) {
  const size_t rows_b = (size_t)p.rp * p.w * p.S, rrec_b = (size_t)p.rp * p.w * p.R;
  int rc;
  if ((rc = ensure(c, c->sp_ods, (size_t)p.rp * p.k * p.S)) || (rc = ensure(c, c->sp_C, (size_t)p.w * p.cp * p.S)) ||
      (rc = ensure(c, c->sp_LC, (size_t)p.w * p.cp * p.R)) ||
      (rc = ensure(c, c->sp_scratch,
                   std::max({(size_t)p.w * (p.rp + p.cp), (size_t)p.k * p.cp, (size_t)p.k * p.G}) * p.R)) ||
      (rc = ensure(c, c->sp_meta, p.meta_recs() * p.R)))
    return rc;
  if (p.G > 1) {
    if ((rc = ensure(c, c->sp_R, rows_b)) || (rc = ensure(c, c->sp_LR, rrec_b)) ||
        (rc = ensure(c, c->sp_S, (size_t)p.G * p.rp * p.cp * (p.S + p.R))))
      return rc;
  }
  // device 0: G meta arrays | 4k root records | DAH | G status words
  if (g == 0 && (rc = ensure(c, c->sp_gather, ((size_t)p.G * p.meta_recs() + 4 * (size_t)p.k) * p.R + 32 + 8 * p.G)))
    return rc;
  for (auto& e : c->sp_ev)
    if (!e && !dev_ok(c, hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate")) return CDA_E_DEVICE;
  return CDA_OK;
}

// Row slab / row leaf records of device g (at G = 1 the top half of the column slab itself).
uint8_t* row_slab(cda_ctx* c, const Plan& p) { return (uint8_t*)(p.G > 1 ? c->sp_R.p : c->sp_C.p); }
uint8_t* row_recs(cda_ctx* c, const Plan& p) { return (uint8_t*)(p.G > 1 ? c->sp_LR.p : c->sp_LC.p); }
uint8_t* send_sh(cda_ctx* c, const Plan& p, uint32_t h) {
  return (uint8_t*)c->sp_S.p + (size_t)h * p.rp * p.cp * p.S;
}
uint8_t* send_rec(cda_ctx* c, const Plan& p, uint32_t h) {
  return (uint8_t*)c->sp_S.p + (size_t)p.G * p.rp * p.cp * p.S + (size_t)h * p.rp * p.cp * p.R;
}

#define TRY(x)                    \
  do {                            \
    if (int rc_ = (x)) return rc_; \
  } while (0)
#define HIPC(c, x, what)                                       \
  do {                                                         \
    if (!dev_ok((c), (x), (what))) return CDA_E_DEVICE;        \
  } while (0)

// Step 1 on device g: row encode, row leaves (+ row push order), top-row roots, pack the send blocks.
int row_pass(cda_ctx* c, const Plan& p, uint32_t g, const uint8_t* d_slab) {
  hipStream_t s = c->stream;
  const uint32_t r0 = g * p.rp;
  uint8_t* R = row_slab(c, p);
  uint8_t* LR = row_recs(c, p);
  uint8_t* meta = (uint8_t*)c->sp_meta.p;
  unsigned long long* st = (unsigned long long*)(meta + (p.meta_recs() - 1) * p.R);
  HIPC(c, hipMemsetAsync(meta + (p.meta_recs() - 1) * p.R, 0, p.R, s), "memset");
  HIPC(c, hipMemsetAsync(st, 0xFF, 8, s), "memset");
  {
    RsJob j{};
    j.src = d_slab;
    j.src_cw = (long long)p.k * p.S;
    j.src_sh = p.S;
    j.dst = R + (size_t)p.k * p.S;
    j.dst_cw = (long long)p.w * p.S;
    j.dst_sh = p.S;
    j.cpy = R;
    j.cpy_cw = j.dst_cw;
    j.cpy_sh = p.S;
    j.k = (int)p.k;
    j.cw_per_blk = (int)p.rp;
    j.nblk = 1;
    j.shard_len = CDA_SHARE;
    ProfScope ps(c, 2 * p.k <= 256 ? "split_rs_rows8" : "split_rs_rows16", s);
    const int lr = 2 * p.k <= 256 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  {
    ProfScope ps(c, "split_leaf_rows", s);
    if (launch_region_leaf(R, (long long)p.w * p.S, (int)r0, 0, (int)p.rp, (int)p.w, (int)p.k, LR, p.w, st, true, s))
      return CDA_E_DEVICE;
  }
  if (p.G > 1) {  // block h = this device's rows x h's columns: shares and leaf records, packed contiguous
    uint8_t* C = (uint8_t*)c->sp_C.p;
    uint8_t* LC = (uint8_t*)c->sp_LC.p;
    for (uint32_t h = 0; h < p.G; h++) {
      const size_t c0 = (size_t)h * p.cp;
      uint8_t* dsh = h == g ? C + (size_t)r0 * p.cp * p.S : send_sh(c, p, h);
      uint8_t* drec = h == g ? LC + (size_t)r0 * p.cp * p.R : send_rec(c, p, h);
      HIPC(c, hipMemcpy2DAsync(dsh, p.cp * p.S, R + c0 * p.S, p.w * p.S, p.cp * p.S, p.rp, hipMemcpyDeviceToDevice, s),
           "pack");
      HIPC(c, hipMemcpy2DAsync(drec, p.cp * p.R, LR + c0 * p.R, p.w * p.R, p.cp * p.R, p.rp, hipMemcpyDeviceToDevice, s),
           "pack");
    }
  }
  return CDA_OK;
}

// Step 3 on device h: column order, column encode, bottom leaves, column roots, bottom-row subtree roots.
int col_pass(cda_ctx* c, const Plan& p, uint32_t h) {
  hipStream_t s = c->stream;
  const uint32_t c0 = h * p.cp;
  uint8_t* C = (uint8_t*)c->sp_C.p;
  uint8_t* LC = (uint8_t*)c->sp_LC.p;
  uint8_t* meta = (uint8_t*)c->sp_meta.p;
  unsigned long long* st = (unsigned long long*)(meta + (p.meta_recs() - 1) * p.R);
  if (launch_records_col_order(LC, p.cp, (int)p.k, (int)c0, (int)p.cp, (int)p.k, st, s)) return CDA_E_DEVICE;
  {
    RsJob j{};
    j.src = C;
    j.src_cw = p.S;
    j.src_sh = (long long)p.cp * p.S;
    j.dst = C + (size_t)p.k * p.cp * p.S;
    j.dst_cw = p.S;
    j.dst_sh = (long long)p.cp * p.S;
    j.k = (int)p.k;
    j.cw_per_blk = (int)p.cp;
    j.nblk = 1;
    j.shard_len = CDA_SHARE;
    ProfScope ps(c, 2 * p.k <= 256 ? "split_rs_cols8" : "split_rs_cols16", s);
    const int lr = 2 * p.k <= 256 ? launch_rs_encode8(j, s) : launch_rs_encode16(j, s);
    if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  }
  {
    ProfScope ps(c, "split_leaf_bottom", s);
    if (launch_region_leaf(C + (size_t)p.k * p.cp * p.S, (long long)p.cp * p.S, (int)p.k, (int)c0, (int)p.k,
                           (int)p.cp, (int)p.k, LC + (size_t)p.k * p.cp * p.R, p.cp, st, false, s))
      return CDA_E_DEVICE;
  }
  int L = 0, Lc = 0;
  while ((1u << L) < p.w) L++;
  while ((1u << Lc) < p.cp) Lc++;
  {  // the roots of this device's top rows (row leaf records LR, tree-major) and of its columns (LC, node-major)
     // in one launch sequence, so neither set's thin top levels run alone
    ProfScope ps(c, "split_trees", s);
    uint8_t* sc = (uint8_t*)c->sp_scratch.p;
    const TreeSpec sets[2] = {
        {row_recs(c, p), p.w, 1, p.rp, false, sc, meta, 1},
        {LC, 1, p.cp, p.cp, true, sc + (size_t)p.rp * p.w * p.R, meta + (size_t)p.rp * p.R, 1}};
    if (launch_tree_roots(sets, 2, L, s)) return CDA_E_DEVICE;
  }
  {  // bottom rows: the subtree over this device's cp columns
    ProfScope ps(c, "split_tree_bottom", s);
    uint8_t* sub = meta + ((size_t)p.rp + p.cp) * p.R;
    const uint8_t* leaves = LC + (size_t)p.k * p.cp * p.R;
    if (Lc == 0) {
      HIPC(c, hipMemcpyAsync(sub, leaves, (size_t)p.k * p.R, hipMemcpyDeviceToDevice, s), "copy");
    } else {
      const TreeSpec set{leaves, p.cp, 1, p.k, false, c->sp_scratch.p, sub, 1};
      if (launch_tree_roots(&set, 1, Lc, s)) return CDA_E_DEVICE;
    }
  }
  return CDA_OK;
}

// Step 4 on device 0: fold the bottom-row subtrees, assemble rowRoots ‖ colRoots, DAH.
int finish_pass(cda_ctx* c0, const Plan& p) {
  hipStream_t s = c0->stream;
  const size_t mr = p.meta_recs();
  uint8_t* gat = (uint8_t*)c0->sp_gather.p;           // [G][mr] records
  uint8_t* fin = gat + (size_t)p.G * mr * p.R;         // [4k] records: top rows | bottom rows | columns
  uint8_t* dah = fin + 4 * (size_t)p.k * p.R;          // 32 B
  HIPC(c0, hipMemcpy2DAsync(fin, p.rp * p.R, gat, mr * p.R, p.rp * p.R, p.G, hipMemcpyDeviceToDevice, s), "assemble");
  HIPC(c0, hipMemcpy2DAsync(fin + 2 * (size_t)p.k * p.R, p.cp * p.R, gat + (size_t)p.rp * p.R, mr * p.R, p.cp * p.R,
                            p.G, hipMemcpyDeviceToDevice, s),
       "assemble");
  const uint8_t* sub = gat + ((size_t)p.rp + p.cp) * p.R;  // node g of bottom row r: sub[g * mr + r]
  uint8_t* bottom = fin + (size_t)p.k * p.R;
  if (p.G == 1) {
    HIPC(c0, hipMemcpyAsync(bottom, sub, (size_t)p.k * p.R, hipMemcpyDeviceToDevice, s), "copy");
  } else {
    int Lg = 0;
    while ((1u << Lg) < p.G) Lg++;
    ProfScope ps(c0, "split_fold", s);
    const TreeSpec set{sub, 1, mr, p.k, true, c0->sp_scratch.p, bottom, 1};
    if (launch_tree_roots(&set, 1, Lg, s)) return CDA_E_DEVICE;
  }
  ProfScope ps(c0, "dah", s);
  const int lr = launch_dah(fin, dah, (int)(4 * p.k), 1, s);
  if (lr) return lr == -2 ? CDA_E_UNSUPPORTED : CDA_E_DEVICE;
  return CDA_OK;
}

// Exchange of the top half (step 2).  RCCL: every send and receive of every device in one group.  Replicas: the
// receiver's stream waits for each sender's pack and copies the block.
int exchange(cda_multi* m, const Plan& p) {
  const uint32_t G = p.G;
  if (G == 1) return CDA_OK;
  const size_t bsh = (size_t)p.rp * p.cp * p.S, brec = (size_t)p.rp * p.cp * p.R;
  if (m->replicas) {
    for (uint32_t g = 0; g < G; g++) HIPC(m->ctx[g], hipEventRecord(m->ctx[g]->sp_ev[0], m->ctx[g]->stream), "event");
    for (uint32_t h = 0; h < G; h++) {
      cda_ctx* ch = m->ctx[h];
      for (uint32_t g = 0; g < G; g++) {
        if (g == h) continue;
        cda_ctx* cg = m->ctx[g];
        HIPC(ch, hipStreamWaitEvent(ch->stream, cg->sp_ev[0], 0), "wait");
        HIPC(ch, hipMemcpyAsync((uint8_t*)ch->sp_C.p + (size_t)g * p.rp * p.cp * p.S, send_sh(cg, p, h), bsh,
                                hipMemcpyDeviceToDevice, ch->stream),
             "exchange");
        HIPC(ch, hipMemcpyAsync((uint8_t*)ch->sp_LC.p + (size_t)g * p.rp * p.cp * p.R, send_rec(cg, p, h), brec,
                                hipMemcpyDeviceToDevice, ch->stream),
             "exchange");
      }
    }
    // the senders' send blocks are rewritten by the next call's row pass only after this call's copies
    for (uint32_t h = 0; h < G; h++) HIPC(m->ctx[h], hipEventRecord(m->ctx[h]->sp_ev[1], m->ctx[h]->stream), "event");
    for (uint32_t g = 0; g < G; g++)
      for (uint32_t h = 0; h < G; h++)
        if (g != h) HIPC(m->ctx[g], hipStreamWaitEvent(m->ctx[g]->stream, m->ctx[h]->sp_ev[1], 0), "wait");
    return CDA_OK;
  }
  cda_ctx* c0 = m->ctx[0];
  TRY(nccl_ok(c0, ncclGroupStart(), "ncclGroupStart"));
  int rc = CDA_OK;
  for (uint32_t g = 0; g < G && rc == CDA_OK; g++) {
    cda_ctx* cg = m->ctx[g];
    (void)hipSetDevice(cg->device);
    ncclComm_t cm = m->comm->comms[g];
    for (uint32_t h = 0; h < G && rc == CDA_OK; h++) {
      if (h == g) continue;
      if ((rc = nccl_ok(cg, ncclSend(send_sh(cg, p, h), bsh, ncclUint8, (int)h, cm, cg->stream), "ncclSend")) ||
          (rc = nccl_ok(cg, ncclSend(send_rec(cg, p, h), brec, ncclUint8, (int)h, cm, cg->stream), "ncclSend")) ||
          (rc = nccl_ok(cg, ncclRecv((uint8_t*)cg->sp_C.p + (size_t)h * p.rp * p.cp * p.S, bsh, ncclUint8, (int)h, cm,
                                     cg->stream),
                        "ncclRecv")) ||
          (rc = nccl_ok(cg, ncclRecv((uint8_t*)cg->sp_LC.p + (size_t)h * p.rp * p.cp * p.R, brec, ncclUint8, (int)h,
                                     cm, cg->stream),
                        "ncclRecv")))
        break;
    }
  }
  const int rc2 = nccl_ok(c0, ncclGroupEnd(), "ncclGroupEnd");
  return rc ? rc : rc2;
}

// Gather of every device's meta records to device 0 (step 4).
int gather(cda_multi* m, const Plan& p) {
  const uint32_t G = p.G;
  const size_t mb = p.meta_recs() * p.R;
  cda_ctx* c0 = m->ctx[0];
  (void)hipSetDevice(c0->device);
  HIPC(c0, hipMemcpyAsync(c0->sp_gather.p, c0->sp_meta.p, mb, hipMemcpyDeviceToDevice, c0->stream), "gather");
  if (G == 1) return CDA_OK;
  if (m->replicas) {
    for (uint32_t g = 1; g < G; g++) {
      cda_ctx* cg = m->ctx[g];
      HIPC(cg, hipEventRecord(cg->sp_ev[0], cg->stream), "event");
      HIPC(c0, hipStreamWaitEvent(c0->stream, cg->sp_ev[0], 0), "wait");
      HIPC(c0, hipMemcpyAsync((uint8_t*)c0->sp_gather.p + (size_t)g * mb, cg->sp_meta.p, mb, hipMemcpyDeviceToDevice,
                              c0->stream),
           "gather");
    }
    HIPC(c0, hipEventRecord(c0->sp_ev[1], c0->stream), "event");
    for (uint32_t g = 1; g < G; g++) HIPC(m->ctx[g], hipStreamWaitEvent(m->ctx[g]->stream, c0->sp_ev[1], 0), "wait");
    return CDA_OK;
  }
  TRY(nccl_ok(c0, ncclGroupStart(), "ncclGroupStart"));
  int rc = CDA_OK;
  for (uint32_t g = 1; g < G && rc == CDA_OK; g++) {
    cda_ctx* cg = m->ctx[g];
    (void)hipSetDevice(cg->device);
    rc = nccl_ok(cg, ncclSend(cg->sp_meta.p, mb, ncclUint8, 0, m->comm->comms[g], cg->stream), "ncclSend");
    if (!rc) {
      (void)hipSetDevice(c0->device);
      rc = nccl_ok(c0, ncclRecv((uint8_t*)c0->sp_gather.p + (size_t)g * mb, mb, ncclUint8, (int)g, m->comm->comms[0],
                                c0->stream),
                   "ncclRecv");
    }
  }
  const int rc2 = nccl_ok(c0, ncclGroupEnd(), "ncclGroupEnd");
  return rc ? rc : rc2;
}

int ensure_comms(cda_multi* m) {
  if (m->replicas || m->ctx.size() == 1 || m->comm) return CDA_OK;
  auto* sc = new SplitComm();
  sc->comms.assign(m->ctx.size(), nullptr);
  const ncclResult_t r = ncclCommInitAll(sc->comms.data(), (int)m->ctx.size(), m->devices.data());
  if (r != ncclSuccess) {
    m->ctx[0]->last_err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
    delete sc;
    return CDA_E_DEVICE;
  }
  m->comm = sc;
  return CDA_OK;
}

// The whole split.  Input: host ODS (h_ods, k*k*512, row-major) or per-device slabs already in device memory
// (d_slabs[g] on device g: rows [g rp, (g+1) rp) of the ODS).  Outputs on the host.
int split_impl(cda_multi* m, uint32_t k, const uint8_t* h_ods, const void* const* d_slabs, uint8_t* eds,
               uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah_out, cda_err_info* err) {
  const uint32_t G = (uint32_t)m->ctx.size();
  Plan p{k, 2 * k, G, k / G, 2 * k / G};
  std::lock_guard<std::mutex> sl(m->split_mu);
  std::vector<std::unique_ptr<Lock>> locks;
  for (auto* c : m->ctx) locks.emplace_back(new Lock(c));
  TRY(ensure_comms(m));
  for (uint32_t g = 0; g < G; g++) {
    (void)hipSetDevice(m->ctx[g]->device);
    TRY(ensure_split(m->ctx[g], p, (int)g));
  }
  // upload the slabs (pageable host memory blocks the issuing thread: one thread per device when G > 1)
  std::vector<const uint8_t*> slab(G);
  if (h_ods) {
    std::vector<int> rcs(G, CDA_OK);
    auto up = [&](uint32_t g) {
      cda_ctx* c = m->ctx[g];
      try {
        (void)hipSetDevice(c->device);
        rcs[g] = dev_ok(c, hipMemcpyAsync(c->sp_ods.p, h_ods + (size_t)g * p.rp * p.k * p.S, (size_t)p.rp * p.k * p.S,
                                          hipMemcpyHostToDevice, c->stream),
                        "H2D")
                     ? CDA_OK
                     : CDA_E_DEVICE;
      } catch (...) {
        rcs[g] = api_exception(c);
      }
    };
    if (G == 1) {
      up(0);
    } else {
      std::vector<std::thread> th;
      th.reserve(G);
      struct JoinAll {
        std::vector<std::thread>& v;
        ~JoinAll() {
          for (auto& t : v)
            if (t.joinable()) t.join();
        }
      } join_all{th};
      for (uint32_t g = 0; g < G; g++) th.emplace_back(up, g);
      for (auto& t : th) t.join();
    }
    for (uint32_t g = 0; g < G; g++) {
      TRY(rcs[g]);
      slab[g] = (const uint8_t*)m->ctx[g]->sp_ods.p;
    }
  } else {
    for (uint32_t g = 0; g < G; g++) slab[g] = (const uint8_t*)d_slabs[g];
  }
  cda_ctx* c0 = m->ctx[0];
  if (G == 1) {
    // one device: its column slab is the whole 2k x 2k EDS, so the split is the block pipeline itself (RS rows and
    // columns, leaf hashing shared by row and column trees, all 4k trees, DAH) into the result area
    // (the pipeline sets its status word itself; it sits behind the DAH, where the results copy reads it)
    uint8_t* fin = (uint8_t*)c0->sp_gather.p + p.meta_recs() * p.R;
    unsigned long long* st = (unsigned long long*)(fin + 4 * (size_t)k * p.R + 32);
    TRY(enqueue_pipeline(c0, k, 1, slab[0], (uint8_t*)c0->sp_C.p, fin, fin + 4 * (size_t)k * p.R, st, c0->stream));
  } else {
    for (uint32_t g = 0; g < G; g++) {
      (void)hipSetDevice(m->ctx[g]->device);
      TRY(row_pass(m->ctx[g], p, g, slab[g]));
    }
    TRY(exchange(m, p));
    for (uint32_t h = 0; h < G; h++) {
      (void)hipSetDevice(m->ctx[h]->device);
      TRY(col_pass(m->ctx[h], p, h));
    }
    TRY(gather(m, p));
    (void)hipSetDevice(c0->device);
    TRY(finish_pass(c0, p));
  }
  // results: 4k roots + DAH + the G status words, gathered behind the DAH on device 0 and fetched by ONE copy into a
  // pinned buffer of the handle; the EDS from where each part lives
  const size_t mr = p.meta_recs();
  uint8_t* gat = (uint8_t*)c0->sp_gather.p;
  uint8_t* fin = gat + (size_t)G * mr * p.R;
  const size_t res_b = 4 * (size_t)k * p.R + 32 + 8 * (size_t)G;
  if (G > 1)
    HIPC(c0, hipMemcpy2DAsync(fin + 4 * (size_t)k * p.R + 32, 8, gat + (mr - 1) * p.R, mr * p.R, 8, G,
                              hipMemcpyDeviceToDevice, c0->stream),
         "status");
  if (m->pin_cap < res_b) {
    if (m->pin_res) (void)hipHostFree(m->pin_res);
    m->pin_res = nullptr;
    m->pin_cap = 0;
    (void)hipSetDevice(c0->device);
    HIPC(c0, hipHostMalloc((void**)&m->pin_res, res_b, hipHostMallocDefault), "hipHostMalloc");
    m->pin_cap = res_b;
  }
  (void)hipSetDevice(c0->device);
  HIPC(c0, hipMemcpyAsync(m->pin_res, fin, res_b, hipMemcpyDeviceToHost, c0->stream), "D2H");
  if (eds && G == 1) {
    HIPC(c0, hipMemcpyAsync(eds, c0->sp_C.p, (size_t)p.w * p.w * p.S, hipMemcpyDeviceToHost, c0->stream), "D2H");
  } else if (eds) {
    for (uint32_t g = 0; g < G; g++) {  // top rows from each row slab, bottom half from each column slab
      cda_ctx* c = m->ctx[g];
      (void)hipSetDevice(c->device);
      HIPC(c, hipMemcpyAsync(eds + (size_t)g * p.rp * p.w * p.S, row_slab(c, p), (size_t)p.rp * p.w * p.S,
                             hipMemcpyDeviceToHost, c->stream),
           "D2H");
      HIPC(c, hipMemcpy2DAsync(eds + ((size_t)k * p.w + (size_t)g * p.cp) * p.S, p.w * p.S,
                               (const uint8_t*)c->sp_C.p + (size_t)k * p.cp * p.S, p.cp * p.S, p.cp * p.S, k,
                               hipMemcpyDeviceToHost, c->stream),
           "D2H");
    }
  }
  // device 0's stream ends after every device's part (the gather receives from all of them); the others are
  // synchronised too so that the call returns with no work of it in flight
  for (uint32_t g = 0; g < G; g++) {
    (void)hipSetDevice(m->ctx[g]->device);
    HIPC(m->ctx[g], hipStreamSynchronize(m->ctx[g]->stream), "sync");
    flush_profile(m->ctx[g]);
  }
  pack_roots(m->pin_res, 2 * k, row_roots);
  pack_roots(m->pin_res + 2 * (size_t)k * p.R, 2 * k, col_roots);
  memcpy(dah_out, m->pin_res + 4 * (size_t)k * p.R, 32);
  uint64_t st = ~0ull;
  for (uint32_t g = 0; g < G; g++) {
    uint64_t v;
    memcpy(&v, m->pin_res + 4 * (size_t)k * p.R + 32 + 8 * (size_t)g, 8);
    st = std::min(st, v);
  }
  return map_status(st, -1, err);
}

// A failure on any device of the handle (an RCCL group call is issued per device; ncclCommInitAll reports into
// device 0) is surfaced through cda_last_device_error(cda_multi_context(m, 0)): every device's message, each named
// by its handle index and HIP device, with the RCCL error string.
// Every context's lock is held from the clearing of last_err to the combined message (a concurrent call on
// a handle from cda_multi_context writes the same string under that lock); split_impl takes the handle's split mutex
// and re-enters these (recursive) locks.
int split_call(cda_multi* m, uint32_t k, const uint8_t* h_ods, const void* const* d_slabs, uint8_t* eds,
               uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, cda_err_info* err) {
  std::vector<std::unique_ptr<Lock>> locks;
  for (auto* c : m->ctx) locks.emplace_back(new Lock(c));
  for (auto* c : m->ctx) c->last_err.clear();
  const int rc = split_impl(m, k, h_ods, d_slabs, eds, row_roots, col_roots, dah, err);
  if (rc == CDA_E_DEVICE || rc == CDA_E_NOMEM || rc == CDA_E_INTERNAL) {
    std::string all;
    for (size_t g = 0; g < m->ctx.size(); g++)
      if (!m->ctx[g]->last_err.empty())
        all += (all.empty() ? "" : "; ") + std::string("split device ") + std::to_string(g) + " (HIP " +
               std::to_string(m->ctx[g]->device) + "): " + m->ctx[g]->last_err;
    m->ctx[0]->last_err = all.empty() ? std::string("split: device error (no detail recorded)") : all;
  }
  return rc;
}

int check_split_args(cda_multi* m, uint32_t k, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah) {
  if (!m || m->ctx.empty() || !row_roots || !col_roots || !dah) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  const uint32_t G = (uint32_t)m->ctx.size();
  if (!is_pow2(G) || k % G) return CDA_E_ARG;  // devices must be a power of two dividing k
  return CDA_OK;
}

}  // namespace

extern "C" {

int cda_multi_init_replicas(int device, uint32_t count, cda_multi** out) {
  CDA_API_TRY
  if (!out || count == 0 || count > 64) return CDA_E_ARG;
  *out = nullptr;
  cda_multi* m = new cda_multi();
  struct Owner {
    cda_multi* m;
    ~Owner() {
      if (m) cda_multi_free(m);
    }
  } own{m};
  m->replicas = true;
  for (uint32_t i = 0; i < count; i++) {
    cda_ctx* c = nullptr;
    if (cda_init(device, &c) != CDA_OK) return CDA_E_DEVICE;
    m->ctx.reserve(m->ctx.size() + 1);
    m->ctx.push_back(c);
    m->devices.push_back(device);
  }
  own.m = nullptr;
  *out = m;
  return CDA_OK;
  CDA_API_CATCH(nullptr)
}

int cda_multi_extend_commit_split(cda_multi* m, uint32_t k, const uint8_t* ods, uint8_t* eds_or_null,
                                  uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!ods) return CDA_E_ARG;
  if (int rc = check_split_args(m, k, row_roots, col_roots, dah)) return rc;
  return split_call(m, k, ods, nullptr, eds_or_null, row_roots, col_roots, dah, err);
  CDA_API_CATCH(m && !m->ctx.empty() ? m->ctx[0] : nullptr)
}

int cda_multi_extend_commit_split_device(cda_multi* m, uint32_t k, const void* const* d_ods_slabs, uint8_t* row_roots,
                                         uint8_t* col_roots, uint8_t* dah, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!d_ods_slabs) return CDA_E_ARG;
  if (int rc = check_split_args(m, k, row_roots, col_roots, dah)) return rc;
  for (size_t g = 0; g < m->ctx.size(); g++)
    if (!d_ods_slabs[g]) return CDA_E_ARG;
  return split_call(m, k, nullptr, d_ods_slabs, nullptr, row_roots, col_roots, dah, err);
  CDA_API_CATCH(m && !m->ctx.empty() ? m->ctx[0] : nullptr)
}

}  // extern "C"
