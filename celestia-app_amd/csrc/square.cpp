// square.cpp — square construction on the device (include/cda.h "square construction"): validates a
// host layout plan and assembles the ODS in HBM (square_kernels.hip); cda_construct_extend_commit then
// runs the block path on it, so the host never materialises the k*k shares.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "ctx.h"
#include "plan.h"

using namespace cda;


extern "C" {

int cda_build_ods_device(cda_ctx* c, uint32_t k, uint32_t nseg, const cda_share_segment* segs, const uint8_t* data,
                         uint64_t data_len, const uint32_t* reserved, uint32_t nreserved, void* d_ods, void* stream) {
  CDA_API_TRY
  if (!c || !d_ods || !is_pow2(k) || k > kMaxDeviceK) return CDA_E_ARG;
  if (int rc = plan::check_square_plan(k, nseg, segs, data_len, nreserved)) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : nullptr;
  DevLock l(c, s);
  const size_t seg_b = (size_t)nseg * sizeof(cda_share_segment), res_b = (size_t)nreserved * 4;
  int rc;
  if ((rc = ensure(c, c->plan, seg_b + res_b + 16)) || (rc = ensure(c, c->payload, data_len + 16))) return rc;
  uint8_t* d_plan = (uint8_t*)c->plan.p;
  if (!dev_ok(c, hipMemcpyAsync(d_plan, segs, seg_b, hipMemcpyHostToDevice, s), "H2D") ||
      (nreserved && !dev_ok(c, hipMemcpyAsync(d_plan + seg_b, reserved, res_b, hipMemcpyHostToDevice, s), "H2D")) ||
      (data_len && !dev_ok(c, hipMemcpyAsync(c->payload.p, data, data_len, hipMemcpyHostToDevice, s), "H2D")))
    return CDA_E_DEVICE;
  ProfScope ps(c, "build_ods", s);
  const int lr = launch_build_ods((const cda_share_segment*)d_plan, (int)nseg, (const uint8_t*)c->payload.p,
                                  (const uint32_t*)(d_plan + seg_b), k * k, d_ods, s);
  return lr == 0 ? CDA_OK : (lr == -2 ? CDA_E_ARG : CDA_E_DEVICE);
  CDA_API_CATCH(c)
}

int cda_construct_extend_commit(cda_ctx* c, uint32_t k, uint32_t nseg, const cda_share_segment* segs,
                                const uint8_t* data, uint64_t data_len, const uint32_t* reserved, uint32_t nreserved,
                                uint8_t* ods_or_null, uint8_t* eds_or_null, uint8_t* row_roots, uint8_t* col_roots,
                                uint8_t* dah, cda_err_info* err) {
  CDA_API_TRY
  set_err(err, CDA_OK, -1, -1, -1, -1);
  if (!c || !row_roots || !col_roots || !dah) return CDA_E_ARG;
  if (!is_pow2(k)) return CDA_E_NOT_POW2;
  if (k > kMaxDeviceK) return CDA_E_UNSUPPORTED;
  Lock l(c);
  const uint32_t w = 2 * k;
  const size_t ods_b = (size_t)k * k * CDA_SHARE, eds_b = (size_t)w * w * CDA_SHARE;
  const size_t roots_b = (size_t)2 * w * CDA_REC_BYTES;
  int rc;
  if ((rc = ensure(c, c->ods, ods_b)) || (rc = ensure(c, c->eds, eds_b)) || (rc = ensure(c, c->roots, roots_b)) ||
      (rc = ensure(c, c->dah, 32)) || (rc = ensure(c, c->status, 8)))
    return rc;
  if ((rc = cda_build_ods_device(c, k, nseg, segs, data, data_len, reserved, nreserved, c->ods.p, c->stream)))
    return rc;
  rc = enqueue_pipeline(c, k, 1, (const uint8_t*)c->ods.p, (uint8_t*)c->eds.p, c->roots.p, c->dah.p,
                        (unsigned long long*)c->status.p, c->stream);
  if (rc) return rc;
  std::vector<uint8_t> recs(roots_b);
  uint64_t st = 0;
  hipStream_t s = c->stream;
  if ((ods_or_null && !dev_ok(c, hipMemcpyAsync(ods_or_null, c->ods.p, ods_b, hipMemcpyDeviceToHost, s), "D2H")) ||
      (eds_or_null && !dev_ok(c, hipMemcpyAsync(eds_or_null, c->eds.p, eds_b, hipMemcpyDeviceToHost, s), "D2H")) ||
      !dev_ok(c, hipMemcpyAsync(recs.data(), c->roots.p, roots_b, hipMemcpyDeviceToHost, s), "D2H") ||
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

}  // extern "C"
