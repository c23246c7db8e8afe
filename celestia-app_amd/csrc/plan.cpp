// plan.cpp — host-only planners (plan.h).  No HIP: built into libcda and, alone, under the CPU sanitizers.
#include "plan.h"

#include <string.h>

#include <algorithm>

namespace cda {
namespace plan {

namespace {
// 8 presence bytes (any nonzero = present) -> 8 bits, byte i -> bit i
inline uint64_t pack8(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  v = (((v & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | v) & 0x8080808080808080ull;
  return ((v >> 7) * 0x0102040810204080ull) >> 56;
}
// in place: a[i] bit j <-> a[j] bit i
void transpose64(uint64_t a[64]) {
  uint64_t m = 0x00000000FFFFFFFFull;
  for (int j = 32; j; j >>= 1, m ^= m << j)
    for (int k = 0; k < 64; k = ((k | j) + 1) & ~j) {
      const uint64_t t = ((a[k] >> j) ^ a[k | j]) & m;
      a[k] ^= t << j;
      a[k | j] ^= t;
    }
}
}  // namespace

void Presence::init(int w_, const uint8_t* p) {
  w = w_;
  words = (w + 63) / 64;
  full = w >= 64 ? ~0ull : ((1ull << w) - 1);
  for (int a = 0; a < 2; a++) {
    bits[a].assign((size_t)w * words, 0);
    cnt[a].assign(w, 0);
  }
  uint64_t* rb = bits[CDA_AXIS_ROW].data();
  for (int r = 0; r < w; r++) {
    const uint8_t* row = p + (size_t)r * w;
    if (w < 8) {
      for (int q = 0; q < w; q++) rb[(size_t)r * words] |= (uint64_t)(row[q] != 0) << q;
    } else {
      for (int q = 0; q < w; q += 8) rb[(size_t)r * words + (q >> 6)] |= pack8(row + q) << (q & 63);
    }
    int n = 0;
    for (int wd = 0; wd < words; wd++) n += __builtin_popcountll(rb[(size_t)r * words + wd]);
    cnt[CDA_AXIS_ROW][r] = n;
  }
  // column bitsets: 64 x 64 bit-block transposes of the row bitsets
  uint64_t blk[64];
  for (int R = 0; R < words; R++)
    for (int C = 0; C < words; C++) {
      for (int i = 0; i < 64; i++) blk[i] = R * 64 + i < w ? rb[(size_t)(R * 64 + i) * words + C] : 0;
      transpose64(blk);
      for (int j = 0; j < 64 && C * 64 + j < w; j++) bits[CDA_AXIS_COL][(size_t)(C * 64 + j) * words + R] = blk[j];
    }
  for (int q = 0; q < w; q++) {
    int n = 0;
    for (int wd = 0; wd < words; wd++) n += __builtin_popcountll(bits[CDA_AXIS_COL][(size_t)q * words + wd]);
    cnt[CDA_AXIS_COL][q] = n;
  }
}

void Presence::bytes(int a, int idx, uint8_t* out) const {
  static const struct Expand {
    uint64_t t[256];
    Expand() {
      for (int v = 0; v < 256; v++) {
        t[v] = 0;
        for (int i = 0; i < 8; i++) t[v] |= (uint64_t)((v >> i) & 1) << (8 * i);
      }
    }
  } ex;
  const uint64_t* b = bits[a].data() + (size_t)idx * words;
  if (w < 8) {
    for (int j = 0; j < w; j++) out[j] = (b[0] >> j) & 1;
    return;
  }
  for (int j = 0; j < w; j += 8) {
    const uint64_t v = ex.t[(b[j >> 6] >> (j & 63)) & 0xFF];
    memcpy(out + j, &v, 8);
  }
}

int plan_repair(const Presence& P, int K, RepairPlan& out, uint8_t* pres_out) {
  const int w = P.w;
  const size_t W = (size_t)w;
  out = RepairPlan{};
  for (int i = 0; i < w; i++) {
    if (P.cnt[CDA_AXIS_ROW][i] == w) out.sane.push_back(enc_axis(CDA_AXIS_ROW, i));
    if (P.cnt[CDA_AXIS_COL][i] == w) out.sane.push_back(enc_axis(CDA_AXIS_COL, i));
  }
  std::vector<RepairOp>& ops = out.ops;
  ops.reserve(2 * W);
  out.vall.reserve(4 * W);
  out.blast.assign(w, -1);
  Presence Pq = P;  // the optimistic presence at the start of the next batch
  for (;;) {
    // replay one sweep: row i, then column i, for i = 0..w-1
    Presence Ps = Pq;
    const size_t first = ops.size();
    bool sweep_solved = true;
    for (int i = 0; i < w; i++) {
      for (int axis = 0; axis < 2; axis++) {
        const int n = Ps.cnt[axis][i];
        if (n == w) continue;
        if (n < K) {
          sweep_solved = false;
          continue;
        }
        ops.push_back(RepairOp{axis, i, {}});
        // orthogonal axis j is completed by this operation iff (i, j) is its only missing cell
        Ps.fill(axis, i, [&](int o, int j, int n) {
          if (n == w) ops.back().ortho.push_back(enc_axis(o, j));
        });
      }
    }
    if (ops.size() > 2 * W) return CDA_E_ARG;  // cannot happen: each operation completes an axis
    // batches of operations already decodable at the batch start
    for (size_t b0 = first; b0 < ops.size();) {
      size_t b1 = b0;
      while (b1 < ops.size() && Pq.cnt[ops[b1].axis][ops[b1].idx] >= K) b1++;
      if (b1 == b0) return CDA_E_ARG;  // cannot happen: the replay guarantees decodability in order
      RepairBatch bt{b0, b1, out.vall.size(), 0};
      for (size_t q = b0; q < b1; q++) {
        const RepairOp& op = ops[q];
        Pq.bytes(op.axis, op.idx, pres_out + q * W);  // the presence at the batch start
        out.vall.push_back(enc_axis(op.axis, op.idx));
        for (int o : op.ortho) out.vall.push_back(o);
        // blast[r] = the last batch that writes a cell of row r (a row operation on r, or a column operation
        // with (r, c) missing at its batch start)
        if (op.axis == CDA_AXIS_ROW)
          out.blast[op.idx] = (int)out.bat.size();
        else
          Pq.missing(CDA_AXIS_COL, op.idx, [&](int r) { out.blast[r] = (int)out.bat.size(); });
      }
      bt.v1 = out.vall.size();
      out.bat.push_back(bt);
      for (size_t q = b0; q < b1; q++) Pq.fill(ops[q].axis, ops[q].idx, [](int, int, int) {});
      b0 = b1;
    }
    if (sweep_solved) {
      out.solved = true;
      break;
    }
    if (ops.size() == first) break;  // no progress: unrepairable once every batch has passed
  }
  if (out.vall.size() > 4 * W) return CDA_E_ARG;  // each axis is verified by its own and at most one other op
  return CDA_OK;
}

namespace {
constexpr uint32_t kShare = 512;
constexpr uint32_t kFirstSparse = kShare - CDA_NAMESPACE_SIZE - 1 - 4;  // 478 (specs shares.md:31-60)
constexpr uint32_t kContSparse = kShare - CDA_NAMESPACE_SIZE - 1;       // 482
uint32_t round_up_pow2(uint32_t v) {
  uint32_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
}  // namespace

uint32_t sparse_shares_needed(uint64_t len) {
  if (len == 0) return 0;
  if (len <= kFirstSparse) return 1;
  return 1 + (uint32_t)((len - kFirstSparse + kContSparse - 1) / kContSparse);
}

uint32_t round_down_pow2(uint32_t v) {
  uint32_t p = 1;
  while (p * 2 <= v) p <<= 1;
  return p;
}

uint32_t subtree_width(uint32_t n, uint32_t threshold) {
  const uint32_t s = round_up_pow2(n / threshold + (n % threshold ? 1 : 0));
  uint32_t r = 0;
  while ((uint64_t)r * r < n) r++;
  return std::min(s, round_up_pow2(r));
}

void mountains(uint32_t n, uint32_t width, uint32_t first, std::vector<uint32_t>& out) {
  for (uint32_t j = 0, rem = n; rem;) {
    const uint32_t t = rem >= width ? width : round_down_pow2(rem);
    out.push_back(first + j);
    j += t;
    rem -= t;
  }
}

namespace {
void prove_rec(int h, uint32_t p, uint32_t s, uint32_t e, std::vector<std::pair<int, uint32_t>>& out) {
  const uint64_t lo = (uint64_t)p << h, hi = (uint64_t)(p + 1) << h;
  if (hi <= s || lo >= e) {
    out.emplace_back(h, p);
    return;
  }
  if (h == 0) return;  // a leaf inside the range
  prove_rec(h - 1, 2 * p, s, e, out);
  prove_rec(h - 1, 2 * p + 1, s, e, out);
}
}  // namespace

void prove_range(int L, uint32_t s, uint32_t e, std::vector<std::pair<int, uint32_t>>& out) {
  prove_rec(L, 0, s, e, out);
}

uint64_t segment_shares_needed(uint32_t kind, uint64_t len) {
  if (kind == CDA_SEG_PADDING || len == 0) return kind == CDA_SEG_PADDING ? 1 : 0;
  const uint64_t first = kind == CDA_SEG_COMPACT ? 474 : 478, cont = kind == CDA_SEG_COMPACT ? 478 : 482;
  return len <= first ? 1 : 1 + (len - first + cont - 1) / cont;
}

int check_square_plan(uint32_t k, uint32_t nseg, const cda_share_segment* segs, uint64_t data_len,
                      uint32_t nreserved) {
  if (!segs || nseg == 0) return CDA_E_ARG;
  uint64_t next = 0;
  for (uint32_t i = 0; i < nseg; i++) {
    const cda_share_segment& s = segs[i];
    if (s.kind > CDA_SEG_PADDING || s.first_share != next || s.nshares == 0) return CDA_E_ARG;
    if (s.share_version != 0) return CDA_E_SHARE_VERSION;  // appconsts.SupportedShareVersions = {0}
    if (s.kind != CDA_SEG_PADDING) {
      if (s.data_off > data_len || s.data_len > data_len - s.data_off || s.data_len > 0xFFFFFFFFull) return CDA_E_ARG;
      if (segment_shares_needed(s.kind, s.data_len) != s.nshares) return CDA_E_ARG;
    } else if (s.data_len != 0) {
      return CDA_E_ARG;
    }
    if (s.kind == CDA_SEG_COMPACT && ((uint64_t)s.reserved_off + s.nshares > nreserved)) return CDA_E_ARG;
    next += s.nshares;
  }
  return next == (uint64_t)k * k ? CDA_OK : CDA_E_ARG;
}

}  // namespace plan
}  // namespace cda
