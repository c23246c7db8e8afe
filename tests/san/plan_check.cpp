// plan_check.cpp — CPU check of libcda's host planners (celestia-app_amd/csrc/plan.cpp), built and run under
// AddressSanitizer + UndefinedBehaviorSanitizer by scripts/sanitize.sh (tests/test_sanitize.py runs it when
// asked).  Each planner is compared with a naive restatement written here, on random and edge-case inputs:
//
//   plan_repair          rsmt2d solveCrossword (v0.12.0, extendeddatacrossword.go: sweeps of "row i, then col i",
//                        an axis with >= k present cells is decoded) replayed on a byte matrix
//   sparse_shares_needed go-square shares.SparseSharesNeeded by share-by-share subtraction
//   subtree_width,       inclusion.SubTreeWidth / MerkleMountainRangeSizes by their definitions
//   mountains
//   prove_range          the leaves outside [s, e) covered by maximal subtrees, checked leaf by leaf
//   check_square_plan    random and corrupted share-layout plans (no UB on any field value)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../celestia-app_amd/csrc/plan.h"

using namespace cda::plan;

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      if (g_fail++ < 20) {                                 \
        fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        fprintf(stderr, __VA_ARGS__);                      \
        fprintf(stderr, "\n");                             \
      }                                                    \
    }                                                      \
  } while (0)

// ---- repair: the crossword order on a byte matrix ----
struct NaiveOp {
  int axis, idx;
  std::vector<int> ortho;
};
static int count_axis(const std::vector<uint8_t>& m, int w, int axis, int i) {
  int n = 0;
  for (int j = 0; j < w; j++) n += axis == CDA_AXIS_ROW ? m[(size_t)i * w + j] : m[(size_t)j * w + i];
  return n;
}
static uint8_t& cell(std::vector<uint8_t>& m, int w, int axis, int i, int j) {
  return axis == CDA_AXIS_ROW ? m[(size_t)i * w + j] : m[(size_t)j * w + i];
}
static bool naive_crossword(std::vector<uint8_t> m, int w, int K, std::vector<NaiveOp>& ops) {
  for (;;) {
    bool solved = true, progress = false;
    for (int i = 0; i < w; i++)
      for (int axis = 0; axis < 2; axis++) {
        const int n = count_axis(m, w, axis, i);
        if (n == w) continue;
        if (n < K) {
          solved = false;
          continue;
        }
        NaiveOp op{axis, i, {}};
        for (int j = 0; j < w; j++)
          if (!cell(m, w, axis, i, j) && count_axis(m, w, 1 - axis, j) == w - 1) op.ortho.push_back(enc_axis(1 - axis, j));
        for (int j = 0; j < w; j++) cell(m, w, axis, i, j) = 1;
        ops.push_back(op);
        progress = true;
      }
    if (solved) return true;
    if (!progress) return false;
  }
}

static void check_repair(const std::vector<uint8_t>& raw, int w, int K) {
  Presence P;
  P.init(w, raw.data());
  std::vector<uint8_t> present(raw.size());
  for (size_t i = 0; i < raw.size(); i++) present[i] = raw[i] != 0;
  for (int a = 0; a < 2; a++)  // the bitsets and counts against the byte matrix
    for (int i = 0; i < w; i++) {
      int n = 0;
      for (int j = 0; j < w; j++) {
        const bool want = a == CDA_AXIS_ROW ? present[(size_t)i * w + j] != 0 : present[(size_t)j * w + i] != 0;
        const bool got = (P.bits[a][(size_t)i * P.words + (j >> 6)] >> (j & 63)) & 1;
        CHECK(want == got, "presence bit axis %d (%d, %d) (w=%d)", a, i, j, w);
        n += want;
      }
      CHECK(P.cnt[a][i] == n, "presence count axis %d idx %d (w=%d)", a, i, w);
    }
  RepairPlan rp;
  std::vector<uint8_t> pres(2 * (size_t)w * w, 0xAA);
  const int rc = plan_repair(P, K, rp, pres.data());
  CHECK(rc == CDA_OK, "plan_repair rc %d (w=%d)", rc, w);
  if (rc) return;
  std::vector<NaiveOp> nops;
  const bool solved = naive_crossword(present, w, K, nops);
  CHECK(solved == rp.solved, "solved %d vs naive %d (w=%d)", rp.solved, solved, w);
  CHECK(nops.size() == rp.ops.size(), "ops %zu vs naive %zu (w=%d)", rp.ops.size(), nops.size(), w);
  for (size_t q = 0; q < nops.size() && q < rp.ops.size(); q++)
    CHECK(nops[q].axis == rp.ops[q].axis && nops[q].idx == rp.ops[q].idx && nops[q].ortho == rp.ops[q].ortho,
          "op %zu differs (w=%d)", q, w);
  // sanity axes: complete axes at the start, i ascending, row before column
  std::vector<int> sane;
  for (int i = 0; i < w; i++)
    for (int axis = 0; axis < 2; axis++)
      if (count_axis(present, w, axis, i) == w) sane.push_back(enc_axis(axis, i));
  CHECK(sane == rp.sane, "sanity axes differ (w=%d)", w);
  // batches partition the operations in order; each operation is decodable with the presence at its batch
  // start, which pres records; vall lists each operation's axis then its orthogonal completions
  std::vector<uint8_t> m = present;
  std::vector<int> blast(w, -1);
  size_t next_q = 0, next_v = 0;
  for (size_t b = 0; b < rp.bat.size(); b++) {
    const RepairBatch& bt = rp.bat[b];
    CHECK(bt.q0 == next_q && bt.q1 > bt.q0 && bt.v0 == next_v && bt.v1 >= bt.v0, "batch %zu bounds (w=%d)", b, w);
    if (bt.q0 != next_q || bt.q1 <= bt.q0 || bt.q1 > rp.ops.size()) return;
    size_t v = bt.v0;
    for (size_t q = bt.q0; q < bt.q1; q++) {
      const RepairOp& op = rp.ops[q];
      CHECK(count_axis(m, w, op.axis, op.idx) >= K, "op %zu not decodable at its batch start (w=%d)", q, w);
      for (int j = 0; j < w; j++) {
        const uint8_t want = cell(m, w, op.axis, op.idx, j);
        CHECK(pres[q * w + j] == want, "pres of op %zu cell %d (w=%d)", q, j, w);
        if (!want) blast[op.axis == CDA_AXIS_ROW ? op.idx : j] = (int)b;
      }
      if (op.axis == CDA_AXIS_ROW) blast[op.idx] = (int)b;
      CHECK(v < rp.vall.size() && rp.vall[v] == enc_axis(op.axis, op.idx), "vall own axis, op %zu (w=%d)", q, w);
      v++;
      for (int o : op.ortho) {
        CHECK(v < rp.vall.size() && rp.vall[v] == o, "vall ortho, op %zu (w=%d)", q, w);
        v++;
      }
    }
    CHECK(v == bt.v1, "batch %zu vall end (w=%d)", b, w);
    for (size_t q = bt.q0; q < bt.q1; q++)
      for (int j = 0; j < w; j++) cell(m, w, rp.ops[q].axis, rp.ops[q].idx, j) = 1;
    next_q = bt.q1;
    next_v = bt.v1;
  }
  CHECK(next_q == rp.ops.size(), "batches cover %zu of %zu ops (w=%d)", next_q, rp.ops.size(), w);
  CHECK(blast == rp.blast, "blast differs (w=%d)", w);
  CHECK(rp.ops.size() <= 2 * (size_t)w && rp.vall.size() <= 4 * (size_t)w, "bounds (w=%d)", w);
}

static void repair_cases(std::mt19937_64& rng) {
  int ncase = 0;
  for (int k = 1; k <= 128; k *= 2) {
    const int w = 2 * k;
    const int reps = k <= 16 ? 60 : (k <= 64 ? 12 : 4);
    for (int r = 0; r < reps; r++) {
      std::vector<uint8_t> p((size_t)w * w);
      const int mode = r % 6;
      const double keep = mode == 0 ? 0.25 : mode == 1 ? 0.5 : mode == 2 ? 0.7 : 0.9;
      for (auto& x : p) x = (rng() % 1000) < keep * 1000 ? (uint8_t)(1 + rng() % 255) : 0;  // any nonzero byte = present
      if (mode == 4) {  // the minimal repairable pattern: Q0 present only
        for (int i = 0; i < w; i++)
          for (int j = 0; j < w; j++) p[(size_t)i * w + j] = i < k && j < k;
      } else if (mode == 5) {  // an unrepairable corner: (k + 1) x (k + 1) missing
        for (auto& x : p) x = 1;
        for (int i = 0; i <= k && i < w; i++)
          for (int j = 0; j <= k && j < w; j++) p[(size_t)i * w + j] = 0;
      }
      check_repair(p, w, k);
      ncase++;
    }
    std::vector<uint8_t> full((size_t)w * w, 1), none((size_t)w * w, 0);
    check_repair(full, w, k);
    check_repair(none, w, k);
    ncase += 2;
  }
  printf("plan_repair: %d presence maps\n", ncase);
}

// ---- blob commitments ----
static void blob_cases(std::mt19937_64& rng) {
  int n = 0;
  for (uint64_t len = 0; len < 20000; len += 1 + rng() % 97, n++) {
    uint64_t shares = 0;
    for (int64_t rem = (int64_t)len; rem > 0; shares++) rem -= shares == 0 ? 478 : 482;
    CHECK(sparse_shares_needed(len) == shares, "sparse_shares_needed(%llu)", (unsigned long long)len);
  }
  CHECK(sparse_shares_needed(0xFFFFFFFFull) == 1 + (0xFFFFFFFFull - 478 + 481) / 482, "sparse_shares_needed(max)");
  for (uint32_t shares = 1; shares < 5000; shares += 1 + (uint32_t)(rng() % 13))
    for (uint32_t thr : {1u, 2u, 7u, 64u, 128u}) {
      uint32_t c = 1;
      while (c < (shares + thr - 1) / thr) c <<= 1;
      uint32_t sq = 1;  // BlobMinSquareSize: the smallest power of two whose square holds the shares
      while ((uint64_t)sq * sq < shares) sq <<= 1;
      const uint32_t want = c < sq ? c : sq, got = subtree_width(shares, thr);
      CHECK(got == want, "subtree_width(%u, %u) = %u, want %u", shares, thr, got, want);
      std::vector<uint32_t> starts;
      mountains(shares, got, 100, starts);
      uint32_t pos = 100;
      for (size_t i = 0; i < starts.size(); i++) {
        CHECK(starts[i] == pos, "mountain %zu start", i);
        const uint32_t end = i + 1 < starts.size() ? starts[i + 1] : 100 + shares;
        const uint32_t sz = end - starts[i];
        const uint32_t rem = 100 + shares - starts[i];
        uint32_t want_sz = 1;  // MerkleMountainRangeSizes: full-width mountains, then the largest power of two left
        while (want_sz * 2 <= rem) want_sz *= 2;
        if (rem >= got) want_sz = got;
        CHECK(sz == want_sz, "mountain size %u, want %u (width %u)", sz, want_sz, got);
        pos = end;
      }
      n++;
    }
  printf("blob planners: %d cases\n", n);
}

// ---- range proofs ----
static void proof_cases(std::mt19937_64& rng) {
  int n = 0;
  for (int L = 0; L <= 10; L++) {
    const uint32_t nl = 1u << L;
    for (int r = 0; r < 200; r++, n++) {
      uint32_t s = (uint32_t)(rng() % nl), e = s + 1 + (uint32_t)(rng() % (nl - s));
      if (r == 0) s = 0, e = nl;
      std::vector<std::pair<int, uint32_t>> nodes;
      prove_range(L, s, e, nodes);
      std::vector<int> cover(nl, 0);
      uint32_t last_end = 0;
      for (auto& [h, p] : nodes) {
        CHECK(h >= 0 && h <= L && p < (nl >> h), "node (%d, %u) outside the tree", h, p);
        const uint32_t lo = p << h, hi = (p + 1) << h;
        CHECK(lo >= last_end, "nodes not left to right");
        last_end = hi;
        for (uint32_t x = lo; x < hi && x < nl; x++) cover[x]++;
        // maximal: the parent intersects [s, e)
        if (h < L) {
          const uint32_t plo = (p >> 1) << (h + 1), phi = ((p >> 1) + 1) << (h + 1);
          CHECK(!(phi <= s || plo >= e), "node (%d, %u) not maximal", h, p);
        }
      }
      for (uint32_t x = 0; x < nl; x++) CHECK(cover[x] == (x < s || x >= e ? 1 : 0), "leaf %u coverage (L=%d)", x, L);
      CHECK(nodes.size() <= 2 * (size_t)L, "too many nodes (L=%d)", L);
    }
  }
  printf("prove_range: %d ranges\n", n);
}

// ---- square plans ----
static void square_cases(std::mt19937_64& rng) {
  int n = 0, ok = 0;
  for (int r = 0; r < 4000; r++, n++) {
    const uint32_t k = 1u << (rng() % 6);
    std::vector<cda_share_segment> segs;
    uint64_t next = 0, data_off = 0;
    uint32_t reserved = 0;
    while (next < (uint64_t)k * k) {
      cda_share_segment s;
      memset(&s, 0, sizeof s);
      s.kind = (uint32_t)(rng() % 3);
      s.first_share = (uint32_t)next;
      s.data_len = s.kind == CDA_SEG_PADDING ? 0 : 1 + rng() % 3000;
      s.nshares = (uint32_t)segment_shares_needed(s.kind, s.data_len);
      if (next + s.nshares > (uint64_t)k * k) {
        s.kind = CDA_SEG_PADDING;
        s.data_len = 0;
        s.nshares = 1;
      }
      s.data_off = data_off;
      data_off += s.data_len;
      if (s.kind == CDA_SEG_COMPACT) {
        s.reserved_off = reserved;
        reserved += s.nshares;
      }
      next += s.nshares;
      segs.push_back(s);
    }
    const int mut = r % 4 == 0 ? 0 : (int)(rng() % 8);
    if (mut && !segs.empty()) {  // corrupt one field with an extreme value
      cda_share_segment& s = segs[rng() % segs.size()];
      const uint64_t big = rng() % 2 ? ~0ull : (1ull << 63) + rng() % 1000;
      switch (mut) {
        case 1: s.data_off = big; break;
        case 2: s.data_len = big; break;
        case 3: s.nshares = (uint32_t)big; break;
        case 4: s.first_share = (uint32_t)big; break;
        case 5: s.reserved_off = (uint32_t)big; break;
        case 6: s.share_version = 1 + (uint32_t)(rng() % 255); break;
        default: s.kind = (uint32_t)big; break;
      }
    }
    const int rc = check_square_plan(k, (uint32_t)segs.size(), segs.data(), data_off, reserved);
    if (!mut) CHECK(rc == CDA_OK, "valid plan rejected (%d)", rc);
    ok += rc == CDA_OK;
  }
  CHECK(check_square_plan(4, 0, nullptr, 0, 0) == CDA_E_ARG, "empty plan");
  printf("check_square_plan: %d plans (%d accepted)\n", n, ok);
}

int main() {
  std::mt19937_64 rng(0xC0FFEE);
  repair_cases(rng);
  blob_cases(rng);
  proof_cases(rng);
  square_cases(rng);
  if (g_fail) {
    fprintf(stderr, "plan_check: %d failures\n", g_fail);
    return 1;
  }
  printf("plan_check: all passed\n");
  return 0;
}
