// plan.h — the host-only planners behind the C ABI: pure C++ with no HIP runtime dependency, so they build and
// run under AddressSanitizer / UndefinedBehaviorSanitizer on the CPU (tests/san, scripts/sanitize.sh) exactly as
// libcda compiles them.
//
//   Presence / plan_repair   rsmt2d (*ExtendedDataSquare).Repair's crossword order (repair.cpp)
//   sparse_shares_needed,    go-square shares.SparseSharesNeeded, inclusion.SubTreeWidth and
//   subtree_width, mountains MerkleMountainRangeSizes (inclusion.cpp, cda_blob_commitments)
//   prove_range              nmt buildRangeProof on a perfect tree (inclusion.cpp, cda_share_inclusion_proof)
//   check_square_plan        the share-layout plan of cda_build_ods_device (square.cpp)
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <utility>
#include <vector>

#include "../../include/cda.h"

namespace cda {
namespace plan {

inline int enc_axis(int axis, int idx) { return (axis << 24) | idx; }

// Presence of the w x w cells as row and column bitsets with per-axis counts: a crossword step
// costs O(w / 64 + cells it fills) on the host instead of O(w) byte scans.
struct Presence {
  int w = 0, words = 0;
  uint64_t full = 0;              // valid bits of each word (w < 64: one partial word)
  std::vector<uint64_t> bits[2];  // [axis][idx * words + j / 64] bit j % 64 = cell j of axis idx present
  std::vector<int> cnt[2];        // present cells per axis
  void init(int w_, const uint8_t* p);
  // f(j) for every missing cell j of axis (a, idx), j ascending
  template <class F>
  void missing(int a, int idx, F f) const {
    const uint64_t* b = bits[a].data() + (size_t)idx * words;
    for (int wd = 0; wd < words; wd++)
      for (uint64_t m = ~b[wd] & full; m; m &= m - 1) f(wd * 64 + __builtin_ctzll(m));
  }
  // mark every cell of axis (a, idx) present; f(o, j, n) for each cell (a, idx) x (o = 1 - a, j) that was
  // missing, n = axis (o, j)'s new count, j ascending
  template <class F>
  void fill(int a, int idx, F f) {
    const int o = 1 - a;
    uint64_t* b = bits[a].data() + (size_t)idx * words;
    const uint64_t bit = 1ull << (idx & 63);
    for (int wd = 0; wd < words; wd++) {
      for (uint64_t m = ~b[wd] & full; m; m &= m - 1) {
        const int j = wd * 64 + __builtin_ctzll(m);
        bits[o][(size_t)j * words + (idx >> 6)] |= bit;
        f(o, j, ++cnt[o][j]);
      }
      b[wd] = full;
    }
    cnt[a][idx] = w;
  }
  void fill(int a, int idx) {
    fill(a, idx, [](int, int, int) {});
  }
  void bytes(int a, int idx, uint8_t* out) const;  // presence of axis (a, idx)'s cells, one byte (0/1) each
};

// One crossword operation: decode axis (axis, idx); `ortho` = the orthogonal axes it completes (enc_axis codes).
struct RepairOp {
  int axis, idx;
  std::vector<int> ortho;
};
// Operations [q0, q1) are all decodable at the batch start; their verified axes are vall[v0, v1).
struct RepairBatch {
  size_t q0, q1, v0, v1;
};
struct RepairPlan {
  std::vector<int> sane;  // complete axes at the start (prerepairSanityCheck): i ascending, row before column
  std::vector<RepairOp> ops;
  std::vector<RepairBatch> bat;
  std::vector<int> vall;  // per batch: each operation's own axis, then its orthogonal completions
  std::vector<int> blast;  // per row: the last batch writing a cell of it (-1: none)
  bool solved = false;     // every axis complete after the last sweep (if every check passes)
};

// rsmt2d solveCrossword (v0.12.0): sweeps of "row i, then column i" for i = 0..w-1 on the optimistic presence
// (every check passes) starting from P; an incomplete axis with >= K present cells is an operation.  pres_out
// (capacity 2 * w * w bytes) receives, per operation, its axis' presence at its batch start.  Returns CDA_OK or
// CDA_E_ARG (a bound violated: cannot happen for a w x w presence map).
int plan_repair(const Presence& P, int K, RepairPlan& out, uint8_t* pres_out);

// go-square shares.SparseSharesNeeded (specs shares.md:31-60: 478 B in the first share, 482 after)
uint32_t sparse_shares_needed(uint64_t len);
// inclusion.SubTreeWidth: min(RoundUpPowerOfTwo(ceil(n / threshold)), BlobMinSquareSize(n))
uint32_t subtree_width(uint32_t n, uint32_t threshold);
// inclusion MerkleMountainRangeSizes: append the first share of every mountain of n shares of width `width`
void mountains(uint32_t n, uint32_t width, uint32_t first, std::vector<uint32_t>& out);
uint32_t round_down_pow2(uint32_t v);

// nmt buildRangeProof on a perfect tree of 2^L leaves: the maximal subtrees outside [s, e), left to right, as
// (height, position) pairs.
void prove_range(int L, uint32_t s, uint32_t e, std::vector<std::pair<int, uint32_t>>& out);

// shares a sequence of `len` bytes needs (compact: 474 / 478 per share; sparse: 478 / 482; padding: 1)
uint64_t segment_shares_needed(uint32_t kind, uint64_t len);
// cda_build_ods_device's plan check: the segments tile [0, k*k) in order, every payload lies inside `data`
// and fits its sequence.  CDA_OK, CDA_E_ARG or CDA_E_SHARE_VERSION.
int check_square_plan(uint32_t k, uint32_t nseg, const cda_share_segment* segs, uint64_t data_len,
                      uint32_t nreserved);

}  // namespace plan
}  // namespace cda
