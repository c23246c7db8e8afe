// gf8_prog_check — host check of the RS encoder's compile-time multiply programs (csrc/gf8_const.h).
// For every skew index i of the GF(2^8) FFT (kCpoly8, the constants the g2 encoder multiplies by) it runs the
// XOR3 program of gf8_prog() on the bit-planes of every byte x and prints the 256 products as one hex line;
// tests/test_gf8_prog.py compares each line with the oracle's Leopard multiply, x * exp(skew[i])
// (oracle/leopard.c).  Built with hipcc (constexpr functions of gf8_const.h are host-callable).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../celestia-app_amd/csrc/gf8_const.h"

static unsigned run_prog(const cda::Gf8Prog& p, unsigned x) {
  unsigned V[24] = {}, X[8] = {};
  for (int j = 0; j < 8; j++) V[j] = (x >> j) & 1u;
  for (int i = 0; i < p.n; i++) {
    unsigned t = V[p.s[i][0]];
    if (p.s[i][1] >= 0) t ^= V[p.s[i][1]];
    if (p.s[i][2] >= 0) t ^= V[p.s[i][2]];
    if (p.dst[i] < 0)
      V[-p.dst[i]] = t;
    else
      X[p.dst[i]] ^= t;
  }
  unsigned r = 0;
  for (int j = 0; j < 8; j++) r |= (X[j] & 1u) << j;
  return r;
}

int main() {
  int ops = 0, maxops = 0;
  for (int i = 0; i < 255; i++) {
    const unsigned c = cda::kCpoly8.v[i];
    const cda::Gf8Prog p = cda::gf8_prog(c);
    ops += p.n;
    maxops = p.n > maxops ? p.n : maxops;
    printf("%d %u ", i, c);
    for (unsigned x = 0; x < 256; x++) printf("%02x", c ? run_prog(p, x) : x * 0u);
    printf("\n");
  }
  fprintf(stderr, "programs: %d ops over 255 constants, max %d\n", ops, maxops);
  return 0;
}
