// leopard_tables.cpp — host construction of the Leopard GF(2^8)/GF(2^16) tables
// used by the device kernels (product code; the oracle has its own restatement).
//
// Table construction follows klauspost/reedsolomon v1.12.1 initConstants8/16 and
// initFFT8/16 (upstream, go.mod:153): LFSR exp/log, Cantor-basis conversion,
// then the FFT skew vector.
#include <mutex>
#include <vector>

#include "cda_internal.h"

namespace cda {
namespace {

struct Field {
  int bits = 0;
  unsigned order = 0, modulus = 0;
  std::vector<uint16_t> exp_t, log_t, skew;
  LeoTables view{};

  unsigned add_mod(unsigned a, unsigned b) const {
    const unsigned s = a + b;
    return (s + (s >> bits)) & modulus;
  }
  unsigned mul_log(unsigned a, unsigned log_b) const { return a == 0 ? 0 : exp_t[add_mod(log_t[a], log_b)]; }

  void build(int nbits, unsigned poly, const uint16_t* basis) {
    bits = nbits;
    order = 1u << bits;
    modulus = order - 1;
    exp_t.assign(order, 0);
    log_t.assign(order, 0);
    skew.assign(modulus, 0);
    unsigned state = 1;
    for (unsigned i = 0; i < modulus; i++) {
      exp_t[state] = (uint16_t)i;
      state <<= 1;
      if (state >= order) state ^= poly;
    }
    exp_t[0] = (uint16_t)modulus;
    log_t[0] = 0;
    for (int i = 0; i < bits; i++) {
      const unsigned width = 1u << i;
      for (unsigned j = 0; j < width; j++) log_t[j + width] = log_t[j] ^ basis[i];
    }
    for (unsigned i = 0; i < order; i++) log_t[i] = exp_t[log_t[i]];
    for (unsigned i = 0; i < order; i++) exp_t[log_t[i]] = (uint16_t)i;
    exp_t[modulus] = exp_t[0];

    std::vector<unsigned> temp(bits > 1 ? bits - 1 : 1);
    for (int i = 1; i < bits; i++) temp[i - 1] = 1u << i;
    for (int m = 0; m < bits - 1; m++) {
      const unsigned step = 1u << (m + 1);
      skew[(1u << m) - 1] = 0;
      for (int i = m; i < bits - 1; i++) {
        const unsigned s = 1u << (i + 1);
        for (unsigned j = (1u << m) - 1; j < s; j += step) skew[j + s] = skew[j] ^ (uint16_t)temp[i];
      }
      temp[m] = modulus - log_t[mul_log(temp[m], log_t[temp[m] ^ 1])];
      for (int i = m + 1; i < bits - 1; i++) temp[i] = mul_log(temp[i], add_mod(log_t[temp[i] ^ 1], temp[m]));
    }
    for (unsigned i = 0; i < modulus; i++) skew[i] = log_t[skew[i]];
    view.bits = bits;
    view.order = order;
    view.modulus = modulus;
    view.exp_t = exp_t.data();
    view.log_t = log_t.data();
    view.skew = skew.data();
  }
};

const uint16_t kCantor8[8] = {1, 214, 152, 146, 86, 200, 88, 230};
const uint16_t kCantor16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

Field g_f8, g_f16;
std::once_flag g_once;

void build_all() {
  g_f8.build(8, 0x11D, kCantor8);
  g_f16.build(16, 0x1002D, kCantor16);
}

}  // namespace

const LeoTables& leo_tables(int bits) {
  std::call_once(g_once, build_all);
  return bits == 8 ? g_f8.view : g_f16.view;
}

uint64_t leo8_colbits(unsigned log_m) {
  leo_tables(8);
  if (log_m >= 255) return 0;
  uint64_t v = 0;
  for (int b = 0; b < 8; b++) v |= (uint64_t)g_f8.mul_log(1u << b, log_m) << (8 * b);
  return v;
}

void leo16_colbits(unsigned log_m, uint16_t out[16]) {
  leo_tables(16);
  for (int b = 0; b < 16; b++) out[b] = log_m >= 65535 ? 0 : (uint16_t)g_f16.mul_log(1u << b, log_m);
}

}  // namespace cda
