/*
 * leopard.c — CPU restatement of klauspost/reedsolomon v1.12.1 Leopard GF(2^8) /
 * GF(2^16) systematic encoding as called by rsmt2d v0.12.0 LeoRSCodec
 * (reedsolomon.New(k, k, WithLeopardGF(true)); codec selected at
 * /root/reference/pkg/appconsts/global_consts.go:92, called from
 * pkg/da/data_availability_header.go:74).
 *
 * TEST INFRASTRUCTURE ONLY (checker + CPU baseline).  Not part of libcda.
 *
 * The upstream module is not vendored in /root/reference (go.mod:153,
 * go.sum:945-946); this restates its published algorithm (SURVEY.md
 * Appendix A): LFSR + Cantor-basis log/exp tables, FFT skew table, IFFT-DIT
 * over the data placed at points m..m+k-1 followed by FFT-DIT to points
 * 0..k-1 ("mtrunc" loop bounds, multiplier log == modulus => XOR only).
 *
 * ora_leo_decode is deliberately NOT the Leopard error-locator path: it is
 * Lagrange interpolation in Leopard's field, an independent decoder.  Because
 * the code is MDS every correct decoder returns identical bytes, so agreement
 * between this decoder and the FFT encoder pins the closed form used on the GPU.
 * ora_leo_decode_fft restates klauspost's own reconstruct (error locators,
 * IFFT, formal derivative, FFT: O(k log k) per shard byte) -- the CPU baseline
 * of the repair path (bench.py cpu_baseline.repair_c4), checked against the
 * Lagrange decoder in tests/test_oracle.py.
 */
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "oracle.h"

#if defined(__x86_64__)
#include <immintrin.h>
#define ORA_HAVE_X86 1
#endif

/* ------------------------------------------------------------------ */
/* Field tables                                                        */
/* ------------------------------------------------------------------ */

typedef struct {
  int bits;
  unsigned order, modulus, poly;
  uint16_t* exp_t; /* [order] */
  uint16_t* log_t; /* [order] */
  uint16_t* skew;  /* [modulus] */
} field_t;

static field_t F8, F16;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static const uint16_t kCantor8[8] = {1, 214, 152, 146, 86, 200, 88, 230};
static const uint16_t kCantor16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E,
                                       0x914C, 0x4012, 0x6C98, 0x10D8, 0x6A72, 0xB900,
                                       0xFDB8, 0xFB34, 0xFF38, 0x991E};

static inline unsigned add_mod(const field_t* f, unsigned a, unsigned b) {
  unsigned s = a + b;
  return (s + (s >> f->bits)) & f->modulus;
}

static inline unsigned mul_log(const field_t* f, unsigned a, unsigned log_b) {
  if (a == 0) return 0;
  return f->exp_t[add_mod(f, f->log_t[a], log_b)];
}

static void init_field(field_t* f, int bits, unsigned poly, const uint16_t* basis) {
  f->bits = bits;
  f->order = 1u << bits;
  f->modulus = f->order - 1;
  f->poly = poly;
  f->exp_t = (uint16_t*)calloc(f->order, sizeof(uint16_t));
  f->log_t = (uint16_t*)calloc(f->order, sizeof(uint16_t));
  f->skew = (uint16_t*)calloc(f->modulus, sizeof(uint16_t));
  /* 1. LFSR table */
  unsigned state = 1;
  for (unsigned i = 0; i < f->modulus; i++) {
    f->exp_t[state] = (uint16_t)i;
    state <<= 1;
    if (state >= f->order) state ^= poly;
  }
  f->exp_t[0] = (uint16_t)f->modulus;
  /* 2. Cantor basis */
  f->log_t[0] = 0;
  for (int i = 0; i < bits; i++) {
    unsigned width = 1u << i;
    for (unsigned j = 0; j < width; j++) f->log_t[j + width] = f->log_t[j] ^ basis[i];
  }
  for (unsigned i = 0; i < f->order; i++) f->log_t[i] = f->exp_t[f->log_t[i]];
  for (unsigned i = 0; i < f->order; i++) f->exp_t[f->log_t[i]] = (uint16_t)i;
  f->exp_t[f->modulus] = f->exp_t[0];
  /* FFT skew */
  unsigned temp[16];
  for (int i = 1; i < bits; i++) temp[i - 1] = 1u << i;
  for (int m = 0; m < bits - 1; m++) {
    unsigned step = 1u << (m + 1);
    f->skew[(1u << m) - 1] = 0;
    for (int i = m; i < bits - 1; i++) {
      unsigned s = 1u << (i + 1);
      for (unsigned j = (1u << m) - 1; j < s; j += step) f->skew[j + s] = f->skew[j] ^ (uint16_t)temp[i];
    }
    temp[m] = f->modulus - f->log_t[mul_log(f, temp[m], f->log_t[temp[m] ^ 1])];
    for (int i = m + 1; i < bits - 1; i++) {
      unsigned sum = add_mod(f, f->log_t[temp[i] ^ 1], temp[m]);
      temp[i] = mul_log(f, temp[i], sum);
    }
  }
  for (unsigned i = 0; i < f->modulus; i++) f->skew[i] = f->log_t[f->skew[i]];
}

static void init_all(void) {
  init_field(&F8, 8, 0x11D, kCantor8);
  init_field(&F16, 16, 0x1002D, kCantor16);
}

static const field_t* field_for_bits(int bits) {
  pthread_once(&g_once, init_all);
  return bits == 8 ? &F8 : &F16;
}

int ora_leo_bits_for(int k) { return (2 * k > 256) ? 16 : 8; }

unsigned ora_leo_mul(int bits, unsigned a, unsigned b) {
  const field_t* f = field_for_bits(bits);
  if (a == 0 || b == 0) return 0;
  return mul_log(f, a, f->log_t[b]);
}
int ora_leo_skew(int bits, int i) { return field_for_bits(bits)->skew[i]; }
int ora_leo_log(int bits, unsigned a) { return field_for_bits(bits)->log_t[a]; }
int ora_leo_exp(int bits, unsigned l) { return field_for_bits(bits)->exp_t[l]; }

/* ------------------------------------------------------------------ */
/* Vector kernels: x ^= y, x ^= y * exp(log_m)                         */
/* ------------------------------------------------------------------ */

static void slice_xor(uint8_t* out, const uint8_t* in, size_t n) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t a, b;
    memcpy(&a, out + i, 8);
    memcpy(&b, in + i, 8);
    a ^= b;
    memcpy(out + i, &a, 8);
  }
  for (; i < n; i++) out[i] ^= in[i];
}

#ifdef ORA_HAVE_X86
static int g_avx2 = -1;
static int have_avx2(void) {
  if (g_avx2 < 0) g_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
  return g_avx2;
}

__attribute__((target("avx2"))) static void muladd8_avx2(uint8_t* x, const uint8_t* y, size_t n,
                                                         const uint8_t lo[16], const uint8_t hi[16]) {
  __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)lo));
  __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)hi));
  __m256i m4 = _mm256_set1_epi8(0x0F);
  for (size_t i = 0; i < n; i += 32) {
    __m256i v = _mm256_loadu_si256((const __m256i*)(y + i));
    __m256i l = _mm256_and_si256(v, m4);
    __m256i h = _mm256_and_si256(_mm256_srli_epi64(v, 4), m4);
    __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
    __m256i o = _mm256_loadu_si256((const __m256i*)(x + i));
    _mm256_storeu_si256((__m256i*)(x + i), _mm256_xor_si256(o, p));
  }
}

/* FF16 element t of a 64-B block = byte[t] | byte[t+32] << 8. */
__attribute__((target("avx2"))) static void muladd16_avx2(uint8_t* x, const uint8_t* y, size_t n,
                                                          const uint8_t tab[8][16]) {
  __m256i t[8];
  for (int i = 0; i < 8; i++) t[i] = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)tab[i]));
  __m256i m4 = _mm256_set1_epi8(0x0F);
  for (size_t i = 0; i < n; i += 64) {
    __m256i vl = _mm256_loadu_si256((const __m256i*)(y + i));
    __m256i vh = _mm256_loadu_si256((const __m256i*)(y + i + 32));
    __m256i n0 = _mm256_and_si256(vl, m4), n1 = _mm256_and_si256(_mm256_srli_epi64(vl, 4), m4);
    __m256i n2 = _mm256_and_si256(vh, m4), n3 = _mm256_and_si256(_mm256_srli_epi64(vh, 4), m4);
    /* tab[2q] = low byte of product contribution of nibble q, tab[2q+1] = high byte */
    __m256i pl = _mm256_xor_si256(_mm256_xor_si256(_mm256_shuffle_epi8(t[0], n0), _mm256_shuffle_epi8(t[2], n1)),
                                  _mm256_xor_si256(_mm256_shuffle_epi8(t[4], n2), _mm256_shuffle_epi8(t[6], n3)));
    __m256i ph = _mm256_xor_si256(_mm256_xor_si256(_mm256_shuffle_epi8(t[1], n0), _mm256_shuffle_epi8(t[3], n1)),
                                  _mm256_xor_si256(_mm256_shuffle_epi8(t[5], n2), _mm256_shuffle_epi8(t[7], n3)));
    __m256i ol = _mm256_loadu_si256((const __m256i*)(x + i));
    __m256i oh = _mm256_loadu_si256((const __m256i*)(x + i + 32));
    _mm256_storeu_si256((__m256i*)(x + i), _mm256_xor_si256(ol, pl));
    _mm256_storeu_si256((__m256i*)(x + i + 32), _mm256_xor_si256(oh, ph));
  }
}
#endif

/* x[] ^= y[] * exp(log_m)   (refMulAdd8 / refMulAdd in klauspost) */
static void mul_add(const field_t* f, uint8_t* x, const uint8_t* y, unsigned log_m, size_t n) {
  if (f->bits == 8) {
    uint8_t lo[16], hi[16];
    for (unsigned i = 0; i < 16; i++) {
      lo[i] = (uint8_t)mul_log(f, i, log_m);
      hi[i] = (uint8_t)mul_log(f, i << 4, log_m);
    }
#ifdef ORA_HAVE_X86
    if (have_avx2() && (n % 32) == 0) {
      muladd8_avx2(x, y, n, lo, hi);
      return;
    }
#endif
    for (size_t i = 0; i < n; i++) x[i] ^= lo[y[i] & 15] ^ hi[y[i] >> 4];
  } else {
    uint16_t nib[4][16];
    for (unsigned q = 0; q < 4; q++)
      for (unsigned i = 0; i < 16; i++) nib[q][i] = (uint16_t)mul_log(f, i << (4 * q), log_m);
#ifdef ORA_HAVE_X86
    if (have_avx2()) {
      uint8_t tab[8][16];
      for (int q = 0; q < 4; q++)
        for (int i = 0; i < 16; i++) {
          tab[2 * q][i] = (uint8_t)(nib[q][i] & 0xFF);
          tab[2 * q + 1][i] = (uint8_t)(nib[q][i] >> 8);
        }
      muladd16_avx2(x, y, n, (const uint8_t(*)[16])tab);
      return;
    }
#endif
    for (size_t b = 0; b < n; b += 64) {
      for (int t = 0; t < 32; t++) {
        unsigned v = y[b + t] | ((unsigned)y[b + t + 32] << 8);
        unsigned p = nib[0][v & 15] ^ nib[1][(v >> 4) & 15] ^ nib[2][(v >> 8) & 15] ^ nib[3][v >> 12];
        x[b + t] ^= (uint8_t)p;
        x[b + t + 32] ^= (uint8_t)(p >> 8);
      }
    }
  }
}

/* ------------------------------------------------------------------ */
/* Butterflies                                                         */
/* ------------------------------------------------------------------ */

/* IFFT2: y ^= x; x ^= y * exp(lm)   (lm == modulus => XOR only) */
static inline void ifft2(const field_t* f, uint8_t* x, uint8_t* y, unsigned lm, size_t n) {
  slice_xor(y, x, n);
  if (lm != f->modulus) mul_add(f, x, y, lm, n);
}
/* FFT2: x ^= y * exp(lm); y ^= x */
static inline void fft2(const field_t* f, uint8_t* x, uint8_t* y, unsigned lm, size_t n) {
  if (lm != f->modulus) mul_add(f, x, y, lm, n);
  slice_xor(y, x, n);
}

static void ifft_dit_encoder(const field_t* f, uint8_t** work, int mtrunc, int m, const uint16_t* skew_lut,
                             size_t n) {
  int dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (int r = 0; r < mtrunc; r += dist4) {
      int iend = r + dist;
      unsigned l01 = skew_lut[iend], l02 = skew_lut[iend + dist], l23 = skew_lut[iend + 2 * dist];
      for (int i = r; i < iend; i++) {
        ifft2(f, work[i], work[i + dist], l01, n);
        ifft2(f, work[i + 2 * dist], work[i + 3 * dist], l23, n);
        ifft2(f, work[i], work[i + 2 * dist], l02, n);
        ifft2(f, work[i + dist], work[i + 3 * dist], l02, n);
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    unsigned logm = skew_lut[dist];
    for (int i = 0; i < dist; i++) ifft2(f, work[i], work[i + dist], logm, n);
  }
}

static void fft_dit(const field_t* f, uint8_t** work, int mtrunc, int m, const uint16_t* skew, size_t n) {
  int dist4 = m, dist = m >> 2;
  while (dist != 0) {
    for (int r = 0; r < mtrunc; r += dist4) {
      int iend = r + dist;
      unsigned l01 = skew[iend - 1], l02 = skew[iend + dist - 1], l23 = skew[iend + 2 * dist - 1];
      for (int i = r; i < iend; i++) {
        fft2(f, work[i], work[i + 2 * dist], l02, n);
        fft2(f, work[i + dist], work[i + 3 * dist], l02, n);
        fft2(f, work[i], work[i + dist], l01, n);
        fft2(f, work[i + 2 * dist], work[i + 3 * dist], l23, n);
      }
    }
    dist4 = dist;
    dist >>= 2;
  }
  if (dist4 == 2) {
    for (int r = 0; r < mtrunc; r += 2) fft2(f, work[r], work[r + 1], skew[r], n);
  }
}

static int ceil_pow2(int n) {
  int m = 1;
  while (m < n) m <<= 1;
  return m;
}

int ora_leo_encode(int k, size_t shard_len, const uint8_t* const* data, uint8_t* const* parity) {
  if (k <= 0 || k > 32768) return ORA_E_ARG;
  if (shard_len == 0 || shard_len % 64 != 0) return ORA_E_SHARD_SIZE;
  const field_t* f = field_for_bits(ora_leo_bits_for(k));
  int m = ceil_pow2(k);
  uint8_t* buf = (uint8_t*)aligned_alloc(64, (size_t)m * shard_len);
  uint8_t** work = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)m);
  for (int i = 0; i < m; i++) work[i] = buf + (size_t)i * shard_len;
  int mtrunc = k < m ? k : m;
  for (int i = 0; i < mtrunc; i++) memcpy(work[i], data[i], shard_len);
  for (int i = mtrunc; i < m; i++) memset(work[i], 0, shard_len);
  ifft_dit_encoder(f, work, mtrunc, m, f->skew + (m - 1), shard_len);
  fft_dit(f, work, k, m, f->skew, shard_len);
  for (int i = 0; i < k; i++) memcpy(parity[i], work[i], shard_len);
  free(work);
  free(buf);
  return ORA_OK;
}

/* ------------------------------------------------------------------ */
/* Lagrange erasure decoder                                            */
/* ------------------------------------------------------------------ */

static inline unsigned fmul(const field_t* f, unsigned a, unsigned b) {
  if (!a || !b) return 0;
  return f->exp_t[add_mod(f, f->log_t[a], f->log_t[b])];
}
static inline unsigned finv(const field_t* f, unsigned a) { return f->exp_t[(f->modulus - f->log_t[a]) % f->modulus]; }

int ora_leo_decode(int k, size_t shard_len, uint8_t* const* shards, const uint8_t* present) {
  if (k <= 0 || k > 32768) return ORA_E_ARG;
  if (shard_len == 0 || shard_len % 64 != 0) return ORA_E_SHARD_SIZE;
  const field_t* f = field_for_bits(ora_leo_bits_for(k));
  int m = ceil_pow2(k);
  int n = 2 * k;
  /* shard s (0..2k): data i=s<k at point m+i; parity j=s-k at point j */
  int npresent = 0;
  for (int s = 0; s < n; s++) npresent += present[s] ? 1 : 0;
  if (npresent < k) return ORA_E_TOO_FEW;
  if (npresent == n) return ORA_OK;
  /* nodes: first k present shards (data first, like the systematic order) + zero points m+k..2m-1 */
  int nn = m;
  unsigned* xs = (unsigned*)malloc(sizeof(unsigned) * nn);
  int* src = (int*)malloc(sizeof(int) * nn);
  int c = 0;
  for (int s = 0; s < n && c < k; s++)
    if (present[s]) {
      xs[c] = s < k ? (unsigned)(m + s) : (unsigned)(s - k);
      src[c] = s;
      c++;
    }
  for (int z = m + k; z < 2 * m; z++) {
    xs[c] = (unsigned)z;
    src[c] = -1;
    c++;
  }
  /* barycentric denominators w_j = 1 / prod_{l != j} (x_j - x_l) */
  unsigned* w = (unsigned*)malloc(sizeof(unsigned) * nn);
  for (int j = 0; j < nn; j++) {
    unsigned d = 1;
    for (int l = 0; l < nn; l++)
      if (l != j) d = fmul(f, d, xs[j] ^ xs[l]);
    w[j] = finv(f, d);
  }
  for (int s = 0; s < n; s++) {
    if (present[s]) continue;
    unsigned x = s < k ? (unsigned)(m + s) : (unsigned)(s - k);
    unsigned num = 1; /* prod_l (x - x_l) */
    for (int l = 0; l < nn; l++) num = fmul(f, num, x ^ xs[l]);
    memset(shards[s], 0, shard_len);
    for (int j = 0; j < nn; j++) {
      if (src[j] < 0) continue;
      /* L_j(x) = num / (x - x_j) * w_j */
      unsigned coef = fmul(f, fmul(f, num, finv(f, x ^ xs[j])), w[j]);
      if (coef) mul_add(f, shards[s], shards[src[j]], f->log_t[coef], shard_len);
    }
  }
  free(xs);
  free(src);
  free(w);
  return ORA_OK;
}

/* ------------------------------------------------------------------ */
/* Leopard reconstruct (klauspost/reedsolomon v1.12.1 leopardFF8/FF16  */
/* reconstruct, upstream; restated for the CPU baseline)               */
/* ------------------------------------------------------------------ */

/* ifftDITDecoder: as the encoder's IFFT but with skew[iend - 1] and an mtrunc bound */
static void ifft_dit_decoder(const field_t* f, uint8_t** work, int mtrunc, int m, const uint16_t* skew, size_t n) {
  int dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (int r = 0; r < mtrunc; r += dist4) {
      int iend = r + dist;
      unsigned l01 = skew[iend - 1], l02 = skew[iend + dist - 1], l23 = skew[iend + 2 * dist - 1];
      for (int i = r; i < iend; i++) {
        ifft2(f, work[i], work[i + dist], l01, n);
        ifft2(f, work[i + 2 * dist], work[i + 3 * dist], l23, n);
        ifft2(f, work[i], work[i + 2 * dist], l02, n);
        ifft2(f, work[i + dist], work[i + 3 * dist], l02, n);
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    unsigned logm = skew[dist - 1];
    for (int i = 0; i < dist; i++) ifft2(f, work[i], work[i + dist], logm, n);
  }
}

/* FormalDerivative: for i = 1..n-1, width = ((i ^ (i-1)) + 1) / 2, work[i-width..i) ^= work[i..i+width) */
static void formal_derivative(uint8_t** work, int nn, size_t n) {
  for (int i = 1; i < nn; i++) {
    int width = ((i ^ (i - 1)) + 1) >> 1;
    for (int j = 0; j < width; j++) slice_xor(work[i - width + j], work[i + j], n);
  }
}

int ora_leo_decode_fft(int k, size_t shard_len, uint8_t* const* shards, const uint8_t* present) {
  if (k <= 0 || k > 32768) return ORA_E_ARG;
  if (shard_len == 0 || shard_len % 64 != 0) return ORA_E_SHARD_SIZE;
  const field_t* f = field_for_bits(ora_leo_bits_for(k));
  const int m = ceil_pow2(k), nn = 2 * m;
  int npresent = 0;
  for (int s = 0; s < 2 * k; s++) npresent += present[s] ? 1 : 0;
  if (npresent < k) return ORA_E_TOO_FEW;
  if (npresent == 2 * k) return ORA_OK;
  /* erasures in the n-space: parity i -> i, the padding [k, m), data i -> m + i */
  uint8_t* erased = (uint8_t*)calloc((size_t)nn, 1);
  for (int i = 0; i < k; i++)
    if (!present[k + i]) erased[i] = 1;
  for (int i = k; i < m; i++) erased[i] = 1;
  for (int i = 0; i < k; i++)
    if (!present[i]) erased[m + i] = 1;
  /* error locators: errLocs[p] = sum_{j erased} log(p ^ j) mod modulus, log(0) := 0 (the value klauspost's two
   * Walsh-Hadamard transforms produce) */
  unsigned* loc = (unsigned*)malloc(sizeof(unsigned) * (size_t)nn);
  for (int p = 0; p < nn; p++) {
    unsigned long long acc = 0;
    for (int j = 0; j < nn; j++)
      if (erased[j] && j != p) acc += f->log_t[p ^ j];
    loc[p] = (unsigned)(acc % f->modulus);
  }
  uint8_t* buf = (uint8_t*)aligned_alloc(64, (size_t)nn * shard_len);
  uint8_t** work = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)nn);
  memset(buf, 0, (size_t)nn * shard_len);
  for (int i = 0; i < nn; i++) work[i] = buf + (size_t)i * shard_len;
  for (int i = 0; i < k; i++) {
    if (present[k + i]) mul_add(f, work[i], shards[k + i], loc[i], shard_len);
    if (present[i]) mul_add(f, work[m + i], shards[i], loc[m + i], shard_len);
  }
  ifft_dit_decoder(f, work, m + k, nn, f->skew, shard_len);
  formal_derivative(work, nn, shard_len);
  fft_dit(f, work, m + k, nn, f->skew, shard_len);
  for (int i = 0; i < k; i++) {
    if (!present[i]) {
      memset(shards[i], 0, shard_len);
      mul_add(f, shards[i], work[m + i], (f->modulus - loc[m + i]) % f->modulus, shard_len);
    }
    if (!present[k + i]) {
      memset(shards[k + i], 0, shard_len);
      mul_add(f, shards[k + i], work[i], (f->modulus - loc[i]) % f->modulus, shard_len);
    }
  }
  free(work);
  free(buf);
  free(loc);
  free(erased);
  return ORA_OK;
}
