/*
 * TEST / BASELINE INFRASTRUCTURE ONLY -- never part of the product path.
 *
 * Vectorisable CPU port of the layered normalised min-sum decoder, used as bench.py's cpu_baseline ("kind": "port").
 * Same semantics as orc_ldpc_decode (ldpc_oracle.c, which restates ldpc_decoder_impl.cpp:60-308 and
 * ldpc_decoder_generic.cpp:30-128) and bit-exact with it (tests/test_oracle.py::test_cpu_port_matches_oracle), but
 * organised for SIMD the way the reference's AVX2 decoder is (ldpc_decoder_avx2.cpp): every inner loop runs over the
 * Z lanes of a lifted node with branch-free int8/int16 arithmetic, and the cyclic shift is applied by copying the
 * two contiguous segments of a node instead of a per-element modulo. Check-to-variable messages are kept per edge in
 * the check-node domain (c2v[e][t]); an all-zero c2v is the reference's "not initialised" state (soft (-) 0 = soft).
 */
#include "ldpc_oracle.h"

#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define PORT_MAX_Z 384
#define PORT_MAX_EDGES 316
#define PORT_MAX_DEG 19

typedef struct {
  int8_t soft[68 * PORT_MAX_Z];            /* node-major soft bits                                  */
  int8_t c2v[PORT_MAX_EDGES * PORT_MAX_Z]; /* per edge, check-node domain, stride Zp                */
  int8_t sv[PORT_MAX_DEG][PORT_MAX_Z];     /* soft bits of the row's edges, rotated; then soft'     */
  int8_t v2c[PORT_MAX_DEG][PORT_MAX_Z];    /* variable-to-check, rotated                            */
} port_state;

typedef struct {
  unsigned Z, K, M, N_full, N_short;
  int      deg[46];
  uint16_t cols[46][PORT_MAX_DEG + 8];
  uint16_t shifts[46][PORT_MAX_DEG + 8];
} port_graph;

static int port_graph_build(port_graph* g, int bg, unsigned Z)
{
  if (orc_lifting_index(Z) < 0 || (bg != 1 && bg != 2)) {
    return -1;
  }
  g->Z       = Z;
  g->M       = (bg == 1) ? 46 : 42;
  g->N_full  = (bg == 1) ? 68 : 52;
  g->N_short = g->N_full - 2;
  g->K       = g->N_full - g->M;
  for (unsigned m = 0; m != g->M; ++m) {
    g->deg[m] = orc_graph_row(bg, Z, m, g->cols[m], g->shifts[m]);
  }
  return 0;
}

/* The lifted graphs, built once per process (pthread_once): building one walks the whole base-graph edge table per row
 * (about 24k entries), which cost every call tens of microseconds while the reference builds its graph once per
 * decoder configuration (ldpc_graph_impl.cpp:29-53) and per call only resets per-layer state
 * (ldpc_decoder_impl.cpp:33-58, 97). */
static port_graph     g_graphs[2][51];
static int            g_graph_ok[2][51];
static pthread_once_t g_graphs_once = PTHREAD_ONCE_INIT;
static const unsigned k_port_lifting[51] = {2,  3,  4,  5,  6,  7,  8,  9,  10, 11,  12,  13,  14,  15,  16,  18,  20,
                                            22, 24, 26, 28, 30, 32, 36, 40, 44, 48,  52,  56,  60,  64,  72,  80,  88,
                                            96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320, 352, 384};
static void port_graphs_build(void)
{
  for (int b = 0; b != 2; ++b) {
    for (int i = 0; i != 51; ++i) {
      g_graph_ok[b][i] = port_graph_build(&g_graphs[b][i], b + 1, k_port_lifting[i]) == 0;
    }
  }
}
static const port_graph* port_graph_get(int bg, unsigned Z)
{
  const int pos = orc_lifting_position(Z);
  if (pos < 0 || (bg != 1 && bg != 2)) {
    return NULL;
  }
  pthread_once(&g_graphs_once, port_graphs_build);
  return g_graph_ok[bg - 1][pos] ? &g_graphs[bg - 1][pos] : NULL;
}

/* One layer over Zp = Z rounded up to 32 lanes (AVX2; lanes >= Z carry junk that never reaches the soft bits).
 * Arithmetic per lane, with c2v never infinite (|c2v| <= round(0.8 * 120)):
 *   v2c   = +-127 soft passes through, else clamp(s - c, +-120)                 llr.cpp:56-71
 *   min1 / min2 / idx / sign over the edges in order, strict '<'               gen.cpp:46-68
 *   c2v'  = sign * round(0.8 * (k == idx ? min2 : min1)) = (205 m + 128) >> 8   gen.cpp:70-106
 *   soft' = promotion_sum(c2v', v2c)                                           llr.cpp:73-86, gen.cpp:108-120 */
static void port_layer(port_state* st, const port_graph* g, unsigned m, unsigned e0, unsigned Zp, int first)
{
  const unsigned Z  = g->Z;
  const int      D  = g->deg[m];
  const __m256i  p120 = _mm256_set1_epi8(120), m120 = _mm256_set1_epi8(-120);
  const __m256i  p127 = _mm256_set1_epi8(127), m127 = _mm256_set1_epi8(-127);
  const __m256i  one  = _mm256_set1_epi8(1);
  for (int k = 0; k != D; ++k) {
    const int8_t*  node = st->soft + (size_t)g->cols[m][k] * Z;
    const unsigned s    = g->shifts[m][k];
    memcpy(st->sv[k], node + s, Z - s);
    memcpy(st->sv[k] + (Z - s), node, s);
  }
  for (unsigned t = 0; t < Zp; t += 32) {
    __m256i m1 = p120, m2 = p120, idx = _mm256_setzero_si256(), sgn = _mm256_setzero_si256();
    for (int k = 0; k != D; ++k) {
      const __m256i sv   = _mm256_loadu_si256((const __m256i*)(st->sv[k] + t));
      /* first iteration: no c2v yet (the reference's per-layer "initialised" flag, ldpc_decoder_impl.cpp:196-200) */
      const __m256i c    = first ? _mm256_setzero_si256()
                                 : _mm256_loadu_si256((const __m256i*)(st->c2v + (size_t)(e0 + k) * Zp + t));
      const __m256i inf  = _mm256_or_si256(_mm256_cmpeq_epi8(sv, p127), _mm256_cmpeq_epi8(sv, m127));
      __m256i       v    = _mm256_min_epi8(_mm256_max_epi8(_mm256_subs_epi8(sv, c), m120), p120);
      v                  = _mm256_blendv_epi8(v, sv, inf);
      _mm256_storeu_si256((__m256i*)(st->v2c[k] + t), v);
      const __m256i a    = _mm256_abs_epi8(v);
      const __m256i ismn = _mm256_cmpgt_epi8(m1, a);
      m2                 = _mm256_min_epi8(m2, _mm256_max_epi8(m1, a));
      m1                 = _mm256_min_epi8(m1, a);
      idx                = _mm256_blendv_epi8(idx, _mm256_set1_epi8((char)k), ismn);
      sgn                = _mm256_xor_si256(sgn, v);
    }
    /* scaled magnitudes in 16-bit lanes */
    const __m256i c205 = _mm256_set1_epi16(205), c128 = _mm256_set1_epi16(128);
    const __m256i lo1  = _mm256_srli_epi16(_mm256_add_epi16(_mm256_mullo_epi16(_mm256_unpacklo_epi8(m1, _mm256_setzero_si256()), c205), c128), 8);
    const __m256i hi1  = _mm256_srli_epi16(_mm256_add_epi16(_mm256_mullo_epi16(_mm256_unpackhi_epi8(m1, _mm256_setzero_si256()), c205), c128), 8);
    const __m256i lo2  = _mm256_srli_epi16(_mm256_add_epi16(_mm256_mullo_epi16(_mm256_unpacklo_epi8(m2, _mm256_setzero_si256()), c205), c128), 8);
    const __m256i hi2  = _mm256_srli_epi16(_mm256_add_epi16(_mm256_mullo_epi16(_mm256_unpackhi_epi8(m2, _mm256_setzero_si256()), c205), c128), 8);
    const __m256i n1   = _mm256_packus_epi16(lo1, hi1);
    const __m256i n2   = _mm256_packus_epi16(lo2, hi2);
    for (int k = 0; k != D; ++k) {
      const __m256i v   = _mm256_loadu_si256((const __m256i*)(st->v2c[k] + t));
      const __m256i mag = _mm256_blendv_epi8(n1, n2, _mm256_cmpeq_epi8(idx, _mm256_set1_epi8((char)k)));
      const __m256i cc  = _mm256_sign_epi8(mag, _mm256_or_si256(_mm256_xor_si256(sgn, v), one));
      _mm256_storeu_si256((__m256i*)(st->c2v + (size_t)(e0 + k) * Zp + t), cc);
      __m256i       r   = _mm256_adds_epi8(cc, v);
      r                 = _mm256_blendv_epi8(r, p127, _mm256_cmpgt_epi8(r, p120));
      r                 = _mm256_blendv_epi8(r, m127, _mm256_cmpgt_epi8(m120, r));
      const __m256i inf = _mm256_or_si256(_mm256_cmpeq_epi8(v, p127), _mm256_cmpeq_epi8(v, m127));
      r                 = _mm256_blendv_epi8(r, v, inf);
      _mm256_storeu_si256((__m256i*)(st->sv[k] + t), r);
    }
  }
  for (int k = 0; k != D; ++k) {
    int8_t*        node = st->soft + (size_t)g->cols[m][k] * Z;
    const unsigned s    = g->shifts[m][k];
    memcpy(node + s, st->sv[k], Z - s);
    memcpy(node, st->sv[k] + (Z - s), s);
  }
}

/* The early-stop check at the speed of the reference's CPU path (its AVX2 hard decision, log_likelihood_ratio.cpp:
 * 226-252, and its byte-table CRC calculator, crc_calculator_lut_impl): the oracle's bit-serial restatements cost the
 * port tens of microseconds per iteration on a BG1 Z=384 codeblock. Same results: hard bit = (llr <= 0), MSB first;
 * the CRC is the remainder of M(x) x^order mod G with zero initial state (crc_calculator_generic_impl.cpp:111-133). */
static uint8_t  g_rev8[256];
static uint32_t g_crc_tab[3][256]; /* CRC24A, CRC24B, CRC16 */
static pthread_once_t g_tabs_once = PTHREAD_ONCE_INIT;
static const unsigned k_crc_order[3] = {24, 24, 16};
static const uint32_t k_crc_poly[3]  = {0x864cfbU, 0x800063U, 0x1021U}; /* without the x^order term */
static void port_tabs_build(void)
{
  for (unsigned b = 0; b != 256; ++b) {
    unsigned r = 0;
    for (unsigned k = 0; k != 8; ++k) {
      r |= ((b >> k) & 1U) << (7 - k);
    }
    g_rev8[b] = (uint8_t)r;
    for (int p = 0; p != 3; ++p) {
      const unsigned order = k_crc_order[p];
      const uint32_t mask  = (1U << order) - 1U;
      uint32_t       c     = (uint32_t)b << (order - 8);
      for (int k = 0; k != 8; ++k) {
        c = (c & (1U << (order - 1))) ? ((c << 1) ^ k_crc_poly[p]) & mask : (c << 1) & mask;
      }
      g_crc_tab[p][b] = c;
    }
  }
}
static int port_crc_index(int crc_poly)
{
  return crc_poly == ORC_CRC24A ? 0 : (crc_poly == ORC_CRC24B ? 1 : (crc_poly == ORC_CRC16 ? 2 : -1));
}
/* CRC remainder of the first nbits of the packed (MSB-first) message; falls back to the oracle for other polynomials */
uint32_t orc_crc_port(int crc_poly, const uint8_t* packed, unsigned nbits)
{
  const int p = port_crc_index(crc_poly);
  if (p < 0) {
    return orc_crc_packed(crc_poly, packed, nbits);
  }
  pthread_once(&g_tabs_once, port_tabs_build);
  const unsigned order = k_crc_order[p];
  const uint32_t mask  = (1U << order) - 1U;
  uint32_t       c     = 0;
  const unsigned nb    = nbits / 8;
  for (unsigned i = 0; i != nb; ++i) {
    c = ((c << 8) & mask) ^ g_crc_tab[p][((c >> (order - 8)) ^ packed[i]) & 0xffU];
  }
  for (unsigned i = nb * 8; i != nbits; ++i) {
    const uint32_t bit = (packed[i / 8] >> (7 - i % 8)) & 1U;
    const uint32_t top = ((c >> (order - 1)) ^ bit) & 1U;
    c                  = (c << 1) & mask;
    c ^= top ? k_crc_poly[p] : 0U;
  }
  return c;
}
/* hard_decision of n soft bits into packed bytes (every byte rewritten); returns 1 iff no soft bit is zero */
static int port_hard_decision(uint8_t* out, const int8_t* soft, unsigned n)
{
  pthread_once(&g_tabs_once, port_tabs_build);
  const __m256i one = _mm256_set1_epi8(1), zero = _mm256_setzero_si256();
  int           any_zero = 0;
  unsigned      i        = 0;
  for (; i + 32 <= n; i += 32) {
    const __m256i  x = _mm256_loadu_si256((const __m256i*)(soft + i));
    const uint32_t h = (uint32_t)_mm256_movemask_epi8(_mm256_cmpgt_epi8(one, x)); /* x <= 0 */
    any_zero |= _mm256_movemask_epi8(_mm256_cmpeq_epi8(x, zero)) != 0;
    out[i / 8]     = g_rev8[h & 0xffU];
    out[i / 8 + 1] = g_rev8[(h >> 8) & 0xffU];
    out[i / 8 + 2] = g_rev8[(h >> 16) & 0xffU];
    out[i / 8 + 3] = g_rev8[h >> 24];
  }
  for (; i < n; i += 8) {
    uint8_t b = 0;
    for (unsigned k = 0; k != 8 && i + k < n; ++k) {
      b |= (uint8_t)((soft[i + k] <= 0 ? 1U : 0U) << (7 - k));
      any_zero |= soft[i + k] == 0;
    }
    out[i / 8] = b;
  }
  return !any_zero;
}

int orc_ldpc_decode_port(int bg, unsigned Z, unsigned nof_filler_bits, const int8_t* llr, unsigned llr_len,
                         unsigned max_iterations, int crc_poly, uint8_t* out_packed)
{
  const port_graph* gp = port_graph_get(bg, Z);
  if (gp == NULL || max_iterations == 0) {
    return -1;
  }
  const port_graph* g = gp;
  const unsigned msg_len = g->K * Z;
  if (llr_len > g->N_short * Z || llr_len < msg_len + 2 * Z || nof_filler_bits >= msg_len) {
    return -1;
  }
  const unsigned out_bytes = (msg_len + 7) / 8;
  unsigned       last      = llr_len;
  while (last != 0 && llr[last - 1] == 0) {
    --last;
  }
  if (last == 0) { /* ldpc_decoder_impl.cpp:86-94 */
    if (crc_poly < 0) {
      memset(out_packed, 0, out_bytes);
      for (unsigned i = 0; i != msg_len; ++i) {
        out_packed[i / 8] |= (uint8_t)(1U << (7 - i % 8));
      }
    }
    return 0;
  }
  /* one decoder state per thread, reused across calls (the reference keeps one decoder object per worker thread,
   * pusch_decoder_impl.h:48); a fresh allocation per call would page-fault 160 KiB of zeroed memory every time and
   * serialise threads on the address-space lock */
  static __thread port_state* tls_state = NULL;
  if (tls_state == NULL) {
    tls_state = (port_state*)malloc(sizeof(port_state));
    if (tls_state == NULL) {
      return -1;
    }
  }
  port_state* st = tls_state;
  /* only what this codeblock reads: [0, 2Z) and the tail past its LLRs; c2v needs no clearing (first-iteration
   * flag, port_layer) */
  const unsigned Zp = (Z + 31) / 32 * 32;
  memset(st->soft, 0, 2 * Z);
  memcpy(st->soft + 2 * Z, llr, llr_len);
  memset(st->soft + 2 * Z + llr_len, 0, g->N_full * Z - 2 * Z - llr_len);
  unsigned cb_len = last + 2 * Z;
  if (cb_len < (g->K + 4) * Z) {
    cb_len = (g->K + 4) * Z;
  }
  cb_len                    = (cb_len + Z - 1) / Z * Z;
  const unsigned nof_layers = cb_len / Z - g->K;
  unsigned       e0[46];
  for (unsigned m = 0, e = 0; m != g->M; ++m) {
    e0[m] = e;
    e += (unsigned)g->deg[m];
  }
  int ret = 0;
  for (unsigned it = 0; it != max_iterations; ++it) {
    for (unsigned m = 0; m != nof_layers; ++m) {
      port_layer(st, g, m, e0[m], Zp, it == 0);
    }
    if (crc_poly >= 0) {
      const int ok = port_hard_decision(out_packed, st->soft, msg_len);
      if (ok && orc_crc_port(crc_poly, out_packed, msg_len - nof_filler_bits) == 0) {
        ret = (int)it + 1;
        break;
      }
    }
  }
  if (crc_poly < 0) {
    port_hard_decision(out_packed, st->soft, msg_len);
  }
  return ret;
}
