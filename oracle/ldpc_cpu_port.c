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

static int port_graph_init(port_graph* g, int bg, unsigned Z)
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

/* One layer over Zp = Z rounded up to 32 lanes (AVX2; lanes >= Z carry junk that never reaches the soft bits).
 * Arithmetic per lane, with c2v never infinite (|c2v| <= round(0.8 * 120)):
 *   v2c   = +-127 soft passes through, else clamp(s - c, +-120)                 llr.cpp:56-71
 *   min1 / min2 / idx / sign over the edges in order, strict '<'               gen.cpp:46-68
 *   c2v'  = sign * round(0.8 * (k == idx ? min2 : min1)) = (205 m + 128) >> 8   gen.cpp:70-106
 *   soft' = promotion_sum(c2v', v2c)                                           llr.cpp:73-86, gen.cpp:108-120 */
static void port_layer(port_state* st, const port_graph* g, unsigned m, unsigned e0, unsigned Zp)
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
      const __m256i c    = _mm256_loadu_si256((const __m256i*)(st->c2v + (size_t)(e0 + k) * Zp + t));
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

int orc_ldpc_decode_port(int bg, unsigned Z, unsigned nof_filler_bits, const int8_t* llr, unsigned llr_len,
                         unsigned max_iterations, int crc_poly, uint8_t* out_packed)
{
  port_graph g;
  if (port_graph_init(&g, bg, Z) != 0 || max_iterations == 0) {
    return -1;
  }
  const unsigned msg_len = g.K * Z;
  if (llr_len > g.N_short * Z || llr_len < msg_len + 2 * Z || nof_filler_bits >= msg_len) {
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
  memset(st->soft, 0, sizeof(st->soft));
  memset(st->c2v, 0, sizeof(st->c2v));
  const unsigned Zp = (Z + 31) / 32 * 32;
  memcpy(st->soft + 2 * Z, llr, llr_len);
  unsigned cb_len = last + 2 * Z;
  if (cb_len < (g.K + 4) * Z) {
    cb_len = (g.K + 4) * Z;
  }
  cb_len                    = (cb_len + Z - 1) / Z * Z;
  const unsigned nof_layers = cb_len / Z - g.K;
  unsigned       e0[46];
  for (unsigned m = 0, e = 0; m != g.M; ++m) {
    e0[m] = e;
    e += (unsigned)g.deg[m];
  }
  int ret = 0;
  for (unsigned it = 0; it != max_iterations; ++it) {
    for (unsigned m = 0; m != nof_layers; ++m) {
      port_layer(st, &g, m, e0[m], Zp);
    }
    if (crc_poly >= 0) {
      memset(out_packed, 0, out_bytes);
      const int ok = orc_hard_decision(out_packed, st->soft, msg_len);
      if (ok && orc_crc_packed(crc_poly, out_packed, msg_len - nof_filler_bits) == 0) {
        ret = (int)it + 1;
        break;
      }
    }
  }
  if (crc_poly < 0) {
    memset(out_packed, 0, out_bytes);
    orc_hard_decision(out_packed, st->soft, msg_len);
  }
  return ret;
}
