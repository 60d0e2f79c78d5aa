/*
 * CPU ORACLE for the MI355X LDPC decode path -- TEST INFRASTRUCTURE ONLY (see ldpc_oracle.h for the contract and
 * the parity-pinning status). Plain C restatement of the reference srsRAN algorithms; every function cites the
 * reference file:line it follows. Never linked into the product library.
 */
#include "ldpc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define LLR_MAX 120
#define LLR_INF 127

/* ------------------------------------------------------------------------------------------------------------ */
/* LLR arithmetic -- lib/phy/upper/log_likelihood_ratio.cpp:37-97                                                 */
/* ------------------------------------------------------------------------------------------------------------ */

static int llr_isinf(int8_t v) { return v > LLR_MAX || v < -LLR_MAX; } /* header isinf/isfinite */

/* tackle_special_sums (:39-54): a == -b -> 0; an infinite summand wins (a first). Returns 1 if handled. */
static int special_sum(int8_t a, int8_t b, int8_t* r)
{
  if ((int)a == -(int)b) {
    *r = 0;
    return 1;
  }
  if (llr_isinf(a)) {
    *r = a;
    return 1;
  }
  if (llr_isinf(b)) {
    *r = b;
    return 1;
  }
  return 0;
}

int8_t orc_llr_add(int8_t a, int8_t b) /* operator+= (:56-71): special cases, then saturate at +-LLR_MAX */
{
  int8_t r;
  if (special_sum(a, b, &r)) {
    return r;
  }
  int tmp = (int)a + (int)b;
  if (abs(tmp) > LLR_MAX) {
    return (int8_t)(tmp > 0 ? LLR_MAX : -LLR_MAX);
  }
  return (int8_t)tmp;
}

/* operator-: a + (-b) (log_likelihood_ratio.h, "Saturated difference"); note rhs += *this order of operator+ is
 * symmetric in the special cases except "a infinite wins first", which for a - b means: a == b -> 0,
 * isinf(-b) checked after isinf(a)... operator+(rhs) calls rhs += *this, i.e. special_sum(-b, a). */
int8_t orc_llr_sub(int8_t a, int8_t b)
{
  /* a - b = a + (-b) = operator+(a, -b) = (-b) += a  ->  tackle_special_sums(-b, a) */
  int8_t nb = (int8_t)(-(int)b);
  int8_t r;
  if (special_sum(nb, a, &r)) {
    return r;
  }
  int tmp = (int)nb + (int)a;
  if (abs(tmp) > LLR_MAX) {
    return (int8_t)(tmp > 0 ? LLR_MAX : -LLR_MAX);
  }
  return (int8_t)tmp;
}

int8_t orc_llr_promotion_sum(int8_t a, int8_t b) /* promotion_sum (:73-86): overflow promotes to +-LLR_INFTY */
{
  int8_t r;
  if (special_sum(a, b, &r)) {
    return r;
  }
  int tmp = (int)a + (int)b;
  if (abs(tmp) > LLR_MAX) {
    return (int8_t)(tmp > 0 ? LLR_INF : -LLR_INF);
  }
  return (int8_t)tmp;
}

int8_t orc_llr_quantize(float value, float range) /* quantize (:88-97) */
{
  float clipped = value;
  if (fabsf(value) > range) {
    clipped = copysignf(range, value);
  }
  return (int8_t)roundf(clipped / range * (float)LLR_MAX);
}

/* hard_decision (:226-252): bit = (llr <= 0) packed MSB-first (bit_buffer.h:98-150); true iff no zero LLR. */
int orc_hard_decision(uint8_t* out_packed, const int8_t* llr, unsigned n)
{
  int no_zero = 1;
  for (unsigned i = 0; i != n; ++i) {
    unsigned bit  = (llr[i] <= 0) ? 1U : 0U;
    unsigned byte = i / 8, pos = 7 - (i % 8);
    out_packed[byte] = (uint8_t)((out_packed[byte] & ~(1U << pos)) | (bit << pos));
    if (llr[i] == 0) {
      no_zero = 0;
    }
  }
  return no_zero;
}

/* ------------------------------------------------------------------------------------------------------------ */
/* CRC -- crc_calculator_generic_impl.cpp:28-133 (MSB-first long division, init 0, `order` zero bits appended)   */
/* ------------------------------------------------------------------------------------------------------------ */

static void crc_params(int poly, unsigned* order, uint64_t* polynom)
{
  switch (poly) {
    case ORC_CRC24A: *order = 24; *polynom = 0x1864cfb; break;
    case ORC_CRC24B: *order = 24; *polynom = 0x1800063; break;
    case ORC_CRC24C: *order = 24; *polynom = 0x1b2b117; break;
    case ORC_CRC16: *order = 16; *polynom = 0x11021; break;
    case ORC_CRC11: *order = 11; *polynom = 0xe21; break;
    default: *order = 6; *polynom = 0x61; break;
  }
}

static uint32_t crc_finish(uint64_t rem, unsigned order, uint64_t polynom)
{
  uint64_t highbit = 1ULL << order;
  for (unsigned i = 0; i != order; ++i) {
    rem <<= 1;
    if (rem & highbit) {
      rem ^= polynom;
    }
  }
  return (uint32_t)(rem & (highbit - 1));
}

uint32_t orc_crc_packed(int poly, const uint8_t* packed, unsigned nbits)
{
  unsigned order;
  uint64_t polynom;
  crc_params(poly, &order, &polynom);
  uint64_t highbit = 1ULL << order, rem = 0;
  for (unsigned i = 0; i != nbits; ++i) {
    rem = (rem << 1) | ((packed[i / 8] >> (7 - (i % 8))) & 1U);
    if (rem & highbit) {
      rem ^= polynom;
    }
  }
  return crc_finish(rem, order, polynom);
}

uint32_t orc_crc_bytes(int poly, const uint8_t* bytes, unsigned nbytes)
{
  return orc_crc_packed(poly, bytes, nbytes * 8);
}

uint32_t orc_crc_bits(int poly, const uint8_t* bits, unsigned nbits)
{
  unsigned order;
  uint64_t polynom;
  crc_params(poly, &order, &polynom);
  uint64_t highbit = 1ULL << order, rem = 0;
  for (unsigned i = 0; i != nbits; ++i) {
    rem = (rem << 1) | (bits[i] & 1U);
    if (rem & highbit) {
      rem ^= polynom;
    }
  }
  return crc_finish(rem, order, polynom);
}

/* ------------------------------------------------------------------------------------------------------------ */
/* Graph tables -- ldpc_luts_impl.cpp:57 (LSindex), :4521-4566 (get_graph: shift %= Z); ldpc_graph_impl.h:38-67 */
/* ------------------------------------------------------------------------------------------------------------ */

typedef struct {
  uint8_t  bg, row, col;
  uint16_t shift[8];
} edge_entry;

static const edge_entry k_edges[] = {
#define LDPC_EDGE(bg, r, c, s0, s1, s2, s3, s4, s5, s6, s7) {bg, r, c, {s0, s1, s2, s3, s4, s5, s6, s7}},
#include "ldpc_base_graphs.inc"
#undef LDPC_EDGE
};
static const unsigned k_nof_edges = sizeof(k_edges) / sizeof(k_edges[0]);

static const unsigned k_lifting_sizes[51] = {2,  3,  4,  5,  6,  7,  8,  9,  10,  11,  12,  13,  14,  15,  16,  18, 20,
                                             22, 24, 26, 28, 30, 32, 36, 40, 44, 48, 52, 56, 60, 64, 72, 80, 88,
                                             96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320,
                                             352, 384};

/* TS 38.212 Table 5.3.2-1: Z = a * 2^j, iLS is the index of a in {2,3,5,7,9,11,13,15}. */
int orc_lifting_index(unsigned Z)
{
  static const unsigned a_set[8] = {2, 3, 5, 7, 9, 11, 13, 15};
  if (orc_lifting_position(Z) < 0) {
    return -1;
  }
  for (int i = 0; i != 8; ++i) {
    for (unsigned z = a_set[i]; z <= 384; z *= 2) {
      if (z == Z) {
        return i;
      }
    }
  }
  return -1;
}

int orc_lifting_position(unsigned Z)
{
  for (int i = 0; i != 51; ++i) {
    if (k_lifting_sizes[i] == Z) {
      return i;
    }
  }
  return -1;
}

int orc_graph_row(int bg, unsigned Z, unsigned m, uint16_t* cols, uint16_t* shifts)
{
  int ils = orc_lifting_index(Z);
  if (ils < 0 || (bg != 1 && bg != 2)) {
    return -1;
  }
  int deg = 0;
  for (unsigned e = 0; e != k_nof_edges; ++e) {
    if (k_edges[e].bg == bg && k_edges[e].row == m) {
      cols[deg]   = k_edges[e].col;
      shifts[deg] = (uint16_t)(k_edges[e].shift[ils] % Z);
      ++deg;
    }
  }
  return deg;
}

typedef struct {
  int      bg;
  unsigned Z, K, M, N_full, N_short;
  int      deg[46];
  uint16_t cols[46][20];
  uint16_t shifts[46][20];
} graph_t;

static int graph_init(graph_t* g, int bg, unsigned Z) /* ldpc_graph_impl.cpp:29-53, ldpc_decoder_impl.cpp:33-58 */
{
  if (orc_lifting_index(Z) < 0 || (bg != 1 && bg != 2)) {
    return -1;
  }
  g->bg      = bg;
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

/* ------------------------------------------------------------------------------------------------------------ */
/* Layered normalised min-sum decoder -- ldpc_decoder_impl.cpp:60-308 with ldpc_decoder_generic.cpp:30-128       */
/* (generic: node_size_byte == lifting_size, ldpc_decoder_generic.h:36)                                          */
/* ------------------------------------------------------------------------------------------------------------ */

#define MAX_Z 384
#define MAX_SLOTS 27 /* MAX_CHECK_NODE_DEGREE = MAX_BG_K + 5 (ldpc_decoder_impl.h:45) */

typedef struct {
  graph_t g;
  unsigned hr;                           /* bg_N_high_rate = K + 4 */
  float    sf;
  int8_t   soft[68 * MAX_Z];             /* soft_bits, node-major */
  int8_t   v2c[2 * MAX_SLOTS * MAX_Z];   /* var_to_check, two copies per slot (ldpc_decoder_impl.h:220) */
  int8_t   c2v[46][MAX_SLOTS * MAX_Z];   /* check_to_var[layer][slot][j] (ldpc_decoder_impl.h:224) */
  int      c2v_init[46];
  int8_t   min1[MAX_Z], min2[MAX_Z];
  uint8_t  idx[MAX_Z], sgn[MAX_Z];
} dec_state;

static int8_t* soft_of(dec_state* s, unsigned n) { return s->soft + n * s->g.Z; }
static int8_t* c2v_of(dec_state* s, unsigned m, unsigned slot) { return s->c2v[m] + slot * s->g.Z; }
static int8_t* v2c_of(dec_state* s, unsigned slot, unsigned shift) { return s->v2c + 2 * slot * s->g.Z + shift; }

/* scale_llr (ldpc_decoder_generic.cpp:70-79) */
static int8_t scale_llr(int8_t v, float sf)
{
  if (llr_isinf(v)) {
    return v;
  }
  return (int8_t)roundf((float)v * sf);
}

/* update_variable_to_check_messages (ldpc_decoder_impl.cpp:176-219) + compute_var_to_check_msgs (gen.cpp:30-44) */
static void update_v2c(dec_state* s, unsigned m)
{
  const unsigned Z = s->g.Z;
  for (int k = 0; k != s->g.deg[m]; ++k) {
    unsigned n = s->g.cols[m][k];
    if (n >= s->hr) {
      break;
    }
    const int8_t* soft = soft_of(s, n);
    const int8_t* c2v  = c2v_of(s, m, n);
    int8_t*       v2c  = v2c_of(s, n, 0);
    if (s->c2v_init[m]) {
      for (unsigned j = 0; j != Z; ++j) {
        v2c[j] = orc_llr_sub(soft[j], c2v[j]);
      }
    } else {
      memcpy(v2c, soft, Z);
    }
    memcpy(v2c + Z, v2c, Z);
  }
  if (m >= 4) {
    unsigned      n    = s->hr + m - 4;
    const int8_t* soft = soft_of(s, n);
    const int8_t* c2v  = c2v_of(s, m, s->hr);
    int8_t*       v2c  = v2c_of(s, s->hr, 0);
    if (s->c2v_init[m]) {
      for (unsigned j = 0; j != Z; ++j) {
        v2c[j] = orc_llr_sub(soft[j], c2v[j]);
      }
    } else {
      memcpy(v2c, soft, Z);
    }
    memcpy(v2c + Z, v2c, Z);
  }
}

/* update_check_to_variable_messages (ldpc_decoder_impl.cpp:236-308) with analyze_var_to_check_msgs
 * (gen.cpp:46-68) and compute_check_to_var_msgs (gen.cpp:83-106). */
static void update_c2v(dec_state* s, unsigned m)
{
  const unsigned Z = s->g.Z;
  for (unsigned j = 0; j != Z; ++j) {
    s->min1[j] = LLR_MAX;
    s->min2[j] = LLR_MAX;
    s->idx[j]  = 0;
    s->sgn[j]  = 0;
  }
  for (int k = 0; k != s->g.deg[m]; ++k) {
    unsigned      n       = s->g.cols[m][k];
    unsigned      shift   = s->g.shifts[m][k];
    unsigned      slot    = n < s->hr ? n : s->hr;
    const int8_t* rotated = v2c_of(s, slot, shift);
    for (unsigned j = 0; j != Z; ++j) {
      int8_t a      = (int8_t)abs((int)rotated[j]);
      int    is_min = a < s->min1[j];
      int8_t new2   = is_min ? s->min1[j] : a;
      int    best2  = a < s->min2[j];
      s->min2[j]    = best2 ? new2 : s->min2[j];
      s->min1[j]    = is_min ? a : s->min1[j];
      s->idx[j]     = is_min ? (uint8_t)k : s->idx[j];
      s->sgn[j] ^= (rotated[j] >= 0) ? 0U : 1U;
    }
  }
  for (int k = 0; k != s->g.deg[m]; ++k) {
    unsigned      n     = s->g.cols[m][k];
    unsigned      shift = s->g.shifts[m][k];
    unsigned      slot  = n < s->hr ? n : s->hr;
    int8_t*       c2v   = c2v_of(s, m, slot);
    const int8_t* v2c   = v2c_of(s, slot, 0);
    for (unsigned j = 0; j != Z; ++j) {
      unsigned t     = (j + Z - shift) % Z;
      int8_t   mag   = ((unsigned)k != s->idx[t]) ? s->min1[t] : s->min2[t];
      mag            = scale_llr(mag, s->sf);
      unsigned fsign = s->sgn[t] ^ ((v2c[j] >= 0) ? 0U : 1U);
      int      am    = abs((int)mag);
      c2v[j]         = (int8_t)(fsign ? -am : am); /* copysign(mag, 1 - 2*fsign), header :185-192 */
    }
  }
  s->c2v_init[m] = 1;
}

/* update_soft_bits (ldpc_decoder_impl.cpp:221-234) + compute_soft_bits (gen.cpp:108-120) */
static void update_soft(dec_state* s, unsigned m)
{
  const unsigned Z = s->g.Z;
  for (int k = 0; k != s->g.deg[m]; ++k) {
    unsigned      n    = s->g.cols[m][k];
    unsigned      slot = n < s->hr ? n : s->hr;
    const int8_t* c2v  = c2v_of(s, m, slot);
    const int8_t* v2c  = v2c_of(s, slot, 0);
    int8_t*       soft = soft_of(s, n);
    for (unsigned j = 0; j != Z; ++j) {
      soft[j] = orc_llr_promotion_sum(c2v[j], v2c[j]);
    }
  }
}

int orc_ldpc_decode(int bg, unsigned Z, unsigned nof_filler_bits, const int8_t* llr, unsigned llr_len,
                    unsigned max_iterations, float scaling_factor, int crc_poly, uint8_t* out_packed)
{
  dec_state* s = (dec_state*)calloc(1, sizeof(dec_state)); /* fresh object: all soft bits zero */
  if (s == NULL || graph_init(&s->g, bg, Z) != 0 || max_iterations == 0 || !(scaling_factor > 0) ||
      !(scaling_factor < 1)) {
    free(s);
    return -1;
  }
  s->hr = s->g.K + 4;
  s->sf = scaling_factor;

  const unsigned K = s->g.K;
  const unsigned msg_len = K * Z, max_in = s->g.N_short * Z, min_in = msg_len + 2 * Z;
  if (llr_len > max_in || llr_len < min_in || nof_filler_bits >= msg_len) {
    free(s);
    return -1;
  }
  const unsigned nof_significant_bits = msg_len - nof_filler_bits;
  const unsigned out_bytes            = (msg_len + 7) / 8;

  /* Last non-zero soft bit (impl.cpp:85-94). */
  unsigned last = llr_len;
  while (last != 0 && llr[last - 1] == 0) {
    --last;
  }
  if (last == 0) {
    if (crc_poly < 0) {
      memset(out_packed, 0, out_bytes);
      for (unsigned i = 0; i != msg_len; ++i) {
        out_packed[i / 8] |= (uint8_t)(1U << (7 - i % 8));
      }
    }
    free(s);
    return 0;
  }

  /* load_soft_bits (impl.cpp:149-174): two punctured nodes are zero, then the LLRs; the rest stays zero. */
  memcpy(s->soft + 2 * Z, llr, llr_len);

  /* Codeblock length and number of layers (impl.cpp:103-114). */
  unsigned cb_len = last + 2 * Z;
  if (cb_len < (K + 4) * Z) {
    cb_len = (K + 4) * Z;
  }
  if (cb_len % Z != 0) {
    cb_len = (cb_len / Z + 1) * Z;
  }
  unsigned nof_layers = cb_len / Z - K;

  for (unsigned it = 0; it != max_iterations; ++it) {
    for (unsigned m = 0; m != nof_layers; ++m) {
      update_v2c(s, m);
      update_c2v(s, m);
      update_soft(s, m);
    }
    if (crc_poly >= 0) {
      memset(out_packed, 0, out_bytes);
      int ok = orc_hard_decision(out_packed, s->soft, msg_len);
      if (ok && orc_crc_packed(crc_poly, out_packed, nof_significant_bits) == 0) {
        free(s);
        return (int)it + 1;
      }
    }
  }
  if (crc_poly < 0) {
    memset(out_packed, 0, out_bytes);
    orc_hard_decision(out_packed, s->soft, msg_len);
  }
  free(s);
  return 0;
}

/* ------------------------------------------------------------------------------------------------------------ */
/* Rate dematcher -- ldpc_rate_dematcher_impl.cpp:33-213                                                        */
/* ------------------------------------------------------------------------------------------------------------ */

int orc_rate_dematch(int8_t* out, unsigned cb_len, const int8_t* in, unsigned E, int new_data, unsigned rv,
                     unsigned Qm, unsigned Nref, unsigned nof_filler_bits)
{
  static const double sf_bg1[4] = {0, 17, 33, 56}, sf_bg2[4] = {0, 13, 25, 43}; /* :33-34 */
  if (rv > 3 || Qm == 0 || E % Qm != 0 || cb_len > 66 * 384) {
    return -1;
  }
  unsigned       block_length  = cb_len;
  unsigned       buffer_length = (Nref > 0) ? (Nref < block_length ? Nref : block_length) : block_length;
  const double*  shift_factor;
  unsigned       bg_k;
  if (block_length % 66 == 0) { /* :76-90: BG1 is tested first */
    shift_factor = sf_bg1;
    bg_k         = 22;
  } else if (block_length % 50 == 0) {
    shift_factor = sf_bg2;
    bg_k         = 10;
  } else {
    return -1;
  }
  unsigned Z = block_length / (bg_k == 22 ? 66 : 50);
  if (orc_lifting_index(Z) < 0) {
    return -1;
  }
  unsigned nof_systematic = (bg_k - 2) * Z;
  if (nof_filler_bits >= nof_systematic) {
    return -1;
  }
  unsigned shift_k0 = (unsigned)floor((shift_factor[rv] * buffer_length) / block_length) * Z; /* :104-105 */

  /* deinterleave_bits_Qm (:203-213): out[(E/Qm)*j + i] = in[i*Qm + j] */
  int8_t* aux = (int8_t*)malloc(E ? E : 1);
  if (aux == NULL) {
    return -1;
  }
  if (Qm == 1) {
    memcpy(aux, in, E);
  } else {
    unsigned K = E / Qm;
    for (unsigned idx = 0, i = 0; i != K; ++i) {
      for (unsigned j = 0; j != Qm; ++j, ++idx) {
        aux[K * j + i] = in[idx];
      }
    }
  }

  /* allot_llrs (:128-201) */
  unsigned       nof_info = nof_systematic - nof_filler_bits;
  int            copy     = new_data ? 1 : 0;
  unsigned       tmp_idx  = shift_k0;
  const int8_t*  cur      = aux;
  unsigned       left     = E;
  while (left != 0) {
    if (tmp_idx < nof_info) {
      unsigned n = nof_info - tmp_idx;
      if (n > left) {
        n = left;
      }
      if (copy) {
        memset(out, 0, tmp_idx);
        memcpy(out + tmp_idx, cur, n);
      } else {
        for (unsigned i = 0; i != n; ++i) {
          out[tmp_idx + i] = orc_llr_add(out[tmp_idx + i], cur[i]);
        }
      }
      tmp_idx += n;
      cur += n;
      left -= n;
    } else if (copy) {
      memset(out, 0, nof_info);
    }
    if (copy) {
      memset(out + nof_info, LLR_INF, nof_filler_bits);
    }
    if (tmp_idx < nof_systematic) {
      tmp_idx = nof_systematic;
    }
    unsigned np = buffer_length - tmp_idx;
    if (np > left) {
      np = left;
    }
    if (copy) {
      memcpy(out + tmp_idx, cur, np);
    } else {
      for (unsigned i = 0; i != np; ++i) {
        out[tmp_idx + i] = orc_llr_add(out[tmp_idx + i], cur[i]);
      }
    }
    tmp_idx = (tmp_idx + np) % buffer_length;
    cur += np;
    left -= np;
    if (left != 0) {
      copy = 0;
    }
  }
  if (copy && tmp_idx != 0) {
    /* out.last(buffer_length - tmp_idx): the LAST (Ncb - tmp_idx) entries of the N-sized output (:197-200). */
    unsigned cnt = buffer_length - tmp_idx;
    memset(out + block_length - cnt, 0, cnt);
  }
  free(aux);
  return 0;
}

/* ------------------------------------------------------------------------------------------------------------ */
/* Encoder (TS 38.212 §5.3.2) -- test-vector generation. Core parity solved by GF(2) elimination (not the        */
/* reference's closed forms), extension parity by the row equations.                                             */
/* ------------------------------------------------------------------------------------------------------------ */

typedef struct {
  int       bg;
  unsigned  Z;
  unsigned  n;     /* 4Z */
  unsigned  words; /* ceil(n/64) */
  uint64_t* inv;   /* n x words rows of A^{-1} */
} core_inverse;

static core_inverse g_inv = {0, 0, 0, 0, NULL};

static int build_core_inverse(const graph_t* g)
{
  if (g_inv.inv != NULL && g_inv.bg == g->bg && g_inv.Z == g->Z) {
    return 0;
  }
  free(g_inv.inv);
  g_inv.inv = NULL;
  const unsigned Z = g->Z, K = g->K, n = 4 * Z, W = (2 * n + 63) / 64;
  uint64_t*      aug = (uint64_t*)calloc((size_t)n * W, sizeof(uint64_t));
  if (aug == NULL) {
    return -1;
  }
  /* Row (m,t): sum over core edges (m, K+c, s) of p_c[(t + s) % Z]. Columns 0..n-1 = unknowns, n..2n-1 = I. */
  for (unsigned m = 0; m != 4; ++m) {
    for (unsigned t = 0; t != Z; ++t) {
      uint64_t* row = aug + (size_t)(m * Z + t) * W;
      for (int k = 0; k != g->deg[m]; ++k) {
        unsigned col = g->cols[m][k];
        if (col >= K && col < K + 4) {
          unsigned u = (col - K) * Z + (t + g->shifts[m][k]) % Z;
          row[u / 64] ^= 1ULL << (u % 64);
        }
      }
      unsigned u = n + m * Z + t;
      row[u / 64] |= 1ULL << (u % 64);
    }
  }
  for (unsigned c = 0; c != n; ++c) {
    unsigned piv = c;
    while (piv < n && !((aug[(size_t)piv * W + c / 64] >> (c % 64)) & 1ULL)) {
      ++piv;
    }
    if (piv == n) {
      free(aug);
      return -1;
    }
    if (piv != c) {
      for (unsigned w = 0; w != W; ++w) {
        uint64_t tmp                 = aug[(size_t)piv * W + w];
        aug[(size_t)piv * W + w]     = aug[(size_t)c * W + w];
        aug[(size_t)c * W + w]       = tmp;
      }
    }
    for (unsigned r = 0; r != n; ++r) {
      if (r != c && ((aug[(size_t)r * W + c / 64] >> (c % 64)) & 1ULL)) {
        for (unsigned w = 0; w != W; ++w) {
          aug[(size_t)r * W + w] ^= aug[(size_t)c * W + w];
        }
      }
    }
  }
  const unsigned IW = (n + 63) / 64;
  g_inv.inv         = (uint64_t*)calloc((size_t)n * IW, sizeof(uint64_t));
  for (unsigned r = 0; r != n; ++r) {
    for (unsigned c = 0; c != n; ++c) {
      unsigned u = n + c;
      if ((aug[(size_t)r * W + u / 64] >> (u % 64)) & 1ULL) {
        g_inv.inv[(size_t)r * IW + c / 64] |= 1ULL << (c % 64);
      }
    }
  }
  free(aug);
  g_inv.bg    = g->bg;
  g_inv.Z     = Z;
  g_inv.n     = n;
  g_inv.words = IW;
  return 0;
}

int orc_ldpc_encode(int bg, unsigned Z, const uint8_t* msg_bits, uint8_t* cw_bits, unsigned cb_len)
{
  graph_t g;
  if (graph_init(&g, bg, Z) != 0 || build_core_inverse(&g) != 0) {
    return -1;
  }
  const unsigned K = g.K, N_full = g.N_full;
  if (cb_len > (N_full - 2) * Z) {
    return -1;
  }
  uint8_t* c = (uint8_t*)calloc((size_t)N_full * Z, 1);
  if (c == NULL) {
    return -1;
  }
  for (unsigned i = 0; i != K * Z; ++i) {
    c[i] = (msg_bits[i] == ORC_FILLER_BIT) ? 0 : (msg_bits[i] & 1U);
  }
  /* syndrome of the core rows from the systematic part */
  const unsigned n  = 4 * Z;
  uint8_t*       b  = (uint8_t*)calloc(n, 1);
  for (unsigned m = 0; m != 4; ++m) {
    for (int k = 0; k != g.deg[m]; ++k) {
      unsigned col = g.cols[m][k];
      if (col < K) {
        for (unsigned t = 0; t != Z; ++t) {
          b[m * Z + t] ^= c[col * Z + (t + g.shifts[m][k]) % Z];
        }
      }
    }
  }
  for (unsigned r = 0; r != n; ++r) {
    unsigned acc = 0;
    for (unsigned cidx = 0; cidx != n; ++cidx) {
      if ((g_inv.inv[(size_t)r * g_inv.words + cidx / 64] >> (cidx % 64)) & 1ULL) {
        acc ^= b[cidx];
      }
    }
    c[K * Z + r] = (uint8_t)acc;
  }
  free(b);
  /* extension parity: row m >= 4 has identity on column K + m */
  for (unsigned m = 4; m != g.M; ++m) {
    for (int k = 0; k != g.deg[m]; ++k) {
      unsigned col = g.cols[m][k];
      if (col < K + 4) {
        for (unsigned t = 0; t != Z; ++t) {
          c[(K + m) * Z + t] ^= c[col * Z + (t + g.shifts[m][k]) % Z];
        }
      }
    }
  }
  for (unsigned i = 0; i != cb_len; ++i) {
    unsigned p = 2 * Z + i;
    cw_bits[i] = (p < K * Z && msg_bits[p] == ORC_FILLER_BIT) ? ORC_FILLER_BIT : c[p];
  }
  free(c);
  return 0;
}

/* Rate matching (TS 38.212 §5.4.2.1 bit selection, §5.4.2.2 bit interleaving). */
int orc_rate_match(uint8_t* out_bits, unsigned E, const uint8_t* cw_bits, unsigned N, unsigned rv, unsigned Qm,
                   unsigned Nref, int bg, unsigned Z)
{
  static const unsigned sf_bg1[4] = {0, 17, 33, 56}, sf_bg2[4] = {0, 13, 25, 43};
  if (rv > 3 || Qm == 0 || E % Qm != 0) {
    return -1;
  }
  unsigned Ncb  = (Nref > 0 && Nref < N) ? Nref : N;
  unsigned nsh  = (bg == 1) ? 66 : 50;
  unsigned k0   = (unsigned)(((unsigned long long)(bg == 1 ? sf_bg1[rv] : sf_bg2[rv]) * Ncb) / (nsh * Z)) * Z;
  uint8_t* e    = (uint8_t*)malloc(E ? E : 1);
  unsigned k = 0, j = 0, guard = 0;
  while (k < E) {
    uint8_t v = cw_bits[(k0 + j) % Ncb];
    if (v != ORC_FILLER_BIT) {
      e[k++] = v;
      guard  = 0;
    } else if (++guard > Ncb) {
      free(e);
      return -1;
    }
    ++j;
  }
  unsigned EQ = E / Qm;
  for (unsigned jj = 0; jj != EQ; ++jj) {
    for (unsigned i = 0; i != Qm; ++i) {
      out_bits[i + jj * Qm] = e[i * EQ + jj];
    }
  }
  free(e);
  return 0;
}

/* ------------------------------------------------------------------------------------------------------------ */
/* RX segmenter -- ldpc_segmenter_impl.cpp:58-69, 254-331; ldpc.h:124-217                                        */
/* ------------------------------------------------------------------------------------------------------------ */

int orc_segment_rx(unsigned tbs, int bg, unsigned nof_ch_symbols, unsigned Qm, unsigned nof_layers,
                   orc_cb_meta* out, unsigned max_cbs)
{
  if ((bg != 1 && bg != 2) || nof_layers < 1 || nof_layers > 4 || nof_ch_symbols % nof_layers != 0) {
    return -1;
  }
  unsigned tb_crc  = (tbs <= 3824) ? 16 : 24;           /* compute_tb_crc_size */
  unsigned B       = tbs + tb_crc;
  unsigned max_seg = (bg == 1) ? 8448 : 3840;
  unsigned C       = (B <= max_seg) ? 1 : (B + (max_seg - 24) - 1) / (max_seg - 24); /* compute_nof_codeblocks */
  if (C > max_cbs) {
    return -1;
  }
  unsigned Bp = B + ((C > 1) ? 24 * C : 0);
  unsigned kb = 22;                                     /* compute_lifting_size */
  if (bg == 2) {
    kb = (B > 640) ? 10 : (B > 560) ? 9 : (B > 192) ? 8 : 6;
  }
  unsigned Z = 0;
  for (int i = 0; i != 51; ++i) {
    if (k_lifting_sizes[i] * C * kb >= Bp) {
      Z = k_lifting_sizes[i];
      break;
    }
  }
  if (Z == 0) {
    return -1;
  }
  unsigned seg_len    = ((bg == 1) ? 22 : 10) * Z;      /* compute_codeblock_size */
  unsigned crc_len    = (C > 1) ? 24 : 0;
  unsigned max_info   = (Bp + C - 1) / C - crc_len;
  unsigned sym_layer  = nof_ch_symbols / nof_layers;
  unsigned nof_short  = C - (sym_layer % C);
  unsigned cw_offset  = 0;
  for (unsigned r = 0; r != C; ++r) {
    out[r].bg              = bg;
    out[r].lifting_size    = Z;
    out[r].nof_segments    = C;
    out[r].full_length     = seg_len * ((bg == 1) ? 3 : 5);
    out[r].nof_filler_bits = seg_len - (max_info + crc_len);
    out[r].nof_crc_bits    = (C == 1) ? tb_crc : 24;
    unsigned tmp           = (r < nof_short) ? sym_layer / C : (sym_layer + C - 1) / C;
    out[r].rm_length       = tmp * nof_layers * Qm;
    out[r].cw_offset       = cw_offset;
    cw_offset += out[r].rm_length;
  }
  return (int)C;
}

/* ------------------------------------------------------------------------------------------------------------ */
/* pusch_codeblock_decoder::decode -- pusch_codeblock_decoder.cpp:35-71                                          */
/* ------------------------------------------------------------------------------------------------------------ */

int orc_pusch_cb_decode(uint8_t* out_packed, int8_t* soft_buf, unsigned cb_len, const int8_t* llr_E, unsigned E,
                        int new_data, int bg, unsigned Z, unsigned rv, unsigned Qm, unsigned Nref,
                        unsigned nof_filler_bits, int crc_poly, int use_early_stop, unsigned nof_iterations)
{
  if (orc_rate_dematch(soft_buf, cb_len, llr_E, E, new_data, rv, Qm, Nref, nof_filler_bits) != 0) {
    return -1;
  }
  if (use_early_stop) {
    return orc_ldpc_decode(bg, Z, nof_filler_bits, soft_buf, cb_len, nof_iterations, 0.8f, crc_poly, out_packed);
  }
  int r = orc_ldpc_decode(bg, Z, nof_filler_bits, soft_buf, cb_len, nof_iterations, 0.8f, -1, out_packed);
  if (r < 0) {
    return r;
  }
  unsigned K = (bg == 1) ? 22 : 10;
  if (orc_crc_packed(crc_poly, out_packed, K * Z - nof_filler_bits) == 0) {
    return (int)nof_iterations;
  }
  return 0;
}

/* ---- pusch_decoder_impl::join_and_notify (pusch_decoder_impl.cpp:384-444) and concatenate_codeblocks (:446-497) -- */
static unsigned orc_get_bit(const uint8_t* packed, unsigned i) { return (packed[i / 8] >> (7 - i % 8)) & 1U; }
static void     orc_set_bit(uint8_t* packed, unsigned i, unsigned b)
{
  const uint8_t m = (uint8_t)(0x80U >> (i % 8));
  packed[i / 8]   = b ? (uint8_t)(packed[i / 8] | m) : (uint8_t)(packed[i / 8] & ~m);
}

int orc_tb_join(const uint8_t* msgs, unsigned msg_stride, unsigned nof_cbs, unsigned cb_msg_bits,
                unsigned nof_filler_bits, unsigned cb_crc_bits, unsigned tbs, const uint8_t* cb_crc_ok,
                uint8_t* tb_out)
{
  if (nof_cbs == 0) {
    return 0;
  }
  if (nof_cbs == 1) {
    /* one CB: its CRC is the TB CRC; the TB bits are copied only when it passed (:409-417) */
    if (!cb_crc_ok[0]) {
      return 0;
    }
    for (unsigned i = 0; i != tbs; ++i) {
      orc_set_bit(tb_out, i, orc_get_bit(msgs, i));
    }
    return 1;
  }
  for (unsigned r = 0; r != nof_cbs; ++r) {
    if (!cb_crc_ok[r]) {
      return 0; /* :418 -- nothing to do when a CB CRC failed */
    }
  }
  /* concatenate_codeblocks (:446-497): data bits per CB = K*Z - CRC - filler (get_cblk_bit_breakdown :62-64) */
  const unsigned nof_data_bits = cb_msg_bits - cb_crc_bits - nof_filler_bits;
  unsigned       tb_offset     = 0;
  uint32_t       checksum      = 0;
  for (unsigned r = 0; r != nof_cbs; ++r) {
    const uint8_t* cb           = msgs + (size_t)r * msg_stride;
    const unsigned free_tb_bits = tbs - tb_offset;
    const unsigned nof_new_bits = free_tb_bits < nof_data_bits ? free_tb_bits : nof_data_bits;
    for (unsigned i = 0; i != nof_new_bits; ++i) {
      orc_set_bit(tb_out, tb_offset + i, orc_get_bit(cb, i));
    }
    if (r == nof_cbs - 1) {
      for (unsigned i = 0; i != 24; ++i) {
        checksum = (checksum << 1) | orc_get_bit(cb, nof_new_bits + i);
      }
    }
    tb_offset += nof_new_bits;
  }
  /* crc24A over the TB bytes (:424-425), as a bit_buffer of tbs bits */
  return orc_crc_packed(ORC_CRC24A, tb_out, tbs) == checksum ? 1 : 0;
}

/* ------------------------------------------------------------------------------------------------------------ */
/* Soft demodulation mapper -- lib/phy/upper/channel_modulation/demodulation_mapper_*.cpp   */
/* The reference's portable scalar paths, in float arithmetic without contraction (built -ffp-contract=off).      */
/* ------------------------------------------------------------------------------------------------------------ */

/* demodulation_mapper_intervals.h:33-39 compute_interval_idx, :52-63 interval_function */
static float orc_interval_function(float value, float rcp_noise, float width, int nof, const float* slopes,
                                   const float* intercepts)
{
  /* static_cast<int>(std::floor(.)) as x86-64 executes it (cvttss2si): NaN or out of range -> INT_MIN */
  const float q   = floorf(value / width);
  int         idx = (q >= -2147483648.0F && q < 2147483648.0F) ? (int)q : (-2147483647 - 1);
  idx             = (idx < -nof) ? -nof : idx; /* keeps + nof / 2 from overflowing; clamped below anyway */
  idx += nof / 2;
  idx     = idx < 0 ? 0 : (idx > nof - 1 ? nof - 1 : idx);
  float l = slopes[idx] * value + intercepts[idx];
  l *= rcp_noise;
  return l;
}

/* math_utils.h:37,85-94 is_near_zero(cf_t): |z|^2 < 1e-9 */
static int orc_near_zero(float re, float im) { return re * re + im * im < 1e-9F; }

/* demodulation_mapper_impl.cpp:33-41 demod_BPSK_symbol (range limit 24) */
static int8_t orc_bpsk(float re, float im, float nv)
{
  if (!(nv > 0)) {
    return 0;
  }
  const float gain = 2.0F * 1.41421356237309504880F;
  return orc_llr_quantize(gain * (re + im) / nv, 24.0F);
}

/* demodulation_mapper_qpsk.cpp:133-141 demod_QPSK_symbol (range limit 24) */
static int8_t orc_qpsk(float x, float nv)
{
  if (!(nv > 0)) {
    return 0;
  }
  const float gain = 2.0F * 1.41421356237309504880F;
  return orc_llr_quantize(gain * x / nv, 24.0F);
}

int orc_demodulate_soft(int mod, unsigned nof_symbols, const float* sym, const float* nv, int8_t* llr)
{
  unsigned qm = (mod == 0 || mod == 1) ? 1U : (unsigned)mod;
  if (!(mod == 0 || mod == 1 || mod == 2 || mod == 4 || mod == 6 || mod == 8)) {
    return -1;
  }
  /* constants as the reference computes them, in float */
  const float s10 = 1.0F / sqrtf(10.0F), s42 = 1.0F / sqrtf(42.0F), s170 = 1.0F / sqrtf(170.0F);
  /* demodulation_mapper_qam64.cpp:36-67 */
  const float w64a = 2 * s42, w64c = 4 * s42;
  const float sl64_01[8] = {16 * s42, 12 * s42, 8 * s42, 4 * s42, 4 * s42, 8 * s42, 12 * s42, 16 * s42};
  const float ic64_01[8] = {24.0F / 21, 12.0F / 21, 4.0F / 21, 0.0F, 0.0F, -4.0F / 21, -12.0F / 21, -24.0F / 21};
  const float sl64_23[8] = {8 * s42, 4 * s42, 4 * s42, 8 * s42, -8 * s42, -4 * s42, -4 * s42, -8 * s42};
  const float ic64_23[8] = {20.0F / 21, 8.0F / 21, 8.0F / 21, 12.0F / 21, 12.0F / 21, 8.0F / 21, 8.0F / 21, 20.0F / 21};
  const float sl64_45[8] = {4 * s42, -4 * s42, 4 * s42, -4 * s42, 0, 0, 0, 0};
  const float ic64_45[8] = {12.0F / 21, -4.0F / 21, -4.0F / 21, 12.0F / 21, 0, 0, 0, 0};
  /* demodulation_mapper_qam256.cpp:37-160 */
  const float w256a = 2 * s170, w256c = 4 * s170;
  float       sl256_01[16], ic256_01[16], sl256_23[16], ic256_23[16], sl256_45[16], ic256_45[16], sl256_67[8],
      ic256_67[8];
  {
    static const int   k01[16] = {32, 28, 24, 20, 16, 12, 8, 4, 4, 8, 12, 16, 20, 24, 28, 32};
    static const float n01[16] = {112, 84, 60, 40, 24, 12, 4, 0, 0, -4, -12, -24, -40, -60, -84, -112};
    static const int   k23[16] = {16, 12, 8, 4, 4, 8, 12, 16, -16, -12, -8, -4, -4, -8, -12, -16};
    static const float n23[16] = {88, 60, 36, 16, 16, 28, 36, 40, 40, 36, 28, 16, 16, 36, 60, 88};
    static const int   k45[16] = {8, 4, 4, 8, -8, -4, -4, -8, 8, 4, 4, 8, -8, -4, -4, -8};
    static const float n45[16] = {52, 24, 24, 44, -20, -8, -8, -12, -12, -8, -8, -20, 44, 24, 24, 52};
    static const int   k67[8]  = {4, -4, 4, -4, 4, -4, 4, -4};
    static const float n67[8]  = {28, -20, 12, -4, -4, 12, -20, 28};
    for (int i = 0; i != 16; ++i) {
      sl256_01[i] = (float)k01[i] * s170;
      ic256_01[i] = n01[i] / 85;
      sl256_23[i] = (float)k23[i] * s170;
      ic256_23[i] = n23[i] / 85;
      sl256_45[i] = (float)k45[i] * s170;
      ic256_45[i] = n45[i] / 85;
    }
    for (int i = 0; i != 8; ++i) {
      sl256_67[i] = (float)k67[i] * s170;
      ic256_67[i] = n67[i] / 85;
    }
  }
  for (unsigned i = 0; i != nof_symbols; ++i) {
    const float re = sym[2 * i], im = sym[2 * i + 1], n = nv[i];
    int8_t*     o  = llr + (size_t)i * qm;
    switch (mod) {
      case 1: /* demodulation_mapper_impl.cpp:43-51 */
        o[0] = orc_bpsk(re, im, n);
        break;
      case 0: /* :53-76: odd-indexed symbols rotated by -pi/2: (im, -re) */
        o[0] = (i % 2 == 0) ? orc_bpsk(re, im, n) : orc_bpsk(im, -re, n);
        break;
      case 2: /* demodulation_mapper_qpsk.cpp:143-169 (scalar loop) */
        o[0] = orc_qpsk(re, n);
        o[1] = orc_qpsk(im, n);
        break;
      case 4: /* demodulation_mapper_qam16.cpp:230-273 (scalar loop), demod_16QAM_symbol_01/_23 :201-228 */
        if (orc_near_zero(re, im)) {
          memset(o, 0, 4);
          break;
        }
        for (int c = 0; c != 2; ++c) {
          const float x = c == 0 ? re : im;
          if (!(n > 0)) {
            o[c] = 0;
            o[2 + c] = 0;
            continue;
          }
          float l01 = 4 * s10 * x;
          if (fabsf(x) > 2 * s10) {
            l01 = 2 * l01 - copysignf(0.8F, x);
          }
          l01 /= n;
          o[c]      = orc_llr_quantize(l01, 24.0F);
          float l23 = 0.8F - 4 * s10 * fabsf(x);
          l23 /= n;
          o[2 + c] = orc_llr_quantize(l23, 24.0F);
        }
        break;
      case 6: /* demodulation_mapper_qam64.cpp:404-463 (scalar loop, range limit 20) */
      case 8: /* demodulation_mapper_qam256.cpp:378-427 (scalar loop, range limit 20) */
      {
        if (orc_near_zero(re, im)) {
          memset(o, 0, qm);
          break;
        }
        const float rn = (n > 0) ? 1 / n : 0.0F;
        for (int c = 0; c != 2; ++c) {
          const float x = c == 0 ? re : im;
          if (mod == 6) {
            o[c]     = orc_llr_quantize(orc_interval_function(x, rn, w64a, 8, sl64_01, ic64_01), 20.0F);
            o[2 + c] = orc_llr_quantize(orc_interval_function(x, rn, w64a, 8, sl64_23, ic64_23), 20.0F);
            o[4 + c] = orc_llr_quantize(orc_interval_function(x, rn, w64c, 4, sl64_45, ic64_45), 20.0F);
          } else {
            o[c]     = orc_llr_quantize(orc_interval_function(x, rn, w256a, 16, sl256_01, ic256_01), 20.0F);
            o[2 + c] = orc_llr_quantize(orc_interval_function(x, rn, w256a, 16, sl256_23, ic256_23), 20.0F);
            o[4 + c] = orc_llr_quantize(orc_interval_function(x, rn, w256a, 16, sl256_45, ic256_45), 20.0F);
            o[6 + c] = orc_llr_quantize(orc_interval_function(x, rn, w256c, 8, sl256_67, ic256_67), 20.0F);
          }
        }
        break;
      }
    }
  }
  return 0;
}
