/* Compile-time step schedules for the specialised decoders (ldpc_decode_kernel with a spec::sgraph).
 *
 * The generic kernel reads every step's work from a task table and every edge's (column, shift) from an LDS edge
 * table at run time. For the lifting sizes that carry the throughput, the schedule is built here as a constexpr object
 * from the same base-graph table (ldpc_base_graphs.inc) and the kernel unrolls a whole iteration with every column,
 * shift and c2v slot as an instruction immediate.
 *
 * Schedule (bit-identical to the layer-serial order of ldpc_decoder_impl.cpp:116-123): consecutive rows whose column
 * sets are pairwise disjoint form one step (at most two rows per step; a longer run is cut into steps of two), one
 * barrier per step. A single-row step of degree >= SPLIT_MIN_DEGREE splits each check node's edges over lanes l and
 * l ^ 32 (P = 2) so that twice as many waves work on it.
 *
 *
 * Edge pairs. The kernel keeps two edges of a check node in the two 16-bit halves of one register and updates both
 * with one packed instruction (v_pk_*). Each role's edges are listed as positions (P = 1: the row's edges in order;
 * P = 2: e0[j] for lanes 0-31, e1[j] for lanes 32-63, the upper half taking the row's second half); positions 2i and
 * 2i + 1 form pair i, and a position without an edge (-1) is a dummy: a scratch soft bit at +infinity, which never
 * changes the minima or the sign parity. One c2v register per pair slot.
 */
#pragma once

#include <cstdint>

namespace ldpc_hip {
namespace spec {

struct cedge {
  int bg, row, col;
  int sh[8];
};

constexpr cedge k_edges[] = {
#define LDPC_EDGE(bg, r, c, s0, s1, s2, s3, s4, s5, s6, s7) {bg, r, c, {s0, s1, s2, s3, s4, s5, s6, s7}},
#include "ldpc_base_graphs.inc"
#undef LDPC_EDGE
};
constexpr int k_nof_edges = static_cast<int>(sizeof(k_edges) / sizeof(k_edges[0]));

constexpr int MAX_ROWS  = 46;
constexpr int MAX_DEG   = 19;
constexpr int MAX_STEPS = 48;
#ifndef LDPC_SPEC_MAX_POS
#define LDPC_SPEC_MAX_POS 12
#endif
constexpr int MAX_POS   = LDPC_SPEC_MAX_POS; /* positions (edge slots) per lane and step */

/* A single-row step of this degree or more is split over lane pairs (P = 2). Splitting doubles the waves on the row
 * but costs a per-lane address select per edge and the partner merge; below degree 12 the unsplit row (6 waves, two
 * on the busiest SIMD) is faster (C2 batch: 163 us against 167 us with every single row of degree >= 6 split). */
#ifndef LDPC_SPEC_SPLIT_MIN_DEGREE
#define LDPC_SPEC_SPLIT_MIN_DEGREE 12
#endif
constexpr int SPLIT_MIN_DEGREE = LDPC_SPEC_SPLIT_MIN_DEGREE;
/* Graphs with fewer waves per row (Z <= 320: at most 5) and BG2 (no row of degree 12) take their own thresholds;
 * splitting their single rows from degree 8, 6 or 4 was 1-12% slower on every graph (profiles/r02/split_variants.txt),
 * so none is split. */
#ifndef LDPC_SPEC_SPLIT_SMALL
#define LDPC_SPEC_SPLIT_SMALL 12
#endif
#ifndef LDPC_SPEC_SPLIT_BG2
#define LDPC_SPEC_SPLIT_BG2 12
#endif
/* Graphs with one wave per row (Z <= 64) keep their single rows unsplit too: splitting from degree 4 or 6 was 1-12%
 * slower on every such graph (BG2 Z=36: 63.1 -> 71.0 / 66.0 us per 128-CB batch, profiles/r04/small_z_split_ab.txt):
 * at one wave per SIMD a step's time is its wave's instruction count, and the partner merge adds more than the
 * halved edge work removes. */
constexpr int split_min_degree(int bg, int W)
{
  return W <= 5 ? LDPC_SPEC_SPLIT_SMALL : (bg == 2 ? LDPC_SPEC_SPLIT_BG2 : SPLIT_MIN_DEGREE);
}

/* Precomputed addresses of BG1's split rows (0-3, degree 19: five address pairs per lane each): rows
 * [0, LDPC_SPEC_SPLIT_ADDR_ROWS) in registers, rows [LDPC_SPEC_SPLIT_ADDR_ROWS, LDPC_SPEC_SPLIT_LDS_ROWS) in an LDS
 * table (ldpc_decode_body.h, dec::fill_split), the rest computed in the step. */
#ifndef LDPC_SPEC_SPLIT_ADDR_ROWS
#define LDPC_SPEC_SPLIT_ADDR_ROWS 0
#endif
#ifndef LDPC_SPEC_SPLIT_LDS_ROWS
#define LDPC_SPEC_SPLIT_LDS_ROWS 4
#endif
/* 1: the LDS table is copied from the context's global copy (written once per context by ldpc_split_table_kernel) in
 * each codeblock's prologue; 0: computed by every codeblock (dec::fill_split) */
#ifndef LDPC_SPEC_SPLIT_COPY
#define LDPC_SPEC_SPLIT_COPY 1
#endif
/* LDS table size in address pairs per lane (a BG1 workgroup's waves x 64 lanes, 4 bytes each) */
constexpr int SPLIT_LDS_PAIRS = LDPC_SPEC_SPLIT_LDS_ROWS > LDPC_SPEC_SPLIT_ADDR_ROWS
                                    ? 5 * (LDPC_SPEC_SPLIT_LDS_ROWS - LDPC_SPEC_SPLIT_ADDR_ROWS) : 0;

/* Soft-bit copies per column in LDS: 1 (one write per edge; the lane computes (t + shift) mod Z, three VALU
 * instructions) or 4 (reads and writes at t + shift without a modulo, three writes per edge). An LDS write costs
 * 4 cycles of the CU's LDS pipe whatever its width or active lanes (tools/ubench/lds3.hip, lds4.hip); on the C2 batch
 * one copy is 172 us, four copies 182 us (profiles/r02/variants.txt). */
#ifndef LDPC_SPEC_SOFT_COPIES
#define LDPC_SPEC_SOFT_COPIES 1
#endif
constexpr int SOFT_COPIES = LDPC_SPEC_SOFT_COPIES;
static_assert(SOFT_COPIES == 1 || SOFT_COPIES == 4, "soft-bit copies");

/* Soft-bit element of the specialised decoders, in LDS and in their registers: 1 = int8; 2 = IEEE binary16 holding
 * the same integers (exact: every value the decoder forms is an integer of magnitude below 2048). In binary16 a
 * value's sign and magnitude are separate bits, so |v2c|, the sign parity and every sign application of the
 * check-node update become full-rate bitwise VOP2 instructions (v_and / v_xor / v_or on both halves at once) instead
 * of half-rate packed ones (sp::pass1 / pass2: 474 fewer packed and 612 more full-rate instructions per BG1 Z=384
 * iteration, tools/step_isa.py), with ds_read_u16 / ds_write_b16 at even addresses. Bit-exact (tests/test_f16_arith.py
 * exhaustively, the whole -m gpu suite on the GPU), and no faster: C2 137.5 against 137.0 us, every other graph within
 * +-2% (profiles/r05/ab_f16_vs_i8.txt) -- as round 3's XOR-sign variant found, trading packed instructions for more
 * full-rate ones does not pay in this kernel. Off by default; -DLDPC_SPEC_F16=1 builds it. */
#ifndef LDPC_SPEC_F16
#define LDPC_SPEC_F16 0
#endif
constexpr int SOFT_BYTES = LDPC_SPEC_F16 ? 2 : 1;
static_assert(SOFT_BYTES == 1 || SOFT_COPIES == 1, "binary16 soft bits: one copy per column");

struct srow {
  int deg = 0;
  int e0  = 0; /* first edge of the row in row-major edge order */
  int col[MAX_DEG] = {};
  int sh[MAX_DEG]  = {}; /* shift mod Z */
};

/* One role of a step: one row, its edge list per position. P = 1: e0[j]; P = 2: e0[j] (lanes 0-31) and e1[j]
 * (lanes 32-63), -1 = dummy. grp: the wave group that runs it (P = 1: waves [grp W, (grp + 1) W); P = 2: every wave).
 * nearly: positions [0, nearly) (whole pairs) were read and passed through pass 1 in the previous step by the same
 * wave group (see sstep::e). q0: first c2v pair slot (slots q0 .. q0 + (npos + 1) / 2 - 1 of the group's lanes). */
struct srole {
  int row = -1, p = 1, npos = 0, grp = 0, nearly = 0, q0 = 0;
  int e0[MAX_POS] = {};
  int e1[MAX_POS] = {};
};

/* Pipelined single-row chains. Two consecutive single-row steps (P = 1, one row each) of rows r and r + 1 alternate
 * wave groups: while group g runs row r, the idle group 1 - g reads row r + 1's soft bits of the columns row r does
 * not write and runs pass 1 of those edges (the two-minimum scan and the sign parity are independent of the edge
 * order), keeping the partial minima, parity, v2c magnitudes, signs and addresses in registers across the barrier; in
 * the next step it reads the remaining (shared-column) edges, finishes pass 1 and updates the row. Every soft bit is
 * read after the last write to it in layer order, so the result is bit-identical to the serial schedule. */
#ifndef LDPC_SPEC_PIPELINE
#define LDPC_SPEC_PIPELINE 1
#endif

struct sstep {
  srole r[2]; /* r[1].row < 0 for a single-row step */
  srole e;    /* e.row >= 0: the next step's row whose early positions group e.grp runs in this step */
};

struct sgraph {
  int   bg = 0, Z = 0, M = 0, N_full = 0, K = 0, n_steps = 0, ils = 0;
  int   W     = 0; /* waves per unsplit row, ceil(Z / 64)              */
  int   waves = 0; /* waves per workgroup: max(2 W, ceil(Z / 32))     */
  int   slots = 0; /* c2v pair slots (registers) per lane per iteration */
  bool  valid = false;
  srow  rows[MAX_ROWS]   = {};
  sstep steps[MAX_STEPS] = {};
};

constexpr bool rows_share_column(const srow& a, const srow& b)
{
  for (int i = 0; i < a.deg; ++i) {
    for (int j = 0; j < b.deg; ++j) {
      if (a.col[i] == b.col[j]) {
        return true;
      }
    }
  }
  return false;
}

constexpr bool row_has_column(const srow& r, int c)
{
  for (int i = 0; i < r.deg; ++i) {
    if (r.col[i] == c) {
      return true;
    }
  }
  return false;
}

constexpr bool is_single_p1(const sstep& st) { return st.r[1].row < 0 && st.r[0].p == 1; }

constexpr void make_role(const sgraph& g, srole& ro)
{
  const int d = g.rows[ro.row].deg;
  if (ro.p == 1) {
    for (int k = 0; k < d; ++k) {
      ro.e0[ro.npos++] = k;
    }
    return;
  }
  const int h = (d + 1) / 2; /* lanes 0-31: edges [0, h), lanes 32-63: [h, d) */
  for (int j = 0; j < h; ++j) {
    ro.e0[j] = j;
    ro.e1[j] = (h + j < d) ? h + j : -1;
  }
  ro.npos = h;
}


/* ils: lifting-set index of Z (TS 38.212 Table 5.3.2-1). */
constexpr sgraph make(int bg, int Z, int ils)
{
  sgraph g{};
  g.bg     = bg;
  g.Z      = Z;
  g.ils    = ils;
  g.M      = (bg == 1) ? 46 : 42;
  g.N_full = (bg == 1) ? 68 : 52;
  g.K      = g.N_full - g.M;
  g.W      = (Z + 63) / 64;
  g.waves  = (2 * g.W > (Z + 31) / 32) ? 2 * g.W : (Z + 31) / 32;
  int e    = 0;
  for (int m = 0; m < g.M; ++m) {
    g.rows[m].e0 = e;
    for (int i = 0; i < k_nof_edges; ++i) {
      if (k_edges[i].bg == bg && k_edges[i].row == m) {
        srow& r      = g.rows[m];
        r.col[r.deg] = k_edges[i].col;
        r.sh[r.deg]  = k_edges[i].sh[ils] % Z;
        ++r.deg;
        ++e;
      }
    }
  }
  bool ok = Z >= 2 && g.waves <= 12;
  int  m  = 0;
  while (m < g.M && g.n_steps < MAX_STEPS) {
    const bool pair = m + 1 < g.M && !rows_share_column(g.rows[m], g.rows[m + 1]);
    sstep&     st   = g.steps[g.n_steps];
    st.r[0].row     = m;
    st.r[1].row     = pair ? m + 1 : -1;
    st.r[0].p       = (!pair && g.rows[m].deg >= split_min_degree(bg, g.W)) ? 2 : 1;
    ++g.n_steps;
    m += pair ? 2 : 1;
  }
  ok = ok && m == g.M;
  /* wave groups: pairs take groups 0 and 1, a single-row step after another single-row P = 1 step the other group */
  for (int s = 0; s < g.n_steps; ++s) {
    sstep& st = g.steps[s];
    for (srole& ro : st.r) {
      if (ro.row >= 0) {
        make_role(g, ro);
        ok = ok && ro.npos <= MAX_POS;
      }
    }
    if (st.r[1].row >= 0) {
      st.r[1].grp = 1;
    } else if (st.r[0].p == 1 && s > 0 && is_single_p1(g.steps[s - 1])) {
      st.r[0].grp = 1 - g.steps[s - 1].r[0].grp;
    }
  }
  /* early positions: the next single row's edges on columns this step's row does not write, first (whole pairs) */
  for (int s = 0; LDPC_SPEC_PIPELINE && s + 1 < g.n_steps; ++s) {
    if (!is_single_p1(g.steps[s]) || !is_single_p1(g.steps[s + 1])) {
      continue;
    }
    srole&      nx   = g.steps[s + 1].r[0];
    const srow& prev = g.rows[g.steps[s].r[0].row];
    const srow& row  = g.rows[nx.row];
    int         ne   = 0;
    for (int pass = 0; pass < 2; ++pass) { /* non-shared edges first, then the shared ones */
      for (int k = 0; k < row.deg; ++k) {
        if (row_has_column(prev, row.col[k]) == (pass == 1)) {
          nx.e0[ne++] = k;
        }
      }
    }
    int early = 0;
    for (int k = 0; k < row.deg; ++k) {
      early += row_has_column(prev, row.col[k]) ? 0 : 1;
    }
    nx.nearly = early & ~1;
    if (nx.nearly > 0) {
      g.steps[s].e = nx;
    }
  }
  /* c2v pair slots: the two wave groups have separate registers, so each group's rows take consecutive slots of
   * their own; a P = 2 row uses every wave (both groups' cursors) */
  int cur[2] = {0, 0};
  for (int s = 0; s < g.n_steps; ++s) {
    for (srole& ro : g.steps[s].r) {
      if (ro.row < 0) {
        continue;
      }
      const int np = (ro.npos + 1) / 2;
      if (ro.p == 2) {
        ro.q0  = cur[0] > cur[1] ? cur[0] : cur[1];
        cur[0] = cur[1] = ro.q0 + np;
      } else {
        ro.q0 = cur[ro.grp];
        cur[ro.grp] += np;
      }
    }
    if (g.steps[s].e.row >= 0) {
      g.steps[s].e.q0 = cur[g.steps[s].e.grp]; /* the next step's role takes exactly these slots */
    }
  }
  g.slots = cur[0] > cur[1] ? cur[0] : cur[1];
  g.valid = ok;
  return g;
}

/* Every early role equals the role that completes it in the next step (same row, group, positions and slots). */
constexpr bool early_roles_match(const sgraph& g)
{
  for (int s = 0; s < g.n_steps; ++s) {
    const srole& e = g.steps[s].e;
    if (e.row < 0) {
      continue;
    }
    if (s + 1 >= g.n_steps) {
      return false;
    }
    const srole& c = g.steps[s + 1].r[0];
    if (c.row != e.row || c.grp != e.grp || c.q0 != e.q0 || c.nearly != e.nearly || c.npos != e.npos || c.p != 1 ||
        e.grp == g.steps[s].r[0].grp || g.steps[s].r[1].row >= 0) {
      return false;
    }
    for (int j = 0; j < c.npos; ++j) {
      if (c.e0[j] != e.e0[j]) {
        return false;
      }
    }
    /* the early positions' columns are not written by this step's row */
    for (int j = 0; j < e.nearly; ++j) {
      if (row_has_column(g.rows[g.steps[s].r[0].row], g.rows[e.row].col[e.e0[j]])) {
        return false;
      }
    }
  }
  return true;
}

/* Is this step's pairing the layer-serial order? (consecutive rows, disjoint columns) */
constexpr bool schedule_is_layer_serial(const sgraph& g)
{
  int next = 0;
  for (int s = 0; s < g.n_steps; ++s) {
    const sstep& st = g.steps[s];
    if (st.r[0].row != next) {
      return false;
    }
    ++next;
    if (st.r[1].row >= 0) {
      if (st.r[1].row != next || rows_share_column(g.rows[st.r[0].row], g.rows[st.r[1].row])) {
        return false;
      }
      ++next;
    }
  }
  return next == g.M;
}

/* Every edge of every row appears exactly once in its role's positions (per half for P = 2). */
constexpr bool roles_cover_edges(const sgraph& g)
{
  for (int s = 0; s < g.n_steps; ++s) {
    for (const srole& ro : g.steps[s].r) {
      if (ro.row < 0) {
        continue;
      }
      const int d = g.rows[ro.row].deg;
      for (int k = 0; k < d; ++k) {
        int n = 0;
        for (int j = 0; j < ro.npos; ++j) {
          n += (ro.e0[j] == k) ? 1 : 0;
          n += (ro.p == 2 && ro.e1[j] == k) ? 1 : 0;
        }
        if (n != 1) {
          return false;
        }
      }
    }
  }
  return true;
}

/* ---- Register-resident schedules of the one-wave graphs (Z <= 64) --------------------------------------------------
 * A Z <= 64 codeblock runs on ONE wave, one lane per check node, with every column's Z soft bits in a register (lane t
 * of column c's register: the soft bit of position (t + rho_c) mod Z, in one 16-bit half). Row r reads edge (c, s) as
 * the value at lane (t + s - rho_c) mod Z of that register (one ds_bpermute_b32, none when s == rho_c), and its
 * updated value for position (t + s) mod Z is computed by lane t: so the result register IS column c's register from
 * then on, with rho_c = s -- writes cost nothing, no LDS round trip, no barrier, and the whole iteration is one
 * straight-line instruction stream the compiler schedules across rows (the next row's reads of columns this row does
 * not write overlap its update). The layer order is still ldpc_decoder_impl.cpp:116-123's, one row after the other.
 *
 * Everything about the registers is compile-time: which column lives in which register half with which rotation at
 * every row (make_reg simulates the iteration), so each read is a constant rotation k = (s - rho_c) mod Z. The state at
 * the iteration boundary is the state after a full iteration (every column is written each iteration), and the
 * codeblock's registers are loaded from LDS in that state. Rows beyond the codeblock's layer count (impl.cpp:103-114)
 * are skipped in chunks: every LDPC_SPEC_REG_EXIT_EVERY rows a uniform branch leaves the iteration, re-rotating the
 * columns the skipped rows would have left elsewhere; rows in the last, partly active chunk run as the identity
 * (their c2v stays zero and their scaled magnitudes are forced to zero: v2c = soft, soft' = soft).
 *
 * Measured (round 5): bit-exact on every graph, and SLOWER than the lane-split decoder below on every one-wave graph
 * (128-CB batches, 8 it: BG2 Z=36 67 against 58 us, BG1 Z=36 120 against 71 us; profiles/r05/ab_reg_vs_quad_v1.txt,
 * ab_reg_nobarrier.txt). One iteration is 2,800 (BG2) to 4,300 (BG1) VALU instructions on ONE SIMD -- an issue floor
 * of 4.4-6.7 us per iteration before any stall -- and the row-to-row dependency chain stalls the lone wave for about
 * as long again (profiles/r05/reg_decoder_isa.txt); the LDS decoders spread the same work over 2-4 waves on
 * different SIMDs. Off by default; -DLDPC_SPEC_REG=1 builds it. */
#ifndef LDPC_SPEC_REG
#define LDPC_SPEC_REG 0
#endif
#ifndef LDPC_SPEC_REG_EXIT_EVERY
#define LDPC_SPEC_REG_EXIT_EVERY 6
#endif
constexpr int REG_MAX_COLS  = 68;
constexpr int REG_MAX_EXITS = 8;
constexpr int REG_ROW_PAIRS = 10; /* register id of row r's pair i: r * REG_ROW_PAIRS + i */

/* a column's register: lane t holds position (t + rho) mod Z in 16-bit half `half` of register `reg` */
struct rcol {
  int rho = 0, half = 0, reg = -1;
};
/* an edge of a row (pair i = edges 2i, 2i + 1): its column, read rotation k = (shift - rho) mod Z, and source state */
struct redge {
  int col = 0, k = 0, half = 0, reg = -1;
};
struct rrow {
  int   deg = 0, q0 = 0; /* q0: first c2v pair register */
  redge e[MAX_DEG] = {};
};
struct rgraph {
  int   n_pairs = 0, n_exits = 0;
  bool  valid = false;
  rrow  rows[MAX_ROWS]      = {};
  rcol  end[REG_MAX_COLS]   = {}; /* at the iteration boundary */
  int   partner[REG_MAX_COLS] = {}; /* the other column of its boundary register, or -1 */
  int   exit_row[REG_MAX_EXITS] = {};
  rcol  at_exit[REG_MAX_EXITS][REG_MAX_COLS] = {}; /* before row exit_row[x] */
};

constexpr bool is_reg(const sgraph& g) { return LDPC_SPEC_REG != 0 && g.Z <= 64; }

constexpr rgraph make_reg(const sgraph& g)
{
  rgraph R{};
  if (!is_reg(g) || !g.valid || g.N_full > REG_MAX_COLS) {
    return R;
  }
  rcol st[REG_MAX_COLS] = {};
  for (int pass = 0; pass < 2; ++pass) { /* pass 0: the boundary state; pass 1: from it, every row's edges */
    int q = 0;
    for (int r = 0; r < g.M; ++r) {
      const srow& row = g.rows[r];
      if (pass == 1 && r >= LDPC_SPEC_REG_EXIT_EVERY && r % LDPC_SPEC_REG_EXIT_EVERY == 0 &&
          R.n_exits < REG_MAX_EXITS) {
        R.exit_row[R.n_exits] = r;
        for (int c = 0; c < g.N_full; ++c) {
          R.at_exit[R.n_exits][c] = st[c];
        }
        ++R.n_exits;
      }
      if (pass == 1) {
        R.rows[r].deg = row.deg;
        R.rows[r].q0  = q;
        for (int e = 0; e < row.deg; ++e) {
          const rcol& s  = st[row.col[e]];
          R.rows[r].e[e] = redge{row.col[e], (row.sh[e] - s.rho + g.Z) % g.Z, s.half, s.reg};
        }
      }
      q += (row.deg + 1) / 2;
      for (int e = 0; e < row.deg; ++e) {
        st[row.col[e]] = rcol{row.sh[e], e & 1, r * REG_ROW_PAIRS + e / 2};
      }
    }
    if (pass == 0) {
      for (int c = 0; c < g.N_full; ++c) {
        R.end[c] = st[c];
      }
    } else {
      R.n_pairs = q;
    }
  }
  bool ok = true;
  for (int c = 0; c < g.N_full; ++c) {
    ok = ok && st[c].reg >= 0 && st[c].reg == R.end[c].reg && st[c].rho == R.end[c].rho && st[c].half == R.end[c].half;
    R.partner[c] = -1;
    for (int o = 0; o < g.N_full; ++o) {
      if (o != c && R.end[o].reg == R.end[c].reg) {
        R.partner[c] = o;
      }
    }
  }
  R.valid = ok;
  return R;
}

/* ---- Lane-split schedules of the one-wave graphs (W == 1, Z <= 64) -------------------------------------------------
 * With one lane per check node a row of a Z <= 64 graph is one wave, whose instruction stream (every edge of the row
 * in turn: about 12 issue slots per edge, 14 per row) sets the step time at one wave per SIMD: the BG2 Z=36 batch spent
 * ~0.25 us per step whatever Z. Here each check node's edges are dealt over P lanes instead:
 * P = P2 (4 up to Z = 32, else 2) for the rows of a two-row step (each row on its own wave group of WH = ceil(P2 Z / 64)
 * waves), P = 2 P2 for a single-row step (both groups), so a lane handles ceil(degree / P) edges -- one or two edge
 * pairs for most rows -- and the check node's two minima and sign parity are merged across its P lanes by DPP
 * (quad_perm within a quad, row_half_mirror between two quads). The two minima of a multiset and the parity do not
 * depend on the order edges are scanned in, and the reference's tie rule is applied per edge from the merged minima
 * (sp::pass2), so the results are those of the layer-serial decoder bit for bit. A lane's edge k + P j of a row has a
 * per-lane column and shift, so its soft-bit addresses are precomputed once per context (two 16-bit LDS addresses per
 * register, written by ldpc_split_table_kernel) and held in registers with the c2v pairs: one of each per step. */
#ifndef LDPC_SPEC_QUAD
#define LDPC_SPEC_QUAD 1
#endif
constexpr int QUAD_MAX_SLOTS = 64;

struct qrole {
  int row = -1, P = 4, npos = 0; /* npos: positions (edges) per lane, ceil(degree / P) */
};
struct qstep {
  qrole r[2];  /* r[1].row < 0: a single-row step (P = 8, every wave) */
  int   q0 = 0; /* the step's first register slot (address pair and c2v pair) */
  int   nq = 0; /* its slots: ceil(npos / 2) of its larger role */
};
struct qgraph {
  int   P2 = 4;  /* lanes per check node in a two-row step; 2 P2 in a single-row step */
  int   WH = 0, waves = 0, slots = 0, n_steps = 0;
  bool  valid = false;
  qstep steps[MAX_STEPS] = {};
};

/* the register-resident decoder (is_reg) takes precedence */
constexpr bool is_quad(const sgraph& g) { return LDPC_SPEC_QUAD != 0 && g.W == 1 && !is_reg(g); }

constexpr qgraph make_quad(const sgraph& g)
{
  qgraph q{};
  /* four lanes per check node up to Z = 32 and two above (a row group of two waves either way): four lanes at Z = 36
   * put three waves in a group, two of them on one SIMD, and the 128-CB BG2 Z=36 batch took 67.8 us against 60.5 us
   * for the one-lane decoder (profiles/r05/z_sweep_quad_p4.txt) */
  q.P2      = g.Z <= 32 ? 4 : 2;
  q.WH      = (q.P2 * g.Z + 63) / 64;
  q.waves   = 2 * q.WH;
  q.n_steps = g.n_steps;
  int cur   = 0;
  for (int s = 0; s < g.n_steps; ++s) {
    const sstep& st   = g.steps[s];
    qstep&       qs   = q.steps[s];
    const bool   pair = st.r[1].row >= 0;
    int          nq   = 0;
    for (int k = 0; k < (pair ? 2 : 1); ++k) {
      qrole& ro = qs.r[k];
      ro.row    = st.r[k].row;
      ro.P      = pair ? q.P2 : 2 * q.P2;
      ro.npos   = (g.rows[ro.row].deg + ro.P - 1) / ro.P;
      const int np = (ro.npos + 1) / 2;
      nq           = np > nq ? np : nq;
    }
    qs.q0 = cur;
    qs.nq = nq;
    cur += nq;
  }
  q.slots = cur;
  q.valid = g.valid && q.waves <= 16 && cur <= QUAD_MAX_SLOTS && 2 * q.P2 * g.Z <= 64 * q.waves;
  return q;
}

/* The (BG, Z) pairs with a specialised kernel, X(id, bg, Z, ils); ils is the lifting set of Z (TS 38.212 Table
 * 5.3.2-1). The kernel is instantiated per id.
 *  - core (ids 0-9, ldpc_hip_kernels.hip, also bodies of the mixed kernel): BG1 Z = 384 (the BASELINE metric's graph)
 *    and the other large lifting sizes the codeblocks of large transport blocks use, BG1 and BG2 with Z in {384, 352,
 *    320, 288, 256};
 *  - mid (ids 10-41, ldpc_spec_kernels_{a..h}.hip, own launches only): BG1 and BG2 with Z in {240, 224, 208, 192,
 *    176, 160, 144, 128} (C3's BG2 Z = 208 among them) and {120, 112, 104, 96, 88, 80, 72, 64};
 *  - small (ids 42-101, ldpc_spec_kernels_{i..p}.hip, own launches only): every lifting size below 64 (a row is less
 *    than one wave: lanes t >= Z idle, two waves per codeblock).
 * In a mixed launch the mid and small graphs run the generic body. */
#define LDPC_SPEC_GRAPHS_CORE(X)                                                                                       \
  X(0, 1, 384, 1) X(1, 1, 352, 5) X(2, 1, 320, 2) X(3, 1, 288, 4) X(4, 1, 256, 0)                                      \
  X(5, 2, 384, 1) X(6, 2, 352, 5) X(7, 2, 320, 2) X(8, 2, 288, 4) X(9, 2, 256, 0)
#define LDPC_SPEC_GRAPHS_MID_A(X) X(10, 1, 240, 7) X(11, 1, 224, 3) X(12, 1, 208, 6) X(13, 1, 192, 1)
#define LDPC_SPEC_GRAPHS_MID_B(X) X(14, 1, 176, 5) X(15, 1, 160, 2) X(16, 1, 144, 4) X(17, 1, 128, 0)
#define LDPC_SPEC_GRAPHS_MID_C(X) X(18, 2, 240, 7) X(19, 2, 224, 3) X(20, 2, 208, 6) X(21, 2, 192, 1)
#define LDPC_SPEC_GRAPHS_MID_D(X) X(22, 2, 176, 5) X(23, 2, 160, 2) X(24, 2, 144, 4) X(25, 2, 128, 0)
#define LDPC_SPEC_GRAPHS_MID_E(X) X(26, 1, 120, 7) X(27, 1, 112, 3) X(28, 1, 104, 6) X(29, 1, 96, 1)
#define LDPC_SPEC_GRAPHS_MID_F(X) X(30, 1, 88, 5) X(31, 1, 80, 2) X(32, 1, 72, 4) X(33, 1, 64, 0)
#define LDPC_SPEC_GRAPHS_MID_G(X) X(34, 2, 120, 7) X(35, 2, 112, 3) X(36, 2, 104, 6) X(37, 2, 96, 1)
#define LDPC_SPEC_GRAPHS_MID_H(X) X(38, 2, 88, 5) X(39, 2, 80, 2) X(40, 2, 72, 4) X(41, 2, 64, 0)
#define LDPC_SPEC_GRAPHS_SMALL_I(X) X(42, 1, 60, 7) X(43, 1, 56, 3) X(44, 1, 52, 6) X(45, 1, 48, 1) X(46, 1, 44, 5) X(47, 1, 40, 2) X(48, 1, 36, 4) X(49, 1, 32, 0)
#define LDPC_SPEC_GRAPHS_SMALL_J(X) X(50, 1, 30, 7) X(51, 1, 28, 3) X(52, 1, 26, 6) X(53, 1, 24, 1) X(54, 1, 22, 5) X(55, 1, 20, 2) X(56, 1, 18, 4) X(57, 1, 16, 0)
#define LDPC_SPEC_GRAPHS_SMALL_K(X) X(58, 1, 15, 7) X(59, 1, 14, 3) X(60, 1, 13, 6) X(61, 1, 12, 1) X(62, 1, 11, 5) X(63, 1, 10, 2) X(64, 1, 9, 4) X(65, 1, 8, 0)
#define LDPC_SPEC_GRAPHS_SMALL_L(X) X(66, 1, 7, 3) X(67, 1, 6, 1) X(68, 1, 5, 2) X(69, 1, 4, 0) X(70, 1, 3, 1) X(71, 1, 2, 0) X(72, 2, 60, 7) X(73, 2, 56, 3)
#define LDPC_SPEC_GRAPHS_SMALL_M(X) X(74, 2, 52, 6) X(75, 2, 48, 1) X(76, 2, 44, 5) X(77, 2, 40, 2) X(78, 2, 36, 4) X(79, 2, 32, 0) X(80, 2, 30, 7) X(81, 2, 28, 3)
#define LDPC_SPEC_GRAPHS_SMALL_N(X) X(82, 2, 26, 6) X(83, 2, 24, 1) X(84, 2, 22, 5) X(85, 2, 20, 2) X(86, 2, 18, 4) X(87, 2, 16, 0) X(88, 2, 15, 7) X(89, 2, 14, 3)
#define LDPC_SPEC_GRAPHS_SMALL_O(X) X(90, 2, 13, 6) X(91, 2, 12, 1) X(92, 2, 11, 5) X(93, 2, 10, 2) X(94, 2, 9, 4) X(95, 2, 8, 0) X(96, 2, 7, 3) X(97, 2, 6, 1)
#define LDPC_SPEC_GRAPHS_SMALL_P(X) X(98, 2, 5, 2) X(99, 2, 4, 0) X(100, 2, 3, 1) X(101, 2, 2, 0)
#define LDPC_SPEC_GRAPHS(X)                                                                                            \
  LDPC_SPEC_GRAPHS_CORE(X)                                                                                             \
  LDPC_SPEC_GRAPHS_MID_A(X) LDPC_SPEC_GRAPHS_MID_B(X) LDPC_SPEC_GRAPHS_MID_C(X) LDPC_SPEC_GRAPHS_MID_D(X)              \
  LDPC_SPEC_GRAPHS_MID_E(X) LDPC_SPEC_GRAPHS_MID_F(X) LDPC_SPEC_GRAPHS_MID_G(X) LDPC_SPEC_GRAPHS_MID_H(X)              \
  LDPC_SPEC_GRAPHS_SMALL_I(X) LDPC_SPEC_GRAPHS_SMALL_J(X) LDPC_SPEC_GRAPHS_SMALL_K(X) LDPC_SPEC_GRAPHS_SMALL_L(X)      \
  LDPC_SPEC_GRAPHS_SMALL_M(X) LDPC_SPEC_GRAPHS_SMALL_N(X) LDPC_SPEC_GRAPHS_SMALL_O(X) LDPC_SPEC_GRAPHS_SMALL_P(X)
constexpr int NOF_CORE_SPECS = 10; /* ids [0, 10): bodies of the mixed kernel */

/* A translation unit may define LDPC_SPEC_TU_GRAPHS to the list of the graphs it instantiates before including this
 * header: the schedules of the other graphs are then not evaluated (the constexpr evaluation of one schedule costs
 * about a second per compilation pass). Only a unit with the full list has k_specs[] (ldpc_graph.cpp). */
#ifndef LDPC_SPEC_TU_GRAPHS
#define LDPC_SPEC_TU_GRAPHS LDPC_SPEC_GRAPHS
#define LDPC_SPEC_ALL_GRAPHS 1
#endif

#define LDPC_SPEC_DEFINE(id, bg, z, ils)                                                                               \
  constexpr sgraph k_spec##id = make(bg, z, ils);                                                                      \
  static_assert(k_spec##id.valid && schedule_is_layer_serial(k_spec##id) && roles_cover_edges(k_spec##id) &&         \
                    early_roles_match(k_spec##id),                                                                     \
                "specialised schedule " #id);                                                                          \
  constexpr qgraph k_quad##id = make_quad(k_spec##id);                                                                 \
  static_assert(!is_quad(k_spec##id) || k_quad##id.valid, "lane-split schedule " #id);                              \
  constexpr rgraph k_reg##id = make_reg(k_spec##id);                                                                   \
  static_assert(!is_reg(k_spec##id) || k_reg##id.valid, "register-resident schedule " #id);
LDPC_SPEC_TU_GRAPHS(LDPC_SPEC_DEFINE)
#undef LDPC_SPEC_DEFINE

#define LDPC_SPEC_COUNT(id, bg, z, ils) +1
constexpr int NOF_SPECS = 0 LDPC_SPEC_GRAPHS(LDPC_SPEC_COUNT);
#undef LDPC_SPEC_COUNT

#ifdef LDPC_SPEC_ALL_GRAPHS
#define LDPC_SPEC_PTR(id, bg, z, ils) &k_spec##id,
constexpr const sgraph* k_specs[] = {LDPC_SPEC_GRAPHS(LDPC_SPEC_PTR)};
#undef LDPC_SPEC_PTR
#define LDPC_QUAD_PTR(id, bg, z, ils) &k_quad##id,
constexpr const qgraph* k_quads[] = {LDPC_SPEC_GRAPHS(LDPC_QUAD_PTR)};
#undef LDPC_QUAD_PTR
static_assert(sizeof(k_specs) / sizeof(k_specs[0]) == NOF_SPECS, "specialised graph list");
static_assert(k_spec0.bg == 1 && k_spec0.Z == 384 && k_spec0.n_steps == 32, "BG1 Z=384 schedule");
#endif

/* spec_graph<id>::g: the compile-time graph of a specialised kernel instantiation */
template <int I>
struct spec_graph;
#define LDPC_SPEC_SEL(id, bg, z, ils)                                                                                  \
  template <>                                                                                                          \
  struct spec_graph<id> {                                                                                              \
    static constexpr const sgraph& g = k_spec##id;                                                                     \
    static constexpr const qgraph& q = k_quad##id;                                                                     \
    static constexpr const rgraph& r = k_reg##id;                                                                      \
  };
LDPC_SPEC_TU_GRAPHS(LDPC_SPEC_SEL)
#undef LDPC_SPEC_SEL

} // namespace spec
} // namespace ldpc_hip
