#include "ldpc_graph.h"
#include "ldpc_spec.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace ldpc_hip {

namespace {

struct base_edge {
  uint8_t  bg, row, col;
  uint16_t shift[8];
};

const base_edge k_base_edges[] = {
#define LDPC_EDGE(bg, r, c, s0, s1, s2, s3, s4, s5, s6, s7) {bg, r, c, {s0, s1, s2, s3, s4, s5, s6, s7}},
#include "ldpc_base_graphs.inc"
#undef LDPC_EDGE
};

uint32_t align16(uint32_t x) { return (x + 15U) & ~15U; }

/* A single-row step splits each check node's edges over two lanes when the row degree reaches this value (timed in
 * round 1: thresholds 7-11 were 1-3% slower on C2). The specialised schedules have their own (ldpc_spec.h). */
#ifndef LDPC_SPEC_SPLIT_MIN_DEGREE
#define LDPC_SPEC_SPLIT_MIN_DEGREE 6
#endif
constexpr unsigned split_min_degree() { return LDPC_SPEC_SPLIT_MIN_DEGREE; }

} // namespace

const uint16_t k_lifting_sizes[51] = {2,   3,   4,   5,   6,   7,   8,   9,   10,  11,  12,  13,  14,
                                      15,  16,  18,  20,  22,  24,  26,  28,  30,  32,  36,  40,  44,
                                      48,  52,  56,  60,  64,  72,  80,  88,  96,  104, 112, 120, 128,
                                      144, 160, 176, 192, 208, 224, 240, 256, 288, 320, 352, 384};

uint32_t layer_edges(int bg, unsigned nof_layers)
{
  /* cumulative row degrees of both base graphs, counted once from the edge table */
  static const auto cum = [] {
    std::vector<uint32_t> c(2 * 47, 0);
    for (const base_edge& e : k_base_edges) {
      for (unsigned r = e.row + 1U; r <= 46U; ++r) {
        ++c[(e.bg - 1U) * 47U + r];
      }
    }
    return c;
  }();
  if (bg != 1 && bg != 2) {
    return 0;
  }
  const unsigned M = bg == 1 ? 46U : 42U;
  return cum[static_cast<unsigned>(bg - 1) * 47U + std::min(nof_layers, M)];
}

int lifting_position(unsigned Z)
{
  for (int i = 0; i != 51; ++i) {
    if (k_lifting_sizes[i] == Z) {
      return i;
    }
  }
  return -1;
}

int lifting_index(unsigned Z)
{
  static const unsigned a_set[8] = {2, 3, 5, 7, 9, 11, 13, 15};
  if (lifting_position(Z) < 0) {
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

bool build_graph(int bg, unsigned Z, graph_desc& g)
{
  const int ils = lifting_index(Z);
  if (ils < 0 || (bg != 1 && bg != 2)) {
    return false;
  }
  g          = graph_desc{};
  g.bg       = static_cast<uint8_t>(bg);
  g.Z        = static_cast<uint16_t>(Z);
  g.M        = (bg == 1) ? 46 : 42;
  g.N_full   = (bg == 1) ? 68 : 52;
  g.K        = static_cast<uint16_t>(g.N_full - g.M);
  g.maxdeg   = 0;
  g.ils      = static_cast<uint8_t>(ils);
  unsigned e = 0;
  std::vector<std::vector<uint16_t>> row_cols(g.M);
  for (unsigned m = 0; m != g.M; ++m) {
    const unsigned e0 = e;
    for (const base_edge& be : k_base_edges) {
      if (be.bg == bg && be.row == m) {
        g.edges[e++] = static_cast<uint32_t>(be.col) * Z | (static_cast<uint32_t>(be.shift[ils] % Z) << 16);
        row_cols[m].push_back(be.col);
      }
    }
    const unsigned deg = e - e0;
    g.rows[m]          = e0 | (deg << 16);
    g.maxdeg           = std::max<uint8_t>(g.maxdeg, static_cast<uint8_t>(deg));
  }
  g.n_edges = static_cast<uint16_t>(e);
  /* per-edge int8 c2v, edge-major with stride Z (ldpc_hip_kernels.hip "Check-to-variable storage") */
  for (unsigned m = 0; m != g.M; ++m) {
    g.c2v_off[m] = (g.rows[m] & 0xffffU) * Z;
  }
  g.c2v_bytes = static_cast<uint32_t>(e) * Z;

  /* Greedy grouping of consecutive rows with pairwise-disjoint column sets: updating them concurrently reads and
   * writes disjoint soft bits, hence equals the layer-serial schedule of ldpc_decoder_impl.cpp:116-123. */
  unsigned ng = 0, maxg = 0;
  unsigned m  = 0;
  while (m < g.M) {
    std::vector<uint16_t> used(row_cols[m]);
    unsigned              nr = 1;
    while (m + nr < g.M) {
      bool clash = false;
      for (uint16_t c : row_cols[m + nr]) {
        if (std::find(used.begin(), used.end(), c) != used.end()) {
          clash = true;
          break;
        }
      }
      if (clash) {
        break;
      }
      used.insert(used.end(), row_cols[m + nr].begin(), row_cols[m + nr].end());
      ++nr;
    }
    /* a single-row step splits each check node's edges over two lanes to keep every SIMD busy */
    const unsigned deg   = g.rows[m] >> 16;
    const bool     split = (nr == 1) && deg >= split_min_degree();
    g.groups[ng++]       = m | (nr << 8) | ((split ? 2U : 1U) << 16);
    maxg           = std::max(maxg, nr);
    m += nr;
  }
  g.n_groups       = static_cast<uint16_t>(ng);
  g.max_group_rows = static_cast<uint16_t>(maxg);
  std::vector<step_task> unused;
  build_tasks(g, unused); /* step counts and block size; the context keeps the records themselves */
  g.task_offset = 0;
  return true;
}

lds_layout make_lds_layout(const graph_desc& g, bool spec)
{
  lds_layout l{};
  uint32_t   off = 0;
  l.soft         = off; /* must stay 0: the decode kernel addresses soft bits from the LDS base */
  if (spec) {
    /* specialised kernel: spec::SOFT_COPIES copies per column, c2v in registers (ldpc_hip_kernels.hip, namespace sp) */
    l.soft_stride = static_cast<uint32_t>(spec::SOFT_COPIES * spec::SOFT_BYTES) * g.Z; /* bytes per column */
    l.soft_read   = spec::SOFT_COPIES == 1 ? 0U : g.Z;
    off += align16(static_cast<uint32_t>(g.N_full + 1) * l.soft_stride + 64); /* + one column of dummy-edge scratch */
    l.c2v = off; /* c2v lives in registers; the region holds the split rows' address table (BG1 rows 0-3) */
    int  qid = -1; /* a one-wave graph: the lane-split decoder, its address table in global memory (registers) */
    bool reg = false; /* ... or the register-resident decoder: no table */
    for (int i = 0; i != spec::NOF_SPECS; ++i) {
      if (spec::k_specs[i]->bg == g.bg && spec::k_specs[i]->Z == g.Z) {
        qid = spec::is_quad(*spec::k_specs[i]) ? i : -1;
        reg = spec::is_reg(*spec::k_specs[i]);
      }
    }
    if (reg) {
      l.split_tab = 0;
    } else if (qid >= 0) {
      l.split_tab = static_cast<uint32_t>(quad_table_offset(qid));
    } else if (g.bg == 1) {
      const uint32_t waves = std::max<uint32_t>(2U * ((g.Z + 63U) / 64U), (g.Z + 31U) / 32U);
      off += align16(static_cast<uint32_t>(spec::SPLIT_LDS_PAIRS) * waves * 64U * 4U);
      l.split_tab = static_cast<uint32_t>(SPLIT_TAB_OFFSET + lifting_position(g.Z) * SPLIT_TAB_STRIDE);
    }
  } else {
    l.soft_stride = g.Z;
    l.soft_read   = 0;
    off += align16(static_cast<uint32_t>(g.N_full) * g.Z + g.Z + 64); /* + scratch for dummy-edge stores */
    l.c2v = off;
    off += align16(g.c2v_bytes);
  }
  l.hard = off;
  off += align16((static_cast<uint32_t>(g.K) * g.Z + 7) / 8 + 16);
  l.red = off;
  off += 128;
  l.crct = off;
  off += align16(static_cast<uint32_t>(CRC_LDS_WORDS) * 4U);
  l.edges = off;
  off += static_cast<uint32_t>(g.M) * EDGE_SLOT * 4U;
  l.total = off;
  return l;
}

int decoder_block_size(const graph_desc& g) { return 64 * static_cast<int>(g.task_waves); }

void build_tasks(graph_desc& g, std::vector<step_task>& tasks, int max_waves)
{
  struct chunk {
    unsigned row, t0, split;
  };
  /* chunks of every row group: 64 check nodes per wave, or 32 when the edges are split */
  std::vector<std::vector<chunk>> steps;
  std::vector<unsigned>           row0;
  for (unsigned i = 0; i != g.n_groups; ++i) {
    const unsigned r0    = g.groups[i] & 0xffU;
    const unsigned nr    = (g.groups[i] >> 8) & 0xffU;
    const unsigned gsplit = ((g.groups[i] >> 16) & 0xffU) == 2U ? 1U : 0U;
    std::vector<chunk> all;
    for (unsigned r = r0; r != r0 + nr; ++r) {
      const unsigned split = gsplit;
      const unsigned per   = split ? 32U : 64U;
      for (unsigned t0 = 0; t0 < g.Z; t0 += per) {
        all.push_back({r, t0, split});
      }
    }
    /* rows of a group are independent, so a group wider than the workgroup runs as consecutive steps */
    for (size_t b = 0; b < all.size(); b += max_waves) {
      const size_t e = std::min(all.size(), b + max_waves);
      steps.emplace_back(all.begin() + static_cast<long>(b), all.begin() + static_cast<long>(e));
      row0.push_back(all[b].row);
    }
  }
  size_t waves = 4;
  for (const auto& st : steps) {
    waves = std::max(waves, st.size());
  }
  g.n_steps     = static_cast<uint16_t>(steps.size());
  g.task_waves  = static_cast<uint16_t>(waves);
  g.task_offset = static_cast<uint32_t>(tasks.size());
  for (size_t s = 0; s != steps.size(); ++s) {
    g.step_row0[s] = static_cast<uint8_t>(row0[s]);
    for (size_t w = 0; w != waves; ++w) {
      step_task tk{};
      if (w < steps[s].size()) {
        const chunk&   c   = steps[s][w];
        const unsigned e0  = g.rows[c.row] & 0xffffU;
        const unsigned deg = g.rows[c.row] >> 16;
        tk.w[0]            = deg | (c.split << 5) | (1U << 6) | (c.row << 8) | (c.t0 << 16);
        tk.w[1]            = g.c2v_off[c.row];
        tk.w[2]            = make_lds_layout(g).edges + c.row * EDGE_SLOT * 4U;
        (void)e0;
      }
      tasks.push_back(tk);
    }
  }
}

/* Is the specialised kernel's compile-time graph (ldpc_spec.h) the graph build_graph made for g: same (BG, Z), and
 * every row with the same edges (columns and shifts mod Z) in the same order? Its step schedule is its own (checked
 * layer-serial at compile time, spec::schedule_is_layer_serial). */
int spec_index(const graph_desc& g, const lds_layout& lay)
{
  for (int i = 0; i != spec::NOF_SPECS; ++i) {
    if (spec::k_specs[i]->bg == g.bg && spec::k_specs[i]->Z == g.Z) {
      return spec_matches(g, lay, *spec::k_specs[i]) ? i : -1;
    }
  }
  return -1;
}

int spec_waves(int id)
{
  if (id < 0 || id >= spec::NOF_SPECS) {
    return 0;
  }
  if (spec::is_reg(*spec::k_specs[id])) {
    return 1; /* the register-resident decoder: one wave per codeblock */
  }
  return spec::is_quad(*spec::k_specs[id]) ? spec::k_quads[id]->waves : spec::k_specs[id]->waves;
}

namespace {
const std::vector<long>& quad_offsets()
{
  static const std::vector<long> o = [] {
    std::vector<long> v(spec::NOF_SPECS + 1, -1);
    long              cur = QUAD_TAB_OFFSET;
    for (int id = 0; id != spec::NOF_SPECS; ++id) {
      if (spec::is_quad(*spec::k_specs[id])) {
        v[id] = cur;
        cur += static_cast<long>(spec::k_quads[id]->slots) * spec::k_quads[id]->waves * 64;
        cur = (cur + 3) / 4 * 4;
      }
    }
    v[spec::NOF_SPECS] = cur;
    return v;
  }();
  return o;
}
} // namespace

long quad_table_offset(int id) { return (id >= 0 && id < spec::NOF_SPECS) ? quad_offsets()[id] : -1; }
long quad_tables_end() { return quad_offsets()[spec::NOF_SPECS]; }

int spec_core_count() { return spec::NOF_CORE_SPECS; }

int spec_unit(int id)
{
  /* unit of each graph list: 0 core (ldpc_hip_kernels.hip), 1 + u for ldpc_spec_kernels_<'a' + u>.hip */
  static const int units[] = {
#define X0(id, bg, z, ils) 0,
#define XA(id, bg, z, ils) 1,
#define XB(id, bg, z, ils) 2,
#define XC(id, bg, z, ils) 3,
#define XD(id, bg, z, ils) 4,
#define XE(id, bg, z, ils) 5,
#define XF(id, bg, z, ils) 6,
#define XG(id, bg, z, ils) 7,
#define XH(id, bg, z, ils) 8,
#define XI(id, bg, z, ils) 9,
#define XJ(id, bg, z, ils) 10,
#define XK(id, bg, z, ils) 11,
#define XL(id, bg, z, ils) 12,
#define XM(id, bg, z, ils) 13,
#define XN(id, bg, z, ils) 14,
#define XO(id, bg, z, ils) 15,
#define XP(id, bg, z, ils) 16,
      LDPC_SPEC_GRAPHS_CORE(X0) LDPC_SPEC_GRAPHS_MID_A(XA) LDPC_SPEC_GRAPHS_MID_B(XB) LDPC_SPEC_GRAPHS_MID_C(XC)
          LDPC_SPEC_GRAPHS_MID_D(XD) LDPC_SPEC_GRAPHS_MID_E(XE) LDPC_SPEC_GRAPHS_MID_F(XF) LDPC_SPEC_GRAPHS_MID_G(XG)
              LDPC_SPEC_GRAPHS_MID_H(XH) LDPC_SPEC_GRAPHS_SMALL_I(XI) LDPC_SPEC_GRAPHS_SMALL_J(XJ)
                  LDPC_SPEC_GRAPHS_SMALL_K(XK) LDPC_SPEC_GRAPHS_SMALL_L(XL) LDPC_SPEC_GRAPHS_SMALL_M(XM)
                      LDPC_SPEC_GRAPHS_SMALL_N(XN) LDPC_SPEC_GRAPHS_SMALL_O(XO) LDPC_SPEC_GRAPHS_SMALL_P(XP)};
#undef X0
#undef XA
#undef XB
#undef XC
#undef XD
#undef XE
#undef XF
#undef XG
#undef XH
#undef XI
#undef XJ
#undef XK
#undef XL
#undef XM
#undef XN
#undef XO
#undef XP
  static_assert(sizeof(units) / sizeof(units[0]) == spec::NOF_SPECS, "unit table");
  return (id >= 0 && id < spec::NOF_SPECS) ? units[id] : -1;
}

bool spec_matches(const graph_desc& g, const lds_layout& lay, const spec::sgraph& k)
{
  if (g.bg != k.bg || g.Z != k.Z || g.M != k.M || g.N_full != k.N_full || lay.soft != 0 ||
      lay.soft_stride != static_cast<uint32_t>(spec::SOFT_COPIES * spec::SOFT_BYTES) * g.Z) {
    return false;
  }
  for (int m = 0; m < k.M; ++m) {
    const uint32_t rw = g.rows[m];
    if (static_cast<int>(rw >> 16) != k.rows[m].deg || static_cast<int>(rw & 0xffffU) != k.rows[m].e0) {
      return false;
    }
    for (int e = 0; e < k.rows[m].deg; ++e) {
      const uint32_t ew = g.edges[k.rows[m].e0 + e];
      if (static_cast<int>(ew & 0xffffU) != k.rows[m].col[e] * k.Z || static_cast<int>(ew >> 16) != k.rows[m].sh[e]) {
        return false;
      }
    }
  }
  return true;
}

std::vector<uint32_t> build_crc_tables()
{
  /* split and lane-split address tables: filled on the device; demod tables: by the context */
  std::vector<uint32_t> t(static_cast<size_t>(quad_tables_end()), 0);
  static_assert(CRC_XPOW_OFFSET >= DTAB_OFFSET + DTAB_WORDS + 1024 * 8 * 2 &&
                    QUAD_TAB_OFFSET >= CRC_XPOW_OFFSET + 3 * CRC_XPOW_WORDS,
                "table buffer regions");
  for (int p = 0; p != 3; ++p) {
    unsigned order = (p == LDPC_HIP_CRC16) ? 16 : 24;
    uint64_t poly  = (p == LDPC_HIP_CRC16) ? 0x11021ULL : (p == LDPC_HIP_CRC24B) ? 0x1800063ULL : 0x1864cfbULL;
    uint64_t hi    = 1ULL << order;
    uint32_t* tab  = t.data() + p * CRC_TABLE_SIZE;
    for (unsigned b = 0; b != 256; ++b) {
      /* (b(x) * x^order) mod G by bitwise long division, b MSB first */
      uint64_t rem = 0;
      for (int i = 7; i >= 0; --i) {
        rem = (rem << 1) | ((b >> i) & 1U);
        if (rem & hi) {
          rem ^= poly;
        }
      }
      for (unsigned i = 0; i != order; ++i) {
        rem <<= 1;
        if (rem & hi) {
          rem ^= poly;
        }
      }
      tab[b] = static_cast<uint32_t>(rem);
    }
    /* slicing-by-4: T_k[b] = T_0[b] x^(8k) mod G, k = 1..3 (eight zero bits through the byte table per k) */
    const uint32_t mask = (1U << order) - 1U;
    for (int k = 1; k != 4; ++k) {
      uint32_t*       tk   = t.data() + CRC_SLICE_OFFSET + p * CRC_SLICE_WORDS + (k - 1) * 256;
      const uint32_t* prev = (k == 1) ? tab : tk - 256;
      for (unsigned b = 0; b != 256; ++b) {
        const uint32_t c = prev[b];
        tk[b]            = ((c << 8) ^ tab[(c >> (order - 8)) & 0xffU]) & mask;
      }
    }
    /* x^(32 e + i) mod G, i < order: the columns of multiplication by x^(32 e) */
    {
      uint64_t y = 1;
      for (int e = 0; e != CRC_POW_WORDS; ++e) {
        uint64_t z = y;
        for (unsigned i = 0; i != order; ++i) {
          t[CRC_MCOL_OFFSET + (p * CRC_POW_WORDS + e) * 24 + i] = static_cast<uint32_t>(z);
          z <<= 1;
          if (z & hi) {
            z ^= poly;
          }
        }
        for (int i = 0; i != 32; ++i) {
          y <<= 1;
          if (y & hi) {
            y ^= poly;
          }
        }
      }
    }
    /* x^k mod G, k < CRC_XPOW_WORDS */
    {
      uint64_t z = 1;
      for (int k = 0; k != CRC_XPOW_WORDS; ++k) {
        t[CRC_XPOW_OFFSET + p * CRC_XPOW_WORDS + k] = static_cast<uint32_t>(z);
        z <<= 1;
        if (z & hi) {
          z ^= poly;
        }
      }
    }
    /* x^(32 e) mod G */
    uint64_t x = 1;
    for (int e = 0; e != CRC_POW_WORDS; ++e) {
      tab[256 + e] = static_cast<uint32_t>(x);
      for (int i = 0; i != 32; ++i) {
        x <<= 1;
        if (x & hi) {
          x ^= poly;
        }
      }
    }
    if (p == LDPC_HIP_CRC24A) { /* TB-join combination powers (ldpc_hip_device.h TBJ_*) */
      uint32_t* pw = t.data() + TBJ_POW_OFFSET;
      uint64_t  y  = 1;
      for (int k = 0; k != TBJ_THREADS * TBJ_MAX_CHUNKS; ++k) {
        if (k < TBJ_THREADS) {
          pw[k] = static_cast<uint32_t>(y); /* x^(8 * 16 * k) */
        }
        if (k % TBJ_THREADS == 0) {
          pw[TBJ_THREADS + k / TBJ_THREADS] = static_cast<uint32_t>(y); /* x^(8 * 4096 * k / 256) */
        }
        for (int i = 0; i != 8 * TBJ_BYTES; ++i) {
          y <<= 1;
          if (y & hi) {
            y ^= poly;
          }
        }
      }
    }
  }
  return t;
}

} // namespace ldpc_hip
