/* Compile-time step schedules for the specialised decoder (ldpc_decode_kernel<SF08, true>).
 *
 * The generic kernel reads every step's work from a task table and every edge's (column, shift) from an LDS edge
 * table at run time. For the lifting sizes that carry the throughput (BG1 Z = 384, the BASELINE metric) the same
 * schedule is built here as a constexpr object from the same base-graph table (ldpc_base_graphs.inc) with the same
 * rules as build_graph / build_tasks (ldpc_graph.cpp): consecutive rows with pairwise-disjoint column sets form one
 * step; a single-row step of degree >= split_min_degree() splits each check node's edges over a lane pair. The kernel
 * then unrolls the whole iteration, with columns, shifts and c2v offsets as instruction immediates.
 * spec_matches() (ldpc_graph.cpp) compares this schedule with build_graph's before the specialised kernel is used. */
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

struct srow {
  int deg = 0;
  int e0  = 0; /* first edge of the row in row-major edge order (c2v offset e0 * Z) */
  int col[MAX_DEG] = {};
  int sh[MAX_DEG]  = {}; /* shift mod Z */
};

/* One step: up to two rows; p = 2 when the (single) row's edges are split over lane pairs. */
struct sstep {
  int ra = -1, rb = -1, p = 1;
};

struct sgraph {
  int   bg = 0, Z = 0, M = 0, N_full = 0, n_steps = 0;
  bool  valid = false; /* every step fits the kernel's wave mapping (see make) */
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

/* ils: lifting-set index of Z (TS 38.212 Table 5.3.2-1). The wave mapping needs Z = 6 * 64 (six 64-check-node chunks
 * per row, twelve waves for two rows or for one split row). */
constexpr sgraph make(int bg, int Z, int ils, int split_min_degree)
{
  sgraph g{};
  g.bg     = bg;
  g.Z      = Z;
  g.M      = (bg == 1) ? 46 : 42;
  g.N_full = (bg == 1) ? 68 : 52;
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
  bool ok = (Z == 384);
  int  m  = 0;
  while (m < g.M) {
    int nr = 1;
    while (m + nr < g.M) {
      bool clash = false;
      for (int q = m; q < m + nr; ++q) {
        clash = clash || rows_share_column(g.rows[q], g.rows[m + nr]);
      }
      if (clash) {
        break;
      }
      ++nr;
    }
    sstep st{};
    st.ra = m;
    st.rb = (nr >= 2) ? m + 1 : -1;
    st.p  = (nr == 1 && g.rows[m].deg >= split_min_degree) ? 2 : 1;
    ok    = ok && nr <= 2 && g.n_steps < MAX_STEPS && (st.p == 1 || (g.rows[m].deg + 1) / 2 <= 10) &&
         (st.p == 2 || g.rows[m].deg <= 10);
    if (g.n_steps < MAX_STEPS) {
      g.steps[g.n_steps++] = st;
    }
    m += nr;
  }
  g.valid = ok;
  return g;
}

/* Does edge k of row r (its column) belong to one of the rows a, b (-1 = none)? */
constexpr bool edge_in_rows(const sgraph& g, int r, int k, int a, int b)
{
  const int c = g.rows[r].col[k];
  for (int q : {a, b}) {
    if (q >= 0) {
      for (int j = 0; j < g.rows[q].deg; ++j) {
        if (g.rows[q].col[j] == c) {
          return true;
        }
      }
    }
  }
  return false;
}

/* Soft-bit copies per column in the specialised kernel's LDS: 4 (column stride 4Z, no modulo in any address, three
 * stores per update) or 1 (stride Z, (t + shift) mod Z computed per edge, one store). */
#ifndef LDPC_SPEC_COPIES
#define LDPC_SPEC_COPIES 4
#endif
constexpr int k_spec_copies = LDPC_SPEC_COPIES;
static_assert(k_spec_copies == 1 || k_spec_copies == 4, "LDPC_SPEC_COPIES is 1 or 4");

/* BG1, Z = 384 (iLS 1), split threshold 6 (split_min_degree()'s default): the C2 configuration. */
#ifndef LDPC_SPEC_SPLIT_MIN_DEGREE
#define LDPC_SPEC_SPLIT_MIN_DEGREE 6
#endif
constexpr sgraph k_bg1_z384 = make(1, 384, 1, LDPC_SPEC_SPLIT_MIN_DEGREE);
static_assert(k_bg1_z384.valid && k_bg1_z384.n_steps == 32, "BG1 Z=384 schedule");

} // namespace spec
} // namespace ldpc_hip
