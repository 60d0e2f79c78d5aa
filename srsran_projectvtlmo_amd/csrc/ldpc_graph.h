/*
 * Host-side construction of the lifted LDPC graph schedules and CRC tables consumed by the gfx950 kernels.
 *
 * Graph: TS 38.212 Tables 5.3.2-2/-3 (ldpc_base_graphs.inc); lifting-set index per Table 5.3.2-1; shift values
 * reduced modulo Z as ldpc_luts_impl.cpp:4521-4544 (get_graph) does. Rows are kept in the reference's adjacency order
 * (ldpc_luts_impl.cpp:4383/4477: ascending column), which fixes the edge index k used by the min-index tie-break.
 */
#pragma once

#include <cstdint>
#include <vector>

#include "ldpc_hip_device.h"

namespace ldpc_hip {

/* Valid 5G-NR lifting sizes (TS 38.212 Table 5.3.2-1), ascending. */
extern const uint16_t k_lifting_sizes[51];

int lifting_position(unsigned Z); /* index in k_lifting_sizes, or -1 */
/* Edges of base-graph rows [0, nof_layers) (the first nof_layers layers a codeblock decodes) */
uint32_t layer_edges(int bg, unsigned nof_layers);
int lifting_index(unsigned Z);    /* iLS 0..7, or -1                 */

/* Builds the graph for (bg, Z); returns false for an invalid pair. */
bool build_graph(int bg, unsigned Z, graph_desc& g);

/* LDS layout of one decoder workgroup for graph g. */
lds_layout make_lds_layout(const graph_desc& g, bool spec = false);

/* Threads per decoder workgroup for graph g (64 * g.task_waves, after build_tasks). */
int decoder_block_size(const graph_desc& g);

/* Per-(step, wave) task records of graph g, appended to `tasks`; sets g.n_steps, g.task_waves, g.task_offset and
 * g.step_row0. Row groups wider than max_waves waves are issued as several consecutive steps (check nodes of one
 * row, and rows of one group, are independent). max_waves = 16 gives the widest steps (lowest latency per CB);
 * NARROW_WAVES the "narrow" schedule whose workgroups fit twice per CU (throughput at large batches). */
void build_tasks(graph_desc& g, std::vector<step_task>& tasks, int max_waves = 16);

/* Graph slots: [0, 102) wide schedules; NARROW_SLOT_BASE + slot the narrow schedule of the same (BG, Z). */
constexpr int NARROW_SLOT_BASE = 102;
constexpr int NARROW_WAVES     = 8;
constexpr int NOF_GRAPH_SLOTS  = 2 * NARROW_SLOT_BASE;

/* CRC tables: for poly id p in {CRC16, CRC24B, CRC24A} (hw_dec_cb_crc_type numbering), CRC_TABLE_SIZE words at
 * p * CRC_TABLE_SIZE: [0,256) byte table (b(x) x^r mod G), [256, 256 + CRC_POW_WORDS) x^(32 e) mod G. */
std::vector<uint32_t> build_crc_tables();

namespace spec {
struct sgraph;
}
/* True when a specialised decoder's compile-time graph (ldpc_spec.h) is exactly build_graph's g. */
bool spec_matches(const graph_desc& g, const lds_layout& lay, const spec::sgraph& k);
/* The specialised kernel id (spec::k_specs index) for g, or -1; and that kernel's waves per workgroup. */
int spec_index(const graph_desc& g, const lds_layout& lay);
int spec_waves(int id);
/* One-wave graphs run the lane-split decoder (ldpc_spec.h qgraph): the word offset of specialised graph id's address
 * table in the context's table buffer, or -1 for other graphs; and the end of the last table (the buffer's size). */
long quad_table_offset(int id);
long quad_tables_end();
/* Specialised kernels [0, spec_core_count()) are also bodies of the mixed kernel; the others run standalone only. */
int spec_core_count();
/* The translation unit holding specialised kernel `id` (and its work-queue body): 0 core, 1..16 units a..p. */
int spec_unit(int id);
constexpr int NOF_SPEC_UNITS = 17;

} // namespace ldpc_hip
