/*
 * Device-side data layouts shared by the host runtime (ldpc_hip_api.cpp) and the gfx950 kernels
 * (ldpc_hip_kernels.hip). Plain structs only; the C ABI in include/srsran_ldpc_hip.h never exposes them.
 */
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

#include "srsran_ldpc_hip.h"

namespace ldpc_hip {

constexpr int MAX_Z          = 384;
constexpr int MAX_EDGES      = 316; /* BG1 base-graph edges (ldpc_luts_impl.cpp:4383) */
constexpr int MAX_ROWS       = 46;  /* BG1_M */
constexpr int BG1_MAXDEG     = 19;  /* BG1 rows 0..3 */
constexpr int BG2_MAXDEG     = 10;  /* BG2 rows 1, 3 */
constexpr int CRC_POW_WORDS  = 272; /* x^(32e) mod G for e < 272 (8448 bits = 264 words) */
constexpr int CRC_TABLE_SIZE = 256 + CRC_POW_WORDS;
/* Transport-block join (ldpc_tb_join_kernel): 16 TB bytes per thread, 256 threads = one 4 KiB chunk per workgroup,
 * up to 64 chunks per TB (max TBS 1,277,992 bits = 39 chunks). Appended to the CRC tables (build_crc_tables):
 * x^(8*16*j) mod G_24A for j < 256, then x^(8*4096*k) mod G_24A for k < 64. */
constexpr int TBJ_BYTES      = 16;
constexpr int TBJ_THREADS    = 256;
constexpr int TBJ_CHUNK      = TBJ_BYTES * TBJ_THREADS;
constexpr int TBJ_MAX_CHUNKS = 64;
constexpr int TBJ_POW_OFFSET = 3 * CRC_TABLE_SIZE;
constexpr int TBJ_WORK_WORDS = TBJ_MAX_CHUNKS + 1; /* per TB: chunk CRCs, then the arrival counter */
/* Slicing-by-4 byte tables for the decoder's early-stop CRC, after the TB-join powers: for poly id p, three tables of
 * 256 words at CRC_SLICE_OFFSET + p * 768, T_k[b] = b(x) x^(8k + r) mod G for k = 1, 2, 3 (T_0 is the byte table). */
constexpr int CRC_SLICE_OFFSET = TBJ_POW_OFFSET + TBJ_THREADS + TBJ_MAX_CHUNKS;
constexpr int CRC_SLICE_WORDS  = 3 * 256;
/* Multiplication by x^(32 e) mod G as 24 columns: for poly id p and e < CRC_POW_WORDS, words
 * CRC_MCOL_OFFSET + (p * CRC_POW_WORDS + e) * 24 + i = x^(32 e + i) mod G (i < order): a CRC word c times x^(32 e) is
 * the XOR of the columns of c's set bits (independent operations instead of a 24-step dependent Horner chain). */
constexpr int CRC_MCOL_OFFSET = CRC_SLICE_OFFSET + 3 * CRC_SLICE_WORDS;
constexpr int CRC_MCOL_WORDS  = 24 * CRC_POW_WORDS;
/* The decoder's LDS copy for one poly: T_0..T_3 (1024 words), then x^(32 e) mod G for e < CRC_POW_WORDS. */
constexpr int CRC_LDS_WORDS = 4 * 256 + CRC_POW_WORDS;
/* BG1's split-row address tables (the specialised decoder's LDS table, ldpc_decode_body.h dec::fill_split), one per
 * BG1 lifting size p at SPLIT_TAB_OFFSET + p * SPLIT_TAB_STRIDE words: pair k of lane tid at word k * (waves * 64) + tid.
 * Written once per context by ldpc_split_table_kernel, copied into LDS by each codeblock's prologue. */
constexpr int SPLIT_TAB_OFFSET = (CRC_MCOL_OFFSET + 3 * CRC_MCOL_WORDS + 3) / 4 * 4;
constexpr int SPLIT_TAB_STRIDE = 20 * 768; /* 20 pairs (rows 0-3, 5 each) x up to 12 waves of 64 lanes */
constexpr int SPLIT_TAB_WORDS  = 51 * SPLIT_TAB_STRIDE;
/* The demodulation tables (demod_tables, below) for the decode kernels' fused dematcher, after the split tables. */
constexpr int DTAB_OFFSET = SPLIT_TAB_OFFSET + SPLIT_TAB_WORDS;
constexpr int DTAB_WORDS  = 192; /* >= sizeof(demod_tables) / 4, static_assert in ldpc_graph.cpp */
#ifdef LDPC_HIP_DIAG_CB /* diagnostic build: per-workgroup decoder phase stamps (8 uint64 per workgroup) after them */
constexpr int DIAG_CB_OFFSET = DTAB_OFFSET + DTAB_WORDS;
constexpr int DIAG_CB_WORDS  = 1024 * 8 * 2;
#endif
/* The one-wave graphs' lane-split address tables (ldpc_spec.h qgraph, ldpc_decode_body.h sp::qdec), after the
 * diagnostic region: graph by graph at the offsets ldpc_graph.cpp quad_table_offset gives, slot q of lane tid at word
 * q * (waves * 64) + tid. Written once per context by ldpc_split_table_kernel, held in registers by each codeblock. */
/* x^k mod G for k < CRC_XPOW_WORDS, per poly id p at CRC_XPOW_OFFSET + p * CRC_XPOW_WORDS: the register-resident
 * decoder's early-stop CRC (sp::rdec::et_setup), bit i of an L-bit message contributing x^(L - 1 - i + order) mod G;
 * K Z + order <= 22 * 64 + 24 for its graphs (Z <= 64). */
constexpr int CRC_XPOW_OFFSET = DTAB_OFFSET + DTAB_WORDS + 1024 * 8 * 2;
constexpr int CRC_XPOW_WORDS  = 1536;
constexpr int QUAD_TAB_OFFSET = CRC_XPOW_OFFSET + 3 * CRC_XPOW_WORDS;
/* One TB-join workgroup's record: its TB's descriptor, the TB's index (result slot, work words) and its chunk, so that
 * the workgroup starts with one load instead of a table lookup followed by a descriptor load. */
struct tbj_block {
  ldpc_hip_tb_desc d;
  uint32_t         tb;
  uint32_t         chunk;
};
constexpr int MAX_STEPS      = 64;  /* decoder steps per iteration (BG1: 32, BG2: 28, more after splitting) */
constexpr int TASK_DWORDS    = 4;   /* header, c2v offset, edge-slot offset, spare                          */
constexpr int EDGE_SLOT      = 20;  /* words per row in the LDS edge table: degree <= 19 + one dummy edge    */

/* What one wave does in one decoder step: one 64-lane chunk of one row (check nodes t0 .. t0 + 63), or with edge
 * splitting 32 check nodes whose edges are shared by lanes l and l ^ 32. Built on the host per (graph, step, wave) and
 * fetched one step ahead (ldpc_graph.cpp build_tasks, ldpc_hip_kernels.hip).
 *   w[0] = degree | split << 5 | active << 6 | row << 8 | t0 << 16
 *   w[1] = byte offset of the row's c2v messages in the LDS c2v area
 *   w[2] = byte offset of the row's slot in the LDS edge table (EDGE_SLOT words: shift | (col * Z) << 16 per edge,
 *          then dummy edges that point at the scratch bytes after the soft bits)                           */
struct step_task {
  uint32_t w[TASK_DWORDS];
};

/* Lifted graph for one (BG, Z), built on the host from the TS 38.212 tables (ldpc_base_graphs.inc).
 * edges[e]   = (col * Z) | (shift mod Z) << 16        in row-major edge order (the reference's adjacency order)
 * rows[m]    = first edge index | degree << 16
 * groups[g]  = first row | rows << 8 | P << 16      consecutive rows that share no variable node; P = 2 splits
 *              each check node's edges over lanes l and l ^ 32
 * c2v_off[m] = byte offset of row m's check-to-variable messages in the LDS c2v area: int8 c2v[e][t] for the
 *              row's edges e, stride Z (ldpc_hip_kernels.hip "Check-to-variable storage").               */
struct graph_desc {
  uint8_t  bg;
  uint8_t  maxdeg;
  uint16_t Z;
  uint16_t K;
  uint16_t M;
  uint16_t N_full;
  uint16_t n_edges;
  uint16_t n_groups;
  uint16_t max_group_rows;
  uint32_t edges[MAX_EDGES];
  uint32_t rows[MAX_ROWS];
  uint32_t groups[MAX_ROWS];
  uint32_t c2v_off[MAX_ROWS];
  uint32_t c2v_bytes;
  uint16_t n_steps;              /* steps per iteration                                    */
  uint16_t task_waves;           /* waves per workgroup = step_task entries per step      */
  uint32_t task_offset;          /* first step_task of this graph in the context's table  */
  uint8_t  step_row0[MAX_STEPS]; /* first row of each step (adaptive layer count)         */
  uint8_t  ils;                  /* lifting-set index iLS (TS 38.212 Table 5.3.2-1)       */
  uint8_t  pad[3];
};

/* LDS carve-up for one decoder launch (every offset a multiple of 16; cdna_hip_programming.md G17). */
struct lds_layout {
  uint32_t soft;   /* soft bits, N_full columns of soft_stride bytes (int8; binary16 in the specialised kernels) */
  uint32_t soft_stride; /* Z; specialised kernels: SOFT_BYTES Z (4 Z with ldpc_spec.h SOFT_COPIES = 4) */
  uint32_t soft_read;   /* offset of the copy the decoder reads inside a column: 0; Z for the specialised kernel */
  uint32_t c2v;    /* int8 c2v per edge, n_edges * Z        */
  uint32_t hard;   /* packed hard bits, ceil(K*Z/8) + 16    */
  uint32_t red;    /* uint32 reduction scratch, 32 words    */
  uint32_t crct;   /* uint32 CRC byte table, 256 words      */
  uint32_t edges;  /* uint32 edge table, M * EDGE_SLOT words */
  uint32_t total;
  uint32_t split_tab; /* specialised BG1: word offset of the graph's split-row address table in the table buffer */
};

/* One (BG, Z) group of a mixed decoder launch (ldpc_decode_mixed_kernel): workgroups [first_block, next group's
 * first_block) decode with graph c_graphs[graph_slot], its step tasks at task_offset and LDS layout lay. */
struct mixed_group {
  uint32_t   first_block;
  int32_t    graph_slot;
  uint32_t   task_offset;
  uint32_t   spec; /* 1: specialised body (ldpc_spec.h) */
  lds_layout lay;
};
constexpr int MIXED_BLOCK = 768;

/* One decoder work item (one workgroup). Offsets are relative to the launch's base pointers. */
struct dec_cb {
  uint64_t llr_offset;
  uint64_t out_offset;
  uint32_t llr_length;
  uint32_t result_index;
  uint16_t nof_filler_bits;
  uint8_t  max_iterations;
  uint8_t  crc_mode;
  int8_t   crc_poly;
  uint8_t  keep_passed; /* LDPC_HIP_CRC_MODE_FLAG_KEEP_PASSED */
  uint8_t  pad[2];
  float    scaling_factor;
};

/* One encoder work item (one workgroup): packed message in, packed shortened codeword out. The message is data_bits
 * bits from bit msg_bit_off (< 8) of byte msg_offset, then zeros up to K Z; crc_at > 0 attaches the CRC24B of bits
 * [0, crc_at) at bit crc_at (the HAL's TB mode: one staged TB, every segment read in place). */
struct enc_cb {
  uint64_t msg_offset;
  uint64_t cw_offset;
  uint32_t cw_length; /* output bits, <= N_short * Z */
  int32_t  graph_slot;
  uint32_t msg_bit_off;
  uint32_t data_bits; /* <= K Z        */
  uint32_t crc_at;    /* 0: no CRC     */
  uint32_t pad;
};

/* One rate-matcher work item: packed shortened codeword in, packed E bits out (ldpc_rate_matcher_impl.cpp). */
struct ratematch_cb {
  uint64_t cw_offset;
  uint64_t out_offset;
  uint32_t cb_length; /* N = N_short * Z */
  uint32_t rm_length; /* E                */
  uint32_t Ncb;
  uint32_t k0;
  uint32_t fill_lo;   /* filler range [fill_lo, fill_hi) in the shortened codeword */
  uint32_t fill_hi;
  uint32_t Qm;
  uint32_t pad;
};

/* One codeblock of the PDSCH encoder queue's fused encode + rate match (ldpc_pdsch_encode_kernel): rm.cw_offset unused. */
struct pdsch_enc_cb {
  enc_cb       enc;
  ratematch_cb rm;
};
constexpr int ENC_THREADS = 256; /* encoder workgroup */

/* Rate dematcher: threads per workgroup (one workgroup per CB) and the largest E staged in LDS. */
constexpr int      DM_THREADS = 512;
constexpr unsigned DM_STAGE   = 32768;

/* One rate-dematch work item. llr / soft are absolute device pointers. With sym != nullptr the E LLRs are not read
 * from llr but produced in LDS by soft-demodulating the CB's E / Qm symbols (sym, noise variances nv, modulation
 * demod = modulation_scheme value; E <= DM_STAGE): ldpc_hip_demod_dematch_launch. */
struct dematch_cb {
  const int8_t* llr;
  int8_t*       soft;
  const float*  sym; /* interleaved (re, im) */
  const float*  nv;
  uint32_t      cb_length;
  uint32_t      rm_length;
  uint32_t      Nref;
  uint32_t      nof_filler_bits;
  uint8_t       modulation_order;
  uint8_t       rv;
  uint8_t       new_data;
  uint8_t       demod;
  uint32_t      stage_bytes; /* LDS staging the launch reserved for the LLRs (E <= stage_bytes is staged); 0: DM_STAGE */
};

/* One soft-demodulation segment (ldpc_hip_demodulate_launch): nof_symbols symbols of one modulation. Blocks
 * [block0, block0 + ceil(nof_symbols / DEMOD_BLOCK)) of the launch work on it. */
constexpr int DEMOD_BLOCK = 256;
struct demod_seg {
  uint64_t sym_offset;   /* complex symbols (float re, im) from the symbol base */
  uint64_t noise_offset; /* floats from the noise-variance base                  */
  uint64_t llr_offset;   /* bytes from the LLR base                              */
  uint32_t nof_symbols;
  uint32_t block0;
  uint8_t  modulation;   /* modulation_scheme value                              */
  uint8_t  qm;
  uint8_t  pad[6];
};

/* Slopes, intercepts and interval widths of the piecewise-linear LLR approximations, computed on the host in float
 * exactly as the reference computes its tables (demodulation_mapper_qam{16,64,256}.cpp), passed by value. */
struct demod_tables {
  float s10;                                         /* 1 / sqrt(10): 16-QAM */
  float w64a, w64c;                                  /* 64-QAM interval widths */
  float sl64[3][8], ic64[3][8];
  float w256a, w256c;                                /* 256-QAM interval widths */
  float sl256[4][16], ic256[4][16];
};
/* Dynamic LDS a decode launch with the fused dematcher needs at least: the staging buffer, then the tables' copy. */
constexpr uint32_t DM_FUSED_LDS = DM_STAGE + ((sizeof(demod_tables) + 15U) & ~15U);

/* ---- the device work queue (ldpc_hip_dwq.cpp): single-codeblock operations handed to a resident grid ----------
 * One work item: a fused dematch + decode of one codeblock on a specialised body (spec = id + 1), or a dematch alone
 * (spec = 0). Written by the host into a ring slot of pinned memory; a workgroup of the unit's persistent grid claims
 * it, copies it into LDS and runs it. Offsets in cb are relative to llr_base / out_base, result_index to res_base. */
struct dwq_item {
  dec_cb              cb;
  lds_layout          lay;
  dematch_cb          dm;   /* dm.soft != nullptr: the dematcher runs first (fused) */
  const int8_t*       llr_base;
  uint8_t*            out_base;
  ldpc_hip_cb_result* res_base;
  const uint32_t*     crc_tables;
  uint32_t            spec; /* specialised kernel id + 1; 0: dematch only */
  uint32_t            ticket;
  uint32_t            pad[4];
};
constexpr uint32_t DWQ_ITEM_WORDS = sizeof(dwq_item) / 4;
static_assert(sizeof(dwq_item) % 16 == 0, "dwq_item copied as words");
/* A ring slot: the item's words 0-44 (every field through pad[0]) in three 64-byte lines of 15 words, each line
 * followed by a sequence word = ticket + 1 that the host writes after the line's payload. A poller reads the whole slot
 * in one round trip and accepts it only when all three sequence words match (a line is read as one snapshot), so the
 * item arrives with the poll. */
constexpr uint32_t DWQ_WIRE_WORDS = 48;
constexpr uint32_t DWQ_WIRE_PAYLOAD = 45;
static_assert(DWQ_ITEM_WORDS == DWQ_WIRE_WORDS && offsetof(dwq_item, pad) / 4 + 1 == DWQ_WIRE_PAYLOAD,
              "wire slot: item words 0-44 carried");
/* Word 44 of an item on the wire (pad[0]) is the checksum of its words 0-43, the ticket included: XOR over i of
 * dwq_mix(word_i, i). The poller accepts a slot only when the checksum of the 44 words it read matches, so an item is
 * self-validating however the slot's lines are fetched (a read that mixed two publications, or a line that arrived
 * torn, fails the check and is polled again) instead of resting on a 64-byte line being read as one snapshot. */
__host__ __device__ inline uint32_t dwq_mix(uint32_t w, uint32_t i)
{
  uint32_t h = (w ^ (i * 0x9E3779B9U)) * 0x85EBCA77U;
  h ^= h >> 15;
  h *= 0xC2B2AE3DU;
  h ^= h >> 13;
  return h;
}
/* A PDSCH encoder item (queue key DWQ_KEY_ENC, ldpc_dwq_encode_kernel): this payload in the item's first words, spec
 * = 1. */
struct dwq_enc_payload {
  pdsch_enc_cb    c;
  const uint8_t*  msg_base;
  uint8_t*        out_base;
  const uint32_t* crc_tables;
};
static_assert(sizeof(dwq_enc_payload) <= offsetof(dwq_item, spec), "encoder payload before the item's spec word");

/* A copy item (queue key DWQ_KEY_COPY, ldpc_dwq_copy_kernel): n16 16-byte words from src (pinned host memory, device
 * address) to dst (HBM), this payload in the item's first words, spec = 1. */
struct dwq_copy_payload {
  const uint8_t* src;
  uint8_t*       dst;
  uint64_t       n16;
};
static_assert(sizeof(dwq_copy_payload) <= offsetof(dwq_item, spec), "copy payload before the item's spec word");
constexpr int COPY_THREADS = 256;
constexpr int COPY_UNROLL  = 16; /* 16-byte loads in flight per thread: 64 KiB per workgroup and round */

inline uint32_t dwq_item_checksum(const dwq_item& it)
{
  uint32_t w[DWQ_ITEM_WORDS];
  std::memcpy(w, &it, sizeof(w));
  uint32_t x = 0;
  for (uint32_t i = 0; i != DWQ_WIRE_PAYLOAD - 1; ++i) {
    x ^= dwq_mix(w[i], i);
  }
  return x;
}
/* dwq_item::spec of an item that does nothing when claimed (a published item whose grid could not be launched: its
 * ticket must still be served in order, without touching the caller's buffers) */
constexpr uint32_t DWQ_SPEC_NOOP = 0xffffffffU;

/* Control words of a unit's queue. Host-written (pinned): published ticket count (for diagnostics), stop. Device
 * memory: the claim counter. done (pinned, device-written): ticket + 1 of the last item completed in each ring slot. */
enum : uint32_t { DWQ_H_PUBLISHED = 0, DWQ_H_STOP = 1, DWQ_H_EXITED = 2, DWQ_H_WORDS = 16 };
enum : uint32_t { DWQ_D_CLAIMED = 0, DWQ_D_PUBLISHED = 1, DWQ_D_STOP = 2, DWQ_D_STAMP = 4, DWQ_D_EXITS = 5, DWQ_D_WORDS = 16 };
struct dwq_args {
  const uint32_t* ring;       /* device address of the pinned ring (DWQ_WIRE_WORDS per slot) */
  const uint32_t* host_ctl;   /* device address of the pinned host control words */
  uint32_t*       dev_ctl;    /* device memory */
  uint32_t*       done;       /* device address of the pinned done flags */
  uint32_t        ring_mask;  /* ring size - 1 (a power of two) */
  uint32_t        ctl_lds;    /* byte offset of the LDS control words and item copy (after the bodies' LDS) */
  uint32_t        idle_ticks; /* exit after this long without a claim (100 MHz ticks) */
  uint32_t        life_ticks; /* exit after this long at the latest */
  uint32_t*       host_exit;  /* device address of the pinned word host_ctl[DWQ_H_EXITED] */
  uint32_t        exit_target; /* workgroups launched on this queue so far, this grid's included: the workgroup whose
                                  exit brings dev_ctl[DWQ_D_EXITS] to it stores it into host_exit (the grid is gone) */
  uint32_t        slot_ticks;  /* idle polling: one slot read per slot_ticks (100 MHz) for the whole grid, in turns */
  uint32_t        poll_flags;  /* DWQ_POLL_* */
};
/* poll_flags: DWQ_POLL_LONG_SLEEP: a workgroup waiting for its polling turn sleeps in long steps (one clock read per
 * ~0.85 us) instead of reading the clock every ~130 cycles; DWQ_POLL_TEST_NO_CLAIM (tests only): the grid claims
 * nothing, a stalled queue on demand, for the timed-out-wait fallback's test */
enum : uint32_t { DWQ_POLL_LONG_SLEEP = 1, DWQ_POLL_TEST_NO_CLAIM = 2 };
constexpr uint32_t DWQ_LDS_EXTRA = 32 + sizeof(dwq_item); /* control words + the claimed item */

/* The fused dematcher's LDS budget for a launch over dm[0, n): DM_FUSED_LDS when a CB soft-demodulates symbols (the
 * tables sit at DM_STAGE), else the largest staged E rounded to 16 bytes (a C4 slot's small TBs stage 1,248 LLRs, not
 * 32 KiB, so a small graph's workgroups keep the occupancy their own layout allows). Writes the budget into every
 * descriptor's stage_bytes, which decides in the kernel what is staged. */
inline uint32_t dm_fused_budget(dematch_cb* dm, size_t n)
{
  uint32_t b = 16;
  for (size_t i = 0; i != n; ++i) {
    if (dm[i].sym != nullptr) {
      b = DM_FUSED_LDS;
      break;
    }
    if (dm[i].rm_length <= DM_STAGE) {
      b = b > ((dm[i].rm_length + 15U) & ~15U) ? b : ((dm[i].rm_length + 15U) & ~15U);
    }
  }
  for (size_t i = 0; i != n; ++i) {
    dm[i].stage_bytes = b == DM_FUSED_LDS ? DM_STAGE : b;
  }
  return b;
}

} // namespace ldpc_hip
