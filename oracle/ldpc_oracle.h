/*
 * CPU ORACLE for the MI355X LDPC decode path -- TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of the reference srsRAN algorithms on the PUSCH LDPC decode path. It exists to
 * check the HIP product path; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (srsran_projectvtlmo_amd/) never links or calls anything in this directory.
 *
 * Parity status: PARTIALLY PINNED. The reference's golden .dat fixtures are absent from the snapshot and building
 * or running the reference is denied, so this restatement is pinned by (i) the reference's in-source
 * known-answer tests (log_likelihood_ratio_test.cpp:32-87, crc_calculator_test.cpp:32-110,
 * ldpc_enc_dec_test.cpp:334-358, hard_decision_test.cpp), (ii) noiseless encode->decode and
 * rate-match->dematch round trips, and (iii) the survey's record that a restatement of the same pseudo-code matched
 * the reference generic decoder bit-exactly on 48/48 randomised cases. See DESIGN.md "Oracle".
 *
 * Each function cites the reference file:line it follows.
 */
#ifndef LDPC_ORACLE_H
#define LDPC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- LLR arithmetic: lib/phy/upper/log_likelihood_ratio.cpp:39-97, include/.../log_likelihood_ratio.h:46-244 ---- */
int8_t orc_llr_add(int8_t a, int8_t b);            /* saturated sum (operator+=, :56-71)            */
int8_t orc_llr_sub(int8_t a, int8_t b);            /* a + (-b) (operator-, header)                   */
int8_t orc_llr_promotion_sum(int8_t a, int8_t b);  /* promotion_sum (:73-86)                        */
int8_t orc_llr_quantize(float value, float range); /* quantize (:88-97)                             */
/* hard_decision (:226-252): packs (llr <= 0) MSB-first into out; returns 1 iff no llr == 0. */
int orc_hard_decision(uint8_t* out_packed, const int8_t* llr, unsigned n);

/* ---- CRC: lib/phy/upper/channel_coding/crc_calculator_generic_impl.cpp:28-133 ---- */
enum { ORC_CRC24A = 0, ORC_CRC24B = 1, ORC_CRC24C = 2, ORC_CRC16 = 3, ORC_CRC11 = 4, ORC_CRC6 = 5 };
uint32_t orc_crc_packed(int poly, const uint8_t* packed, unsigned nbits); /* calculate(bit_buffer) :111-133 */
uint32_t orc_crc_bytes(int poly, const uint8_t* bytes, unsigned nbytes); /* calculate_byte :59-86         */
uint32_t orc_crc_bits(int poly, const uint8_t* bits, unsigned nbits);    /* calculate_bit :88-109          */

/* ---- Graph: ldpc_graph_impl.{h,cpp}, ldpc_luts_impl.cpp:57 (LSindex), :4521-4566 (get_graph) ---- */
int orc_lifting_index(unsigned Z);    /* 0..7, or -1 if Z is not a valid lifting size */
int orc_lifting_position(unsigned Z); /* 0..50, or -1                                 */
/* Fills (col, shift mod Z) for every edge of row m; returns the row degree, or -1 on error. */
int orc_graph_row(int bg, unsigned Z, unsigned m, uint16_t* cols, uint16_t* shifts);

/* ---- Decoder: ldpc_decoder_impl.cpp:33-308 + ldpc_decoder_generic.cpp:30-128 (fresh decoder object) ----
 * out_packed: ceil(K*Z/8) bytes, MSB-first. crc_poly < 0 disables early stopping (crc == nullptr).
 * Returns the number of iterations when the CRC passed (std::optional has_value), 0 for std::nullopt, -1 on a
 * contract violation (the reference would srsran_assert). When all LLRs are zero and crc_poly >= 0 the output
 * is left untouched (ldpc_decoder_impl.cpp:86-94). */
int orc_ldpc_decode(int bg, unsigned Z, unsigned nof_filler_bits, const int8_t* llr, unsigned llr_len,
                    unsigned max_iterations, float scaling_factor, int crc_poly, uint8_t* out_packed);

/* ---- Rate dematcher: ldpc_rate_dematcher_impl.cpp:46-213 ----
 * out: N = cb_len LLRs (HARQ soft buffer, in/out). Qm = bits per symbol (1,2,4,6,8). Returns 0, -1 on error. */
int orc_rate_dematch(int8_t* out, unsigned cb_len, const int8_t* in, unsigned E, int new_data, unsigned rv,
                     unsigned Qm, unsigned Nref, unsigned nof_filler_bits);

/* ---- Encoder (TS 38.212 §5.3.2) and rate matcher (§5.4.2): test-vector generation only ----
 * msg_bits: K*Z unpacked bits; filler positions hold ORC_FILLER_BIT. cw_bits receives cb_len bits of the
 * shortened codeblock (codeblock bits 2Z .. 2Z+cb_len), filler positions as ORC_FILLER_BIT. */
#define ORC_FILLER_BIT 254
int orc_ldpc_encode(int bg, unsigned Z, const uint8_t* msg_bits, uint8_t* cw_bits, unsigned cb_len);
/* cw_bits: N = N_short*Z codeblock bits (filler = ORC_FILLER_BIT). out_bits: E rate-matched bits. */
int orc_rate_match(uint8_t* out_bits, unsigned E, const uint8_t* cw_bits, unsigned N, unsigned rv, unsigned Qm,
                   unsigned Nref, int bg, unsigned Z);

/* ---- RX segmenter: ldpc_segmenter_impl.cpp:58-69, 254-331; ldpc.h:140-193 ---- */
typedef struct {
  int      bg;
  unsigned lifting_size;
  unsigned nof_segments;
  unsigned full_length;     /* N_full-ish codeblock length before shortening handling, per the reference */
  unsigned nof_filler_bits;
  unsigned nof_crc_bits;    /* per-CB CRC length (TB CRC length when one segment) */
  unsigned rm_length;       /* E_r */
  unsigned cw_offset;
} orc_cb_meta;
/* Returns number of segments (<= max_cbs), -1 on error. */
int orc_segment_rx(unsigned tbs, int bg, unsigned nof_ch_symbols, unsigned Qm, unsigned nof_layers,
                   orc_cb_meta* out, unsigned max_cbs);

/* ---- pusch_codeblock_decoder::decode (pusch_codeblock_decoder.cpp:35-71) ----
 * rate-dematch into soft_buf (N LLRs) then decode; returns iterations (>0) when the CB CRC passes, 0 otherwise. */
int orc_pusch_cb_decode(uint8_t* out_packed, int8_t* soft_buf, unsigned cb_len, const int8_t* llr_E, unsigned E,
                        int new_data, int bg, unsigned Z, unsigned rv, unsigned Qm, unsigned Nref,
                        unsigned nof_filler_bits, int crc_poly, int use_early_stop, unsigned nof_iterations);

/* ---- transport-block join: pusch_decoder_impl::join_and_notify / concatenate_codeblocks
 * (pusch_decoder_impl.cpp:384-497, get_cblk_bit_breakdown :50-67) ----
 * msgs: C decoded CB messages, packed MSB-first, msg_stride bytes apart, each K*Z = cb_msg_bits bits.
 * cb_crc_ok: per-CB CRC flags. tb_out: ceil(tbs/8) bytes, written as the reference writes transport_block
 * (C = 1: only when the CB CRC passed; C > 1: only when every CB CRC passed). cb_crc_bits: the CB's CRC length
 * (the TB CRC length when C = 1). Returns 1 when the TB CRC is OK, 0 otherwise. */
int orc_tb_join(const uint8_t* msgs, unsigned msg_stride, unsigned nof_cbs, unsigned cb_msg_bits,
                unsigned nof_filler_bits, unsigned cb_crc_bits, unsigned tbs, const uint8_t* cb_crc_ok,
                uint8_t* tb_out);

/* ---- vectorisable CPU port (ldpc_cpu_port.c): orc_ldpc_decode's semantics at scaling factor 0.8, organised for
 * SIMD like the reference AVX2 decoder; bench.py's cpu_baseline. Same return convention as orc_ldpc_decode. ---- */
int orc_ldpc_decode_port(int bg, unsigned Z, unsigned nof_filler_bits, const int8_t* llr, unsigned llr_len,
                         unsigned max_iterations, int crc_poly, uint8_t* out_packed);

/* The port's table-driven CRC (same remainder as orc_crc_packed for CRC24A/24B/16; other polynomials fall back to it) */
uint32_t orc_crc_port(int poly, const uint8_t* packed, unsigned nbits);

/* bench.py's cpu_baseline timing loop (ldpc_cpu_bench.c): `threads` threads, each one warm-up and `reps` timed decodes
 * of `llr` (no CRC) with the port; per-decode latencies in lat_ns[thread * reps + r], the run's wall time in *wall_s.
 * Returns 0, -1 on an invalid argument or a failed decode. */
int orc_bench_port(int bg, unsigned Z, const int8_t* llr, unsigned llr_len, unsigned iters, unsigned threads,
                   unsigned reps, uint32_t* lat_ns, double* wall_s);

/* The CPU leg of bench.py's software-route figure (ldpc_cpu_slot.c): a slot's codeblocks on `threads` workers in
 * pusch_decoder_impl's per-CB task order (pusch_decoder_impl.cpp:309-382, pusch_codeblock_decoder.cpp:35-71). */
typedef struct {
  int           bg;
  unsigned      Z, F, Qm, rv, iters, E;
  int           crc_poly; /* ORC CRC id (CRC24A 0, CRC24B 1, CRC16 3) */
  const int8_t* llr;      /* E rate-matched LLRs */
} orc_slot_cb;
/* with_dematch 1: rate dematch + decode per task; 0: decode only (soft buffers dematched beforehand). Two warm-up
 * slots, then `reps` timed: slot_us[reps], per-CB dec_us / dm_us[reps * n]; crc_ok: CRC-passed CBs of the last slot.
 * Returns 0, -1 on an invalid argument or a failed call. */
int orc_bench_slot(const orc_slot_cb* cbs, unsigned n, unsigned threads, unsigned reps, int with_dematch,
                   double* slot_us, double* dec_us, double* dm_us, unsigned* crc_ok);

/* ---- soft demodulation mapper: demodulation_mapper::demodulate_soft (demodulation_mapper_impl.cpp:78-106) with the
 * reference's portable scalar per-symbol functions (demodulation_mapper_{qpsk,qam16,qam64,qam256}.cpp scalar loops),
 * float arithmetic without contraction. sym: nof_symbols complex symbols as (re, im) float pairs; nv: one noise
 * variance per symbol; llr: nof_symbols * Qm outputs. mod: modulation_scheme value (PI_2_BPSK 0, BPSK 1, QPSK 2,
 * QAM16 4, QAM64 6, QAM256 8). Returns 0, -1 for an invalid modulation. ---- */
int orc_demodulate_soft(int mod, unsigned nof_symbols, const float* sym, const float* nv, int8_t* llr);

#ifdef __cplusplus
}
#endif

#endif /* LDPC_ORACLE_H */
