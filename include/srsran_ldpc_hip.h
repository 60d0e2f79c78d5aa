/*
 * srsran_ldpc_hip.h -- C ABI of the MI355X-native (gfx950) 5G-NR PUSCH LDPC decode path.
 *
 * This is the drop-in boundary. It is a plain C interface: POD structs, raw pointers and sizes, integer status codes,
 * no exceptions and no torch/HIP C++ types in the signatures. srsRAN-side adapters (C++: ldpc_decoder_hip,
 * ldpc_rate_dematcher_hip, hw_accelerator_pusch_dec_hip; Python mirror in srsran_projectvtlmo_amd/) sit on top of it.
 * Reference interfaces replaced (paths relative to the srsRAN tree):
 *
 *   ldpc_decoder::decode                  include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:73-74
 *       -> ldpc_hip_decode_sync / ldpc_hip_decode_plan_create + ldpc_hip_decode_launch (batched, device pointers)
 *   ldpc_rate_dematcher::rate_dematch     include/srsran/phy/upper/channel_coding/ldpc/ldpc_rate_dematcher.h:52-55
 *       -> ldpc_hip_rate_dematch_sync
 *   demodulation_mapper::demodulate_soft  include/srsran/phy/upper/channel_modulation/demodulation_mapper.h:66-69
 *       -> ldpc_hip_demodulate_sync / ldpc_hip_demodulate_launch (device pointers)
 *   hal::hw_accelerator_pusch_dec         include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h:83-115
 *   hal::hw_accelerator<int8_t,uint8_t>   include/srsran/hal/hw_accelerator.h:35-57
 *       reserve_queue()/free_queue()      -> ldpc_hip_queue_reserve / ldpc_hip_queue_free
 *       configure_operation + enqueue_operation -> ldpc_hip_enqueue
 *       dequeue_operation                 -> ldpc_hip_dequeue (launches the staged batch on first call; polls)
 *       read_operation_outputs            -> ldpc_hip_read_outputs
 *       free_harq_context_entry           -> ldpc_hip_harq_free
 *       is_external_harq_supported        -> ldpc_hip_external_harq_supported
 *   hal::hw_accelerator_pdsch_enc         include/srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc.h:75-102
 *   hal::hw_accelerator<uint8_t,uint8_t>  include/srsran/hal/hw_accelerator.h:35-57
 *       reserve_queue()/free_queue()      -> ldpc_hip_enc_reserve / ldpc_hip_enc_free
 *       configure_operation               -> ldpc_hip_enc_configure
 *       enqueue_operation                 -> ldpc_hip_enc_enqueue
 *       dequeue_operation                 -> ldpc_hip_enc_dequeue (launches the staged batch on first call; polls)
 *       get_cb_mode / get_max_tb_size     -> ldpc_hip_enc_cb_mode / ldpc_hip_enc_max_tb_size
 *
 * Threading: a context is single-producer (like one pusch_decoder_hw_impl / one decoder object per worker thread,
 * pusch_decoder_impl.h:48); use one context per thread. A context is bound to one GPU and owns its device memory,
 * its HIP stream and the per-(BG,Z) graph schedules; its HAL queue's HBM HARQ soft buffers live in an external HARQ
 * repository (ldpc_hip_harq_repo) that the contexts of one GPU share, as srsRAN's PUSCH decoders share one
 * ext_harq_buffer_context_repository. Repository calls are thread-safe.
 *
 * Status codes: 0 ok, 1 not ready (dequeue/poll), negative on error (see LDPC_HIP_E*). ldpc_hip_last_error() gives a
 * message for the last error on a context.
 */
#ifndef SRSRAN_LDPC_HIP_H
#define SRSRAN_LDPC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC_HIP_OK 0
#define LDPC_HIP_NOT_READY 1
#define LDPC_HIP_DROPPED 2     /* enqueue accepted the operation as dropped: it dequeues as a CRC failure with the
                                  maximum number of iterations (acc100 drop_op, acc100_impl.cpp:179-186, 233-247)  */
#define LDPC_HIP_EINVAL (-1)   /* contract violation (the reference would srsran_assert)          */
#define LDPC_HIP_EDEVICE (-2)  /* HIP runtime error                                                */
#define LDPC_HIP_EFULL (-3)    /* HAL queue cannot take the operation now: dequeue what was enqueued, then retry  */
#define LDPC_HIP_ENOMEM (-4)   /* allocation failure                                               */
#define LDPC_HIP_ESTATE (-5)   /* call out of order (e.g. dequeue before enqueue)                  */

/* CRC polynomials, numbered as hal::hw_dec_cb_crc_type (hw_accelerator_pusch_dec.h:36). */
#define LDPC_HIP_CRC16 0
#define LDPC_HIP_CRC24B 1
#define LDPC_HIP_CRC24A 2
#define LDPC_HIP_CRC_NONE (-1)

/* CRC use by the decoder. */
#define LDPC_HIP_CRC_MODE_NONE 0        /* ldpc_decoder::decode(..., crc = nullptr, ...)                          */
#define LDPC_HIP_CRC_MODE_EARLY_STOP 1  /* ldpc_decoder::decode(..., crc, ...): CRC checked every iteration     */
#define LDPC_HIP_CRC_MODE_CHECK_AFTER 2 /* pusch_codeblock_decoder.cpp:61-70: decode w/o CRC, then check once   */
/* OR-ed into crc_mode: skip the CB (message and result kept from the previous launch) when its d_results entry already
 * reports a passed CRC -- the HARQ retransmission rule of pusch_decoder_impl.cpp:336-346 (only dematch a CB whose
 * CRC passed before). The caller clears the results on new data. */
#define LDPC_HIP_CRC_MODE_FLAG_KEEP_PASSED 0x80

/* result.status bits */
#define LDPC_HIP_STATUS_OUTPUT_WRITTEN 0x1 /* the packed message was written (not the all-zero+CRC case)        */
#define LDPC_HIP_STATUS_DROPPED 0x2        /* operation was dropped (reported as CRC fail, max iterations)       */

typedef struct ldpc_hip_ctx ldpc_hip_ctx;
typedef struct ldpc_hip_plan ldpc_hip_plan;

/* ldpc_hip_params.launch_flags: schedule controls for tests and diagnostics; 0 (the default) picks the fastest
 * launch form for every plan. All forms give bit-identical results. */
#define LDPC_HIP_LAUNCH_NO_SPEC 0x1       /* generic kernel for every graph (no compile-time schedules)               */
#define LDPC_HIP_LAUNCH_NO_MIXED 0x2      /* one launch per (BG, Z) group instead of one mixed launch                 */
#define LDPC_HIP_LAUNCH_NARROW_ALWAYS 0x4 /* narrow (two workgroups per CU) schedules wherever a graph has one      */
#define LDPC_HIP_LAUNCH_NARROW_NEVER 0x8  /* wide schedules only                                                   */
#define LDPC_HIP_LAUNCH_HAL_COPY 0x10     /* HAL queue: always stage through device buffers (no zero-copy batches)    */
#define LDPC_HIP_LAUNCH_SEPARATE_DEMATCH 0x20 /* HAL queue: rate dematching as its own kernel, not fused into decode  */
/* HAL queue without a dedicated hardware queue (hw_accelerator_pusch_dec_configuration::dedicated_queue == false,
 * include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_factories.h:42-43): ldpc_hip_queue_reserve
 * borrows one of the device's shared HIP streams (LDPC_HIP_SHARED_QUEUES of them, environment, default 4), spinning
 * until one is free, and ldpc_hip_queue_free returns it -- acc100's hw_reserve_queue / hw_free_queue
 * (hw_accelerator_pusch_dec_acc100_impl.cpp:70-98). Without the flag the context's own stream is the queue. */
#define LDPC_HIP_LAUNCH_SHARED_QUEUE 0x40
/* No device work queue: one-codeblock operations (ldpc_hip_decode_sync / ldpc_hip_rate_dematch_sync with one CB, small
 * HAL batches) are launched as kernels instead of handed to the resident grid of their graph's unit. */
#define LDPC_HIP_LAUNCH_NO_DWQ 0x80
/* HAL queue, external HARQ, batches of more codeblocks than the work queue takes (hw_pusch_decoder_configuration::
 * nof_segments > 16): with this flag (or LDPC_HIP_HAL_EARLY_COPY=1 in the environment) each chunk of staged LLRs
 * (LDPC_HIP_HAL_COPY_CHUNK bytes, default 256 KiB) is copied to device memory by the copy engine as soon as it is
 * enqueued, and the batch's kernel reads its LLRs from HBM. Without it (the default: measured faster) the kernel reads
 * them from the pinned staging buffer over PCIe. */
#define LDPC_HIP_LAUNCH_HAL_EARLY_COPY 0x100

typedef struct {
  uint32_t max_queue_cbs;   /* CBs one HAL batch holds (162 = MAX_NOF_SEGMENTS when 0); enqueue beyond: EFULL  */
  uint32_t max_cb_llrs;     /* largest rate-matched length E accepted by the HAL queue (4 x 25344 when 0)      */
  uint32_t nof_harq_slots;  /* HBM HARQ arena entries (external HARQ); 0 disables external HARQ               */
  uint32_t launch_flags;    /* LDPC_HIP_LAUNCH_* (0 = default)                                                 */
} ldpc_hip_params;

/* One codeblock for the pure decoder (ldpc_decoder::decode semantics, one fresh decoder per CB). */
typedef struct {
  uint8_t  base_graph;      /* 1 or 2                                                                         */
  uint8_t  max_iterations;  /* > 0                                                                            */
  uint8_t  crc_mode;        /* LDPC_HIP_CRC_MODE_*                                                            */
  int8_t   crc_poly;        /* LDPC_HIP_CRC16/24B/24A when crc_mode != NONE                                    */
  uint16_t lifting_size;    /* Z                                                                              */
  uint16_t nof_filler_bits; /* F (codeblock_metadata::cb_specific::nof_filler_bits)                           */
  uint32_t llr_length;      /* (K+2)Z <= llr_length <= N_short*Z                                              */
  float    scaling_factor;  /* normalised min-sum factor in (0,1); 0 selects the reference default 0.8        */
  uint64_t llr_offset;      /* byte offset of this CB's LLRs from the batch LLR base pointer                  */
  uint64_t out_offset;      /* byte offset of this CB's packed message (ceil(K*Z/8) bytes) from the out base   */
} ldpc_hip_dec_desc;

/* One codeblock for the rate dematcher (ldpc_rate_dematcher::rate_dematch semantics). */
typedef struct {
  uint8_t  modulation_order; /* Qm: 1, 2, 4, 6, 8                                                             */
  uint8_t  rv;               /* 0..3                                                                          */
  uint8_t  new_data;         /* 1: first transmission (copy), 0: combine                                      */
  uint8_t  reserved;
  uint32_t cb_length;        /* N = output size: 66Z (BG1) or 50Z (BG2)                                       */
  uint32_t rm_length;        /* E = input size, multiple of Qm                                                */
  uint32_t Nref;             /* limited-buffer length, 0 = unlimited                                          */
  uint32_t nof_filler_bits;  /* F                                                                             */
} ldpc_hip_dematch_desc;

/* HAL operation configuration: hal::hw_pusch_decoder_configuration (hw_accelerator_pusch_dec.h:39-72). */
typedef struct {
  uint8_t  base_graph;              /* 1 or 2                                       */
  uint8_t  modulation_order;        /* Qm                                           */
  uint8_t  rv;
  uint8_t  new_data;
  uint32_t nof_segments;
  uint32_t cw_length;               /* E                                            */
  uint32_t lifting_size;
  uint32_t Ncb;
  uint32_t Nref;
  uint32_t nof_segment_bits;
  uint32_t nof_filler_bits;
  uint32_t max_nof_ldpc_iterations;
  uint8_t  use_early_stop;
  uint8_t  cb_crc_type;             /* LDPC_HIP_CRC16/24B/24A                       */
  uint16_t cb_crc_len;
  uint32_t absolute_cb_id;
} ldpc_hip_hw_config;

typedef struct {
  uint8_t  crc_pass;        /* hw_pusch_decoder_outputs::CRC_pass / optional<unsigned>::has_value()            */
  uint8_t  nof_iterations;  /* iterations used (value of the optional), or max_iterations when failed           */
  uint16_t status;          /* LDPC_HIP_STATUS_* bits                                                           */
} ldpc_hip_cb_result;

/* One transport block joined on the device from its decoded codeblocks: pusch_decoder_impl::join_and_notify and
 * concatenate_codeblocks (pusch_decoder_impl.cpp:384-497). SURVEY.md section 8 row f3. */
typedef struct {
  uint64_t msg_offset;      /* byte offset of CB 0's decoded message (packed, MSB first) in d_msgs           */
  uint64_t tb_offset;       /* byte offset of the transport block in d_tb                                     */
  uint32_t msg_stride;      /* bytes between consecutive CB messages                                         */
  uint32_t tbs;             /* transport block size in bits, a multiple of 8                                 */
  uint32_t result_index;    /* CB 0's entry in d_cb_results; CB r uses result_index + r                       */
  uint16_t nof_cbs;         /* C >= 1                                                                          */
  uint16_t cb_msg_bits;     /* K * Z                                                                           */
  uint16_t nof_filler_bits; /* F                                                                               */
  uint8_t  cb_crc_bits;     /* 24 when C > 1; the TB CRC length (16 or 24) when C = 1 (codeblock_metadata)    */
  uint8_t  pad;
} ldpc_hip_tb_desc;

typedef struct {
  uint8_t  tb_crc_ok;       /* pusch_decoder_result::tb_crc_ok                                                 */
  uint8_t  written;         /* 1 when the TB bytes were written (the reference writes them only in that case) */
  uint16_t nof_cbs_ok;      /* codeblocks whose CRC passed                                                      */
} ldpc_hip_tb_result;

/* LDPC encoding of one codeblock (ldpc_encoder::encode, ldpc_encoder_impl.cpp:47-81): message of K*Z bits (filler bits
 * as 0), packed MSB first, into the shortened codeword bits [2Z, 2Z + cw_length). SURVEY.md section 8 row f2. */
typedef struct {
  uint64_t msg_offset;   /* byte offset of the packed message in d_msgs */
  uint64_t cw_offset;    /* byte offset of the packed codeword in d_cws */
  uint32_t cw_length;    /* codeword bits to produce, <= N_short * Z      */
  uint16_t lifting_size;
  uint8_t  base_graph;
  uint8_t  pad;
} ldpc_hip_enc_desc;

/* Rate matching of one codeblock (ldpc_rate_matcher::rate_match, ldpc_rate_matcher_impl.cpp:36-160): E bits selected
 * from k0 around the circular buffer of the shortened codeword (length cb_length = N_short * Z, limited to Nref when
 * Nref > 0), skipping the filler bits, then bit-interleaved for Qm. Input and output packed MSB first. */
typedef struct {
  uint64_t cw_offset;        /* byte offset of the packed codeword in d_cws */
  uint64_t out_offset;       /* byte offset of the packed E bits in d_out   */
  uint32_t cb_length;        /* N                                            */
  uint32_t rm_length;        /* E, a multiple of Qm                          */
  uint32_t Nref;             /* 0: no limited buffer                         */
  uint16_t nof_filler_bits;
  uint8_t  modulation_order; /* Qm                                           */
  uint8_t  rv;
} ldpc_hip_rm_desc;

/* Modulation schemes, numbered as srsran::modulation_scheme (include/srsran/ran/sch/modulation_scheme.h:39-52). */
#define LDPC_HIP_MOD_PI_2_BPSK 0
#define LDPC_HIP_MOD_BPSK 1
#define LDPC_HIP_MOD_QPSK 2
#define LDPC_HIP_MOD_QAM16 4
#define LDPC_HIP_MOD_QAM64 6
#define LDPC_HIP_MOD_QAM256 8

/* One soft-demodulation segment (demodulation_mapper::demodulate_soft over one span of symbols): nof_symbols complex
 * symbols (interleaved float re, im) with one noise variance each, into nof_symbols * Qm int8 LLRs. For pi/2-BPSK
 * the symbol parity counts from the segment's first symbol, as in the reference span. SURVEY.md section 8 row f4. */
typedef struct {
  uint64_t symbol_offset; /* complex symbols from d_symbols (8 bytes each)      */
  uint64_t noise_offset;  /* floats from d_noise_vars                            */
  uint64_t llr_offset;    /* bytes from d_llrs                                   */
  uint32_t nof_symbols;
  uint8_t  modulation;    /* LDPC_HIP_MOD_*                                      */
  uint8_t  pad[3];
} ldpc_hip_demod_desc;

/* ---- external HARQ buffer repository (one per GPU, shared by every HAL context on it) ---------------------------
 * hal::ext_harq_buffer_context_repository (include/srsran/hal/phy/upper/channel_processors/pusch/
 * ext_harq_buffer_context_repository.h:44-96) together with the device HARQ memory it describes: nof_codeblocks soft
 * buffers of LDPC_HIP_HARQ_STRIDE int8 each in HBM, direct-indexed by absolute_cb_id, and per entry the soft-data
 * length and empty flag. The reference creates ONE repository (create_ext_harq_buffer_context_repository,
 * ext_harq_buffer_context_repository_factory.cpp:28-34) and hands it to every hw_accelerator_pusch_dec its factory
 * creates (hw_accelerator_factories.h:41, hw_accelerator_factories.cpp:46-65), so a retransmission may be decoded by
 * a different PUSCH decoder (thread) than the first transmission; here every context opened with ldpc_hip_open_harq on
 * the repository's GPU shares it. Entry updates are atomic: contexts on different threads may use one repository.
 * debug_mode keeps entries on free (the reference's HARQ unit-test mode, :92-95).
 * Reference-counted: the creator holds one reference, every context opened on it another; the HBM is released with
 * the last reference. */
typedef struct ldpc_hip_harq_repo ldpc_hip_harq_repo;
#define LDPC_HIP_HARQ_STRIDE 25344u /* bytes per entry: MAX_CODEBLOCK_SIZE, 66 x 384 LLRs (ldpc.h:113) */
int ldpc_hip_harq_repo_create(int device, uint32_t nof_codeblocks, int debug_mode, ldpc_hip_harq_repo** repo);
int ldpc_hip_harq_repo_release(ldpc_hip_harq_repo* repo);
/* Entry state of absolute_cb_id: returns 1 when the entry is empty, 0 when it holds soft data of *soft_data_len LLRs
 * (0 until the first decode of the entry completes), LDPC_HIP_EINVAL when the id is out of bounds. */
int ldpc_hip_harq_repo_entry(const ldpc_hip_harq_repo* repo, uint32_t absolute_cb_id, uint32_t* soft_data_len);
/* Copies the first len (<= LDPC_HIP_HARQ_STRIDE) soft bits of entry absolute_cb_id to host memory (synchronous;
 * tests and diagnostics). */
int ldpc_hip_harq_repo_read(ldpc_hip_harq_repo* repo, uint32_t absolute_cb_id, int8_t* dst, uint32_t len);

/* The GPU's HARQ memory, the way acc100 splits HARQ state: the caller's hal::ext_harq_buffer_context_repository
 * (ext_harq_buffer_context_repository.h:48-105) keeps each entry's {soft_data_len, empty} and the caller decides which
 * operations to drop (hw_accelerator_pusch_dec_acc100_impl.cpp:113, 123-125, 184-186, 206-211, 270), while the soft
 * bits live in the accelerator's own HARQ memory at absolute_cb_id (bbdev_ldpc_decoder.cpp:146). Here that memory is
 * HBM owned by the library: ONE per device and process, shared by every context opened on it with
 * ldpc_hip_open_harq, LDPC_HIP_HARQ_STRIDE int8 per absolute_cb_id. A context on it never drops an operation itself,
 * ldpc_hip_harq_free is a no-op for it and ldpc_hip_harq_repo_entry reports LDPC_HIP_ESTATE (the caller holds the
 * state). It grows on demand to any absolute_cb_id below 2^20 (waiting once for the device's queued work), starting
 * from LDPC_HIP_HARQ_CODEBLOCKS entries (environment; default 2048, 52 MB). Returns a new reference
 * (ldpc_hip_harq_repo_release); the library keeps the memory for the process lifetime. */
int      ldpc_hip_harq_device_memory(int device, ldpc_hip_harq_repo** memory);
/* Entries a repository or the device's HARQ memory currently holds. */
uint32_t ldpc_hip_harq_capacity(const ldpc_hip_harq_repo* repo);

/* The GPU a factory type "auto" resolves to (ldpc_decoder_factory_sw::create, channel_coding_factories.cpp:100-124):
 * LDPC_HIP_AUTO_DEVICE (environment; default 0) when that device is visible and a gfx950 (MI355X), else -1 (no GPU:
 * "auto" keeps the CPU decoders). */
int ldpc_hip_auto_device(void);

/* Decoder work of one codeblock, for the "auto" decoder type's CPU/GPU choice (host only, no GPU needed): edges of the
 * layers the codeblock decodes x Z x max_iterations, the layer count from the last non-zero of llr[0, llr_length) as
 * ldpc_decoder_impl.cpp:97-114 derives it; 0 for an all-zero input or an invalid descriptor. */
uint64_t ldpc_hip_decode_work(const ldpc_hip_dec_desc* desc, const int8_t* llr);
/* (with CRC early stop the iterations counted are min(max_iterations, 2), the typical count) */
/* The work above which "auto" decodes a codeblock on the GPU and below which it keeps the reference's CPU decoder
 * (channel_coding_factories.cpp:100-121): LDPC_HIP_AUTO_MIN_WORK (environment) or the measured crossover (DESIGN.md
 * section 4.8). */
uint64_t ldpc_hip_auto_min_work(void);

/* ---- context ---------------------------------------------------------------------------------------------- */
/* params->nof_harq_slots != 0 gives the context a private repository of that many entries (ldpc_hip_open_harq with a
 * repository of its own). */
int         ldpc_hip_open(int device, const ldpc_hip_params* params, ldpc_hip_ctx** ctx);
/* A context whose HAL queue keeps its soft buffers in `repo` (external HARQ, shared with the repository's other
 * contexts; params->nof_harq_slots is ignored). repo must live on `device`. repo == NULL: as ldpc_hip_open. */
int         ldpc_hip_open_harq(int device, const ldpc_hip_params* params, ldpc_hip_harq_repo* repo, ldpc_hip_ctx** ctx);
int         ldpc_hip_close(ldpc_hip_ctx* ctx);
const char* ldpc_hip_last_error(const ldpc_hip_ctx* ctx);
/* HIP stream the context launches on (hipStream_t as void*); callers may pass it to their own frameworks.
 * Every entry point's `stream` argument: NULL = this context stream; hipStreamLegacy = the legacy default (null)
 * stream; hipStreamPerThread = the calling thread's default stream; otherwise a stream of the context's device.
 * ldpc_hip_capture_begin refuses the two default streams (LDPC_HIP_EINVAL), which HIP cannot capture. */
void*       ldpc_hip_stream(ldpc_hip_ctx* ctx);

/* ---- batched decoder on device-resident data (the throughput path) ------------------------------------------ */
/* Uploads the descriptors and builds per-(BG,Z) launch groups once; a plan can be launched many times. */
int ldpc_hip_decode_plan_create(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dec_desc* descs,
                                ldpc_hip_plan** plan);
int ldpc_hip_decode_plan_destroy(ldpc_hip_plan* plan);
/* Asynchronous on `stream` (hipStream_t as void*, NULL = the context stream). d_llr/d_out/d_results are device
 * pointers; d_results holds nof_cbs entries (may be NULL). */
int ldpc_hip_decode_launch(ldpc_hip_plan* plan, const int8_t* d_llr, uint8_t* d_out, ldpc_hip_cb_result* d_results,
                           void* stream);

/* Rate-dematches nof_cbs codeblocks on device-resident buffers, asynchronously on `stream` (NULL = the context
 * stream): CB i reads descs[i].rm_length LLRs at d_llr + llr_offsets[i] and combines into / overwrites the
 * descs[i].cb_length soft bits at d_soft + soft_offsets[i] (ldpc_rate_dematcher_impl.cpp:46-213). The soft bits are
 * the decoder's input for the same CB (ldpc_hip_decode_launch). */
int ldpc_hip_rate_dematch_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dematch_desc* descs,
                                 const int8_t* d_llr, const uint64_t* llr_offsets, int8_t* d_soft,
                                 const uint64_t* soft_offsets, void* stream);

/* Encodes / rate-matches nof_cbs codeblocks on device buffers, asynchronously on `stream` (NULL = the context
 * stream). The downlink counterpart of the decode path (hw_accelerator_pdsch_enc's operations); also used to build
 * device-resident test and benchmark codewords. */
int ldpc_hip_encode_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_enc_desc* descs, const uint8_t* d_msgs,
                           uint8_t* d_cws, void* stream);
int ldpc_hip_rate_match_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_rm_desc* descs,
                               const uint8_t* d_cws, uint8_t* d_out, void* stream);

/* Joins nof_tbs transport blocks on the device, asynchronously on `stream` (NULL = the context stream): the CB data
 * bits are concatenated into d_tb and the TB CRC24A is checked against the checksum carried by the last CB; with one
 * CB its CRC is the TB CRC. d_msgs / d_cb_results are typically the outputs of ldpc_hip_decode_launch. When every CB
 * passed but the TB CRC fails, the TB's CB results are marked failed (crc_pass = 0), as reset_codeblocks_crc does
 * (pusch_decoder_impl.cpp:423-428), so a retransmission decodes them again. */
int ldpc_hip_tb_join_launch(ldpc_hip_ctx* ctx, uint32_t nof_tbs, const ldpc_hip_tb_desc* descs, const uint8_t* d_msgs,
                            ldpc_hip_cb_result* d_cb_results, uint8_t* d_tb, ldpc_hip_tb_result* d_tb_results,
                            void* stream);

/* Soft-demodulates nof_segs segments on device buffers, asynchronously on `stream` (NULL = the context stream):
 * the LLRs a PUSCH demodulator hands to the rate dematcher (ldpc_hip_rate_dematch_launch). Bit-exact with the
 * reference's portable per-symbol functions (demodulation_mapper_*.cpp), including the noise-variance <= 0 / NaN and
 * near-zero-symbol rules (LLR 0). */
int ldpc_hip_demodulate_launch(ldpc_hip_ctx* ctx, uint32_t nof_segs, const ldpc_hip_demod_desc* descs,
                               const float* d_symbols, const float* d_noise_vars, int8_t* d_llrs, void* stream);

/* Soft demodulation fused into rate dematching (the PUSCH demodulator's output feeding pusch_codeblock_decoder's
 * ldpc_rate_dematcher::rate_dematch, pusch_codeblock_decoder.cpp:35-71): CB i's descs[i].rm_length LLRs are
 * demod[i].nof_symbols symbols of demod[i].modulation at d_symbols + 2 * demod[i].symbol_offset floats, demodulated
 * exactly as ldpc_hip_demodulate_launch does (demod[i].llr_offset is not used) and dematched into d_soft +
 * soft_offsets[i] without an LLR round trip through HBM. Requires nof_symbols * Qm == rm_length <= 32768. */
int ldpc_hip_demod_dematch_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dematch_desc* descs,
                                  const ldpc_hip_demod_desc* demod, const float* d_symbols,
                                  const float* d_noise_vars, int8_t* d_soft, const uint64_t* soft_offsets,
                                  void* stream);

/* Rate dematching fused into decoding, one launch: equivalent to ldpc_hip_rate_dematch_launch (or, with demod !=
 * NULL, ldpc_hip_demod_dematch_launch) of plan's nof_cbs codeblocks followed by ldpc_hip_decode_launch(plan, d_soft,
 * d_out, d_results, stream), where dematch descriptor i writes the soft buffer decode descriptor i of the plan reads
 * (d_soft + its llr_offset). Each decoder workgroup first dematches its codeblock (pusch_codeblock_decoder.cpp:35-71
 * calls rate_dematch then decode per codeblock): one kernel boundary, one launch and one pass over the soft buffers
 * less. descs / llr_offsets / demod are indexed like the plan's decode descriptors; d_llr / llr_offsets are unused
 * with demod (then d_symbols / d_noise_vars as in ldpc_hip_demod_dematch_launch, rm_length <= 32768). */
int ldpc_hip_dematch_decode_launch(ldpc_hip_plan* plan, const ldpc_hip_dematch_desc* descs, const int8_t* d_llr,
                                   const uint64_t* llr_offsets, const ldpc_hip_demod_desc* demod,
                                   const float* d_symbols, const float* d_noise_vars, int8_t* d_soft, uint8_t* d_out,
                                   ldpc_hip_cb_result* d_results, void* stream);

/* ---- launch graphs: one submission per slot ---------------------------------------------------------------- */
/* srsRAN runs the PUSCH decode chain once per slot with the same shape slot after slot (pusch_decoder_impl /
 * pusch_decoder_hw_impl call the decoder per codeblock and join per TB). Here the chain's *_launch calls on `stream`
 * (NULL = the context stream) can be recorded once between ldpc_hip_capture_begin and ldpc_hip_capture_end (a HIP
 * graph) and replayed by ldpc_hip_graph_launch with one submission. Launch the same sequence once before capturing:
 * a launch that would upload new descriptors inside the capture fails (LDPC_HIP_EDEVICE). The device buffers the
 * captured launches use must outlive the graph. */
typedef struct ldpc_hip_graph ldpc_hip_graph;
int ldpc_hip_capture_begin(ldpc_hip_ctx* ctx, void* stream);
int ldpc_hip_capture_end(ldpc_hip_ctx* ctx, void* stream, ldpc_hip_graph** graph);
int ldpc_hip_graph_launch(ldpc_hip_graph* graph, void* stream);
int ldpc_hip_graph_destroy(ldpc_hip_graph* graph);

/* ---- synchronous host-buffer entry points (ldpc_decoder / ldpc_rate_dematcher adapters) ---------------------- */
/* Decodes nof_cbs CBs from host LLR buffers into host packed outputs. Output bytes are left untouched when the
 * reference leaves them untouched (all-zero LLRs with a CRC, ldpc_decoder_impl.cpp:86-94). */
int ldpc_hip_decode_sync(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dec_desc* descs,
                         const int8_t* const* llrs, uint8_t* const* outs, ldpc_hip_cb_result* results);
/* Dematches nof_cbs CBs; soft_bufs[i] (cb_length LLRs) is read (combine) and written (HARQ state). */
int ldpc_hip_rate_dematch_sync(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dematch_desc* descs,
                               int8_t* const* soft_bufs, const int8_t* const* llrs);

/* demodulation_mapper::demodulate_soft on host buffers: symbols = nof_symbols (re, im) float pairs. */
int ldpc_hip_demodulate_sync(ldpc_hip_ctx* ctx, uint32_t nof_symbols, int modulation, const float* symbols,
                             const float* noise_vars, int8_t* llrs);

/* ---- HAL queue: hw_accelerator_pusch_dec ------------------------------------------------------------------- */
/* The queue stages operations in pinned host memory and runs them as one batch: the first dequeue of a staged batch
 * issues ONE host-to-device copy of all staged LLRs (and, without external HARQ, soft buffers), ONE descriptor upload,
 * the dematch and decode launches and ONE device-to-host copy of all messages and results. Once every operation of a
 * launched batch has been dequeued, the next enqueue starts a new batch on the same reservation -- the order
 * pusch_decoder_hw_impl uses without external HARQ (enqueue, dequeue, enqueue, ..., pusch_decoder_hw_impl.cpp:246-261).
 * Call order per TB: reserve -> (enqueue ... dequeue ...)* -> free (pusch_decoder_hw_impl.cpp:141, 404). */
int ldpc_hip_queue_reserve(ldpc_hip_ctx* ctx);
int ldpc_hip_queue_free(ldpc_hip_ctx* ctx);
/* configure_operation + enqueue_operation. soft_in: host soft buffer (N LLRs) when external HARQ is NOT used,
 * otherwise NULL (the repository entry cfg->absolute_cb_id is used: get(absolute_cb_id, new_data) of
 * ext_harq_buffer_context_repository.h:69-83, which resets the entry on new data or when it is empty).
 * Returns LDPC_HIP_OK (staged), LDPC_HIP_DROPPED (accepted as dropped: a retransmission -- new_data == 0 -- whose entry
 * holds no soft data; acc100 soft_data_len_ok, hw_accelerator_pusch_dec_acc100_impl.cpp:123-125, 182-185), or
 * LDPC_HIP_EFULL when the batch is full or still has undequeued operations: the caller dequeues, then enqueues again
 * (enqueue_operation() == false). Contract violations return LDPC_HIP_EINVAL, among them an absolute_cb_id beyond the
 * repository's capacity (the reference asserts, :70-73) and a cb_index >= 4 x MAX_NOF_SEGMENTS. */
int ldpc_hip_enqueue(ldpc_hip_ctx* ctx, uint32_t cb_index, const ldpc_hip_hw_config* cfg, const int8_t* llrs,
                     uint32_t nof_llrs, const int8_t* soft_in, uint32_t soft_len);
/* dequeue_operation: launches the staged batch if needed; returns LDPC_HIP_NOT_READY until it completes. Copies the
 * packed message (ceil(K*Z/8) bytes) and, without external HARQ, the updated soft buffer. */
int ldpc_hip_dequeue(ldpc_hip_ctx* ctx, uint32_t cb_index, uint8_t* packed_msg, uint32_t msg_bytes, int8_t* soft_out,
                     uint32_t soft_len);
int ldpc_hip_read_outputs(ldpc_hip_ctx* ctx, uint32_t cb_index, uint32_t absolute_cb_id, ldpc_hip_cb_result* out);
/* free_harq_context_entry: marks the repository entry empty (kept in debug mode). */
int ldpc_hip_harq_free(ldpc_hip_ctx* ctx, uint32_t absolute_cb_id);
int ldpc_hip_external_harq_supported(const ldpc_hip_ctx* ctx);

/* ---- HAL queue: hw_accelerator_pdsch_enc ------------------------------------------------------------------- */
/* hal::hw_pdsch_encoder_configuration (include/srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc.h:
 * 37-76), the fields in the same order and meaning. modulation: LDPC_HIP_MOD_*. tb_crc: the TB checksum bytes the caller
 * computed (nof_tb_crc_bits / 8 of them, most significant first); used in TB mode only. */
typedef struct {
  uint32_t nof_tb_bits;
  uint32_t nof_tb_crc_bits;    /* 16 or 24                                                            */
  uint8_t  base_graph;         /* 1 or 2                                                              */
  uint8_t  modulation;         /* LDPC_HIP_MOD_*                                                      */
  uint8_t  rv;                 /* 0..3                                                                */
  uint8_t  cb_mode;            /* 1: CB mode (one segment per operation), 0: TB mode (the whole TB)   */
  uint32_t nof_segments;
  uint32_t nof_short_segments; /* segments with the short rate-matched length cw_length_a             */
  uint32_t cw_length_a;        /* Ea                                                                  */
  uint32_t cw_length_b;        /* Eb                                                                  */
  uint32_t lifting_size;
  uint32_t Ncb;                /* circular buffer length N (66 Z / 50 Z)                              */
  uint32_t Nref;               /* limited-buffer rate matching length, 0 = unlimited                 */
  uint32_t nof_segment_bits;   /* TB data bits per segment (CB CRC excluded)                          */
  uint32_t nof_filler_bits;
  uint32_t rm_length;          /* E of this segment (CB mode)                                         */
  uint8_t  tb_crc[3];
  uint8_t  reserved;
} ldpc_hip_enc_hw_config;

/* A PDSCH encoder queue on a context's GPU and stream (hw_accelerator_pdsch_enc). Operations are staged in pinned host
 * memory and run as one batch at the first dequeue: ONE host-to-device copy of all staged messages (TB mode: TB CRC
 * attached, segmented, CB CRC24B attached and filler bits added on the host), ldpc_encode_kernel and
 * ldpc_rate_match_kernel over every codeblock of the batch, ONE device-to-host copy of the packed rate-matched bits.
 * Call order per TB (pdsch_encoder_hw_impl.cpp:31-170): reserve -> (configure + enqueue ... dequeue ...)* -> free.
 * max_queue_cbs: codeblocks one batch holds (0: 162 = MAX_NOF_SEGMENTS); max_tb_bytes: get_max_tb_size() (0: 159,749,
 * the largest NR TBS in bytes). */
typedef struct ldpc_hip_enc_queue ldpc_hip_enc_queue;
int ldpc_hip_enc_queue_create(ldpc_hip_ctx* ctx, int cb_mode, uint32_t max_queue_cbs, uint32_t max_tb_bytes,
                              ldpc_hip_enc_queue** queue);
int ldpc_hip_enc_queue_destroy(ldpc_hip_enc_queue* queue);
int ldpc_hip_enc_reserve(ldpc_hip_enc_queue* queue);   /* reserve_queue */
int ldpc_hip_enc_free(ldpc_hip_enc_queue* queue);      /* free_queue    */
/* configure_operation(config, cb_index) */
int ldpc_hip_enc_configure(ldpc_hip_enc_queue* queue, uint32_t cb_index, const ldpc_hip_enc_hw_config* cfg);
/* enqueue_operation(data, {}, cb_index): CB mode: the segment's ceil((K Z - F) / 8) packed bytes (CB CRC included,
 * filler excluded); TB mode: the nof_tb_bits / 8 TB bytes. LDPC_HIP_OK (staged) or LDPC_HIP_EFULL (the batch is full
 * or still has undequeued operations: the caller dequeues, then enqueues again -- enqueue_operation() == false). */
int ldpc_hip_enc_enqueue(ldpc_hip_enc_queue* queue, uint32_t cb_index, const uint8_t* data, uint32_t nof_bytes);
/* dequeue_operation(data, packed_data, segment_index): launches the staged batch if needed; LDPC_HIP_NOT_READY until it
 * completes. bits: the rate-matched bits, one per byte (CB mode: E; TB mode: all segments concatenated); packed: the same
 * bits packed MSB first, each segment starting on a byte boundary (as the bbdev output), up to packed_bytes. */
int ldpc_hip_enc_dequeue(ldpc_hip_enc_queue* queue, uint32_t segment_index, uint8_t* bits, uint32_t nof_bits,
                         uint8_t* packed, uint32_t packed_bytes);
int      ldpc_hip_enc_cb_mode(const ldpc_hip_enc_queue* queue);      /* get_cb_mode()     */
uint32_t ldpc_hip_enc_max_tb_size(const ldpc_hip_enc_queue* queue);  /* get_max_tb_size() */

/* ---- introspection (tests / benchmarks) -------------------------------------------------------------------- */
/* Number of sequential layer groups the schedule uses for (bg, Z) with all layers active (row groups whose rows
 * share no variable node run concurrently; bit-identical to the layer-serial order). */
int ldpc_hip_schedule_groups(int bg, uint32_t lifting_size);
/* 1 when a specialised kernel (compile-time schedule, ldpc_spec.h) exists for (bg, Z), 0 when (bg, Z) has only the
 * generic one, LDPC_HIP_EINVAL for an invalid pair. A context opened with LDPC_HIP_LAUNCH_NO_SPEC uses the generic
 * kernel whatever this reports. */
int ldpc_hip_specialised(int bg, uint32_t lifting_size);
const char* ldpc_hip_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_LDPC_HIP_H */
