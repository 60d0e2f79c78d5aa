/*
 * Host runtime behind the C ABI of include/srsran_ldpc_hip.h: context (device, stream, graph schedules, CRC tables,
 * HBM HARQ arena), batched decode plans, synchronous decoder/dematcher entry points and the HAL operation queue
 * (hw_accelerator_pusch_dec semantics, include/srsran/hal/phy/upper/channel_processors/pusch/
 * hw_accelerator_pusch_dec.h:83-115; caller flow pusch_decoder_hw_impl.cpp:132-410).
 */
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "ldpc_graph.h"
#include "ldpc_hip_buffers.h"
#include "ldpc_hip_device.h"
#include "ldpc_hip_dwq.h"
#include "srsran_ldpc_hip.h"

namespace ldpc_hip {
hipError_t launch_decode(bool sf08, int spec, const dec_cb* d_cbs, uint32_t n, int graph_slot,
                         const step_task* tasks, const lds_layout& lay, int block, const int8_t* llr, uint8_t* out,
                         ldpc_hip_cb_result* res, const uint32_t* d_crc, hipStream_t stream,
                         const dec_cb* host_one = nullptr, const dematch_cb* d_dm = nullptr,
                         const dematch_cb* host_dm_one = nullptr, uint32_t dm_lds = 0);
hipError_t upload_graphs(const graph_desc* graphs, int n);
hipError_t write_split_tables(uint32_t* d_tables, const int* spec_ids, hipStream_t stream);
hipError_t launch_decode_mixed(bool sf08, const dec_cb* d_cbs, uint32_t n, const mixed_group* d_groups,
                               uint32_t ngroups, uint32_t lds_bytes, const step_task* tasks, const int8_t* llr,
                               uint8_t* out, ldpc_hip_cb_result* res, const uint32_t* d_crc, hipStream_t stream,
                               const dematch_cb* d_dm = nullptr, uint32_t dm_lds = 0);
hipError_t launch_encode(const enc_cb* d_cbs, uint32_t n, const uint8_t* msg, uint8_t* cw, const uint32_t* d_crc,
                         hipStream_t stream);
hipError_t launch_rate_match(const ratematch_cb* d_cbs, uint32_t n, const uint8_t* cw, uint8_t* out,
                             hipStream_t stream);
hipError_t launch_pdsch_encode(const pdsch_enc_cb* d_cbs, const pdsch_enc_cb* host_one, uint32_t n,
                               const uint8_t* msg, uint8_t* out, const uint32_t* d_crc, hipStream_t stream);
hipError_t launch_tb_join(const tbj_block* d_blocks, uint32_t nblocks, const uint8_t* msgs, ldpc_hip_cb_result* cb,
                          uint8_t* tb, ldpc_hip_tb_result* res, const uint32_t* d_crc, uint32_t* d_work,
                          hipStream_t stream);
hipError_t launch_dematch(const dematch_cb* d_cbs, uint32_t n, const demod_tables& tab, hipStream_t stream,
                          const dematch_cb* host_one = nullptr);
hipError_t configure_kernels(uint32_t max_lds);
hipError_t launch_demodulate(const demod_seg* d_segs, uint32_t nseg, uint32_t nblocks, const demod_tables& tab,
                             const float* d_sym, const float* d_nv, int8_t* d_llr, hipStream_t stream);
} // namespace ldpc_hip

using namespace ldpc_hip;

/* "auto" decoder type: the codeblock work (layer edges x Z x expected iterations, ldpc_hip_decode_work) from which a
 * decode call is faster on the GPU than on the host CPU. Measured on the GPU box (AMD EPYC 9575F, bench.py
 * extra.sw_route, profiles/r05/bench_a_line.json): a GPU call costs 21-22 us whatever the codeblock (PCIe and work-queue
 * round trips included), the CPU decoder port 12.2 us for C4's 6-layer BG1 Z=384 codeblocks with early stop (66 k
 * work) and 87.8 us for a full 8-iteration BG1 Z=384 codeblock without it (970 k); the crossover is ~150 k. */
constexpr uint64_t LDPC_HIP_AUTO_MIN_WORK_DEFAULT = 150000ULL;
/* iterations a decode with CRC early stop is expected to run (the C4 slot's mean is 1.8, C3's 1.14) */
constexpr uint64_t LDPC_HIP_AUTO_ET_ITERATIONS = 2ULL;

/* the C ABI's struct layouts are part of the contract (tests/test_abi.py checks the same sizes from Python) */
static_assert(sizeof(ldpc_hip_dec_desc) == 32, "ldpc_hip_dec_desc layout");
static_assert(sizeof(ldpc_hip_dematch_desc) == 20, "ldpc_hip_dematch_desc layout");
static_assert(sizeof(ldpc_hip_hw_config) == 44, "ldpc_hip_hw_config layout");
static_assert(sizeof(ldpc_hip_cb_result) == 4, "ldpc_hip_cb_result layout");
static_assert(sizeof(ldpc_hip_tb_desc) == 40, "ldpc_hip_tb_desc layout");
static_assert(sizeof(ldpc_hip_tb_result) == 4, "ldpc_hip_tb_result layout");
static_assert(sizeof(ldpc_hip_enc_desc) == 24, "ldpc_hip_enc_desc layout");
static_assert(sizeof(ldpc_hip_rm_desc) == 32, "ldpc_hip_rm_desc layout");
static_assert(sizeof(ldpc_hip_demod_desc) == 32, "ldpc_hip_demod_desc layout");

namespace {

constexpr uint32_t MAX_CB_LEN = 66U * 384U; /* MAX_CODEBLOCK_SIZE (ldpc.h:113) */
constexpr size_t   MAX_AUX_STREAMS = 3;       /* GPU_MAX_HW_QUEUES defaults to 4: the context stream + 3 */

/* The reference's demodulator tables, computed the way it computes them (float; demodulation_mapper_qam16.cpp:39,
 * demodulation_mapper_qam64.cpp:36-67, demodulation_mapper_qam256.cpp:37-160). */
demod_tables make_demod_tables()
{
  demod_tables t{};
  const float  s10 = 1.0F / std::sqrt(10.0F), s42 = 1.0F / std::sqrt(42.0F), s170 = 1.0F / std::sqrt(170.0F);
  t.s10            = s10;
  t.w64a           = 2 * s42;
  t.w64c           = 4 * s42;
  const int   k64[3][8] = {{16, 12, 8, 4, 4, 8, 12, 16}, {8, 4, 4, 8, -8, -4, -4, -8}, {4, -4, 4, -4, 0, 0, 0, 0}};
  const float n64[3][8] = {{24, 12, 4, 0, 0, -4, -12, -24}, {20, 8, 8, 12, 12, 8, 8, 20}, {12, -4, -4, 12, 0, 0, 0, 0}};
  for (int j = 0; j != 3; ++j) {
    for (int i = 0; i != 8; ++i) {
      t.sl64[j][i] = static_cast<float>(k64[j][i]) * s42;
      t.ic64[j][i] = n64[j][i] / 21;
    }
  }
  t.w256a                = 2 * s170;
  t.w256c                = 4 * s170;
  const int   k256[4][16] = {{32, 28, 24, 20, 16, 12, 8, 4, 4, 8, 12, 16, 20, 24, 28, 32},
                             {16, 12, 8, 4, 4, 8, 12, 16, -16, -12, -8, -4, -4, -8, -12, -16},
                             {8, 4, 4, 8, -8, -4, -4, -8, 8, 4, 4, 8, -8, -4, -4, -8},
                             {4, -4, 4, -4, 4, -4, 4, -4, 0, 0, 0, 0, 0, 0, 0, 0}};
  const float n256[4][16] = {{112, 84, 60, 40, 24, 12, 4, 0, 0, -4, -12, -24, -40, -60, -84, -112},
                             {88, 60, 36, 16, 16, 28, 36, 40, 40, 36, 28, 16, 16, 36, 60, 88},
                             {52, 24, 24, 44, -20, -8, -8, -12, -12, -8, -8, -20, 44, 24, 24, 52},
                             {28, -20, 12, -4, -4, 12, -20, 28, 0, 0, 0, 0, 0, 0, 0, 0}};
  for (int j = 0; j != 4; ++j) {
    for (int i = 0; i != 16; ++i) {
      t.sl256[j][i] = static_cast<float>(k256[j][i]) * s170;
      t.ic256[j][i] = n256[j][i] / 85;
    }
  }
  return t;
}

bool valid_modulation(int m) { return m == 0 || m == 1 || m == 2 || m == 4 || m == 6 || m == 8; }
unsigned bits_per_symbol(int m) { return (m == 0 || m == 1) ? 1U : static_cast<unsigned>(m); }

/* Descriptor upload of the *_launch entry points. A slot pipeline relaunches the same descriptors slot after slot,
 * and a host-to-device copy from pageable memory is performed synchronously by HIP (the host waits for the stream),
 * so an upload equal to the previous one into the same buffer, on the same stream, is skipped. */
struct desc_cache {
  std::vector<uint8_t> bytes;
  void*                ptr    = nullptr;
  hipStream_t          stream = nullptr;
};

hipError_t upload_descs(dev_buffer& buf, desc_cache& last, const void* src, size_t n, hipStream_t s)
{
  hipError_t e = buf.reserve(n);
  if (e != hipSuccess) {
    return e;
  }
  const auto* b = static_cast<const uint8_t*>(src);
  if (last.ptr == buf.ptr && last.stream == s && last.bytes.size() == n && std::memcmp(last.bytes.data(), b, n) == 0) {
    return hipSuccess;
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    return hipErrorStreamCaptureUnsupported; /* new descriptors inside a graph capture: launch once before capturing */
  }
  e = hipMemcpyAsync(buf.ptr, src, n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    last.bytes.assign(b, b + n);
    last.ptr    = buf.ptr;
    last.stream = s;
  } else {
    last = desc_cache{};
  }
  return e;
}

int graph_slot(int bg, unsigned Z)
{
  int pos = lifting_position(Z);
  if (pos < 0 || (bg != 1 && bg != 2)) {
    return -1;
  }
  return (bg - 1) * 51 + pos;
}

} // namespace

/* One operation of the HAL batch (hw_accelerator_pusch_dec configure + enqueue). */
struct hal_op {
  uint32_t           cb_index = 0;
  ldpc_hip_hw_config cfg{};
  uint32_t           N         = 0; /* codeblock length 66Z / 50Z                                   */
  uint32_t           msg_bytes = 0;
  uint64_t           llr_off   = 0; /* in the LLR staging arena (h_llr / q_llr)                    */
  uint64_t           soft_off  = 0; /* external HARQ: in the arena; otherwise in h_soft / q_soft    */
  uint64_t           out_off   = 0; /* in the message arena (h_out / q_out)                         */
  uint32_t           pos       = 0; /* decode position in the launched batch (result index)          */
  dwq*               q         = nullptr; /* the work queue running this op (a work-queue batch), else null */
  uint32_t           ticket    = 0;
  bool               dropped   = false;
  bool               dequeued  = false;
  ldpc_hip_cb_result res{};
};

/* failed: a launch failed after work was queued; the batch cannot be relaunched (its dematch may already have combined
 * into the HARQ soft buffers) and reads as an error until the queue is reserved or freed again. */
enum class hal_state { idle, staging, launched, failed };

/* The external HARQ buffer repository (ext_harq_buffer_context_repository.h:44-96) and the HBM it describes. One
 * atomic word per entry: bit 31 = entry in use (not empty), bits 0-30 = soft-data length.
 * caller_state (ldpc_hip_harq_device_memory): the device's HARQ memory only -- the caller keeps the entry state in its
 * own ext_harq_buffer_context_repository and decides drops (acc100's split: the repository holds the metadata, the
 * accelerator's HARQ memory the soft bits, bbdev_ldpc_decoder.cpp:146); then there is no state array and the arena
 * grows on demand (grow), under arena_mu: launches read the arena pointer under a shared lock, a growth takes it
 * exclusively and waits for the device before it moves the soft bits. */
struct ldpc_hip_harq_repo {
  static constexpr uint32_t IN_USE = 0x80000000U;
  static constexpr uint32_t MAX_CODEBLOCKS = 1U << 20;
  int                                    device         = 0;
  uint32_t                               nof_codeblocks = 0;
  bool                                   debug_mode     = false;
  bool                                   caller_state   = false;
  dev_buffer                             arena; /* nof_codeblocks x LDPC_HIP_HARQ_STRIDE int8 */
  std::unique_ptr<std::atomic<uint32_t>[]> state;
  std::atomic<int>                       refs{1};
  std::shared_mutex                      arena_mu;
  /* What may still use the arena's address after a batch has been issued: the work-queue items of HAL batches (a grid
   * may claim one after its batch's arena lock is gone), and the launch-path batches of every context attached to the
   * arena (each records its done event after its batch). grow() waits for exactly these, not for the whole device (a
   * hipDeviceSynchronize also waited for the persistent work-queue grids, up to their 50 ms lifetime). */
  std::mutex                             inflight_mu;
  std::vector<std::pair<dwq*, uint32_t>> inflight;
  std::vector<hipEvent_t>                user_events;

  void track_item(dwq* q, uint32_t ticket)
  {
    std::lock_guard<std::mutex> lock(inflight_mu);
    inflight.erase(std::remove_if(inflight.begin(), inflight.end(),
                                  [](const std::pair<dwq*, uint32_t>& it) { return dwq_done(it.first, it.second); }),
                   inflight.end());
    inflight.emplace_back(q, ticket);
  }
  void add_user(hipEvent_t ev)
  {
    std::lock_guard<std::mutex> lock(inflight_mu);
    user_events.push_back(ev);
  }
  void remove_user(hipEvent_t ev)
  {
    std::lock_guard<std::mutex> lock(inflight_mu);
    user_events.erase(std::remove(user_events.begin(), user_events.end(), ev), user_events.end());
  }
  /* with arena_mu held exclusively (no batch can be issued): every issued user of the arena has finished */
  hipError_t wait_users()
  {
    std::lock_guard<std::mutex> lock(inflight_mu);
    hipError_t                  e = hipSuccess;
    for (const auto& it : inflight) {
      /* a timed-out item is harmless only once its queue's grid has left (a stopped grid claims nothing); while the
       * grid is still resident the arena must not be freed: the error goes to the caller and the arena stays */
      if (dwq_wait(it.first, it.second) != hipSuccess && !dwq_quiesced(it.first)) {
        e = hipErrorLaunchTimeOut;
      }
    }
    if (e != hipSuccess) {
      return e;
    }
    inflight.clear();
    for (hipEvent_t ev : user_events) {
      const hipError_t r = hipEventSynchronize(ev);
      e                  = e == hipSuccess ? r : e;
    }
    return e;
  }

  int8_t* entry(uint32_t id) const { return arena.as<int8_t>() + static_cast<size_t>(id) * LDPC_HIP_HARQ_STRIDE; }
  /* caller_state memory: makes absolute_cb_id addressable (doubling, at least to the next multiple of 1024 entries).
   * Waits for every issued user of the arena first (wait_users): a batch already issued holds the old address. */
  hipError_t grow(uint32_t id)
  {
    {
      std::shared_lock<std::shared_mutex> rd(arena_mu);
      if (id < nof_codeblocks) {
        return hipSuccess;
      }
    }
    std::unique_lock<std::shared_mutex> wr(arena_mu);
    if (id < nof_codeblocks) {
      return hipSuccess;
    }
    if (id >= MAX_CODEBLOCKS) {
      return hipErrorInvalidValue;
    }
    const uint32_t n = std::min<uint32_t>(MAX_CODEBLOCKS, std::max<uint32_t>(2U * nof_codeblocks, (id + 1024U) & ~1023U));
    hipError_t     e = hipSetDevice(device);
    void*          p = nullptr;
    const size_t   old_bytes = static_cast<size_t>(nof_codeblocks) * LDPC_HIP_HARQ_STRIDE;
    const size_t   bytes     = static_cast<size_t>(n) * LDPC_HIP_HARQ_STRIDE;
    if (e == hipSuccess) {
      e = wait_users();
    }
    if (e == hipSuccess) {
      e = hipMalloc(&p, bytes);
    }
    if (e == hipSuccess && old_bytes != 0) {
      e = hipMemcpy(p, arena.ptr, old_bytes, hipMemcpyDeviceToDevice);
    }
    if (e == hipSuccess) {
      e = hipMemset(static_cast<int8_t*>(p) + old_bytes, 0, bytes - old_bytes);
    }
    if (e != hipSuccess) {
      if (p != nullptr) {
        (void)hipFree(p);
      }
      return e;
    }
    if (arena.ptr != nullptr) {
      (void)hipFree(arena.ptr);
    }
    arena.ptr      = p;
    arena.size     = bytes;
    nof_codeblocks = n;
    return hipSuccess;
  }
  /* get(absolute_codeblock_id, new_data), :69-83: a fresh entry (soft-data length 0) on new data or when empty;
   * returns the entry's soft-data length. */
  uint32_t get(uint32_t id, bool new_data)
  {
    uint32_t s = state[id].load(std::memory_order_acquire);
    if ((s & IN_USE) == 0 || new_data) {
      s = IN_USE;
      state[id].store(s, std::memory_order_release);
    }
    return s & ~IN_USE;
  }
  /* the soft-data length a completed decode leaves (acc100 reads it back at dequeue, acc100_impl.cpp:206-207) */
  void set_len(uint32_t id, uint32_t len) { state[id].store(IN_USE | len, std::memory_order_release); }
  /* free(absolute_codeblock_id), :86-96: kept in debug mode */
  void free(uint32_t id)
  {
    if (!debug_mode) {
      state[id].store(0U, std::memory_order_release);
    }
  }
  void release()
  {
    if (refs.fetch_sub(1, std::memory_order_acq_rel) == 1) {
      (void)hipSetDevice(device);
      delete this;
    }
  }
};

struct ldpc_hip_plan;

struct ldpc_hip_ctx {
  int                     device = 0;
  hipStream_t             stream = nullptr;
  hipEvent_t              done_event = nullptr;
  std::string             err;
  std::vector<graph_desc> graphs;      /* host copy, NOF_GRAPH_SLOTS entries: wide (BG1 then BG2, by lifting
                                          position), then the narrow schedules (NARROW_SLOT_BASE + slot) */
  int                     n_cu = 256;  /* compute units of the device */
  std::vector<uint8_t>    narrow_fits2 = std::vector<uint8_t>(102, 0); /* narrow schedule runs two CBs per CU */
  std::vector<uint8_t>    graph_valid;
  std::vector<uint8_t>    graph_spec; /* id + 1 of the specialised kernel (ldpc_spec.h) for this graph, 0: none */
  dev_buffer              d_crc;
  dev_buffer              d_tasks; /* step_task records of all graphs (ldpc_graph.cpp build_tasks) */
  dev_buffer              d_tbdesc; /* ldpc_hip_tb_join_launch descriptors */
  dev_buffer              d_dmdesc; /* ldpc_hip_rate_dematch_launch descriptors */
  dev_buffer              d_encdesc; /* ldpc_hip_encode_launch descriptors */
  dev_buffer              d_rmdesc;  /* ldpc_hip_rate_match_launch descriptors */
  dev_buffer              d_dmsegs;  /* ldpc_hip_demodulate_launch segments */
  desc_cache              c_dmdesc, c_encdesc, c_rmdesc, c_tbdesc, c_dmsegs, c_tbaux; /* last uploads (upload_descs) */
  dev_buffer              d_tbaux;   /* ldpc_hip_tb_join_launch: TB << 8 | chunk per workgroup */
  dev_buffer              d_tbwork;  /* ldpc_hip_tb_join_launch: per-TB chunk CRCs + arrival counter (zero at rest) */
  demod_tables            dtab{};    /* demodulator slopes / intercepts (make_demod_tables) */
  ldpc_hip_params         params{};
  /* fork/join of multi-group decode plans: groups after the first run on auxiliary streams (created on first use) */
  std::vector<hipStream_t> aux_streams;
  std::vector<hipEvent_t>  aux_events; /* [0]: fork point, [1 + i]: auxiliary stream i done */

  /* scratch for the synchronous entry points */
  dev_buffer d_llr, d_out, d_res, d_soft, d_desc, d_sym, d_nv;
  /* the one-codeblock software route (ldpc_decoder_hip::decode / ldpc_rate_dematcher_hip::rate_dematch, one call per
   * CB): pinned staging the kernel reads and writes in place (zero-copy), an event the caller spins on */
  pinned_buffer s_in, s_out;
  /* the one-CB decode's LLRs in device memory the host writes through the BAR (ldpc_hip_buffers.h bar_buffer), so the
   * kernel reads HBM; s_in serves when it cannot be had (bar_failed: not asked again) */
  bar_buffer    s_bar;
  bool          bar_failed = false;
  /* a one-CB work-queue wait timed out while the queue's grid stayed resident: it may still write s_in / s_out, so the
   * one-CB calls of this context refuse from then on (the context is to be closed) */
  bool          staging_lost = false;
  hipEvent_t    sync_event = nullptr;
  bool          sync_zc    = true; /* LDPC_HIP_SYNC_ZERO_COPY=0 (environment): the copy path, for A/B timing */
  /* the device work queues (ldpc_hip_dwq.h): workgroup size and body LDS of every queue key's persistent kernel */
  int      key_block[DWQ_KEYS] = {};
  uint32_t key_lds[DWQ_KEYS]   = {};
  bool     use_dwq                    = false;
  lds_layout spec_lay[102]            = {}; /* the specialised layout of each graph with a specialised body */

  /* HAL queue (ldpc_hip_enqueue / ldpc_hip_dequeue): staged operations of the current batch in pinned host memory,
   * moved with one copy per direction per batch */
  hal_state            hstate = hal_state::idle;
  std::vector<hal_op>  hops;  /* operations of the current batch, in enqueue order */
  std::vector<int32_t> hslot; /* cb_index -> index in hops, -1 when absent          */
  uint32_t             hdequeued = 0;
  pinned_buffer        h_llr, h_soft, h_out; /* h_llr: LLRs then descriptors; h_out: messages then results */
  dev_buffer           q_llr, q_soft, q_out;
  uint64_t             h_llr_used = 0, h_soft_used = 0, h_out_used = 0, h_res_off = 0;
  /* early copy (LDPC_HIP_LAUNCH_HAL_NO_EARLY_COPY off): h_llr[0, h_llr_copied) is already queued for q_llr on
   * hq_stream; hcopy: the current batch stages this way */
  uint64_t             h_llr_copied = 0;
  bool                 hcopy        = false;
  /* the early copy through the copy work queue (hal_copy_staged): its queue for this batch and its items' tickets */
  dwq*                  hcopy_q = nullptr;
  std::vector<uint32_t> hcopy_tickets;
  ldpc_hip_plan*       hplan = nullptr; /* the batch's decode plan (descriptors in q_llr after the LLRs); owned, see close */

  /* external HARQ: the repository this context's HAL queue keeps its soft buffers in (one reference held) */
  ldpc_hip_harq_repo* repo = nullptr;
  /* the HAL queue's stream: the context stream (dedicated queue), or one of the device's shared queues between
   * ldpc_hip_queue_reserve and ldpc_hip_queue_free (LDPC_HIP_LAUNCH_SHARED_QUEUE) */
  hipStream_t hq_stream = nullptr;
  int         hq_shared = -1; /* index of the borrowed shared queue, -1: none */
  bool        hbatch_done = false; /* the launched batch's event has been seen complete (later dequeues skip the query) */

  int fail(int code, const std::string& msg)
  {
    err = msg;
    return code;
  }
  int hip_fail(hipError_t e, const char* where)
  {
    err = std::string(where) + ": " + hipGetErrorString(e);
    return LDPC_HIP_EDEVICE;
  }
};

namespace {
void release_shared_queue(ldpc_hip_ctx* ctx); /* the HAL queue's borrowed shared stream back to the device's pool */
} // namespace

struct launch_group {
  int        slot;
  uint32_t   first;
  uint32_t   count;
  lds_layout lay;
  int        block;
  bool       sf08; /* scaling factor 0.8f: integer scaling path */
};

struct ldpc_hip_plan {
  ldpc_hip_ctx*             ctx = nullptr;
  uint32_t                  n   = 0;
  dev_buffer                d_cbs;
  std::vector<launch_group> groups;
  /* mixed launch (ldpc_decode_mixed_kernel): all groups in one launch when the plan fits the device at once */
  bool       mixed     = false;
  uint32_t   mixed_lds = 0;
  dev_buffer d_groups; /* mixed_group per launch group */
  /* the device descriptors launch_plan reads: d_cbs / d_groups, or a caller's buffer (the HAL batch's q_llr) */
  const dec_cb*      cbs_dev    = nullptr;
  const mixed_group* groups_dev = nullptr;
  /* a one-CB plan built on launch (the HAL batch): the descriptor also on the host, passed by value */
  bool   has_one = false;
  dec_cb one{};
  /* the device descriptors in block order on the host (block i decodes caller descriptor h_cbs[i].result_index), and
   * the fused dematcher's descriptors in the same order (ldpc_hip_dematch_decode_launch) */
  std::vector<dec_cb> h_cbs;
  dev_buffer          d_dm;
  desc_cache          c_dm;
};

namespace {

int validate_dec_desc(ldpc_hip_ctx* ctx, const ldpc_hip_dec_desc& d)
{
  const int slot = graph_slot(d.base_graph, d.lifting_size);
  if (slot < 0) {
    return ctx->fail(LDPC_HIP_EINVAL, "invalid base graph / lifting size");
  }
  const graph_desc& g  = ctx->graphs[slot];
  const unsigned    KZ = static_cast<unsigned>(g.K) * g.Z;
  if (d.max_iterations == 0) {
    return ctx->fail(LDPC_HIP_EINVAL, "Max iterations must be different to 0");
  }
  if (d.llr_length > static_cast<unsigned>(g.N_full - 2) * g.Z || d.llr_length < KZ + 2U * g.Z) {
    return ctx->fail(LDPC_HIP_EINVAL, "input length out of range [(K+2)Z, N_short Z]");
  }
  if (d.nof_filler_bits >= KZ) {
    return ctx->fail(LDPC_HIP_EINVAL, "invalid number of filler bits");
  }
  const unsigned crc_mode = d.crc_mode & ~LDPC_HIP_CRC_MODE_FLAG_KEEP_PASSED;
  if (crc_mode > LDPC_HIP_CRC_MODE_CHECK_AFTER) {
    return ctx->fail(LDPC_HIP_EINVAL, "invalid CRC mode");
  }
  if (crc_mode != LDPC_HIP_CRC_MODE_NONE && (d.crc_poly < 0 || d.crc_poly > 2)) {
    return ctx->fail(LDPC_HIP_EINVAL, "invalid CRC polynomial");
  }
  const float sf = (d.scaling_factor == 0.0f) ? 0.8f : d.scaling_factor;
  if (!(sf > 0.0f && sf < 1.0f)) {
    return ctx->fail(LDPC_HIP_EINVAL, "Scaling factor must be between 0 and 1 exclusively");
  }
  return LDPC_HIP_OK;
}

/* Host part of a decode plan: validates the descriptors, groups the CBs by (BG, Z, scaling path), picks the launch
 * form (specialised / generic, narrow schedules, one mixed launch) and fills the device descriptors `cbs` (group
 * order) and `mg` (mixed launch groups). Nothing touches the device. */
int plan_host(ldpc_hip_ctx* ctx, uint32_t n, const ldpc_hip_dec_desc* descs, ldpc_hip_plan& plan,
              std::vector<dec_cb>& cbs, std::vector<mixed_group>& mg)
{
  const uint32_t flags = ctx->params.launch_flags;
  plan.ctx             = ctx;
  plan.n               = n;
  plan.groups.clear();
  plan.mixed     = false;
  plan.mixed_lds = 0;
  mg.clear();
  std::vector<uint32_t> order(n);
  for (uint32_t i = 0; i != n; ++i) {
    int r = validate_dec_desc(ctx, descs[i]);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    order[i] = i;
  }
  /* launch groups: one kernel launch per (BG, Z, default-scaling) class */
  auto sf_of  = [](const ldpc_hip_dec_desc& s) { return (s.scaling_factor == 0.0f) ? 0.8f : s.scaling_factor; };
  auto key_of = [&](const ldpc_hip_dec_desc& s) {
    return 2 * graph_slot(s.base_graph, s.lifting_size) + (sf_of(s) == 0.8f ? 0 : 1);
  };
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return key_of(descs[a]) < key_of(descs[b]); });
  cbs.resize(n);
  for (uint32_t i = 0; i != n; ++i) {
    const ldpc_hip_dec_desc& s = descs[order[i]];
    dec_cb&                  d = cbs[i];
    d                          = dec_cb{};
    d.llr_offset               = s.llr_offset;
    d.out_offset               = s.out_offset;
    d.llr_length               = s.llr_length;
    d.result_index             = order[i];
    d.nof_filler_bits          = s.nof_filler_bits;
    d.max_iterations           = s.max_iterations;
    d.crc_mode                 = s.crc_mode & ~LDPC_HIP_CRC_MODE_FLAG_KEEP_PASSED;
    d.keep_passed              = (s.crc_mode & LDPC_HIP_CRC_MODE_FLAG_KEEP_PASSED) != 0 ? 1 : 0;
    d.crc_poly                 = (d.crc_mode == LDPC_HIP_CRC_MODE_NONE) ? 0 : s.crc_poly;
    d.scaling_factor           = sf_of(s);
    const int  slot            = graph_slot(s.base_graph, s.lifting_size);
    const bool sf08            = d.scaling_factor == 0.8f;
    if (plan.groups.empty() || plan.groups.back().slot != slot || plan.groups.back().sf08 != sf08) {
      const graph_desc& g = ctx->graphs[slot];
      /* the specialised kernels implement the default scaling factor only (integer round(0.8 m)) */
      const int spec = sf08 ? static_cast<int>(ctx->graph_spec[slot]) - 1 : -1;
      plan.groups.push_back({slot, i, 0, make_lds_layout(g, spec >= 0),
                             spec >= 0 ? 64 * spec_waves(spec) : decoder_block_size(g), sf08});
    }
    plan.groups.back().count++;
  }
  /* Large groups (more CBs than CUs) of a graph with a narrow schedule take it: two workgroups per CU. */
  for (launch_group& g : plan.groups) {
    const int  ns    = NARROW_SLOT_BASE + g.slot;
    const bool avail = !(g.sf08 && ctx->graph_spec[g.slot] != 0) && ctx->graph_valid[ns] != 0 &&
                       ctx->narrow_fits2[g.slot] != 0;
    const bool want  = (flags & LDPC_HIP_LAUNCH_NARROW_ALWAYS) != 0 ||
                      ((flags & LDPC_HIP_LAUNCH_NARROW_NEVER) == 0 && g.count > static_cast<uint32_t>(ctx->n_cu));
    if (avail && want) {
      g.slot  = ns;
      g.lay   = make_lds_layout(ctx->graphs[ns]);
      g.block = decoder_block_size(ctx->graphs[ns]);
    }
  }
  /* Mixed launch: several groups, one scaling path, every CB resident at once (at most one workgroup per CU with the
   * largest group's LDS) and every group's schedule within MIXED_BLOCK threads (a wider generic schedule takes its
   * narrow form). */
  plan.mixed = plan.groups.size() > 1 && n <= static_cast<uint32_t>(ctx->n_cu) &&
               (flags & LDPC_HIP_LAUNCH_NO_MIXED) == 0;
  for (launch_group& g : plan.groups) {
    if (!plan.mixed) {
      break;
    }
    int slot = g.slot;
    /* the mixed kernel carries the core specialised bodies only; a graph whose specialised kernel is standalone-only
     * runs the generic body there, and a generic schedule wider than the mixed block takes its narrow form */
    const int  sid  = (g.sf08 && slot < NARROW_SLOT_BASE) ? static_cast<int>(ctx->graph_spec[slot]) - 1 : -1;
    const bool spec = sid >= 0 && sid < spec_core_count();
    if (!spec && slot < NARROW_SLOT_BASE && decoder_block_size(ctx->graphs[slot]) > MIXED_BLOCK &&
        ctx->graph_valid[NARROW_SLOT_BASE + slot] != 0) {
      slot = NARROW_SLOT_BASE + slot;
    }
    const lds_layout lay  = make_lds_layout(ctx->graphs[slot], spec);
    const int block = spec ? 64 * spec_waves(sid) : decoder_block_size(ctx->graphs[slot]);
    if (block > MIXED_BLOCK || g.sf08 != plan.groups[0].sf08) {
      plan.mixed = false;
      break;
    }
    mixed_group m{};
    m.first_block  = g.first;
    m.graph_slot   = slot;
    m.task_offset  = ctx->graphs[slot].task_offset;
    m.spec         = spec ? static_cast<uint32_t>(sid + 1) : 0U; /* specialised kernel id + 1 */
    m.lay          = lay;
    mg.push_back(m);
    plan.mixed_lds = std::max(plan.mixed_lds, lay.total);
  }
  if (!plan.mixed) {
    mg.clear();
  }
  return LDPC_HIP_OK;
}

/* A plan that owns its device descriptors (ldpc_hip_decode_plan_create, ldpc_hip_decode_sync). */
int build_plan(ldpc_hip_ctx* ctx, uint32_t n, const ldpc_hip_dec_desc* descs, ldpc_hip_plan& plan)
{
  std::vector<dec_cb>      cbs;
  std::vector<mixed_group> mg;
  int                      r = plan_host(ctx, n, descs, plan, cbs, mg);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  hipError_t e = hipSuccess;
  if (!mg.empty()) {
    e = plan.d_groups.reserve(mg.size() * sizeof(mixed_group));
    if (e == hipSuccess) {
      e = hipMemcpy(plan.d_groups.ptr, mg.data(), mg.size() * sizeof(mixed_group), hipMemcpyHostToDevice);
    }
  }
  if (e == hipSuccess && n != 0) {
    e = plan.d_cbs.reserve(n * sizeof(dec_cb));
    if (e == hipSuccess) {
      e = hipMemcpy(plan.d_cbs.ptr, cbs.data(), n * sizeof(dec_cb), hipMemcpyHostToDevice);
    }
  }
  if (e != hipSuccess) {
    return ctx->hip_fail(e, "decode plan upload");
  }
  plan.cbs_dev    = plan.d_cbs.as<dec_cb>();
  plan.groups_dev = plan.d_groups.as<mixed_group>();
  plan.h_cbs      = std::move(cbs);
  return LDPC_HIP_OK;
}

/* d_dm (block order) / dm_one (a one-CB plan's descriptor by value): the fused rate dematcher in front of each CB's
 * decode (ldpc_dematch_body.h), writing the soft buffers the decode then reads; nullptr: decode only. */
int launch_plan(ldpc_hip_plan& plan, const int8_t* d_llr, uint8_t* d_out, ldpc_hip_cb_result* d_res,
                hipStream_t stream, const dematch_cb* d_dm = nullptr, const dematch_cb* dm_one = nullptr,
                uint32_t dm_lds = 0)
{
  ldpc_hip_ctx* ctx = plan.ctx;
  if (plan.mixed) {
    const hipError_t e = launch_decode_mixed(plan.groups[0].sf08, plan.cbs_dev, plan.n, plan.groups_dev,
                                             static_cast<uint32_t>(plan.groups.size()), plan.mixed_lds,
                                             ctx->d_tasks.as<step_task>(), d_llr, d_out, d_res,
                                             ctx->d_crc.as<uint32_t>(), stream, d_dm, dm_lds);
    return e == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(e, "ldpc_decode_mixed_kernel launch");
  }
  /* One launch per (BG, Z) group. Groups are independent (disjoint CBs, outputs and result slots), so with more than
   * one group (a mixed slot: the large-TB BG1 CBs beside the small-TB BG2 CBs) every group after the first runs on an
   * auxiliary stream forked from and joined back into `stream`: the groups share the GPU instead of queueing behind
   * each other. Stream order as seen by the caller is unchanged. */
  const size_t ng   = plan.groups.size();
  const size_t naux = std::min<size_t>(ng > 1 ? ng - 1 : 0, MAX_AUX_STREAMS);
  while (ctx->aux_streams.size() < naux) {
    hipStream_t s = nullptr;
    hipEvent_t  ev = nullptr;
    if (ctx->aux_events.empty()) {
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        return ctx->fail(LDPC_HIP_EDEVICE, "hipEventCreate(fork)");
      }
      ctx->aux_events.push_back(ev);
    }
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      return ctx->fail(LDPC_HIP_EDEVICE, "hipStreamCreate(aux)");
    }
    ctx->aux_streams.push_back(s);
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      return ctx->fail(LDPC_HIP_EDEVICE, "hipEventCreate(join)");
    }
    ctx->aux_events.push_back(ev);
  }
  hipError_t e = hipSuccess;
  if (naux != 0) {
    e = hipEventRecord(ctx->aux_events[0], stream);
    for (size_t i = 0; i != naux && e == hipSuccess; ++i) {
      e = hipStreamWaitEvent(ctx->aux_streams[i], ctx->aux_events[0], 0);
    }
    if (e != hipSuccess) {
      return ctx->hip_fail(e, "decode fork");
    }
  }
  for (size_t gi = 0; gi != ng; ++gi) {
    const launch_group& g  = plan.groups[gi];
    hipStream_t         gs = (gi == 0 || naux == 0) ? stream : ctx->aux_streams[(gi - 1) % naux];
    const int spec = (g.sf08 && g.slot < NARROW_SLOT_BASE) ? static_cast<int>(ctx->graph_spec[g.slot]) - 1 : -1;
    e = launch_decode(g.sf08, spec, plan.cbs_dev + g.first, g.count, g.slot,
                      ctx->d_tasks.as<step_task>() + ctx->graphs[g.slot].task_offset, g.lay, g.block, d_llr, d_out,
                      d_res, ctx->d_crc.as<uint32_t>(), gs, (plan.has_one && ng == 1) ? &plan.one : nullptr,
                      d_dm != nullptr ? d_dm + g.first : nullptr, (plan.has_one && ng == 1) ? dm_one : nullptr,
                      dm_lds);
    if (e != hipSuccess) {
      return ctx->hip_fail(e, "ldpc_decode_kernel launch");
    }
  }
  for (size_t i = 0; i != naux && e == hipSuccess; ++i) {
    e = hipEventRecord(ctx->aux_events[1 + i], ctx->aux_streams[i]);
    if (e == hipSuccess) {
      e = hipStreamWaitEvent(stream, ctx->aux_events[1 + i], 0);
    }
  }
  if (e != hipSuccess) {
    return ctx->hip_fail(e, "decode join");
  }
  return LDPC_HIP_OK;
}

/* The HIP stream an entry point's `stream` argument names: NULL the context's own stream; hipStreamLegacy
 * ((hipStream_t)1, the legacy default stream) the null stream, which is that stream to every runtime call; any other
 * handle (a stream, or hipStreamPerThread, which the runtime resolves itself) as given. Round 4 passed hipStreamLegacy
 * through unchanged, and a multi-group plan's fork (hipEventRecord / hipStreamWaitEvent on it) crashed in the runtime
 * (tools/ubench/stream_probe.hip). */
hipStream_t abi_stream(hipStream_t ctx_stream, void* stream)
{
  if (stream == nullptr) {
    return ctx_stream;
  }
  if (static_cast<hipStream_t>(stream) == hipStreamLegacy) {
    return nullptr;
  }
  return static_cast<hipStream_t>(stream);
}

unsigned msg_bytes_of(int bg, unsigned Z) { return ((bg == 1 ? 22U : 10U) * Z + 7U) / 8U; }

} // namespace

/* =============================================================================================================== */
extern "C" {

const char* ldpc_hip_version(void) { return "srsran_ldpc_hip 0.2 gfx950"; }

int ldpc_hip_harq_repo_create(int device, uint32_t nof_codeblocks, int debug_mode, ldpc_hip_harq_repo** out)
{
  if (out == nullptr || nof_codeblocks == 0 || nof_codeblocks > (1U << 20)) {
    return LDPC_HIP_EINVAL;
  }
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) {
    return LDPC_HIP_EDEVICE;
  }
  std::unique_ptr<ldpc_hip_harq_repo> r(new (std::nothrow) ldpc_hip_harq_repo());
  if (!r) {
    return LDPC_HIP_ENOMEM;
  }
  r->device         = device;
  r->nof_codeblocks = nof_codeblocks;
  r->debug_mode     = debug_mode != 0;
  r->state.reset(new (std::nothrow) std::atomic<uint32_t>[nof_codeblocks]);
  if (!r->state) {
    return LDPC_HIP_ENOMEM;
  }
  for (uint32_t i = 0; i != nof_codeblocks; ++i) {
    r->state[i].store(0U, std::memory_order_relaxed);
  }
  const size_t bytes = static_cast<size_t>(nof_codeblocks) * LDPC_HIP_HARQ_STRIDE;
  if (r->arena.reserve(bytes) != hipSuccess || hipMemset(r->arena.ptr, 0, bytes) != hipSuccess) {
    return LDPC_HIP_ENOMEM;
  }
  *out = r.release();
  return LDPC_HIP_OK;
}

int ldpc_hip_harq_repo_release(ldpc_hip_harq_repo* repo)
{
  if (repo == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  repo->release();
  return LDPC_HIP_OK;
}

int ldpc_hip_harq_device_memory(int device, ldpc_hip_harq_repo** out)
{
  if (out == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  *out = nullptr;
  static std::mutex                        mu;
  static std::map<int, ldpc_hip_harq_repo*> mems; /* one per device, alive for the process (one reference held) */
  std::lock_guard<std::mutex>              lock(mu);
  ldpc_hip_harq_repo*&                     m = mems[device];
  if (m == nullptr) {
    int dev_count = 0;
    if (hipGetDeviceCount(&dev_count) != hipSuccess || device < 0 || device >= dev_count) {
      return LDPC_HIP_EDEVICE;
    }
    std::unique_ptr<ldpc_hip_harq_repo> r(new (std::nothrow) ldpc_hip_harq_repo());
    if (!r) {
      return LDPC_HIP_ENOMEM;
    }
    r->device       = device;
    r->caller_state = true;
    const char* v   = std::getenv("LDPC_HIP_HARQ_CODEBLOCKS");
    const long  n   = v != nullptr ? std::atol(v) : 2048;
    if (n > 0 && r->grow(static_cast<uint32_t>(std::min<long>(n, ldpc_hip_harq_repo::MAX_CODEBLOCKS)) - 1U) !=
                     hipSuccess) {
      return LDPC_HIP_ENOMEM;
    }
    m = r.release();
  }
  m->refs.fetch_add(1, std::memory_order_acq_rel);
  *out = m;
  return LDPC_HIP_OK;
}

uint32_t ldpc_hip_harq_capacity(const ldpc_hip_harq_repo* repo)
{
  if (repo == nullptr) {
    return 0;
  }
  std::shared_lock<std::shared_mutex> lock(const_cast<ldpc_hip_harq_repo*>(repo)->arena_mu);
  return repo->nof_codeblocks;
}

int ldpc_hip_auto_device(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return -1;
  }
  const char* v   = std::getenv("LDPC_HIP_AUTO_DEVICE");
  const int   dev = v != nullptr ? std::atoi(v) : 0;
  if (dev < 0 || dev >= n) {
    return -1;
  }
  hipDeviceProp_t prop{};
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    (void)hipGetLastError();
    return -1; /* the kernels are built for gfx950 only */
  }
  return dev;
}

uint64_t ldpc_hip_decode_work(const ldpc_hip_dec_desc* d, const int8_t* llr)
{
  if (d == nullptr || (d->base_graph != 1 && d->base_graph != 2) || lifting_position(d->lifting_size) < 0 ||
      (d->llr_length != 0 && llr == nullptr)) {
    return 0;
  }
  const uint64_t Z = d->lifting_size;
  const uint64_t K = d->base_graph == 1 ? 22U : 10U;
  /* last non-zero LLR (ldpc_decoder_impl.cpp:97-101), scanned from the end eight bytes at a time */
  uint64_t last = d->llr_length;
  while (last >= 8) {
    uint64_t w;
    std::memcpy(&w, llr + last - 8, 8);
    if (w != 0) {
      break;
    }
    last -= 8;
  }
  while (last != 0 && llr[last - 1] == 0) {
    --last;
  }
  if (last == 0) {
    return 0;
  }
  /* codeblock length and layers (ldpc_decoder_impl.cpp:103-114) */
  uint64_t cb_len = std::max<uint64_t>(last + 2 * Z, (K + 4) * Z);
  cb_len          = (cb_len + Z - 1) / Z * Z;
  const unsigned nof_layers = static_cast<unsigned>(cb_len / Z - K);
  const uint64_t it         = (d->crc_mode & 0x0fU) == LDPC_HIP_CRC_MODE_EARLY_STOP
                                  ? std::min<uint64_t>(d->max_iterations, LDPC_HIP_AUTO_ET_ITERATIONS)
                                  : d->max_iterations;
  return static_cast<uint64_t>(layer_edges(d->base_graph, nof_layers)) * Z * it;
}

uint64_t ldpc_hip_auto_min_work(void)
{
  static const uint64_t v = [] {
    const char* e = std::getenv("LDPC_HIP_AUTO_MIN_WORK");
    return e != nullptr ? std::strtoull(e, nullptr, 10) : LDPC_HIP_AUTO_MIN_WORK_DEFAULT;
  }();
  return v;
}

int ldpc_hip_harq_repo_entry(const ldpc_hip_harq_repo* repo, uint32_t id, uint32_t* soft_data_len)
{
  if (repo == nullptr || id >= repo->nof_codeblocks) {
    return LDPC_HIP_EINVAL;
  }
  if (repo->caller_state) {
    return LDPC_HIP_ESTATE; /* the device's HARQ memory: the caller's repository holds the entry state */
  }
  const uint32_t s = repo->state[id].load(std::memory_order_acquire);
  if (soft_data_len != nullptr) {
    *soft_data_len = s & ~ldpc_hip_harq_repo::IN_USE;
  }
  return (s & ldpc_hip_harq_repo::IN_USE) != 0 ? 0 : 1;
}

int ldpc_hip_harq_repo_read(ldpc_hip_harq_repo* repo, uint32_t id, int8_t* dst, uint32_t len)
{
  if (repo == nullptr || len > LDPC_HIP_HARQ_STRIDE || (len != 0 && dst == nullptr)) {
    return LDPC_HIP_EINVAL;
  }
  std::shared_lock<std::shared_mutex> lock(repo->arena_mu);
  if (id >= repo->nof_codeblocks) {
    return LDPC_HIP_EINVAL;
  }
  (void)hipSetDevice(repo->device);
  return hipMemcpy(dst, repo->entry(id), len, hipMemcpyDeviceToHost) == hipSuccess ? LDPC_HIP_OK : LDPC_HIP_EDEVICE;
}

int ldpc_hip_open(int device, const ldpc_hip_params* params, ldpc_hip_ctx** out)
{
  return ldpc_hip_open_harq(device, params, nullptr, out);
}

int ldpc_hip_open_harq(int device, const ldpc_hip_params* params, ldpc_hip_harq_repo* repo, ldpc_hip_ctx** out)
{
  if (out == nullptr || (repo != nullptr && repo->device != device)) {
    return LDPC_HIP_EINVAL;
  }
  *out     = nullptr;
  auto ctx = std::make_unique<ldpc_hip_ctx>();
  if (params != nullptr) {
    ctx->params = *params;
  }
  if (ctx->params.max_queue_cbs == 0) {
    ctx->params.max_queue_cbs = 162; /* MAX_NOF_SEGMENTS (sch_constants.h:38) */
  }
  if (ctx->params.max_cb_llrs == 0) {
    ctx->params.max_cb_llrs = 4U * MAX_CB_LEN;
  }
  ctx->device  = device;
  ctx->dtab    = make_demod_tables();
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    return LDPC_HIP_EDEVICE;
  }
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->done_event, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->sync_event, hipEventDisableTiming) != hipSuccess) {
    return LDPC_HIP_EDEVICE;
  }
  ctx->hq_stream = ctx->stream;
  {
    const char* v = std::getenv("LDPC_HIP_SYNC_ZERO_COPY");
    ctx->sync_zc  = v == nullptr || std::strcmp(v, "0") != 0;
  }
  /* the one-CB staging of the software route: a whole codeblock's LLRs plus a 32 KiB rate-matched input */
  if (ctx->s_in.reserve(MAX_CB_LEN + 32768 + 16, 0) != hipSuccess || ctx->s_out.reserve(4096, 0) != hipSuccess) {
    return LDPC_HIP_ENOMEM;
  }
  ctx->bar_failed = ctx->s_bar.reserve(MAX_CB_LEN + 16) != hipSuccess; /* optional: s_in serves without it */
  (void)hipGetLastError();
  ctx->graphs.resize(NOF_GRAPH_SLOTS);
  ctx->graph_valid.assign(NOF_GRAPH_SLOTS, 0);
  if (hipDeviceGetAttribute(&ctx->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      ctx->n_cu <= 0) {
    ctx->n_cu = 256;
  }
  uint32_t max_lds = 0;
  for (int bg = 1; bg <= 2; ++bg) {
    for (int p = 0; p != 51; ++p) {
      const int slot = (bg - 1) * 51 + p;
      if (build_graph(bg, k_lifting_sizes[p], ctx->graphs[slot])) {
        ctx->graph_valid[slot] = 1;
        max_lds                = std::max({max_lds, make_lds_layout(ctx->graphs[slot]).total,
                                           make_lds_layout(ctx->graphs[slot], true).total});
      }
    }
  }
  std::vector<step_task> tasks;
  for (int slot = 0; slot != 102; ++slot) {
    if (ctx->graph_valid[slot]) {
      build_tasks(ctx->graphs[slot], tasks);
    }
  }
  /* Narrow schedules: at most NARROW_WAVES waves per workgroup, so that two workgroups share a CU (LDS and the
   * generic kernel's <= 128 VGPRs permitting). A batch of many more CBs than CUs then keeps two CBs in flight per CU,
   * each hiding the other's step latency, instead of running them one after the other. */
  for (int slot = 0; slot != 102; ++slot) {
    if (!ctx->graph_valid[slot]) {
      continue;
    }
    graph_desc& n = ctx->graphs[NARROW_SLOT_BASE + slot];
    n             = ctx->graphs[slot];
    build_tasks(n, tasks, NARROW_WAVES);
    /* valid: narrower than the wide schedule (also used to fit a mixed launch's workgroup); narrow_fits2: two
     * workgroups fit a CU's LDS (the large-batch rule) */
    ctx->graph_valid[NARROW_SLOT_BASE + slot] = (n.task_waves < ctx->graphs[slot].task_waves) ? 1 : 0;
    ctx->narrow_fits2[slot] = (2U * make_lds_layout(n).total <= 160U * 1024U) ? 1 : 0;
  }
  /* specialised kernel where its compile-time schedule equals build_graph's (LDPC_HIP_LAUNCH_NO_SPEC disables it) */
  ctx->graph_spec.assign(NOF_GRAPH_SLOTS, 0);
  for (int slot = 0; slot != 102; ++slot) {
    if (ctx->graph_valid[slot] && (ctx->params.launch_flags & LDPC_HIP_LAUNCH_NO_SPEC) == 0) {
      ctx->graph_spec[slot] = static_cast<uint8_t>(spec_index(ctx->graphs[slot], make_lds_layout(ctx->graphs[slot], true)) + 1);
    }
  }
  /* the work queues' kernels: per specialised graph, its body's width and layout (at least the fused dematcher's
   * staging); the dematch-only kernel's */
  ctx->use_dwq = dwq_enabled() && (ctx->params.launch_flags & (LDPC_HIP_LAUNCH_NO_DWQ | LDPC_HIP_LAUNCH_NO_SPEC)) == 0;
  for (int slot = 0; slot != 102; ++slot) {
    const int id = static_cast<int>(ctx->graph_spec[slot]) - 1;
    if (id < 0) {
      continue;
    }
    ctx->spec_lay[slot]    = make_lds_layout(ctx->graphs[slot], true);
    ctx->key_block[1 + id] = 64 * spec_waves(id);
    ctx->key_lds[1 + id]   = std::max(ctx->spec_lay[slot].total, DM_FUSED_LDS);
  }
  ctx->key_block[0] = DM_THREADS;
  ctx->key_lds[0]   = DM_FUSED_LDS;
  if (ctx->d_tasks.reserve(tasks.size() * sizeof(step_task)) != hipSuccess ||
      hipMemcpy(ctx->d_tasks.ptr, tasks.data(), tasks.size() * sizeof(step_task), hipMemcpyHostToDevice) !=
          hipSuccess) {
    return LDPC_HIP_EDEVICE;
  }
  {
    /* the graph table in constant memory and the kernels' LDS limit are per process and device: set once, so that a
     * context opened while another context's kernels run on the device does not rewrite them under those kernels */
    static std::mutex    once_mutex;
    static std::set<int> done;
    std::lock_guard<std::mutex> lock(once_mutex);
    if (done.count(device) == 0) {
      if (upload_graphs(ctx->graphs.data(), NOF_GRAPH_SLOTS) != hipSuccess || configure_kernels(max_lds) != hipSuccess) {
        return LDPC_HIP_EDEVICE;
      }
      done.insert(device);
    }
  }
  std::vector<uint32_t> crc = build_crc_tables();
  static_assert(sizeof(demod_tables) <= DTAB_WORDS * 4U, "DTAB_WORDS");
  std::memcpy(crc.data() + DTAB_OFFSET, &ctx->dtab, sizeof(demod_tables)); /* the fused dematcher's tables */
  if (ctx->d_crc.reserve(crc.size() * 4) != hipSuccess ||
      hipMemcpy(ctx->d_crc.ptr, crc.data(), crc.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    return LDPC_HIP_EDEVICE;
  }
  {
    /* the specialised BG1 kernels' split-row address tables, after the CRC tables (SPLIT_TAB_OFFSET) */
    int spec_ids[51];
    for (int p = 0; p != 51; ++p) {
      spec_ids[p] = ctx->graph_valid[p] ? spec_index(ctx->graphs[p], make_lds_layout(ctx->graphs[p], true)) : -1;
    }
    if (write_split_tables(ctx->d_crc.as<uint32_t>(), spec_ids, ctx->stream) != hipSuccess) {
      return LDPC_HIP_EDEVICE;
    }
  }
  if (repo != nullptr) {
    repo->refs.fetch_add(1, std::memory_order_acq_rel);
    ctx->repo = repo;
  } else if (ctx->params.nof_harq_slots != 0) {
    /* a private repository (the context's own external HARQ memory) */
    const int r = ldpc_hip_harq_repo_create(device, ctx->params.nof_harq_slots, 0, &ctx->repo);
    if (r != LDPC_HIP_OK) {
      return r;
    }
  }
  if (ctx->repo != nullptr) {
    ctx->repo->add_user(ctx->done_event); /* grow() waits for this context's issued HAL batches */
  }
  *out = ctx.release();
  return LDPC_HIP_OK;
}

} /* extern "C" */
namespace {
void hal_sync(ldpc_hip_ctx* ctx);
}
extern "C" {

int ldpc_hip_close(ldpc_hip_ctx* ctx)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  (void)hipSetDevice(ctx->device);
  /* a HAL batch still in flight (work-queue items included) reads and writes this context's pinned buffers */
  hal_sync(ctx);
  if (ctx->stream != nullptr) {
    (void)hipStreamSynchronize(ctx->stream);
  }
  if (ctx->repo != nullptr) {
    ctx->repo->remove_user(ctx->done_event);
  }
  if (ctx->hq_shared >= 0) {
    (void)hipStreamSynchronize(ctx->hq_stream);
    release_shared_queue(ctx);
  }
  delete ctx->hplan;
  ctx->hplan = nullptr;
  if (ctx->done_event != nullptr) {
    (void)hipEventDestroy(ctx->done_event);
  }
  if (ctx->sync_event != nullptr) {
    (void)hipEventDestroy(ctx->sync_event);
  }
  for (hipStream_t a : ctx->aux_streams) {
    (void)hipStreamSynchronize(a);
    (void)hipStreamDestroy(a);
  }
  for (hipEvent_t ev : ctx->aux_events) {
    (void)hipEventDestroy(ev);
  }
  hipStream_t         s    = ctx->stream;
  ldpc_hip_harq_repo* repo = ctx->repo;
  delete ctx;
  if (s != nullptr) {
    (void)hipStreamDestroy(s);
  }
  if (repo != nullptr) {
    repo->release();
  }
  return LDPC_HIP_OK;
}

const char* ldpc_hip_last_error(const ldpc_hip_ctx* ctx) { return ctx == nullptr ? "null context" : ctx->err.c_str(); }

struct ldpc_hip_graph {
  ldpc_hip_ctx*  ctx   = nullptr;
  hipGraph_t     graph = nullptr;
  hipGraphExec_t exec  = nullptr;
};

int ldpc_hip_capture_begin(ldpc_hip_ctx* ctx, void* stream)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t      s = abi_stream(ctx->stream, stream);
  if (s == nullptr || s == hipStreamPerThread) {
    return ctx->fail(LDPC_HIP_EINVAL, "a default stream cannot be captured"); /* hipStreamBeginCapture refuses it */
  }
  const hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
  return e == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(e, "hipStreamBeginCapture");
}

int ldpc_hip_capture_end(ldpc_hip_ctx* ctx, void* stream, ldpc_hip_graph** out)
{
  if (ctx == nullptr || out == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  *out          = nullptr;
  hipStream_t s = abi_stream(ctx->stream, stream);
  auto        g = std::make_unique<ldpc_hip_graph>();
  g->ctx        = ctx;
  hipError_t e  = hipStreamEndCapture(s, &g->graph);
  if (e == hipSuccess) {
    e = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
  }
  if (e != hipSuccess) {
    if (g->graph != nullptr) {
      (void)hipGraphDestroy(g->graph);
    }
    return ctx->hip_fail(e, "graph capture");
  }
  *out = g.release();
  return LDPC_HIP_OK;
}

int ldpc_hip_graph_launch(ldpc_hip_graph* g, void* stream)
{
  if (g == nullptr || g->exec == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  hipStream_t      s = abi_stream(g->ctx->stream, stream);
  const hipError_t e = hipGraphLaunch(g->exec, s);
  return e == hipSuccess ? LDPC_HIP_OK : g->ctx->hip_fail(e, "hipGraphLaunch");
}

int ldpc_hip_graph_destroy(ldpc_hip_graph* g)
{
  if (g == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (g->exec != nullptr) {
    (void)hipGraphExecDestroy(g->exec);
  }
  if (g->graph != nullptr) {
    (void)hipGraphDestroy(g->graph);
  }
  delete g;
  return LDPC_HIP_OK;
}

void* ldpc_hip_stream(ldpc_hip_ctx* ctx) { return ctx == nullptr ? nullptr : static_cast<void*>(ctx->stream); }

int ldpc_hip_schedule_groups(int bg, uint32_t lifting_size)
{
  graph_desc g;
  if (!build_graph(bg, lifting_size, g)) {
    return LDPC_HIP_EINVAL;
  }
  return g.n_groups;
}

int ldpc_hip_specialised(int bg, uint32_t lifting_size)
{
  graph_desc g;
  if (!build_graph(bg, lifting_size, g)) {
    return LDPC_HIP_EINVAL;
  }
  return spec_index(g, make_lds_layout(g, true)) >= 0 ? 1 : 0;
}

/* ---- plans ---- */
int ldpc_hip_decode_plan_create(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dec_desc* descs,
                                ldpc_hip_plan** plan)
{
  if (ctx == nullptr || plan == nullptr || (nof_cbs != 0 && descs == nullptr)) {
    return LDPC_HIP_EINVAL;
  }
  *plan  = nullptr;
  auto p = std::make_unique<ldpc_hip_plan>();
  (void)hipSetDevice(ctx->device);
  int r = build_plan(ctx, nof_cbs, descs, *p);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  *plan = p.release();
  return LDPC_HIP_OK;
}

int ldpc_hip_decode_plan_destroy(ldpc_hip_plan* plan)
{
  delete plan;
  return LDPC_HIP_OK;
}

int ldpc_hip_decode_launch(ldpc_hip_plan* plan, const int8_t* d_llr, uint8_t* d_out, ldpc_hip_cb_result* d_results,
                           void* stream)
{
  if (plan == nullptr || (plan->n != 0 && (d_llr == nullptr || d_out == nullptr))) {
    return LDPC_HIP_EINVAL;
  }
  hipStream_t s = abi_stream(plan->ctx->stream, stream);
  return launch_plan(*plan, d_llr, d_out, d_results, s);
}

static int validate_dematch(ldpc_hip_ctx* ctx, const ldpc_hip_dematch_desc& d);

int ldpc_hip_rate_dematch_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dematch_desc* descs,
                                 const int8_t* d_llr, const uint64_t* llr_offsets, int8_t* d_soft,
                                 const uint64_t* soft_offsets, void* stream)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_cbs == 0) {
    return LDPC_HIP_OK;
  }
  if (descs == nullptr || d_llr == nullptr || llr_offsets == nullptr || d_soft == nullptr || soft_offsets == nullptr) {
    return ctx->fail(LDPC_HIP_EINVAL, "rate_dematch_launch: null argument");
  }
  std::vector<dematch_cb> dm(nof_cbs);
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    const int r = validate_dematch(ctx, descs[i]);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    const ldpc_hip_dematch_desc& s = descs[i];
    dm[i]                          = dematch_cb{};
    dm[i].llr                      = d_llr + llr_offsets[i];
    dm[i].soft                     = d_soft + soft_offsets[i];
    dm[i].cb_length                = s.cb_length;
    dm[i].rm_length                = s.rm_length;
    dm[i].Nref                     = s.Nref;
    dm[i].nof_filler_bits          = s.nof_filler_bits;
    dm[i].modulation_order         = s.modulation_order;
    dm[i].rv                       = s.rv;
    dm[i].new_data                 = s.new_data;
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = abi_stream(ctx->stream, stream);
  hipError_t  e = upload_descs(ctx->d_dmdesc, ctx->c_dmdesc, dm.data(), nof_cbs * sizeof(dematch_cb), s);
  if (e == hipSuccess) {
    e = launch_dematch(ctx->d_dmdesc.as<dematch_cb>(), nof_cbs, ctx->dtab, s);
  }
  return e == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(e, "ldpc_rate_dematch_kernel launch");
}

int ldpc_hip_demod_dematch_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dematch_desc* descs,
                                  const ldpc_hip_demod_desc* demod, const float* d_symbols,
                                  const float* d_noise_vars, int8_t* d_soft, const uint64_t* soft_offsets,
                                  void* stream)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_cbs == 0) {
    return LDPC_HIP_OK;
  }
  if (descs == nullptr || demod == nullptr || d_symbols == nullptr || d_noise_vars == nullptr || d_soft == nullptr ||
      soft_offsets == nullptr) {
    return ctx->fail(LDPC_HIP_EINVAL, "demod_dematch_launch: null argument");
  }
  std::vector<dematch_cb> dm(nof_cbs);
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    const int r = validate_dematch(ctx, descs[i]);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    const ldpc_hip_dematch_desc& s = descs[i];
    const ldpc_hip_demod_desc&   m = demod[i];
    if (!valid_modulation(m.modulation) || bits_per_symbol(m.modulation) != s.modulation_order ||
        static_cast<uint64_t>(m.nof_symbols) * s.modulation_order != s.rm_length) {
      return ctx->fail(LDPC_HIP_EINVAL, "demod_dematch_launch: symbols x bits per symbol must equal rm_length");
    }
    if (s.rm_length > DM_STAGE) {
      return ctx->fail(LDPC_HIP_EINVAL, "demod_dematch_launch: rm_length above 32768 (use demodulate + dematch)");
    }
    dm[i]                  = dematch_cb{};
    dm[i].soft             = d_soft + soft_offsets[i];
    dm[i].sym              = d_symbols + 2 * m.symbol_offset;
    dm[i].nv               = d_noise_vars + m.noise_offset;
    dm[i].demod            = m.modulation;
    dm[i].cb_length        = s.cb_length;
    dm[i].rm_length        = s.rm_length;
    dm[i].Nref             = s.Nref;
    dm[i].nof_filler_bits  = s.nof_filler_bits;
    dm[i].modulation_order = s.modulation_order;
    dm[i].rv               = s.rv;
    dm[i].new_data         = s.new_data;
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = abi_stream(ctx->stream, stream);
  hipError_t  e = upload_descs(ctx->d_dmdesc, ctx->c_dmdesc, dm.data(), nof_cbs * sizeof(dematch_cb), s);
  if (e == hipSuccess) {
    e = launch_dematch(ctx->d_dmdesc.as<dematch_cb>(), nof_cbs, ctx->dtab, s);
  }
  return e == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(e, "ldpc_rate_dematch_kernel launch (demodulating)");
}

#ifdef LDPC_HIP_DIAG_CB
/* diagnostic build only: the decoder's per-workgroup phase stamps (tools/diag_cb.py) */
int ldpc_hip_diag_cb_read(ldpc_hip_ctx* ctx, uint64_t* out, uint32_t n)
{
  if (ctx == nullptr || n > DIAG_CB_WORDS / 2) {
    return LDPC_HIP_EINVAL;
  }
  (void)hipSetDevice(ctx->device);
  return hipMemcpy(out, ctx->d_crc.as<uint32_t>() + DIAG_CB_OFFSET, n * sizeof(uint64_t), hipMemcpyDeviceToHost) ==
                 hipSuccess ? LDPC_HIP_OK : LDPC_HIP_EDEVICE;
}
#endif

int ldpc_hip_dematch_decode_launch(ldpc_hip_plan* plan, const ldpc_hip_dematch_desc* descs, const int8_t* d_llr,
                                   const uint64_t* llr_offsets, const ldpc_hip_demod_desc* demod,
                                   const float* d_symbols, const float* d_noise_vars, int8_t* d_soft, uint8_t* d_out,
                                   ldpc_hip_cb_result* d_results, void* stream)
{
  if (plan == nullptr || plan->ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  ldpc_hip_ctx* ctx = plan->ctx;
  if (plan->n == 0) {
    return LDPC_HIP_OK;
  }
  if (descs == nullptr || d_soft == nullptr || d_out == nullptr || plan->h_cbs.size() != plan->n ||
      (demod == nullptr && (d_llr == nullptr || llr_offsets == nullptr)) ||
      (demod != nullptr && (d_symbols == nullptr || d_noise_vars == nullptr))) {
    return ctx->fail(LDPC_HIP_EINVAL, "dematch_decode_launch: null argument");
  }
  std::vector<dematch_cb> dm(plan->n); /* block order: block i dematches caller descriptor h_cbs[i].result_index */
  for (uint32_t i = 0; i != plan->n; ++i) {
    const uint32_t               k = plan->h_cbs[i].result_index;
    const ldpc_hip_dematch_desc& s = descs[k];
    const int                    r = validate_dematch(ctx, s);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    /* the dematcher writes cb_length soft bits at the decode descriptor's offset, inside the workgroup that then
     * decodes them: a length or filler mismatch would write into a neighbour's buffer while it is being decoded */
    if (s.cb_length != plan->h_cbs[i].llr_length || s.nof_filler_bits != plan->h_cbs[i].nof_filler_bits) {
      return ctx->fail(LDPC_HIP_EINVAL, "dematch_decode_launch: dematch descriptor does not match its codeblock "
                                        "(cb_length != llr_length or filler bits differ)");
    }
    dematch_cb& d = dm[i];
    d             = dematch_cb{};
    if (demod != nullptr) {
      const ldpc_hip_demod_desc& m = demod[k];
      if (!valid_modulation(m.modulation) || bits_per_symbol(m.modulation) != s.modulation_order ||
          static_cast<uint64_t>(m.nof_symbols) * s.modulation_order != s.rm_length || s.rm_length > DM_STAGE) {
        return ctx->fail(LDPC_HIP_EINVAL, "dematch_decode_launch: symbols x bits per symbol must equal rm_length "
                                          "<= 32768");
      }
      d.sym   = d_symbols + 2 * m.symbol_offset;
      d.nv    = d_noise_vars + m.noise_offset;
      d.demod = m.modulation;
    } else {
      d.llr = d_llr + llr_offsets[k];
    }
    d.soft             = d_soft + plan->h_cbs[i].llr_offset;
    d.cb_length        = s.cb_length;
    d.rm_length        = s.rm_length;
    d.Nref             = s.Nref;
    d.nof_filler_bits  = s.nof_filler_bits;
    d.modulation_order = s.modulation_order;
    d.rv               = s.rv;
    d.new_data         = s.new_data;
  }
  (void)hipSetDevice(ctx->device);
  const uint32_t   dm_lds = dm_fused_budget(dm.data(), dm.size());
  hipStream_t      hs = abi_stream(ctx->stream, stream);
  const hipError_t e  = upload_descs(plan->d_dm, plan->c_dm, dm.data(), dm.size() * sizeof(dematch_cb), hs);
  if (e != hipSuccess) {
    return ctx->hip_fail(e, "dematch_decode_launch: descriptors");
  }
  return launch_plan(*plan, d_soft, d_out, d_results, hs, plan->d_dm.as<dematch_cb>(), nullptr, dm_lds);
}

} /* extern "C" */
namespace ldpc_hip {
/* an encoder work item from its C-ABI descriptor and (ext) message bit offset, data bits and CRC position; the
 * reason it is invalid, or nullptr */
const char* make_enc_cb(const ldpc_hip_ctx* ctx, const ldpc_hip_enc_desc& d, const uint32_t* ext, enc_cb& out)
{
  const int slot = graph_slot(d.base_graph, d.lifting_size);
  if (slot < 0) {
    return "encode_launch: invalid base graph / lifting size";
  }
  const graph_desc& g  = ctx->graphs[slot];
  const uint32_t    KZ = static_cast<uint32_t>(g.K) * g.Z;
  if (d.cw_length == 0 || d.cw_length > static_cast<uint32_t>(g.N_full - 2) * g.Z) {
    return "encode_launch: codeword length out of range";
  }
  const uint32_t bit_off = ext != nullptr ? ext[0] : 0U;
  const uint32_t data    = ext != nullptr ? ext[1] : KZ;
  const uint32_t crc_at  = ext != nullptr ? ext[2] : 0U;
  if (bit_off > 7 || data > KZ || (crc_at != 0 && (crc_at + 24 > KZ || data > crc_at))) {
    return "encode_launch: message bit range out of range";
  }
  out = enc_cb{d.msg_offset, d.cw_offset, d.cw_length, slot, bit_off, data, crc_at, 0};
  return nullptr;
}

/* a rate-matcher work item from its C-ABI descriptor (ldpc_rate_matcher_impl.cpp:36-160); the reason it is invalid,
 * or nullptr */
const char* make_rm_cb(const ldpc_hip_rm_desc& d, ratematch_cb& out)
{
  static const uint32_t sf_bg1[4] = {0, 17, 33, 56}, sf_bg2[4] = {0, 13, 25, 43}; /* ldpc_rate_matcher_impl.cpp:33-34 */
  const unsigned        N         = d.cb_length;
  const bool            bg1       = (N % 66U) == 0;
  if (!bg1 && (N % 50U) != 0) {
    return "rate_match_launch: invalid codeblock length";
  }
  const unsigned Z = bg1 ? N / 66U : N / 50U;
  if (graph_slot(bg1 ? 1 : 2, Z) < 0 || d.rv > 3 || d.modulation_order == 0 || d.modulation_order > 8 ||
      d.rm_length == 0 || d.rm_length % d.modulation_order != 0) {
    return "rate_match_launch: invalid parameters";
  }
  const unsigned nsys = ((bg1 ? 22U : 10U) - 2U) * Z;
  if (d.nof_filler_bits >= nsys) {
    return "rate_match_launch: invalid number of filler bits";
  }
  const unsigned Ncb = (d.Nref > 0) ? std::min<unsigned>(d.Nref, N) : N;
  const uint64_t sf  = bg1 ? sf_bg1[d.rv] : sf_bg2[d.rv];
  out                = ratematch_cb{};
  out.cw_offset      = d.cw_offset;
  out.out_offset     = d.out_offset;
  out.cb_length      = N;
  out.rm_length      = d.rm_length;
  out.Ncb            = Ncb;
  out.k0             = static_cast<uint32_t>((sf * Ncb) / N) * Z; /* :88-89, floor of an exact ratio */
  out.fill_lo        = nsys - d.nof_filler_bits;
  out.fill_hi        = nsys;
  out.Qm             = d.modulation_order;
  return nullptr;
}

size_t pdsch_enc_desc_bytes() { return sizeof(pdsch_enc_cb); }

const char* make_pdsch_cb(const ldpc_hip_ctx* ctx, const ldpc_hip_enc_desc& ed, const uint32_t* ext,
                          const ldpc_hip_rm_desc& rd, pdsch_enc_cb& c)
{
  const char* why = make_enc_cb(ctx, ed, ext, c.enc);
  if (why == nullptr) {
    why = make_rm_cb(rd, c.rm);
  }
  if (why == nullptr &&
      (c.enc.cw_length != c.rm.cb_length ||
       c.enc.graph_slot != graph_slot(rd.cb_length % 66U == 0 ? 1 : 2, ed.lifting_size))) {
    why = "pdsch_encode: encoder and rate matcher descriptors disagree";
  }
  return why;
}

/* A small PDSCH batch as items of the encoder's work queue (ldpc_hip_dwq.h DWQ_KEY_ENC; ldpc_dwq_encode_kernel) instead
 * of a launch: every codeblock validated first, then one item each, tickets[i] its ticket (0xffffffff when not
 * published). Returns LDPC_HIP_OK with *qo set, 1 when the queue cannot serve the batch now (nothing published: launch
 * instead), or an error after which the published items must still be waited for (pdsch_encode_wait). */
int pdsch_encode_submit(ldpc_hip_ctx* ctx, uint32_t n, const ldpc_hip_enc_desc* ed, const uint32_t* ext,
                        const ldpc_hip_rm_desc* rd, const uint8_t* d_msgs, uint8_t* d_out, void** qo,
                        uint32_t* tickets)
{
  *qo = nullptr;
  if (ctx == nullptr || n == 0 || !ctx->use_dwq) {
    return 1;
  }
  std::vector<pdsch_enc_cb> c(n);
  for (uint32_t i = 0; i != n; ++i) {
    tickets[i] = 0xffffffffU;
    if (const char* why = make_pdsch_cb(ctx, ed[i], ext + 3 * i, rd[i], c[i])) {
      return ctx->fail(LDPC_HIP_EINVAL, why);
    }
  }
  dwq* q = dwq_get(ctx->device, DWQ_KEY_ENC, ENC_THREADS, 0);
  if (q == nullptr || !dwq_admit(q)) {
    return 1;
  }
  *qo = q;
  for (uint32_t i = 0; i != n; ++i) {
    const dwq_enc_payload pl{c[i], d_msgs, d_out, ctx->d_crc.as<uint32_t>()};
    dwq_item              it{};
    std::memcpy(static_cast<void*>(&it), &pl, sizeof(pl));
    it.spec            = 1;
    const hipError_t e = dwq_submit(q, it, tickets[i], false);
    if (e != hipSuccess) {
      dwq_unpin(q);
      return ctx->hip_fail(e, "PDSCH work queue submit");
    }
  }
  dwq_unpin(q);
  return LDPC_HIP_OK;
}

/* whether the item of ticket has completed (its outputs are in host memory) */
bool pdsch_encode_done(void* q, uint32_t ticket) { return ticket == 0xffffffffU || dwq_done(static_cast<dwq*>(q), ticket); }

/* waits for the item of ticket (a no-op for an unpublished one) */
int pdsch_encode_wait(void* q, uint32_t ticket)
{
  return (ticket == 0xffffffffU || dwq_wait(static_cast<dwq*>(q), ticket) == hipSuccess) ? LDPC_HIP_OK
                                                                                          : LDPC_HIP_EDEVICE;
}

/* The PDSCH encoder queue's batch (ldpc_hip_enc_queue.cpp): encoder + rate matcher in one launch
 * (ldpc_pdsch_encode_kernel), codeblock i from ed[i] / ext[3 i..] and rd[i] (whose cw_offset is unused). One codeblock
 * passes its descriptor by value; more are written to h_desc, pinned host memory mapped at d_desc (room for n
 * descriptors of pdsch_enc_desc_bytes()), which the kernel reads in place. */
int pdsch_encode_launch(ldpc_hip_ctx* ctx, uint32_t n, const ldpc_hip_enc_desc* ed, const uint32_t* ext,
                        const ldpc_hip_rm_desc* rd, const uint8_t* d_msgs, uint8_t* d_out, void* h_desc,
                        const void* d_desc, void* stream)
{
  if (ctx == nullptr || (n != 0 && (ed == nullptr || ext == nullptr || rd == nullptr || d_msgs == nullptr ||
                                    d_out == nullptr || (n > 1 && (h_desc == nullptr || d_desc == nullptr))))) {
    return LDPC_HIP_EINVAL;
  }
  if (n == 0) {
    return LDPC_HIP_OK;
  }
  pdsch_enc_cb  one{};
  pdsch_enc_cb* c = n == 1 ? &one : static_cast<pdsch_enc_cb*>(h_desc);
  for (uint32_t i = 0; i != n; ++i) {
    if (const char* why = make_pdsch_cb(ctx, ed[i], ext + 3 * i, rd[i], c[i])) {
      return ctx->fail(LDPC_HIP_EINVAL, why);
    }
  }
  (void)hipSetDevice(ctx->device);
  const hipError_t er = launch_pdsch_encode(static_cast<const pdsch_enc_cb*>(d_desc), n == 1 ? &one : nullptr, n,
                                            d_msgs, d_out, ctx->d_crc.as<uint32_t>(), abi_stream(ctx->stream, stream));
  return er == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(er, "ldpc_pdsch_encode_kernel launch");
}

/* ldpc_hip_encode_launch with, per codeblock i, ext[3 i] = the message's bit offset (< 8), ext[3 i + 1] = its data bits
 * (<= K Z; the rest are zeros) and ext[3 i + 2] = where the CRC24B of the bits before it goes (0: none); ext == nullptr:
 * K Z bits from bit 0, no CRC. The PDSCH encoder queue's TB mode (ldpc_hip_enc_queue.cpp) reads its segments in place. */
int encode_launch_ext(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_enc_desc* descs, const uint32_t* ext,
                      const uint8_t* d_msgs, uint8_t* d_cws, void* stream)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_cbs == 0) {
    return LDPC_HIP_OK;
  }
  if (descs == nullptr || d_msgs == nullptr || d_cws == nullptr) {
    return ctx->fail(LDPC_HIP_EINVAL, "encode_launch: null argument");
  }
  std::vector<enc_cb> e(nof_cbs);
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    const char* why = make_enc_cb(ctx, descs[i], ext != nullptr ? ext + 3 * i : nullptr, e[i]);
    if (why != nullptr) {
      return ctx->fail(LDPC_HIP_EINVAL, why);
    }
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s  = abi_stream(ctx->stream, stream);
  hipError_t  er = upload_descs(ctx->d_encdesc, ctx->c_encdesc, e.data(), nof_cbs * sizeof(enc_cb), s);
  if (er == hipSuccess) {
    er = launch_encode(ctx->d_encdesc.as<enc_cb>(), nof_cbs, d_msgs, d_cws, ctx->d_crc.as<uint32_t>(), s);
  }
  return er == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(er, "ldpc_encode_kernel launch");
}
} // namespace ldpc_hip
extern "C" {

int ldpc_hip_encode_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_enc_desc* descs, const uint8_t* d_msgs,
                           uint8_t* d_cws, void* stream)
{
  return ldpc_hip::encode_launch_ext(ctx, nof_cbs, descs, nullptr, d_msgs, d_cws, stream);
}

int ldpc_hip_rate_match_launch(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_rm_desc* descs,
                               const uint8_t* d_cws, uint8_t* d_out, void* stream)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_cbs == 0) {
    return LDPC_HIP_OK;
  }
  if (descs == nullptr || d_cws == nullptr || d_out == nullptr) {
    return ctx->fail(LDPC_HIP_EINVAL, "rate_match_launch: null argument");
  }
  std::vector<ratematch_cb> r(nof_cbs);
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    const char* why = ldpc_hip::make_rm_cb(descs[i], r[i]);
    if (why != nullptr) {
      return ctx->fail(LDPC_HIP_EINVAL, why);
    }
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s  = abi_stream(ctx->stream, stream);
  hipError_t  er = upload_descs(ctx->d_rmdesc, ctx->c_rmdesc, r.data(), nof_cbs * sizeof(ratematch_cb), s);
  if (er == hipSuccess) {
    er = launch_rate_match(ctx->d_rmdesc.as<ratematch_cb>(), nof_cbs, d_cws, d_out, s);
  }
  return er == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(er, "ldpc_rate_match_kernel launch");
}

int ldpc_hip_tb_join_launch(ldpc_hip_ctx* ctx, uint32_t nof_tbs, const ldpc_hip_tb_desc* descs, const uint8_t* d_msgs,
                            ldpc_hip_cb_result* d_cb_results, uint8_t* d_tb, ldpc_hip_tb_result* d_tb_results,
                            void* stream)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_tbs == 0) {
    return LDPC_HIP_OK;
  }
  if (descs == nullptr || d_msgs == nullptr || d_cb_results == nullptr || d_tb == nullptr || d_tb_results == nullptr) {
    return ctx->fail(LDPC_HIP_EINVAL, "tb_join: null argument");
  }
  for (uint32_t i = 0; i != nof_tbs; ++i) {
    const ldpc_hip_tb_desc& d = descs[i];
    const unsigned          C = d.nof_cbs;
    if (C == 0 || d.tbs == 0 || d.tbs % 8 != 0 || d.msg_stride < (d.cb_msg_bits + 7U) / 8U) {
      return ctx->fail(LDPC_HIP_EINVAL, "tb_join: invalid sizes");
    }
    if (d.cb_crc_bits != 16 && d.cb_crc_bits != 24) {
      return ctx->fail(LDPC_HIP_EINVAL, "tb_join: CRC length must be 16 or 24");
    }
    if (d.tbs / 8U > static_cast<uint32_t>(TBJ_CHUNK * TBJ_MAX_CHUNKS)) {
      return ctx->fail(LDPC_HIP_EINVAL, "tb_join: transport block too large");
    }
    if (C == 1) {
      if (d.tbs + d.cb_crc_bits + d.nof_filler_bits > d.cb_msg_bits) {
        return ctx->fail(LDPC_HIP_EINVAL, "tb_join: TB larger than its codeblock");
      }
    } else {
      const unsigned kd = d.cb_msg_bits - d.cb_crc_bits - d.nof_filler_bits;
      if (d.cb_crc_bits != 24 || d.cb_crc_bits + d.nof_filler_bits >= d.cb_msg_bits ||
          d.tbs <= (C - 1U) * kd || d.tbs - (C - 1U) * kd + 24U > kd) {
        return ctx->fail(LDPC_HIP_EINVAL, "tb_join: segmentation inconsistent with the TB size");
      }
    }
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = abi_stream(ctx->stream, stream);
  std::vector<tbj_block> blocks; /* per workgroup: its TB's descriptor, the TB index and the chunk */
  for (uint32_t i = 0; i != nof_tbs; ++i) {
    const uint32_t nch = (descs[i].tbs / 8U + TBJ_CHUNK - 1) / TBJ_CHUNK;
    for (uint32_t c = 0; c != nch; ++c) {
      blocks.push_back(tbj_block{descs[i], i, c});
    }
  }
  const uint32_t nblocks = static_cast<uint32_t>(blocks.size());
  hipError_t     e       = upload_descs(ctx->d_tbaux, ctx->c_tbaux, blocks.data(), nblocks * sizeof(tbj_block), s);
  const size_t work_bytes = static_cast<size_t>(nof_tbs) * TBJ_WORK_WORDS * 4;
  if (e == hipSuccess && ctx->d_tbwork.size < work_bytes) {
    /* arrival counters start at zero; the kernel returns each to zero after its TB */
    if ((e = hipStreamSynchronize(s)) == hipSuccess && (e = ctx->d_tbwork.reserve(work_bytes)) == hipSuccess) {
      e = hipMemsetAsync(ctx->d_tbwork.ptr, 0, ctx->d_tbwork.size, s);
    }
  }
  if (e == hipSuccess) {
    e = launch_tb_join(ctx->d_tbaux.as<tbj_block>(), nblocks, d_msgs, d_cb_results, d_tb, d_tb_results,
                       ctx->d_crc.as<uint32_t>(), ctx->d_tbwork.as<uint32_t>(), s);
  }
  return e == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(e, "ldpc_tb_join_kernel launch");
}

/* ---- synchronous entry points ---- */
} /* extern "C" */

namespace {

/* Waits for the context's sync event by polling (a blocking synchronize may sleep in the driver and wake late; the
 * software route's calls take tens of microseconds). */
hipError_t spin_event(hipEvent_t ev)
{
  hipError_t q;
  while ((q = hipEventQuery(ev)) == hipErrorNotReady) {
  }
  return q;
}

/* ldpc_decoder::decode of one codeblock from host memory, the software route's call (pusch_codeblock_decoder.cpp:
 * 58-62, one per CB and worker thread): the LLRs are copied into the context's pinned staging buffer, the kernel reads
 * them there and writes the message and result into pinned memory (no DMA either way, descriptor by value in the
 * kernel arguments), and the caller spins on one event. */
/* The decode descriptor of one codeblock for its specialised body (plan_host's dec_cb for a one-CB plan, without
 * building the plan); false when the graph has no specialised body or the scaling factor is not 0.8. */
bool one_spec_cb(const ldpc_hip_ctx* ctx, const ldpc_hip_dec_desc& s, dec_cb& d, int& slot)
{
  const float sf = (s.scaling_factor == 0.0f) ? 0.8f : s.scaling_factor;
  slot           = graph_slot(s.base_graph, s.lifting_size);
  if (sf != 0.8f || slot < 0 || slot >= 102 || ctx->graph_spec[slot] == 0) {
    return false;
  }
  d                = dec_cb{};
  d.llr_offset     = s.llr_offset;
  d.out_offset     = s.out_offset;
  d.llr_length     = s.llr_length;
  d.result_index   = 0;
  d.nof_filler_bits = s.nof_filler_bits;
  d.max_iterations = s.max_iterations;
  d.crc_mode       = s.crc_mode & ~LDPC_HIP_CRC_MODE_FLAG_KEEP_PASSED;
  d.keep_passed    = (s.crc_mode & LDPC_HIP_CRC_MODE_FLAG_KEEP_PASSED) != 0 ? 1 : 0;
  d.crc_poly       = (d.crc_mode == LDPC_HIP_CRC_MODE_NONE) ? 0 : s.crc_poly;
  d.scaling_factor = sf;
  return true;
}

int decode_one_zero_copy(ldpc_hip_ctx* ctx, const ldpc_hip_dec_desc& desc, const int8_t* llr, uint8_t* out,
                         ldpc_hip_cb_result* result)
{
  dwq_diag_entry();
  ldpc_hip_dec_desc d = desc;
  d.llr_offset        = 0;
  d.out_offset        = 0;
  int r = validate_dec_desc(ctx, d);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  /* The decoder works up to the last non-zero LLR (ldpc_decoder_impl.cpp:85-112: layers and length follow it, and the
   * soft bits past it are zero), so the trailing zeros of the caller's soft buffer (a rate-dematched codeblock shorter
   * than N) need not cross PCIe: the call stages and passes the buffer up to its last non-zero 32-byte block, never
   * below the minimum length (K + 2) Z. */
  {
    const uint32_t lmin = (d.base_graph == 1 ? 24U : 12U) * d.lifting_size;
    uint32_t       n    = d.llr_length;
    while (n >= lmin + 32U) {
      uint64_t w[4];
      std::memcpy(w, llr + n - 32U, sizeof(w));
      if ((w[0] | w[1] | w[2] | w[3]) != 0) {
        break;
      }
      n -= 32U;
    }
    d.llr_length = n;
  }
  const unsigned mb    = msg_bytes_of(d.base_graph, d.lifting_size);
  const size_t   res_o = (mb + 15U) & ~15U;
  hipError_t     e;
  if (ctx->staging_lost) {
    return ctx->hip_fail(hipErrorLaunchTimeOut, "sync decode: a stalled work-queue grid may still write this context's "
                                                "staging; close the context");
  }
  if ((e = ctx->s_in.reserve(std::max<size_t>(d.llr_length, 16), 0)) != hipSuccess ||
      (e = ctx->s_out.reserve(res_o + sizeof(ldpc_hip_cb_result), 0)) != hipSuccess || ctx->s_in.dev == nullptr ||
      ctx->s_out.dev == nullptr) {
    return ctx->hip_fail(e != hipSuccess ? e : hipErrorInvalidValue, "pinned staging (sync decode)");
  }
  /* the LLRs into the BAR staging, stores ordered before the hand-off (they may be write-combined), else into s_in */
  const int8_t* llr_dev = nullptr;
  if (!ctx->bar_failed && ctx->s_bar.reserve(std::max<size_t>(d.llr_length, 16)) == hipSuccess) {
    std::memcpy(ctx->s_bar.ptr, llr, d.llr_length);
    _mm_sfence();
    llr_dev = ctx->s_bar.dev_as<int8_t>();
  } else {
    ctx->bar_failed = true;
    std::memcpy(ctx->s_in.ptr, llr, d.llr_length);
    llr_dev = ctx->s_in.dev_as<int8_t>();
  }
  /* the device work queue of the graph's specialised body: no plan and no launch at all */
  dec_cb one{};
  int    slot = -1;
  if (ctx->use_dwq && one_spec_cb(ctx, d, one, slot)) {
    const int sid = ctx->graph_spec[slot] - 1;
    if (dwq* q = dwq_get(ctx->device, 1 + sid, ctx->key_block[1 + sid], ctx->key_lds[1 + sid])) {
      dwq_item it{};
      it.cb         = one;
      it.lay        = ctx->spec_lay[slot];
      it.llr_base   = llr_dev;
      it.out_base   = ctx->s_out.dev_as<uint8_t>();
      it.res_base   = reinterpret_cast<ldpc_hip_cb_result*>(ctx->s_out.dev_as<uint8_t>() + res_o);
      it.crc_tables = ctx->d_crc.as<uint32_t>();
      it.spec       = static_cast<uint32_t>(sid + 1);
      uint32_t ticket = 0;
      e               = dwq_submit(q, it, ticket, true);
      if (e != hipErrorLaunchOutOfResources) { /* refused (residency budget spent): nothing published, launch below */
        if (e != hipSuccess || (e = dwq_wait(q, ticket)) != hipSuccess) {
          ctx->staging_lost = ctx->staging_lost || !dwq_quiesced(q);
          return ctx->hip_fail(e, "work queue (sync decode)");
        }
        const ldpc_hip_cb_result res = *reinterpret_cast<const ldpc_hip_cb_result*>(ctx->s_out.as<uint8_t>() + res_o);
        if (res.status & LDPC_HIP_STATUS_OUTPUT_WRITTEN) {
          std::memcpy(out, ctx->s_out.ptr, mb);
        }
        if (result != nullptr) {
          *result = res;
        }
        return LDPC_HIP_OK;
      }
    }
  }
  ldpc_hip_plan            plan;
  std::vector<dec_cb>      cbs;
  std::vector<mixed_group> mg;
  if ((r = plan_host(ctx, 1, &d, plan, cbs, mg)) != LDPC_HIP_OK) {
    return r;
  }
  plan.has_one = true;
  plan.one     = cbs[0];
  plan.cbs_dev = nullptr;
  r = launch_plan(plan, llr_dev, ctx->s_out.dev_as<uint8_t>(),
                  reinterpret_cast<ldpc_hip_cb_result*>(ctx->s_out.dev_as<uint8_t>() + res_o), ctx->stream);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  if ((e = hipEventRecord(ctx->sync_event, ctx->stream)) != hipSuccess || (e = spin_event(ctx->sync_event)) != hipSuccess) {
    return ctx->hip_fail(e, "sync decode");
  }
  const ldpc_hip_cb_result res = *reinterpret_cast<const ldpc_hip_cb_result*>(ctx->s_out.as<uint8_t>() + res_o);
  if (res.status & LDPC_HIP_STATUS_OUTPUT_WRITTEN) {
    std::memcpy(out, ctx->s_out.ptr, mb);
  }
  if (result != nullptr) {
    *result = res;
  }
  return LDPC_HIP_OK;
}

} // namespace

extern "C" {

int ldpc_hip_decode_sync(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dec_desc* descs,
                         const int8_t* const* llrs, uint8_t* const* outs, ldpc_hip_cb_result* results)
{
  if (ctx == nullptr || (nof_cbs != 0 && (descs == nullptr || llrs == nullptr || outs == nullptr))) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_cbs == 0) {
    return LDPC_HIP_OK;
  }
  (void)hipSetDevice(ctx->device);
  if (nof_cbs == 1 && ctx->sync_zc && ctx->s_in.dev != nullptr) {
    return decode_one_zero_copy(ctx, descs[0], llrs[0], outs[0], results);
  }
  std::vector<ldpc_hip_dec_desc> d(descs, descs + nof_cbs);
  uint64_t                       llr_total = 0, out_total = 0;
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    d[i].llr_offset = llr_total;
    d[i].out_offset = out_total;
    llr_total += (d[i].llr_length + 15U) & ~15U;
    out_total += (msg_bytes_of(d[i].base_graph, d[i].lifting_size) + 15U) & ~15U;
  }
  ldpc_hip_plan plan;
  int           r = build_plan(ctx, nof_cbs, d.data(), plan);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  hipError_t e;
  if ((e = ctx->d_llr.reserve(llr_total)) != hipSuccess || (e = ctx->d_out.reserve(out_total)) != hipSuccess ||
      (e = ctx->d_res.reserve(nof_cbs * sizeof(ldpc_hip_cb_result))) != hipSuccess) {
    return ctx->hip_fail(e, "hipMalloc(sync decode)");
  }
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    e = hipMemcpyAsync(ctx->d_llr.as<int8_t>() + d[i].llr_offset, llrs[i], d[i].llr_length, hipMemcpyHostToDevice,
                       ctx->stream);
    if (e != hipSuccess) {
      return ctx->hip_fail(e, "hipMemcpyAsync(llr)");
    }
  }
  r = launch_plan(plan, ctx->d_llr.as<int8_t>(), ctx->d_out.as<uint8_t>(), ctx->d_res.as<ldpc_hip_cb_result>(),
                  ctx->stream);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  std::vector<ldpc_hip_cb_result> res(nof_cbs);
  std::vector<uint8_t>            host_out(out_total);
  if ((e = hipMemcpyAsync(res.data(), ctx->d_res.ptr, nof_cbs * sizeof(ldpc_hip_cb_result), hipMemcpyDeviceToHost,
                          ctx->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(host_out.data(), ctx->d_out.ptr, out_total, hipMemcpyDeviceToHost, ctx->stream)) !=
          hipSuccess ||
      (e = hipStreamSynchronize(ctx->stream)) != hipSuccess) {
    return ctx->hip_fail(e, "sync decode");
  }
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    if (res[i].status & LDPC_HIP_STATUS_OUTPUT_WRITTEN) {
      std::memcpy(outs[i], host_out.data() + d[i].out_offset, msg_bytes_of(d[i].base_graph, d[i].lifting_size));
    }
    if (results != nullptr) {
      results[i] = res[i];
    }
  }
  return LDPC_HIP_OK;
}

static int validate_dematch(ldpc_hip_ctx* ctx, const ldpc_hip_dematch_desc& d)
{
  const unsigned Qm = d.modulation_order;
  if (d.rv > 3 || !(Qm == 1 || Qm == 2 || Qm == 4 || Qm == 6 || Qm == 8) || d.rm_length % Qm != 0) {
    return ctx->fail(LDPC_HIP_EINVAL, "invalid rv / modulation / rm_length");
  }
  if (d.Nref > MAX_CB_LEN || d.cb_length > MAX_CB_LEN) {
    return ctx->fail(LDPC_HIP_EINVAL, "N_ref / cb_length too large");
  }
  unsigned Z = 0, K = 0;
  if (d.cb_length % 66 == 0) {
    Z = d.cb_length / 66;
    K = 22;
  } else if (d.cb_length % 50 == 0) {
    Z = d.cb_length / 50;
    K = 10;
  } else {
    return ctx->fail(LDPC_HIP_EINVAL, "LDPC rate dematching: invalid input length.");
  }
  if (lifting_index(Z) < 0) {
    return ctx->fail(LDPC_HIP_EINVAL, "LDPC rate dematching: invalid input length.");
  }
  if (d.nof_filler_bits >= (K - 2) * Z) {
    return ctx->fail(LDPC_HIP_EINVAL, "LDPC rate dematching: invalid number of filler bits.");
  }
  return LDPC_HIP_OK;
}

int ldpc_hip_rate_dematch_sync(ldpc_hip_ctx* ctx, uint32_t nof_cbs, const ldpc_hip_dematch_desc* descs,
                               int8_t* const* soft_bufs, const int8_t* const* llrs)
{
  if (ctx == nullptr || (nof_cbs != 0 && (descs == nullptr || soft_bufs == nullptr || llrs == nullptr))) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_cbs == 0) {
    return LDPC_HIP_OK;
  }
  (void)hipSetDevice(ctx->device);
  if (nof_cbs == 1 && ctx->sync_zc) {
    /* the software route's call (pusch_codeblock_decoder.cpp:42-46): LLRs and the old soft bits copied into pinned
     * staging, the dematcher kernel working on it in place, descriptor by value */
    dwq_diag_entry();
    const ldpc_hip_dematch_desc& s = descs[0];
    int                          r = validate_dematch(ctx, s);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    const size_t soft_o = (s.rm_length + 15U) & ~15U;
    hipError_t   e;
    if (ctx->staging_lost) {
      return ctx->hip_fail(hipErrorLaunchTimeOut, "rate dematch: a stalled work-queue grid may still write this "
                                                  "context's staging; close the context");
    }
    if ((e = ctx->s_in.reserve(soft_o + s.cb_length, 0)) == hipSuccess && ctx->s_in.dev != nullptr) {
      /* the LLRs into the BAR staging as the one-CB decode's (else into s_in); the soft bits, which the host reads
       * back, stay in pinned memory */
      const int8_t* llr_dev = ctx->s_in.dev_as<int8_t>();
      if (s.rm_length != 0) {
        if (!ctx->bar_failed && ctx->s_bar.reserve(s.rm_length) == hipSuccess) {
          std::memcpy(ctx->s_bar.ptr, llrs[0], s.rm_length);
          llr_dev = ctx->s_bar.dev_as<int8_t>();
        } else {
          ctx->bar_failed = true;
          std::memcpy(ctx->s_in.ptr, llrs[0], s.rm_length);
        }
      }
      /* the old soft bits also on new data: positions the dematcher does not write keep them (the limited-buffer
       * gap between the last written index and the zeroed tail, ldpc_rate_dematcher_impl.cpp:197-200) */
      std::memcpy(ctx->s_in.as<int8_t>() + soft_o, soft_bufs[0], s.cb_length);
      _mm_sfence(); /* the write-combined LLR stores before the hand-off */
      dematch_cb one{};
      one.llr              = llr_dev;
      one.soft             = ctx->s_in.dev_as<int8_t>() + soft_o;
      one.cb_length        = s.cb_length;
      one.rm_length        = s.rm_length;
      one.Nref             = s.Nref;
      one.nof_filler_bits  = s.nof_filler_bits;
      one.modulation_order = s.modulation_order;
      one.rv               = s.rv;
      one.new_data         = s.new_data;
      dwq* q               = ctx->use_dwq ? dwq_get(ctx->device, 0, ctx->key_block[0], ctx->key_lds[0]) : nullptr;
      if (q != nullptr) { /* the dematch-only work queue */
        dwq_item it{};
        it.dm           = one;
        it.crc_tables   = ctx->d_crc.as<uint32_t>();
        it.spec         = 0;
        uint32_t ticket = 0;
        e               = dwq_submit(q, it, ticket, true);
        if (e != hipErrorLaunchOutOfResources) { /* refused (residency budget spent): launch below */
          if (e != hipSuccess || (e = dwq_wait(q, ticket)) != hipSuccess) {
            ctx->staging_lost = ctx->staging_lost || !dwq_quiesced(q);
            return ctx->hip_fail(e, "work queue (rate dematch)");
          }
          std::memcpy(soft_bufs[0], ctx->s_in.as<int8_t>() + soft_o, s.cb_length);
          return LDPC_HIP_OK;
        }
      }
      if ((e = launch_dematch(nullptr, 1, ctx->dtab, ctx->stream, &one)) != hipSuccess ||
          (e = hipEventRecord(ctx->sync_event, ctx->stream)) != hipSuccess ||
          (e = spin_event(ctx->sync_event)) != hipSuccess) {
        return ctx->hip_fail(e, "rate dematch (one CB)");
      }
      std::memcpy(soft_bufs[0], ctx->s_in.as<int8_t>() + soft_o, s.cb_length);
      return LDPC_HIP_OK;
    }
    (void)hipGetLastError();
  }
  uint64_t              llr_total = 0, soft_total = 0;
  std::vector<uint64_t> lo(nof_cbs), so(nof_cbs);
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    int r = validate_dematch(ctx, descs[i]);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    lo[i] = llr_total;
    so[i] = soft_total;
    llr_total += (descs[i].rm_length + 15U) & ~15U;
    soft_total += (descs[i].cb_length + 15U) & ~15U;
  }
  hipError_t e;
  if ((e = ctx->d_llr.reserve(std::max<uint64_t>(llr_total, 16))) != hipSuccess ||
      (e = ctx->d_soft.reserve(soft_total)) != hipSuccess ||
      (e = ctx->d_desc.reserve(nof_cbs * sizeof(dematch_cb))) != hipSuccess) {
    return ctx->hip_fail(e, "hipMalloc(dematch)");
  }
  std::vector<dematch_cb> dm(nof_cbs);
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    const ldpc_hip_dematch_desc& s = descs[i];
    dm[i]                          = dematch_cb{};
    dm[i].llr                      = ctx->d_llr.as<int8_t>() + lo[i];
    dm[i].soft                     = ctx->d_soft.as<int8_t>() + so[i];
    dm[i].cb_length                = s.cb_length;
    dm[i].rm_length                = s.rm_length;
    dm[i].Nref                     = s.Nref;
    dm[i].nof_filler_bits          = s.nof_filler_bits;
    dm[i].modulation_order         = s.modulation_order;
    dm[i].rv                       = s.rv;
    dm[i].new_data                 = s.new_data;
    if (s.rm_length != 0 &&
        (e = hipMemcpyAsync(ctx->d_llr.as<int8_t>() + lo[i], llrs[i], s.rm_length, hipMemcpyHostToDevice,
                            ctx->stream)) != hipSuccess) {
      return ctx->hip_fail(e, "hipMemcpyAsync(llr)");
    }
    if ((e = hipMemcpyAsync(ctx->d_soft.as<int8_t>() + so[i], soft_bufs[i], s.cb_length, hipMemcpyHostToDevice,
                            ctx->stream)) != hipSuccess) {
      return ctx->hip_fail(e, "hipMemcpyAsync(soft)");
    }
  }
  if ((e = hipMemcpyAsync(ctx->d_desc.ptr, dm.data(), nof_cbs * sizeof(dematch_cb), hipMemcpyHostToDevice,
                          ctx->stream)) != hipSuccess ||
      (e = launch_dematch(ctx->d_desc.as<dematch_cb>(), nof_cbs, ctx->dtab, ctx->stream)) != hipSuccess) {
    return ctx->hip_fail(e, "rate dematch launch");
  }
  for (uint32_t i = 0; i != nof_cbs; ++i) {
    if ((e = hipMemcpyAsync(soft_bufs[i], ctx->d_soft.as<int8_t>() + so[i], descs[i].cb_length,
                            hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess) {
      return ctx->hip_fail(e, "hipMemcpyAsync(soft out)");
    }
  }
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) {
    return ctx->hip_fail(e, "rate dematch sync");
  }
  return LDPC_HIP_OK;
}

/* ---- HAL queue ---- */
} /* extern "C" */

namespace {

/* Waits for a launched batch (queue_reserve / queue_free / close while operations are in flight). */
/* waits for the batch's early-copy items (they read h_llr and write q_llr); the first error */
hipError_t hal_wait_copies(ldpc_hip_ctx* ctx)
{
  hipError_t r = hipSuccess;
  for (uint32_t t : ctx->hcopy_tickets) {
    const hipError_t e = dwq_wait(ctx->hcopy_q, t);
    r                  = r == hipSuccess ? e : r;
  }
  ctx->hcopy_tickets.clear();
  return r;
}

void hal_sync(ldpc_hip_ctx* ctx)
{
  (void)hal_wait_copies(ctx);
  if (ctx->hstate == hal_state::launched || ctx->hstate == hal_state::failed) {
    /* every work-queue item submitted (a failed batch may have submitted some before its error) */
    for (const hal_op& op : ctx->hops) {
      if (op.q != nullptr) {
        (void)dwq_wait(op.q, op.ticket);
      }
    }
  }
  if (ctx->hstate == hal_state::launched) {
    (void)hipEventSynchronize(ctx->done_event);
  } else if (ctx->hstate == hal_state::failed) {
    (void)hipStreamSynchronize(ctx->hq_stream); /* whatever part of the failed launch was queued */
  } else if (ctx->hstate == hal_state::staging && ctx->h_llr_copied != 0) {
    (void)hipStreamSynchronize(ctx->hq_stream); /* early copies of a batch never launched still read h_llr */
  }
}

/* Drops the batch's staged operations (the HARQ arena keeps its entries). */
void hal_reset(ldpc_hip_ctx* ctx, hal_state next)
{
  for (const hal_op& op : ctx->hops) {
    if (op.cb_index < ctx->hslot.size()) {
      ctx->hslot[op.cb_index] = -1;
    }
  }
  ctx->hops.clear();
  ctx->hdequeued    = 0;
  ctx->h_llr_copied = 0;
  ctx->hcopy        = false;
  dwq_unpin(ctx->hcopy_q); /* admitted (pinned) when the batch began */
  ctx->hcopy_q      = nullptr;
  ctx->hcopy_tickets.clear(); /* waited for by hal_sync / the launch */
  ctx->h_llr_used   = 0;
  ctx->h_soft_used = 0;
  ctx->h_out_used  = 0;
  ctx->hstate      = next;
}

/* Zero-copy batches: with the HARQ soft buffers in the HBM arena, a batch whose staged LLRs and descriptors take at
 * most hal_zero_copy_max_bytes() (LDPC_HIP_HAL_ZERO_COPY_MAX, default 4 MiB: C4's 128-CB TB, 1.25 MB of LLRs, first
 * dequeue 92-110 -> 74 us against 256 KiB, profiles/r04/route_ab.json) is read by the kernels straight from the
 * pinned staging buffer, and the decoder writes messages and results straight into the pinned readback buffer: no DMA copy either way, and two fewer dependent operations in
 * the stream (a small TB's latency). Larger batches (a large TB's LLRs) go through one DMA copy each way. */
uint64_t hal_zero_copy_max_bytes()
{
  static const uint64_t v = [] {
    const char* e = std::getenv("LDPC_HIP_HAL_ZERO_COPY_MAX"); /* bytes; A/B timing of the threshold */
    return e != nullptr ? std::strtoull(e, nullptr, 10) : 4ULL * 1024ULL * 1024ULL;
  }();
  return v;
}
/* a zero-copy batch of at most this many codeblocks goes to the device work queue (one item per codeblock; the queue's
 * grid has 32 workgroups by default), a larger one is one launch with a workgroup per codeblock */
constexpr size_t HAL_DWQ_MAX_CBS = 16;

/* Early copy of a large batch's LLRs (LDPC_HIP_LAUNCH_HAL_NO_EARLY_COPY). Round 4's zero-copy launch of C4's 128-CB TB
 * read its 1.25 MB of LLRs from pinned memory over PCIe after the last enqueue (the fused kernel 57.6 us at ~30 GB/s,
 * profiles/r04/hal_kernel_trace.txt). Now each chunk of staged LLRs goes to q_llr by the copy engine while the caller
 * is still enqueueing, and at the first dequeue only the last chunk and the descriptors cross: the kernel reads HBM.
 * Not per-item work-queue traffic (measured slower in round 4, profiles/r04/route_ab_eager_v1.json). */
uint64_t hal_copy_chunk_bytes()
{
  static const uint64_t v = [] {
    const char* e = std::getenv("LDPC_HIP_HAL_COPY_CHUNK"); /* bytes; A/B timing of the chunk size */
    return e != nullptr ? std::max<uint64_t>(4096, std::strtoull(e, nullptr, 10)) : 256ULL * 1024ULL;
  }();
  return v;
}

/* Early copy on (LDPC_HIP_LAUNCH_HAL_EARLY_COPY or LDPC_HIP_HAL_EARLY_COPY=1) by hipMemcpyAsync per chunk: measured
 * slower than the zero-copy read on the GPU box (C4's 128-CB TB 100 -> 123 us, profiles/r05), so it is off by default.
 * The work-queue form (hal_dwq_copy) is the other way to copy early. */
bool hal_early_copy(const ldpc_hip_ctx* ctx)
{
  static const bool env = [] {
    const char* e = std::getenv("LDPC_HIP_HAL_EARLY_COPY");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return (env || (ctx->params.launch_flags & LDPC_HIP_LAUNCH_HAL_EARLY_COPY) != 0) &&
         (ctx->params.launch_flags & LDPC_HIP_LAUNCH_HAL_COPY) == 0;
}

/* Early copy through the copy work queue (LDPC_HIP_HAL_DWQ_COPY=1; needs the work queues): a large batch's
 * staged LLRs go to HBM in 64 KiB items of a resident grid while the caller enqueues (no runtime call per piece), and
 * the batch kernel reads HBM instead of pinned memory over PCIe. */
bool hal_dwq_copy(const ldpc_hip_ctx* ctx)
{
  static const bool env = [] {
    const char* e = std::getenv("LDPC_HIP_HAL_DWQ_COPY");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return env && ctx->use_dwq && (ctx->params.launch_flags & LDPC_HIP_LAUNCH_HAL_COPY) == 0;
}

constexpr uint64_t HAL_COPY_PIECE = 64U * 1024U; /* bytes per copy item */

/* Queues h_llr[h_llr_copied, upto) for q_llr once at least a chunk (force: anything) is staged: as copy items when
 * the batch has a copy queue (hcopy_q; upto a multiple of 16), else on hq_stream. */
hipError_t hal_copy_staged(ldpc_hip_ctx* ctx, bool force, uint64_t upto)
{
  const uint64_t n = upto - ctx->h_llr_copied;
  if (n == 0 || (!force && n < (ctx->hcopy_q != nullptr ? HAL_COPY_PIECE : hal_copy_chunk_bytes()))) {
    return hipSuccess;
  }
  if (upto > ctx->q_llr.size) { /* the device copy moves: what was queued is lost, copy from the start again */
    (void)hal_wait_copies(ctx);
    hipError_t e = hipStreamSynchronize(ctx->hq_stream);
    if (e == hipSuccess) {
      e = ctx->q_llr.reserve(std::max<uint64_t>(upto, 2 * ctx->q_llr.size));
    }
    if (e != hipSuccess) {
      return e;
    }
    ctx->h_llr_copied = 0;
  }
  if (ctx->hcopy_q != nullptr) {
    while (ctx->h_llr_copied < upto) {
      const uint64_t m = std::min<uint64_t>(HAL_COPY_PIECE, upto - ctx->h_llr_copied);
      if (!force && m < HAL_COPY_PIECE) {
        break;
      }
      const dwq_copy_payload pl{ctx->h_llr.dev_as<uint8_t>() + ctx->h_llr_copied,
                                ctx->q_llr.as<uint8_t>() + ctx->h_llr_copied, (m + 15U) / 16U};
      dwq_item it{};
      std::memcpy(static_cast<void*>(&it), &pl, sizeof(pl));
      it.spec           = 1;
      uint32_t   ticket = 0xffffffffU;
      hipError_t e      = dwq_submit(ctx->hcopy_q, it, ticket, false);
      if (ticket != 0xffffffffU) {
        ctx->hcopy_tickets.push_back(ticket);
      }
      if (e != hipSuccess) {
        return e;
      }
      ctx->h_llr_copied += m;
    }
    return hipSuccess;
  }
  const hipError_t e = hipMemcpyAsync(ctx->q_llr.as<uint8_t>() + ctx->h_llr_copied,
                                      ctx->h_llr.as<uint8_t>() + ctx->h_llr_copied, upto - ctx->h_llr_copied,
                                      hipMemcpyHostToDevice, ctx->hq_stream);
  if (e == hipSuccess) {
    ctx->h_llr_copied = upto;
  }
  return e;
}

/* h_llr may move in reserve(): copies still reading the old allocation finish first */
hipError_t hal_reserve_llr(ldpc_hip_ctx* ctx, uint64_t n, uint64_t keep)
{
  if (n > ctx->h_llr.size && ctx->h_llr_copied != 0) {
    (void)hal_wait_copies(ctx);
    const hipError_t e = hipStreamSynchronize(ctx->hq_stream);
    if (e != hipSuccess) {
      return e;
    }
  }
  return ctx->h_llr.reserve(n, keep);
}

/* The first dequeue of a staged batch: one H2D of the staged LLRs (and host soft buffers), one descriptor upload,
 * dematch + decode of the live operations, one D2H of messages, results (and soft buffers), then an event; or, for a
 * zero-copy batch, the two kernels on the pinned buffers alone. */
int hal_launch_issue(ldpc_hip_ctx* ctx, bool& issued)
{
  const bool ext = ctx->repo != nullptr;
  /* the HARQ memory's address stays fixed until this batch is queued (ldpc_hip_harq_repo::grow) */
  std::shared_lock<std::shared_mutex> arena_lock;
  if (ext) {
    arena_lock = std::shared_lock<std::shared_mutex>(ctx->repo->arena_mu);
  }
  std::vector<uint32_t> live;
  for (uint32_t i = 0; i != ctx->hops.size(); ++i) {
    if (!ctx->hops[i].dropped) {
      live.push_back(i);
    }
  }
  hipError_t e = hipSuccess;
  if (!live.empty()) {
    int8_t* soft_base = nullptr;
    /* one readback: the result records follow the messages in q_out / h_out */
    ctx->h_res_off       = (ctx->h_out_used + 15U) & ~static_cast<uint64_t>(15U);
    const uint64_t rback = ctx->h_res_off + live.size() * sizeof(ldpc_hip_cb_result);
    if ((e = ctx->q_out.reserve(rback)) != hipSuccess ||
        (!ext && (e = ctx->q_soft.reserve(std::max<uint64_t>(ctx->h_soft_used, 16))) != hipSuccess) ||
        (e = ctx->h_out.reserve(rback, 0)) != hipSuccess) {
      return ctx->hip_fail(e, "HAL buffers");
    }
    soft_base = ext ? ctx->repo->arena.as<int8_t>() : ctx->q_soft.as<int8_t>();
    /* descriptors: dematch_cb[live], then the decode plan's dec_cb[live] and mixed_group[groups] */
    std::vector<ldpc_hip_dec_desc> dd(live.size());
    std::vector<dematch_cb>        dm(live.size());
    for (uint32_t k = 0; k != live.size(); ++k) {
      hal_op& op = ctx->hops[live[k]];
      op.pos     = k;
      dematch_cb& d      = dm[k];
      d                  = dematch_cb{};
      d.llr              = nullptr; /* set once q_llr has its final size (below) */
      d.soft             = soft_base + op.soft_off;
      d.cb_length        = op.N;
      d.rm_length        = op.cfg.cw_length;
      d.Nref             = op.cfg.Nref;
      d.nof_filler_bits  = op.cfg.nof_filler_bits;
      d.modulation_order = op.cfg.modulation_order;
      d.rv               = op.cfg.rv;
      d.new_data         = op.cfg.new_data;
      ldpc_hip_dec_desc& x = dd[k];
      x                    = ldpc_hip_dec_desc{};
      x.base_graph         = op.cfg.base_graph;
      x.max_iterations     = static_cast<uint8_t>(op.cfg.max_nof_ldpc_iterations);
      x.crc_mode = op.cfg.use_early_stop ? LDPC_HIP_CRC_MODE_EARLY_STOP : LDPC_HIP_CRC_MODE_CHECK_AFTER;
      x.crc_poly        = static_cast<int8_t>(op.cfg.cb_crc_type);
      x.lifting_size    = static_cast<uint16_t>(op.cfg.lifting_size);
      x.nof_filler_bits = static_cast<uint16_t>(op.cfg.nof_filler_bits);
      x.llr_length      = op.N;
      x.scaling_factor  = 0.8f; /* pusch_decoder default (ldpc_decoder.h:50) */
      x.llr_offset      = op.soft_off;
      x.out_offset      = op.out_off;
    }
    if (ctx->hplan == nullptr) {
      ctx->hplan = new ldpc_hip_plan();
    }
    std::vector<dec_cb>      cbs;
    std::vector<mixed_group> mg;
    int r = plan_host(ctx, static_cast<uint32_t>(dd.size()), dd.data(), *ctx->hplan, cbs, mg);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    /* the dematcher runs fused into the decode kernels (one launch; LDPC_HIP_LAUNCH_SEPARATE_DEMATCH: its own kernel
     * first): its descriptors then go in the plan's block order */
    const bool fuse_dm = (ctx->params.launch_flags & LDPC_HIP_LAUNCH_SEPARATE_DEMATCH) == 0;
    if (fuse_dm) {
      std::vector<dematch_cb> dmp(dm.size());
      for (size_t i = 0; i != cbs.size(); ++i) {
        dmp[i] = dm[cbs[i].result_index];
      }
      dm.swap(dmp);
    }
    const uint32_t dm_lds  = fuse_dm ? dm_fused_budget(dm.data(), dm.size()) : 0U;
    const size_t dm_bytes  = dm.size() * sizeof(dematch_cb);
    const size_t cb_off    = (dm_bytes + 15) & ~static_cast<size_t>(15);
    const size_t cb_bytes  = cbs.size() * sizeof(dec_cb);
    const size_t mg_off    = (cb_off + cb_bytes + 15) & ~static_cast<size_t>(15);
    const size_t desc_size = mg_off + mg.size() * sizeof(mixed_group);
    /* one upload: the descriptors follow the staged LLRs in h_llr / q_llr */
    const uint64_t d0    = (ctx->h_llr_used + 15U) & ~static_cast<uint64_t>(15U);
    const uint64_t up    = (d0 + desc_size + 15U) & ~static_cast<uint64_t>(15U); /* copy items move 16-byte words */
    if ((e = hal_reserve_llr(ctx, up, ctx->h_llr_used)) != hipSuccess) {
      return ctx->hip_fail(e, "HAL descriptors");
    }
    if (up > ctx->q_llr.size) { /* q_llr moves: a copy queued early is lost (hal_copy_staged copies it again) */
      (void)hal_wait_copies(ctx);
      if ((e = hipStreamSynchronize(ctx->hq_stream)) != hipSuccess || (e = ctx->q_llr.reserve(up)) != hipSuccess) {
        return ctx->hip_fail(e, "HAL descriptors");
      }
      ctx->h_llr_copied = 0;
    }
    const bool zc = ext && up <= hal_zero_copy_max_bytes() &&
                    (ctx->params.launch_flags & LDPC_HIP_LAUNCH_HAL_COPY) == 0 && ctx->h_llr.dev != nullptr &&
                    ctx->h_out.dev != nullptr;
    /* early-copied batch: the LLRs (and descriptors) in HBM, the outputs still written straight into pinned memory */
    const bool early = zc && ctx->hcopy && live.size() > HAL_DWQ_MAX_CBS;
    if (!early) {
      (void)hal_wait_copies(ctx); /* copies of a batch that reads pinned memory after all (nothing reads q_llr) */
    }
    /* LLRs and descriptors as the kernels see them: the device copy, or (zero-copy) the pinned buffer itself */
    uint8_t* const llr_dev = (zc && !early) ? ctx->h_llr.dev_as<uint8_t>() : ctx->q_llr.as<uint8_t>();
    uint8_t* const out_dev = zc ? ctx->h_out.dev_as<uint8_t>() : ctx->q_out.as<uint8_t>();
    for (uint32_t k = 0; k != live.size(); ++k) { /* q_llr may have moved in reserve(): device pointers only now */
      const uint32_t c = fuse_dm ? cbs[k].result_index : k; /* dm[k] is live CB c's */
      dm[k].llr        = reinterpret_cast<int8_t*>(llr_dev) + ctx->hops[live[c]].llr_off;
    }
    uint8_t* hd = ctx->h_llr.as<uint8_t>() + d0;
    std::memcpy(hd, dm.data(), dm_bytes);
    std::memcpy(hd + cb_off, cbs.data(), cb_bytes);
    if (!mg.empty()) {
      std::memcpy(hd + mg_off, mg.data(), mg.size() * sizeof(mixed_group));
    }
    uint8_t* qd            = llr_dev + d0;
    ctx->hplan->cbs_dev    = reinterpret_cast<const dec_cb*>(qd + cb_off);
    ctx->hplan->groups_dev = reinterpret_cast<const mixed_group*>(qd + mg_off);
    ctx->hplan->has_one    = cbs.size() == 1; /* one-CB batch: both descriptors by value (no host-memory table read) */
    if (ctx->hplan->has_one) {
      ctx->hplan->one = cbs[0];
    }
    /* A zero-copy batch whose graphs all have specialised bodies goes to the device work queues: one item per
     * codeblock (fused dematch + decode), no launch, and each dequeue waits for its own codeblock only. */
    bool via_dwq = zc && !early && fuse_dm && ctx->use_dwq && cbs.size() <= HAL_DWQ_MAX_CBS;
    std::vector<const launch_group*> cb_grp(cbs.size(), nullptr);
    std::vector<dwq*>                cb_q(cbs.size(), nullptr);
    for (size_t i = 0; i != cbs.size() && via_dwq; ++i) {
      via_dwq = false;
      for (const launch_group& g : ctx->hplan->groups) {
        if (i >= g.first && i < g.first + g.count) {
          via_dwq   = g.sf08 && g.slot < NARROW_SLOT_BASE && ctx->graph_spec[g.slot] != 0;
          cb_grp[i] = &g;
        }
      }
      if (via_dwq) {
        const int sid = ctx->graph_spec[cb_grp[i]->slot] - 1;
        cb_q[i]       = dwq_get(ctx->device, 1 + sid, ctx->key_block[1 + sid], ctx->key_lds[1 + sid]);
        via_dwq       = cb_q[i] != nullptr;
      }
    }
    /* every queue the batch uses has a grid running (or one started now) within the residency budget; otherwise the
     * whole batch takes the launch path, so no item is ever left waiting for a stream */
    std::vector<dwq*> pinned; /* the distinct queues admitted (pinned) until the batch's items are submitted */
    for (size_t i = 0; i != cbs.size() && via_dwq; ++i) {
      if (std::find(pinned.begin(), pinned.end(), cb_q[i]) != pinned.end()) {
        continue;
      }
      via_dwq = dwq_admit(cb_q[i]);
      if (via_dwq) {
        pinned.push_back(cb_q[i]);
      }
    }
    struct unpin_all {
      std::vector<dwq*>& v;
      ~unpin_all()
      {
        for (dwq* q : v) {
          dwq_unpin(q);
        }
      }
    } unpin_guard{pinned};
    if (via_dwq) {
      issued = true;
      for (size_t i = 0; i != cbs.size(); ++i) {
        const launch_group* grp = cb_grp[i];
        const int           sid = ctx->graph_spec[grp->slot] - 1;
        dwq*                q   = cb_q[i];
        dwq_item it{};
        it.cb         = cbs[i];
        it.lay        = grp->lay;
        it.dm         = dm[i];
        it.llr_base   = soft_base;
        it.out_base   = out_dev;
        it.res_base   = reinterpret_cast<ldpc_hip_cb_result*>(out_dev + ctx->h_res_off);
        it.crc_tables = ctx->d_crc.as<uint32_t>();
        it.spec       = static_cast<uint32_t>(sid + 1);
        hal_op&  op     = ctx->hops[live[cbs[i].result_index]];
        uint32_t ticket = 0xffffffffU;
        e               = dwq_submit(q, it, ticket, false);
        if (ticket != 0xffffffffU) { /* published (also when an error follows): hal_sync waits for it */
          op.q      = q;
          op.ticket = ticket;
          if (ext) {
            ctx->repo->track_item(q, ticket); /* the arena may not move before this item is done (grow) */
          }
        }
        if (e != hipSuccess) {
          return ctx->hip_fail(e, "HAL work queue submit");
        }
      }
      ctx->hstate      = hal_state::launched;
      ctx->hbatch_done = false;
      return LDPC_HIP_OK;
    }
    hipStream_t s = ctx->hq_stream;
    issued        = true; /* from here on the stream may hold part of the batch */
    if (early && (e = hal_copy_staged(ctx, true, up)) == hipSuccess && ctx->hcopy_q != nullptr) {
      e = hal_wait_copies(ctx); /* the kernel reads q_llr: every copy item done (they run on the queue's own stream) */
    }
    if ((early && e != hipSuccess) || /* the last chunk and the descriptors */
        (!zc && (e = hipMemcpyAsync(ctx->q_llr.ptr, ctx->h_llr.ptr, up, hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (!ext && (e = hipMemcpyAsync(ctx->q_soft.ptr, ctx->h_soft.ptr, ctx->h_soft_used, hipMemcpyHostToDevice, s)) !=
                     hipSuccess)) {
      return ctx->hip_fail(e, "HAL upload");
    }
    if (!fuse_dm && (e = launch_dematch(reinterpret_cast<const dematch_cb*>(qd), static_cast<uint32_t>(dm.size()),
                                        ctx->dtab, s, dm.size() == 1 ? dm.data() : nullptr)) != hipSuccess) {
      return ctx->hip_fail(e, "HAL dematch");
    }
    r = launch_plan(*ctx->hplan, soft_base, out_dev, reinterpret_cast<ldpc_hip_cb_result*>(out_dev + ctx->h_res_off),
                    s, fuse_dm ? reinterpret_cast<const dematch_cb*>(qd) : nullptr,
                    fuse_dm && dm.size() == 1 ? dm.data() : nullptr, dm_lds);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    if ((!zc && (e = hipMemcpyAsync(ctx->h_out.ptr, ctx->q_out.ptr, rback, hipMemcpyDeviceToHost, s)) != hipSuccess) ||
        (!ext && (e = hipMemcpyAsync(ctx->h_soft.ptr, ctx->q_soft.ptr, ctx->h_soft_used, hipMemcpyDeviceToHost, s)) !=
                     hipSuccess)) {
      return ctx->hip_fail(e, "HAL readback");
    }
  }
  issued = true;
  if ((e = hipEventRecord(ctx->done_event, ctx->hq_stream)) != hipSuccess) {
    return ctx->hip_fail(e, "hipEventRecord");
  }
  ctx->hstate      = hal_state::launched;
  ctx->hbatch_done = false;
  return LDPC_HIP_OK;
}

/* hal_launch_issue, and on an error after any part of the batch was queued the batch is marked failed: a later dequeue
 * must not launch it again (its dematch may already have combined the LLRs into the HARQ soft buffers). */
int hal_launch(ldpc_hip_ctx* ctx)
{
  bool issued = false;
  int  r      = LDPC_HIP_ENOMEM;
  try {
    r = hal_launch_issue(ctx, issued);
  } catch (const std::bad_alloc&) {
    ctx->err = "out of host memory (HAL launch)";
  }
  if (r != LDPC_HIP_OK && issued) {
    ctx->hstate = hal_state::failed;
    /* whatever part of the batch reached the stream ends before the done event (the HARQ memory's grow waits on it) */
    (void)hipEventRecord(ctx->done_event, ctx->hq_stream);
  }
  return r;
}

/* The device's shared hardware queues: HIP streams a context borrows per TB when opened with
 * LDPC_HIP_LAUNCH_SHARED_QUEUE, as acc100 without a dedicated queue reserves a bbdev queue in reserve_queue, spinning
 * until one is free, and frees it in free_queue (hw_accelerator_pusch_dec_acc100_impl.cpp:70-98). The pool holds
 * LDPC_HIP_SHARED_QUEUES streams (environment; default 4 = GPU_MAX_HW_QUEUES' default, one stream per hardware queue)
 * and lives as long as the process. */
struct shared_queue_pool {
  std::mutex               mu;
  std::vector<hipStream_t> streams;
  std::vector<uint8_t>     busy;
};

shared_queue_pool* queue_pool(int device)
{
  static std::mutex                                       mu;
  static std::map<int, std::unique_ptr<shared_queue_pool>> pools;
  std::lock_guard<std::mutex>                             lock(mu);
  std::unique_ptr<shared_queue_pool>&                     p = pools[device];
  if (!p) {
    p            = std::make_unique<shared_queue_pool>();
    const char* v = std::getenv("LDPC_HIP_SHARED_QUEUES");
    const int   n = std::max(1, std::min(64, v != nullptr ? std::atoi(v) : 4));
    (void)hipSetDevice(device);
    for (int i = 0; i != n; ++i) {
      hipStream_t st = nullptr;
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        break;
      }
      p->streams.push_back(st);
      p->busy.push_back(0);
    }
  }
  return p->streams.empty() ? nullptr : p.get();
}

/* reserve_queue without a dedicated queue: the index of a free shared queue, spinning (yielding) until one is */
int acquire_shared_queue(shared_queue_pool* p, hipStream_t& s)
{
  while (true) {
    {
      std::lock_guard<std::mutex> lock(p->mu);
      for (size_t i = 0; i != p->streams.size(); ++i) {
        if (p->busy[i] == 0) {
          p->busy[i] = 1;
          s          = p->streams[i];
          return static_cast<int>(i);
        }
      }
    }
    std::this_thread::yield();
  }
}

void release_shared_queue(ldpc_hip_ctx* ctx)
{
  if (ctx->hq_shared >= 0) {
    shared_queue_pool*          p = queue_pool(ctx->device);
    std::lock_guard<std::mutex> lock(p->mu);
    p->busy[static_cast<size_t>(ctx->hq_shared)] = 0;
    ctx->hq_shared                                = -1;
    ctx->hq_stream                                = ctx->stream;
  }
}

hal_op* hal_find(ldpc_hip_ctx* ctx, uint32_t cb_index)
{
  if (cb_index >= ctx->hslot.size() || ctx->hslot[cb_index] < 0) {
    return nullptr;
  }
  return &ctx->hops[static_cast<size_t>(ctx->hslot[cb_index])];
}

} // namespace

extern "C" {

} /* extern "C" */
namespace ldpc_hip {
/* the context's launch flags, for the PDSCH encoder queue (ldpc_hip_enc_queue.cpp) */
uint32_t ctx_launch_flags(const ldpc_hip_ctx* ctx) { return ctx != nullptr ? ctx->params.launch_flags : 0U; }
hipStream_t ctx_hal_stream(const ldpc_hip_ctx* ctx) { return ctx != nullptr ? ctx->hq_stream : nullptr; }
} // namespace ldpc_hip
extern "C" {

int ldpc_hip_external_harq_supported(const ldpc_hip_ctx* ctx)
{
  return (ctx != nullptr && ctx->repo != nullptr) ? 1 : 0;
}

int ldpc_hip_queue_reserve(ldpc_hip_ctx* ctx)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  hal_sync(ctx);
  hal_reset(ctx, hal_state::staging);
  if ((ctx->params.launch_flags & LDPC_HIP_LAUNCH_SHARED_QUEUE) != 0 && ctx->hq_shared < 0) {
    shared_queue_pool* p = queue_pool(ctx->device);
    if (p == nullptr) {
      return ctx->fail(LDPC_HIP_EDEVICE, "no shared hardware queue could be created");
    }
    ctx->hq_shared = acquire_shared_queue(p, ctx->hq_stream);
  }
  return LDPC_HIP_OK;
}

int ldpc_hip_queue_free(ldpc_hip_ctx* ctx)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  hal_sync(ctx);
  hal_reset(ctx, hal_state::idle);
  release_shared_queue(ctx);
  return LDPC_HIP_OK;
}

/* HAL operation indices: a TB has at most MAX_NOF_SEGMENTS = 162 codeblocks (sch_constants.h:38); larger indices are
 * contract violations, not a reason to grow the index table without bound */
constexpr uint32_t HAL_MAX_CB_INDEX = 4U * 162U;

static int hal_enqueue(ldpc_hip_ctx* ctx, uint32_t cb_index, const ldpc_hip_hw_config* cfg, const int8_t* llrs,
                       uint32_t nof_llrs, const int8_t* soft_in, uint32_t soft_len)
{
  if (ctx->hstate == hal_state::idle) {
    return ctx->fail(LDPC_HIP_ESTATE, "enqueue without a reserved queue");
  }
  if (ctx->hstate == hal_state::failed) {
    return ctx->fail(LDPC_HIP_ESTATE, "the batch failed to launch: free or reserve the queue again");
  }
  if (ctx->hstate == hal_state::launched) {
    if (ctx->hdequeued != ctx->hops.size()) {
      /* the batch is in flight: dequeue its operations first, then enqueue again (pusch_decoder_hw_impl.cpp:
       * 237-241 breaks out of its enqueue loop on false and dequeues) */
      return ctx->fail(LDPC_HIP_EFULL, "batch in flight");
    }
    hal_reset(ctx, hal_state::staging); /* every operation dequeued: a new batch on the same reservation */
  }
  const int      bg = cfg->base_graph;
  const unsigned Z  = cfg->lifting_size;
  const unsigned N  = (bg == 1 ? 66U : 50U) * Z;
  ldpc_hip_dematch_desc dd{static_cast<uint8_t>(cfg->modulation_order), static_cast<uint8_t>(cfg->rv),
                           static_cast<uint8_t>(cfg->new_data), 0, N, cfg->cw_length, cfg->Nref,
                           cfg->nof_filler_bits};
  if (cb_index >= HAL_MAX_CB_INDEX || graph_slot(bg, Z) < 0 || validate_dematch(ctx, dd) != LDPC_HIP_OK ||
      cfg->cw_length != nof_llrs || nof_llrs > ctx->params.max_cb_llrs || cfg->max_nof_ldpc_iterations == 0 ||
      cfg->max_nof_ldpc_iterations > 255 || cfg->cb_crc_type > 2) {
    return ctx->fail(LDPC_HIP_EINVAL, "invalid HAL operation configuration");
  }
  const bool ext = ctx->repo != nullptr;
  if (ext && ctx->repo->caller_state) {
    /* the device's HARQ memory holds any absolute_cb_id the caller's repository hands out: grow to it */
    const hipError_t ge = ctx->repo->grow(cfg->absolute_cb_id);
    if (ge != hipSuccess) {
      return ge == hipErrorInvalidValue ? ctx->fail(LDPC_HIP_EINVAL, "absolute CB index beyond 2^20")
                                        : ctx->hip_fail(ge, "HARQ memory growth");
    }
  } else if (ext && cfg->absolute_cb_id >= ctx->repo->nof_codeblocks) {
    /* ext_harq_buffer_context_repository::get asserts (ext_harq_buffer_context_repository.h:70-73) */
    return ctx->fail(LDPC_HIP_EINVAL, "absolute CB index out of the HARQ repository's bounds");
  }
  if (!ext && soft_in != nullptr && soft_len != 0 && soft_len != N) {
    return ctx->fail(LDPC_HIP_EINVAL, "soft buffer size differs from the codeblock length");
  }
  hal_op* existing = hal_find(ctx, cb_index);
  if (existing == nullptr && ctx->hops.size() >= ctx->params.max_queue_cbs) {
    return ctx->fail(LDPC_HIP_EFULL, "HAL batch full"); /* dequeue the batch, then enqueue again */
  }
  /* staging space (pinned; grows, keeping what is staged) */
  const uint64_t llr_off  = ctx->h_llr_used;
  const uint64_t soft_off = ctx->h_soft_used;
  const uint64_t out_off  = ctx->h_out_used;
  const unsigned mb       = msg_bytes_of(bg, Z);
  hipError_t     e;
  /* a large batch (more codeblocks than the work queue takes) with external HARQ stages its LLRs into HBM early */
  if (ctx->hops.empty()) {
    ctx->hcopy   = ext && cfg->nof_segments > HAL_DWQ_MAX_CBS && (hal_early_copy(ctx) || hal_dwq_copy(ctx));
    dwq_unpin(ctx->hcopy_q);
    ctx->hcopy_q = nullptr;
    if (ctx->hcopy && !hal_early_copy(ctx)) { /* the copy work queue, if a grid can serve it now */
      dwq* q       = dwq_get(ctx->device, DWQ_KEY_COPY, COPY_THREADS, 0);
      ctx->hcopy_q = (q != nullptr && dwq_admit(q)) ? q : nullptr;
      ctx->hcopy   = ctx->hcopy_q != nullptr;
    }
    if (ctx->hcopy) { /* room for the whole batch up front, so the staging buffers do not move under queued copies */
      const uint64_t want = static_cast<uint64_t>(cfg->nof_segments) * (((nof_llrs + 15U) & ~15U) + 256U) + 65536U;
      if ((e = hal_reserve_llr(ctx, want, 0)) != hipSuccess || (e = ctx->q_llr.reserve(want)) != hipSuccess) {
        return ctx->hip_fail(e, "HAL staging");
      }
    }
  }
  if ((e = hal_reserve_llr(ctx, llr_off + ((nof_llrs + 15U) & ~15U), llr_off)) != hipSuccess ||
      (e = ctx->h_out.reserve(out_off + ((mb + 15U) & ~15U), 0)) != hipSuccess ||
      (!ext && (e = ctx->h_soft.reserve(soft_off + ((N + 15U) & ~15U), soft_off)) != hipSuccess)) {
    return ctx->hip_fail(e, "hipHostMalloc(HAL staging)");
  }
  hal_op op{};
  op.cb_index  = cb_index;
  op.cfg       = *cfg;
  op.N         = N;
  op.msg_bytes = mb;
  op.llr_off   = llr_off;
  op.out_off   = out_off;
  if (ext) {
    /* hw_config + hw_enqueue of hw_accelerator_pusch_dec_acc100_impl.cpp:113, 123-125, 182-185: the entry is
     * (re)initialised on new data; a retransmission whose entry holds no soft data is dropped */
    /* (with the caller keeping the entry state, the caller has decided already: nothing is dropped here) */
    const uint32_t soft_len_now = ctx->repo->caller_state ? 1U : ctx->repo->get(cfg->absolute_cb_id, cfg->new_data != 0);
    op.dropped                  = cfg->new_data == 0 && soft_len_now == 0;
    op.soft_off                 = static_cast<uint64_t>(cfg->absolute_cb_id) * LDPC_HIP_HARQ_STRIDE;
  } else {
    op.soft_off = soft_off;
    int8_t* dst = ctx->h_soft.as<int8_t>() + soft_off;
    if (soft_in != nullptr && soft_len != 0) {
      std::memcpy(dst, soft_in, N);
    } else {
      std::memset(dst, 0, N); /* a clean buffer (rx_buffer, pusch_decoder_impl.cpp:327) */
    }
    ctx->h_soft_used = soft_off + ((N + 15U) & ~15U);
  }
  if (nof_llrs != 0) {
    std::memcpy(ctx->h_llr.as<int8_t>() + llr_off, llrs, nof_llrs);
  }
  ctx->h_llr_used = llr_off + ((nof_llrs + 15U) & ~15U);
  ctx->h_out_used = out_off + ((mb + 15U) & ~15U);
  if (ctx->hcopy && existing == nullptr && (e = hal_copy_staged(ctx, false, ctx->h_llr_used)) != hipSuccess) {
    return ctx->hip_fail(e, "HAL early copy");
  }
  if (existing != nullptr) {
    *existing = op; /* the same codeblock enqueued again before the launch: the later configuration wins */
  } else {
    if (cb_index >= ctx->hslot.size()) {
      ctx->hslot.resize(static_cast<size_t>(cb_index) + 1, -1);
    }
    ctx->hslot[cb_index] = static_cast<int32_t>(ctx->hops.size());
    ctx->hops.push_back(op);
  }
  return op.dropped ? LDPC_HIP_DROPPED : LDPC_HIP_OK;
}

int ldpc_hip_enqueue(ldpc_hip_ctx* ctx, uint32_t cb_index, const ldpc_hip_hw_config* cfg, const int8_t* llrs,
                     uint32_t nof_llrs, const int8_t* soft_in, uint32_t soft_len)
{
  if (ctx == nullptr || cfg == nullptr || (nof_llrs != 0 && llrs == nullptr)) {
    return LDPC_HIP_EINVAL;
  }
  try {
    return hal_enqueue(ctx, cb_index, cfg, llrs, nof_llrs, soft_in, soft_len);
  } catch (const std::bad_alloc&) {
    return ctx->fail(LDPC_HIP_ENOMEM, "out of host memory (enqueue)");
  }
}

int ldpc_hip_dequeue(ldpc_hip_ctx* ctx, uint32_t cb_index, uint8_t* packed_msg, uint32_t msg_bytes, int8_t* soft_out,
                     uint32_t soft_len)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  hal_op* op = hal_find(ctx, cb_index);
  if (op == nullptr) {
    return ctx->fail(LDPC_HIP_ESTATE, "dequeue of an operation that was not enqueued");
  }
  if (ctx->hstate == hal_state::failed) {
    return ctx->fail(LDPC_HIP_EDEVICE, "the batch failed to launch: " + ctx->err);
  }
  if (ctx->hstate == hal_state::staging) {
    int r = hal_launch(ctx);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    op = hal_find(ctx, cb_index);
  }
  if (op->q != nullptr) {
    if (!dwq_done(op->q, op->ticket)) {
      return LDPC_HIP_NOT_READY; /* this codeblock's work item (a work-queue batch completes CB by CB) */
    }
  } else if (!ctx->hbatch_done) {
    hipError_t q = hipEventQuery(ctx->done_event);
    if (q == hipErrorNotReady) {
      return LDPC_HIP_NOT_READY;
    }
    if (q != hipSuccess) {
      return ctx->hip_fail(q, "hipEventQuery");
    }
    ctx->hbatch_done = true;
  }
  if (op->dropped) {
    op->res.crc_pass       = 0;
    op->res.nof_iterations = static_cast<uint8_t>(op->cfg.max_nof_ldpc_iterations);
    op->res.status         = LDPC_HIP_STATUS_DROPPED;
  } else {
    op->res = reinterpret_cast<const ldpc_hip_cb_result*>(ctx->h_out.as<uint8_t>() + ctx->h_res_off)[op->pos];
    if (op->res.crc_pass == 0) {
      op->res.nof_iterations = static_cast<uint8_t>(op->cfg.max_nof_ldpc_iterations); /* acc100_impl.cpp:246 */
    }
    if (packed_msg != nullptr && (op->res.status & LDPC_HIP_STATUS_OUTPUT_WRITTEN)) {
      std::memcpy(packed_msg, ctx->h_out.as<uint8_t>() + op->out_off, std::min(op->msg_bytes, msg_bytes));
    }
    if (ctx->repo == nullptr && soft_out != nullptr) {
      std::memcpy(soft_out, ctx->h_soft.as<int8_t>() + op->soft_off, std::min<uint32_t>(op->N, soft_len));
    }
    if (ctx->repo != nullptr && !ctx->repo->caller_state && !op->dequeued) {
      /* the entry now holds the codeblock's soft data (acc100 hw_dequeue, acc100_impl.cpp:206-207) */
      ctx->repo->set_len(op->cfg.absolute_cb_id, op->N);
    }
  }
  if (!op->dequeued) {
    op->dequeued = true;
    ++ctx->hdequeued;
  }
  return LDPC_HIP_OK;
}

int ldpc_hip_read_outputs(ldpc_hip_ctx* ctx, uint32_t cb_index, uint32_t absolute_cb_id, ldpc_hip_cb_result* out)
{
  (void)absolute_cb_id;
  if (ctx == nullptr || out == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  const hal_op* op = hal_find(ctx, cb_index);
  if (op == nullptr || !op->dequeued) {
    return ctx->fail(LDPC_HIP_ESTATE, "read_operation_outputs before dequeue");
  }
  *out = op->res;
  return LDPC_HIP_OK;
}

int ldpc_hip_harq_free(ldpc_hip_ctx* ctx, uint32_t absolute_cb_id)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (ctx->repo != nullptr && !ctx->repo->caller_state) { /* caller_state: the caller frees its own entry */
    if (absolute_cb_id >= ctx->repo->nof_codeblocks) {
      return ctx->fail(LDPC_HIP_EINVAL, "absolute CB index out of the HARQ repository's bounds"); /* :89-91 */
    }
    ctx->repo->free(absolute_cb_id);
  }
  return LDPC_HIP_OK;
}

} /* extern "C" */

/* ---- soft demodulation mapper ----------------------------------------------------- */
namespace {
int demodulate_segments(ldpc_hip_ctx* ctx, uint32_t nof_segs, const ldpc_hip_demod_desc* descs, const float* d_sym,
                        const float* d_nv, int8_t* d_llr, hipStream_t s)
{
  std::vector<demod_seg> sg;
  sg.reserve(nof_segs);
  uint32_t blocks = 0;
  for (uint32_t i = 0; i != nof_segs; ++i) {
    const ldpc_hip_demod_desc& d = descs[i];
    if (!valid_modulation(d.modulation)) {
      return ctx->fail(LDPC_HIP_EINVAL, "demodulate: invalid modulation scheme");
    }
    if (d.nof_symbols == 0) {
      continue;
    }
    demod_seg g{};
    g.sym_offset   = d.symbol_offset;
    g.noise_offset = d.noise_offset;
    g.llr_offset   = d.llr_offset;
    g.nof_symbols  = d.nof_symbols;
    g.block0       = blocks;
    g.modulation   = d.modulation;
    g.qm           = static_cast<uint8_t>(bits_per_symbol(d.modulation));
    sg.push_back(g);
    blocks += (d.nof_symbols + DEMOD_BLOCK - 1) / DEMOD_BLOCK;
  }
  if (sg.empty()) {
    return LDPC_HIP_OK;
  }
  hipError_t e = upload_descs(ctx->d_dmsegs, ctx->c_dmsegs, sg.data(), sg.size() * sizeof(demod_seg), s);
  if (e == hipSuccess) {
    e = launch_demodulate(ctx->d_dmsegs.as<demod_seg>(), static_cast<uint32_t>(sg.size()), blocks, ctx->dtab, d_sym,
                          d_nv, d_llr, s);
  }
  return e == hipSuccess ? LDPC_HIP_OK : ctx->hip_fail(e, "ldpc_demodulate_kernel launch");
}
} // namespace

int ldpc_hip_demodulate_launch(ldpc_hip_ctx* ctx, uint32_t nof_segs, const ldpc_hip_demod_desc* descs,
                               const float* d_symbols, const float* d_noise_vars, int8_t* d_llrs, void* stream)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (nof_segs == 0) {
    return LDPC_HIP_OK;
  }
  if (descs == nullptr || d_symbols == nullptr || d_noise_vars == nullptr || d_llrs == nullptr) {
    return ctx->fail(LDPC_HIP_EINVAL, "demodulate_launch: null argument");
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = abi_stream(ctx->stream, stream);
  return demodulate_segments(ctx, nof_segs, descs, d_symbols, d_noise_vars, d_llrs, s);
}

int ldpc_hip_demodulate_sync(ldpc_hip_ctx* ctx, uint32_t nof_symbols, int modulation, const float* symbols,
                             const float* noise_vars, int8_t* llrs)
{
  if (ctx == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (!valid_modulation(modulation)) {
    return ctx->fail(LDPC_HIP_EINVAL, "demodulate: invalid modulation scheme");
  }
  if (nof_symbols == 0) {
    return LDPC_HIP_OK;
  }
  if (symbols == nullptr || noise_vars == nullptr || llrs == nullptr) {
    return ctx->fail(LDPC_HIP_EINVAL, "demodulate_sync: null argument");
  }
  (void)hipSetDevice(ctx->device);
  const size_t nllr = static_cast<size_t>(nof_symbols) * bits_per_symbol(modulation);
  hipError_t   e;
  if ((e = ctx->d_sym.reserve(static_cast<size_t>(nof_symbols) * 8)) != hipSuccess ||
      (e = ctx->d_nv.reserve(static_cast<size_t>(nof_symbols) * 4)) != hipSuccess ||
      (e = ctx->d_llr.reserve(nllr)) != hipSuccess) {
    return ctx->hip_fail(e, "hipMalloc(demodulate)");
  }
  if ((e = hipMemcpyAsync(ctx->d_sym.ptr, symbols, static_cast<size_t>(nof_symbols) * 8, hipMemcpyHostToDevice,
                          ctx->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(ctx->d_nv.ptr, noise_vars, static_cast<size_t>(nof_symbols) * 4, hipMemcpyHostToDevice,
                          ctx->stream)) != hipSuccess) {
    return ctx->hip_fail(e, "hipMemcpyAsync(demodulate in)");
  }
  ldpc_hip_demod_desc d{};
  d.nof_symbols = nof_symbols;
  d.modulation  = static_cast<uint8_t>(modulation);
  const int r   = demodulate_segments(ctx, 1, &d, ctx->d_sym.as<float>(), ctx->d_nv.as<float>(),
                                      ctx->d_llr.as<int8_t>(), ctx->stream);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  if ((e = hipMemcpyAsync(llrs, ctx->d_llr.ptr, nllr, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(ctx->stream)) != hipSuccess) {
    return ctx->hip_fail(e, "demodulate_sync");
  }
  return LDPC_HIP_OK;
}
