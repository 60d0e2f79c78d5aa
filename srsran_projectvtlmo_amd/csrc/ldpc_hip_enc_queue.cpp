/*
 * PDSCH encoder queue behind the C ABI (include/srsran_ldpc_hip.h, "HAL queue: hw_accelerator_pdsch_enc"): the
 * hal::hw_accelerator_pdsch_enc operations (include/srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc.h:
 * 75-102) on one GPU, in the call order pdsch_encoder_hw_impl::encode uses (pdsch_encoder_hw_impl.cpp:31-170).
 *
 * What an operation computes is what the reference's accelerator returns (hw_accelerator_pdsch_enc_acc100_impl.cpp,
 * bbdev_ldpc_encoder.cpp:188-241): the rate-matched bits of one codeblock (CB mode) or of every codeblock of a TB
 * (TB mode: TB CRC attached, segmented into nof_segments codeblocks of nof_segment_bits data bits, CB CRC24B attached
 * when there is more than one, filler bits added; TS 38.212 5.1-5.2), each LDPC-encoded (ldpc_encoder_impl.cpp:47-81)
 * and rate-matched to E bits (ldpc_rate_matcher_impl.cpp:36-160; Ea for the first nof_short_segments codeblocks, Eb
 * for the others). The encoding and rate matching run on the device (ldpc_encode_kernel, ldpc_rate_match_kernel); the
 * segmentation of a TB is a byte-level host copy into the pinned staging buffer.
 */
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "ldpc_hip_buffers.h"
#include "srsran_ldpc_hip.h"

using namespace ldpc_hip;

namespace ldpc_hip {
uint32_t    ctx_launch_flags(const ldpc_hip_ctx* ctx); /* ldpc_hip_api.cpp */
hipStream_t ctx_hal_stream(const ldpc_hip_ctx* ctx);   /* the HAL queue's current stream (ldpc_hip_api.cpp) */
size_t pdsch_enc_desc_bytes(); /* ldpc_hip_api.cpp */
int    pdsch_encode_submit(ldpc_hip_ctx* ctx, uint32_t n, const ldpc_hip_enc_desc* ed, const uint32_t* ext,
                           const ldpc_hip_rm_desc* rd, const uint8_t* d_msgs, uint8_t* d_out, void** qo,
                           uint32_t* tickets);
bool   pdsch_encode_done(void* q, uint32_t ticket);
int    pdsch_encode_wait(void* q, uint32_t ticket);
int    pdsch_encode_launch(ldpc_hip_ctx* ctx, uint32_t n, const ldpc_hip_enc_desc* ed, const uint32_t* ext,
                           const ldpc_hip_rm_desc* rd, const uint8_t* d_msgs, uint8_t* d_out, void* h_desc,
                           const void* d_desc, void* stream);
} // namespace ldpc_hip

namespace {

constexpr uint32_t MAX_NOF_SEGMENTS = 162;    /* sch_constants.h:38 */
constexpr uint32_t MAX_TB_BYTES     = 159749; /* the largest NR TBS (1,277,992 bits) in bytes */

uint64_t align16(uint64_t x) { return (x + 15U) & ~static_cast<uint64_t>(15U); }

bool valid_lifting_size(uint32_t z)
{
  static const uint32_t a_set[8] = {2, 3, 5, 7, 9, 11, 13, 15};
  for (uint32_t a : a_set) {
    for (uint32_t v = a; v <= 384; v *= 2) {
      if (v == z) {
        return true;
      }
    }
  }
  return false;
}

uint32_t bits_per_symbol(uint8_t m) { return (m == 0 || m == 1) ? 1U : m; }
bool     valid_modulation(uint8_t m) { return m == 0 || m == 1 || m == 2 || m == 4 || m == 6 || m == 8; }

/* byte -> its eight bits, MSB first, one per byte (little-endian uint64 image) */
struct unpack_table {
  uint64_t t[256];
  unpack_table()
  {
    for (uint32_t b = 0; b != 256; ++b) {
      uint64_t v = 0;
      for (int i = 0; i != 8; ++i) {
        v |= static_cast<uint64_t>((b >> (7 - i)) & 1U) << (8 * i);
      }
      t[b] = v;
    }
  }
};

/* src's first n bytes -> 8 n bytes of one bit each, MSB first: four source bytes per 32 output bytes (broadcast,
 * byte shuffle, bit mask, compare); the host's AVX2 when it has it, else the table */
__attribute__((target("avx2"))) void unpack_bits_avx2(uint8_t* dst, const uint8_t* src, uint32_t n)
{
  const __m256i shuf = _mm256_setr_epi8(0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3,
                                        3, 3, 3, 3, 3);
  const __m256i bitm = _mm256_setr_epi8(-128, 64, 32, 16, 8, 4, 2, 1, -128, 64, 32, 16, 8, 4, 2, 1, -128, 64, 32, 16, 8,
                                        4, 2, 1, -128, 64, 32, 16, 8, 4, 2, 1);
  const __m256i one  = _mm256_set1_epi8(1);
  uint32_t      j    = 0;
  for (; j + 4 <= n; j += 4) {
    uint32_t w;
    std::memcpy(&w, src + j, 4);
    const __m256i v = _mm256_shuffle_epi8(_mm256_set1_epi32(static_cast<int>(w)), shuf);
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + 8 * j),
                        _mm256_and_si256(_mm256_cmpeq_epi8(_mm256_and_si256(v, bitm), bitm), one));
  }
  static const unpack_table tab;
  for (; j < n; ++j) {
    std::memcpy(dst + 8 * j, &tab.t[src[j]], 8);
  }
}

void unpack_bits(uint8_t* dst, const uint8_t* src, uint32_t n)
{
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) {
    unpack_bits_avx2(dst, src, n);
    return;
  }
  static const unpack_table tab;
  for (uint32_t j = 0; j != n; ++j) {
    std::memcpy(dst + 8 * j, &tab.t[src[j]], 8);
  }
}

/* One codeblock of the batch. */
struct enc_unit {
  uint64_t msg_off; /* its message's first byte in the message staging arena */
  uint32_t bit_off; /* its first bit in that byte (a TB-mode segment read in place) */
  uint32_t data_bits;
  uint32_t crc_at;  /* TB mode with more than one segment: the CRC24B the device attaches at bit S */
  uint64_t out_off; /* ceil(E / 8) bytes in the output arena       */
  uint32_t E;
  uint32_t N;
  uint16_t Z;
  uint8_t  bg;
  uint8_t  Qm;
  uint8_t  rv;
  uint32_t Nref;
  uint32_t F;
};

/* One enqueued operation: a codeblock (CB mode) or a TB (a run of codeblocks). */
struct enc_op {
  uint32_t cb_index  = 0;
  uint32_t unit0     = 0;
  uint32_t nof_units = 0;
  bool     dequeued  = false;
};

enum class enc_state { idle, staging, launched };

} // namespace

struct ldpc_hip_enc_queue {
  ldpc_hip_ctx*                       ctx    = nullptr;
  hipStream_t                         stream = nullptr;
  int                                 device = 0;
  bool                                cb_mode = true;
  uint32_t                            max_cbs = MAX_NOF_SEGMENTS;
  uint32_t                            max_tb  = MAX_TB_BYTES;
  std::vector<ldpc_hip_enc_hw_config> cfgs;
  std::vector<uint8_t>                cfg_set;
  std::vector<enc_unit>               units;
  std::vector<enc_op>                 ops;
  std::vector<int32_t>                op_of_cb; /* cb_index -> ops index, -1 */
  uint32_t                            ndequeued = 0;
  enc_state                           state     = enc_state::idle;
  uint64_t                            msg_used = 0, out_used = 0;
  pinned_buffer                       h_msg, h_out, h_desc;
  void*                               wq = nullptr; /* the batch went through the encoder's work queue      */
  std::vector<uint32_t>               tickets;      /* its items' tickets (0xffffffff: not published)      */
  bool                                complete = false;
  dev_buffer                          d_msg, d_out;
  hipEvent_t                          done = nullptr;

  /* small zero-copy batches go through the encoder's device work queue (no launch per batch) */
  static constexpr size_t ENC_DWQ_MAX_CBS = 8;
  void reset(enc_state next)
  {
    wq = nullptr;
    tickets.clear();
    complete = false;
    for (const enc_op& op : ops) {
      if (op.cb_index < op_of_cb.size()) {
        op_of_cb[op.cb_index] = -1;
      }
    }
    ops.clear();
    units.clear();
    ndequeued = 0;
    msg_used = out_used = 0;
    state                         = next;
  }
  void sync()
  {
    if (wq != nullptr) { /* every published item, also after a failed submit */
      for (uint32_t t : tickets) {
        (void)ldpc_hip::pdsch_encode_wait(wq, t);
      }
      complete = true;
    } else if (state == enc_state::launched) {
      (void)hipEventSynchronize(done);
    }
  }
  /* the batch: encode + rate match of every unit in one launch (ldpc_pdsch_encode_kernel: the codeword stays in
   * LDS; one codeblock's descriptor goes by value, more are read in place from the pinned h_desc, so no descriptor
   * upload precedes the kernel). For a zero-copy batch (at most ENC_ZERO_COPY_MAX_BYTES staged and produced) the
   * kernel reads the messages straight from the pinned staging buffer and writes straight into the pinned output
   * buffer (mapped host memory; the HAL decoder queue does the same, ldpc_hip_api.cpp hal_launch); otherwise one H2D
   * of the messages and one D2H of the packed outputs around it. */
  static constexpr uint64_t ENC_ZERO_COPY_MAX_BYTES = 1024U * 1024U;
  int launch()
  {
    if (wq != nullptr) { /* items a failed submit left published still use the staging buffers */
      sync();
      wq = nullptr;
      tickets.clear();
      complete = false;
    }
    if (units.empty()) {
      state = enc_state::launched;
      return hipEventRecord(done, stream) == hipSuccess ? LDPC_HIP_OK : LDPC_HIP_EDEVICE;
    }
    (void)hipSetDevice(device);
    if (d_msg.reserve(msg_used) != hipSuccess || d_out.reserve(out_used) != hipSuccess ||
        h_out.reserve(out_used, 0) != hipSuccess ||
        h_desc.reserve(units.size() * ldpc_hip::pdsch_enc_desc_bytes(), 0) != hipSuccess) {
      return LDPC_HIP_EDEVICE;
    }
    std::vector<ldpc_hip_enc_desc> ed(units.size());
    std::vector<ldpc_hip_rm_desc>  rd(units.size());
    std::vector<uint32_t>          ext(3 * units.size());
    for (size_t i = 0; i != units.size(); ++i) {
      const enc_unit& u = units[i];
      ed[i]             = ldpc_hip_enc_desc{u.msg_off, 0, u.N, u.Z, u.bg, 0};
      ext[3 * i]        = u.bit_off;
      ext[3 * i + 1]    = u.data_bits;
      ext[3 * i + 2]    = u.crc_at;
      rd[i]             = ldpc_hip_rm_desc{0, u.out_off, u.N, u.E, u.Nref, static_cast<uint16_t>(u.F), u.Qm, u.rv};
    }
    const bool zc = msg_used + out_used <= ENC_ZERO_COPY_MAX_BYTES && h_msg.dev != nullptr && h_out.dev != nullptr &&
                    (ldpc_hip::ctx_launch_flags(ctx) & LDPC_HIP_LAUNCH_HAL_COPY) == 0;
    uint8_t* const msg = zc ? h_msg.dev_as<uint8_t>() : d_msg.as<uint8_t>();
    uint8_t* const out = zc ? h_out.dev_as<uint8_t>() : d_out.as<uint8_t>();
    if (zc && units.size() <= ENC_DWQ_MAX_CBS) {
      tickets.assign(units.size(), 0xffffffffU);
      const int w = ldpc_hip::pdsch_encode_submit(ctx, static_cast<uint32_t>(units.size()), ed.data(), ext.data(),
                                                  rd.data(), msg, out, &wq, tickets.data());
      if (w == LDPC_HIP_OK) {
        state = enc_state::launched;
        return LDPC_HIP_OK;
      }
      if (w != 1) {
        return w; /* sync() waits for the items published before the error */
      }
      wq = nullptr;
      tickets.clear();
    }
    if (!zc && hipMemcpyAsync(d_msg.ptr, h_msg.ptr, msg_used, hipMemcpyHostToDevice, stream) != hipSuccess) {
      return LDPC_HIP_EDEVICE;
    }
    const int r = ldpc_hip::pdsch_encode_launch(ctx, static_cast<uint32_t>(units.size()), ed.data(), ext.data(),
                                                rd.data(), msg, out, h_desc.ptr, h_desc.dev, stream);
    if (r != LDPC_HIP_OK) {
      return r;
    }
    if ((!zc && hipMemcpyAsync(h_out.ptr, d_out.ptr, out_used, hipMemcpyDeviceToHost, stream) != hipSuccess) ||
        hipEventRecord(done, stream) != hipSuccess) {
      return LDPC_HIP_EDEVICE;
    }
    state = enc_state::launched;
    return LDPC_HIP_OK;
  }
  /* a region of `bytes` message bytes in the staging arena (8 zero bytes after them: the device reads a 40-bit window),
   * nullptr on failure; its offset in *off */
  uint8_t* stage(uint64_t bytes, uint64_t* off)
  {
    *off            = msg_used;
    const uint64_t n = align16(msg_used + bytes + 8);
    if (h_msg.reserve(n, msg_used) != hipSuccess) {
      return nullptr;
    }
    uint8_t* p = h_msg.as<uint8_t>() + msg_used;
    std::memset(p + bytes, 0, n - msg_used - bytes);
    msg_used = n;
    return p;
  }
  /* appends a codeblock unit whose message is data_bits bits from bit bit_off of staged byte msg_off */
  void add_unit(uint8_t bg, uint32_t Z, uint32_t E, const ldpc_hip_enc_hw_config& c, uint64_t msg_off,
                uint32_t bit_off, uint32_t data_bits, uint32_t crc_at)
  {
    enc_unit u{};
    u.bg        = bg;
    u.Z         = static_cast<uint16_t>(Z);
    u.N         = (bg == 1 ? 66U : 50U) * Z;
    u.E         = E;
    u.Qm        = static_cast<uint8_t>(bits_per_symbol(c.modulation));
    u.rv        = c.rv;
    u.Nref      = c.Nref;
    u.F         = c.nof_filler_bits;
    u.msg_off   = msg_off;
    u.bit_off   = bit_off;
    u.data_bits = data_bits;
    u.crc_at    = crc_at;
    u.out_off   = out_used;
    out_used    = align16(out_used + (E + 7) / 8);
    units.push_back(u);
  }
};

extern "C" {

int ldpc_hip_enc_queue_create(ldpc_hip_ctx* ctx, int cb_mode, uint32_t max_queue_cbs, uint32_t max_tb_bytes,
                              ldpc_hip_enc_queue** queue)
{
  if (ctx == nullptr || queue == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  *queue = nullptr;
  auto* q = new (std::nothrow) ldpc_hip_enc_queue();
  if (q == nullptr) {
    return LDPC_HIP_EDEVICE;
  }
  q->ctx     = ctx;
  q->stream  = static_cast<hipStream_t>(ldpc_hip_stream(ctx));
  q->cb_mode = cb_mode != 0;
  q->max_cbs = max_queue_cbs != 0 ? max_queue_cbs : MAX_NOF_SEGMENTS;
  q->max_tb  = max_tb_bytes != 0 ? max_tb_bytes : MAX_TB_BYTES;
  if (hipStreamGetDevice(q->stream, &q->device) != hipSuccess || hipSetDevice(q->device) != hipSuccess ||
      hipEventCreateWithFlags(&q->done, hipEventDisableTiming) != hipSuccess) {
    delete q;
    return LDPC_HIP_EDEVICE;
  }
  *queue = q;
  return LDPC_HIP_OK;
}

int ldpc_hip_enc_queue_destroy(ldpc_hip_enc_queue* q)
{
  if (q == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  q->sync();
  (void)hipEventDestroy(q->done);
  delete q;
  return LDPC_HIP_OK;
}

int ldpc_hip_enc_reserve(ldpc_hip_enc_queue* q)
{
  if (q == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  q->sync();
  q->reset(enc_state::staging);
  /* the context's HAL queue: its own stream, or (LDPC_HIP_LAUNCH_SHARED_QUEUE, dedicated_queue == false) one of the
   * device's shared streams until free_queue (hw_accelerator_pdsch_enc_acc100_impl.cpp:62-88) */
  const int r = ldpc_hip_queue_reserve(q->ctx);
  if (r != LDPC_HIP_OK) {
    return r;
  }
  q->stream = ldpc_hip::ctx_hal_stream(q->ctx);
  return LDPC_HIP_OK;
}

int ldpc_hip_enc_free(ldpc_hip_enc_queue* q)
{
  if (q == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  q->sync();
  q->reset(enc_state::idle);
  const int r = ldpc_hip_queue_free(q->ctx);
  q->stream   = ldpc_hip::ctx_hal_stream(q->ctx);
  return r;
}

int ldpc_hip_enc_configure(ldpc_hip_enc_queue* q, uint32_t cb_index, const ldpc_hip_enc_hw_config* cfg)
{
  if (q == nullptr || cfg == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  const ldpc_hip_enc_hw_config& c = *cfg;
  const uint32_t                Qm = bits_per_symbol(c.modulation);
  /* cb_index: a segment index (CB mode) or 0 (TB mode); bounded so that a stray index cannot grow the tables */
  if (cb_index >= 4U * MAX_NOF_SEGMENTS || (c.base_graph != 1 && c.base_graph != 2) ||
      !valid_lifting_size(c.lifting_size) || !valid_modulation(c.modulation) || c.rv > 3 || c.nof_segments == 0 ||
      c.nof_segments > MAX_NOF_SEGMENTS) {
    return LDPC_HIP_EINVAL;
  }
  const uint32_t KZ = (c.base_graph == 1 ? 22U : 10U) * c.lifting_size;
  if (c.cb_mode != 0) {
    if (c.rm_length == 0 || c.rm_length % Qm != 0 || c.nof_filler_bits >= KZ) {
      return LDPC_HIP_EINVAL;
    }
  } else {
    const uint32_t crc = c.nof_segments > 1 ? 24U : 0U;
    if ((c.nof_tb_crc_bits != 16 && c.nof_tb_crc_bits != 24) || c.nof_tb_bits % 8 != 0 ||
        c.nof_segment_bits + crc + c.nof_filler_bits != KZ || c.nof_short_segments > c.nof_segments ||
        c.cw_length_a == 0 || c.cw_length_a % Qm != 0 || c.cw_length_b % Qm != 0 ||
        (c.nof_short_segments < c.nof_segments && c.cw_length_b == 0) ||
        static_cast<uint64_t>(c.nof_segment_bits) * c.nof_segments < static_cast<uint64_t>(c.nof_tb_bits) + c.nof_tb_crc_bits) {
      return LDPC_HIP_EINVAL;
    }
  }
  if (cb_index >= q->cfgs.size()) {
    q->cfgs.resize(cb_index + 1);
    q->cfg_set.resize(cb_index + 1, 0);
  }
  q->cfgs[cb_index]    = c;
  q->cfg_set[cb_index] = 1;
  return LDPC_HIP_OK;
}

int ldpc_hip_enc_enqueue(ldpc_hip_enc_queue* q, uint32_t cb_index, const uint8_t* data, uint32_t nof_bytes)
{
  if (q == nullptr || (nof_bytes != 0 && data == nullptr)) {
    return LDPC_HIP_EINVAL;
  }
  if (q->state == enc_state::idle || cb_index >= q->cfg_set.size() || q->cfg_set[cb_index] == 0) {
    return LDPC_HIP_ESTATE; /* enqueue without reserve_queue / configure_operation */
  }
  if (q->state == enc_state::launched) {
    if (q->ndequeued != q->ops.size()) {
      return LDPC_HIP_EFULL; /* the batch is in flight: dequeue it first (pdsch_encoder_hw_impl.cpp:93-96) */
    }
    q->reset(enc_state::staging);
  }
  const ldpc_hip_enc_hw_config& c  = q->cfgs[cb_index];
  const uint32_t                Z  = c.lifting_size;
  const uint32_t                KZ = (c.base_graph == 1 ? 22U : 10U) * Z;
  const uint32_t                nu = c.cb_mode != 0 ? 1U : c.nof_segments;
  if (cb_index < q->op_of_cb.size() && q->op_of_cb[cb_index] >= 0) {
    return LDPC_HIP_EINVAL; /* the same cb_index twice in one batch */
  }
  if (q->units.size() + nu > q->max_cbs) {
    return q->units.empty() ? LDPC_HIP_EINVAL : LDPC_HIP_EFULL;
  }
  enc_op op;
  op.cb_index  = cb_index;
  op.unit0     = static_cast<uint32_t>(q->units.size());
  op.nof_units = nu;
  if (c.cb_mode != 0) {
    const uint32_t nbits = KZ - c.nof_filler_bits;
    if (nof_bytes != (nbits + 7) / 8) {
      return LDPC_HIP_EINVAL;
    }
    uint64_t off = 0;
    uint8_t* m   = q->stage(nof_bytes, &off);
    if (m == nullptr) {
      return LDPC_HIP_EDEVICE;
    }
    std::memcpy(m, data, nof_bytes); /* CB data + CB CRC; the device zeroes the bits after nbits (filler) */
    q->add_unit(c.base_graph, Z, c.rm_length, c, off, 0, nbits, 0);
  } else {
    if (nof_bytes != c.nof_tb_bits / 8 || nof_bytes > q->max_tb) {
      return LDPC_HIP_EINVAL;
    }
    /* TB + TB CRC, byte aligned (the TBS is a whole number of bytes, TS 38.214 5.1.3.2), staged once; segment r is
     * bits [r S, r S + n) of it, read in place by the device, which attaches the CB CRC24B when there is more than
     * one segment (TS 38.212 5.2.2) */
    const uint32_t crc_bytes = c.nof_tb_crc_bits / 8;
    uint64_t       off       = 0;
    uint8_t*       m         = q->stage(static_cast<uint64_t>(nof_bytes) + crc_bytes, &off);
    if (m == nullptr) {
      return LDPC_HIP_EDEVICE;
    }
    std::memcpy(m, data, nof_bytes);
    std::memcpy(m + nof_bytes, c.tb_crc, crc_bytes);
    const uint64_t B = static_cast<uint64_t>(c.nof_tb_bits) + c.nof_tb_crc_bits;
    const uint32_t S = c.nof_segment_bits;
    for (uint32_t r = 0; r != c.nof_segments; ++r) {
      const uint32_t E   = r < c.nof_short_segments ? c.cw_length_a : c.cw_length_b;
      const uint64_t bo  = static_cast<uint64_t>(r) * S;
      const uint32_t n   = bo >= B ? 0U : static_cast<uint32_t>(std::min<uint64_t>(S, B - bo));
      /* a segment past the TB's end (n = 0) reads nothing; its message is all zero */
      const uint64_t mo  = n != 0 ? off + bo / 8 : off;
      q->add_unit(c.base_graph, Z, E, c, mo, n != 0 ? static_cast<uint32_t>(bo % 8) : 0U, n,
                  c.nof_segments > 1 ? S : 0U);
    }
  }
  if (cb_index >= q->op_of_cb.size()) {
    q->op_of_cb.resize(cb_index + 1, -1);
  }
  q->op_of_cb[cb_index] = static_cast<int32_t>(q->ops.size());
  q->ops.push_back(op);
  return LDPC_HIP_OK;
}

int ldpc_hip_enc_dequeue(ldpc_hip_enc_queue* q, uint32_t segment_index, uint8_t* bits, uint32_t nof_bits,
                         uint8_t* packed, uint32_t packed_bytes)
{
  if (q == nullptr) {
    return LDPC_HIP_EINVAL;
  }
  if (segment_index >= q->op_of_cb.size() || q->op_of_cb[segment_index] < 0) {
    return LDPC_HIP_ESTATE; /* nothing enqueued under this index */
  }
  enc_op& op = q->ops[static_cast<size_t>(q->op_of_cb[segment_index])];
  if (op.dequeued) {
    return LDPC_HIP_ESTATE;
  }
  if (q->state == enc_state::staging) {
    const int r = q->launch();
    if (r != LDPC_HIP_OK) {
      return r;
    }
  }
  if (!q->complete) {
    if (q->wq != nullptr) { /* every item of the batch done (the work queue's done flags, no runtime call) */
      for (uint32_t t : q->tickets) {
        if (!ldpc_hip::pdsch_encode_done(q->wq, t)) {
          return LDPC_HIP_NOT_READY;
        }
      }
    } else {
      const hipError_t e = hipEventQuery(q->done);
      if (e == hipErrorNotReady) {
        return LDPC_HIP_NOT_READY;
      }
      if (e != hipSuccess) {
        return LDPC_HIP_EDEVICE;
      }
    }
    q->complete = true;
  }
  uint64_t total = 0;
  for (uint32_t u = op.unit0; u != op.unit0 + op.nof_units; ++u) {
    total += q->units[u].E;
  }
  if (bits != nullptr && nof_bits < total) {
    return LDPC_HIP_EINVAL;
  }
  uint64_t bo = 0, po = 0;
  for (uint32_t u = op.unit0; u != op.unit0 + op.nof_units; ++u) {
    const enc_unit& un = q->units[u];
    const uint8_t*  src = q->h_out.as<uint8_t>() + un.out_off;
    if (bits != nullptr) { /* one bit per byte */
      const uint32_t full = un.E / 8;
      unpack_bits(bits + bo, src, full);
      for (uint32_t i = 8 * full; i != un.E; ++i) {
        bits[bo + i] = static_cast<uint8_t>((src[i / 8] >> (7 - (i % 8))) & 1U);
      }
    }
    const uint32_t nb = (un.E + 7) / 8;
    if (packed != nullptr && po < packed_bytes) {
      std::memcpy(packed + po, src, std::min<uint64_t>(nb, packed_bytes - po));
    }
    bo += un.E;
    po += nb;
  }
  op.dequeued = true;
  ++q->ndequeued;
  return LDPC_HIP_OK;
}

int ldpc_hip_enc_cb_mode(const ldpc_hip_enc_queue* q) { return (q != nullptr && q->cb_mode) ? 1 : 0; }

uint32_t ldpc_hip_enc_max_tb_size(const ldpc_hip_enc_queue* q) { return q != nullptr ? q->max_tb : 0U; }

} /* extern "C" */
