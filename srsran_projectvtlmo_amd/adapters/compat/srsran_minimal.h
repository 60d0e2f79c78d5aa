/*
 * Minimal stand-ins for the srsRAN interface types the MI355X adapters implement, used ONLY to build and test the
 * adapters outside an srsRAN tree. Inside srsRAN (SRSRAN_LDPC_HIP_IN_TREE defined) the adapters include the real
 * headers instead:
 *   srsran/adt/span.h, srsran/adt/bit_buffer.h, srsran/phy/upper/log_likelihood_ratio.h,
 *   srsran/phy/upper/codeblock_metadata.h, srsran/phy/upper/channel_coding/crc_calculator.h,
 *   srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h, .../ldpc/ldpc_rate_dematcher.h,
 *   srsran/phy/upper/channel_coding/channel_coding_factories.h, srsran/hal/hw_accelerator.h,
 *   srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h (+ _factory.h),
 *   srsran/hal/phy/upper/channel_processors/pusch/ext_harq_buffer_context_repository.h (+ _factory.h),
 *   srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_factories.h,
 *   srsran/hal/phy/upper/channel_processors/hw_accelerator_factories.h.
 * Only the members the adapters use are provided; names, layouts and semantics follow those headers.
 */
#pragma once

#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#define srsran_assert(cond, ...)                                                                                     \
  do {                                                                                                               \
    if (!(cond)) {                                                                                                   \
      std::fprintf(stderr, "srsran_assert: %s (%s:%d)\n", #cond, __FILE__, __LINE__);                                \
      std::abort();                                                                                                  \
    }                                                                                                                \
  } while (0)

namespace srsran {

template <typename T>
class span
{
public:
  span() = default;
  span(T* p, std::size_t n) : ptr(p), len(n) {}
  template <typename U>
  span(std::vector<U>& v) : ptr(v.data()), len(v.size())
  {
  }
  template <typename U>
  span(const std::vector<U>& v) : ptr(v.data()), len(v.size())
  {
  }
  template <typename U>
  span(span<U> o) : ptr(o.data()), len(o.size())
  {
  }
  T*          data() const { return ptr; }
  std::size_t size() const { return len; }
  bool        empty() const { return len == 0; }
  T&          operator[](std::size_t i) const { return ptr[i]; }
  span        first(std::size_t n) const { return span(ptr, n); }
  T*          begin() const { return ptr; }
  T*          end() const { return ptr + len; }

private:
  T*          ptr = nullptr;
  std::size_t len = 0;
};

/* Packed bit buffer, MSB-first in uint8_t words (bit_buffer.h:31-150). */
class bit_buffer
{
public:
  bit_buffer() = default;
  bit_buffer(span<uint8_t> storage, unsigned nbits) : buf(storage), nof_bits(nbits) {}
  unsigned      size() const { return nof_bits; }
  span<uint8_t> get_buffer() const { return buf.first((nof_bits + 7) / 8); }
  uint8_t       extract(unsigned i) const { return (buf[i / 8] >> (7 - i % 8)) & 1U; }

private:
  span<uint8_t> buf;
  unsigned      nof_bits = 0;
};

/* int8 LLR, +-120 finite, +-127 infinite (log_likelihood_ratio.h:46-244). */
class log_likelihood_ratio
{
public:
  constexpr log_likelihood_ratio() = default;
  constexpr log_likelihood_ratio(int v) : value(static_cast<int8_t>(v)) {}
  constexpr int8_t to_value_type() const { return value; }
  constexpr int    to_int() const { return static_cast<int>(value); }

private:
  int8_t value = 0;
};
static_assert(sizeof(log_likelihood_ratio) == 1, "LLR must be one byte");

enum class crc_generator_poly { CRC24A, CRC24B, CRC24C, CRC16, CRC11, CRC6 };

class crc_calculator
{
public:
  virtual ~crc_calculator()                                = default;
  virtual crc_generator_poly get_generator_poly() const    = 0;
  virtual unsigned           calculate(const bit_buffer& d) = 0;
};

enum class ldpc_base_graph_type : uint8_t { BG1 = 1, BG2 = 2 };
enum class modulation_scheme { PI_2_BPSK = 0, BPSK = 1, QPSK = 2, QAM16 = 4, QAM64 = 6, QAM256 = 8 };
inline unsigned get_bits_per_symbol(modulation_scheme m)
{
  return m == modulation_scheme::PI_2_BPSK ? 1U : static_cast<unsigned>(m);
}

namespace ldpc {
enum lifting_size_t : unsigned {}; /* values are the lifting sizes themselves (ldpc.h) */
}

struct codeblock_metadata {
  struct tb_common_metadata {
    ldpc_base_graph_type base_graph   = ldpc_base_graph_type::BG1;
    ldpc::lifting_size_t lifting_size = ldpc::lifting_size_t(2);
    unsigned             rv           = 0;
    modulation_scheme    mod          = modulation_scheme::BPSK;
    unsigned             Nref         = 0;
    unsigned             cw_length    = 0;
  };
  struct cb_specific_metadata {
    unsigned full_length     = 0;
    unsigned rm_length       = 0;
    unsigned nof_filler_bits = 0;
    unsigned cw_offset       = 0;
    unsigned nof_crc_bits    = 16;
  };
  tb_common_metadata   tb_common;
  cb_specific_metadata cb_specific;
};

class ldpc_decoder
{
public:
  virtual ~ldpc_decoder() = default;
  struct configuration {
    struct algorithm_details {
      unsigned max_iterations = 6;
      float    scaling_factor = 0.8;
    };
    codeblock_metadata block_conf;
    algorithm_details  algorithm_conf;
  };
  virtual std::optional<unsigned>
  decode(bit_buffer& output, span<const log_likelihood_ratio> input, crc_calculator* crc, const configuration& cfg) = 0;
};

class ldpc_rate_dematcher
{
public:
  virtual ~ldpc_rate_dematcher() = default;
  virtual void rate_dematch(span<log_likelihood_ratio>       output,
                            span<const log_likelihood_ratio> input,
                            bool                             new_data,
                            const codeblock_metadata&        cfg) = 0;
};

class ldpc_decoder_factory
{
public:
  virtual ~ldpc_decoder_factory()                = default;
  virtual std::unique_ptr<ldpc_decoder> create() = 0;
};

class ldpc_rate_dematcher_factory
{
public:
  virtual ~ldpc_rate_dematcher_factory()                = default;
  virtual std::unique_ptr<ldpc_rate_dematcher> create() = 0;
};

/* channel_coding_factories.h:52-59, :70-77. In srsRAN these build the CPU decoders ("auto", "generic", "avx2", ...);
 * out of tree (ldpc_hip_adapters.cpp) only the types that resolve to the GPU exist: "hip", "hip:<n>", and "auto"
 * for the decoder when a gfx950 is visible -- the branches INTEGRATION.md section 2.1 adds to the real factories. */
std::shared_ptr<ldpc_decoder_factory>        create_ldpc_decoder_factory_sw(const std::string& dec_type);
std::shared_ptr<ldpc_rate_dematcher_factory> create_ldpc_rate_dematcher_factory_sw(const std::string& dematcher_type);

/* demodulation_mapper.h:46-70, channel_modulation_factories.h:32-39 (the EVM calculator is outside the path) */
using cf_t = std::complex<float>;
class demodulation_mapper
{
public:
  virtual ~demodulation_mapper() = default;
  virtual void demodulate_soft(span<log_likelihood_ratio> llrs,
                               span<const cf_t>           symbols,
                               span<const float>          noise_vars,
                               modulation_scheme          mod) = 0;
};
class evm_calculator
{
public:
  virtual ~evm_calculator() = default;
};
class channel_modulation_factory
{
public:
  virtual ~channel_modulation_factory()                                     = default;
  virtual std::unique_ptr<demodulation_mapper> create_demodulation_mapper() = 0;
  virtual std::unique_ptr<evm_calculator>      create_evm_calculator()      = 0;
};

namespace dpdk {
class bbdev_acc; /* include/srsran/hal/dpdk/bbdev/bbdev_acc.h: the DPDK bbdev accelerator (not used by "mi355x") */
}

namespace hal {

/* ext_harq_buffer_context_repository.h: the per-codeblock HARQ metadata the HAL caller owns (the soft bits stay in
 * the accelerator's memory). Same members and semantics: entries direct-indexed by absolute_cb_id; get() opens a
 * fresh entry (soft_data_len 0) on new data or when the entry is empty; free() empties it except in debug mode; an
 * out-of-range id asserts. */
constexpr uint64_t HARQ_INCR_BYTES = 32768; /* HARQ_INCR (units::bytes{32768}): one accelerator HARQ slot */

struct ext_harq_buffer_context_entry {
  unsigned soft_data_len = 0;
  bool     empty         = true;
};

class ext_harq_buffer_context_repository
{
public:
  ext_harq_buffer_context_repository(unsigned nof_codeblocks_, uint64_t ext_harq_buff_size, bool debug_mode_) :
    entries(nof_codeblocks_), debug_mode(debug_mode_)
  {
    srsran_assert(static_cast<uint64_t>(nof_codeblocks_) * HARQ_INCR_BYTES <= ext_harq_buff_size,
                  "external HARQ buffer too small for the requested codeblocks");
  }
  ext_harq_buffer_context_entry* get(unsigned absolute_codeblock_id, bool new_data)
  {
    srsran_assert(absolute_codeblock_id < entries.size(), "absolute CB index out of the repository's bounds");
    ext_harq_buffer_context_entry& e = entries[absolute_codeblock_id];
    if (new_data || e.empty) {
      e = ext_harq_buffer_context_entry{0, false};
    }
    return &e;
  }
  void free(unsigned absolute_codeblock_id)
  {
    srsran_assert(absolute_codeblock_id < entries.size(), "absolute CB index out of the repository's bounds");
    if (!debug_mode) {
      entries[absolute_codeblock_id].empty = true;
    }
  }

private:
  std::vector<ext_harq_buffer_context_entry> entries;
  bool                                       debug_mode;
};

/* ext_harq_buffer_context_repository_factory.h */
std::shared_ptr<ext_harq_buffer_context_repository>
create_ext_harq_buffer_context_repository(unsigned nof_codeblocks, uint64_t ext_harq_buff_size, bool debug_mode);

template <typename T, typename U>
class hw_accelerator
{
public:
  virtual ~hw_accelerator()                                                                               = default;
  virtual bool enqueue_operation(span<const T> data, span<const T> aux_data = {}, unsigned cb_index = 0) = 0;
  virtual bool dequeue_operation(span<U> data, span<T> aux_data = {}, unsigned segment_index = 0)        = 0;
};

enum class hw_dec_cb_crc_type : uint8_t { CRC16 = 0, CRC24B = 1, CRC24A = 2 };

struct hw_pusch_decoder_configuration {
  ldpc_base_graph_type base_graph_index;
  modulation_scheme    modulation;
  unsigned             nof_segments;
  unsigned             rv;
  unsigned             cw_length;
  unsigned             lifting_size;
  unsigned             Ncb;
  unsigned             Nref;
  unsigned             nof_segment_bits;
  unsigned             nof_filler_bits;
  unsigned             max_nof_ldpc_iterations;
  bool                 use_early_stop;
  bool                 new_data;
  unsigned             cb_crc_len;
  hw_dec_cb_crc_type   cb_crc_type;
  unsigned             absolute_cb_id;
};

struct hw_pusch_decoder_outputs {
  bool     CRC_pass;
  unsigned nof_ldpc_iterations;
};

class hw_accelerator_pusch_dec : public hw_accelerator<int8_t, uint8_t>
{
public:
  virtual ~hw_accelerator_pusch_dec()                                                                          = default;
  virtual void reserve_queue()                                                                                  = 0;
  virtual void free_queue()                                                                                     = 0;
  virtual void configure_operation(const hw_pusch_decoder_configuration& config, unsigned cb_index = 0)        = 0;
  virtual void read_operation_outputs(hw_pusch_decoder_outputs& out, unsigned cb_index = 0, unsigned id = 0)   = 0;
  virtual void free_harq_context_entry(unsigned absolute_cb_id)                                                 = 0;
  virtual bool is_external_harq_supported() const                                                              = 0;
};

class hw_accelerator_pusch_dec_factory
{
public:
  virtual ~hw_accelerator_pusch_dec_factory()                      = default;
  virtual std::unique_ptr<hw_accelerator_pusch_dec> create()        = 0;
};

/* pusch/hw_accelerator_factories.h:33-51: the configuration every HAL caller fills, field for field */
struct hw_accelerator_pusch_dec_configuration {
  std::string                                         acc_type;
  std::shared_ptr<dpdk::bbdev_acc>                    bbdev_accelerator;
  bool                                                ext_softbuffer;
  std::shared_ptr<ext_harq_buffer_context_repository> harq_buffer_context;
  bool                                                dedicated_queue = true;
};
std::shared_ptr<hw_accelerator_pusch_dec_factory>
create_hw_accelerator_pusch_dec_factory(const hw_accelerator_pusch_dec_configuration& accelerator_config);

/* hw_accelerator_pdsch_enc.h:37-102 (static_vector<uint8_t, 3> tb_crc as a std::vector here) */
struct hw_pdsch_encoder_configuration {
  unsigned             nof_tb_bits;
  unsigned             nof_tb_crc_bits;
  ldpc_base_graph_type base_graph_index;
  modulation_scheme    modulation;
  unsigned             nof_segments;
  unsigned             nof_short_segments;
  unsigned             rv;
  unsigned             cw_length_a;
  unsigned             cw_length_b;
  unsigned             lifting_size;
  unsigned             Ncb;
  unsigned             Nref;
  unsigned             nof_segment_bits;
  unsigned             nof_filler_bits;
  unsigned             rm_length;
  std::vector<uint8_t> tb_crc;
  bool                 cb_mode = false;
};

class hw_accelerator_pdsch_enc : public hw_accelerator<uint8_t, uint8_t>
{
public:
  virtual ~hw_accelerator_pdsch_enc()                                                                   = default;
  virtual void     reserve_queue()                                                                       = 0;
  virtual void     free_queue()                                                                          = 0;
  virtual void     configure_operation(const hw_pdsch_encoder_configuration& config, unsigned cb_index = 0) = 0;
  virtual bool     get_cb_mode() const                                                                   = 0;
  virtual unsigned get_max_tb_size() const                                                               = 0;
};

class hw_accelerator_pdsch_enc_factory
{
public:
  virtual ~hw_accelerator_pdsch_enc_factory()                = default;
  virtual std::unique_ptr<hw_accelerator_pdsch_enc> create() = 0;
};

/* channel_processors/hw_accelerator_factories.h:31-51 */
struct hw_accelerator_pdsch_enc_configuration {
  std::string                      acc_type;
  std::shared_ptr<dpdk::bbdev_acc> bbdev_accelerator;
  bool                             cb_mode = false;
  unsigned                         max_tb_size;
  bool                             dedicated_queue;
};
std::shared_ptr<hw_accelerator_pdsch_enc_factory>
create_hw_accelerator_pdsch_enc_factory(const hw_accelerator_pdsch_enc_configuration& accelerator_config);

} // namespace hal
} // namespace srsran
