/*
 * srsRAN-side adapters of the MI355X LDPC decode path: see ldpc_hip_adapters.h.
 * Reference semantics: ldpc_decoder_impl.cpp:60-147 (decode contract, return value), ldpc_rate_dematcher_impl.cpp
 * :46-114 (dematch contract), hw_accelerator_pusch_dec_acc100_impl.cpp (HAL queue semantics incl. dropped ops).
 */
#include "ldpc_hip_adapters.h"

#include <algorithm>
#include <cstring>

using namespace srsran;

namespace {

int8_t hip_crc_of(crc_generator_poly p)
{
  switch (p) {
    case crc_generator_poly::CRC16:
      return LDPC_HIP_CRC16;
    case crc_generator_poly::CRC24B:
      return LDPC_HIP_CRC24B;
    case crc_generator_poly::CRC24A:
      return LDPC_HIP_CRC24A;
    default:
      srsran_assert(false, "Invalid number of CRC bits.");
      return LDPC_HIP_CRC_NONE;
  }
}

void check_rc(ldpc_hip_ctx* ctx, int rc)
{
  if (rc < 0) {
    std::fprintf(stderr, "ldpc_hip: %s\n", ldpc_hip_last_error(ctx));
    srsran_assert(rc >= 0, "ldpc_hip call failed");
  }
}

} // namespace

ldpc_hip_context::ldpc_hip_context(int device, ldpc_hip_harq_repo* harq_repo, uint32_t launch_flags)
{
  ldpc_hip_params p{};
  p.launch_flags = launch_flags;
  const int rc   = ldpc_hip_open_harq(device, &p, harq_repo, &ctx);
  srsran_assert(rc == LDPC_HIP_OK, "ldpc_hip_open failed");
}

ldpc_hip_context::~ldpc_hip_context()
{
  if (ctx != nullptr) {
    ldpc_hip_close(ctx);
  }
}

namespace {
/* the C ABI descriptor of one ldpc_decoder::decode call (ldpc_decoder.h:37-75) */
ldpc_hip_dec_desc dec_desc_of(span<const log_likelihood_ratio> input, crc_calculator* crc,
                              const ldpc_decoder::configuration& cfg)
{
  ldpc_hip_dec_desc d{};
  d.base_graph      = static_cast<uint8_t>(cfg.block_conf.tb_common.base_graph);
  d.lifting_size    = static_cast<uint16_t>(cfg.block_conf.tb_common.lifting_size);
  d.nof_filler_bits = static_cast<uint16_t>(cfg.block_conf.cb_specific.nof_filler_bits);
  d.max_iterations  = static_cast<uint8_t>(cfg.algorithm_conf.max_iterations);
  d.scaling_factor  = cfg.algorithm_conf.scaling_factor;
  d.llr_length      = static_cast<uint32_t>(input.size());
  d.crc_mode        = (crc == nullptr) ? LDPC_HIP_CRC_MODE_NONE : LDPC_HIP_CRC_MODE_EARLY_STOP;
  d.crc_poly        = (crc == nullptr) ? LDPC_HIP_CRC_NONE : hip_crc_of(crc->get_generator_poly());
  return d;
}
} // namespace

std::optional<unsigned> ldpc_decoder_hip::decode(bit_buffer&                      output,
                                                 span<const log_likelihood_ratio> input,
                                                 crc_calculator*                  crc,
                                                 const configuration&             cfg)
{
  const ldpc_hip_dec_desc d = dec_desc_of(input, crc, cfg);
  const unsigned K  = (d.base_graph == 1) ? 22U : 10U;
  srsran_assert(output.size() == K * d.lifting_size, "The output size is not equal to the message length.");

  const int8_t*      llr = reinterpret_cast<const int8_t*>(input.data());
  uint8_t*           out = output.get_buffer().data();
  ldpc_hip_cb_result res{};
  check_rc(ctx.get(), ldpc_hip_decode_sync(ctx.get(), 1, &d, &llr, &out, &res));
  if (res.crc_pass) {
    return res.nof_iterations;
  }
  return std::nullopt;
}

ldpc_decoder_hip_auto::ldpc_decoder_hip_auto(int dev, std::unique_ptr<ldpc_decoder> cpu_, uint64_t min_work_) :
  device(dev), cpu(std::move(cpu_)), min_work(min_work_)
{
}

std::optional<unsigned> ldpc_decoder_hip_auto::decode(bit_buffer&                      output,
                                                      span<const log_likelihood_ratio> input,
                                                      crc_calculator*                  crc,
                                                      const configuration&             cfg)
{
  const ldpc_hip_dec_desc d = dec_desc_of(input, crc, cfg);
  if (cpu && ldpc_hip_decode_work(&d, reinterpret_cast<const int8_t*>(input.data())) < min_work) {
    ++n_cpu;
    return cpu->decode(output, input, crc, cfg);
  }
  if (!gpu) {
    gpu = std::make_unique<ldpc_decoder_hip>(device);
  }
  ++n_gpu;
  return gpu->decode(output, input, crc, cfg);
}

void ldpc_rate_dematcher_hip::rate_dematch(span<log_likelihood_ratio>       output,
                                           span<const log_likelihood_ratio> input,
                                           bool                             new_data,
                                           const codeblock_metadata&        cfg)
{
  ldpc_hip_dematch_desc d{};
  d.modulation_order = static_cast<uint8_t>(get_bits_per_symbol(cfg.tb_common.mod));
  d.rv               = static_cast<uint8_t>(cfg.tb_common.rv);
  d.new_data         = new_data ? 1 : 0;
  d.cb_length        = static_cast<uint32_t>(output.size());
  d.rm_length        = static_cast<uint32_t>(input.size());
  d.Nref             = cfg.tb_common.Nref;
  d.nof_filler_bits  = cfg.cb_specific.nof_filler_bits;
  int8_t*       soft = reinterpret_cast<int8_t*>(output.data());
  const int8_t* llr  = reinterpret_cast<const int8_t*>(input.data());
  check_rc(ctx.get(), ldpc_hip_rate_dematch_sync(ctx.get(), 1, &d, &soft, &llr));
}

namespace {

class ldpc_decoder_factory_hip : public ldpc_decoder_factory
{
public:
  explicit ldpc_decoder_factory_hip(int dev) : device(dev) {}
  std::unique_ptr<ldpc_decoder> create() override { return std::make_unique<ldpc_decoder_hip>(device); }

private:
  int device;
};

class ldpc_rate_dematcher_factory_hip : public ldpc_rate_dematcher_factory
{
public:
  explicit ldpc_rate_dematcher_factory_hip(int dev) : device(dev) {}
  std::unique_ptr<ldpc_rate_dematcher> create() override { return std::make_unique<ldpc_rate_dematcher_hip>(device); }

private:
  int device;
};

} // namespace

int srsran::hip_device_of(const char* type)
{
  if (type == nullptr) {
    return -1;
  }
  if (std::strcmp(type, "hip") == 0) {
    return 0;
  }
  if (std::strncmp(type, "hip:", 4) != 0 || type[4] == '\0') {
    return -1;
  }
  int dev = 0;
  for (const char* p = type + 4; *p != '\0'; ++p) {
    if (*p < '0' || *p > '9' || dev > 1000) {
      return -1;
    }
    dev = dev * 10 + (*p - '0');
  }
  return dev;
}

int srsran::hip_device_of_decoder_type(const std::string& dec_type)
{
  return dec_type == "auto" ? ldpc_hip_auto_device() : hip_device_of(dec_type.c_str());
}

int srsran::hip_device_of_dematcher_type(const std::string& dematcher_type)
{
  return hip_device_of(dematcher_type.c_str());
}

std::shared_ptr<ldpc_decoder_factory> srsran::create_ldpc_decoder_factory_hip(int device)
{
  return std::make_shared<ldpc_decoder_factory_hip>(device);
}

namespace {
class ldpc_decoder_factory_hip_auto : public ldpc_decoder_factory
{
public:
  ldpc_decoder_factory_hip_auto(int dev, std::shared_ptr<ldpc_decoder_factory> cpu_factory, uint64_t min_work_) :
    device(dev), cpu(std::move(cpu_factory)), min_work(min_work_)
  {
  }
  std::unique_ptr<ldpc_decoder> create() override
  {
    return std::make_unique<ldpc_decoder_hip_auto>(device, cpu ? cpu->create() : nullptr, min_work);
  }

private:
  int                                   device;
  std::shared_ptr<ldpc_decoder_factory> cpu;
  uint64_t                              min_work;
};
} // namespace

std::shared_ptr<ldpc_decoder_factory>
srsran::create_ldpc_decoder_factory_hip_auto(int device, std::shared_ptr<ldpc_decoder_factory> cpu_factory,
                                             uint64_t min_work)
{
  return std::make_shared<ldpc_decoder_factory_hip_auto>(device, std::move(cpu_factory), min_work);
}

std::shared_ptr<ldpc_rate_dematcher_factory> srsran::create_ldpc_rate_dematcher_factory_hip(int device)
{
  return std::make_shared<ldpc_rate_dematcher_factory_hip>(device);
}

/* ---- soft demodulation mapper ---- */
void demodulation_mapper_hip::demodulate_soft(span<log_likelihood_ratio> llrs,
                                              span<const cf_t>           symbols,
                                              span<const float>          noise_vars,
                                              modulation_scheme          mod)
{
  /* demodulation_mapper_impl.cpp:82-83 */
  srsran_assert(symbols.size() == noise_vars.size(), "Inputs symbols and noise_vars must have the same length.");
  srsran_assert(symbols.size() * get_bits_per_symbol(mod) == llrs.size(), "Input and output lengths are incompatible.");
  check_rc(ctx.get(),
           ldpc_hip_demodulate_sync(ctx.get(), static_cast<uint32_t>(symbols.size()), static_cast<int>(mod),
                                    reinterpret_cast<const float*>(symbols.data()), noise_vars.data(),
                                    reinterpret_cast<int8_t*>(llrs.data())));
}

namespace {
class channel_modulation_factory_hip : public channel_modulation_factory
{
public:
  channel_modulation_factory_hip(int dev, std::shared_ptr<channel_modulation_factory> evm) :
    device(dev), evm_source(std::move(evm))
  {
  }
  std::unique_ptr<demodulation_mapper> create_demodulation_mapper() override
  {
    return std::make_unique<demodulation_mapper_hip>(device);
  }
  std::unique_ptr<evm_calculator> create_evm_calculator() override
  {
    return evm_source ? evm_source->create_evm_calculator() : nullptr;
  }

private:
  int                                         device;
  std::shared_ptr<channel_modulation_factory> evm_source;
};
} // namespace

std::shared_ptr<channel_modulation_factory>
srsran::create_channel_modulation_factory_hip(int device, std::shared_ptr<channel_modulation_factory> evm_source)
{
  return std::make_shared<channel_modulation_factory_hip>(device, std::move(evm_source));
}

/* ---- HAL ---- */
using namespace srsran::hal;

int srsran::hal::hip_device_of_acc_type(const std::string& acc_type)
{
  if (acc_type == "mi355x") {
    return 0;
  }
  if (acc_type.rfind("mi355x:", 0) != 0) {
    return -1;
  }
  return hip_device_of(("hip:" + acc_type.substr(7)).c_str());
}

namespace {

/* the GPU's HARQ memory (ldpc_hip_harq_device_memory): one reference per device, held for the process */
ldpc_hip_harq_repo* device_harq_memory(int device)
{
  ldpc_hip_harq_repo* m = nullptr;
  srsran_assert(ldpc_hip_harq_device_memory(device, &m) == LDPC_HIP_OK, "the GPU's HARQ memory is unavailable");
  (void)ldpc_hip_harq_repo_release(m); /* the library keeps it for the process; contexts hold their own references */
  return m;
}

int acc_device(const std::string& acc_type)
{
  const int dev = hip_device_of_acc_type(acc_type);
  srsran_assert(dev >= 0, "acc_type is not an MI355X accelerator");
  return dev;
}

} // namespace

hw_accelerator_pusch_dec_hip::hw_accelerator_pusch_dec_hip(const hw_accelerator_pusch_dec_configuration& cfg) :
  ext_softbuffer(cfg.ext_softbuffer),
  harq_buffer_context(cfg.harq_buffer_context),
  ctx(acc_device(cfg.acc_type),
      cfg.ext_softbuffer ? device_harq_memory(acc_device(cfg.acc_type)) : nullptr,
      cfg.dedicated_queue ? 0U : static_cast<uint32_t>(LDPC_HIP_LAUNCH_SHARED_QUEUE)),
  cfgs(162)
{
  /* acc100 takes the entry of every configured codeblock from this repository (acc100_impl.cpp:113) */
  srsran_assert(harq_buffer_context != nullptr, "hw_accelerator_pusch_dec_configuration without harq_buffer_context");
}

void hw_accelerator_pusch_dec_hip::reserve_queue()
{
  check_rc(ctx.get(), ldpc_hip_queue_reserve(ctx.get()));
}

void hw_accelerator_pusch_dec_hip::free_queue()
{
  check_rc(ctx.get(), ldpc_hip_queue_free(ctx.get()));
}

void hw_accelerator_pusch_dec_hip::configure_operation(const hw_pusch_decoder_configuration& c, unsigned cb_index)
{
  /* a TB has at most MAX_NOF_SEGMENTS = 162 codeblocks (sch_constants.h:38); the library rejects larger indices */
  srsran_assert(cb_index < 4U * 162U, "Codeblock index {} out of bounds.", cb_index);
  if (cb_index == 0) { /* acc100 hw_config: the drop bits are reset with the first CB of the TB (acc100_impl.cpp:106-110) */
    drop_op.assign(std::max<size_t>(c.nof_segments, 1), 0);
    harq_context_entries.assign(std::max<size_t>(c.nof_segments, 1), nullptr);
  }
  if (cb_index >= cfgs.size()) {
    cfgs.resize(cb_index + 1);
  }
  if (cb_index >= drop_op.size()) {
    drop_op.resize(cb_index + 1, 0);
    harq_context_entries.resize(cb_index + 1, nullptr);
  }
  /* the CB's entry in the caller's repository, opened afresh on new data (acc100_impl.cpp:113) */
  harq_context_entries[cb_index] = harq_buffer_context->get(c.absolute_cb_id, c.new_data);
  ldpc_hip_hw_config& h          = cfgs[cb_index];
  h                              = ldpc_hip_hw_config{};
  h.base_graph                   = static_cast<uint8_t>(c.base_graph_index);
  h.modulation_order             = static_cast<uint8_t>(get_bits_per_symbol(c.modulation));
  h.rv                           = static_cast<uint8_t>(c.rv);
  h.new_data                     = c.new_data ? 1 : 0;
  h.nof_segments                 = c.nof_segments;
  h.cw_length                    = c.cw_length;
  h.lifting_size                 = c.lifting_size;
  h.Ncb                          = c.Ncb;
  h.Nref                         = c.Nref;
  h.nof_segment_bits             = c.nof_segment_bits;
  h.nof_filler_bits              = c.nof_filler_bits;
  h.max_nof_ldpc_iterations      = c.max_nof_ldpc_iterations;
  h.use_early_stop               = c.use_early_stop ? 1 : 0;
  h.cb_crc_type                  = static_cast<uint8_t>(c.cb_crc_type);
  h.cb_crc_len                   = static_cast<uint16_t>(c.cb_crc_len);
  h.absolute_cb_id               = c.absolute_cb_id;
}

bool hw_accelerator_pusch_dec_hip::enqueue_operation(span<const int8_t> data, span<const int8_t> aux, unsigned cb)
{
  srsran_assert(cb < harq_context_entries.size() && harq_context_entries[cb] != nullptr,
                "enqueue_operation without configure_operation");
  /* acc100 hw_enqueue (acc100_impl.cpp:123-125, 184-186): a retransmission whose entry holds no soft data is
   * dropped -- accepted, and read back as a CRC failure with the maximum number of iterations */
  if (cfgs[cb].new_data == 0 && harq_context_entries[cb]->soft_data_len == 0) {
    drop_op[cb] = 1;
    return true;
  }
  const int rc = ldpc_hip_enqueue(ctx.get(), cb, &cfgs[cb], data.data(), static_cast<uint32_t>(data.size()),
                                  aux.empty() ? nullptr : aux.data(), static_cast<uint32_t>(aux.size()));
  if (rc == LDPC_HIP_EFULL) {
    return false; /* the batch cannot take it now: the caller dequeues, then enqueues again */
  }
  check_rc(ctx.get(), rc);
  drop_op[cb] = 0;
  return true;
}

bool hw_accelerator_pusch_dec_hip::dequeue_operation(span<uint8_t> data, span<int8_t> aux, unsigned segment_index)
{
  if (segment_index < drop_op.size() && drop_op[segment_index] != 0) {
    return true; /* acc100 hw_dequeue: a dropped operation dequeues at once (acc100_impl.cpp:217-219) */
  }
  const int rc = ldpc_hip_dequeue(ctx.get(), segment_index, data.data(), static_cast<uint32_t>(data.size()),
                                  aux.empty() ? nullptr : aux.data(), static_cast<uint32_t>(aux.size()));
  if (rc == LDPC_HIP_NOT_READY) {
    return false;
  }
  check_rc(ctx.get(), rc);
  /* the entry now holds the codeblock's soft data: its length, as acc100 reads harq_combined_output.length back
   * (acc100_impl.cpp:211-212, bbdev_ldpc_decoder.cpp:323) */
  const ldpc_hip_hw_config& c = cfgs[segment_index];
  harq_context_entries[segment_index]->soft_data_len = (c.base_graph == 1 ? 66U : 50U) * c.lifting_size;
  return true;
}

void hw_accelerator_pusch_dec_hip::read_operation_outputs(hw_pusch_decoder_outputs& out, unsigned cb, unsigned id)
{
  if (cb < drop_op.size() && drop_op[cb] != 0) { /* acc100_impl.cpp:233-247 */
    out.CRC_pass            = false;
    out.nof_ldpc_iterations = cfgs[cb].max_nof_ldpc_iterations;
    drop_op[cb]             = 0;
    return;
  }
  ldpc_hip_cb_result r{};
  check_rc(ctx.get(), ldpc_hip_read_outputs(ctx.get(), cb, id, &r));
  out.CRC_pass            = r.crc_pass != 0;
  out.nof_ldpc_iterations = r.nof_iterations;
}

void hw_accelerator_pusch_dec_hip::free_harq_context_entry(unsigned absolute_cb_id)
{
  harq_buffer_context->free(absolute_cb_id); /* acc100_impl.cpp:268-271 */
}

bool hw_accelerator_pusch_dec_hip::is_external_harq_supported() const
{
  return ext_softbuffer;
}

namespace {

class hw_accelerator_pusch_dec_factory_hip : public hw_accelerator_pusch_dec_factory
{
public:
  explicit hw_accelerator_pusch_dec_factory_hip(const hw_accelerator_pusch_dec_configuration& c) : cfg(c) {}
  std::unique_ptr<hw_accelerator_pusch_dec> create() override
  {
    return std::make_unique<hw_accelerator_pusch_dec_hip>(cfg);
  }

private:
  hw_accelerator_pusch_dec_configuration cfg;
};

} // namespace

std::shared_ptr<hw_accelerator_pusch_dec_factory>
srsran::hal::create_hw_accelerator_pusch_dec_factory_hip(const hw_accelerator_pusch_dec_configuration& cfg)
{
  if (hip_device_of_acc_type(cfg.acc_type) < 0) {
    return nullptr;
  }
  return std::make_shared<hw_accelerator_pusch_dec_factory_hip>(cfg);
}

/* ---- hw_accelerator_pdsch_enc (hw_accelerator_pdsch_enc_acc100_impl.cpp semantics on the GPU) ---- */

hw_accelerator_pdsch_enc_hip::hw_accelerator_pdsch_enc_hip(const hw_accelerator_pdsch_enc_configuration& cfg) :
  ctx(acc_device(cfg.acc_type), nullptr, cfg.dedicated_queue ? 0U : static_cast<uint32_t>(LDPC_HIP_LAUNCH_SHARED_QUEUE))
{
  check_rc(ctx.get(), ldpc_hip_enc_queue_create(ctx.get(), cfg.cb_mode ? 1 : 0, 0, cfg.max_tb_size, &queue));
}

hw_accelerator_pdsch_enc_hip::~hw_accelerator_pdsch_enc_hip()
{
  if (queue != nullptr) {
    (void)ldpc_hip_enc_queue_destroy(queue);
  }
}

void hw_accelerator_pdsch_enc_hip::reserve_queue()
{
  check_rc(ctx.get(), ldpc_hip_enc_reserve(queue));
}

void hw_accelerator_pdsch_enc_hip::free_queue()
{
  check_rc(ctx.get(), ldpc_hip_enc_free(queue));
}

void hw_accelerator_pdsch_enc_hip::configure_operation(const hw_pdsch_encoder_configuration& c, unsigned cb_index)
{
  ldpc_hip_enc_hw_config h{};
  h.nof_tb_bits        = c.nof_tb_bits;
  h.nof_tb_crc_bits    = c.nof_tb_crc_bits;
  h.base_graph         = static_cast<uint8_t>(c.base_graph_index);
  h.modulation         = static_cast<uint8_t>(c.modulation);
  h.rv                 = static_cast<uint8_t>(c.rv);
  h.cb_mode            = c.cb_mode ? 1 : 0;
  h.nof_segments       = c.nof_segments;
  h.nof_short_segments = c.nof_short_segments;
  h.cw_length_a        = c.cw_length_a;
  h.cw_length_b        = c.cw_length_b;
  h.lifting_size       = c.lifting_size;
  h.Ncb                = c.Ncb;
  h.Nref               = c.Nref;
  h.nof_segment_bits   = c.nof_segment_bits;
  h.nof_filler_bits    = c.nof_filler_bits;
  h.rm_length          = c.rm_length;
  for (size_t i = 0; i != c.tb_crc.size() && i != 3; ++i) {
    h.tb_crc[i] = c.tb_crc[i];
  }
  check_rc(ctx.get(), ldpc_hip_enc_configure(queue, cb_index, &h));
}

bool hw_accelerator_pdsch_enc_hip::enqueue_operation(span<const uint8_t> data, span<const uint8_t>, unsigned cb_index)
{
  const int rc = ldpc_hip_enc_enqueue(queue, cb_index, data.data(), static_cast<uint32_t>(data.size()));
  if (rc == LDPC_HIP_EFULL) {
    return false; /* pdsch_encoder_hw_impl.cpp:93-96: dequeue what was enqueued, then enqueue again */
  }
  check_rc(ctx.get(), rc);
  return true;
}

bool hw_accelerator_pdsch_enc_hip::dequeue_operation(span<uint8_t> data, span<uint8_t> packed, unsigned segment_index)
{
  const int rc = ldpc_hip_enc_dequeue(queue, segment_index, data.data(), static_cast<uint32_t>(data.size()),
                                      packed.empty() ? nullptr : packed.data(), static_cast<uint32_t>(packed.size()));
  if (rc == LDPC_HIP_NOT_READY) {
    return false;
  }
  check_rc(ctx.get(), rc);
  return true;
}

bool hw_accelerator_pdsch_enc_hip::get_cb_mode() const
{
  return ldpc_hip_enc_cb_mode(queue) != 0;
}

unsigned hw_accelerator_pdsch_enc_hip::get_max_tb_size() const
{
  return ldpc_hip_enc_max_tb_size(queue);
}

namespace {

class hw_accelerator_pdsch_enc_factory_hip : public hw_accelerator_pdsch_enc_factory
{
public:
  explicit hw_accelerator_pdsch_enc_factory_hip(const hw_accelerator_pdsch_enc_configuration& c) : cfg(c) {}
  std::unique_ptr<hw_accelerator_pdsch_enc> create() override
  {
    return std::make_unique<hw_accelerator_pdsch_enc_hip>(cfg);
  }

private:
  hw_accelerator_pdsch_enc_configuration cfg;
};

} // namespace

std::shared_ptr<hw_accelerator_pdsch_enc_factory>
srsran::hal::create_hw_accelerator_pdsch_enc_factory_hip(const hw_accelerator_pdsch_enc_configuration& cfg)
{
  if (hip_device_of_acc_type(cfg.acc_type) < 0) {
    return nullptr;
  }
  return std::make_shared<hw_accelerator_pdsch_enc_factory_hip>(cfg);
}

#ifndef SRSRAN_LDPC_HIP_IN_TREE
/* Out of tree only: the reference's factory entry points, reduced to the branches INTEGRATION.md adds to them (the
 * "mi355x" HAL accelerators, the "hip" / "auto" software decoders). In srsRAN these functions are the reference's own
 * (hw_accelerator_factories.cpp, channel_coding_factories.cpp, ext_harq_buffer_context_repository_factory.cpp). */
std::shared_ptr<hw_accelerator_pusch_dec_factory>
srsran::hal::create_hw_accelerator_pusch_dec_factory(const hw_accelerator_pusch_dec_configuration& accelerator_config)
{
  return create_hw_accelerator_pusch_dec_factory_hip(accelerator_config); /* nullptr unless acc_type is "mi355x[:n]" */
}

std::shared_ptr<hw_accelerator_pdsch_enc_factory>
srsran::hal::create_hw_accelerator_pdsch_enc_factory(const hw_accelerator_pdsch_enc_configuration& accelerator_config)
{
  return create_hw_accelerator_pdsch_enc_factory_hip(accelerator_config);
}

std::shared_ptr<ext_harq_buffer_context_repository>
srsran::hal::create_ext_harq_buffer_context_repository(unsigned nof_codeblocks, uint64_t ext_harq_buff_size,
                                                      bool debug_mode)
{
  return std::make_shared<ext_harq_buffer_context_repository>(nof_codeblocks, ext_harq_buff_size, debug_mode);
}

std::shared_ptr<ldpc_decoder_factory> srsran::create_ldpc_decoder_factory_sw(const std::string& dec_type)
{
  /* out of tree there are no CPU decoders: "auto" is the hybrid without a CPU side (every call on the GPU); in an
   * srsRAN tree the factory branch of INTEGRATION.md 2.1 gives it the reference's own CPU decoder */
  const int dev = hip_device_of_decoder_type(dec_type);
  if (dev < 0) {
    return nullptr;
  }
  return dec_type == "auto" ? create_ldpc_decoder_factory_hip_auto(dev, nullptr) : create_ldpc_decoder_factory_hip(dev);
}

std::shared_ptr<ldpc_rate_dematcher_factory> srsran::create_ldpc_rate_dematcher_factory_sw(const std::string& type)
{
  const int dev = hip_device_of_dematcher_type(type);
  return dev >= 0 ? create_ldpc_rate_dematcher_factory_hip(dev) : nullptr;
}
#endif
