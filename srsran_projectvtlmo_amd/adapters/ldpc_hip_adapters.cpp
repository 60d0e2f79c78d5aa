/*
 * srsRAN-side adapters of the MI355X LDPC decode path: see ldpc_hip_adapters.h.
 * Reference semantics: ldpc_decoder_impl.cpp:60-147 (decode contract, return value), ldpc_rate_dematcher_impl.cpp
 * :46-114 (dematch contract), hw_accelerator_pusch_dec_acc100_impl.cpp (HAL queue semantics incl. dropped ops).
 */
#include "ldpc_hip_adapters.h"

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

ldpc_hip_context::ldpc_hip_context(int device, unsigned nof_harq_slots, unsigned max_queue_cbs,
                                   ldpc_hip_harq_repo* harq_repo)
{
  ldpc_hip_params p{};
  p.max_queue_cbs  = max_queue_cbs;
  p.nof_harq_slots = nof_harq_slots;
  const int rc     = ldpc_hip_open_harq(device, &p, harq_repo, &ctx);
  srsran_assert(rc == LDPC_HIP_OK, "ldpc_hip_open failed");
}

ldpc_hip_context::~ldpc_hip_context()
{
  if (ctx != nullptr) {
    ldpc_hip_close(ctx);
  }
}

std::optional<unsigned> ldpc_decoder_hip::decode(bit_buffer&                      output,
                                                 span<const log_likelihood_ratio> input,
                                                 crc_calculator*                  crc,
                                                 const configuration&             cfg)
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

std::shared_ptr<ldpc_decoder_factory> srsran::create_ldpc_decoder_factory_hip(int device)
{
  return std::make_shared<ldpc_decoder_factory_hip>(device);
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

ext_harq_buffer_context_repository_hip::ext_harq_buffer_context_repository_hip(int device,
                                                                               unsigned nof_codeblocks,
                                                                               bool     debug_mode) :
  dev(device)
{
  const int rc = ldpc_hip_harq_repo_create(device, nof_codeblocks, debug_mode ? 1 : 0, &repo);
  srsran_assert(rc == LDPC_HIP_OK, "ldpc_hip_harq_repo_create failed");
}

ext_harq_buffer_context_repository_hip::~ext_harq_buffer_context_repository_hip()
{
  if (repo != nullptr) {
    (void)ldpc_hip_harq_repo_release(repo);
  }
}

std::shared_ptr<ext_harq_buffer_context_repository_hip>
srsran::hal::create_ext_harq_buffer_context_repository_hip(int device, unsigned nof_codeblocks, bool debug_mode)
{
  return std::make_shared<ext_harq_buffer_context_repository_hip>(device, nof_codeblocks, debug_mode);
}

hw_accelerator_pusch_dec_hip::hw_accelerator_pusch_dec_hip(const hw_accelerator_pusch_dec_hip_configuration& cfg) :
  harq(cfg.ext_softbuffer ? cfg.harq_buffer_context : nullptr),
  ctx(cfg.device,
      (cfg.ext_softbuffer && !harq) ? cfg.nof_harq_slots : 0,
      cfg.max_queue_cbs,
      harq ? harq->get() : nullptr),
  cfgs(cfg.max_queue_cbs != 0 ? cfg.max_queue_cbs : 162)
{
  srsran_assert(!harq || harq->device() == cfg.device, "The HARQ repository lives on another GPU.");
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
  if (cb_index >= cfgs.size()) {
    cfgs.resize(cb_index + 1); /* a TB may have more CBs than one batch holds (MAX_NOF_SEGMENTS) */
  }
  ldpc_hip_hw_config& h     = cfgs[cb_index];
  h                         = ldpc_hip_hw_config{};
  h.base_graph              = static_cast<uint8_t>(c.base_graph_index);
  h.modulation_order        = static_cast<uint8_t>(get_bits_per_symbol(c.modulation));
  h.rv                      = static_cast<uint8_t>(c.rv);
  h.new_data                = c.new_data ? 1 : 0;
  h.nof_segments            = c.nof_segments;
  h.cw_length               = c.cw_length;
  h.lifting_size            = c.lifting_size;
  h.Ncb                     = c.Ncb;
  h.Nref                    = c.Nref;
  h.nof_segment_bits        = c.nof_segment_bits;
  h.nof_filler_bits         = c.nof_filler_bits;
  h.max_nof_ldpc_iterations = c.max_nof_ldpc_iterations;
  h.use_early_stop          = c.use_early_stop ? 1 : 0;
  h.cb_crc_type             = static_cast<uint8_t>(c.cb_crc_type);
  h.cb_crc_len              = static_cast<uint16_t>(c.cb_crc_len);
  h.absolute_cb_id          = c.absolute_cb_id;
}

bool hw_accelerator_pusch_dec_hip::enqueue_operation(span<const int8_t> data, span<const int8_t> aux, unsigned cb)
{
  srsran_assert(cb < cfgs.size(), "enqueue_operation without configure_operation");
  const int rc = ldpc_hip_enqueue(ctx.get(), cb, &cfgs[cb], data.data(), static_cast<uint32_t>(data.size()),
                                  aux.empty() ? nullptr : aux.data(), static_cast<uint32_t>(aux.size()));
  if (rc == LDPC_HIP_EFULL) {
    return false; /* the batch cannot take it now: the caller dequeues, then enqueues again */
  }
  if (rc == LDPC_HIP_DROPPED) {
    return true; /* acc100 drop_op: dequeues as a CRC failure with max iterations (acc100_impl.cpp:179-186) */
  }
  check_rc(ctx.get(), rc);
  return true;
}

bool hw_accelerator_pusch_dec_hip::dequeue_operation(span<uint8_t> data, span<int8_t> aux, unsigned segment_index)
{
  const int rc = ldpc_hip_dequeue(ctx.get(), segment_index, data.data(), static_cast<uint32_t>(data.size()),
                                  aux.empty() ? nullptr : aux.data(), static_cast<uint32_t>(aux.size()));
  if (rc == LDPC_HIP_NOT_READY) {
    return false;
  }
  check_rc(ctx.get(), rc);
  return true;
}

void hw_accelerator_pusch_dec_hip::read_operation_outputs(hw_pusch_decoder_outputs& out, unsigned cb, unsigned id)
{
  ldpc_hip_cb_result r{};
  check_rc(ctx.get(), ldpc_hip_read_outputs(ctx.get(), cb, id, &r));
  out.CRC_pass            = r.crc_pass != 0;
  out.nof_ldpc_iterations = r.nof_iterations;
}

void hw_accelerator_pusch_dec_hip::free_harq_context_entry(unsigned absolute_cb_id)
{
  check_rc(ctx.get(), ldpc_hip_harq_free(ctx.get(), absolute_cb_id));
}

bool hw_accelerator_pusch_dec_hip::is_external_harq_supported() const
{
  return ldpc_hip_external_harq_supported(ctx.get()) != 0;
}

namespace {

class hw_accelerator_pusch_dec_factory_hip : public hw_accelerator_pusch_dec_factory
{
public:
  explicit hw_accelerator_pusch_dec_factory_hip(const hw_accelerator_pusch_dec_hip_configuration& c) : cfg(c)
  {
    /* every accelerator of this factory shares one external HARQ repository (hw_accelerator_factories.cpp:46-65) */
    if (cfg.ext_softbuffer && !cfg.harq_buffer_context) {
      cfg.harq_buffer_context = create_ext_harq_buffer_context_repository_hip(cfg.device, cfg.nof_harq_slots);
    }
  }
  std::unique_ptr<hw_accelerator_pusch_dec> create() override
  {
    return std::make_unique<hw_accelerator_pusch_dec_hip>(cfg);
  }

private:
  hw_accelerator_pusch_dec_hip_configuration cfg;
};

} // namespace

std::shared_ptr<hw_accelerator_pusch_dec_factory>
srsran::hal::create_hw_accelerator_pusch_dec_factory_hip(const hw_accelerator_pusch_dec_hip_configuration& cfg)
{
  return std::make_shared<hw_accelerator_pusch_dec_factory_hip>(cfg);
}

/* ---- hw_accelerator_pdsch_enc (hw_accelerator_pdsch_enc_acc100_impl.cpp semantics on the GPU) ---- */

hw_accelerator_pdsch_enc_hip::hw_accelerator_pdsch_enc_hip(const hw_accelerator_pdsch_enc_hip_configuration& cfg) :
  ctx(cfg.device)
{
  check_rc(ctx.get(), ldpc_hip_enc_queue_create(ctx.get(), cfg.cb_mode ? 1 : 0, cfg.max_queue_cbs, cfg.max_tb_size,
                                                &queue));
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
  explicit hw_accelerator_pdsch_enc_factory_hip(const hw_accelerator_pdsch_enc_hip_configuration& c) : cfg(c) {}
  std::unique_ptr<hw_accelerator_pdsch_enc> create() override
  {
    return std::make_unique<hw_accelerator_pdsch_enc_hip>(cfg);
  }

private:
  hw_accelerator_pdsch_enc_hip_configuration cfg;
};

} // namespace

std::shared_ptr<hw_accelerator_pdsch_enc_factory>
srsran::hal::create_hw_accelerator_pdsch_enc_factory_hip(const hw_accelerator_pdsch_enc_hip_configuration& cfg)
{
  return std::make_shared<hw_accelerator_pdsch_enc_factory_hip>(cfg);
}
