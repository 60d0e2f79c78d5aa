/*
 * srsRAN-side adapters of the MI355X LDPC decode path (C++ host code above the C ABI of include/srsran_ldpc_hip.h).
 *
 *   srsran::ldpc_decoder_hip            : ldpc_decoder         (ldpc_decoder.h:37-75)        factory type "hip"
 *   srsran::ldpc_rate_dematcher_hip     : ldpc_rate_dematcher  (ldpc_rate_dematcher.h:35-56) factory type "hip"
 *   srsran::demodulation_mapper_hip     : demodulation_mapper  (demodulation_mapper.h:46-70)  channel_modulation_factory
 *   srsran::hal::hw_accelerator_pusch_dec_hip : hal::hw_accelerator_pusch_dec (hw_accelerator_pusch_dec.h:83-115)
 *                                                                                       acc_type "mi355x"
 *   srsran::hal::hw_accelerator_pdsch_enc_hip : hal::hw_accelerator_pdsch_enc (hw_accelerator_pdsch_enc.h:75-102)
 *                                                                                       acc_type "mi355x"
 *
 * In an srsRAN tree (SRSRAN_LDPC_HIP_IN_TREE) they build against the real headers and plug into
 * create_ldpc_decoder_factory_sw("hip"), create_ldpc_rate_dematcher_factory_sw("hip") and
 * hal::create_hw_accelerator_pusch_dec_factory. Outside it, compat/srsran_minimal.h supplies
 * the interface types so the adapters can be built and tested here.
 *
 * Objects are not thread-safe (like the reference decoders, one per worker thread); each owns one ldpc_hip_ctx. The
 * external HARQ repository is shared by the accelerators of a GPU and is thread-safe.
 * Contract violations abort through srsran_assert, as the reference's implementations do.
 */
#pragma once

#ifdef SRSRAN_LDPC_HIP_IN_TREE
#include "srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc_factory.h"
#include "srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec_factory.h"
#include "srsran/phy/upper/channel_coding/channel_coding_factories.h"
#include "srsran/phy/upper/channel_modulation/channel_modulation_factories.h"
#include "srsran/support/srsran_assert.h"
#else
#include "compat/srsran_minimal.h"
#endif

#include "srsran_ldpc_hip.h"

#include <memory>
#include <vector>

namespace srsran {

/* Owns an ldpc_hip_ctx (one GPU, one stream). With `harq_repo` its HAL queue keeps the soft buffers in that shared
 * external HARQ repository; otherwise nof_harq_slots != 0 gives it a private one. */
class ldpc_hip_context
{
public:
  explicit ldpc_hip_context(int device = 0, unsigned nof_harq_slots = 0, unsigned max_queue_cbs = 0,
                            ldpc_hip_harq_repo* harq_repo = nullptr);
  ~ldpc_hip_context();
  ldpc_hip_context(const ldpc_hip_context&)            = delete;
  ldpc_hip_context& operator=(const ldpc_hip_context&) = delete;
  ldpc_hip_ctx* get() const { return ctx; }

private:
  ldpc_hip_ctx* ctx = nullptr;
};

class ldpc_decoder_hip : public ldpc_decoder
{
public:
  explicit ldpc_decoder_hip(int device = 0) : ctx(device) {}
  std::optional<unsigned> decode(bit_buffer&                      output,
                                 span<const log_likelihood_ratio> input,
                                 crc_calculator*                  crc,
                                 const configuration&             cfg) override;

private:
  ldpc_hip_context ctx;
};

class ldpc_rate_dematcher_hip : public ldpc_rate_dematcher
{
public:
  explicit ldpc_rate_dematcher_hip(int device = 0) : ctx(device) {}
  void rate_dematch(span<log_likelihood_ratio>       output,
                    span<const log_likelihood_ratio> input,
                    bool                             new_data,
                    const codeblock_metadata&        cfg) override;

private:
  ldpc_hip_context ctx;
};

std::shared_ptr<ldpc_decoder_factory>        create_ldpc_decoder_factory_hip(int device = 0);
std::shared_ptr<ldpc_rate_dematcher_factory> create_ldpc_rate_dematcher_factory_hip(int device = 0);

/* The GPU a software-factory type string selects: "hip" -> 0, "hip:<n>" -> n; -1 when the string is not a HIP type.
 * One cell per GPU: cell c's upper PHY gets ldpc_decoder_type / ldpc_rate_dematcher_type = "hip:" + (c mod G). */
int hip_device_of(const char* type);

/* Soft demodulation on the GPU: bit-exact with the reference's portable per-symbol
 * demappers (demodulation_mapper_*.cpp). */
class demodulation_mapper_hip : public demodulation_mapper
{
public:
  explicit demodulation_mapper_hip(int device = 0) : ctx(device) {}
  void demodulate_soft(span<log_likelihood_ratio> llrs,
                       span<const cf_t>           symbols,
                       span<const float>          noise_vars,
                       modulation_scheme          mod) override;

private:
  ldpc_hip_context ctx;
};

/* channel_modulation_factory whose demodulation mappers run on the GPU; EVM calculators come from `evm_source`
 * (e.g. create_channel_modulation_sw_factory()) when given, else nullptr. */
std::shared_ptr<channel_modulation_factory>
create_channel_modulation_factory_hip(int device = 0, std::shared_ptr<channel_modulation_factory> evm_source = nullptr);

namespace hal {

/* The external HARQ buffer context repository with its HBM soft buffers, on one GPU: hal::
 * ext_harq_buffer_context_repository (ext_harq_buffer_context_repository.h:44-96) plus the accelerator HARQ memory it
 * describes. ONE is shared by every hw_accelerator_pusch_dec_hip of a cell (all PUSCH decoder threads), as the
 * reference shares one repository among the accelerators its factory creates (hw_accelerator_factories.h:41,
 * hw_accelerator_factories.cpp:46-65): a retransmission may reach a different decoder than the first transmission. */
class ext_harq_buffer_context_repository_hip
{
public:
  ext_harq_buffer_context_repository_hip(int device, unsigned nof_codeblocks, bool debug_mode);
  ~ext_harq_buffer_context_repository_hip();
  ext_harq_buffer_context_repository_hip(const ext_harq_buffer_context_repository_hip&)            = delete;
  ext_harq_buffer_context_repository_hip& operator=(const ext_harq_buffer_context_repository_hip&) = delete;
  ldpc_hip_harq_repo* get() const { return repo; }
  int                 device() const { return dev; }

private:
  ldpc_hip_harq_repo* repo = nullptr;
  int                 dev  = 0;
};

/* create_ext_harq_buffer_context_repository (ext_harq_buffer_context_repository_factory.cpp:28-34) on a GPU. */
std::shared_ptr<ext_harq_buffer_context_repository_hip>
create_ext_harq_buffer_context_repository_hip(int device, unsigned nof_codeblocks, bool debug_mode = false);

/* hw_accelerator_pusch_dec_configuration (hw_accelerator_factories.h:33-44) for acc_type "mi355x". */
struct hw_accelerator_pusch_dec_hip_configuration {
  int      device         = 0;
  bool     ext_softbuffer = true; /* soft buffers in HBM, in the external HARQ repository */
  /* the shared external HARQ repository (harq_buffer_context); when null, the factory creates one of nof_harq_slots
   * entries on `device` and shares it among every accelerator it creates */
  std::shared_ptr<ext_harq_buffer_context_repository_hip> harq_buffer_context;
  unsigned nof_harq_slots = 1024;
  unsigned max_queue_cbs  = 162;
};

class hw_accelerator_pusch_dec_hip : public hw_accelerator_pusch_dec
{
public:
  explicit hw_accelerator_pusch_dec_hip(const hw_accelerator_pusch_dec_hip_configuration& cfg);
  void reserve_queue() override;
  void free_queue() override;
  void configure_operation(const hw_pusch_decoder_configuration& config, unsigned cb_index = 0) override;
  bool enqueue_operation(span<const int8_t> data, span<const int8_t> aux_data = {}, unsigned cb_index = 0) override;
  bool dequeue_operation(span<uint8_t> data, span<int8_t> aux_data = {}, unsigned segment_index = 0) override;
  void read_operation_outputs(hw_pusch_decoder_outputs& out, unsigned cb_index = 0, unsigned id = 0) override;
  void free_harq_context_entry(unsigned absolute_cb_id) override;
  bool is_external_harq_supported() const override;

private:
  std::shared_ptr<ext_harq_buffer_context_repository_hip> harq; /* keeps the shared repository alive */
  ldpc_hip_context                                        ctx;
  std::vector<ldpc_hip_hw_config>                         cfgs;
};

std::shared_ptr<hw_accelerator_pusch_dec_factory>
create_hw_accelerator_pusch_dec_factory_hip(const hw_accelerator_pusch_dec_hip_configuration& cfg);

struct hw_accelerator_pdsch_enc_hip_configuration {
  int      device        = 0;
  bool     cb_mode       = false; /* get_cb_mode(): CB mode (one codeblock per operation) or TB mode */
  unsigned max_tb_size   = 0;     /* get_max_tb_size() in bytes; 0: the largest NR TBS */
  unsigned max_queue_cbs = 162;   /* codeblocks one batch holds */
};

/* PDSCH encoder plugin: LDPC encoding + rate matching of a codeblock (CB mode) or of a whole TB (TB mode: TB CRC,
 * segmentation, CB CRC) on the GPU (ldpc_hip_enc_* in srsran_ldpc_hip.h). */
class hw_accelerator_pdsch_enc_hip : public hw_accelerator_pdsch_enc
{
public:
  explicit hw_accelerator_pdsch_enc_hip(const hw_accelerator_pdsch_enc_hip_configuration& cfg);
  ~hw_accelerator_pdsch_enc_hip() override;
  void     reserve_queue() override;
  void     free_queue() override;
  void     configure_operation(const hw_pdsch_encoder_configuration& config, unsigned cb_index = 0) override;
  bool     enqueue_operation(span<const uint8_t> data, span<const uint8_t> aux_data = {}, unsigned cb_index = 0) override;
  bool     dequeue_operation(span<uint8_t> data, span<uint8_t> packed_data = {}, unsigned segment_index = 0) override;
  bool     get_cb_mode() const override;
  unsigned get_max_tb_size() const override;

private:
  ldpc_hip_context    ctx;
  ldpc_hip_enc_queue* queue = nullptr;
};

std::shared_ptr<hw_accelerator_pdsch_enc_factory>
create_hw_accelerator_pdsch_enc_factory_hip(const hw_accelerator_pdsch_enc_hip_configuration& cfg);

} // namespace hal
} // namespace srsran
