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
 * GPU's HARQ memory is shared by the accelerators of a GPU and is thread-safe; the caller's
 * ext_harq_buffer_context_repository holds the entry state, as with acc100.
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
#include <string>
#include <vector>

namespace srsran {

/* Owns an ldpc_hip_ctx (one GPU, one stream). With `harq_repo` (the device's HARQ memory) its HAL queue keeps the
 * soft buffers there; launch_flags: LDPC_HIP_LAUNCH_* (e.g. LDPC_HIP_LAUNCH_SHARED_QUEUE). */
class ldpc_hip_context
{
public:
  explicit ldpc_hip_context(int device = 0, ldpc_hip_harq_repo* harq_repo = nullptr, uint32_t launch_flags = 0);
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

/* The "auto" decoder type on a host with a gfx950: each codeblock goes to the decoder
 * that measured faster for its work (ldpc_hip_decode_work: layer edges x Z x max_iterations). Below min_work
 * (ldpc_hip_auto_min_work(): LDPC_HIP_AUTO_MIN_WORK or the measured crossover) it stays on `cpu`, the CPU decoder the
 * reference's "auto" would have built (channel_coding_factories.cpp:100-121: AVX-512, AVX2 or generic); above it the
 * GPU decodes it (created on first use). The calling thread waits for a GPU call (it spins on the done word), so a
 * GPU call frees no CPU time: the choice is by latency only. */
class ldpc_decoder_hip_auto : public ldpc_decoder
{
public:
  ldpc_decoder_hip_auto(int device, std::unique_ptr<ldpc_decoder> cpu, uint64_t min_work);
  std::optional<unsigned> decode(bit_buffer&                      output,
                                 span<const log_likelihood_ratio> input,
                                 crc_calculator*                  crc,
                                 const configuration&             cfg) override;
  uint64_t cpu_calls() const { return n_cpu; }
  uint64_t gpu_calls() const { return n_gpu; }

private:
  int                               device;
  std::unique_ptr<ldpc_decoder>     cpu;
  std::unique_ptr<ldpc_decoder_hip> gpu;
  uint64_t                          min_work;
  uint64_t                          n_cpu = 0, n_gpu = 0;
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
/* "auto" with a GPU: decoders of type ldpc_decoder_hip_auto, each with a CPU decoder from `cpu_factory` (the factory of
 * the CPU type the reference's "auto" picks) and the threshold ldpc_hip_auto_min_work() unless min_work is given. */
std::shared_ptr<ldpc_decoder_factory> create_ldpc_decoder_factory_hip_auto(int                                   device,
                                                                           std::shared_ptr<ldpc_decoder_factory> cpu_factory,
                                                                           uint64_t min_work = ldpc_hip_auto_min_work());
std::shared_ptr<ldpc_rate_dematcher_factory> create_ldpc_rate_dematcher_factory_hip(int device = 0);

/* The GPU a software-factory type string selects: "hip" -> 0, "hip:<n>" -> n; -1 when the string is not a HIP type.
 * One cell per GPU: cell c's upper PHY gets ldpc_decoder_type / ldpc_rate_dematcher_type = "hip:" + (c mod G). */
int hip_device_of(const char* type);

/* The GPU ldpc_decoder_factory_sw::create (channel_coding_factories.cpp:100-124) hands a decoder type to: "hip" /
 * "hip:<n>" as hip_device_of, and "auto" -- the type du_low_config_translator.cpp:160-162 sets -- to
 * ldpc_hip_auto_device() (a visible gfx950, else -1: the CPU decoders). */
int hip_device_of_decoder_type(const std::string& dec_type);
/* The same for ldpc_rate_dematcher_factory_sw::create (:166-192): "hip" / "hip:<n>" only. "auto" keeps the CPU
 * dematcher: on the software route its output is the caller's host soft buffer (rx_buffer), so on the GPU every
 * codeblock's N soft bits would cross PCIe twice for E + N bytes of work. */
int hip_device_of_dematcher_type(const std::string& dematcher_type);

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

/* The GPU an acc_type string selects: "mi355x" -> 0, "mi355x:<n>" -> n (one cell per GPU: cell c takes
 * "mi355x:" + (c mod G)); -1 when the string names another accelerator. */
int hip_device_of_acc_type(const std::string& acc_type);

/* hal::hw_accelerator_pusch_dec on an MI355X, built from the reference's own hw_accelerator_pusch_dec_configuration
 * (pusch/hw_accelerator_factories.h:33-44) exactly as acc100 is (hw_accelerator_pusch_dec_acc100_impl.{h,cpp}):
 *   acc_type            "mi355x" / "mi355x:<n>" (the GPU);
 *   ext_softbuffer      true: soft bits in the GPU's HARQ memory (HBM, owned by the library, one per device, indexed
 *                       by absolute_cb_id: ldpc_hip_harq_device_memory); false: in the caller's host soft buffers;
 *   harq_buffer_context the caller's repository: configure_operation takes the CB's entry (get(absolute_cb_id,
 *                       new_data)), enqueue_operation drops a retransmission whose entry holds no soft data,
 *                       dequeue_operation records the soft-data length, free_harq_context_entry frees the entry
 *                       (acc100_impl.cpp:113, 123-125, 184-186, 206-211, 270);
 *   dedicated_queue     true: the accelerator's own HIP stream; false: reserve_queue borrows one of the device's
 *                       shared streams (spinning until one is free) and free_queue returns it (acc100_impl.cpp:70-98);
 *   bbdev_accelerator   unused (no DPDK device).
 * Not thread-safe, like the reference's accelerators: one per PUSCH decoder. */
class hw_accelerator_pusch_dec_hip : public hw_accelerator_pusch_dec
{
public:
  explicit hw_accelerator_pusch_dec_hip(const hw_accelerator_pusch_dec_configuration& cfg);
  void reserve_queue() override;
  void free_queue() override;
  void configure_operation(const hw_pusch_decoder_configuration& config, unsigned cb_index = 0) override;
  bool enqueue_operation(span<const int8_t> data, span<const int8_t> aux_data = {}, unsigned cb_index = 0) override;
  bool dequeue_operation(span<uint8_t> data, span<int8_t> aux_data = {}, unsigned segment_index = 0) override;
  void read_operation_outputs(hw_pusch_decoder_outputs& out, unsigned cb_index = 0, unsigned id = 0) override;
  void free_harq_context_entry(unsigned absolute_cb_id) override;
  bool is_external_harq_supported() const override;

private:
  bool                                                ext_softbuffer;
  std::shared_ptr<ext_harq_buffer_context_repository> harq_buffer_context;
  ldpc_hip_context                                    ctx;
  std::vector<ldpc_hip_hw_config>                     cfgs;
  std::vector<ext_harq_buffer_context_entry*>         harq_context_entries;
  std::vector<uint8_t>                                drop_op; /* acc100's drop_op bitset */
};

/* The factory the reference's create_hw_accelerator_pusch_dec_factory returns for acc_type "mi355x[:n]"
 * (INTEGRATION.md section 2.2): every accelerator it creates shares the caller's repository and the GPU's HARQ
 * memory, so a retransmission may be decoded by another PUSCH decoder than the first transmission. */
std::shared_ptr<hw_accelerator_pusch_dec_factory>
create_hw_accelerator_pusch_dec_factory_hip(const hw_accelerator_pusch_dec_configuration& cfg);

/* PDSCH encoder plugin: LDPC encoding + rate matching of a codeblock (CB mode) or of a whole TB (TB mode: TB CRC,
 * segmentation, CB CRC) on the GPU (ldpc_hip_enc_* in srsran_ldpc_hip.h), built from the reference's
 * hw_accelerator_pdsch_enc_configuration (channel_processors/hw_accelerator_factories.h:31-43): acc_type "mi355x[:n]",
 * cb_mode, max_tb_size (bytes; 0: the largest NR TBS), dedicated_queue as for the PUSCH decoder. */
class hw_accelerator_pdsch_enc_hip : public hw_accelerator_pdsch_enc
{
public:
  explicit hw_accelerator_pdsch_enc_hip(const hw_accelerator_pdsch_enc_configuration& cfg);
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
create_hw_accelerator_pdsch_enc_factory_hip(const hw_accelerator_pdsch_enc_configuration& cfg);

} // namespace hal
} // namespace srsran
