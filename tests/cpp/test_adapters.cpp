/*
 * C++ test of the srsRAN-side adapters (ldpc_decoder_hip, ldpc_rate_dematcher_hip, hw_accelerator_pusch_dec_hip,
 * demodulation_mapper_hip, hw_accelerator_pdsch_enc_hip)
 * against the CPU oracle, in the style of the reference's gtest suites (ldpc_enc_dec_test.cpp, ldpc_rm_test.cpp,
 * pusch_decoder_vectortest.cpp). Needs a GPU. Exit code 0 = all checks passed.
 */
#include "ldpc_hip_adapters.h"

extern "C" {
#include "ldpc_oracle.h"
}

#include <cstdio>
#include <random>
#include <vector>

using namespace srsran;

static int failures = 0;
#define CHECK(cond, what)                                                                                            \
  do {                                                                                                               \
    if (!(cond)) {                                                                                                   \
      std::printf("FAIL: %s (%s:%d)\n", what, __FILE__, __LINE__);                                                   \
      ++failures;                                                                                                    \
    }                                                                                                                \
  } while (0)

class crc_poly_only : public crc_calculator
{
public:
  explicit crc_poly_only(crc_generator_poly p) : poly(p) {}
  crc_generator_poly get_generator_poly() const override { return poly; }
  unsigned           calculate(const bit_buffer&) override { return 0; }

private:
  crc_generator_poly poly;
};

static void test_decoder(std::mt19937& rng)
{
  auto factory = create_ldpc_decoder_factory_hip(0);
  auto dec     = factory->create();
  struct tc {
    int      bg;
    unsigned Z, F, iters;
    bool     crc;
  };
  const tc cases[] = {{2, 52, 0, 6, false}, {1, 384, 0, 8, false}, {2, 208, 0, 10, true}, {1, 36, 40, 4, true}};
  for (const tc& c : cases) {
    const unsigned K = c.bg == 1 ? 22 : 10, N = (c.bg == 1 ? 66 : 50) * c.Z, KZ = K * c.Z;
    std::vector<uint8_t> msg(KZ);
    for (unsigned i = 0; i != KZ; ++i) {
      msg[i] = (i >= KZ - c.F) ? ORC_FILLER_BIT : static_cast<uint8_t>(rng() & 1U);
    }
    if (c.crc) { /* CRC24B over the significant bits before the filler */
      const unsigned L = KZ - c.F;
      uint32_t       r = orc_crc_bits(ORC_CRC24B, msg.data(), L - 24);
      for (unsigned i = 0; i != 24; ++i) {
        msg[L - 24 + i] = (r >> (23 - i)) & 1U;
      }
    }
    std::vector<uint8_t> cw(N);
    orc_ldpc_encode(c.bg, c.Z, msg.data(), cw.data(), N);
    std::normal_distribution<float>   noise(0.0f, 1.0f);
    std::vector<log_likelihood_ratio> llr(N);
    std::vector<int8_t>               llr8(N);
    for (unsigned i = 0; i != N; ++i) {
      const float x = (cw[i] == ORC_FILLER_BIT) ? 100.0f : (cw[i] ? -2.0f : 2.0f) + 0.9f * noise(rng);
      llr8[i]       = orc_llr_quantize(x, 8.0f);
      llr[i]        = llr8[i];
    }
    std::vector<uint8_t> out((KZ + 7) / 8, 0), ref((KZ + 7) / 8, 0);
    bit_buffer           bb(span<uint8_t>(out.data(), out.size()), KZ);
    ldpc_decoder::configuration cfg;
    cfg.block_conf.tb_common.base_graph       = static_cast<ldpc_base_graph_type>(c.bg);
    cfg.block_conf.tb_common.lifting_size     = static_cast<ldpc::lifting_size_t>(c.Z);
    cfg.block_conf.cb_specific.nof_filler_bits = c.F;
    cfg.algorithm_conf.max_iterations          = c.iters;
    crc_poly_only                crc(crc_generator_poly::CRC24B);
    std::optional<unsigned>      r   = dec->decode(bb, span<const log_likelihood_ratio>(llr), c.crc ? &crc : nullptr, cfg);
    const int                    rr  = orc_ldpc_decode(c.bg, c.Z, c.F, llr8.data(), N, c.iters, 0.8f,
                                                       c.crc ? ORC_CRC24B : -1, ref.data());
    CHECK(out == ref, "decoder output differs from the oracle");
    CHECK((r.has_value() ? static_cast<int>(*r) : 0) == rr, "decoder iteration count differs from the oracle");
  }
}

static void test_dematcher(std::mt19937& rng)
{
  auto dm = create_ldpc_rate_dematcher_factory_hip(0)->create();
  struct tc {
    unsigned N, E, rv, F, Nref;
    modulation_scheme mod;
  };
  const tc cases[] = {{66 * 384, 9728, 0, 0, 0, modulation_scheme::QAM256}, {50 * 36, 1248, 2, 88, 0, modulation_scheme::QPSK},
                      {50 * 52, 3000, 3, 20, 0, modulation_scheme::QAM16}, {66 * 52, 1500, 1, 0, 2000, modulation_scheme::QAM64}};
  for (const tc& c : cases) {
    for (int new_data = 1; new_data >= 0; --new_data) {
      std::vector<log_likelihood_ratio> buf(c.N), in(c.E);
      std::vector<int8_t>               ref(c.N), in8(c.E);
      for (unsigned i = 0; i != c.N; ++i) {
        ref[i] = static_cast<int8_t>(static_cast<int>(rng() % 241) - 120);
        buf[i] = ref[i];
      }
      for (unsigned i = 0; i != c.E; ++i) {
        in8[i] = static_cast<int8_t>(static_cast<int>(rng() % 241) - 120);
        in[i]  = in8[i];
      }
      codeblock_metadata m;
      m.tb_common.rv              = c.rv;
      m.tb_common.mod             = c.mod;
      m.tb_common.Nref            = c.Nref;
      m.cb_specific.nof_filler_bits = c.F;
      dm->rate_dematch(span<log_likelihood_ratio>(buf), span<const log_likelihood_ratio>(in), new_data != 0, m);
      orc_rate_dematch(ref.data(), c.N, in8.data(), c.E, new_data, c.rv, get_bits_per_symbol(c.mod), c.Nref, c.F);
      bool same = true;
      for (unsigned i = 0; i != c.N; ++i) {
        same = same && (buf[i].to_value_type() == ref[i]);
      }
      CHECK(same, "rate dematcher output differs from the oracle");
    }
  }
}

static void test_hal(std::mt19937& rng)
{
  for (int ext = 1; ext >= 0; --ext) {
    hal::hw_accelerator_pusch_dec_hip_configuration hc;
    hc.ext_softbuffer = ext != 0;
    hc.nof_harq_slots = 16;
    /* with external HARQ, two accelerators of one factory share its HARQ repository: A takes the first transmission,
     * B (another PUSCH decoder thread) the retransmissions, combining with A's soft bits in HBM */
    auto factory = hal::create_hw_accelerator_pusch_dec_factory_hip(hc);
    auto acc_a   = factory->create();
    auto acc_b   = factory->create();
    CHECK(acc_a->is_external_harq_supported() == (ext != 0), "external HARQ flag");
    const unsigned Z = 208, K = 10, N = 50 * Z, KZ = K * Z, E = 4000;
    std::vector<uint8_t> msg(KZ);
    for (auto& b : msg) {
      b = rng() & 1U;
    }
    uint32_t crc = orc_crc_bits(ORC_CRC16, msg.data(), KZ - 16);
    for (unsigned i = 0; i != 16; ++i) {
      msg[KZ - 16 + i] = (crc >> (15 - i)) & 1U;
    }
    std::vector<uint8_t> cw(N), e(E);
    orc_ldpc_encode(2, Z, msg.data(), cw.data(), N);
    std::vector<int8_t> soft_hw(N, 0), soft_ref(N, 0);
    std::normal_distribution<float> noise(0.0f, 1.0f);
    const unsigned rvs[4] = {0, 2, 3, 1};
    for (unsigned t = 0; t != 4; ++t) {
      orc_rate_match(e.data(), E, cw.data(), N, rvs[t], 2, 0, 2, Z);
      std::vector<int8_t> llr(E);
      for (unsigned i = 0; i != E; ++i) {
        llr[i] = orc_llr_quantize((e[i] ? -1.0f : 1.0f) + 1.6f * noise(rng), 8.0f);
      }
      hal::hw_pusch_decoder_configuration c{};
      c.base_graph_index        = ldpc_base_graph_type::BG2;
      c.modulation              = modulation_scheme::QPSK;
      c.nof_segments            = 1;
      c.rv                      = rvs[t];
      c.cw_length               = E;
      c.lifting_size            = Z;
      c.Ncb                     = N;
      c.nof_filler_bits         = 0;
      c.max_nof_ldpc_iterations = 6;
      c.use_early_stop          = true;
      c.new_data                = t == 0;
      c.cb_crc_len              = 16;
      c.cb_crc_type             = hal::hw_dec_cb_crc_type::CRC16;
      c.absolute_cb_id          = 7;
      auto& acc                 = (ext != 0 && t > 0) ? acc_b : acc_a;
      acc->reserve_queue();
      acc->configure_operation(c, 0);
      CHECK(acc->enqueue_operation(span<const int8_t>(llr), ext ? span<const int8_t>() : span<const int8_t>(soft_hw), 0),
            "enqueue");
      std::vector<uint8_t> out((KZ + 7) / 8, 0), ref((KZ + 7) / 8, 0);
      while (!acc->dequeue_operation(span<uint8_t>(out), ext ? span<int8_t>() : span<int8_t>(soft_hw), 0)) {
      }
      hal::hw_pusch_decoder_outputs o{};
      acc->read_operation_outputs(o, 0, 7);
      acc->free_queue();
      const int rr = orc_pusch_cb_decode(ref.data(), soft_ref.data(), N, llr.data(), E, t == 0, 2, Z, rvs[t], 2, 0, 0,
                                         ORC_CRC16, 1, 6);
      CHECK(out == ref, "HAL message differs from the oracle");
      CHECK(o.CRC_pass == (rr > 0), "HAL CRC status differs from the oracle");
      CHECK(!o.CRC_pass || static_cast<int>(o.nof_ldpc_iterations) == rr, "HAL iterations differ from the oracle");
      if (!ext) {
        CHECK(soft_hw == soft_ref, "HAL soft buffer differs from the oracle");
      }
      if (o.CRC_pass) {
        acc->free_harq_context_entry(7);
        break;
      }
    }
  }
}

static void test_demodulator(std::mt19937& rng)
{
  auto factory = create_channel_modulation_factory_hip(0);
  auto demod   = factory->create_demodulation_mapper();
  CHECK(factory->create_evm_calculator() == nullptr, "no EVM source -> no EVM calculator");
  std::normal_distribution<float> g(0.0F, 0.7F);
  for (modulation_scheme m : {modulation_scheme::PI_2_BPSK, modulation_scheme::BPSK, modulation_scheme::QPSK,
                              modulation_scheme::QAM16, modulation_scheme::QAM64, modulation_scheme::QAM256}) {
    const unsigned    n = 1031, qm = get_bits_per_symbol(m);
    std::vector<cf_t> sym(n);
    std::vector<float> nv(n);
    for (unsigned i = 0; i != n; ++i) {
      sym[i] = cf_t(g(rng), g(rng));
      nv[i]  = (i % 97 == 0) ? 0.0F : 0.05F + 0.01F * static_cast<float>(i % 7);
    }
    sym[5] = cf_t(0, 0);
    std::vector<log_likelihood_ratio> llr(n * qm);
    demod->demodulate_soft(span<log_likelihood_ratio>(llr), span<const cf_t>(sym), span<const float>(nv), m);
    std::vector<int8_t> ref(n * qm);
    orc_demodulate_soft(static_cast<int>(m), n, reinterpret_cast<const float*>(sym.data()), nv.data(), ref.data());
    bool same = true;
    for (unsigned i = 0; i != n * qm; ++i) {
      same = same && llr[i].to_int() == ref[i];
    }
    CHECK(same, "demodulation_mapper_hip differs from the oracle");
  }
}

/* pdsch_encoder_hw_impl::encode's call order (pdsch_encoder_hw_impl.cpp:31-170) through hw_accelerator_pdsch_enc_hip,
 * TB mode and CB mode, against the oracle's TB CRC -> segments -> CB CRC24B -> encoder -> rate matcher. */
static void test_pdsch_encoder(std::mt19937& rng)
{
  struct tc {
    unsigned          tbs;
    int               bg;
    unsigned          nsym, layers, rv, Nref;
    modulation_scheme mod;
  };
  const tc cases[] = {{1078248, 1, 250 * 156 * 4, 4, 0, 0, modulation_scheme::QAM256},
                      {256, 2, 156 * 4, 4, 0, 0, modulation_scheme::QPSK},
                      {40000, 2, 52 * 156, 2, 2, 0, modulation_scheme::QAM64},
                      {30000, 1, 40 * 156, 2, 1, 12672, modulation_scheme::QPSK}};
  for (bool cb_mode : {false, true}) {
    hal::hw_accelerator_pdsch_enc_hip_configuration acfg;
    acfg.cb_mode = cb_mode;
    auto enc     = hal::create_hw_accelerator_pdsch_enc_factory_hip(acfg)->create();
    CHECK(enc->get_cb_mode() == cb_mode, "get_cb_mode");
    for (const tc& c : cases) {
      const unsigned Qm = get_bits_per_symbol(c.mod);
      std::vector<orc_cb_meta> meta(200);
      const int C = orc_segment_rx(c.tbs, c.bg, c.nsym, Qm, c.layers, meta.data(), 200);
      CHECK(C > 0, "segmentation");
      const unsigned Z = meta[0].lifting_size, F = meta[0].nof_filler_bits, KZ = (c.bg == 1 ? 22U : 10U) * Z;
      const unsigned N = (c.bg == 1 ? 66U : 50U) * Z, L = c.tbs > 3824 ? 24U : 16U, cbc = C > 1 ? 24U : 0U;
      std::vector<uint8_t> tb(c.tbs / 8);
      for (uint8_t& b : tb) {
        b = static_cast<uint8_t>(rng());
      }
      /* expected codeword (oracle) */
      std::vector<uint8_t> bits(c.tbs + L);
      for (unsigned i = 0; i != c.tbs; ++i) {
        bits[i] = (tb[i / 8] >> (7 - i % 8)) & 1U;
      }
      const uint32_t tbcrc = orc_crc_bytes(L == 24 ? ORC_CRC24A : ORC_CRC16, tb.data(), c.tbs / 8);
      for (unsigned i = 0; i != L; ++i) {
        bits[c.tbs + i] = (tbcrc >> (L - 1 - i)) & 1U;
      }
      const unsigned kd = KZ - F - cbc;
      std::vector<std::vector<uint8_t>> msgs(C, std::vector<uint8_t>(KZ, 0));
      std::vector<uint8_t>              want;
      for (int r = 0; r != C; ++r) {
        for (unsigned i = 0; i != kd && r * kd + i < bits.size(); ++i) {
          msgs[r][i] = bits[r * kd + i];
        }
        if (C > 1) {
          const uint32_t cc = orc_crc_bits(ORC_CRC24B, msgs[r].data(), kd);
          for (unsigned i = 0; i != 24; ++i) {
            msgs[r][kd + i] = (cc >> (23 - i)) & 1U;
          }
        }
        std::vector<uint8_t> m = msgs[r];
        for (unsigned i = KZ - F; i != KZ; ++i) {
          m[i] = ORC_FILLER_BIT;
        }
        std::vector<uint8_t> cw(N), e(meta[r].rm_length);
        orc_ldpc_encode(c.bg, Z, m.data(), cw.data(), N);
        orc_rate_match(e.data(), meta[r].rm_length, cw.data(), N, c.rv, Qm, c.Nref, c.bg, Z);
        want.insert(want.end(), e.begin(), e.end());
      }
      /* the plugin, in pdsch_encoder_hw_impl's order */
      hal::hw_pdsch_encoder_configuration h{};
      const unsigned per_layer = c.nsym / c.layers;
      h.nof_tb_bits            = c.tbs;
      h.nof_tb_crc_bits        = L;
      h.base_graph_index       = static_cast<ldpc_base_graph_type>(c.bg);
      h.modulation             = c.mod;
      h.nof_segments           = static_cast<unsigned>(C);
      h.nof_short_segments     = C - per_layer % C;
      h.rv                     = c.rv;
      h.cw_length_a            = meta[0].rm_length;
      h.cw_length_b            = meta[C - 1].rm_length;
      h.lifting_size           = Z;
      h.Ncb                    = N;
      h.Nref                   = c.Nref;
      h.nof_segment_bits       = kd;
      h.nof_filler_bits        = F;
      h.rm_length              = meta[0].rm_length;
      h.cb_mode                = cb_mode;
      h.tb_crc = L == 24 ? std::vector<uint8_t>{static_cast<uint8_t>(tbcrc >> 16), static_cast<uint8_t>(tbcrc >> 8),
                                                static_cast<uint8_t>(tbcrc)}
                         : std::vector<uint8_t>{static_cast<uint8_t>(tbcrc >> 8), static_cast<uint8_t>(tbcrc)};
      std::vector<uint8_t> got(want.size(), 0xEE);
      enc->reserve_queue();
      if (!cb_mode) {
        enc->configure_operation(h, 0);
        CHECK(enc->enqueue_operation(span<const uint8_t>(tb.data(), tb.size()), {}, 0), "TB enqueue");
        std::vector<uint8_t> packed((got.size() + 7) / 8 + C);
        while (!enc->dequeue_operation(span<uint8_t>(got.data(), got.size()), span<uint8_t>(packed), 0)) {
        }
      } else {
        for (int r = 0; r != C; ++r) {
          h.nof_filler_bits = meta[r].nof_filler_bits;
          h.rm_length       = meta[r].rm_length;
          enc->configure_operation(h, r);
          std::vector<uint8_t> data((KZ - F + 7) / 8, 0);
          for (unsigned i = 0; i != KZ - F; ++i) {
            data[i / 8] = static_cast<uint8_t>(data[i / 8] | (msgs[r][i] << (7 - i % 8)));
          }
          CHECK(enc->enqueue_operation(span<const uint8_t>(data.data(), data.size()), {}, r), "CB enqueue");
        }
        unsigned off = 0;
        for (int r = 0; r != C; ++r) {
          std::vector<uint8_t> packed((meta[r].rm_length + 7) / 8);
          while (!enc->dequeue_operation(span<uint8_t>(got.data() + off, meta[r].rm_length), span<uint8_t>(packed),
                                         r)) {
          }
          off += meta[r].rm_length;
        }
      }
      enc->free_queue();
      CHECK(got == want, cb_mode ? "PDSCH encoder (CB mode) differs from the oracle"
                                 : "PDSCH encoder (TB mode) differs from the oracle");
    }
  }
}

int main()
{
  std::mt19937 rng(0);
  CHECK(hip_device_of("hip") == 0 && hip_device_of("hip:3") == 3 && hip_device_of("hip:") == -1 &&
            hip_device_of("generic") == -1 && hip_device_of("hip:x") == -1,
        "hip_device_of");
  test_decoder(rng);
  test_dematcher(rng);
  test_hal(rng);
  test_demodulator(rng);
  test_pdsch_encoder(rng);
  std::printf("%s: %d failure(s)\n", failures == 0 ? "PASS" : "FAIL", failures);
  return failures == 0 ? 0 : 1;
}
