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

#include <algorithm>
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

/* Test stand-in for the reference's CPU decoder (the "auto" type's CPU side): the oracle's ldpc_decoder_generic
 * restatement behind the ldpc_decoder interface. */
class ldpc_decoder_oracle : public ldpc_decoder
{
public:
  std::optional<unsigned> decode(bit_buffer& output, span<const log_likelihood_ratio> input, crc_calculator* crc,
                                 const configuration& cfg) override
  {
    int poly = -1;
    if (crc != nullptr) {
      const crc_generator_poly p = crc->get_generator_poly();
      poly = p == crc_generator_poly::CRC16 ? ORC_CRC16 : (p == crc_generator_poly::CRC24A ? ORC_CRC24A : ORC_CRC24B);
    }
    const int r = orc_ldpc_decode(static_cast<int>(cfg.block_conf.tb_common.base_graph),
                                  static_cast<unsigned>(cfg.block_conf.tb_common.lifting_size),
                                  cfg.block_conf.cb_specific.nof_filler_bits,
                                  reinterpret_cast<const int8_t*>(input.data()), static_cast<unsigned>(input.size()),
                                  cfg.algorithm_conf.max_iterations, cfg.algorithm_conf.scaling_factor, poly,
                                  output.get_buffer().data());
    return r > 0 ? std::optional<unsigned>(static_cast<unsigned>(r)) : std::nullopt;
  }
};
class ldpc_decoder_oracle_factory : public ldpc_decoder_factory
{
public:
  std::unique_ptr<ldpc_decoder> create() override { return std::make_unique<ldpc_decoder_oracle>(); }
};

static void test_decoder_with(std::mt19937& rng, ldpc_decoder& dec_ref);

static void test_decoder(std::mt19937& rng)
{
  auto factory = create_ldpc_decoder_factory_hip(0);
  auto dec     = factory->create();
  test_decoder_with(rng, *dec);
}

/* The "auto" type with a GPU (ldpc_decoder_hip_auto): every codeblock bit-exact with the oracle on whichever side it
 * runs; threshold 0 sends every call to the GPU, an unreachable one every call to the CPU decoder, the default splits
 * them by ldpc_hip_decode_work. */
static void test_decoder_auto(std::mt19937& rng)
{
  auto cpu = std::make_shared<ldpc_decoder_oracle_factory>();
  for (uint64_t thr : {uint64_t(0), ~uint64_t(0), ldpc_hip_auto_min_work()}) {
    auto dec  = create_ldpc_decoder_factory_hip_auto(0, cpu, thr)->create();
    auto* hyb = static_cast<ldpc_decoder_hip_auto*>(dec.get());
    test_decoder_with(rng, *dec);
    CHECK(hyb->cpu_calls() + hyb->gpu_calls() == 4, "auto decoder: every call routed once");
    if (thr == 0) {
      CHECK(hyb->gpu_calls() == 4, "auto decoder, threshold 0: every call on the GPU");
    } else if (thr == ~uint64_t(0)) {
      CHECK(hyb->cpu_calls() == 4, "auto decoder, unreachable threshold: every call on the CPU decoder");
    } else {
      /* BG1 Z=384, 8 it, no CRC (971 k) on the GPU; BG2 Z=52 (6 it, 61 k), BG2 Z=208 with early stop (82 k) and
       * BG1 Z=36 with early stop (23 k) on the CPU */
      CHECK(hyb->gpu_calls() >= 1 && hyb->cpu_calls() >= 2, "auto decoder, default threshold: split by work");
    }
  }
}

/* A CPU stub for the "auto" type's CPU side: counts its calls and decodes nothing (the split, not
 * the arithmetic, is under test here). */
class ldpc_decoder_counting_stub : public ldpc_decoder
{
public:
  explicit ldpc_decoder_counting_stub(unsigned& n) : calls(n) {}
  std::optional<unsigned> decode(bit_buffer&, span<const log_likelihood_ratio>, crc_calculator*,
                                 const configuration&) override
  {
    ++calls;
    return std::nullopt;
  }

private:
  unsigned& calls;
};
class ldpc_decoder_counting_stub_factory : public ldpc_decoder_factory
{
public:
  unsigned                      calls = 0;
  std::unique_ptr<ldpc_decoder> create() override { return std::make_unique<ldpc_decoder_counting_stub>(calls); }
};

/* Per call: ldpc_decoder_hip_auto sends the codeblock to the CPU side exactly when ldpc_hip_decode_work of its
 * descriptor (computed here from the same configuration, through the C ABI) is below the threshold. Cases of many
 * works: both base graphs, several Z, iteration counts, early stop, shortened inputs (fewer layers), and an all-zero
 * input (work 0); thresholds between them, so both routes occur. */
static void test_decoder_auto_split(std::mt19937& rng)
{
  struct tc {
    int      bg;
    unsigned Z, iters, len;
    bool     crc;
  };
  const tc cases[] = {{1, 384, 8, 66 * 384, false}, {1, 384, 8, 26 * 384, true},  {2, 208, 10, 50 * 208, true},
                      {2, 52, 6, 50 * 52, false},    {1, 36, 4, 30 * 36, true},     {2, 384, 1, 14 * 384, false},
                      {1, 120, 3, 66 * 120, false},  {2, 16, 25, 50 * 16, false},   {1, 2, 8, 0, false}};
  std::vector<uint64_t> works;
  std::vector<std::vector<log_likelihood_ratio>> inputs;
  for (const tc& c : cases) {
    const unsigned                    N = (c.bg == 1 ? 66 : 50) * c.Z;
    std::vector<log_likelihood_ratio> llr(N);
    for (unsigned i = 0; i != c.len; ++i) {
      llr[i] = static_cast<int8_t>((rng() & 1U) != 0 ? 10 : -10);
    }
    ldpc_hip_dec_desc d{};
    d.base_graph     = static_cast<uint8_t>(c.bg);
    d.lifting_size   = static_cast<uint16_t>(c.Z);
    d.max_iterations = static_cast<uint8_t>(c.iters);
    d.crc_mode       = c.crc ? LDPC_HIP_CRC_MODE_EARLY_STOP : LDPC_HIP_CRC_MODE_NONE;
    d.crc_poly       = c.crc ? LDPC_HIP_CRC24B : -1;
    d.llr_length     = N;
    works.push_back(ldpc_hip_decode_work(&d, reinterpret_cast<const int8_t*>(llr.data())));
    inputs.push_back(std::move(llr));
  }
  CHECK(works.back() == 0, "decode work of an all-zero input is 0");
  std::vector<uint64_t> thresholds = {1, ldpc_hip_auto_min_work()};
  std::vector<uint64_t> sorted     = works;
  std::sort(sorted.begin(), sorted.end());
  thresholds.push_back(sorted[sorted.size() / 2]); /* the median: about half the cases on each side */
  for (uint64_t thr : thresholds) {
    auto  cpu  = std::make_shared<ldpc_decoder_counting_stub_factory>();
    auto  dec  = create_ldpc_decoder_factory_hip_auto(0, cpu, thr)->create();
    auto* hyb  = static_cast<ldpc_decoder_hip_auto*>(dec.get());
    bool  both = false, seen_cpu = false, seen_gpu = false;
    for (size_t i = 0; i != std::size(cases); ++i) {
      const tc&            c  = cases[i];
      const unsigned       KZ = (c.bg == 1 ? 22 : 10) * c.Z;
      std::vector<uint8_t> out((KZ + 7) / 8, 0);
      bit_buffer           bb(span<uint8_t>(out.data(), out.size()), KZ);
      ldpc_decoder::configuration cfg;
      cfg.block_conf.tb_common.base_graph   = static_cast<ldpc_base_graph_type>(c.bg);
      cfg.block_conf.tb_common.lifting_size = static_cast<ldpc::lifting_size_t>(c.Z);
      cfg.algorithm_conf.max_iterations      = c.iters;
      crc_poly_only  crc(crc_generator_poly::CRC24B);
      const unsigned cpu0 = hyb->cpu_calls(), gpu0 = hyb->gpu_calls(), stub0 = cpu->calls;
      (void)dec->decode(bb, span<const log_likelihood_ratio>(inputs[i]), c.crc ? &crc : nullptr, cfg);
      const bool want_cpu = works[i] < thr;
      CHECK(hyb->cpu_calls() == cpu0 + (want_cpu ? 1U : 0U) && hyb->gpu_calls() == gpu0 + (want_cpu ? 0U : 1U),
            "auto decoder: the call went to the side ldpc_hip_decode_work < threshold names");
      CHECK(cpu->calls == stub0 + (want_cpu ? 1U : 0U), "auto decoder: the CPU side saw exactly its calls");
      seen_cpu = seen_cpu || want_cpu;
      seen_gpu = seen_gpu || !want_cpu;
    }
    both = seen_cpu && seen_gpu;
    CHECK(thr == 1 || both, "auto decoder split test: both routes exercised");
  }
}

static void test_decoder_with(std::mt19937& rng, ldpc_decoder& dec_ref)
{
  ldpc_decoder* dec = &dec_ref;
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

/* ---- the HAL route in pusch_decoder_vectortest's setup ------------------------------------------------------------
 * A transport block on the transmit side (TS 38.212 5.1-5.4, built from the oracle: TB CRC, segmentation, CB CRC24B,
 * LDPC encoding, rate matching per RV), the oracle's pusch_decoder_impl flow as the checker (sw_flow), and
 * pusch_decoder_hw_impl::on_end_softbits driving a hw_accelerator_pusch_dec (hw_flow) -- the C++ counterparts of
 * tests/tb_chain.py. */
struct tb_chain {
  unsigned                          tbs, C, Z, F, K, N, Qm, tb_crc_len, nof_data_bits;
  int                               bg, cb_crc_poly;
  std::vector<orc_cb_meta>          metas;
  std::vector<uint8_t>              tb_and_crc;
  std::vector<std::vector<uint8_t>> cws;

  tb_chain(std::mt19937& rng, unsigned tbs_, int bg_, unsigned nsym, unsigned qm, unsigned layers) :
    tbs(tbs_), Qm(qm), bg(bg_)
  {
    metas.resize(200);
    const int n = orc_segment_rx(tbs, bg, nsym, qm, layers, metas.data(), 200);
    srsran_assert(n > 0, "segmentation");
    C = static_cast<unsigned>(n);
    metas.resize(C);
    Z          = metas[0].lifting_size;
    F          = metas[0].nof_filler_bits;
    K          = bg == 1 ? 22U : 10U;
    N          = (bg == 1 ? 66U : 50U) * Z;
    tb_crc_len = tbs > 3824 ? 24U : 16U;
    /* select_crc (pusch_decoder_impl.cpp:35-46) */
    cb_crc_poly = C > 1 ? ORC_CRC24B : (tbs > 3824 ? ORC_CRC24A : ORC_CRC16);
    const unsigned cbc = C > 1 ? 24U : 0U;
    nof_data_bits      = K * Z - F - cbc;
    tb_and_crc.resize(tbs + tb_crc_len);
    for (unsigned i = 0; i != tbs; ++i) {
      tb_and_crc[i] = rng() & 1U;
    }
    const uint32_t tc = orc_crc_bits(tb_crc_len == 24 ? ORC_CRC24A : ORC_CRC16, tb_and_crc.data(), tbs);
    for (unsigned i = 0; i != tb_crc_len; ++i) {
      tb_and_crc[tbs + i] = (tc >> (tb_crc_len - 1 - i)) & 1U;
    }
    for (unsigned r = 0, off = 0; r != C; ++r) {
      std::vector<uint8_t> msg(K * Z, 0);
      for (unsigned i = 0; i != nof_data_bits && off + i < tb_and_crc.size(); ++i) {
        msg[i] = tb_and_crc[off + i];
      }
      off += nof_data_bits;
      if (C > 1) {
        const uint32_t cc = orc_crc_bits(ORC_CRC24B, msg.data(), nof_data_bits);
        for (unsigned i = 0; i != 24; ++i) {
          msg[nof_data_bits + i] = (cc >> (23 - i)) & 1U;
        }
      }
      for (unsigned i = K * Z - F; i != K * Z; ++i) {
        msg[i] = ORC_FILLER_BIT;
      }
      cws.emplace_back(N);
      orc_ldpc_encode(bg, Z, msg.data(), cws.back().data(), N);
    }
  }
  /* every CB rate-matched for rv, soft bits amp (1 - 2b) + noise N(0, 1), quantised with range 8 */
  std::vector<std::vector<int8_t>> llrs(std::mt19937& rng, unsigned rv, float amp, float noise) const
  {
    std::normal_distribution<float>  g(0.0f, 1.0f);
    std::vector<std::vector<int8_t>> out;
    for (unsigned r = 0; r != C; ++r) {
      std::vector<uint8_t> e(metas[r].rm_length);
      orc_rate_match(e.data(), metas[r].rm_length, cws[r].data(), N, rv, Qm, 0, bg, Z);
      out.emplace_back(e.size());
      for (size_t i = 0; i != e.size(); ++i) {
        out.back()[i] = orc_llr_quantize((e[i] ? -amp : amp) + noise * g(rng), 8.0f);
      }
    }
    return out;
  }
  unsigned msg_bytes() const { return (K * Z + 7) / 8; }
};

/* per-CB HARQ state of one receive flow */
struct flow_state {
  std::vector<std::vector<uint8_t>> msgs;
  std::vector<uint8_t>              crc_ok;
  std::vector<unsigned>             iters;
  explicit flow_state(const tb_chain& t) : msgs(t.C, std::vector<uint8_t>(t.msg_bytes(), 0)), crc_ok(t.C, 0), iters(t.C, 0) {}
  /* join_and_notify (pusch_decoder_impl.cpp:384-497): the TB CRC over the concatenated data bits */
  bool join(const tb_chain& t)
  {
    std::vector<uint8_t> flat;
    for (const auto& m : msgs) {
      flat.insert(flat.end(), m.begin(), m.end());
    }
    std::vector<uint8_t> tb((t.tbs + 7) / 8);
    const bool ok = orc_tb_join(flat.data(), t.msg_bytes(), t.C, t.K * t.Z, t.F, t.C > 1 ? 24U : t.tb_crc_len, t.tbs,
                                crc_ok.data(), tb.data()) == 1;
    if (!ok && t.C > 1 && std::all_of(crc_ok.begin(), crc_ok.end(), [](uint8_t x) { return x != 0; })) {
      std::fill(crc_ok.begin(), crc_ok.end(), 0); /* reset_codeblocks_crc (:423-428) */
    }
    return ok;
  }
};

/* the checker: pusch_decoder_impl + pusch_codeblock_decoder with the oracle, soft buffers on the host */
struct sw_flow : flow_state {
  std::vector<std::vector<int8_t>> soft;
  unsigned                         nof_iters;
  bool                             es;
  sw_flow(const tb_chain& t, unsigned it, bool early_stop) :
    flow_state(t), soft(t.C, std::vector<int8_t>(t.N, 0)), nof_iters(it), es(early_stop)
  {
  }
  bool transmission(const tb_chain& t, const std::vector<std::vector<int8_t>>& llr, unsigned rv, bool new_data)
  {
    if (new_data) {
      std::fill(crc_ok.begin(), crc_ok.end(), 0);
    }
    for (unsigned r = 0; r != t.C; ++r) {
      if (crc_ok[r]) {
        orc_rate_dematch(soft[r].data(), t.N, llr[r].data(), static_cast<unsigned>(llr[r].size()), new_data, rv, t.Qm, 0,
                         t.F);
        continue; /* pusch_decoder_impl.cpp:336-346 */
      }
      const int it = orc_pusch_cb_decode(msgs[r].data(), soft[r].data(), t.N, llr[r].data(),
                                         static_cast<unsigned>(llr[r].size()), new_data, t.bg, t.Z, rv, t.Qm, 0, t.F,
                                         t.cb_crc_poly, es ? 1 : 0, nof_iters);
      crc_ok[r] = it > 0;
      iters[r]  = it > 0 ? static_cast<unsigned>(it) : nof_iters;
    }
    return join(t);
  }
};

/* the product path: pusch_decoder_hw_impl::on_end_softbits (pusch_decoder_hw_impl.cpp:132-342) over the plugin. With
 * external HARQ every CB not yet passed is enqueued until enqueue_operation returns false, then the enqueued ones are
 * dequeued (spinning) and read; with host HARQ one CB at a time, its soft buffer in host memory. */
struct hw_flow : flow_state {
  std::vector<std::vector<int8_t>> soft;
  unsigned                         nof_iters, abs_base;
  bool                             es;
  hw_flow(const tb_chain& t, unsigned it, bool early_stop, unsigned base) :
    flow_state(t), soft(t.C, std::vector<int8_t>(t.N, 0)), nof_iters(it), abs_base(base), es(early_stop)
  {
  }
  bool transmission(hal::hw_accelerator_pusch_dec& acc, const tb_chain& t, const std::vector<std::vector<int8_t>>& llr,
                    unsigned rv, bool new_data)
  {
    const bool ext = acc.is_external_harq_supported();
    acc.reserve_queue();
    if (new_data) {
      std::fill(crc_ok.begin(), crc_ok.end(), 0);
    }
    hal::hw_pusch_decoder_configuration c{};
    c.base_graph_index        = static_cast<ldpc_base_graph_type>(t.bg);
    c.modulation              = static_cast<modulation_scheme>(t.Qm);
    c.nof_segments            = t.C;
    c.rv                      = rv;
    c.lifting_size            = t.Z;
    c.Ncb                     = t.N;
    c.Nref                    = 0;
    c.nof_segment_bits        = t.nof_data_bits;
    c.nof_filler_bits         = t.F;
    c.max_nof_ldpc_iterations = nof_iters;
    c.use_early_stop          = es;
    c.new_data                = new_data;
    c.cb_crc_len              = t.C > 1 ? 24U : t.tb_crc_len;
    c.cb_crc_type             = t.cb_crc_poly == ORC_CRC24B   ? hal::hw_dec_cb_crc_type::CRC24B
                                : t.cb_crc_poly == ORC_CRC24A ? hal::hw_dec_cb_crc_type::CRC24A
                                                              : hal::hw_dec_cb_crc_type::CRC16;
    unsigned next = 0;
    while (next != t.C) {
      std::vector<unsigned> batch;
      for (; next != t.C; ++next) {
        if (crc_ok[next]) {
          continue;
        }
        c.cw_length      = static_cast<unsigned>(llr[next].size());
        c.absolute_cb_id = abs_base + next;
        acc.configure_operation(c, next);
        const bool enq = acc.enqueue_operation(span<const int8_t>(llr[next].data(), llr[next].size()),
                                               ext ? span<const int8_t>() : span<const int8_t>(soft[next]), next);
        if (!enq) {
          break;
        }
        batch.push_back(next);
        if (!ext) {
          ++next;
          break;
        }
      }
      for (unsigned r : batch) {
        while (!acc.dequeue_operation(span<uint8_t>(msgs[r]), ext ? span<int8_t>() : span<int8_t>(soft[r]), r)) {
        }
        hal::hw_pusch_decoder_outputs o{};
        acc.read_operation_outputs(o, r, abs_base + r);
        crc_ok[r] = o.CRC_pass ? 1 : 0;
        iters[r]  = o.nof_ldpc_iterations;
      }
    }
    acc.free_queue();
    const bool ok = join(t);
    if (ok) { /* copy_tb_and_notify frees the TB's entries (pusch_decoder_hw_impl.cpp:372-389) */
      for (unsigned r = 0; r != t.C; ++r) {
        acc.free_harq_context_entry(abs_base + r);
      }
    }
    return ok;
  }
};

/* pusch_decoder_vectortest.cpp:207-223 with acc_type = "mi355x" the only change (no DPDK EAL / bbdev accelerator:
 * the repository's capacity is what the GPU's HARQ memory holds, which grows to any absolute_cb_id) */
static std::shared_ptr<hal::hw_accelerator_pusch_dec_factory>
create_hw_accelerator_pusch_dec_factory_vectortest(bool ext_softbuffer, bool dedicated_queue, bool test_harq)
{
  unsigned nof_cbs                   = 162; /* MAX_NOF_SEGMENTS */
  uint64_t acc100_ext_harq_buff_size = static_cast<uint64_t>(nof_cbs) * hal::HARQ_INCR_BYTES;
  std::shared_ptr<hal::ext_harq_buffer_context_repository> harq_buffer_context =
      hal::create_ext_harq_buffer_context_repository(nof_cbs, acc100_ext_harq_buff_size, test_harq);

  hal::hw_accelerator_pusch_dec_configuration hw_decoder_config;
  hw_decoder_config.acc_type            = "mi355x";
  hw_decoder_config.bbdev_accelerator   = nullptr;
  hw_decoder_config.ext_softbuffer      = ext_softbuffer;
  hw_decoder_config.harq_buffer_context = harq_buffer_context;
  hw_decoder_config.dedicated_queue     = dedicated_queue;
  return hal::create_hw_accelerator_pusch_dec_factory(hw_decoder_config);
}

/* RV {0, 2, 3, 1} (pusch_decoder_vectortest's rv_sequence) through the plugin vs the oracle flow, with external and
 * host soft buffers, dedicated and shared queues, early stop on and off, and -- external HARQ -- the retransmissions
 * decoded by a second accelerator of the same factory (another PUSCH processor thread). */
static void test_hal_vectortest_setup(std::mt19937& rng)
{
  struct tc {
    unsigned tbs;
    int      bg;
    unsigned nsym, qm, layers;
    float    noise;
  };
  const tc cases[] = {{25000, 1, 2496 * 4, 4, 2, 1.05f}, {256, 2, 156 * 4, 2, 4, 1.75f},
                      {2000, 2, 1872, 2, 1, 1.2f},      {6000, 1, 4000, 2, 2, 1.1f}};
  unsigned combined = 0, runs = 0;
  for (int ext = 1; ext >= 0; --ext) {
    for (int dedicated = 1; dedicated >= 0; --dedicated) {
      for (int es = 1; es >= 0; --es) {
        auto factory = create_hw_accelerator_pusch_dec_factory_vectortest(ext != 0, dedicated != 0, false);
        CHECK(factory != nullptr, "create_hw_accelerator_pusch_dec_factory(acc_type = \"mi355x\")");
        auto acc_a = factory->create();
        auto acc_b = factory->create();
        CHECK(acc_a->is_external_harq_supported() == (ext != 0), "is_external_harq_supported follows ext_softbuffer");
        for (const tc& k : cases) {
          const tb_chain t(rng, k.tbs, k.bg, k.nsym, k.qm, k.layers);
          sw_flow        sw(t, 6, es != 0);
          hw_flow        hw(t, 6, es != 0, 0);
          const unsigned rvs[4] = {0, 2, 3, 1};
          for (unsigned i = 0; i != 4; ++i) {
            const auto llr    = t.llrs(rng, rvs[i], 1.0f, k.noise);
            const bool ok_sw  = sw.transmission(t, llr, rvs[i], i == 0);
            auto&      acc    = (ext != 0 && i > 0) ? *acc_b : *acc_a; /* cross-instance retransmissions */
            const bool ok_hw  = hw.transmission(acc, t, llr, rvs[i], i == 0);
            ++runs;
            CHECK(ok_sw == ok_hw, "HAL TB CRC differs from the oracle flow");
            CHECK(sw.crc_ok == hw.crc_ok, "HAL CB CRC flags differ from the oracle flow");
            CHECK(sw.iters == hw.iters, "HAL iteration counts differ from the oracle flow");
            CHECK(sw.msgs == hw.msgs, "HAL messages differ from the oracle flow");
            if (ext == 0) {
              bool same = true;
              for (unsigned r = 0; r != t.C; ++r) {
                same = same && (sw.crc_ok[r] || sw.soft[r] == hw.soft[r]);
              }
              CHECK(same, "HAL host soft buffers differ from the oracle flow");
            }
            if (ok_sw) {
              break;
            }
            combined += i < 3 ? 1U : 0U;
          }
        }
      }
    }
  }
  CHECK(combined >= 4, "the noise levels must leave TBs for retransmission (HARQ combining exercised)");
  std::printf("hal vectortest setup: %u transmissions, %u needed a retransmission\n", runs, combined);
}

/* acc100's drop contract and the repository's debug mode (ext_harq_buffer_context_repository.h:92-95): after
 * free_harq_context_entry a retransmission of the entry is dropped (CRC failure, maximum iterations) unless the
 * repository keeps entries (debug mode), in which case it combines with the soft bits left in the GPU's memory. */
static void test_hal_drop_and_debug_mode(std::mt19937& rng)
{
  for (int debug = 0; debug != 2; ++debug) {
    auto       factory = create_hw_accelerator_pusch_dec_factory_vectortest(true, true, debug != 0);
    auto       acc     = factory->create();
    tb_chain   t(rng, 256, 2, 156 * 4, 2, 4);
    hw_flow    hw(t, 6, true, 40);
    sw_flow    sw(t, 6, true);
    const auto llr0 = t.llrs(rng, 0, 1.0f, 0.3f);
    CHECK(hw.transmission(*acc, t, llr0, 0, true), "clean first transmission decodes");
    (void)sw.transmission(t, llr0, 0, true);
    /* the TB passed, so hw_flow freed the entry; a retransmission of the same CB now */
    const auto llr1 = t.llrs(rng, 0, 1.0f, 0.3f);
    hw.crc_ok.assign(t.C, 0);
    const bool ok = hw.transmission(*acc, t, llr1, 0, false);
    if (debug == 0) {
      CHECK(!ok && hw.iters[0] == 6, "retransmission of a freed entry is dropped (CRC fail, max iterations)");
    } else {
      sw.crc_ok.assign(t.C, 0);
      const bool ok_sw = sw.transmission(t, llr1, 0, false);
      CHECK(ok == ok_sw && hw.msgs == sw.msgs && hw.iters == sw.iters,
            "debug mode: the kept entry combines like the oracle flow");
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
    hal::hw_accelerator_pdsch_enc_configuration acfg; /* pdsch_encoder_test.cpp:176-182 with acc_type "mi355x" */
    acfg.acc_type        = "mi355x";
    acfg.cb_mode         = cb_mode;
    acfg.max_tb_size     = 0;
    acfg.dedicated_queue = !cb_mode; /* both queue modes */
    auto enc             = hal::create_hw_accelerator_pdsch_enc_factory(acfg)->create();
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
  test_decoder_auto(rng);
  test_decoder_auto_split(rng);
  test_dematcher(rng);
  CHECK(hal::hip_device_of_acc_type("mi355x") == 0 && hal::hip_device_of_acc_type("mi355x:2") == 2 &&
            hal::hip_device_of_acc_type("acc100") == -1 && hal::hip_device_of_acc_type("mi355x:") == -1,
        "hip_device_of_acc_type");
  {
    hal::hw_accelerator_pusch_dec_configuration other;
    other.acc_type = "acc100";
    CHECK(hal::create_hw_accelerator_pusch_dec_factory(other) == nullptr, "acc_type acc100 is not this plugin's");
  }
  /* "auto" reaches the GPU decoder (a gfx950 is visible when this test runs), the dematcher stays on the CPU */
  CHECK(create_ldpc_decoder_factory_sw("auto") != nullptr, "decoder type auto resolves to the GPU");
  CHECK(create_ldpc_rate_dematcher_factory_sw("auto") == nullptr, "dematcher type auto stays on the CPU");
  CHECK(create_ldpc_rate_dematcher_factory_sw("hip") != nullptr, "dematcher type hip");
  test_hal_vectortest_setup(rng);
  test_hal_drop_and_debug_mode(rng);
  test_demodulator(rng);
  test_pdsch_encoder(rng);
  std::printf("%s: %d failure(s)\n", failures == 0 ? "PASS" : "FAIL", failures);
  return failures == 0 ? 0 : 1;
}
