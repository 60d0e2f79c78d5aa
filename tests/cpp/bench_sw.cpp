/*
 * Benchmark of the software-factory route -- the one the untouched upper PHY builds (upper_phy_factories.cpp:394-445
 * creates only create_pusch_decoder_factory_sw): pusch_decoder_impl forks one task per codeblock onto its executor
 * (pusch_decoder_impl.cpp:309-382) and each task runs pusch_codeblock_decoder::decode (pusch_codeblock_decoder.cpp:
 * 35-71) with the decoder pair of its thread (the concurrent_thread_local_object_pool of pusch_decoder_impl.h:48):
 * ldpc_rate_dematcher::rate_dematch into the codeblock's host soft buffer (rx_buffer), then
 * ldpc_decoder::decode(message, soft buffer, crc, {max_iterations, 0.8}) with CRC early stop.
 *
 * Here the pairs are ldpc_rate_dematcher_hip + ldpc_decoder_hip from the factories' "hip" type (one pair per thread),
 * T worker threads take the slot's codeblocks from a shared counter (largest TB first), host buffers in and out, so
 * every PCIe crossing and every per-call latency counts. Three pairings:
 *   gpu_pair      dematcher and decoder on the GPU ("hip" / "hip");
 *   decoder_only  the decoder on the GPU with each codeblock's soft buffer already dematched (the dematcher stays on
 *                 the CPU; its CPU time is not in these figures);
 *   auto_decoder_only  as decoder_only with the "auto" type's hybrid (ldpc_decoder_hip_auto): codeblocks below
 *                 ldpc_hip_auto_min_work() on a CPU decoder, the others on the GPU. Its CPU side is the oracle's AVX2
 *                 decoder port (oracle/ldpc_cpu_port.c), standing in for the reference's AVX2/AVX-512 decoders, which
 *                 cannot be built here; it is the only oracle code this program links (the GPU pairings are
 *                 product code only).
 * Reported per T: slot time (release of the workers to the last codeblock) p50 / p99 and per-call latencies.
 *
 * Input: bench_hal's slot file (u32 nof_tbs; per TB: u32 tbs, bg, Z, F, C, Qm, rv, iters; per CB: u32 E, E int8 LLRs).
 * Output: one JSON object on stdout. Links the product libraries only.
 */
#include "ldpc_hip_adapters.h"

extern "C" {
#include "ldpc_oracle.h"
}

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

using namespace srsran;
using clk = std::chrono::steady_clock;

namespace {

struct cb_in {
  unsigned            bg, Z, F, Qm, rv, iters, tbs, C;
  std::vector<int8_t> llr;
};

class crc_poly_only : public crc_calculator
{
public:
  explicit crc_poly_only(crc_generator_poly p) : poly(p) {}
  crc_generator_poly get_generator_poly() const override { return poly; }
  unsigned           calculate(const bit_buffer&) override { return 0; }

private:
  crc_generator_poly poly;
};

double us_between(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

double pct(std::vector<double> v, double p)
{
  if (v.empty()) {
    return 0;
  }
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, static_cast<size_t>(p * static_cast<double>(v.size() - 1) + 0.5))];
}

modulation_scheme mod_of(unsigned qm) { return qm == 1 ? modulation_scheme::BPSK : static_cast<modulation_scheme>(qm); }

codeblock_metadata meta_of(const cb_in& c)
{
  codeblock_metadata m;
  m.tb_common.base_graph        = static_cast<ldpc_base_graph_type>(c.bg);
  m.tb_common.lifting_size      = static_cast<ldpc::lifting_size_t>(c.Z);
  m.tb_common.rv                = c.rv;
  m.tb_common.mod               = mod_of(c.Qm);
  m.tb_common.Nref              = 0;
  m.cb_specific.rm_length       = static_cast<unsigned>(c.llr.size());
  m.cb_specific.nof_filler_bits = c.F;
  m.cb_specific.nof_crc_bits    = c.C > 1 ? 24 : (c.tbs > 3824 ? 24 : 16);
  return m;
}

crc_generator_poly crc_of(const cb_in& c)
{
  /* select_crc (pusch_decoder_impl.cpp:35-46) */
  return c.C > 1 ? crc_generator_poly::CRC24B : (c.tbs > 3824 ? crc_generator_poly::CRC24A : crc_generator_poly::CRC16);
}

struct result {
  std::vector<double>                        slot_us, dematch_us, decode_us;
  std::vector<std::pair<std::string, double>> decode_by_graph; /* ("BG<bg>Z<Z>", us) per call */
  unsigned                                   ok = 0;
  uint64_t                                   cpu_calls = 0, gpu_calls = 0;
};

/* The auto pairing's CPU side (see the header comment): the AVX2 decoder port behind the ldpc_decoder interface */
class ldpc_decoder_cpu_port : public ldpc_decoder
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
    const int r = orc_ldpc_decode_port(static_cast<int>(cfg.block_conf.tb_common.base_graph),
                                       static_cast<unsigned>(cfg.block_conf.tb_common.lifting_size),
                                       cfg.block_conf.cb_specific.nof_filler_bits,
                                       reinterpret_cast<const int8_t*>(input.data()),
                                       static_cast<unsigned>(input.size()), cfg.algorithm_conf.max_iterations, poly,
                                       output.get_buffer().data());
    return r > 0 ? std::optional<unsigned>(static_cast<unsigned>(r)) : std::nullopt;
  }
};
class ldpc_decoder_cpu_port_factory : public ldpc_decoder_factory
{
public:
  std::unique_ptr<ldpc_decoder> create() override { return std::make_unique<ldpc_decoder_cpu_port>(); }
};

/* The slot's codeblocks on T threads, each with its own decoder pair; with_dematch false: decode only, from soft
 * buffers dematched beforehand; hybrid: the decoders are the "auto" type's ldpc_decoder_hip_auto. */
result run(const std::vector<cb_in>& cbs, unsigned T, int reps, int device, bool with_dematch, bool hybrid = false)
{
  const std::string type = "hip:" + std::to_string(device);
  auto              dfac = hybrid ? create_ldpc_decoder_factory_hip_auto(device,
                                                                         std::make_shared<ldpc_decoder_cpu_port_factory>())
                                  : create_ldpc_decoder_factory_sw(type);
  auto              rfac = create_ldpc_rate_dematcher_factory_sw(type);
  struct pair {
    std::unique_ptr<ldpc_decoder>        dec;
    std::unique_ptr<ldpc_rate_dematcher> dm;
  };
  std::vector<pair> pairs;
  for (unsigned t = 0; t != T; ++t) {
    pairs.push_back({dfac->create(), rfac->create()});
  }
  const size_t                      n = cbs.size();
  std::vector<std::vector<int8_t>>  soft(n), soft0(n);
  std::vector<std::vector<uint8_t>> msg(n);
  std::vector<codeblock_metadata>   meta(n);
  for (size_t i = 0; i != n; ++i) {
    const cb_in& c = cbs[i];
    soft[i].assign((c.bg == 1 ? 66U : 50U) * c.Z, 0);
    msg[i].assign(((c.bg == 1 ? 22U : 10U) * c.Z + 7) / 8, 0);
    meta[i] = meta_of(c);
  }
  if (!with_dematch) { /* the soft buffers the CPU dematcher would hand over */
    for (size_t i = 0; i != n; ++i) {
      pairs[0].dm->rate_dematch(span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(soft[i].data()),
                                                           soft[i].size()),
                                span<const log_likelihood_ratio>(
                                    reinterpret_cast<const log_likelihood_ratio*>(cbs[i].llr.data()), cbs[i].llr.size()),
                                true, meta[i]);
      soft0[i] = soft[i];
    }
  }
  result                   res;
  std::vector<double>      dm_us(n), dec_us(n);
  std::atomic<int>         gen{0};
  std::atomic<size_t>      next{0}, done{0};
  std::atomic<unsigned>    ok{0};
  std::atomic<bool>        quit{false};
  std::vector<std::thread> workers;
  for (unsigned w = 0; w != T; ++w) {
    workers.emplace_back([&, w] {
      int seen = 0;
      while (true) {
        int g;
        while ((g = gen.load(std::memory_order_acquire)) == seen && !quit.load(std::memory_order_acquire)) {
        }
        if (quit.load(std::memory_order_acquire)) {
          return;
        }
        seen = g;
        for (size_t i; (i = next.fetch_add(1, std::memory_order_acq_rel)) < n;) {
          const cb_in& c  = cbs[i];
          auto         t0 = clk::now();
          if (with_dematch) {
            std::fill(soft[i].begin(), soft[i].end(), 0); /* a clean rx_buffer codeblock (new data) */
            pairs[w].dm->rate_dematch(
                span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(soft[i].data()), soft[i].size()),
                span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(c.llr.data()),
                                                 c.llr.size()),
                true, meta[i]);
          } else {
            std::copy(soft0[i].begin(), soft0[i].end(), soft[i].begin());
          }
          auto                        t1 = clk::now();
          ldpc_decoder::configuration cfg;
          cfg.block_conf                    = meta[i];
          cfg.algorithm_conf.max_iterations = c.iters;
          cfg.algorithm_conf.scaling_factor = 0.8f;
          crc_poly_only crc(crc_of(c));
          bit_buffer    bb(span<uint8_t>(msg[i].data(), msg[i].size()), (c.bg == 1 ? 22U : 10U) * c.Z);
          const auto    r = pairs[w].dec->decode(
              bb, span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(soft[i].data()),
                                                   soft[i].size()),
              &crc, cfg);
          auto t2 = clk::now();
          dm_us[i]  = us_between(t0, t1);
          dec_us[i] = us_between(t1, t2);
          ok.fetch_add(r.has_value() ? 1U : 0U, std::memory_order_relaxed);
          done.fetch_add(1, std::memory_order_acq_rel);
        }
      }
    });
  }
  for (int rep = -2; rep != reps; ++rep) {
    next.store(0);
    done.store(0);
    ok.store(0);
    const auto t0 = clk::now();
    gen.fetch_add(1, std::memory_order_acq_rel);
    while (done.load(std::memory_order_acquire) != n) {
    }
    const auto t1 = clk::now();
    if (rep >= 0) {
      res.slot_us.push_back(us_between(t0, t1));
      if (with_dematch) {
        res.dematch_us.insert(res.dematch_us.end(), dm_us.begin(), dm_us.end());
      }
      res.decode_us.insert(res.decode_us.end(), dec_us.begin(), dec_us.end());
      for (size_t i = 0; i != n; ++i) {
        res.decode_by_graph.emplace_back("BG" + std::to_string(cbs[i].bg) + "Z" + std::to_string(cbs[i].Z), dec_us[i]);
      }
    }
  }
  quit.store(true, std::memory_order_release);
  for (std::thread& t : workers) {
    t.join();
  }
  res.ok = ok.load();
  if (hybrid) {
    for (const pair& p : pairs) {
      const auto* h = static_cast<const ldpc_decoder_hip_auto*>(p.dec.get());
      res.cpu_calls += h->cpu_calls();
      res.gpu_calls += h->gpu_calls();
    }
  }
  return res;
}

} // namespace

int main(int argc, char** argv)
{
  if (argc < 2) {
    std::fprintf(stderr, "usage: bench_sw <slot.bin> [reps] [device] [threads,...]\n");
    return 2;
  }
  const int reps   = argc > 2 ? std::atoi(argv[2]) : 20;
  const int device = argc > 3 ? std::atoi(argv[3]) : 0;
  std::vector<unsigned> ts = {1, 4, 8, 16};
  if (argc > 4) {
    ts.clear();
    for (const char* p = argv[4]; *p != '\0';) {
      ts.push_back(static_cast<unsigned>(std::strtoul(p, const_cast<char**>(&p), 10)));
      if (*p == ',') {
        ++p;
      }
    }
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (f == nullptr) {
    return 2;
  }
  auto rd = [&](void* p, size_t n) {
    if (std::fread(p, 1, n, f) != n) {
      std::exit(3);
    }
  };
  unsigned ntb = 0;
  rd(&ntb, 4);
  std::vector<cb_in> cbs;
  uint64_t           payload = 0;
  for (unsigned t = 0; t != ntb; ++t) {
    unsigned h[8];
    rd(h, sizeof(h));
    payload += h[0];
    for (unsigned r = 0; r != h[4]; ++r) {
      cb_in c{h[1], h[2], h[3], h[5], h[6], h[7], h[0], h[4], {}};
      unsigned E = 0;
      rd(&E, 4);
      c.llr.resize(E);
      rd(c.llr.data(), E);
      cbs.push_back(std::move(c));
    }
  }
  std::fclose(f);

  std::printf("{\"cbs\": %zu, \"reps\": %d, \"auto_min_work\": %llu", cbs.size(), reps,
              static_cast<unsigned long long>(ldpc_hip_auto_min_work()));
  const char* names[3] = {"gpu_pair", "decoder_only", "auto_decoder_only"};
  for (int mode = 0; mode != 3; ++mode) {
    std::printf(", \"%s\": {", names[mode]);
    for (size_t k = 0; k != ts.size(); ++k) {
      const result r = run(cbs, ts[k], reps, device, mode == 0, mode == 2);
      const double s = pct(r.slot_us, 0.5);
      std::printf("%s\"T%u\": {\"slot_us_p50\": %.1f, \"slot_us_p99\": %.1f, \"tb_payload_gbit_per_s\": %.4f, "
                  "\"cb_decode_us_p50\": %.1f, \"cb_decode_us_p99\": %.1f, \"cb_dematch_us_p50\": %.1f, "
                  "\"cb_dematch_us_p99\": %.1f, \"cbs_crc_ok\": %u}",
                  k ? ", " : "", ts[k], s, pct(r.slot_us, 0.99), static_cast<double>(payload) / s / 1e3,
                  pct(r.decode_us, 0.5), pct(r.decode_us, 0.99), pct(r.dematch_us, 0.5), pct(r.dematch_us, 0.99),
                  r.ok);
      /* per graph: decode call p50 (the crossover calibration of the auto type) */
      std::vector<std::string> keys;
      for (const auto& kv : r.decode_by_graph) {
        if (std::find(keys.begin(), keys.end(), kv.first) == keys.end()) {
          keys.push_back(kv.first);
        }
      }
      std::printf(", \"T%u_decode_us_p50_by_graph\": {", ts[k]);
      for (size_t q = 0; q != keys.size(); ++q) {
        std::vector<double> v;
        for (const auto& kv : r.decode_by_graph) {
          if (kv.first == keys[q]) {
            v.push_back(kv.second);
          }
        }
        std::printf("%s\"%s\": %.1f", q ? ", " : "", keys[q].c_str(), pct(v, 0.5));
      }
      std::printf("}");
      if (mode == 2) {
        std::printf(", \"T%u_calls\": {\"cpu\": %llu, \"gpu\": %llu}", ts[k],
                    static_cast<unsigned long long>(r.cpu_calls), static_cast<unsigned long long>(r.gpu_calls));
      }
    }
    std::printf("}");
  }
  std::printf("}\n");
  return 0;
}
