/*
 * Benchmark of the HAL route (the plugin surfaces a srsRAN build drives), host buffers in and out, PCIe included:
 *
 *  PUSCH: hw_accelerator_pusch_dec_hip driven per TB in pusch_decoder_hw_impl's order with external HARQ
 *         (pusch_decoder_hw_impl.cpp:132-342): reserve -> configure + enqueue every CB -> dequeue (spin) +
 *         read_operation_outputs per CB -> free -> free_harq_context_entry; timed per TB like
 *         tests/benchmarks/phy/upper/channel_processors/pusch/pusch_decoder_hwacc_benchmark.cpp:383-502.
 *  PDSCH: hw_accelerator_pdsch_enc_hip in pdsch_encoder_hw_impl's order (pdsch_encoder_hw_impl.cpp:31-170), TB mode
 *         and CB mode, like tests/benchmarks/phy/upper/channel_processors/pdsch_encoder_hwacc_benchmark.cpp.
 *
 *  PUSCH, concurrent: T worker threads, each with its own hw_accelerator_pusch_dec_hip from ONE factory (so one
 *         shared external HARQ repository), take the slot's TBs from a shared counter (largest TB first) -- the shape
 *         of pusch_processor_benchmark.cpp:434-466 driving the accelerator from nof_threads lcores; slot time from the
 *         release of the workers to the last TB's free, p50/p99 for T = 1, 4, 8.
 *
 * Input (written by bench.py from device-generated slot LLRs): a little-endian binary file of
 *   u32 nof_tbs; per TB: u32 tbs, bg, Z, F, C, Qm, rv, iters; per CB: u32 E, then E int8 LLRs.
 * Output: one JSON object on stdout. Links the product libraries only.
 */
#include "ldpc_hip_adapters.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

using namespace srsran;
using clk = std::chrono::steady_clock;

namespace {

struct tb_in {
  unsigned                         tbs, bg, Z, F, C, Qm, rv, iters;
  std::vector<std::vector<int8_t>> llr;
};

double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

double pct(std::vector<double> v, double p)
{
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, static_cast<size_t>(p * static_cast<double>(v.size() - 1) + 0.5))];
}

/* the configuration pusch_decoder_hwacc_benchmark.cpp:233-243 builds for acc100, with acc_type "mi355x:<device>":
 * one repository of nof_cbs entries shared by every accelerator of the factory, soft bits in the GPU's HARQ memory */
hal::hw_accelerator_pusch_dec_configuration pusch_dec_config(int device, unsigned nof_cbs, bool dedicated_queue = true)
{
  hal::hw_accelerator_pusch_dec_configuration c;
  c.acc_type            = "mi355x:" + std::to_string(device);
  c.ext_softbuffer      = true;
  c.harq_buffer_context = hal::create_ext_harq_buffer_context_repository(nof_cbs, nof_cbs * hal::HARQ_INCR_BYTES, false);
  c.dedicated_queue     = dedicated_queue;
  return c;
}

modulation_scheme mod_of(unsigned qm)
{
  return qm == 1 ? modulation_scheme::BPSK : static_cast<modulation_scheme>(qm);
}

/* one TB through the PUSCH decoder plugin; returns the number of CBs whose CRC passed. ph (optional): the host time
 * of the TB's phases, us: [0] reserve + configure + enqueue of every CB, [1] the first dequeue (batch launch and wait),
 * [2] the remaining dequeues, output reads, free_queue and the HARQ entry frees */
unsigned decode_tb(hal::hw_accelerator_pusch_dec& acc, const tb_in& t, unsigned abs_base,
                   std::vector<std::vector<uint8_t>>& msgs, double* ph = nullptr)
{
  const auto tp0 = clk::now();
  auto       tp1 = tp0, tp2 = tp0;
  const unsigned K = t.bg == 1 ? 22 : 10;
  hal::hw_pusch_decoder_configuration c{};
  c.base_graph_index        = static_cast<ldpc_base_graph_type>(t.bg);
  c.modulation              = mod_of(t.Qm);
  c.nof_segments            = t.C;
  c.rv                      = t.rv;
  c.lifting_size            = t.Z;
  c.Ncb                     = (t.bg == 1 ? 66 : 50) * t.Z;
  c.Nref                    = 0;
  c.nof_filler_bits         = t.F;
  c.nof_segment_bits        = K * t.Z - t.F - (t.C > 1 ? 24 : 0);
  c.max_nof_ldpc_iterations = t.iters;
  c.use_early_stop          = true;
  c.new_data                = true;
  c.cb_crc_len              = t.C > 1 ? 24 : (t.tbs > 3824 ? 24 : 16);
  c.cb_crc_type = t.C > 1 ? hal::hw_dec_cb_crc_type::CRC24B
                          : (t.tbs > 3824 ? hal::hw_dec_cb_crc_type::CRC24A : hal::hw_dec_cb_crc_type::CRC16);
  acc.reserve_queue();
  unsigned next_enq = 0, next_deq = 0, ok = 0;
  while (next_deq != t.C) {
    for (; next_enq != t.C; ++next_enq) {
      c.cw_length      = static_cast<unsigned>(t.llr[next_enq].size());
      c.absolute_cb_id = abs_base + next_enq;
      acc.configure_operation(c, next_enq);
      if (!acc.enqueue_operation(span<const int8_t>(t.llr[next_enq].data(), t.llr[next_enq].size()), {}, next_enq)) {
        break;
      }
    }
    if (next_deq == 0) {
      tp1 = clk::now();
    }
    for (; next_deq != next_enq; ++next_deq) {
      while (!acc.dequeue_operation(span<uint8_t>(msgs[next_deq].data(), msgs[next_deq].size()), {}, next_deq)) {
      }
      if (next_deq == 0) {
        tp2 = clk::now();
      }
      hal::hw_pusch_decoder_outputs o{};
      acc.read_operation_outputs(o, next_deq, abs_base + next_deq);
      ok += o.CRC_pass ? 1 : 0;
    }
  }
  acc.free_queue();
  for (unsigned r = 0; r != t.C; ++r) {
    acc.free_harq_context_entry(abs_base + r);
  }
  if (ph != nullptr) {
    using us = std::chrono::duration<double, std::micro>;
    ph[0]    = us(tp1 - tp0).count();
    ph[1]    = us(tp2 - tp1).count();
    ph[2]    = us(clk::now() - tp2).count();
  }
  return ok;
}

/* one TB through the PDSCH encoder plugin */
void encode_tb(hal::hw_accelerator_pdsch_enc& enc, const tb_in& t, const std::vector<uint8_t>& tb,
               const std::vector<std::vector<uint8_t>>& cb_data, std::vector<uint8_t>& cw, std::vector<uint8_t>& packed)
{
  const unsigned K = t.bg == 1 ? 22 : 10, L = t.tbs > 3824 ? 24 : 16;
  hal::hw_pdsch_encoder_configuration c{};
  c.nof_tb_bits        = t.tbs;
  c.nof_tb_crc_bits    = L;
  c.base_graph_index   = static_cast<ldpc_base_graph_type>(t.bg);
  c.modulation         = mod_of(t.Qm);
  c.nof_segments       = t.C;
  c.nof_short_segments = t.C;
  c.rv                 = t.rv;
  c.cw_length_a        = static_cast<unsigned>(t.llr[0].size());
  c.cw_length_b        = static_cast<unsigned>(t.llr[t.C - 1].size());
  for (unsigned r = 0; r != t.C; ++r) {
    if (t.llr[r].size() != t.llr[0].size()) {
      c.nof_short_segments = r;
      break;
    }
  }
  c.lifting_size     = t.Z;
  c.Ncb              = (t.bg == 1 ? 66 : 50) * t.Z;
  c.nof_segment_bits = K * t.Z - t.F - (t.C > 1 ? 24 : 0);
  c.nof_filler_bits  = t.F;
  c.tb_crc           = L == 24 ? std::vector<uint8_t>{1, 2, 3} : std::vector<uint8_t>{1, 2};
  c.cb_mode          = enc.get_cb_mode();
  enc.reserve_queue();
  if (!c.cb_mode) {
    enc.configure_operation(c, 0);
    enc.enqueue_operation(span<const uint8_t>(tb.data(), tb.size()), {}, 0);
    while (!enc.dequeue_operation(span<uint8_t>(cw.data(), cw.size()), span<uint8_t>(packed.data(), packed.size()),
                                  0)) {
    }
  } else {
    for (unsigned r = 0; r != t.C; ++r) {
      c.rm_length = static_cast<unsigned>(t.llr[r].size());
      enc.configure_operation(c, r);
      enc.enqueue_operation(span<const uint8_t>(cb_data[r].data(), cb_data[r].size()), {}, r);
    }
    size_t off = 0, poff = 0;
    for (unsigned r = 0; r != t.C; ++r) {
      const size_t E = t.llr[r].size();
      while (!enc.dequeue_operation(span<uint8_t>(cw.data() + off, E), span<uint8_t>(packed.data() + poff, (E + 7) / 8),
                                    r)) {
      }
      off += E;
      poff += (E + 7) / 8;
    }
  }
  enc.free_queue();
}

/* The slot's TBs decoded by T threads, each with its own accelerator from one factory (one shared HARQ repository).
 * Returns the per-slot times; ok_cbs: CBs whose CRC passed in the last slot. */
std::vector<double> decode_slot_concurrent(const std::vector<tb_in>& tbs, unsigned T, int reps, int device,
                                           unsigned& ok_cbs, std::vector<double>* tb0_start_end = nullptr)
{
  const unsigned ntb = static_cast<unsigned>(tbs.size());
  std::vector<unsigned> abs_base(ntb, 0);
  for (unsigned i = 1; i != ntb; ++i) {
    abs_base[i] = abs_base[i - 1] + tbs[i - 1].C;
  }
  auto factory = hal::create_hw_accelerator_pusch_dec_factory(pusch_dec_config(device, abs_base.back() + tbs.back().C));
  std::vector<std::unique_ptr<hal::hw_accelerator_pusch_dec>> accs;
  for (unsigned w = 0; w != T; ++w) {
    accs.push_back(factory->create());
  }
  std::vector<std::vector<std::vector<uint8_t>>> msgs(ntb);
  for (unsigned i = 0; i != ntb; ++i) {
    msgs[i].assign(tbs[i].C, std::vector<uint8_t>(((tbs[i].bg == 1 ? 22 : 10) * tbs[i].Z + 7) / 8));
  }
  /* each accelerator decodes the largest TB once before timing: its pinned staging and device buffers grow to size
   * on first use (hipHostMalloc / hipMalloc take milliseconds), which a deployment pays once per decoder */
  for (unsigned w = 0; w != T; ++w) {
    decode_tb(*accs[w], tbs[0], abs_base[0], msgs[0]);
  }
  std::atomic<int>      gen{0};
  std::atomic<unsigned> next{0}, done{0}, ok{0};
  clk::time_point       slot_t0{}, tb0_t0{}, tb0_t1{}; /* TB 0 (the largest): when its worker took and finished it */
  std::atomic<bool>     quit{false};
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
        for (unsigned i; (i = next.fetch_add(1, std::memory_order_acq_rel)) < ntb;) {
          const clk::time_point ts = clk::now();
          ok.fetch_add(decode_tb(*accs[w], tbs[i], abs_base[i], msgs[i]), std::memory_order_relaxed);
          if (i == 0) {
            tb0_t0 = ts;
            tb0_t1 = clk::now();
          }
          done.fetch_add(1, std::memory_order_acq_rel);
        }
      }
    });
  }
  std::vector<double> slot_us;
  for (int rep = -2; rep != reps; ++rep) {
    next.store(0);
    done.store(0);
    ok.store(0);
    const auto t0 = clk::now();
    slot_t0       = t0;
    gen.fetch_add(1, std::memory_order_acq_rel);
    while (done.load(std::memory_order_acquire) != ntb) {
    }
    if (rep >= 0) {
      slot_us.push_back(us_since(t0));
      if (tb0_start_end != nullptr) {
        using us = std::chrono::duration<double, std::micro>;
        tb0_start_end->push_back(us(tb0_t0 - slot_t0).count());
        tb0_start_end->push_back(us(tb0_t1 - slot_t0).count());
      }
    }
  }
  quit.store(true, std::memory_order_release);
  for (std::thread& t : workers) {
    t.join();
  }
  ok_cbs = ok.load();
  return slot_us;
}

} // namespace

int main(int argc, char** argv)
{
  if (argc < 2) {
    std::fprintf(stderr, "usage: bench_hal <slot.bin> [reps] [device]\n");
    return 2;
  }
  const int reps   = argc > 2 ? std::atoi(argv[2]) : 20;
  const int device = argc > 3 ? std::atoi(argv[3]) : 0;
  FILE*     f      = std::fopen(argv[1], "rb");
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
  std::vector<tb_in> tbs(ntb);
  uint64_t           payload = 0, llr_bytes = 0;
  for (tb_in& t : tbs) {
    unsigned h[8];
    rd(h, sizeof(h));
    t = tb_in{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], {}};
    t.llr.resize(t.C);
    for (auto& v : t.llr) {
      unsigned E = 0;
      rd(&E, 4);
      v.resize(E);
      rd(v.data(), E);
      llr_bytes += E;
    }
    payload += t.tbs;
  }
  std::fclose(f);

  /* PUSCH decoder plugin */
  unsigned nof_cbs_slot = 0;
  for (const tb_in& t : tbs) {
    nof_cbs_slot += t.C;
  }
  auto acc = hal::create_hw_accelerator_pusch_dec_factory(pusch_dec_config(device, nof_cbs_slot))->create();
  std::vector<std::vector<std::vector<uint8_t>>> msgs(ntb);
  for (unsigned i = 0; i != ntb; ++i) {
    msgs[i].assign(tbs[i].C, std::vector<uint8_t>(((tbs[i].bg == 1 ? 22 : 10) * tbs[i].Z + 7) / 8));
  }
  std::vector<double> slot_us, tb0_us, ph_tb0[3], ph_small[3];
  unsigned            ok_cbs = 0, cbs = 0;
  for (int rep = -2; rep != reps; ++rep) {
    const auto t0 = clk::now();
    unsigned   ok = 0, base = 0;
    for (unsigned i = 0; i != ntb; ++i) {
      const auto ti = clk::now();
      double     ph[3];
      ok += decode_tb(*acc, tbs[i], base, msgs[i], ph);
      if (i == 0 && rep >= 0) {
        tb0_us.push_back(us_since(ti));
      }
      for (int k = 0; rep >= 0 && k != 3; ++k) {
        (tbs[i].C > 1 ? ph_tb0 : ph_small)[k].push_back(ph[k]);
      }
      base += tbs[i].C;
    }
    if (rep >= 0) {
      slot_us.push_back(us_since(t0));
      ok_cbs = ok;
      cbs    = base;
    }
  }

  /* the same slot from T concurrent accelerators sharing one HARQ repository */
  const unsigned      conc_t[3] = {1, 4, 8};
  std::vector<double> conc_p50(3), conc_p99(3), conc_tb0_start(3), conc_tb0_end(3);
  unsigned            conc_ok[3] = {0, 0, 0};
  for (int k = 0; k != 3; ++k) {
    std::vector<double> se;
    std::vector<double> v = decode_slot_concurrent(tbs, conc_t[k], reps, device, conc_ok[k], &se);
    conc_p50[k]           = pct(v, 0.5);
    conc_p99[k]           = pct(v, 0.99);
    std::vector<double> st, en;
    for (size_t j = 0; j + 1 < se.size(); j += 2) {
      st.push_back(se[j]);
      en.push_back(se[j + 1]);
    }
    conc_tb0_start[k] = pct(st, 0.5);
    conc_tb0_end[k]   = pct(en, 0.5);
  }

  /* PDSCH encoder plugin: the same TBs, TB mode and CB mode */
  std::mt19937 rng(5);
  std::vector<std::vector<uint8_t>>              tb_bytes(ntb);
  std::vector<std::vector<std::vector<uint8_t>>> cb_bytes(ntb);
  std::vector<std::vector<uint8_t>>              cws(ntb), packs(ntb);
  for (unsigned i = 0; i != ntb; ++i) {
    const tb_in& t = tbs[i];
    tb_bytes[i].resize(t.tbs / 8);
    for (uint8_t& b : tb_bytes[i]) {
      b = static_cast<uint8_t>(rng());
    }
    const unsigned kb = ((t.bg == 1 ? 22 : 10) * t.Z - t.F + 7) / 8;
    cb_bytes[i].assign(t.C, std::vector<uint8_t>(kb));
    size_t total = 0, ptotal = 0;
    for (unsigned r = 0; r != t.C; ++r) {
      for (uint8_t& b : cb_bytes[i][r]) {
        b = static_cast<uint8_t>(rng());
      }
      total += t.llr[r].size();
      ptotal += (t.llr[r].size() + 7) / 8;
    }
    cws[i].resize(total);
    packs[i].resize(ptotal + 8);
  }
  double enc_p50[2] = {0, 0}, enc_tb0_p50[2] = {0, 0};
  for (int mode = 0; mode != 2; ++mode) {
    hal::hw_accelerator_pdsch_enc_configuration ecfg;
    ecfg.acc_type        = "mi355x:" + std::to_string(device);
    ecfg.cb_mode         = mode == 1;
    ecfg.max_tb_size     = 0;
    ecfg.dedicated_queue = true;
    auto                enc = hal::create_hw_accelerator_pdsch_enc_factory(ecfg)->create();
    std::vector<double> s_us, t0_us;
    for (int rep = -2; rep != reps; ++rep) {
      const auto t0 = clk::now();
      for (unsigned i = 0; i != ntb; ++i) {
        const auto ti = clk::now();
        encode_tb(*enc, tbs[i], tb_bytes[i], cb_bytes[i], cws[i], packs[i]);
        if (i == 0 && rep >= 0) {
          t0_us.push_back(us_since(ti));
        }
      }
      if (rep >= 0) {
        s_us.push_back(us_since(t0));
      }
    }
    enc_p50[mode]     = pct(s_us, 0.5);
    enc_tb0_p50[mode] = pct(t0_us, 0.5);
  }

  const double s50 = pct(slot_us, 0.5);
  std::printf("{\"pusch_dec\": {\"slot_us_p50\": %.1f, \"slot_us_p99\": %.1f, \"tb0_us_p50\": %.1f, \"tb0_us_p99\": "
              "%.1f, \"tb_payload_gbit_per_s_pcie\": %.4f, \"llr_gbyte_per_s_h2d\": %.4f, \"cbs\": %u, "
              "\"cbs_crc_ok\": %u, \"tbs\": %u, \"reps\": %d}, ",
              s50, pct(slot_us, 0.99), pct(tb0_us, 0.5), pct(tb0_us, 0.99), static_cast<double>(payload) / s50 / 1e3,
              static_cast<double>(llr_bytes) / s50 / 1e3, cbs, ok_cbs, ntb, reps);
  std::printf("\"pusch_dec_phases_us_p50\": {\"multi_cb_tb\": [%.1f, %.1f, %.1f], \"one_cb_tb\": [%.1f, %.1f, %.1f], "
              "\"order\": \"reserve+configure+enqueue, first dequeue, rest\"}, ",
              pct(ph_tb0[0], 0.5), pct(ph_tb0[1], 0.5), pct(ph_tb0[2], 0.5), pct(ph_small[0], 0.5),
              pct(ph_small[1], 0.5), pct(ph_small[2], 0.5));
  std::printf("\"pusch_dec_concurrent\": {");
  for (int k = 0; k != 3; ++k) {
    std::printf("%s\"T%u\": {\"slot_us_p50\": %.1f, \"slot_us_p99\": %.1f, \"tb_payload_gbit_per_s_pcie\": %.4f, "
                "\"cbs_crc_ok\": %u, \"tb0_start_end_us_p50\": [%.1f, %.1f]}",
                k ? ", " : "", conc_t[k], conc_p50[k], conc_p99[k], static_cast<double>(payload) / conc_p50[k] / 1e3,
                conc_ok[k], conc_tb0_start[k], conc_tb0_end[k]);
  }
  std::printf("}, ");
  std::printf("\"pdsch_enc\": {\"tb_mode_slot_us_p50\": %.1f, \"tb_mode_tb0_us_p50\": %.1f, \"cb_mode_slot_us_p50\": "
              "%.1f, \"cb_mode_tb0_us_p50\": %.1f, \"tb_mode_payload_gbit_per_s_pcie\": %.4f}}\n",
              enc_p50[0], enc_tb0_p50[0], enc_p50[1], enc_tb0_p50[1], static_cast<double>(payload) / enc_p50[0] / 1e3);
  return 0;
}
