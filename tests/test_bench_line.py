"""CPU tests of bench.py's output contract: the headline line the driver parses carries the contract's keys and stays
under 8 KB; the extras go to a file plus a digest line (round 5's 21.5 KB line with every extra inline was not parsed,
VERDICT r5 item 1); the "auto" software-route figures are labelled by which decoder produced them."""
import json
from pathlib import Path

import bench

ROOT = Path(__file__).resolve().parents[1]


def _stub_cpu():
    one = {"threads": 1, "codeblocks": 10000, "wall_s": 0.87, "gbit_per_s": 0.0974, "info_mbit_per_s_per_thread": 97.5,
           "p50_us": 86.6, "p99_us": 87.5}
    allc = dict(one, threads=16, codeblocks=160000, gbit_per_s=1.42)
    return {"value": 1.42, "unit": "Gbit/s", "cores": 16, "kind": "port", "sample": "x" * 300,
            "cpu_model": "AMD EPYC 9575F 64-Core Processor", "affinity_cores": 256, "cgroup_cpu_quota_cores": 16,
            "job_cpu_share": 16, "single_core": one, "single_core_awgn_codeword": dict(one, p50_us=95.2),
            "all_cores": allc, "p50_us": 86.6, "p99_us": 87.5}


def _stub_secondary():
    return {"bound": "valu", "achieved": 1.0e12, "peak": 1.2e12, "unit": "VALU-busy SIMD cycles/s", "frac": 0.72,
            "issue_frac": 0.4, "cus": 128, "valu_insts_per_launch": 29700000, "valu_active_cycles_per_launch": 1.2e8,
            "lds_insts_per_launch": 4000000, "source": "profiles/pmc_traffic.json " + "y" * 80}


def _headline(world=1, devices=None):
    prov = {"file": "profiles/pmc_traffic.json", "round": 6, "same_build": True, "csrc_sha256": "a" * 64,
            "rocprof_avg_kernel_ns": 134930.0}
    return bench.headline_line(gbps=8.11, world=world, steps=20, warmup=5, elapsed=20 * 1.333e-4, kernel_ms=0.1327,
                               n=128, total_cbs=world * 128 * 20, traffic=4345716, prov=prov,
                               secondary=_stub_secondary(), cpu_base=_stub_cpu() if world == 1 else None,
                               devices=devices, devices_distinct=True if devices else None)


def test_headline_has_contract_keys_and_is_small():
    line = _headline()
    for k in bench.HEADLINE_KEYS:
        assert k in line, k
    assert "extra" not in line
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"]
    assert line["n_gpus"] == 1 and line["steps"] == 20 and line["warmup"] == 5
    assert abs(line["roofline"]["frac"] - line["roofline"]["achieved"] / line["roofline"]["peak"]) < 1e-5
    assert len(json.dumps(line).encode()) < bench.HEADLINE_MAX_BYTES


def test_headline_with_eight_devices_is_small():
    devs = [{"host": "node0", "device": i, "pci": f"0000:{0x11 + i:02x}:00", "uuid": "GPU-" + "f" * 32,
             "name": "AMD Instinct MI355X", "rank": i} for i in range(8)]
    line = _headline(world=8, devices=devs)
    assert line["config"]["devices_distinct"] is True and len(line["config"]["devices"]) == 8
    assert len(json.dumps(line).encode()) < bench.HEADLINE_MAX_BYTES


def test_extras_digest_of_round5_record_is_small():
    # the round-5 line (profiles/r05_bench_line.json) carried every extra inline; its digest must be a few KB
    rec = json.loads((ROOT / "profiles" / "r05_bench_line.json").read_text())
    extra = dict(rec["extra"])
    extra["sw_route"] = bench.label_auto_route(json.loads(json.dumps(extra["sw_route"])))
    s = bench.extras_summary(extra)
    txt = bench.EXTRAS_PREFIX + json.dumps({"bench_extras_summary": s, "full_record": "gpurun_out/bench_extras.json"})
    assert not txt.startswith("{")  # the contract's one JSON line is the headline
    assert len(txt.encode()) < 6144, len(txt)
    assert s["hal"]["pusch_dec"]["slot_us_p50"] == rec["extra"]["hal"]["pusch_dec"]["slot_us_p50"]
    assert s["c4"]["us_per_slot"] == rec["extra"]["c4"]["us_per_slot"]
    # round 5's auto pairing sent every call to the CPU port: the block is renamed to say so
    assert "auto_decoder_only" not in s["sw_route"]
    assert "auto_decoder_only_all_calls_on_cpu_port" in s["sw_route"]
    # together with the headline the whole stdout stays well under the size round 4's parsed line had
    assert len(txt.encode()) + len(json.dumps(_headline()).encode()) < 12288


def test_auto_route_with_gpu_calls_keeps_its_name():
    sw = {"auto_decoder_only": {"T1": {"slot_us_p50": 1.0}, "T1_calls": {"cpu": 10, "gpu": 3}}}
    out = bench.label_auto_route(sw)
    assert "auto_decoder_only" in out and "cpu_port" in out["auto_decoder_only"]["cpu_decoder"]
