"""GPU box: A/B of the host-memory routes under environment / library variants. The C4 slot blob
(bench.hal_slot_blob) goes through tests/cpp/build/bench_sw (decoder_only and gpu_pair) and bench_hal once per
configuration, the configurations alternating over ROUNDS rounds; prints one JSON object (per configuration and
round: slot p50 per T and the per-phase HAL times).

usage: python tools/route_ab.py ROUNDS NAME[:K=V[,K=V...]] ...
  a value LIB=<suffix> runs the library variant srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip_<suffix>.so (through
  LD_LIBRARY_PATH: the benches' RUNPATH gives way to it)"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def run(cmd, env):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    if r.returncode != 0:
        return {"error": r.stderr[-300:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    import torch
    import bench
    from srsran_projectvtlmo_amd import _lib
    rounds = int(sys.argv[1])
    cfgs = []
    for a in sys.argv[2:]:
        name, _, kv = a.partition(":")
        cfgs.append((name, dict(p.split("=", 1) for p in kv.split(",") if p)))
    ctx = _lib.Context(0)
    blob = bench.hal_slot_blob(ctx)
    ctx.close()
    torch.cuda.synchronize()
    tmp = Path(tempfile.mkdtemp())
    path = tmp / "slot.bin"
    path.write_bytes(blob)
    out = {name: [] for name, _ in cfgs}
    try:
        for rnd in range(rounds):
            for name, kv in cfgs:
                env = {**os.environ, **{k: v for k, v in kv.items() if k != "LIB"}}
                if "LIB" in kv:
                    d = tmp / name
                    d.mkdir(exist_ok=True)
                    shutil.copy(ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{kv['LIB']}.so",
                                d / "libsrsran_ldpc_hip.so")
                    env["LD_LIBRARY_PATH"] = f"{d}:{env.get('LD_LIBRARY_PATH', '')}"
                sw = run([str(ROOT / "tests/cpp/build/bench_sw"), str(path), "10", "0", "1,8"], env)
                hal = run([str(ROOT / "tests/cpp/build/bench_hal"), str(path), "10", "0"], env)
                r = {"round": rnd}
                if "error" in sw:
                    r["sw"] = sw
                else:
                    for m in ("decoder_only", "gpu_pair"):
                        r[m] = {t: (v["slot_us_p50"], v["cb_decode_us_p50"]) for t, v in sw[m].items()
                                if isinstance(v, dict) and "slot_us_p50" in v}
                if "error" in hal:
                    r["hal"] = hal
                else:
                    r["hal_slot"] = {t: v["slot_us_p50"] for t, v in hal["pusch_dec_concurrent"].items()}
                    r["hal_serial_slot"] = hal["pusch_dec"]["slot_us_p50"]
                    r["hal_phases"] = hal.get("pusch_dec_phases_us_p50")
                out[name].append(r)
                print(name, rnd, json.dumps(r), file=sys.stderr, flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
