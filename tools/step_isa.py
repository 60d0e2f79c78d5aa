#!/usr/bin/env python3
"""Diagnostic (not product): per-step instruction histogram of the specialised BG1 Z=384 decoder's iteration
(ldpc_decode_kernel<true, 0>), from its gfx950 assembly. The kernel body is split at s_barrier; the full iteration
loop is the first run of 32 step segments after the prologue. Per step: the instructions of both roles (a wave runs
one of them; split steps have one role), split into full-rate VALU, packed (v_pk_*), SALU, LDS and other, with
the VALU cost estimate of tools/asm_cost.py (cycles per wave-instruction issue).

usage: python tools/step_isa.py [extra hipcc -D flags]"""
import collections
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import asm_cost  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "srsran_projectvtlmo_amd" / "csrc"
out = "/tmp/step_isa.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{ROOT / 'include'}",
                f"-I{CSRC}", "-mllvm", "-simplifycfg-sink-common=false", "--cuda-device-only", "-S", "-o", out,
                str(CSRC / "ldpc_hip_kernels.hip")] + sys.argv[1:], check=True, stderr=subprocess.DEVNULL)
src = open(out).read().split("\n")
pat = "_ZN8ldpc_hip18ldpc_decode_kernelILb1ELi0EEEv"
start = next(i for i, l in enumerate(src) if l.startswith(pat))
end = start
while not src[end].startswith(".Lfunc_end"):
    end += 1
lines = [l.strip() for l in src[start:end]]
lines = [l for l in lines if l and not l.startswith((".", ";")) and not l.endswith(":")]
bars = [i for i, l in enumerate(lines) if l.startswith("s_barrier")]
print(f"{len(lines)} instructions, {len(bars)} barriers in ldpc_decode_kernel<true, 0> (BG1 Z=384)")
print("step insts  valu  pk  salu  lds  other  valu_cycles~  (both roles of a step; step 0 also holds the once-per-CB setup before the loop: lanes, role masks, c2v zeroing)")
tot = collections.Counter()
segs = list(zip(bars, bars[1:]))
# the full iteration loop starts at the first step holding a split row's partner merge (v_permlane32_swap): step 0
first = next(k for k, (a, b) in enumerate(segs) if any(l.startswith("v_permlane32_swap") for l in lines[a + 1:b]))
for k, (a, b) in enumerate(segs[first:first + 32]):
    seg = lines[a + 1:b]
    c = collections.Counter()
    cyc = 0.0
    for l in seg:
        op = l.split()[0]
        cls = asm_cost.classify(op, l)
        cyc += asm_cost.COST.get(cls, 0)
        kind = ("lds" if op.startswith("ds_") else "salu" if op.startswith("s_") else "pk" if op.startswith("v_pk")
                else "valu" if op.startswith("v_") else "other")
        c[kind] += 1
    tot.update(c)
    print(f"{k:3d} {len(seg):6d} {c['valu']:5d} {c['pk']:3d} {c['salu']:5d} {c['lds']:4d} {c['other']:6d} {cyc:12.0f}")
print("total", dict(tot))
