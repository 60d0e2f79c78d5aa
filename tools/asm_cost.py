#!/usr/bin/env python3
"""Diagnostic (not product): static issue-cost estimate of the specialised decoder's iteration body.

Compiles ldpc_hip_kernels.hip to gfx950 assembly (extra -D flags from argv), splits the SPEC kernel at s_barrier and
weights each instruction by its measured issue class (tools/ubench/README.md). Prints per-class counts and cycles for
the iteration (both roles of a two-row step are listed: a wave runs one of them)."""
import collections
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "srsran_projectvtlmo_amd" / "csrc"
FULL = re.compile(r"^v_(add|sub|subrev)_(u32|co_u32|u16|i16|f32|f16)|^v_(and|or|xor|not)_b32|^v_ashrrev_i(32|16)|"
                  r"^v_lshrrev_b(32|16)|^v_lshlrev_b16|^v_mov_b32|^v_(min|max)_(i16|u16|f16)|^v_mul_lo_u16|^v_fmac|"
                  r"^v_mul_f(16|32)")
QUARTER = re.compile(r"^v_(mad|fma)_(u16|i16|f16)|^v_swap")


def classify(ins, line):
    if ins.startswith("ds_read"):
        return "lds_rd"
    if ins.startswith("ds_"):
        return "lds_wr"
    if ins.startswith("s_"):
        return "salu"
    if not ins.startswith("v_"):
        return "other"
    if QUARTER.match(ins):
        return "quarter"
    if "_sdwa" in ins or "_dpp" in ins or ins.endswith("_e64") or ins.startswith("v_pk_"):
        return "half"
    if FULL.match(ins):
        return "full_lit" if re.search(r"0x[0-9a-f]{3,}", line) else "full"
    return "half"


COST = {"full": 2.1, "full_lit": 2.6, "half": 4.25, "quarter": 8.3}


def main():
    out = "/tmp/asm_cost.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{ROOT / 'include'}",
                    f"-I{CSRC}", "--cuda-device-only", "-S", "-o", out, str(CSRC / "ldpc_hip_kernels.hip")] + sys.argv[1:],
                   check=True, stderr=subprocess.DEVNULL)
    s = open(out).read()
    i = s.index("_ZN8ldpc_hip18ldpc_decode_kernelILb1ELi0EEE")
    i = s.index(":\n", i)
    j = s.index(".Lfunc_end", i)
    body = [l.strip() for l in s[i:j].split("\n")]
    body = [l for l in body if l and not l.startswith((";", ".")) and not l.endswith(":")]
    bars = [k for k, l in enumerate(body) if l.startswith("s_barrier")]
    # the iteration body: the last run of barriers of one unrolled iteration (32 steps for BG1 Z=384)
    seg = body[bars[0]:bars[-1] + 1]
    c = collections.Counter()
    for l in seg:
        ins = l.split()[0]
        c[classify(ins, l)] += 1
    cyc = sum(COST.get(k, 0) * v for k, v in c.items())
    print(" ".join(f"{k}={v}" for k, v in sorted(c.items())), f"valu_cycles~{cyc:.0f}", f"barriers={len(bars)}")
    ops = collections.Counter(l.split()[0] for l in seg)
    print(" ".join(f"{k}:{v}" for k, v in ops.most_common(40)))


if __name__ == "__main__":
    main()
