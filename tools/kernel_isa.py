#!/usr/bin/env python3
"""Diagnostic (not product): instruction mix of one kernel in a device assembly file (hipcc --cuda-device-only -S).

usage: python tools/kernel_isa.py FILE.s KERNEL_SUBSTRING [--top N]

Prints the kernel's instruction count by class (VALU full / half rate per tools/ubench/README.md, packed, LDS incl.
ds_bpermute, SALU, branches, AGPR moves, scratch) and the most frequent opcodes."""
import collections
import re
import sys

HALF = re.compile(r"^v_(pk_|perm|med3|min3|max3|add3|lshl_add|lshl_or|and_or|bfe|bfi|mad_|cvt_|cmp|cndmask_b32_e64|"
                  r"min_i32|max_i32|min_u32|max_u32|lshlrev_b32|mul_u32_u24|mul_i32_i24|readlane|writelane|"
                  r"readfirstlane)")


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(key) or (key in l and l.rstrip().endswith(":")
                                                                         and not l.startswith((".", "\t"))))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    ops = collections.Counter()
    for l in lines[start + 1:end]:
        t = l.strip()
        if not t or t.startswith((".", ";", "/")) or t.endswith(":"):
            continue
        ops[t.split()[0]] += 1
    cls = collections.Counter()
    for op, n in ops.items():
        if op.startswith("v_accvgpr"):
            c = "agpr move"
        elif op.startswith("v_"):
            c = "valu half" if HALF.match(op) or op.endswith("_e64") or "sdwa" in op or "dpp" in op else "valu full"
        elif op.startswith("ds_"):
            c = "lds"
        elif op.startswith(("scratch_", "buffer_")):
            c = "scratch/buffer"
        elif op.startswith(("global_", "flat_")):
            c = "global"
        elif op.startswith(("s_cbranch", "s_branch")):
            c = "branch"
        elif op.startswith("s_"):
            c = "salu/ctl"
        else:
            c = "other"
        cls[c] += n
    print(f"{lines[start].split(':')[0][:90]}: {sum(ops.values())} instructions")
    for c, n in cls.most_common():
        print(f"  {c:16s} {n}")
    for op, n in ops.most_common(top):
        print(f"  {n:6d} {op}")


if __name__ == "__main__":
    main()
