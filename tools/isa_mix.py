#!/usr/bin/env python3
"""Static instruction mix of the kernels in a gfx950 assembly file (hipcc --cuda-device-only -S).

  python3 tools/isa_mix.py build/fused.s [kernel-substring] [--top N]

Prints, per kernel, the instruction count by class (fp64 VALU, other VALU, LDS, VMEM, SMEM, SALU,
branch/wait) and the most frequent opcodes.  Static counts of straight-line code approximate the
per-wave dynamic counts of the fused kernels (no loops in their compute part)."""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_") and ("_f64" in op or op.endswith("_b64") and "mov" in op):
        return "valu_f64/64b"
    if op.startswith("v_cvt"):
        return "valu_cvt"
    if op.startswith("v_pk_"):
        return "valu_packed"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_cbranch", "s_branch", "s_nop", "s_endpgm",
                      "s_setprio", "s_sleep")):
        return "control"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    lines = open(path).read().split("\n")
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\S+):", lines[i])
        if not m or sub not in m.group(1):
            i += 1
            continue
        name = m.group(1)
        ops = collections.Counter()
        j = i + 1
        while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
            t = lines[j].strip()
            j += 1
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            ops[t.split()[0]] += 1
        cls = collections.Counter()
        for op, c in ops.items():
            cls[classify(op)] += c
        print(f"{name}  total {sum(ops.values())}")
        for k, v in sorted(cls.items(), key=lambda kv: -kv[1]):
            print(f"    {k:14s} {v}")
        for op, c in ops.most_common(top):
            print(f"        {op:32s} {c}")
        i = j


if __name__ == "__main__":
    main()
