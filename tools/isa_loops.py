"""Instruction mix of the loops of a kernel in hipcc's --save-temps assembly: for each backward
branch (a loop), counts of MFMA, transcendental, other VALU, LDS, vector-memory and scalar
instructions in the loop body.  Usage: python tools/isa_loops.py <file.s> <kernel-name-substring>"""
import re
import sys
from collections import Counter


def kernel_lines(path, name):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and name in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or
               re.match(r"^\.Lfunc_end", lines[i]))
    return lines[start:end]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_cvt_pk_bf16") or op.startswith("v_cvt"):
        return "cvt"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_mov"):
        return "vmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_"):
        return "ds_other"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, name)
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    total = Counter()
    for l in lines:
        t = l.strip().split()
        if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
            total[classify(t[0])] += 1
    print(f"{name}: whole kernel {dict(total)}")
    for i, l in enumerate(lines):
        m = re.match(r"^\s*s_cbranch_\w+\s+(\.LBB\w+)", l) or re.match(r"^\s*s_branch\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            body = lines[labels[m.group(1)]:i + 1]
            c = Counter()
            for b in body:
                t = b.strip().split()
                if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
                    c[classify(t[0])] += 1
            v = c["valu"] + c["trans"] + c["cvt"] + c["vmov"] + c["accmov"]
            print(f"  loop {m.group(1)} (lines {labels[m.group(1)]}-{i}): {dict(c)}; VALU/MFMA "
                  f"{v / max(c['mfma'], 1):.1f}")


if __name__ == "__main__":
    main()
