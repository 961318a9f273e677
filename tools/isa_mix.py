#!/usr/bin/env python3
"""Instruction mix of the largest loop of a kernel in a hipcc -S listing (static counts per
loop trip, by class), to budget issue cycles without a GPU.

    python tools/isa_mix.py /tmp/f.s <function-name substring>
"""
import re
import sys
from collections import Counter

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_scratch import functions  # noqa: E402


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_read", "ds_load")):
        return "ds_read"
    if op.startswith(("ds_write", "ds_store")):
        return "ds_write"
    if op.startswith("ds_"):
        return "ds_other"
    if op.startswith(("global_load_lds", "buffer_load")) :
        return "vmem_load"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem_other"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith(("s_barrier",)):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("v_perm", "v_and", "v_sub", "v_add", "v_lshl", "v_or", "v_cndmask", "v_mov", "v_fma", "v_mul",
                      "v_pk", "v_cvt", "v_bfi", "v_lshr", "v_xor", "v_max", "v_min", "v_sqrt", "v_rcp", "v_cmp",
                      "v_readlane", "v_readfirstlane", "v_writelane", "v_permlane", "v_accvgpr", "v_exp", "v_log",
                      "v_bfe", "v_ashr", "v_mad", "v_dot", "v_div", "v_sin", "v_cos", "v_not", "v_swap", "v_nop")):
        return "valu"
    if op.startswith("v_"):
        return "valu_other"
    return "other"


def main():
    text = open(sys.argv[1]).read()
    pat = sys.argv[2]
    for name, lines in functions(text):
        if pat not in name:
            continue
        labels = {}
        for i, ln in enumerate(lines):
            m = re.match(r"^(\.LBB\w+):", ln)
            if m:
                labels[m.group(1)] = i
        loops = []
        for i, ln in enumerate(lines):
            m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in labels and labels[tgt] < i:
                    loops.append((labels[tgt], i))
        a, b = max(loops, key=lambda ab: ab[1] - ab[0])
        c = Counter()
        vo = Counter()
        for ln in lines[a:b + 1]:
            t = ln.strip()
            if not t or t.startswith((";", ".")):
                continue
            op = t.split()[0]
            k = klass(op)
            c[k] += 1
            if k in ("valu", "valu_other"):
                vo[op] += 1
        print(name[:70], f"loop lines {a}-{b}")
        for k, v in c.most_common():
            print(f"  {k:12s} {v}")
        print("  top VALU:", ", ".join(f"{o} {n}" for o, n in vo.most_common(14)))


if __name__ == "__main__":
    main()
