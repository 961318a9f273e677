#!/usr/bin/env python3
"""One character per instruction of a kernel's largest loop (M mfma, r ds_read, w ds_write,
D LDS-DMA / buffer load, | s_waitcnt, B barrier, s other scalar, . vector ALU), one line per
basic block: shows at a glance whether VALU work sits between the MFMAs or in blocks.

    python tools/isa_stream.py /tmp/f.s <function-name substring>
"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_scratch import functions  # noqa: E402


def main():
    text = open(sys.argv[1]).read()
    for name, lines in functions(text):
        if sys.argv[2] not in name:
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
        out = []
        for ln in lines[a:b + 1]:
            t = ln.strip()
            if t.startswith(".LBB"):
                out.append("\n" + t.split(":")[0] + ": ")
                continue
            if not t or t.startswith((";", ".")):
                continue
            op = t.split()[0]
            if op.startswith("v_mfma"):
                c = "M"
            elif op.startswith("ds_read"):
                c = "r"
            elif op.startswith("ds_write"):
                c = "w"
            elif op.startswith(("buffer_load", "global_load_lds")):
                c = "D"
            elif op.startswith("s_waitcnt"):
                c = "|"
            elif op.startswith("s_barrier"):
                c = "B"
            elif op.startswith("s_"):
                c = "s"
            elif op.startswith("v_"):
                c = "."
            else:
                c = "?"
            out.append(c)
        print(name[:60])
        print("".join(out))


if __name__ == "__main__":
    main()
