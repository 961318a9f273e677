#!/usr/bin/env python3
"""Where a kernel touches scratch: for each function of a hipcc -S listing whose name matches,
the scratch loads / stores and whether they sit inside a loop (between a label and a later
branch back to it).

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S file.hip -o /tmp/f.s
    python tools/isa_scratch.py /tmp/f.s k_spec_sliceILi2ELi1ELi1E
"""
import re
import sys


def functions(text):
    cur, lines = None, []
    for ln in text.split("\n"):
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            if cur:
                yield cur, lines
            cur, lines = m.group(1), []
        elif cur:
            if ln.startswith(".Lfunc_end"):
                yield cur, lines
                cur, lines = None, []
            else:
                lines.append(ln)


def main():
    text = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, lines in functions(text):
        if pat not in name:
            continue
        labels = {}
        for i, ln in enumerate(lines):
            m = re.match(r"^(\.LBB\w+):", ln)
            if m:
                labels[m.group(1)] = i
        loops = []  # (start, end) of every backward branch
        for i, ln in enumerate(lines):
            m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in labels and labels[tgt] < i:
                    loops.append((labels[tgt], i))
        sc = [i for i, ln in enumerate(lines) if "scratch_" in ln]
        inside = [i for i in sc if any(a <= i <= b for a, b in loops)]
        big = max(loops, key=lambda ab: ab[1] - ab[0]) if loops else None
        print(f"{name[:60]}: {len(lines)} lines, loops {len(loops)} (largest {big}), scratch ops {len(sc)}, "
              f"inside a loop {len(inside)}")
        for i in inside[:12]:
            print("   ", i, lines[i].strip())


if __name__ == "__main__":
    main()
