#!/usr/bin/env python3
"""Inter-kernel gaps of the fit loop from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -- python3 bench.py --config c3 ...
    python tools/kernel_gaps.py gpurun_out/kt/**/kernel_trace.csv [--match tr::]

For every pair of consecutive dispatches on the same queue whose names both contain --match (the
library's kernels), prints the mean kernel duration per name and the mean idle time between the
end of one kernel and the start of the next, per (previous, next) pair.  Idle time is what the
step pays above the sum of its kernels (dispatch, end-of-kernel cache release, event packets).
"""
import argparse
import csv
import glob
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match", default="tr::")
    args = ap.parse_args()
    rows = []
    for pat in args.paths:
        for p in glob.glob(pat, recursive=True):
            with open(p) as f:
                rows += list(csv.DictReader(f))
    if not rows:
        raise SystemExit("no kernel trace rows")
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else None
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                  r.get(qkey, "0") if qkey else "0") for r in rows))
    dur = defaultdict(list)
    gaps = defaultdict(list)
    last = {}
    for s, e, n, q in ev:
        n = short(n)
        if args.match not in n:
            last.pop(q, None)
            continue
        dur[n].append(e - s)
        if q in last:
            pe, pn = last[q]
            gaps[(pn, n)].append(s - pe)
        last[q] = (e, n)
    print("kernel durations (us): name, count, mean")
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:60s} {len(v):6d} {sum(v) / len(v) / 1e3:10.2f}")
    print("gaps end -> start (us): prev -> next, count, mean, median")
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        print(f"  {a:40s} -> {b:40s} {len(v):6d} {sum(v) / len(v) / 1e3:8.2f} {v[len(v) // 2] / 1e3:8.2f}")


if __name__ == "__main__":
    main()
