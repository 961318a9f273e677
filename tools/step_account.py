#!/usr/bin/env python3
"""Where a benchmarked step's time goes: kernels, gaps between them and host time, for the timed
region of one bench.py run recorded under a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d <dir> -- python3 bench.py --steps K ... > b.json
    python tools/step_account.py --trace '<dir>/**/*kernel_trace.csv' --bench b.json --dominant k_linear_fused

The timed region holds the last K launches of the dominant kernel (bench.py's K steps come last;
nothing but the final reads follows them).  Its GPU window runs from the start of the first
kernel of the first timed iteration (the kernel launched right after the (K+1)-th-last dominant
kernel's iteration ended, i.e. the first launch after the previous iteration's last kernel) to the
end of the last kernel.  Per step: each kernel's mean duration, the idle GPU time between
kernels, and (with --bench) the wall time bench.py measured minus the GPU window: the host-side
cost of the fit call spread over the K steps (argument checks, plan lookup, the final host sync).
"""
import argparse
import csv
import glob
import json
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"<.*", "", name)
    return name.replace("tr::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--bench", default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--dominant", required=True)
    args = ap.parse_args()
    rows = []
    for f in glob.glob(args.trace, recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    bench = json.load(open(args.bench)) if args.bench else None
    K = args.steps or (bench["steps"] if bench else None)
    dom = [i for i, r in enumerate(rows) if args.dominant in r[2]]
    if len(dom) < K + 1:
        raise SystemExit(f"{len(dom)} launches of {args.dominant}, need {K + 1}")
    # the timed fit is the last one in the trace: it ends with the last kernel, and it starts with
    # the first kernel after the largest idle gap between the (K+1)-th-last dominant launch (the
    # warm-up fit's last iteration) and the K-th-last one (the host's fit set-up lies in that gap)
    prev, first = dom[-K - 1], dom[-K]
    gaps_b = [(rows[i + 1][0] - rows[i][1], i + 1) for i in range(prev, first)]
    start_idx = max(gaps_b)[1]
    end_idx = len(rows) - 1
    win = rows[start_idx:end_idx + 1]
    t0, t1 = win[0][0], win[-1][1]
    busy = defaultdict(int)
    count = defaultdict(int)
    for s, e, n in win:
        busy[n] += e - s
        count[n] += 1
    gaps = 0
    for a, b in zip(win, win[1:]):
        gaps += max(0, b[0] - a[1])
    out = {"steps": K, "kernels_in_window": len(win), "gpu_window_ms_per_step": (t1 - t0) / 1e6 / K,
           "kernel_ms_per_step": {n: busy[n] / 1e6 / K for n in busy},
           "kernel_mean_us": {n: busy[n] / 1e3 / count[n] for n in busy},
           "kernels_sum_ms_per_step": sum(busy.values()) / 1e6 / K, "gaps_ms_per_step": gaps / 1e6 / K}
    if bench:
        out["bench_ms_per_step"] = bench["ms_per_step"]
        out["host_ms_per_step"] = bench["ms_per_step"] - out["gpu_window_ms_per_step"]
        out["bench_dominant_event_ms"] = bench["roofline"]["kernel_avg_ms"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
