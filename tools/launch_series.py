#!/usr/bin/env python3
"""Per-launch durations of one kernel in a rocprofv3 kernel trace, in launch order, with the idle
time before each launch that follows a gap longer than --gap-us (the host set-up between fits).

    python tools/launch_series.py profiles/r04_drv_c3_kernel_trace.csv k_mnl_duo

Shows what a short timed fit meets after the GPU idled: the compute-bound kernels (c3, c5) run
their first launches at full clock, then slow by a third for several milliseconds while the
power controller pulls the clock back, then recover over ~20 launches.
"""
import csv
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    gap_us = float(sys.argv[3]) if len(sys.argv) > 3 else 1000.0
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    prev_end = None
    series = []
    idle = 0.0  # idle time in long gaps since the previous launch of the kernel
    for s, e, n in rows:
        if prev_end is not None and s - prev_end > gap_us * 1e3:
            idle += (s - prev_end) / 1e6
        if kern in n:
            if idle > 0:
                series.append(f"| idle {idle:.1f} ms |")
                idle = 0.0
            series.append(f"{(e - s) / 1e3:.0f}")
        prev_end = e
    print(f"{kern} launch durations (us) in {path}:")
    print(" ".join(series))


if __name__ == "__main__":
    main()
