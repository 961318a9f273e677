#!/usr/bin/env python3
"""Average per dispatch of every counter in rocprofv3 counter_collection.csv files, for the
kernels whose name matches a regex (tools/, used with tools/pmc_sweep.sh).

    python tools/pmc_summary.py --kernel 'k_mnl_fused' gpurun_out/pmc/*/*counter_collection.csv
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", required=True)
ap.add_argument("csv", nargs="+")
a = ap.parse_args()
rx = re.compile(a.kernel)
acc = collections.defaultdict(list)
for path in a.csv:
    with open(path) as f:
        for row in csv.DictReader(f):
            if rx.search(row["Kernel_Name"]):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:32s} {sum(v) / len(v):16.4g}   ({len(v)} dispatches)")
