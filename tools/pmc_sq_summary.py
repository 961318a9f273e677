#!/usr/bin/env python3
"""Per-launch averages of the SQ counters collected by tools/_pmc_sq.sh for one kernel.

    python tools/pmc_sq_summary.py gpurun_out/pmcsq_<tag> <kernel-name substring>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root, kern = sys.argv[1], sys.argv[2]
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if kern not in row.get("Kernel_Name", ""):
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        by = defaultdict(list)
        for (d, c), v in per.items():
            by[c].append(v)
        for c, v in by.items():
            vals[c] = v
    for c in sorted(vals):
        v = vals[c]
        print(f"{c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
