#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs).

    python tools/pmc_traffic.py --config c2 --fetch <fetch/..._counter_collection.csv> \
        --write <write/..._counter_collection.csv> [--out profiles/traffic.json]

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports exactly half of the bytes of a wide coalesced streaming read (128-B requests tallied at
64 B), so it is doubled; WRITE_SIZE reads exactly for 16-B-per-lane streaming stores.
hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, averaged over the kernel's launches.
"""
import argparse
import csv
import json
import os
import re

KERNELS = {"k_linear_fused": r"k_linear_fused", "k_linear_cluster": r"k_linear_cluster", "k_mnl_fused": r"k_mnl_fused", "k_mnl_duo": r"k_mnl_duo", "k_rows": r"k_rows<", "k_rows_mfma": r"k_rows_mfma<", "k_cols": r"k_cols<",
           "k_reduce_slabs": r"k_reduce_slabs", "k_mttkrp": r"k_mttkrp", "k_update": r"k_update",
           "k_spec_fused": r"k_spec_fused<0", "k_spec_slice": r"k_spec_slice", "k_spec_prep": r"k_spec_prep", "k_spec_chain": r"k_spec_chain"}


def per_kernel(path, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            for k, pat in KERNELS.items():
                if re.search(pat, row["Kernel_Name"]):
                    vals.setdefault(k, []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json"))
    ap.add_argument("--algorithmic", type=float, default=None,
                    help="algorithmic bytes per launch of the dominant kernel (for the ratio column)")
    ap.add_argument("--dominant", default="k_linear_fused")
    args = ap.parse_args()
    fetch, nf = per_kernel(args.fetch, "FETCH_SIZE")
    write, nw = per_kernel(args.write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        fkb, wkb = fetch.get(k), write.get(k)
        ent = {"fetch_size_kb_raw": fkb, "write_size_kb": wkb, "launches_fetch_pass": nf.get(k),
               "launches_write_pass": nw.get(k)}
        if fkb is not None and wkb is not None:
            ent["hbm_bytes_per_launch"] = (2.0 * fkb + wkb) * 1024.0
            ent["read_bytes_per_launch"] = 2.0 * fkb * 1024.0
            ent["write_bytes_per_launch"] = wkb * 1024.0
        res[k] = ent
    dom = args.dominant
    if args.algorithmic and dom in res and "hbm_bytes_per_launch" in res[dom]:
        res[dom]["traffic_over_algorithmic"] = res[dom]["hbm_bytes_per_launch"] / args.algorithmic
    res["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; hbm bytes = "
                      "(2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE half-count correction)")
    out = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            out = json.load(f)
    out[args.config] = res
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
