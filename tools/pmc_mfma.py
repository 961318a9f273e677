#!/usr/bin/env python3
"""Matrix-core utilisation of the dominant kernel from one rocprofv3 PMC pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace ... -- python bench.py ...
    python tools/pmc_mfma.py --csv <..._counter_collection.csv> --kernel k_spec_fused<0 --flops F --ms T

Units (MI355X_MICROARCH.md, PMC table): SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles
summed over every SIMD (4 per CU, 256 CUs); GRBM_GUI_ACTIVE is the GPU-busy cycle count summed
over the 8 XCDs.  busy fraction = MFMA_BUSY / (4 * 256 * GRBM_GUI_ACTIVE / 8).  The effective
clock GRBM_GUI_ACTIVE / 8 / kernel time (DVFS) is reported beside it, and, when the algorithmic
flops per launch are given, the achieved rate against the dense fp32 matrix peak at that clock.
"""
import argparse
import csv
import json
import re

N_SIMD = 4 * 256
FP32_MFMA_FLOP_PER_CLK_PER_CU = 256  # v_mfma_f32_16x16x4_f32: 8 cyc/CU for 2048 flops (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--csv", required=True)
    ap.add_argument("--kernel", required=True, help="regex on Kernel_Name")
    ap.add_argument("--flops", type=float, default=None, help="algorithmic flops per launch")
    ap.add_argument("--config", default="")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    per = {}
    with open(args.csv) as f:
        for row in csv.DictReader(f):
            if not re.search(args.kernel, row["Kernel_Name"]):
                continue
            d = per.setdefault(row.get("Dispatch_Id", row.get("Correlation_Id")), {"ns": None})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            if "Start_Timestamp" in row and row.get("End_Timestamp"):
                d["ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    ds = [d for d in per.values() if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d]
    if not ds:
        raise SystemExit("no dispatch with both counters")
    busy = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in ds) / len(ds)
    gui = sum(d["GRBM_GUI_ACTIVE"] for d in ds) / len(ds)
    cyc = gui / 8.0
    res = {"config": args.config, "kernel": args.kernel, "dispatches": len(ds),
           "mfma_busy_cycles": busy, "grbm_gui_active": gui, "mfma_busy_frac": busy / (N_SIMD * cyc)}
    ns = [d["ns"] for d in ds if d.get("ns")]
    if ns:
        t = sum(ns) / len(ns) * 1e-9
        res["kernel_ms_under_pmc"] = t * 1e3
        res["effective_clock_ghz"] = cyc / t / 1e9
        if args.flops:
            res["tflops"] = args.flops / t / 1e12
            res["fp32_mfma_peak_tflops_at_that_clock"] = FP32_MFMA_FLOP_PER_CLK_PER_CU * 256 * cyc / t / 1e12
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
