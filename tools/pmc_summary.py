#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes for one kernel (mean per dispatch).

usage: pmc_summary.py KERNEL_SUBSTRING DIR [DIR ...]
Each DIR holds a rocprofv3 `*_counter_collection.csv`.  Prints one JSON object:
counter -> mean value over the kernel's dispatches, plus derived figures
(effective clock from GRBM_GUI_ACTIVE, LDS busy fraction, wave-cycle split).
"""
import csv
import glob
import json
import statistics
import sys


def main():
    kern, dirs = sys.argv[1], sys.argv[2:]
    vals, durs = {}, []
    for d in dirs:
        for f in glob.glob(f"{d}/*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if kern not in r["Kernel_Name"]:
                    continue
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {k: statistics.mean(v) for k, v in sorted(vals.items())}
    out["dispatches_per_counter"] = {k: len(v) for k, v in sorted(vals.items())}
    if durs:
        t = statistics.median(durs) * 1e-9
        out["median_dispatch_s"] = t
        if "GRBM_GUI_ACTIVE" in out:  # summed over the 8 XCDs (MI355X_MICROARCH DVFS note)
            out["effective_clock_GHz"] = out["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
    if "SQ_WAVE_CYCLES" in out:
        wc = out["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in out:
                out[k + "_frac_of_wave_cycles"] = out[k] / wc
    if "SQ_LDS_IDX_ACTIVE" in out and "GRBM_GUI_ACTIVE" in out:
        out["lds_busy_frac"] = out["SQ_LDS_IDX_ACTIVE"] / (out["GRBM_GUI_ACTIVE"] / 8 * 256)
    if "SQ_LDS_BANK_CONFLICT" in out and "SQ_LDS_IDX_ACTIVE" in out:
        out["lds_conflict_frac"] = out["SQ_LDS_BANK_CONFLICT"] / max(1.0, out["SQ_LDS_IDX_ACTIVE"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
