#!/usr/bin/env python3
"""Map a rocprofv3 run of tools/cold_probe.py onto the probe's scenarios.

usage: cold_attrib.py PROBE_JSON ROCPROF_DIR [ROCPROF_DIR ...]

PROBE_JSON is the probe's stdout of the SAME run as each ROCPROF_DIR (one
probe JSON per directory: pass them as PROBE_JSON=DIR pairs, or one JSON for
one dir).  Every crc_rows_kernel dispatch of the probe is one labelled pass
(the probe's run-length encoded "order").  Prints per scenario: median
kernel-trace duration, and for --pmc directories the median of every
counter plus the effective clock (GRBM_GUI_ACTIVE / 8 / duration,
MI355X_MICROARCH.md DVFS note) and UTCL1 translation miss rate.
"""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict

KERNEL = "crc_rows_kernel"


def labels(probe):
    out = []
    for lab, n in probe["order"]:
        out += [lab] * n
    return out


def load(d):
    rows = defaultdict(dict)  # dispatch id -> {counter: value, "_dur": ns}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            e = rows[int(r["Dispatch_Id"])]
            e[r["Counter_Name"]] = float(r["Counter_Value"])
            e["_dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            rows[int(r["Dispatch_Id"])]["_dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [rows[k] for k in sorted(rows)]


def main():
    pairs = []
    for a in sys.argv[1:]:
        if "=" in a:
            pairs.append(tuple(a.split("=", 1)))
    if not pairs:
        pairs = [(sys.argv[1], d) for d in sys.argv[2:]]
    agg = defaultdict(lambda: defaultdict(list))
    for pj, d in pairs:
        probe = json.load(open(pj))
        lab = labels(probe)
        disp = load(d)
        if len(disp) != len(lab):
            sys.exit(f"{d}: {len(disp)} {KERNEL} dispatches, probe order lists {len(lab)}")
        for L, e in zip(lab, disp):
            if L == "ramp":
                continue
            for k, v in e.items():
                agg[L][k].append(v)
    out = {}
    for L, cs in agg.items():
        o = {k: statistics.median(v) for k, v in cs.items() if not k.startswith("_")}
        dur = statistics.median(cs["_dur"]) * 1e-9
        o["median_us"] = round(dur * 1e6, 2)
        o["n"] = len(cs["_dur"])
        if "GRBM_GUI_ACTIVE" in o:
            clk = [g / 8 / (t * 1e-9) / 1e9 for g, t in zip(cs["GRBM_GUI_ACTIVE"], cs["_dur"])]
            o["effective_clock_GHz"] = round(statistics.median(clk), 3)
        if "TCP_UTCL1_TRANSLATION_MISS_sum" in o and "TCP_UTCL1_TRANSLATION_HIT_sum" in o:
            m, h = o["TCP_UTCL1_TRANSLATION_MISS_sum"], o["TCP_UTCL1_TRANSLATION_HIT_sum"]
            o["utcl1_miss_rate"] = round(m / max(1.0, m + h), 5)
        if "GRBM_UTCL2_BUSY" in o and "GRBM_GUI_ACTIVE" in o:
            o["utcl2_busy_frac"] = round(o["GRBM_UTCL2_BUSY"] / o["GRBM_GUI_ACTIVE"], 4)  # both summed over XCDs
        out[L] = o
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
