#!/usr/bin/env python3
"""The headline roofline from a rocprofv3 kernel trace of the SAME bench.py run.

usage: ktrace_window.py BENCH_JSON KTRACE_DIR

BENCH_JSON is bench.py's stdout (the one JSON line) or its detail file of a run made under
`rocprofv3 --kernel-trace --stats -d KTRACE_DIR`.  The headline kernel is the
crc_rows_kernel instance dispatched first (warmup + ramp + timed steps come
before every other leg); the line's config.timed_launches names which of its dispatches were
the K timed steps (they follow the W warmup and the untimed ramp).  Prints
one JSON object: mean / median / min / max duration of exactly those K
dispatches, the roofline fraction each gives (algorithmic bytes per launch /
duration / 8 TB/s), and how far the trace's mean-based fraction is from the
line's own HIP-event `roofline.frac`.
"""
import csv
import glob
import json
import re
import statistics
import sys
from collections import defaultdict


def main():
    line = None
    with open(sys.argv[1]) as f:
        text = f.read()
    try:  # bench.py's detail file (gpurun_out/bench_detail.json): one JSON document
        line = json.loads(text)
    except ValueError:  # its stdout: the JSON line among other output
        for ln in text.splitlines():
            ln = ln.strip()
            if ln.startswith("{"):
                line = json.loads(ln)
    if line is None:
        sys.exit("no JSON line in " + sys.argv[1])
    m = re.match(r"dispatches (\d+)\.\.(\d+)", line["config"]["timed_launches"])
    lo, hi = int(m.group(1)), int(m.group(2))
    by_name = defaultdict(list)
    for f in glob.glob(f"{sys.argv[2]}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "crc_rows_kernel" in r["Kernel_Name"]:
                by_name[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) -
                                                  int(r["Start_Timestamp"])))
    # the headline is the first rows kernel the process dispatched (the odd
    # legs' window kernels may have more dispatches in all)
    name = min(by_name, key=lambda k: min(i for i, _ in by_name[k]))
    d = [t for _, t in sorted(by_name[name])]
    win = d[lo - 1:hi]
    if len(win) != hi - lo + 1:
        sys.exit(f"trace holds {len(d)} dispatches of the headline kernel, the line names {lo}..{hi}")
    alg = line["roofline"]["alg_bytes_per_launch"]
    peak = line["roofline"]["peak"]

    def frac(ns):
        return alg / (ns * 1e-9) / 1e9 / peak

    mean, med = statistics.mean(win), statistics.median(win)
    out = {"kernel": name, "dispatches_of_kernel": len(d), "timed_window": [lo, hi], "n": len(win),
           "mean_us": round(mean / 1e3, 2), "median_us": round(med / 1e3, 2),
           "min_us": round(min(win) / 1e3, 2), "max_us": round(max(win) / 1e3, 2),
           "alg_bytes_per_launch": alg, "frac_mean": round(frac(mean), 4), "frac_median": round(frac(med), 4),
           "line_kernel_ms": line["roofline"]["kernel_ms"], "line_frac": line["roofline"]["frac"],
           "frac_mean_vs_line_pct": round((frac(mean) / line["roofline"]["frac"] - 1) * 100, 2),
           "all_dispatches_mean_us": round(statistics.mean(d) / 1e3, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
