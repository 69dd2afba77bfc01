#!/usr/bin/env python3
"""Per-call kernel durations from a rocprofv3 kernel trace of
tools/few_values_trace.py: consecutive dispatches grouped into calls of
`--per-call` kernels, averaged over the timed calls of each (case, path) run
(the script's 30 warm-up + 100 timed calls).  Prints one line per run with
each kernel's mean duration and the mean span first start -> last end.
Tools only."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warm", type=int, default=30)
    ap.add_argument("--timed", type=int, default=100)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if "crc_" in r["Kernel_Name"] and "fill_splitmix" not in r["Kernel_Name"]
          and "xcd_probe" not in r["Kernel_Name"] and "crc_zero" not in r["Kernel_Name"]]
    short = lambda r: r["Kernel_Name"].split("::")[1].split("<")[0].split("(")[0] if "::" in r["Kernel_Name"] else r["Kernel_Name"][:30]
    i, run = 0, 0
    while i < len(ks):
        per = 3 if short(ks[i]) == "crc_seg_plan_kernel" else 1
        calls = ks[i:i + per * (a.warm + a.timed)]
        i += per * (a.warm + a.timed)
        timed = calls[per * a.warm:]
        agg = collections.defaultdict(list)
        spans = []
        for c in range(0, len(timed), per):
            grp = timed[c:c + per]
            for r in grp:
                agg[short(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            spans.append((int(grp[-1]["End_Timestamp"]) - int(grp[0]["Start_Timestamp"])) / 1e3)
        print(run, {k: round(sum(v) / len(v), 2) for k, v in agg.items()},
              "span_us", round(sum(spans) / max(1, len(spans)), 2))
        run += 1


if __name__ == "__main__":
    main()
