#!/usr/bin/env python3
"""HBM traffic per launch of the rows kernel from rocprofv3 --pmc passes.

Usage: pmc_traffic.py OUT_DIR [KEY]
OUT_DIR holds pmc_fetch/, pmc_write/ and optionally pmc_rdreq/, each with
run_counter_collection.csv from `rocprofv3 --pmc <counter> -d ... -o run
--output-format csv -- python3 bench.py ...` (tools/gpu_r2q.sh).  Prints the
profiles/pmc_traffic.json entry for KEY (default "4096x1048576").

Read bytes = FETCH_SIZE (KiB) x 1024 x 2: gfx950 counts 128-B streaming
requests at 64 B (MI355X_MICROARCH.md, HBM / rocprofv3 section);
TCC_EA0_RDREQ_sum x 128 B is the cross-check.  Write bytes = WRITE_SIZE x 1024.
"""
import csv
import json
import os
import statistics
import sys


def counter_means(path, kernel_sub="crc_rows_kernel"):
    vals = {}
    names = set()
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel_sub not in r["Kernel_Name"]:
                continue
            names.add(r["Kernel_Name"])
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}, names


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "4096x1048576"
    bs, nb = (int(x) for x in key.split("x"))
    fetch, nf, names = counter_means(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write, nw, _ = counter_means(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    read_b = fetch["FETCH_SIZE"] * 1024 * 2
    write_b = write["WRITE_SIZE"] * 1024
    alg = nb * (bs + 4)
    e = {
        "hbm_bytes_per_launch": read_b + write_b,
        "read_bytes": read_b,
        "write_bytes": write_b,
        "algorithmic_bytes": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
        "FETCH_SIZE_KiB_mean": fetch["FETCH_SIZE"],
        "WRITE_SIZE_KiB_mean": write["WRITE_SIZE"],
        "dispatches": {"fetch": nf["FETCH_SIZE"], "write": nw["WRITE_SIZE"]},
        "kernel": sorted(names)[0] if names else None,
    }
    rq = os.path.join(d, "pmc_rdreq", "run_counter_collection.csv")
    if os.path.exists(rq):
        r, _, _ = counter_means(rq)
        if "TCC_EA0_RDREQ_sum" in r:
            e["TCC_EA0_RDREQ_sum_mean"] = r["TCC_EA0_RDREQ_sum"]
            e["rdreq_x128_over_read_bytes"] = r["TCC_EA0_RDREQ_sum"] * 128 / read_b
    print(json.dumps({key: e}, indent=1))


if __name__ == "__main__":
    main()
