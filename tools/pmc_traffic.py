#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 --pmc passes.

Usage:
  pmc_traffic.py OUT_DIR [KEY]                      (OUT_DIR/pmc_fetch, pmc_write, pmc_rdreq)
  pmc_traffic.py --fetch D --write D [--rdreq D] [--kernel SUB] [--key BSxNB]
Each directory holds run_counter_collection.csv from `rocprofv3 --pmc <counter>
-d ... -o run --output-format csv -- python3 bench.py ...` (tools/gpu_steps.sh
pmc steps).  Prints the profiles/pmc_traffic.json entry for KEY (block size x
blocks per launch, default "4096x1048576"), averaged over every dispatch of
the kernel whose name contains SUB (default crc_rows_kernel).

Read bytes = FETCH_SIZE (KiB) x 1024 x 2: gfx950 counts 128-B streaming
requests at 64 B (MI355X_MICROARCH.md, HBM / rocprofv3 section);
TCC_EA0_RDREQ_sum x 128 B is the cross-check.  Write bytes = WRITE_SIZE x 1024.
"""
import argparse
import csv
import json
import os
import statistics


def counter_means(path, kernel_sub="crc_rows_kernel", min_value=0.0):
    vals = {}
    names = set()
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel_sub not in r["Kernel_Name"]:
                continue
            v = float(r["Counter_Value"])
            if v < min_value:
                continue
            names.add(r["Kernel_Name"])
            vals.setdefault(r["Counter_Name"], []).append(v)
    return {k: statistics.mean(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir", nargs="?")
    ap.add_argument("key_pos", nargs="?")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--rdreq")
    ap.add_argument("--kernel", default="crc_rows_kernel")
    ap.add_argument("--key", default=None)
    ap.add_argument("--min-fetch-kib", type=float, default=0.0,
                    help="ignore dispatches reading less (e.g. a bench's small warm-up call)")
    a = ap.parse_args()
    key = a.key or a.key_pos or "4096x1048576"
    fd = a.fetch or os.path.join(a.out_dir, "pmc_fetch")
    wd = a.write or os.path.join(a.out_dir, "pmc_write")
    rd = a.rdreq or (os.path.join(a.out_dir, "pmc_rdreq") if a.out_dir else None)
    bs, nb = (int(x) for x in key.split("x"))
    fetch, nf, names = counter_means(os.path.join(fd, "run_counter_collection.csv"), a.kernel, a.min_fetch_kib)
    write, nw, _ = counter_means(os.path.join(wd, "run_counter_collection.csv"), a.kernel)
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
    rq = os.path.join(rd, "run_counter_collection.csv") if rd else None
    if rq and os.path.exists(rq):
        r, _, _ = counter_means(rq, a.kernel)
        if "TCC_EA0_RDREQ_sum" in r:
            e["TCC_EA0_RDREQ_sum_mean"] = r["TCC_EA0_RDREQ_sum"]
            e["rdreq_x128_over_read_bytes"] = r["TCC_EA0_RDREQ_sum"] * 128 / read_b
    print(json.dumps({key: e}, indent=1))


if __name__ == "__main__":
    main()
