#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of tools/profile_round.sh for the match kernel.

Prints per-launch averages of every collected counter for match_kernel dispatches and the
kernel-trace average duration; writes profiles/pmc_summary.json-style JSON to stdout's
last line.  FETCH_SIZE/WRITE_SIZE are in KiB (rocprofv3); per MI355X_MICROARCH.md §HBM,
FETCH_SIZE under-reports wide coalesced streaming reads by 2x on gfx950, so both the raw
and the doubled read figure are given (the kernel's reads are mostly 16-32 B random
accesses, i.e. not the calibrated wide-stream case).
"""
import csv
import glob
import json
import os
import statistics
import sys


def main(out):
    res = {"counters": {}}
    stats = os.path.join(out, "prof_trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            if "match_kernel" in r["Name"]:
                res["kernel"] = r["Name"]
                res["kernel_avg_ns"] = float(r["AverageNs"])
                res["kernel_calls"] = int(r["Calls"])
    for f in sorted(glob.glob(os.path.join(out, "prof_*", "run_counter_collection.csv"))):
        vals = {}
        for r in csv.DictReader(open(f)):
            if "match_kernel" not in r["Kernel_Name"] or "ablate" in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for k, v in vals.items():
            res["counters"][k] = statistics.median(v)
    c = res["counters"]
    if "FETCH_SIZE" in c:
        res["fetch_bytes_per_launch"] = c["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in c:
        res["write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        res["hbm_bytes_per_launch"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    for k, v in sorted(c.items()):
        print(f"{k:>28}: {v:,.1f}")
    for k in ("kernel_avg_ns", "fetch_bytes_per_launch", "write_bytes_per_launch", "hbm_bytes_per_launch"):
        if k in res:
            print(f"{k:>28}: {res[k]:,.1f}")
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1])
