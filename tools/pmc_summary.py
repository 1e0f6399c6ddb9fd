#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (tools/profile_round.sh, tools/pmc_sq.sh) per match kernel.

For every kernel of the match path (probe_kernel, sweep_kernel) prints the kernel-trace
average duration and the per-dispatch median of every collected counter, plus per-wave
instruction counts when SQ_WAVES was collected.  FETCH_SIZE / WRITE_SIZE are KiB
(rocprofv3); per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports half the bytes of wide
coalesced streaming reads on gfx950 (only the staging loads here are that shape), so the
raw figure is given.  The last line is JSON (profiles/pmc_summary.json form).
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("probe_kernel", "sweep_kernel", "fused_kernel", "match_kernel", "fill_pairs_kernel", "filter_mark",
           "filter_select", "filter_place", "order_kernel")


def kname(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def main(out):
    res = {"kernels": {}}
    for stats in glob.glob(os.path.join(out, "**", "run_kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(stats)):
            k = kname(r["Name"])
            if k:
                d = res["kernels"].setdefault(k, {"counters": {}})
                d["name"] = r["Name"]
                d["avg_ns"] = float(r["AverageNs"])
                d["calls"] = int(r["Calls"])
    for f in sorted(glob.glob(os.path.join(out, "**", "run_counter_collection.csv"), recursive=True)):
        vals = {}
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if not k or "diag" in r["Kernel_Name"]:
                continue
            vals.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        for (k, c), v in vals.items():
            res["kernels"].setdefault(k, {"counters": {}})["counters"][c] = statistics.median(v)
    for k, d in res["kernels"].items():
        c = d["counters"]
        if "FETCH_SIZE" in c:
            d["fetch_bytes_per_launch"] = c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            d["write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes_per_launch"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        print(f"== {k}  avg {d.get('avg_ns', 0) / 1e3:.1f} us over {d.get('calls', 0)} calls")
        for n, v in sorted(c.items()):
            per = f"   ({v / c['SQ_WAVES']:,.1f} per wave)" if "SQ_WAVES" in c and n.startswith("SQ_INSTS") else ""
            print(f"{n:>28}: {v:,.1f}{per}")
        for n in ("fetch_bytes_per_launch", "write_bytes_per_launch", "hbm_bytes_per_launch"):
            if n in d:
                print(f"{n:>28}: {d[n]:,.1f}")
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1])
