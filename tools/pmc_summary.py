#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (tools/profile_round.sh, tools/pmc_sq.sh) per kernel AND grid.

Usage: pmc_summary.py OUT_DIR [--config c2] [--bench OUT_DIR/bench.json] [--json PATH]

Every dispatch is grouped by (kernel, Grid_Size): the full-batch launches of the match kernel
(one grid = the whole batch) are kept apart from the end-to-end pipeline's chunk launches and
from other kernels, so "per launch" always means one full-grid launch.  For each group: the
kernel-trace average duration (run_kernel_trace.csv) and the per-dispatch median of every
collected counter.  FETCH_SIZE / WRITE_SIZE are KiB (rocprofv3).

With --json, the match kernel's full-grid group (the largest grid among the match kernels) is
written as the summary bench.py reads for `roofline.traffic`: raw FETCH + WRITE bytes per
full-grid launch, the kernel's name, the bench variant and the kernel-source hash of the
build that was profiled (bench.py refuses a summary whose hash or variant differs from the
running build).  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE counts half the bytes of a
wide (16 B/lane) coalesced streaming read; the raw counter is reported, the note says so.
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("probe_kernel", "sweep_kernel", "fused_kernel", "persist_kernel", "match_kernel", "fill_pairs_kernel",
           "filter_mark", "filter_select", "filter_edges", "filter_count_dup", "filter_count", "filter_place", "rules_insert", "vex_mark",
           "order_kernel", "rh_count_kernel", "rh_scan_kernel", "rh_emit_kernel", "unpack_kernel", "copy_out_kernel",
           "wrapped_scan")
MATCH = ("fused_kernel", "persist_kernel", "match_kernel")


def kname(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def collect(out):
    groups = {}  # (short, full name, grid) -> {"counters": {name: [values]}, "dur": [ns]}

    def grp(r, name_col):
        k = kname(r[name_col])
        if not k or "diag" in r[name_col]:
            return None
        if r.get("Grid_Size"):
            grid = int(float(r["Grid_Size"]))
        else:  # kernel-trace rows give the grid per dimension
            grid = 1
            for ax in "XYZ":
                grid *= int(float(r.get(f"Grid_Size_{ax}") or 1))
        return groups.setdefault((k, r[name_col], grid), {"counters": {}, "dur": []})

    for f in glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            g = grp(r, "Kernel_Name")
            if g is not None:
                g["dur"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for f in sorted(glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            g = grp(r, "Kernel_Name")
            if g is not None:
                g["counters"].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return groups


def main(argv):
    out = argv[0]
    opt = dict(zip(argv[1::2], argv[2::2]))
    groups = collect(out)
    rows = []
    for (k, full, grid), g in sorted(groups.items(), key=lambda x: (x[0][0], -x[0][2])):
        c = {n: statistics.median(v) for n, v in g["counters"].items()}
        d = {"kernel": full, "short": k, "grid": grid, "counters": c,
             "launches_traced": len(g["dur"]), "avg_ns": statistics.mean(g["dur"]) if g["dur"] else None}
        if "FETCH_SIZE" in c:
            d["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            d["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes_raw"] = d["fetch_bytes_raw"] + d["write_bytes"]
        if "TCC_EA0_RDREQ_128B_sum" in c:  # read bytes by request size (profiles/r06/calib.txt)
            r, r32 = c.get("TCC_EA0_RDREQ_sum", 0.0), c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            r64, r128 = c.get("TCC_EA0_RDREQ_64B_sum", 0.0), c["TCC_EA0_RDREQ_128B_sum"]
            d["fetch_bytes_sized"] = 128 * r128 + 64 * r64 + 32 * r32 + 64 * max(0.0, r - r128 - r64 - r32)
            if "write_bytes" in d:
                d["hbm_bytes_sized"] = d["fetch_bytes_sized"] + d["write_bytes"]
        rows.append(d)
        avg = f"avg {d['avg_ns'] / 1e3:.1f} us over {d['launches_traced']} traced launches" if d["avg_ns"] else "no trace"
        print(f"== {k}  grid {grid}  {avg}\n   {full}")
        waves = c.get("SQ_WAVES")
        for n, v in sorted(c.items()):
            per = f"   ({v / waves:,.1f} per wave)" if waves and n.startswith("SQ_INSTS") else ""
            print(f"{n:>28}: {v:,.1f}{per}")
        for n in ("fetch_bytes_raw", "write_bytes", "hbm_bytes_raw", "fetch_bytes_sized", "hbm_bytes_sized"):
            if n in d:
                print(f"{n:>28}: {d[n]:,.0f} per launch")
    if "--json" in opt:
        match = [d for d in rows if d["short"] in MATCH and "hbm_bytes_raw" in d]
        if not match:
            print("no match-kernel FETCH/WRITE counters found", file=sys.stderr)
            return 1
        # one device-resident pass: per match-kernel instantiation without the pipeline's result
        # move (", false>(") its largest-grid group - one launch, or two when an all-grammar
        # batch runs its tiles without Maven on the GM_LEAN kernel (engine.hip Engine::launch)
        parts = {}
        for d in match:
            if ", false>(" in d["kernel"] and (d["kernel"] not in parts or d["grid"] > parts[d["kernel"]]["grid"]):
                parts[d["kernel"]] = d
        parts = sorted(parts.values(), key=lambda d: -d["grid"]) or [max(match, key=lambda d: d["grid"])]
        top = dict(parts[0])
        if len(parts) > 1:
            for k in ("grid", "avg_ns", "fetch_bytes_raw", "write_bytes", "hbm_bytes_raw", "fetch_bytes_sized",
                      "hbm_bytes_sized"):
                if all(d.get(k) is not None for d in parts):
                    top[k] = sum(d[k] for d in parts)
            top["counters"] = {k: sum(d["counters"].get(k, 0.0) for d in parts) for k in parts[0]["counters"]}
        top["launches"] = [{"kernel": d["kernel"], "grid": d["grid"], "avg_ns": d["avg_ns"]} for d in parts]
        bench = {}
        if opt.get("--bench") and os.path.exists(opt["--bench"]):
            txt = open(opt["--bench"]).read().strip().splitlines()
            bench = json.loads(txt[-1]) if txt else {}
        cfg = bench.get("config", {})
        summ = {"config": opt.get("--config"), "workload": cfg.get("workload"), "kernel": top["kernel"],
                "kernel_variant": cfg.get("kernel_variant"), "kernel_source": cfg.get("kernel_source"),
                "grid": top["grid"], "avg_ns_full_grid": top["avg_ns"], "launches": top["launches"],
                "fetch_bytes_raw": top["fetch_bytes_raw"], "write_bytes": top["write_bytes"],
                "hbm_bytes_per_launch": top["hbm_bytes_raw"],
                "fetch_bytes_sized": top.get("fetch_bytes_sized"), "hbm_bytes_sized": top.get("hbm_bytes_sized"),
                "rdreq": {k: top["counters"].get(k) for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum",
                                                               "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")},
                "note": "raw FETCH_SIZE + WRITE_SIZE of one full-grid launch (median over the profiled launches); "
                        "FETCH_SIZE tallies every L2-to-fabric read request at 64 B, but streaming reads go out as "
                        "128-B requests (calibrated on the match kernel's own load shapes, profiles/r06/calib.txt), "
                        "so hbm_bytes_sized = 128 R_128B + 64 R_64B + 32 R_32B + WRITE_SIZE is the corrected figure "
                        "(Infinity-Cache hits are still counted: bytes from beyond L2)"}
        with open(opt["--json"], "w") as f:
            json.dump(summ, f, indent=1)
        print(json.dumps(summ))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
