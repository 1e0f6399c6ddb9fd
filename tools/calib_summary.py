"""Per-kernel FETCH_SIZE / WRITE_SIZE of tools/calib_fetch (gpurun_out/calib) divided by the
bytes each kernel really touched: the counting factor of each access shape (measurement
only).  Usage: python tools/calib_summary.py gpurun_out/calib"""
import csv
import json
import os
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(d):
    truth = {r["kernel"]: int(r["bytes"]) for r in rows(os.path.join(d, "bytes.csv"))}
    out = {}
    for sub, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE"), ("rdreq", None)):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in rows(p):
            k = r["Kernel_Name"].split("(")[0]
            if k not in truth:
                continue
            name = r["Counter_Name"]
            out.setdefault(k, {}).setdefault(name, []).append(float(r["Counter_Value"]))
    dur = {}
    tp = os.path.join(d, "trace", "run_kernel_trace.csv")
    if os.path.exists(tp):
        for r in rows(tp):
            k = r["Kernel_Name"].split("(")[0]
            dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    print(f"{'kernel':<12} {'true MB':>9} {'FETCH MB':>9} {'f_fetch':>8} {'WRITE MB':>9} {'f_write':>8} "
          f"{'RDREQ':>12} {'RDREQ_32B':>12} {'R_64B':>10} {'R_128B':>10} {'sized MB':>9} {'B/RDREQ':>8} {'us':>8} {'GB/s':>7}")
    for k, b in truth.items():
        c = out.get(k, {})
        f = sum(c.get("FETCH_SIZE", [0])) / max(1, len(c.get("FETCH_SIZE", [1]))) * 1024  # KB per launch -> B
        w = sum(c.get("WRITE_SIZE", [0])) / max(1, len(c.get("WRITE_SIZE", [1]))) * 1024
        rq = sum(c.get("TCC_EA0_RDREQ_sum", [0])) / max(1, len(c.get("TCC_EA0_RDREQ_sum", [1])))
        r32 = sum(c.get("TCC_EA0_RDREQ_32B_sum", [0])) / max(1, len(c.get("TCC_EA0_RDREQ_32B_sum", [1])))
        r64 = sum(c.get("TCC_EA0_RDREQ_64B_sum", [0])) / max(1, len(c.get("TCC_EA0_RDREQ_64B_sum", [1])))
        r128 = sum(c.get("TCC_EA0_RDREQ_128B_sum", [0])) / max(1, len(c.get("TCC_EA0_RDREQ_128B_sum", [1])))
        sized = 128 * r128 + 64 * r64 + 32 * r32 + 64 * max(0.0, rq - r128 - r64 - r32)
        us = sorted(dur.get(k, [0]))[len(dur.get(k, [0])) // 2]
        res[k] = {"bytes": b, "fetch": f, "f_fetch": f / b, "write": w, "f_write": w / b, "rdreq": rq,
                  "rdreq_32b": r32, "rdreq_64b": r64, "rdreq_128b": r128, "fetch_by_request_size": sized,
                  "bytes_per_rdreq": b / rq if rq else None, "us": us,
                  "GBs": b / (us * 1e3) if us else None}
        print(f"{k:<12} {b/1e6:9.1f} {f/1e6:9.1f} {f/b:8.3f} {w/1e6:9.1f} {w/b:8.3f} {rq:12.0f} {r32:12.0f} "
              f"{r64:10.0f} {r128:10.0f} {sized/1e6:9.1f} "
              f"{(b / rq if rq else 0):8.1f} {us:8.1f} {(b / (us * 1e3) if us else 0):7.0f}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
