#!/usr/bin/env python3
"""Timeline of the end-to-end pipelined pass from a rocprofv3 --kernel-trace
--memory-copy-trace output directory (CSV or the default SQLite database): per pass (a run of pipeline chunks), when each copy and
kernel ran, relative to the pass start (tools/profile_e2e.sh)."""
import csv
import glob
import os
import sys


def rows(out, pat):
    r = []
    for f in glob.glob(os.path.join(out, "**", pat), recursive=True):
        r += list(csv.DictReader(open(f)))
    return r


def db_rows(out):
    """(start, end, label) from rocprofv3's default SQLite output (rocpd views)."""
    import sqlite3
    ev = []
    for f in glob.glob(os.path.join(out, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        for name, s, e, grid in c.execute("select name, start, end, grid_x from kernels"):
            short = next((k for k in KERNELS if k in name), None)
            if short:
                ev.append((int(s), int(e), f"{short} grid {grid}"))
        for s, e, size, name in c.execute("select start, end, size, name from memory_copies"):
            ev.append((int(s), int(e), f"copy {name} {int(size) / 1e6:.2f}MB"))
    return ev


KERNELS = ("fused_kernel", "order_kernel", "copy_out_kernel", "unpack_kernel")


def main(out):
    ev = db_rows(out)
    for r in rows(out, "*kernel_trace.csv"):
        name = r["Kernel_Name"]
        short = next((k for k in KERNELS if k in name), None)
        if short:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
    for r in rows(out, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   f"copy {r.get('Direction', r.get('Kind', '?'))} {int(r.get('Size', r.get('Bytes', 0)) or 0) >> 20}MiB"))
    ev.sort()
    # the last pass: from the last 'fused_kernel' burst back to the copies before it
    t_last = max(s for s, _, n in ev if n.startswith("fused_kernel"))
    tail = [e for e in ev if e[0] >= t_last - 8_000_000]
    t0 = tail[0][0]
    for s, e, n in tail:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n}")


if __name__ == "__main__":
    main(sys.argv[1])
