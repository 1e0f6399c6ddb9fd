"""Per-kernel summary of a rocprofv3 SQLite output (tools: profiling helper, not product).
usage: python tools/kstats.py <run_results.db> [name filter]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
q = ("select s.kernel_name, count(*), avg(d.end-d.start)/1000.0, sum(d.end-d.start)/1e6 from rocpd_kernel_dispatch d "
     "join rocpd_info_kernel_symbol s on d.kernel_id=s.id group by s.kernel_name order by 4 desc")
print("%-100s %6s %12s %10s" % ("kernel", "calls", "avg_us", "total_ms"))
for name, n, avg, tot in c.execute(q):
    if flt in name:
        print("%-100s %6d %12.1f %10.2f" % (name[:100], n, avg, tot))
