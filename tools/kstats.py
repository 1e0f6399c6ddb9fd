"""Per-kernel count / average duration (us) from a rocprofv3 results database."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
q = "select name, count(*), avg(end-start)/1000.0 from kernels group by name order by sum(end-start) desc limit 25"
for name, n, us in c.execute(q):
    print(f"{n:5d} {us:9.1f}  {name[:100]}")
