#!/bin/bash
# C5 result.Filter breakdown: kernel trace of the C5 bench legs (match,
# Red Hat merge, FillInfo, Filter, Filter+VEX) -> gpurun_out/c5prof/; plus a variant sweep
# of C3 (language packages).  Every GPU step has its own time limit, chained with &&.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/c5prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 5 --warmup 1 --no-cpu --no-e2e > $OUT/bench_c5.log 2>&1
grep '^{"metric"' $OUT/bench_c5.log | tail -1 > $OUT/bench_c5.json
python3 - $OUT <<'PY'
import csv, glob, os, sys
out = sys.argv[1]
rows = {}
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows[r["Name"][:90]] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3)
for n, (c, avg, tot) in sorted(rows.items(), key=lambda x: -x[1][2])[:25]:
    print(f"{c:5d} {avg:9.1f} us avg {tot:10.1f} us total  {n}")
PY
cd $R && timeout -k 10 300 python3 bench.py --config c3 --sweep 4 --steps 5 --no-cpu --no-e2e > $OUT/sweep_c3.json 2> $OUT/sweep_c3.err && grep sweep $OUT/sweep_c3.err
