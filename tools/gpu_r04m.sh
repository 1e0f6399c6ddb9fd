#!/bin/bash
# GPU tests; the round-end flow (smoke, default bench line with its CPU baseline); C5 with
# the filter's survivor-sum scan (kernel trace).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04o}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -3 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
python3 - $OUT/bench_default.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print({k: d[k] for k in ("metric", "value", "ms_per_step", "steps", "warmup")})
print("roofline", {k: d["roofline"].get(k) for k in ("achieved", "frac", "traffic", "kernel_ms")})
print("cpu", d.get("cpu_baseline"))
print("e2e", d["end_to_end"]["ms_per_pass"], "fresh", d["fresh_batch"]["packages_per_s"])
f = d.get("fill_info") or {}
print("fill", f.get("kernel_ms"), "filter", (f.get("result_filter") or {}).get("ms"))
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c5_trace -o run --output-format csv -- python3 bench.py --config c5 --no-cpu --no-e2e --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
f=$(find $OUT/c5_trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" > $OUT/c5_kernel_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print("%6s %10.1f us  %s" % (r.get("Calls"), float(r.get("AverageNs", 0)) / 1e3, r.get("Name", "")[:110]))
PY
cat $OUT/c5_kernel_stats.txt
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_c5.json') if l.startswith('{')][-1]); f=d['fill_info']; print('c5 filter ms', f['result_filter']['ms'], 'vex', f['result_filter']['vex']['ms'], 'merge', f['redhat_merge']['kernel_ms'])"
