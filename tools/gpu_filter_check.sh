#!/bin/bash
# GPU box: result.Filter / export tests, then a kernel trace of the C2 (and $MORE) legs.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-fchk}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fillinfo.py tests/test_gpu_redhat_chain.py ${TESTS:-} -m gpu -x -q \
  --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
cd /tmp
for c in ${CONFIGS:-c2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$c -o run --output-format csv -- \
    python3 -u $R/bench.py --config $c --no-cpu --no-e2e --steps 10 > $OUT/trace_$c.log 2>&1
  f=$(find $OUT/trace_$c -name '*kernel_stats.csv' | head -1)
  python3 $R/tools/kstats.py "$f"
  : <<'PY'
import csv, sys
for r in list(csv.reader(open(sys.argv[1])))[1:]:
    n = r[0].split("(")[0].replace("tvm::(anonymous namespace)::", "")[:60]
    if "filter" in n or "vex" in n or "fill" in n or "fused" in n or "rh_" in n:
        print(f"  {n:60s} {r[1]:>4s} {float(r[3])/1e3:9.1f} us")
PY
  grep '^{"metric"' $OUT/trace_$c.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); f=d.get('fill_info') or {}
print('  filter', json.dumps(f.get('result_filter')))"
done
