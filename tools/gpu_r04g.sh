#!/bin/bash
# GPU tests; C5 Red Hat merge kernels; the delta-form pass timeline (TVM_PIPE_TRACE); Maven-only
# C3 with and without "-rcN" installed versions (the pairwise-program share).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04g}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c5_trace -o run --output-format csv -- python3 bench.py --config c5 --no-cpu --no-e2e --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
f=$(find $OUT/c5_trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" > $OUT/c5_kernel_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print("%6s %10.1f us  %s" % (r.get("Calls"), float(r.get("AverageNs", 0)) / 1e3, r.get("Name", "")[:110]))
PY
grep -E "rh_|scan" $OUT/c5_kernel_stats.txt || true
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_c5.json') if l.startswith('{')][-1]); print('c5 merge', d['fill_info']['redhat_merge'])"
TVM_COPY_WG_DELTA=256 TVM_PIPE_TRACE=1 timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 4 --warmup 1 > $OUT/bench_c2_trace.json 2> $OUT/bench_c2_trace.err
grep "pipe " $OUT/bench_c2_trace.err | tail -40
for pre in 0 0.03; do
  TVM_BENCH_WEIGHTS=0,1,0,0 TVM_SYNTH_MAVEN_PRE=$pre timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e --no-fill > $OUT/bench_c3_mvn$pre.json 2> $OUT/bench_c3_mvn$pre.err
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_c3_mvn$pre.json') if l.startswith('{')][-1]); print('$pre', d['config']['workload'], d['config']['matches_rank0'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done
