#!/bin/bash
# C3 (language packages) cost split: one ecosystem at a time (TVM_BENCH_WEIGHTS, same package
# count), then the measurement-only variants of the diag library over the full C3 mix.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-c3diag}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for w in 1,0,0,0 0,1,0,0 0,0,1,0 0,0,0,1; do
  TVM_BENCH_WEIGHTS=$w timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e --no-fill > $OUT/bench_c3_w$w.json 2> $OUT/bench_c3_w$w.err
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_c3_w$w.json') if l.startswith('{')][-1]); print('$w', d['config']['workload'], d['config']['matches_rank0'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done
if [ -f trivy_amd/libtrivy_amd_diag.so ]; then
  cp trivy_amd/libtrivy_amd_diag.so trivy_amd/libtrivy_amd.so
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu --no-fill --no-e2e --sweep 3 --steps 10 > $OUT/diag_sweep.json 2> $OUT/diag_sweep.err
  grep -E "sweep|bench\]" $OUT/diag_sweep.err || true
fi
