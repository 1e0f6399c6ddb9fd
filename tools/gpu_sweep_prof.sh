#!/bin/bash
# GPU box: interleaved variant sweep (bench.py --sweep) for the configs in $SWEEP, then a
# rocprofv3 kernel trace of the full device-resident legs (match, FillInfo, merge,
# result.Filter) for the configs in $TRACE.  OUT=gpurun_out/$TAG.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-sw}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for c in ${SWEEP:-c2}; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu --no-e2e --no-fill --sweep ${ROUNDS:-5} \
    > $OUT/sweep_$c.json 2> $OUT/sweep_$c.txt
  grep -v "^\[" $OUT/sweep_$c.txt | tail -20
done
cd /tmp
for c in ${TRACE:-c2}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_$c -o run --output-format csv -- \
    python3 -u $R/bench.py --config $c --no-cpu --no-e2e --steps 10 > $OUT/trace_$c.log 2>&1
  f=$(find $OUT/trace_$c -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 "$f" | head -24
done
