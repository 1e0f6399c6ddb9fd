#!/bin/bash
# One GPU box call (gpurun): default bench lines for the configs in $CONFIGS (no CPU leg) and a
# rocprofv3 kernel trace of the first config's device-resident pass.  OUT=gpurun_out/$TAG.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-quick}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c5}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  cat $OUT/bench_$c.json
done
first=$(echo ${CONFIGS:-c2 c5} | cut -d' ' -f1)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u $R/bench.py --config $first --no-cpu --no-e2e --no-fill --steps 10 > $OUT/trace.log 2>&1
cd $R
f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -12
