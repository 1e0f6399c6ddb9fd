#!/bin/bash
# GPU box (measurement): result.Filter kernel times under TVM_FILTER_DIAG = 0..3 (C2), one
# rocprofv3 kernel trace per setting.  OUT=gpurun_out/$TAG.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-fdiag}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for d in ${DIAGS:-0 1 2 3}; do
  TVM_FILTER_DIAG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/d$d -o run --output-format csv -- \
    python3 -u $R/bench.py --config ${CONFIG:-c2} --no-cpu --no-e2e --steps 5 --warmup 1 > $OUT/d$d.log 2>&1
  f=$(find $OUT/d$d -name "*kernel_stats.csv" | head -1)
  echo "== diag $d"; python3 $R/tools/kstats.py "$f" | grep -i "filter\|vex\|scan"
done
