#!/bin/bash
# Benchmark + rocprofv3 evidence for one round (run on the GPU box via gpurun).
#   1. bench.py (default config)                          -> gpurun_out/bench.json
#   2. rocprofv3 --kernel-trace --stats of a short bench  -> gpurun_out/prof_trace/
#   3. rocprofv3 --pmc FETCH_SIZE   (own pass)            -> gpurun_out/prof_fetch/
#   4. rocprofv3 --pmc WRITE_SIZE   (own pass)            -> gpurun_out/prof_write/
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
STEPS=${STEPS:-20}
timeout -k 10 400 python3 $R/bench.py --steps $STEPS > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu > $OUT/prof_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu > $OUT/prof_write.log 2>&1
echo done
