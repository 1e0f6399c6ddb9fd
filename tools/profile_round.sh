#!/bin/bash
# Benchmark + rocprofv3 evidence for one config (run on the GPU box via gpurun).
#   CONFIG=c2|c3|c4|c5 (default c2), EXTRA="bench.py flags" (e.g. --packages 12500000 for c4)
#   1. bench.py (with the CPU baseline)                          -> gpurun_out/<cfg>/bench.json
#   2. rocprofv3 --kernel-trace --stats of a short bench           -> gpurun_out/<cfg>/prof_trace/
#   3. one rocprofv3 --pmc pass per counter group, over bench runs with --no-e2e --no-fill,
#      so every match-kernel dispatch is a full-grid launch       -> gpurun_out/<cfg>/prof_<name>/
#   4. tools/pmc_summary.py: per (kernel, grid) table + gpurun_out/<cfg>/pmc_summary_<cfg>.json
#      (copy it to profiles/ to make it the summary bench.py reports as roofline.traffic)
# Every GPU step has its own time limit; steps are chained by set -e (stop at the first failure).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${CONFIG:-c2}
EXTRA=${EXTRA:-}
OUT=$R/gpurun_out/$CFG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
STEPS=${STEPS:-20}
SHORT="--config $CFG $EXTRA --steps 5 --warmup 1 --no-cpu --no-e2e --no-fill"
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 500 python3 $R/bench.py --config $CFG $EXTRA --steps $STEPS > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 $R/bench.py --config $CFG $EXTRA --steps 10 --warmup 2 --no-cpu > $OUT/prof_trace.log 2>&1
pmc() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $OUT/prof_$name -o run --output-format csv -- python3 $R/bench.py $SHORT > $OUT/prof_$name.log 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
# request sizes (tools/calib_fetch: FETCH_SIZE tallies every request at 64 B; the 128-B requests of
# streaming reads are half-counted): bytes = 128 R_128B + 64 R_64B + 32 R_32B
pmc rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
if [ "${PMC_EXTRA:-0}" == "1" ]; then
  pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
  pmc tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
fi
# the bench line of the PMC runs carries the variant + kernel-source hash of this build
grep '^{"metric"' $OUT/prof_fetch.log | tail -1 > $OUT/bench_pmc.json || true
python3 $R/tools/pmc_summary.py $OUT --config $CFG --bench $OUT/bench_pmc.json --json $OUT/pmc_summary_$CFG.json > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
echo done
