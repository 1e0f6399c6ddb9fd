#!/bin/bash
# Counters for one config (run on the GPU box via gpurun): every kernel of the hot
# path with its FillInfo / Red Hat merge / result.Filter legs, not only the match kernel.
#   CONFIG=c2|c3|c4|c5, EXTRA="bench.py flags", SQ=1 adds the SQ / TCC passes.
#   out: gpurun_out/<TAG>_<cfg>/{prof_trace,prof_fetch,prof_write,prof_sq,prof_tcc}, pmc_summary.txt
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${CONFIG:-c2}
EXTRA=${EXTRA:-}
OUT=$R/gpurun_out/${TAG:-prof}_$CFG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
RUN="--config $CFG $EXTRA --steps 5 --warmup 1 --no-cpu --no-e2e"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 $R/bench.py $RUN > $OUT/prof_trace.log 2>&1
pmc() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" -d $OUT/prof_$name -o run --output-format csv -- python3 $R/bench.py $RUN > $OUT/prof_$name.log 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
if [ "${SQ:-0}" == "1" ]; then
  pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
  pmc tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
fi
grep '^{"metric"' $OUT/prof_fetch.log | tail -1 > $OUT/bench_pmc.json || true
python3 $R/tools/pmc_summary.py $OUT --config $CFG --bench $OUT/bench_pmc.json --json $OUT/pmc_summary_$CFG.json > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
