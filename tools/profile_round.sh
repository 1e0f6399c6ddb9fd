#!/bin/bash
# Benchmark + rocprofv3 evidence for one round (run on the GPU box via gpurun).
#   1. bench.py (default config, with CPU baseline)         -> gpurun_out/bench.json
#   2. rocprofv3 --kernel-trace --stats of a short bench    -> gpurun_out/prof_trace/
#   3..  one rocprofv3 --pmc pass per counter group           -> gpurun_out/prof_<name>/
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
STEPS=${STEPS:-20}
SHORT="--steps 5 --warmup 1 --no-cpu"
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 400 python3 $R/bench.py --steps $STEPS > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof_trace.log 2>&1
pmc() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $OUT/prof_$name -o run --output-format csv -- python3 $R/bench.py $SHORT > $OUT/prof_$name.log 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
if [ "${PMC_EXTRA:-0}" == "1" ]; then
  pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
  pmc tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
  pmc sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH
fi
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt || true
cat $OUT/pmc_summary.txt
echo done
