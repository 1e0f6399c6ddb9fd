#!/bin/bash
# Instruction / stall counters of the match kernel (run on the GPU box via gpurun).
# One rocprofv3 --pmc pass per counter group, each under its own time limit; the bench runs
# the match kernel only (--no-fill --no-cpu).  Extra bench flags: BENCH_ARGS.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PMC_TAG:-sq}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 3 --warmup 1 --no-cpu --no-e2e ${NOFILL---no-fill} ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/prof_trace.log 2>&1
pmc() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/prof_$name -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/prof_$name.log 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
pmc sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU
pmc tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt || true
cat $OUT/pmc_summary.txt
