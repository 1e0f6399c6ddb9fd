#!/bin/bash
# Variant/ablation sweep per workload (run on the GPU box via gpurun): per-variant
# median kernel times go to gpurun_out/sweep_<cfg>.err.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
for cfg in ${CFGS:-c2 c3 c5}; do
  timeout -k 10 300 python3 -u $R/bench.py --config $cfg --no-cpu --sweep ${SWEEP:-3} --steps 10 > $OUT/sweep_$cfg.json 2> $OUT/sweep_$cfg.err || { tail -20 $OUT/sweep_$cfg.err; exit 1; }
  grep -E "sweep|bench\]" $OUT/sweep_$cfg.err
done
