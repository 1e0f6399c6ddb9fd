#!/bin/bash
# Bench lines for every workload (run on the GPU box via gpurun): C2 (headline, with the
# CPU baseline), then the C3 language-package, C5 rpm/apk and C4 mixed OS+language (one
# GPU's 12.5M-package share) mixes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
run() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 -u $R/bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err
  local rc=$?
  cat $OUT/bench_$name.json; tail -3 $OUT/bench_$name.err
  return $rc
}
run c2 400 ${C2_ARGS:-} && run c3 300 --config c3 --cpu-seconds 5 && run c5 500 --config c5 --cpu-seconds 5 &&
  run c4 600 --config c4 --packages 12500000 --cpu-seconds 5
