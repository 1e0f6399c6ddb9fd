#!/bin/bash
# GPU tests, then a variant sweep of each workload (run on the GPU box via gpurun).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
for c in ${CONFIGS:-c2 c5 c3}; do
  timeout -k 10 300 python -u bench.py --config $c --sweep 3 --no-cpu > gpurun_out/sw_$c.json 2> gpurun_out/sw_$c.err || { tail -20 gpurun_out/sw_$c.err; exit 1; }
  grep sweep gpurun_out/sw_$c.err | grep -v ablate
done
