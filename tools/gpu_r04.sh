#!/bin/bash
# Round-4 GPU pass (via gpurun): the GPU suite with the per-test device drain (verbose, so a
# faulting test is named), smoke(), then the default bench line.  OUT=gpurun_out/<name>.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
  tail -1 $OUT/bench.json
fi
