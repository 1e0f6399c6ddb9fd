#!/bin/bash
# Round-end check at HEAD (via gpurun): the GPU test suite, smoke(), the default bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final2
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json
