#!/bin/bash
# One GPU box call (gpurun): the GPU test suite (or $TESTS), smoke(), then default bench lines for
# $CONFIGS (no CPU leg).  Every GPU step has its own time limit; the first failure stops the
# script.  OUT=gpurun_out/$TAG.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-validate}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_LIMIT:-780} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
fi
if [ "${SKIP_SMOKE:-0}" != 1 ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
  tail -1 $OUT/smoke.log
fi
for c in ${CONFIGS:-c2}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { tail -30 $OUT/bench_$c.err; exit 1; }
  cat $OUT/bench_$c.json
done
