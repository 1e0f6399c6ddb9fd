#!/bin/bash
# GPU pass (run on the GPU box via gpurun): pytest -m gpu, smoke(), then a short bench.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
if [ "${SMOKE:-1}" == "1" ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" == "1" ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cat gpurun_out/bench.json; tail -15 gpurun_out/bench.err; exit $rc
fi
