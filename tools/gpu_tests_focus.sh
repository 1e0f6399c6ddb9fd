#!/bin/bash
# Focused GPU pass (gpurun): the given test files first, then the whole -m gpu suite + smoke.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_focus.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_focus.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
tail -3 gpurun_out/smoke.log
exit $rc
