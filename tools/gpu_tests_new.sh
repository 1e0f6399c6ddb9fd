#!/bin/bash
# Round 6: the new / changed GPU tests in one process (per-test timeouts).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06t
mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_spill.py \
  tests/test_gpu_bulk_add.py tests/test_gpu_pipeline_mix.py tests/test_gpu_pipeline.py tests/test_gpu_vulns.py \
  > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 $O/tests.log
exit $rc
