#!/bin/bash
# Round-end evidence on one GPU box (via gpurun): the GPU test suite, smoke(), then the C2
# profile round (bench + kernel trace + PMC passes incl. SQ / TCC).  Every GPU step has its
# own time limit; the first failure stops the script.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
CONFIG=c2 PMC_EXTRA=1 bash $R/tools/profile_round.sh > $OUT/profile_c2.log 2>&1
tail -3 $OUT/profile_c2.log
