#!/bin/bash
# The whole GPU suite in one process (the driver's round-end tier), then smoke() and the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/full
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
