#!/bin/bash
# Filter-kernel check (gpurun): the filter GPU tests, then a kernel trace of the C2 bench
# (no CPU leg) into gpurun_out/fprof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "filter or vex or fill" > gpurun_out/pytest_filter.log 2>&1 || { tail -40 gpurun_out/pytest_filter.log; exit 1; }
tail -2 gpurun_out/pytest_filter.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fprof -o run -- python3 $R/bench.py --no-cpu --steps 5 > $R/gpurun_out/fb.json 2> $R/gpurun_out/fb.err || { tail -20 $R/gpurun_out/fb.err; exit 1; }
