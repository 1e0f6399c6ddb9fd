#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats, CSV) of the C2 bench (match + FillInfo +
# filter kernels) and the C4 bench at HEAD, into gpurun_out/trace_c2, trace_c4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_c2 -o run -- python3 $R/bench.py --no-cpu --steps 10 > $R/gpurun_out/trace_c2.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_c4 -o run -- python3 $R/bench.py --config c4 --packages 12500000 --no-cpu --no-e2e --steps 10 > $R/gpurun_out/trace_c4.log 2>&1
