#!/bin/bash
# PC sampling (host trap) of the C2 match kernel: instruction-level hot spots.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
rocprofv3 --help 2>&1 | grep -i "pc-sampl" > gpurun_out/pcs/help.txt || true
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL:-1} -d $R/gpurun_out/pcs -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 1 --no-cpu --no-fill --no-e2e > gpurun_out/pcs/log 2>&1
rc=$?
tail -5 gpurun_out/pcs/log
find gpurun_out/pcs -type f | head -20
exit $rc
