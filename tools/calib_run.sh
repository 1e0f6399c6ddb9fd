#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the match kernel's load / store shapes (GPU box):
# tools/calib_fetch (built here by hipcc) under a kernel trace and one --pmc pass per counter
# group; tools/calib_summary.py turns the per-kernel counters into factors = counted / true bytes.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/calib
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B=$R/tools/calib_fetch
timeout -k 10 120 $B > $OUT/bytes.csv
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/rdreq -o run --output-format csv -- $B > $OUT/rdreq.log 2>&1 || echo "rdreq pass failed: $?"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list failed: $?"
echo calib done
