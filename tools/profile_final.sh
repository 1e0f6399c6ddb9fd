#!/bin/bash
# Round-end counters at the final kernel build: for each config in CONFIGS the kernel trace,
# FETCH_SIZE / WRITE_SIZE and the SQ / TCC passes (tools/profile_kernels.sh, SQ=1), each pass its
# own rocprofv3 run under its own time limit; stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for c in ${CONFIGS:-c2}; do
  EXTRA=""
  if [ "$c" == "c4" ]; then EXTRA="--packages 12500000"; fi
  CONFIG=$c SQ=1 EXTRA="$EXTRA" bash $R/tools/profile_kernels.sh
done
