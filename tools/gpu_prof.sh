#!/bin/bash
# Round 6: bench + rocprofv3 evidence (trace, FETCH, WRITE, request sizes; SQ / TCC with
# PMC_EXTRA=1) for the configs named in CONFIGS, optionally the FETCH calibration first (CALIB=1).
# Each step has its own time limit; the first failure ends the call.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
if [ "${CALIB:-0}" == "1" ]; then bash tools/calib_run.sh; fi
for c in ${CONFIGS:-c2}; do
  case $c in
    c4) EXTRA="--packages 12500000" ;;
    *) EXTRA="" ;;
  esac
  CONFIG=$c EXTRA="$EXTRA" STEPS=${STEPS:-20} bash tools/profile_round.sh > gpurun_out/prof_$c.log 2>&1
  tail -3 gpurun_out/prof_$c.log
done
echo prof done
