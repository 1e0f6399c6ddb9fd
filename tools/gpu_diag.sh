#!/bin/bash
# Match-kernel evidence on the GPU box: SQ/PMC counters of the product kernel, then the
# measurement-only variants (libtrivy_amd_diag.so, built here with `make DIAG=1
# OUT=../libtrivy_amd_diag.so OBJDIR=build_diag`) swapped into the box's scratch copy.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ "${SKIP_PMC:-0}" != "1" ]; then bash tools/pmc_sq.sh; fi
if [ -f trivy_amd/libtrivy_amd_diag.so ]; then
  cp trivy_amd/libtrivy_amd_diag.so trivy_amd/libtrivy_amd.so
  timeout -k 10 300 python3 -u bench.py --config ${CFG:-c2} --no-cpu --no-fill --no-e2e --sweep 3 --steps 10 > gpurun_out/diag_sweep.json 2> gpurun_out/diag_sweep.err
  grep -E "sweep|bench\]" gpurun_out/diag_sweep.err
fi
