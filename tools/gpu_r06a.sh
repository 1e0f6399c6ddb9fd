#!/bin/bash
# Round 6 first GPU call: the new GPU tests, the FETCH calibration, a quick C2 / C5 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06a
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_spill.py \
  tests/test_gpu_bulk_add.py tests/test_gpu_pipeline_mix.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -le 1 ] || exit $rc
bash tools/calib_run.sh > $O/calib.log 2>&1 || { echo "calib rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --config c2 --steps 20 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 rc=$?"; exit 1; }
timeout -k 10 400 python -u bench.py --config c5 --steps 10 --cpu-seconds 4 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 rc=$?"; exit 1; }
echo all done
