#!/bin/bash
# Full-size whole-batch parity (tests/test_gpu_fullsize.py): CONFIG = c5 (20M) or c4share (12.5M).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fullsize
mkdir -p $O
cd $R
TVM_FULLSIZE=1 timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 1100 --timeout-method thread \
  "tests/test_gpu_fullsize.py::test_fullsize_whole_batch_vs_oracle[${CONFIG:-c5}]" > $O/${CONFIG:-c5}.log 2>&1
rc=$?; tail -8 $O/${CONFIG:-c5}.log; exit $rc
