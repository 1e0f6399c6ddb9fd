#!/bin/bash
# Red Hat merge: its GPU tests, then C5 (merge time) twice on the same box.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-rh}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_redhat_chain.py tests/test_gpu_mix.py tests/test_gpu_fillinfo.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py --config c5 --no-cpu --no-e2e --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_c5.json') if l.startswith('{')][-1]); f=d['fill_info']; print('c5 kernel_ms %.4f merge %.4f filter %.4f' % (d['roofline']['kernel_ms'], f['redhat_merge']['kernel_ms'], f['result_filter']['ms']))"
