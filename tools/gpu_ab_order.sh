#!/bin/bash
# GPU box: filter / export / mix tests, then C2 / C5 bench lines and C3 with and without the
# heavy-first tile order (TVM_NO_TILE_ORDER=1).  OUT=gpurun_out/$TAG.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_fillinfo.py tests/test_gpu_redhat_chain.py tests/test_gpu_vulns.py \
  tests/test_gpu_mix.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for c in c2 c5 c3; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-e2e > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -30 $OUT/bench_$c.err; exit 1; }
done
TVM_NO_TILE_ORDER=1 timeout -k 10 300 python -u bench.py --config c3 --no-cpu --no-e2e > $OUT/bench_c3_noorder.json 2> $OUT/bench_c3_noorder.err
python - <<'PY'
import json, os
out = os.environ.get("OUT_DIR")
PY
for f in $OUT/bench_*.json; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; fi=d.get('fill_info') or {}
print('$f'.split('/')[-1], 'kernel_ms', round(r['kernel_ms'],4), 'frac', round(r['frac'],3), 'vulns_ms', (d.get('vulns') or {}).get('ms'), 'filter_ms', (fi.get('result_filter') or {}).get('ms'))
"; done
