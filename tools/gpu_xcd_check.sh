#!/bin/bash
# XCD-affine order restricted to the all-grammar kernel: C3 default vs TVM_TILE_ORDER=w, C2 / C5
# default (must be unchanged), then the library parity suites.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/xcd2
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_xcd_$i.json 2> $O/c3_xcd_$i.err || exit 1
  TVM_TILE_ORDER=w timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_w_$i.json 2> $O/c3_w_$i.err || exit 1
done
timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5.json 2> $O/c5.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_mix.py tests/test_gpu_vulns.py tests/test_gpu_library.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
