#!/bin/bash
# A/B: XCD-affine runs for the lean launch of a split all-grammar batch (C4's share) vs without
# (TVM_XCD_SPLIT=0), alternated; then the mixed parity suite.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/xcd4
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 5 --no-cpu --no-e2e --no-fill > $O/c4_xcd_$i.json 2> $O/c4_xcd_$i.err || exit 1
  TVM_XCD_SPLIT=0 timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 5 --no-cpu --no-e2e --no-fill > $O/c4_w_$i.json 2> $O/c4_w_$i.err || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_mix.py tests/test_gpu_vulns.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
