#!/bin/bash
# Round 6: the sequential lean / full split with its threshold - mix tests, C3 per ecosystem,
# C3 / C4 share / C5 kernel times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06e
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_mix.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -le 1 ] || exit $rc
for w in 1,0,0,0 0,1,0,0 0,0,1,0 0,0,0,1; do
  TVM_BENCH_WEIGHTS=$w timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_w$w.json 2> $O/c3_w$w.err || exit 1
done
timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 10 --no-cpu --no-e2e --no-fill > $O/c4.json 2> $O/c4.err || exit 1
TVM_NO_LEAN=1 timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 10 --no-cpu --no-e2e --no-fill > $O/c4_nolean.json 2> $O/c4_nolean.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['roofline']['kernel_ms'], d['config']['kernel_variant'], round(d['roofline']['frac'],3))"; done
echo done
