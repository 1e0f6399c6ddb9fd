#!/bin/bash
# Round 6: inline rpm row filters + the two-stream lean / full split: parity tests, then
# C3 (split vs TVM_NO_LEAN), C4 share and C5 benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_mix.py \
  tests/test_gpu_golden.py tests/test_gpu_redhat_chain.py tests/test_gpu_vulns.py tests/test_gpu_fillinfo.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_$i.json 2> $O/c3_$i.err || exit 1
TVM_NO_LEAN=1 timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_nolean_$i.json 2> $O/c3_nolean_$i.err || exit 1
done
timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 10 --no-cpu --no-e2e --no-fill > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 400 python bench.py --config c5 --steps 10 --no-cpu > $O/c5.json 2> $O/c5.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['roofline']['kernel_ms'], d['config']['kernel_variant'], round(d['roofline']['frac'],3))"; done
echo done
