#!/bin/bash
# Round 6: class-0 row lists for library keys (SLOT_CLS_SPLIT) - library / mix / vulns parity,
# then C3 per ecosystem and whole.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_library.py tests/test_gpu_mix.py \
  tests/test_gpu_parity.py "tests/test_gpu_vulns.py::test_vulns_whole_batch_vs_oracle[c3]" "tests/test_gpu_vulns.py::test_vulns_whole_batch_vs_oracle[c4]" \
  "tests/test_gpu_pipeline_mix.py::test_pipeline_whole_batch_vs_oracle[c3]" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -le 1 ] || exit $rc
for w in 0,0,0,1 0,0,1,0; do
  TVM_BENCH_WEIGHTS=$w timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_w$w.json 2> $O/c3_w$w.err || exit 1
done
timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 10 --no-cpu --no-e2e --no-fill > $O/c4.json 2> $O/c4.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['roofline']['kernel_ms'], d['config']['kernel_variant'], round(d['roofline']['frac'],3))"; done
echo done
