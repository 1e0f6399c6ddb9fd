#!/bin/bash
# Round 6: row-run alignment + dpkg tail-store skip - parity (dpkg, pipeline, mix), then C2 / C5 kernel times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
  tests/test_gpu_bench_batch.py tests/test_gpu_mix.py tests/test_gpu_golden.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5.json 2> $O/c5.err || exit 1
timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3.json 2> $O/c3.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['roofline']['kernel_ms'], d['config']['kernel_variant'], round(d['roofline']['frac'],3), d['value']/1e9)"; done
echo done
