#!/bin/bash
# A/B on C2: the dpkg kernel's next-slot head prefetch only within the home slot's 128-B line
# (product) vs always (libtrivy_amd_exp.so built with -DTVM_EXP_Q0N_ALWAYS), alternated.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/q0n
mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_line_$i.json 2> $O/c2_line_$i.err || exit 1
  TVM_LIB_PATH=$R/trivy_amd/libtrivy_amd_exp.so timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_always_$i.json 2> $O/c2_always_$i.err || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_bench_batch.py > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log
