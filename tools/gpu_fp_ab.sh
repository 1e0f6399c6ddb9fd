#!/bin/bash
# A/B: slot fingerprint walk (product) vs none (libtrivy_amd_exp.so built with -DTVM_EXP_NOFP) on
# C2, C3, C5, alternated; then the parity suites on the product build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fp
mkdir -p $O
cd $R
EXP=$R/trivy_amd/libtrivy_amd_exp.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_parity.py > $O/tests_quick.log 2>&1 || exit 1
tail -1 $O/tests_quick.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_fp_$i.json 2> $O/c2_fp_$i.err || exit 1
  TVM_LIB_PATH=$EXP timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_nofp_$i.json 2> $O/c2_nofp_$i.err || exit 1
done
timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_fp.json 2> $O/c3_fp.err || exit 1
TVM_LIB_PATH=$EXP timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_nofp.json 2> $O/c3_nofp.err || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_fp.json 2> $O/c5_fp.err || exit 1
TVM_LIB_PATH=$EXP timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_nofp.json 2> $O/c5_nofp.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
