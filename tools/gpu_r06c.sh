#!/bin/bash
# Round 6: the lean / split launch - mix parity + variant agreement, then C3 / C4 share / C5 benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_mix.py tests/test_gpu_library.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu > $O/c3.json 2> $O/c3.err || exit 1
TVM_NO_LEAN=1 timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_nolean.json 2> $O/c3_nolean.err || exit 1
timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 10 --no-cpu --no-e2e --no-fill > $O/c4.json 2> $O/c4.err || exit 1
TVM_NO_LEAN=1 timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 10 --no-cpu --no-e2e --no-fill > $O/c4_nolean.json 2> $O/c4_nolean.err || exit 1
timeout -k 10 400 python bench.py --config c5 --steps 10 --cpu-seconds 4 > $O/c5.json 2> $O/c5.err || exit 1
# measurement only: every row filter passing (libtrivy_amd_exp.so, TVM_EXP_NOAUX) - the filters' share of C5
TVM_LIB_PATH=$R/trivy_amd/libtrivy_amd_exp.so timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_noaux.json 2> $O/c5_noaux.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['roofline']['kernel_ms'], d['config']['kernel_variant'], round(d['roofline']['frac'],3))"; done
echo done
