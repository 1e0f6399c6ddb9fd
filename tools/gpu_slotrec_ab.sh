#!/bin/bash
# A/B: slot records at the head of each key's row run + a 4-B entry index (product) vs the
# separate 64-B slot table + fingerprint bytes (libtrivy_amd_exp.so built with
# -DTVM_EXP_OLD_SLOTS, run on the old layout: TVM_SLOT_REC=0), alternated; parity suites first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/slotrec
mkdir -p $O
cd $R
EXP=$R/trivy_amd/libtrivy_amd_exp.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_bench_batch.py > $O/tests_quick.log 2>&1 || { tail -30 $O/tests_quick.log; exit 1; }
tail -1 $O/tests_quick.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_rec_$i.json 2> $O/c2_rec_$i.err || exit 1
  TVM_SLOT_REC=0 TVM_LIB_PATH=$EXP timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_table_$i.json 2> $O/c2_table_$i.err || exit 1
done
timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_rec.json 2> $O/c3_rec.err || exit 1
TVM_SLOT_REC=0 TVM_LIB_PATH=$EXP timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_table.json 2> $O/c3_table.err || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_rec.json 2> $O/c5_rec.err || exit 1
TVM_SLOT_REC=0 TVM_LIB_PATH=$EXP timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_table.json 2> $O/c5_table.err || exit 1
timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 5 --no-cpu --no-e2e --no-fill > $O/c4_rec.json 2> $O/c4_rec.err || exit 1
TVM_SLOT_REC=0 TVM_LIB_PATH=$EXP timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 5 --no-cpu --no-e2e --no-fill > $O/c4_table.json 2> $O/c4_table.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
