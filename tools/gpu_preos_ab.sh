#!/bin/bash
# A/B: the OS and lean kernels load slot heads before the encoder
# (libtrivy_amd_exp.so) vs the product build, alternated.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/preos
mkdir -p $O
cd $R
EXP=$R/trivy_amd/libtrivy_amd_exp.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_base_$i.json 2> $O/c5_base_$i.err || exit 1
  TVM_LIB_PATH=$EXP timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_preos_$i.json 2> $O/c5_preos_$i.err || exit 1
done
timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 5 --no-cpu --no-e2e --no-fill > $O/c4_base.json 2> $O/c4_base.err || exit 1
TVM_LIB_PATH=$EXP timeout -k 10 300 python bench.py --config c4 --packages 12500000 --steps 5 --no-cpu --no-e2e --no-fill > $O/c4_preos.json 2> $O/c4_preos.err || exit 1
timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_base.json 2> $O/c2_base.err || exit 1
TVM_LIB_PATH=$EXP timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_preos.json 2> $O/c2_preos.err || exit 1
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
