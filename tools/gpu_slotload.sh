#!/bin/bash
# A/B: the hash index's load factor (TVM_SLOT_LOAD) on C2, C5 and C3, alternated.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/slotload${TAG:-}
mkdir -p $O
cd $R
for i in 1 2; do
  for L in ${LOADS:-0.5 0.75}; do
    TVM_SLOT_LOAD=$L timeout -k 10 200 python bench.py --config c2 --steps 20 --no-cpu --no-e2e --no-fill --no-dropin > $O/c2_${L}_$i.json 2> $O/c2_${L}_$i.err || exit 1
  done
done
for L in ${LOADS:-0.5 0.75}; do
  TVM_SLOT_LOAD=$L timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_$L.json 2> $O/c5_$L.err || exit 1
  TVM_SLOT_LOAD=$L timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_$L.json 2> $O/c3_$L.err || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
