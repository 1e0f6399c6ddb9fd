#!/bin/bash
# A/B: C5's tile order - heaviest first (default) vs the batch's own order (TVM_NO_TILE_ORDER=1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5order
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_w_$i.json 2> $O/c5_w_$i.err || exit 1
  TVM_NO_TILE_ORDER=1 timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu --no-e2e --no-fill > $O/c5_nat_$i.json 2> $O/c5_nat_$i.err || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
