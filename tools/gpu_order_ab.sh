#!/bin/bash
# A/B: tile order of an unsplit all-grammar launch (C3): TVM_TILE_ORDER = lean (the round-6
# order: tiles without Maven / RubyGems first), w (heaviest first across both), full (the
# all-grammar tiles first), alternated.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/order
mkdir -p $O
cd $R
for i in 1 2; do
  for m in lean w full; do
    TVM_TILE_ORDER=$m timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/c3_${m}_$i.json 2> $O/c3_${m}_$i.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"; done
