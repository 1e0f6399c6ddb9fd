#!/bin/bash
# Round 6 A/B: C3 without Maven (go / npm / PEP 440) on the lean kernel (GM_LEAN) vs the
# all-grammar kernel (TVM_NO_LEAN=1), alternated; then the lean kernel's variant sweep.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lean_ab
mkdir -p $O
cd $R
for i in 1 2; do
  TVM_BENCH_WEIGHTS=15,0,40,25 timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/lean_$i.json 2> $O/lean_$i.err
  TVM_NO_LEAN=1 TVM_BENCH_WEIGHTS=15,0,40,25 timeout -k 10 200 python bench.py --config c3 --steps 20 --no-cpu --no-e2e > $O/all_$i.json 2> $O/all_$i.err
done
TVM_BENCH_WEIGHTS=15,0,40,25 timeout -k 10 300 python bench.py --config c3 --steps 10 --no-cpu --no-e2e --sweep 5 > $O/sweep.json 2> $O/sweep.err
for f in $O/*.json; do echo "$f $(python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['roofline']['kernel_ms'], d['config']['kernel_variant'])")"; done
grep sweep $O/sweep.err
