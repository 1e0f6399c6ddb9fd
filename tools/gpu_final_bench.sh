#!/bin/bash
# Round 6 final lines: the default bench (the driver's command) and C4 at its full 100M packages on one GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu --no-e2e --no-fill > $O/bench_c4_100m.json 2> $O/bench_c4_100m.err || exit 1
timeout -k 10 400 python bench.py --config c3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 400 python bench.py --config c5 --steps 10 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
for f in $O/bench_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3), d['roofline']['traffic'])"; done
timeout -k 10 400 python bench.py --config c3 --steps 10 --no-cpu --no-e2e --sweep 4 > $O/sweep_c3.json 2> $O/sweep_c3.err || exit 1
grep sweep $O/sweep_c3.err
