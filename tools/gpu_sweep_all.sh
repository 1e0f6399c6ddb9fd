#!/bin/bash
# Variant sweep of every config at the current table layout (which variant Engine picks vs the rest).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sweep8
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --config c2 --steps 10 --no-cpu --no-e2e --no-fill --sweep 4 > $O/c2.json 2> $O/c2.err || exit 1
grep sweep $O/c2.err
timeout -k 10 400 python bench.py --config c5 --steps 5 --no-cpu --no-e2e --no-fill --sweep 3 > $O/c5.json 2> $O/c5.err || exit 1
grep sweep $O/c5.err
timeout -k 10 400 python bench.py --config c4 --packages 12500000 --steps 5 --no-cpu --no-e2e --no-fill --sweep 3 > $O/c4.json 2> $O/c4.err || exit 1
grep sweep $O/c4.err
