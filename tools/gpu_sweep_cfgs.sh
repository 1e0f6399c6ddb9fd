#!/bin/bash
# Variant sweep of the match kernel on the C3 / C5 / C4 workloads (gpurun; no CPU leg).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in ${CFGS:-c5 c4 c3}; do
  extra=""; [ $c = c4 ] && extra="--packages 12500000"
  timeout -k 10 300 python3 -u bench.py --config $c $extra --no-cpu --no-fill --no-e2e --steps 10 --sweep 2 > gpurun_out/sw_$c.json 2> gpurun_out/sw_$c.err || { tail -20 gpurun_out/sw_$c.err; exit 1; }
  echo "== $c"; grep sweep gpurun_out/sw_$c.err
done
