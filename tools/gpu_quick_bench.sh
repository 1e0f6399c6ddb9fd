#!/bin/bash
# GPU box: kernel-only bench lines (no CPU / e2e / FillInfo legs) for the configs in $CONFIGS and,
# with $MVN=1, the Maven-only C3 batch; prints config, kernel ms, roofline fraction, variant.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-quick}
mkdir -p $OUT
cd $R
if [ "${MVN:-0}" == 1 ]; then
  TVM_BENCH_WEIGHTS=0,1,0,0 timeout -k 10 300 python -u bench.py --config c3 --no-cpu --no-e2e --no-fill > $OUT/mvn.json 2> $OUT/mvn.err
fi
for c in ${CONFIGS:-c3}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-e2e --no-fill ${BENCH_ARGS:-} > $OUT/$c.json 2> $OUT/$c.err
done
for f in $OUT/*.json; do
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']
print(sys.argv[1].split('/')[-1], round(r['kernel_ms'], 4), round(r['frac'], 3), d['config']['kernel_variant'], round(d['value'] / 1e9, 3))" $f
done
