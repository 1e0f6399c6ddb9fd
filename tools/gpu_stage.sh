#!/bin/bash
# Raw-form staging per chunk inside the pass: pipeline GPU tests, then the C2 line's fresh-batch leg.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-stage}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_bench_batch.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
for i in 1 2; do
  timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 8 --warmup 2 > $OUT/bench_$i.json 2> $OUT/bench_$i.err
  python3 - $OUT/bench_$i.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]
print("e2e ms %.3f | fresh prep %.2f pass %.2f (%.3g/s)" % (e["ms_per_pass"], f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
PY
done
