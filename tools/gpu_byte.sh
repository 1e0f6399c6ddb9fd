#!/bin/bash
# The byte result form: pipeline GPU tests (all forms), then the C2 line with the end-to-end
# pass in each form (headline csr / byte), with the pipeline timeline of the byte form.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-byte}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
for form in csr byte; do
  TVM_PIPE_TRACE=$([ $form == byte ] && echo 1 || echo "") timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 8 --warmup 2 --e2e-form $form > $OUT/bench_$form.json 2> $OUT/bench_$form.err
  python3 - $OUT/bench_$form.json $form <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]
print(sys.argv[2], "e2e ms %.3f (%.3g/s) d2h %d | fresh prep %.2f pass %.2f (%.3g/s)" % (e["ms_per_pass"], e["packages_per_s"], e["d2h_bytes"],
      f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
for o in e.get("other_forms", []):
    print("   other", o["result_form"], "ms %.3f d2h %d" % (o["ms_per_pass"], o["d2h_bytes"]))
PY
done
grep "pipe " $OUT/bench_byte.err | tail -16
