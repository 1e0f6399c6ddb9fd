#!/bin/bash
# GPU tests; C3 with the compacted Maven programs (mixed, Maven-only); C2 end-to-end with the
# faster delta decode (timeline); C5 merge.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04h}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e --sweep 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err
grep -E "sweep\]" $OUT/bench_c3.err || true
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_c3.json') if l.startswith('{')][-1]); print('c3 kernel_ms %.4f' % d['roofline']['kernel_ms'], d['config']['kernel_variant'])"
for pre in 0 0.03 0.3; do
  TVM_BENCH_WEIGHTS=0,1,0,0 TVM_SYNTH_MAVEN_PRE=$pre timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e --no-fill > $OUT/bench_c3_mvn$pre.json 2> $OUT/bench_c3_mvn$pre.err
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_c3_mvn$pre.json') if l.startswith('{')][-1]); print('$pre', d['config']['workload'], d['config']['matches_rank0'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done
TVM_PIPE_NODECODE=1 TVM_PIPE_TRACE=1 timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 8 --warmup 2 > $OUT/bench_c2_nodecode.json 2> $OUT/bench_c2_nodecode.err || true
grep "pipe " $OUT/bench_c2_nodecode.err | tail -14
TVM_PIPE_TRACE=1 timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 8 --warmup 2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
grep "pipe " $OUT/bench_c2.err | tail -14
python3 - $OUT/bench_c2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]
print("c2 kernel_ms %.4f e2e ms %.3f (%.3g/s) d2h %d | csr ms %.3f | fresh prep %.2f pass %.2f (%.3g/s)" % (
    d["roofline"]["kernel_ms"], e["ms_per_pass"], e["packages_per_s"], e["d2h_bytes"], (e.get("csr_form") or {}).get("ms_per_pass", 0),
    f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
PY
