#!/bin/bash
# GPU tests; C3 mixed + Maven-only (the parse only where a program row admits the class);
# C4; C2 line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04l}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e > $OUT/bench_c3.json 2> $OUT/bench_c3.err
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_c3.json') if l.startswith('{')][-1]); print('c3 kernel_ms %.4f' % d['roofline']['kernel_ms'], d['config']['kernel_variant'])"
for pre in 0 0.03; do
  TVM_BENCH_WEIGHTS=0,1,0,0 TVM_SYNTH_MAVEN_PRE=$pre timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e --no-fill > $OUT/bench_c3_mvn$pre.json 2> $OUT/bench_c3_mvn$pre.err
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_c3_mvn$pre.json') if l.startswith('{')][-1]); print('$pre', d['config']['workload'], d['config']['matches_rank0'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done
timeout -k 10 500 python bench.py --config c4 --no-cpu --no-e2e --packages 12500000 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_c4.json') if l.startswith('{')][-1]); print('c4 kernel_ms %.4f' % d['roofline']['kernel_ms'], d['config']['workload'])"
timeout -k 10 500 python bench.py --config c2 --no-cpu > $OUT/bench_c2.json 2> $OUT/bench_c2.err
python3 - $OUT/bench_c2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]; o = e.get("other_form") or {}
print("c2 kernel_ms %.4f e2e %s ms %.3f (%.3g/s) | other ms %.3f | fresh prep %.2f pass %.2f (%.3g/s)" % (
    d["roofline"]["kernel_ms"], e["result_form"], e["ms_per_pass"], e["packages_per_s"], o.get("ms_per_pass", 0),
    f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
PY
