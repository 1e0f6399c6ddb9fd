#!/bin/bash
# End-to-end pass vs hardware queues per process (GPU_MAX_HW_QUEUES: HIP's default 4 maps the
# pipeline's copy and kernel streams onto shared queues once the process has more streams), with
# a kernel + memory-copy trace of the default.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-hwq}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 8 --warmup 2 > $OUT/bench_q$q.json 2> $OUT/bench_q$q.err
  python3 - $OUT/bench_q$q.json $q <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]; o = e.get("other_form") or {}
print("hwq", sys.argv[2], "kernel_ms %.4f e2e ms %.3f (%.3g/s) | delta ms %.3f | fresh prep %.2f pass %.2f (%.3g/s)" % (
    d["roofline"]["kernel_ms"], e["ms_per_pass"], e["packages_per_s"], o.get("ms_per_pass", 0),
    f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
PY
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --config c2 --no-cpu --no-fill --steps 2 --warmup 1 > $OUT/trace.log 2>&1
ls $OUT/trace
