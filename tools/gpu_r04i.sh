#!/bin/bash
# GPU tests; C5 Red Hat merge kernels; C2 line (end-to-end in both result forms); the cost split
# (diag variants) of Maven-only and npm-only C3 batches.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04i}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c5_trace -o run --output-format csv -- python3 bench.py --config c5 --no-cpu --no-e2e --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
f=$(find $OUT/c5_trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" > $OUT/c5_kernel_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print("%6s %10.1f us  %s" % (r.get("Calls"), float(r.get("AverageNs", 0)) / 1e3, r.get("Name", "")[:110]))
PY
grep -E "rh_|scan" $OUT/c5_kernel_stats.txt || true
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_c5.json') if l.startswith('{')][-1]); print('c5 merge', d['fill_info']['redhat_merge']['kernel_ms'])"
timeout -k 10 500 python bench.py --config c2 --no-cpu > $OUT/bench_c2.json 2> $OUT/bench_c2.err
python3 - $OUT/bench_c2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]; o = e.get("other_form") or {}
print("c2 kernel_ms %.4f e2e %s ms %.3f (%.3g/s) d2h %d | other %s ms %.3f d2h %s | fresh prep %.2f pass %.2f (%.3g/s)" % (
    d["roofline"]["kernel_ms"], e["result_form"], e["ms_per_pass"], e["packages_per_s"], e["d2h_bytes"], o.get("result_form"),
    o.get("ms_per_pass", 0), o.get("d2h_bytes"), f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
PY
if [ -f trivy_amd/libtrivy_amd_diag.so ]; then
  cp trivy_amd/libtrivy_amd_diag.so trivy_amd/libtrivy_amd.so
  for w in 0,1,0,0 0,0,1,0; do
    TVM_BENCH_WEIGHTS=$w TVM_SYNTH_MAVEN_PRE=0 timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu --no-fill --no-e2e --sweep 3 --steps 10 > $OUT/diag_c3_w$w.json 2> $OUT/diag_c3_w$w.err
    echo "== $w"; grep -E "sweep\]" $OUT/diag_c3_w$w.err || true
  done
fi
