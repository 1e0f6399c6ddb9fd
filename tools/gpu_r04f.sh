#!/bin/bash
# GPU tests; C5 (Red Hat merge); C2 end-to-end with the delta form at three result-move
# widths; C3 cost split (one ecosystem at a time, then the diag variants).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04f}
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
for wg in 64 128 256; do
  TVM_COPY_WG_DELTA=$wg timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill > $OUT/bench_c2_wg$wg.json 2> $OUT/bench_c2_wg$wg.err
  python3 - $OUT/bench_c2_wg$wg.json $wg <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]
print("wg", sys.argv[2], "e2e ms %.3f (%.3g/s) d2h %d | csr ms %.3f | fresh prep %.2f pass %.2f (%.3g/s)" % (
    e["ms_per_pass"], e["packages_per_s"], e["d2h_bytes"], (e.get("csr_form") or {}).get("ms_per_pass", 0),
    f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
PY
done
for w in 1,0,0,0 0,1,0,0 0,0,1,0 0,0,0,1; do
  TVM_BENCH_WEIGHTS=$w timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e --no-fill > $OUT/bench_c3_w$w.json 2> $OUT/bench_c3_w$w.err
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_c3_w$w.json') if l.startswith('{')][-1]); print('$w', d['config']['workload'], d['config']['matches_rank0'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done
if [ -f trivy_amd/libtrivy_amd_diag.so ]; then
  cp trivy_amd/libtrivy_amd_diag.so trivy_amd/libtrivy_amd.so
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu --no-fill --no-e2e --sweep 3 --steps 10 > $OUT/diag_sweep_c3.json 2> $OUT/diag_sweep_c3.err
  grep -E "sweep\]" $OUT/diag_sweep_c3.err || true
fi
