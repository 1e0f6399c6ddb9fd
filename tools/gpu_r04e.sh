#!/bin/bash
# GPU tests + C2 (e2e with the delta form) / C3 / C5 bench lines + a C5 kernel-trace summary
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04e}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 500 python bench.py --config c2 --no-cpu > $OUT/bench_c2.json 2> $OUT/bench_c2.err
timeout -k 10 400 python bench.py --config c3 --no-cpu --no-e2e > $OUT/bench_c3.json 2> $OUT/bench_c3.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c5_trace -o run --output-format csv -- python3 bench.py --config c5 --no-cpu --no-e2e --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
f=$(find $OUT/c5_trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" > $OUT/c5_kernel_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print("%6s %10.1f us  %s" % (r.get("Calls"), float(r.get("AverageNs", 0)) / 1e3, r.get("Name", "")[:110]))
PY
cat $OUT/c5_kernel_stats.txt
NAME=${NAME:-r04e} python3 - <<'PY'
import json, os
for c in ("c2", "c3", "c5"):
    d = json.loads([l for l in open(f"gpurun_out/{os.environ['NAME']}/bench_{c}.json") if l.startswith("{")][-1])
    r = d["roofline"]; f = d.get("fill_info") or {}
    print(c, "kernel_ms %.4f frac %.3f value %.3g" % (r["kernel_ms"], r["frac"], d["value"]), "merge", (f.get("redhat_merge") or {}).get("kernel_ms"))
    e = d.get("end_to_end")
    if e:
        print("  e2e", {k: e.get(k) for k in ("packages_per_s", "ms_per_pass", "d2h_bytes", "h2d_bytes", "decode_ms", "packages_per_s_with_decode")})
        print("  csr", e.get("csr_form"))
        print("  fresh", {k: (d.get("fresh_batch") or {}).get(k) for k in ("prepare_ms", "pass_ms", "packages_per_s", "d2h_bytes")})
PY
