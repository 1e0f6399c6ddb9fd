#!/bin/bash
# GPU tests + C3 / C5 bench lines (round 4 kernel changes)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04c}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py --config c3 --no-cpu --no-e2e > $OUT/bench_c3.json 2> $OUT/bench_c3.err
timeout -k 10 500 python bench.py --config c5 --no-cpu --no-e2e --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
python3 - <<'PY'
import json
for c in ("c3", "c5"):
    d = json.load(open(f"gpurun_out/{__import__('os').environ.get('NAME','r04c')}/bench_{c}.json"))
    r = d["roofline"]; f = d.get("fill_info") or {}
    print(c, "kernel_ms %.4f frac %.3f" % (r["kernel_ms"], r["frac"]), "merge", (f.get("redhat_merge") or {}).get("kernel_ms"))
PY
