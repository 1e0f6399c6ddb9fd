#!/bin/bash
# GPU tests + C3 / C5 bench lines + the C2 variant sweep + the host SBOM decode rate (round 4)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r04c}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py --config c3 --no-cpu --no-e2e > $OUT/bench_c3.json 2> $OUT/bench_c3.err
timeout -k 10 600 python bench.py --config c5 --no-cpu --no-e2e --steps 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
timeout -k 10 400 python bench.py --config c2 --no-cpu --no-e2e --no-fill --sweep 4 > $OUT/sweep_c2.json 2> $OUT/sweep_c2.err
grep sweep $OUT/sweep_c2.err || true
timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 10 > $OUT/bench_c2_e2e.json 2> $OUT/bench_c2_e2e.err
TVM_PIPE_NORAMP=1 timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 10 > $OUT/bench_c2_e2e_noramp.json 2> $OUT/bench_c2_e2e_noramp.err
timeout -k 10 300 python tools/sbom_rate.py 1000000 > $OUT/sbom_rate.txt 2>&1
cat $OUT/sbom_rate.txt
NAME=${NAME:-r04c} python3 - <<'PY'
import json, os
for c in ("c3", "c5"):
    d = json.load(open(f"gpurun_out/{os.environ['NAME']}/bench_{c}.json"))
    r = d["roofline"]; f = d.get("fill_info") or {}
    print(c, "kernel_ms %.4f frac %.3f" % (r["kernel_ms"], r["frac"]), "merge", (f.get("redhat_merge") or {}).get("kernel_ms"))
for n in ("bench_c2_e2e", "bench_c2_e2e_noramp"):
    d = json.load(open(f"gpurun_out/{os.environ['NAME']}/{n}.json"))
    e, fb = d["end_to_end"], d["fresh_batch"]
    print(n, "e2e %.3f ms %.3g pkg/s chunks %d; fresh prepare %.2f pass %.2f ms %.3g pkg/s" % (
        e["ms_per_pass"], e["packages_per_s"], e["chunks"], fb["prepare_ms"], fb["pass_ms"], fb["packages_per_s"]))
PY
