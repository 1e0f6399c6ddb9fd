#!/bin/bash
# End-to-end pass with the wave-per-tile result move: pipeline GPU tests, then the move width
# (TVM_COPY_WG) and the round-3 workgroup-per-tile move (TVM_COPY_BLOCK) on the same box, and
# a kernel trace of the default.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-e2e2}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_bench_dist.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 8 --warmup 2 > $OUT/$name.json 2> $OUT/$name.err
  python3 - $OUT/$name.json $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]
print(sys.argv[2], "e2e ms %.3f (%.3g/s) | delta %.3f | fresh prep %.2f pass %.2f (%.3g/s)" % (e["ms_per_pass"], e["packages_per_s"],
      (e.get("other_form") or {}).get("ms_per_pass", 0), f["prepare_ms"], f["pass_ms"], f["packages_per_s"]))
PY
}
run wave64 TVM_X=0
run block64 TVM_COPY_BLOCK=1
run wave32 TVM_COPY_WG=32
run wave128 TVM_COPY_WG=128
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/ktrace -o run --output-format csv -- python3 $R/bench.py --config c2 --no-cpu --no-fill --steps 2 --warmup 1 > $OUT/ktrace.log 2>&1
f=$(find $OUT/ktrace -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/e2e_kernels.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "unpack_kernel" in n]
if idx:
    start = idx[-1]
    while start > 0 and ("unpack_kernel" in names[start - 1] or "fused_kernel" in names[start - 1]) and start > idx[-1] - 20:
        start -= 1
    t0 = int(rows[start]["Start_Timestamp"])
    for r in rows[start:start + 16]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print("%9.1f %9.1f %8.1f  %s grid %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X", ""))))
PY
cat $OUT/e2e_kernels.txt
