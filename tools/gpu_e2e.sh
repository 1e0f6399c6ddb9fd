#!/bin/bash
# End-to-end pass: the row ends by DMA vs by the result move's stores; chunk sizes; a kernel
# trace of the default (kernel gaps = waits on uploads).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-e2e}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --config c2 --no-cpu --no-fill --steps 8 --warmup 2 > $OUT/$name.json 2> $OUT/$name.err
  python3 - $OUT/$name.json $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["end_to_end"]; f = d["fresh_batch"]
print(sys.argv[2], "e2e ms %.3f (%.3g/s) chunks %s | fresh pass %.2f" % (e["ms_per_pass"], e["packages_per_s"], e["chunks"], f["pass_ms"]))
PY
}
run default TVM_X=0
run rowend_store TVM_PIPE_ROWEND_STORE=1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/ktrace -o run --output-format csv -- python3 $R/bench.py --config c2 --no-cpu --no-fill --steps 2 --warmup 1 > $OUT/ktrace.log 2>&1
f=$(find $OUT/ktrace -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/e2e_kernels.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last pipelined pass: from the last unpack_kernel burst backwards
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "unpack_kernel" in n]
if idx:
    start = idx[-1]
    while start > 0 and ("unpack_kernel" in names[start - 1] or "fused_kernel" in names[start - 1]) and start > idx[-1] - 20:
        start -= 1
    t0 = int(rows[start]["Start_Timestamp"])
    for r in rows[start:start + 30]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print("%9.1f %9.1f %8.1f  %s grid %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X", ""))))
PY
cat $OUT/e2e_kernels.txt
