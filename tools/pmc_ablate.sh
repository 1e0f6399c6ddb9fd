#!/bin/bash
# Per-phase instruction mix of the match kernel (run on the GPU box via gpurun): one
# rocprofv3 --pmc pass of SQ counters per kernel variant (incl. the ablation variants),
# then a per-wave table.  Usage: VARIANTS="6 11 12 13 14" CONFIG=c2 bash tools/pmc_ablate.sh
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ablate
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in ${VARIANTS:-6 11 12 13 14}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $OUT/v$v -o run --output-format csv -- \
    python3 $R/bench.py --config ${CONFIG:-c2} --variant $v --steps 3 --warmup 1 --no-cpu > $OUT/v$v.log 2>&1
done
python3 - $OUT <<'PY'
import csv, glob, os, statistics, sys
out = sys.argv[1]
cols = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY"]
print("variant".ljust(40) + "".join(c.replace("SQ_INSTS_", "").replace("SQ_", "")[:10].rjust(11) for c in cols) + "  (per wave)")
for d in sorted(glob.glob(os.path.join(out, "v*"))):
    if not os.path.isdir(d):
        continue
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        vals, name = {}, ""
        for r in csv.DictReader(open(f)):
            if "match_kernel" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        if not vals:
            continue
        m = {k: statistics.median(v) for k, v in vals.items()}
        w = m.get("SQ_WAVES", 1) or 1
        short = name.split("match_kernel<")[-1].split(">")[0]
        print((os.path.basename(d) + " " + short)[:40].ljust(40) + "".join(f"{m.get(c, 0) / w:11.0f}" for c in cols))
PY
