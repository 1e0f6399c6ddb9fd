#!/bin/bash
# A/B of two builds of the library on one box (ab/lib_old.so vs ab/lib_new.so): GPU tests of the
# new build, then per config the kernel trace of a short bench for each build, alternating.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-ab}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
cp ab/lib_new.so trivy_amd/libtrivy_amd.so
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_fillinfo.py tests/test_gpu_golden.py tests/test_gpu_mix.py tests/test_gpu_redhat_chain.py} -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
for cfg in ${CONFIGS:-c2 c5}; do
  for v in new old new old; do
    cp ab/lib_$v.so trivy_amd/libtrivy_amd.so
    d=$OUT/${cfg}_$v
    rm -rf $d
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu --no-e2e --steps 10 > $d.json 2> $d.err
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$cfg $v" "${KPAT:-filter}" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], " ".join("%s=%.1f" % (r["Name"].split("(")[0].split("::")[-1][:24], float(r["AverageNs"]) / 1e3) for r in rows if sys.argv[3] in r["Name"]))
PY
  done
done
cp ab/lib_new.so trivy_amd/libtrivy_amd.so
