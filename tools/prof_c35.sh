set -euo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
CONFIG=c5 SQ=1 bash tools/profile_r04.sh > gpurun_out/prof_c5.log 2>&1
CONFIG=c3 SQ=1 bash tools/profile_r04.sh > gpurun_out/prof_c3.log 2>&1
timeout -k 10 400 python3 bench.py --config c5 --steps 10 --no-cpu > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
tail -c 1500 gpurun_out/bench_c5.json
