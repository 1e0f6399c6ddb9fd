cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for d in 0 1 2 3; do TVM_PROBE_DIAG=$d timeout -k 10 200 python3 bench.py --no-cpu --no-fill --steps 10 > gpurun_out/d$d.json 2>gpurun_out/d$d.err; python3 -c "import json;d=json.load(open('gpurun_out/d$d.json'));print($d, d['ms_per_step'])"; done
export TMPDIR=/tmp; mkdir -p gpurun_out/kt2 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-fill > gpurun_out/kt2/log 2>&1
