#!/bin/bash
# End-to-end pass: the unpack kernel on the copy stream (overlapping the previous chunk's match
# launch) and the row ends by the move's own stores, against the default.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-e2e3}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
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
run default TVM_X=0
run unpack_on_copy TVM_PIPE_UNPACK_ON_COPY=1
run rowend_store TVM_PIPE_ROWEND_STORE=1
run both TVM_PIPE_UNPACK_ON_COPY=1 TVM_PIPE_ROWEND_STORE=1
run default2 TVM_X=1
