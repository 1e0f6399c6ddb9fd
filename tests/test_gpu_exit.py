"""GPU: a whole bench run (device-resident pass, DetectedVulnerability export, end-to-end and
fresh-batch pipelined passes, FillInfo / result.Filter legs) exits cleanly.  Round 4 saw a
SIGSEGV inside __cxa_finalize after bench.py printed its line (static teardown racing the
HIP runtime's); the library now drains its queues, joins its worker threads and frees its
cached blocks in tvm_shutdown, which the Python binding registers with atexit."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_bench_run_exits_cleanly():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c2", "--keys-per-plat", "3000",
                        "--targets", "200", "--pkgs-per-target", "400", "--steps", "2", "--warmup", "1", "--no-cpu"],
                       cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["end_to_end"]["vulns_ms"] is not None and line["fresh_batch"]["pass_ms"] > 0
    assert line["vulns"]["detected_vulnerabilities"] == line["config"]["matches_rank0"]
    assert "fill_info" in line
