"""GPU: the multi-GPU path on one box - two ranks share the one MI355X (gloo collectives;
RCCL refuses two ranks on one device), each matches its shard of ONE global batch
(target-boundary shards balanced by predicted rows), orders it into per-package lists (CSR)
on the device, and the CSR gather brings them to rank 0 in batch order, where they equal the
oracle's match of the whole batch without a sort (tests/dist_worker.py)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_two_ranks_gather_equals_single_rank():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tests", "dist_worker.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "DIST OK 2 ranks" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
