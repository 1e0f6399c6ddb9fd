"""GPU: `python bench.py --gpus 2` really runs two ranks (bench.py launches them itself through
torch.distributed.run when WORLD_SIZE is unset).  Weak scaling (the default): every rank
matches its own batch of the config and the line counts both; its lists equal the oracle's.
--gather (strong scaling), and the `strong` object the default line carries at N > 1: the
per-package advisory lists the timed step gathers at rank 0 equal the oracle's match of the
whole global batch (oracle/match.c), element for element, in batch order.  Both ranks share the one MI355X of the box, so the collectives run over gloo
(TVM_BENCH_BACKEND=gloo; RCCL refuses two ranks on one device)."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gather", [True, False])
def test_bench_two_ranks_csr_equals_oracle(tmp_path, oracle_built, gather):
    sys.path.insert(0, ROOT)
    import bench
    from oracle import match as om
    dump = str(tmp_path / "csr.npz")
    flags = ["--config", "c2", "--keys-per-plat", "3000", "--targets", "200", "--pkgs-per-target", "400"]
    env = dict(os.environ, TVM_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu", "--no-e2e", "--no-fill", "--dump-csr", dump] + flags + (["--gather"] if gather else []),
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["packages"] == 200 * 400
    if gather:  # rank 0 matched a shard only; the step's packages are the global batch
        assert line["scaling"] == "strong" and line["config"]["packages_rank0"] < line["config"]["packages"]
        assert line["config"]["packages_per_step"] == 200 * 400
    else:  # every rank matched the whole batch of the config; the strong object: one global batch
        assert line["scaling"] == "weak" and line["config"]["packages_rank0"] == 200 * 400
        assert line["config"]["packages_per_step"] == 2 * 200 * 400
        st = line["strong"]
        assert st["packages"] == 200 * 400 and 0 < st["packages_rank0"] < 200 * 400 and st["gather_ms"] > 0
    wl = bench.C2(argparse.Namespace(keys_per_plat=3000, targets=200, pkgs_per_target=400))
    opk, oad = om.match(om.Prepared(wl.sdb, wl.batch), n_threads=8)
    want_end = np.cumsum(np.bincount(opk, minlength=wl.n)).astype(np.uint32)
    for path in [dump] + ([] if gather else [dump.replace(".npz", "_strong.npz")]):
        got = np.load(path)
        assert int(got["n_gpus"]) == 2
        assert np.array_equal(got["adv"], oad.astype(np.uint32)), path
        assert np.array_equal(got["row_end"], want_end), path
