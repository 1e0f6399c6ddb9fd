"""The exact bench workload (bench.py C2: 10k Debian/Ubuntu targets x 400 packages = 4M
packages, 1.7M advisories) matched on the GPU equals the oracle's C restatement
(oracle/match.c, the Debian/Ubuntu driver loops) pair for pair - the full-size parity
check of the headline measurement (bench.py itself never imports the oracle outside its
cpu_baseline leg)."""
import argparse

import numpy as np
import pytest


@pytest.mark.gpu
def test_bench_c2_batch_matches_oracle():
    import bench
    import trivy_amd
    from oracle import match as om
    from trivy_amd.batch import MatchBatch
    args = argparse.Namespace(keys_per_plat=30000, targets=10000, pkgs_per_target=400)
    wl = bench.C2(args)
    db = trivy_amd.DB()
    wl.load(db, vulns=False)
    eng = trivy_amd.Engine(db.finalize(), 0)
    mb = MatchBatch(eng)
    wl.fill(mb)
    total, errp, bits = mb.run()
    assert errp == -1 and bits == 0 and total > 10_000_000
    pairs = mb.pairs()
    opk, oad = om.match(om.Prepared(wl.sdb, wl.batch), n_threads=16)
    assert np.array_equal(pairs[:, 0], opk) and np.array_equal(pairs[:, 1], oad)
    # the DetectedVulnerability set of the batch (tvm_match_vulns): one per pair, each the
    # record of its advisory (Debian / Ubuntu epilogues; fields: tests/test_gpu_vulns.py)
    vs = mb.vulns()
    assert np.array_equal(vs.pkg, opk) and np.array_equal(vs.rec, oad)
    vs.close()
    mb.close()
    # the end-to-end pipelined pass (bench.py end_to_end) on the same 4M batch: CSR == oracle
    mp = MatchBatch(eng)
    wl.fill(mp)
    mp.pipeline_prepare(match_cap=total, chunk_packages=1 << 19)
    got, ep, _ = mp.pipeline_run()
    adv, rend = mp.pipeline_csr()
    counts = np.diff(np.concatenate([[0], rend.astype(np.int64)]))
    assert got == total and ep == -1
    assert np.array_equal(np.repeat(np.arange(len(rend), dtype=np.uint32), counts), opk)
    assert np.array_equal(adv, oad)
    vp = mp.vulns(pipeline=True)
    assert np.array_equal(vp.pkg, opk) and np.array_equal(vp.rec, oad)
    vp.close()
    mp.close()
