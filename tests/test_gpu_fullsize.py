"""GPU, full size: C5 at its bench size (20M rpm / apk packages) and C4 at one GPU's share of the
100M mix (12.5M packages) - the whole batch's DetectedVulnerability set equals the oracle's,
field for field and in the drivers' output order, from the device-resident pass and from the
pipelined pass (whose per-package lists must also equal the device-resident pairs).

The same checks as tests/test_gpu_vulns.py / test_gpu_pipeline_mix.py, which run C5 at 4M and
a 1M slice of C4 in the default suite; at full size the oracle digests the batch column-wise
(oracle/mix_c.py Prepared(columnar=True), pinned to the scalar digest by
tests/test_cport.py::test_columnar_digest_equals_scalar) and one config takes minutes of host
work, so these run only with TVM_FULLSIZE=1 (tools/gpu_fullsize.sh; logs under
profiles/r06/validate/)."""
import os

import numpy as np
import pytest

import vulnset_ref as vr
from tools import synth_mix as sm

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("TVM_FULLSIZE") != "1",
                                 reason="full-size whole-batch checks: TVM_FULLSIZE=1 (tools/gpu_fullsize.sh)")]

# (platforms, weights, keys per platform, packages): bench.py Mix's generator, seed and sizes
CFGS = {"c5": (sm.C5_PLATS, sm.C5_WEIGHTS, 12_000, 20_000_000),
        "c4share": (sm.C4_PLATS, sm.C4_WEIGHTS, 20_000, 12_500_000)}


def _pairs_of(adv, row_end):
    counts = np.diff(np.concatenate([[0], row_end.astype(np.int64)]))
    return np.repeat(np.arange(len(row_end), dtype=np.uint32), counts), adv


def _same_set(vs, keys, want_pkg, want_rec, what):
    got_pkg, got_rec = vr.gpu_side(vs, keys)
    assert len(got_pkg) == len(want_pkg), (what, len(got_pkg), len(want_pkg))
    assert np.array_equal(got_pkg, want_pkg), what
    bad = np.nonzero(got_rec != want_rec)[0]
    assert len(bad) == 0, (what, len(bad), int(got_pkg[bad[0]]))
    assert vs.n_grp_recs > 1000, what  # Red Hat groups of several members: records of their own
    return got_pkg


@pytest.mark.timeout(1100)
@pytest.mark.parametrize("cfg", list(CFGS))
def test_fullsize_whole_batch_vs_oracle(cfg):
    import time

    import trivy_amd
    from trivy_amd.batch import MatchBatch
    t0 = time.time()
    plats, weights, kpp, n = CFGS[cfg]
    sdb = sm.make_mix_db(plats, kpp)
    batch = sm.make_mix_batch(sdb, n, weights, seed=2)
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    print(f"[{cfg}] db + batch {time.time() - t0:.0f} s", flush=True)
    mb = MatchBatch(eng)
    sm.add_to(mb, sdb, batch)
    total, errp, bits = mb.run()
    assert errp == -1 and bits == 0 and total > n // 2
    pairs = mb.pairs()
    vs = mb.vulns()
    keys = vr.Keys()
    want_pkg, want_rec, installed = vr.expected(sm, sdb, batch, keys, threads=16, columnar=True)
    print(f"[{cfg}] {n} packages, {total} pairs, {len(want_pkg)} DetectedVulnerabilities; oracle done "
          f"{time.time() - t0:.0f} s", flush=True)
    got_pkg = _same_set(vs, keys, want_pkg, want_rec, "device-resident")
    vs.close()
    # the package side: InstalledVersion of every package with findings
    _, vers, paths = mb.report()
    for p in np.unique(got_pkg).tolist():
        assert vers[p] == installed[p] and paths[p] == "", p
    mb.close()
    print(f"[{cfg}] device-resident set equal {time.time() - t0:.0f} s", flush=True)
    # the pipelined pass from host memory (transport form, 512k-package chunks)
    mp = MatchBatch(eng)
    sm.add_to(mp, sdb, batch)
    mp.pipeline_prepare(match_cap=total, chunk_packages=1 << 19)
    got_total, errp, _ = mp.pipeline_run()
    assert errp == -1 and got_total == total
    pk, ad = _pairs_of(*mp.pipeline_csr())
    assert np.array_equal(pk, pairs[:, 0]) and np.array_equal(ad, pairs[:, 1])
    vp = mp.vulns(pipeline=True)
    _same_set(vp, keys, want_pkg, want_rec, "pipelined")
    vp.close()
    mp.close()
    print(f"[{cfg}] pipelined lists and set equal {time.time() - t0:.0f} s", flush=True)
