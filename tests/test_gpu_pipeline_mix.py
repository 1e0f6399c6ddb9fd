"""GPU: the end-to-end pipelined pass (tvm_pipeline_*) on the filtered grammar sets - C3's
language packages (Maven / PEP 440 / npm / go, Maven scratch per chunk), C5's rpm / apk fleet
(arch / ksplice / CPE-set attributes carried per chunk, Red Hat merged per CVE) and a 1M slice
of C4 (every driver family of the mix) - equals the oracle over the WHOLE batch:

* the per-package advisory lists (CSR) of every pass equal the device-resident pass's
  (package, advisory) pairs (those are pinned to the oracle drivers by tests/test_gpu_mix.py);
* the DetectedVulnerability set (tvm_pipeline_vulns) equals tests/vulnset_ref.py's - the
  oracle drivers' own epilogues over oracle/mixmatch.c's matches, Red Hat groups merged per
  redhat.go:146-187 - field for field, in the drivers' output order;

for the transport form and the raw form, and for chunk sizes that cut the batch into many
chunks (4096 packages: tiles of Maven programs split across chunk launches) and few."""
import numpy as np
import pytest

import vulnset_ref as vr
from tools import synth_mix as sm

pytestmark = pytest.mark.gpu

# (platforms, weights, keys per platform, packages): the bench's Mix (C3 full size, C5 at 4M,
# a 1M slice of C4), the same generator and seed as tests/test_gpu_vulns.py
CFGS = {"c3": (sm.C3_PLATS, sm.C3_WEIGHTS, 25_000, 1_000_000),
        "c5": (sm.C5_PLATS, sm.C5_WEIGHTS, 12_000, 4_000_000),
        "c4": (sm.C4_PLATS, sm.C4_WEIGHTS, 20_000, 1_000_000)}
# (raw form, chunk packages)
PASSES = [(False, 1 << 19), (True, 4096), (False, 100_000)]


def _pairs_of(adv, row_end):
    counts = np.diff(np.concatenate([[0], row_end.astype(np.int64)]))
    return np.repeat(np.arange(len(row_end), dtype=np.uint32), counts), adv


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("cfg", list(CFGS))
def test_pipeline_whole_batch_vs_oracle(cfg):
    import trivy_amd
    from trivy_amd.batch import MatchBatch
    plats, weights, kpp, n = CFGS[cfg]
    sdb = sm.make_mix_db(plats, kpp)
    batch = sm.make_mix_batch(sdb, n, weights, seed=2)
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    dev = MatchBatch(eng)
    sm.add_to(dev, sdb, batch)
    total, errp, bits = dev.run()
    assert errp == -1 and bits == 0 and total > n // 2
    pairs = dev.pairs()
    dev.close()
    keys = vr.Keys()
    want_pkg, want_rec, _ = vr.expected(sm, sdb, batch, keys, threads=16)
    mb = MatchBatch(eng)
    sm.add_to(mb, sdb, batch)
    for raw, chunk in PASSES:
        mb.pipeline_prepare(match_cap=total, chunk_packages=chunk, raw=raw)
        got_total, errp, _ = mb.pipeline_run()
        assert errp == -1 and got_total == total, (raw, chunk)
        pk, ad = _pairs_of(*mb.pipeline_csr())
        assert np.array_equal(pk, pairs[:, 0]) and np.array_equal(ad, pairs[:, 1]), (raw, chunk)
        assert mb.pipeline_stats()["transport_form"] == (not raw)
        vs = mb.vulns(pipeline=True)
        got_pkg, got_rec = vr.gpu_side(vs, keys)
        assert np.array_equal(got_pkg, want_pkg), (raw, chunk)
        bad = np.nonzero(got_rec != want_rec)[0]
        assert len(bad) == 0, (raw, chunk, len(bad), int(got_pkg[bad[0]]))
        if cfg != "c3":  # Red Hat groups of several members: records of their own
            assert vs.n_grp_recs > 1000
        vs.close()
    mb.close()


def test_pipeline_vulns_dicts_with_package_base():
    """A pipelined shard whose packages are numbered from a non-zero base
    (tvm_batch_set_package_base, as dist_worker.py numbers a rank's shard): its set - Red Hat
    groups merged on the device - as dicts equals the per-target drop-in drivers on the same
    packages, and the device-resident set of the same shard equals it too."""
    import trivy_amd
    from conftest import canon
    from trivy_amd.batch import MatchBatch
    from trivy_amd.detector import library, ospkg
    sdb = sm.make_mix_db(sm.C4_PLATS, 600, seed=7)
    batch = sm.make_mix_batch(sdb, 20_000, sm.C4_WEIGHTS, seed=9)
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    base = 1_000_003
    want, pkgs = [], {}
    firsts = None
    sets = []
    for pipeline in (True, False):
        mb = MatchBatch(eng)
        firsts = sm.add_to(mb, sdb, batch)
        mb.set_package_base(base)
        if pipeline:
            mb.pipeline_prepare(chunk_packages=4096)
            assert mb.pipeline_run()[1] == -1
        else:
            mb.run()
        vs = mb.vulns(pipeline=pipeline)
        assert int(vs.pkg.min()) >= base
        sets.append((mb, vs))
    for (p, g), (_, first) in zip(batch.groups, firsts):
        bucket, kind = sdb.plats[p]
        dp = sm.driver_packages(sdb, p, g, np.arange(len(g["key"])))
        for i, pk in enumerate(dp):
            pk["ID"] = f"p{first + i}"
            pkgs[base + first + i] = pk
        if kind == "redhat":
            for rel in (7, 8, 9):
                want += ospkg.Scanner(eng, "redhat").detect(str(rel), None,
                                                            [pk for pk, r in zip(dp, g["rhrel"]) if int(r) == rel])
        elif kind in sm.LANG_OF:
            want += library.detect(eng, sm.LANG_OF[kind], dp)
        else:
            fam, fmt = sm.DRIVER_OF[kind]
            want += ospkg.Scanner(eng, fam).detect(fmt.format(bucket.split(" ")[-1]), None, dp)
    assert len(want) > 5000
    for mb, vs in sets:
        assert canon(vs.dicts(pkgs)) == canon(want)
        vs.close()
        mb.close()


def test_pipeline_vulns_refused_before_a_pass():
    """tvm_pipeline_vulns hands out nothing before a completed pass (its lists would be
    uninitialised pinned memory)."""
    import trivy_amd
    from trivy_amd.batch import MatchBatch
    sdb = sm.make_mix_db(sm.C5_PLATS, 300, seed=3)
    batch = sm.make_mix_batch(sdb, 3000, sm.C5_WEIGHTS, seed=4)
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    mb = MatchBatch(eng)
    sm.add_to(mb, sdb, batch)
    mb.pipeline_prepare(chunk_packages=1024)
    with pytest.raises(RuntimeError, match="no completed tvm_pipeline_run"):
        mb.vulns(pipeline=True)
    assert mb.pipeline_run()[1] == -1
    vs = mb.vulns(pipeline=True)
    assert len(vs) > 100
    vs.close()
    mb.close()
