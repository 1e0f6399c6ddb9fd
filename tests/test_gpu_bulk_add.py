"""GPU: the parallel bulk add (tvm_batch_add_targets_attrs: every target of a fleet batch in one
call, filled on the host threads) builds the same batch as adding target by target
(tvm_batch_add_many_attrs) - same match pairs, same package side, same DetectedVulnerability
set - for the attribute-carrying workloads (Red Hat CPE sets + arches, Oracle ksplice, Rocky
arches) and the plain one; shards added as package ranges concatenate to the whole; bad
attributes are refused without touching the batch.  And the native consumer of a set
(tvm_vuln_set_walk) sees every DetectedVulnerability (its digest recomputed from the columns)."""
import numpy as np
import pytest

from tools import synth_mix as sm

pytestmark = pytest.mark.gpu


def _engine(plats, kpp, seed):
    import trivy_amd
    sdb = sm.make_mix_db(plats, kpp, seed=seed)
    return sdb, trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)


@pytest.mark.parametrize("cfg", ["c5", "c4", "c3"])
def test_bulk_add_equals_per_target_adds(cfg):
    from trivy_amd.batch import MatchBatch
    plats, weights = {"c5": (sm.C5_PLATS, sm.C5_WEIGHTS), "c4": (sm.C4_PLATS, sm.C4_WEIGHTS),
                      "c3": (sm.C3_PLATS, sm.C3_WEIGHTS)}[cfg]
    sdb, eng = _engine(plats, 1500, seed=41)
    batch = sm.make_mix_batch(sdb, 120_000, weights, seed=43)
    one = MatchBatch(eng)
    sm.add_to(one, sdb, batch)
    bulk = MatchBatch(eng)
    cols = sm.BulkCols(sdb, batch, per_target=400)
    assert cols.add(bulk) == 0 and len(bulk) == len(one) == len(batch)
    got = []
    for mb in (one, bulk):
        total, errp, bits = mb.run()
        assert errp == -1 and bits == 0
        pairs = mb.pairs()  # the raw list (vulns() merges Red Hat packages per CVE on the device)
        vs = mb.vulns()
        got.append((pairs, mb.report(), vs.pkg.copy(), vs.rec.copy(), vs.walk(), vs.digest()))
        vs.close()
    (p1, r1, vp1, vr1, w1, d1), (p2, r2, vp2, vr2, w2, d2) = got
    assert len(p1) > 20_000 and np.array_equal(p1, p2)
    assert r1 == r2
    assert np.array_equal(vp1, vp2) and np.array_equal(vr1, vr2)
    assert w1 == (len(vp1), d1) and w2 == (len(vp2), d2)
    # two shards added as package ranges (whole targets) concatenate to the whole
    cut = int(cols.ends[len(cols.ends) // 2])
    halves = []
    for lo, hi in ((0, cut), (cut, len(batch))):
        mb = MatchBatch(eng)
        assert cols.add(mb, lo, hi) == 0 and len(mb) == hi - lo
        mb.set_package_base(lo)
        mb.run()
        halves.append(mb.pairs())
        mb.close()
    assert np.array_equal(np.concatenate(halves), p2)
    one.close()
    bulk.close()


def test_bulk_add_refuses_bad_attributes():
    import ctypes

    from trivy_amd.batch import ATTR_CPESET, ATTR_KSPLICE, MatchBatch
    sdb, eng = _engine(sm.C5_PLATS, 300, seed=5)
    batch = sm.make_mix_batch(sdb, 4000, sm.C5_WEIGHTS, seed=6)
    cols = sm.BulkCols(sdb, batch)
    mb = MatchBatch(eng)
    n = cols.n
    ends = cols.ends
    args = ([cols.buckets[t] for t in range(len(ends))], ends, cols.arena, cols.noff, cols.nlen, cols.voff, cols.vlen)
    with pytest.raises(RuntimeError):  # one attribute word: a ksplice tag or a CPE set, not both
        mb.add_targets(*args, flags=np.full(len(ends), ATTR_KSPLICE | ATTR_CPESET, np.uint32),
                       cpe_sets=np.zeros(n, np.uint32))
    with pytest.raises(RuntimeError):  # a CPE-set id the batch never registered
        mb.add_targets(*args, flags=np.full(len(ends), ATTR_CPESET, np.uint32), cpe_sets=np.full(n, 7, np.uint32))
    with pytest.raises(RuntimeError):  # arch flags without the arch columns
        mb.add_targets(*args, flags=np.full(len(ends), 1, np.uint32))
    assert len(mb) == 0
    assert cols.add(mb) == 0 and len(mb) == n  # the batch is still usable
    total, errp, bits = mb.run()
    assert errp == -1 and bits == 0 and total > 0
    del ctypes
    mb.close()


def test_walk_digest_dpkg_batch():
    """The consumer over a plain dpkg batch added by tvm_batch_add_targets (C2's form) and over
    its pipelined set: the same DetectedVulnerabilities, the same digest."""
    from test_gpu_parity import build_engine
    from tools.synth import make_batch, make_db
    from trivy_amd.batch import MatchBatch
    sdb = make_db(["debian 12", "ubuntu 22.04"], 2000, seed=12)
    eng = build_engine(sdb)
    batch = make_batch(sdb, 60, 400, [1, 1], seed=13)
    arena, noff, nlen, voff, vlen = batch.arena()
    mb = MatchBatch(eng)
    ends = np.array([b1 for _, _, b1 in batch.targets], dtype=np.uint64)
    mb.add_targets([sdb.platforms[p] for p, _, _ in batch.targets], ends, arena, noff, nlen, voff, vlen)
    total, errp, _ = mb.run()
    vs = mb.vulns()
    n1, d1 = vs.walk()
    assert n1 == len(vs) == total and d1 == vs.digest()
    vs.close()
    mb.pipeline_prepare(match_cap=total, chunk_packages=4096)
    assert mb.pipeline_run()[:2] == (total, -1)
    vp = mb.vulns(pipeline=True)
    assert vp.walk() == (n1, d1)
    vp.close()
    mb.close()
