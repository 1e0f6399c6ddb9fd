"""GPU: the batch path's DetectedVulnerability set (tvm_match_vulns) equals the oracle's over the
WHOLE batch, field for field and in the drivers' output order - C3 at its bench size (1M
language packages, the bench's own DB and batch), C5 at 4M (rpm / apk: Red Hat merged per CVE,
Oracle ksplice, Rocky arch entries, Alpine), and a 1M slice of C4 (every OS driver family of
the mix plus the four lockfile ecosystems).

Checker: tests/vulnset_ref.py (oracle/mixmatch.c over the whole batch, records from the oracle
drivers' own epilogues), pinned to the oracle drivers' per-target output by
tests/test_vulnset_ref.py.  Reference epilogues: pkg/detector/ospkg/debian/debian.go:78-98,
alma/alma.go:64-71, redhat/redhat.go:140-187, library/driver.go:125-132 + detect.go:33-37."""
import numpy as np
import pytest

import vulnset_ref as vr
from tools import synth_mix as sm

pytestmark = pytest.mark.gpu

# (platforms, weights, keys per platform (bench.py Mix), packages)
CFGS = {"c3": (sm.C3_PLATS, sm.C3_WEIGHTS, 25_000, 1_000_000),
        "c5": (sm.C5_PLATS, sm.C5_WEIGHTS, 12_000, 4_000_000),
        "c4": (sm.C4_PLATS, sm.C4_WEIGHTS, 20_000, 1_000_000)}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg", list(CFGS))
def test_vulns_whole_batch_vs_oracle(cfg):
    import trivy_amd
    from trivy_amd.batch import MatchBatch
    plats, weights, kpp, n = CFGS[cfg]
    sdb = sm.make_mix_db(plats, kpp)
    batch = sm.make_mix_batch(sdb, n, weights, seed=2)  # bench.py Mix's generator and seed
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    mb = MatchBatch(eng)
    sm.add_to(mb, sdb, batch)
    total, errp, bits = mb.run()
    assert errp == -1 and bits == 0
    vs = mb.vulns()
    keys = vr.Keys()
    want_pkg, want_rec, installed = vr.expected(sm, sdb, batch, keys, threads=16)
    got_pkg, got_rec = vr.gpu_side(vs, keys)
    assert len(got_pkg) == len(want_pkg) and len(want_pkg) > n // 2
    assert np.array_equal(got_pkg, want_pkg)
    bad = np.nonzero(got_rec != want_rec)[0]
    inv = {v: k for k, v in keys.ids.items()}
    assert len(bad) == 0, (len(bad), int(got_pkg[bad[0]]), inv[int(got_rec[bad[0]])], inv[int(want_rec[bad[0]])])
    # the package side: InstalledVersion of every package with findings
    _, vers, paths = mb.report()
    for p in np.unique(got_pkg).tolist():
        assert vers[p] == installed[p] and paths[p] == "", p
    if cfg != "c3":  # merged Red Hat groups: records of their own
        assert vs.n_grp_recs > 1000
    vs.close()


def test_vulns_dicts_equal_driver_detect():
    """The dict form of a small batch's set equals the per-target drivers (drop-in C-ABI) on the
    same packages, with the caller's package fields copied per the records' flags."""
    import trivy_amd
    from conftest import canon
    from trivy_amd.batch import MatchBatch
    from trivy_amd.detector import library, ospkg
    sdb = sm.make_mix_db(sm.C4_PLATS, 600, seed=7)
    batch = sm.make_mix_batch(sdb, 20_000, sm.C4_WEIGHTS, seed=9)
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    mb = MatchBatch(eng)
    firsts = sm.add_to(mb, sdb, batch)
    mb.run()
    vs = mb.vulns()
    pkgs = {}
    want = []
    for (p, g), (_, first) in zip(batch.groups, firsts):
        bucket, kind = sdb.plats[p]
        dp = sm.driver_packages(sdb, p, g, np.arange(len(g["key"])))
        for i, pk in enumerate(dp):
            pk["ID"] = f"p{first + i}"
            pkgs[first + i] = pk
        if kind == "redhat":
            for rel in (7, 8, 9):
                want += ospkg.Scanner(eng, "redhat").detect(str(rel), None,
                                                            [pk for pk, r in zip(dp, g["rhrel"]) if int(r) == rel])
        elif kind in sm.LANG_OF:
            want += library.detect(eng, sm.LANG_OF[kind], dp)
        else:
            fam, fmt = sm.DRIVER_OF[kind]
            want += ospkg.Scanner(eng, fam).detect(fmt.format(bucket.split(" ")[-1]), None, dp)
    got = vs.dicts(pkgs)
    assert len(got) > 5000 and canon(got) == canon(want)
    vs.close()
