"""GPU: the rpm/apk (BASELINE.json C5), language-package (C3) and mixed OS + language (C4)
workloads through the batch API - 400k packages per run over a generated DB of each config's platform mix - checked
per platform on a random sample against (1) the per-driver C-ABI entry points
(tvm_ospkg_driver_detect / tvm_library_detect, one launch per sample) and (2) the oracle's
drivers (oracle/drivers.py, oracle/library.py).  (2) pins the semantics, (1) vs the batch
pairs checks that a package's result does not depend on the rest of the batch."""
import collections

import numpy as np
import pytest

from conftest import canon
from tools import synth_mix as sm

pytestmark = pytest.mark.gpu

# C4 (BASELINE config 4): the mixed batch - dpkg (Debian / Ubuntu), the Red Hat family
# (Red Hat CPE sets + merge, Oracle ksplice, alma, rocky arches), Alpine and four lockfile
# ecosystems interleaved in one launch of the all-grammar kernel
# c3lean: C3 without Maven (go / npm / PEP 440): the GM_LEAN kernel alone; c3 / c4 run their
# tiles without Maven packages on it too (Engine::launch's split launch)
CFGS = {"c5": (sm.C5_PLATS, sm.C5_WEIGHTS, 3000), "c3": (sm.C3_PLATS, sm.C3_WEIGHTS, 5000),
        "c4": (sm.C4_PLATS, sm.C4_WEIGHTS, 2500), "c3lean": (sm.C3_PLATS, [15, 0, 40, 25], 5000)}


@pytest.mark.parametrize("cfg", list(CFGS))
def test_mix_batch_parity(cfg):
    import oracle.drivers as od
    import oracle.library as ol
    import trivy_amd
    from trivy_amd.batch import MatchBatch, advisory_vuln_id
    from trivy_amd.detector import library, ospkg
    plats, weights, kpp = CFGS[cfg]
    sdb = sm.make_mix_db(plats, kpp, seed=0x5EED + len(cfg))
    db = sdb.put(trivy_amd.DB()).finalize()
    eng = trivy_amd.Engine(db, 0)
    batch = sm.make_mix_batch(sdb, 400_000, weights, seed=17)
    mb = MatchBatch(eng)
    firsts = sm.add_to(mb, sdb, batch)
    total, errp, bits = mb.run()
    assert errp == -1 and bits == 0 and total > 200_000
    pairs = mb.pairs().astype(np.int64)
    assert np.all(np.diff(pairs[:, 0] * (1 << 32) + pairs[:, 1]) > 0)  # (package, advisory) order
    rng = np.random.default_rng(5)
    checked = 0
    for (p, g), (_, first) in zip(batch.groups, firsts):
        bucket, kind = sdb.plats[p]
        idx = np.sort(rng.choice(len(g["key"]), 250, replace=False))
        pkgs = sm.driver_packages(sdb, p, g, idx)
        roots = sm.C3_ROOTS.get(kind, [bucket])
        recs = sdb.records_for({r: {x["Name"] for x in pkgs} for r in roots})
        if kind == "redhat":  # per-CVE merge: the batch epilogue (GPU) vs drop-in vs oracle
            names = {g["name"][i].decode() for i in idx}
            recs = sdb.records_for({"Red Hat": names, "Red Hat CPE": {"repository", "nvr", "cpe"}})
            want, got = [], []
            for rel in (7, 8, 9):
                sub = [pk for pk, i in zip(pkgs, idx) if int(g["rhrel"][i]) == rel]
                want += od.driver_detect("redhat", str(rel), None, sub, od.Records(recs), None)
                got += ospkg.Scanner(eng, "redhat").detect(str(rel), None, sub)
            assert canon(got) == canon(want), bucket
            every = sm.driver_packages(sdb, p, g, np.arange(len(g["key"])))
            batch_vulns = mb.redhat_result({first + i: pk for i, pk in enumerate(every)})
            sampled = {pk["ID"] for pk in pkgs}
            assert canon([v for v in batch_vulns if v.get("PkgID") in sampled]) == canon(want), bucket
            rh_checked = len(want)
            assert rh_checked > 100 and any(len(v.get("VendorIDs", [])) > 1 for v in want)
            checked += len(want)
            continue
        if kind in sm.LANG_OF:
            want = ol.detect(od.Records(recs), sm.LANG_OF[kind], pkgs)
            got = library.detect(eng, sm.LANG_OF[kind], pkgs)
        else:
            fam, fmt = sm.DRIVER_OF[kind]
            os_ver = fmt.format(bucket.split(" ")[-1])
            want = od.driver_detect(fam, os_ver, None, pkgs, od.Records(recs), None)
            got = ospkg.Scanner(eng, fam).detect(os_ver, None, pkgs)
        assert canon(got) == canon(want), bucket
        # the batch pairs of the sampled packages name the same (package, vulnerability) multiset
        rows = {int(first + i): int(i) for i in idx}
        lo, hi = np.searchsorted(pairs[:, 0], [first, first + len(g["key"])])
        seg = pairs[lo:hi]
        seg = seg[np.isin(seg[:, 0], list(rows))]
        from_batch = collections.Counter((rows[int(a)], advisory_vuln_id(db, int(b))) for a, b in seg)
        from_oracle = collections.Counter((int(v["PkgID"][1:]), v["VulnerabilityID"]) for v in want)
        assert from_batch == from_oracle, bucket
        checked += len(want)
    assert checked > 1000


@pytest.mark.parametrize("cfg", list(CFGS))
def test_mix_variants_agree(cfg):
    """rpm/apk/library grammars and row filters: every kernel variant yields variant 0's pairs."""
    import trivy_amd
    from trivy_amd._lib import lib
    from trivy_amd.batch import MatchBatch
    from test_gpu_parity import variants
    plats, weights, kpp = CFGS[cfg]
    sdb = sm.make_mix_db(plats, kpp // 3, seed=0x77 + len(cfg))
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    batch = sm.make_mix_batch(sdb, 60_000, weights, seed=23)
    ref = None
    try:
        for v in variants(grammar_set={"c3": 4, "c4": 4, "c3lean": 8}.get(cfg, 2)):
            lib().tvm_engine_set_variant(eng.h, v)
            mb = MatchBatch(eng)
            sm.add_to(mb, sdb, batch)
            total, errp, bits = mb.run()
            assert errp == -1 and bits == 0
            pairs = mb.pairs()
            if ref is None:
                ref = pairs
                assert total > 10_000
            assert np.array_equal(pairs, ref), lib().tvm_variant_name(v)
    finally:
        lib().tvm_engine_set_variant(eng.h, 0)
