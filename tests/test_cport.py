"""CPU: the native CPU baseline of the mixed workloads (oracle/mixmatch.c + oracle/libcmp.c,
driven by oracle/mix_c.py) equals the Python oracle drivers (oracle/drivers.py,
oracle/library.py) on seeded samples of the C3 / C4 / C5 generators, and its library
comparers agree with oracle/library.py on the reference's compare_test.go tables.  The C port
is what bench.py's cpu_baseline times for those configs (1 thread and the box's threads)."""
import collections

import numpy as np
import pytest

from oracle import drivers as od
from oracle import library as ol
from oracle import mix_c
from tools import synth_mix as sm

CFG = {"c3": (sm.C3_PLATS, sm.C3_WEIGHTS), "c4": (sm.C4_PLATS, sm.C4_WEIGHTS), "c5": (sm.C5_PLATS, sm.C5_WEIGHTS)}


def _sample(which, n=5000, kpp=1500, seed=3):
    plats, weights = CFG[which]
    sdb = sm.make_mix_db(plats, kpp)
    batch = sm.make_mix_batch(sdb, n, weights, seed=seed)
    return sdb, [(p, g, list(range(len(g["key"])))) for p, g in batch.groups]


def _oracle_pairs(sdb, sample):
    """(sample index, VulnerabilityID, FixedVersion) multiset from the Python oracle drivers."""
    out = collections.Counter()
    base = 0
    for p, g, idx in sample:
        bucket, kind = sdb.plats[p]
        pkgs = sm.driver_packages(sdb, p, g, idx)
        roots = sm.C3_ROOTS.get(kind, [bucket])
        if kind == "redhat":
            names = {pk["Name"] if not pk.get("Modularitylabel") else
                     od.add_modular_namespace(pk["Name"], pk["Modularitylabel"]) for pk in pkgs}
            recs = od.Records(sdb.records_for({"Red Hat": names, "Red Hat CPE": {"repository", "nvr", "cpe"}}))
            vs = []
            for rel in (7, 8, 9):
                vs += od.driver_detect("redhat", str(rel), None,
                                       [pk for pk, i in zip(pkgs, idx) if int(g["rhrel"][i]) == rel], recs, None)
        else:
            names = {pk["Name"] for pk in pkgs} | {pk.get("SrcName", pk["Name"]) for pk in pkgs}
            if kind in sm.LANG_OF:
                eco = ol.LANG[sm.LANG_OF[kind]][0]
                names = {ol.normalize_pkg_name(eco, x) for x in names}
            recs = od.Records(sdb.records_for({r: names for r in roots}))
            if kind in sm.LANG_OF:
                vs = ol.detect(recs, sm.LANG_OF[kind], pkgs)
            else:
                fam, fmt = sm.DRIVER_OF[kind]
                vs = od.driver_detect(fam, fmt.format(bucket.split(" ")[-1]), None, pkgs, recs, None)
        pos = {f"p{i}": base + k for k, i in enumerate(idx)}
        for v in vs:
            fixed = v.get("FixedVersion", "") if kind == "redhat" else ""
            out[(pos[v["PkgID"]], v["VulnerabilityID"], fixed)] += 1
        base += len(idx)
    return out


def _c_pairs(prep, pk, en, sdb):
    out = collections.Counter()
    for p, e in zip(pk.tolist(), en.tolist()):
        ent = prep.entries[e]
        kind = sdb.plats[int(prep.plat_of[p])][1]
        fixed = od.rpm_string(ent["fixed"]) if kind == "redhat" and ent.get("fixed") else ""
        out[(p, ent["vid"], fixed)] += 1
    return out


@pytest.mark.parametrize("which", ["c5", "c3", "c4"])
def test_cport_equals_oracle_drivers(which, oracle_built):
    sdb, sample = _sample(which)
    prep = mix_c.Prepared(sm, sdb, sample)
    want = _oracle_pairs(sdb, sample)
    for threads in (1, 4):
        pk, en = mix_c.match(prep, n_threads=threads)
        got = _c_pairs(prep, pk, en, sdb)
        assert sum(want.values()) > 500
        assert got == want, (which, threads, sorted((got - want).items())[:5], sorted((want - got).items())[:5])


@pytest.mark.parametrize("which", ["c5", "c3", "c4"])
def test_columnar_digest_equals_scalar(which, oracle_built):
    """The columnar digest (Prepared(columnar=True): the whole-batch checks at 10-20M packages)
    gives the scalar digest's packages, keys, entries and matches, Red Hat members included, on
    the same sample - and on a shuffled row subset (the digest takes any row order)."""
    sdb, sample = _sample(which, n=20000)
    rng = np.random.default_rng(11)
    for smp in (sample, [(p, g, sorted(rng.choice(len(idx), len(idx) // 2, replace=False).tolist()))
                         for p, g, idx in sample]):
        a = mix_c.Prepared(sm, sdb, smp)
        b = mix_c.Prepared(sm, sdb, smp, columnar=True)
        assert np.array_equal(a.plat_of, b.plat_of)
        assert list(a.installed) == [b.installed[i] for i in range(len(b.installed))]
        assert [(e["vid"], e.get("fixed"), e.get("vul")) for e in a.entries] == \
            [(e["vid"], e.get("fixed"), e.get("vul")) for e in b.entries]
        pa, ea = (x.copy() for x in mix_c.match(a, 4, members=True))
        pb, eb = mix_c.match(b, 4, members=True)
        assert len(pa) > 1000 and np.array_equal(pa, pb) and np.array_equal(ea, eb)


def test_libcmp_is_vulnerable_on_reference_tables(oracle_built):
    """compare.IsVulnerable of the C comparers against the reference's own compare_test.go
    tables (tests/golden/tables: want) for the four grammars the workloads use, and against
    oracle/library.py on the same cases."""
    import ctypes
    import json
    import os
    L = od.lib()
    L.orc_lib_is_vulnerable.restype = ctypes.c_int
    L.orc_lib_is_vulnerable.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32,
                                        ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    here = os.path.join(os.path.dirname(__file__), "golden", "tables")
    checked = 0
    for sub, gram, pyname in (("compare__compare_test", 1, "generic"), ("compare__npm__compare_test", 2, "npm"),
                              ("compare__pep440__compare_test", 3, "pep440"),
                              ("compare__maven__compare_test", 4, "maven")):
        d = json.load(open(os.path.join(here, f"detector__library__{sub}.json")))
        for table in d["tables"]:
            for case in table["cases"]:
                args = case["args"]
                ver, adv = args.get("currentVersion", args.get("ver")), args["advisory"]
                vul = adv.get("VulnerableVersions") or []
                sec = (adv.get("PatchedVersions") or []) + (adv.get("UnaffectedVersions") or [])
                fl = (mix_c.HAS_VULN if vul else 0) | (mix_c.HAS_SECURE if sec else 0)
                if any(v == "" for v in vul + (adv.get("PatchedVersions") or [])):
                    fl |= mix_c.ALWAYS
                vb, ub, sb = ver.encode(), " || ".join(vul).encode(), " || ".join(sec).encode()
                got = L.orc_lib_is_vulnerable(gram, vb, len(vb), fl, ub, len(ub), sb, len(sb))
                assert got == int(bool(case.get("want", False))), (pyname, case["name"], ver, adv)
                assert got == int(ol.is_vulnerable(pyname, ver, adv)), (pyname, case["name"])
                checked += 1
    assert checked >= 30
