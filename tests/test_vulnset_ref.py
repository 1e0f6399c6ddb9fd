"""CPU: the whole-batch DetectedVulnerability checker (tests/vulnset_ref.py - the C oracle's
matches over the whole batch, turned into records by the oracle drivers' epilogues) equals the
oracle drivers' own per-target output (oracle/drivers.py driver_detect, oracle/library.py detect)
field for field, DetectedVulnerability by DetectedVulnerability in each package's output order,
on seeded C3 / C4 / C5 batches.  This pins the checker the GPU whole-batch tests
(tests/test_gpu_vulns.py) use at full size."""
import collections

import numpy as np
import pytest

import vulnset_ref as vr
from oracle import drivers as od
from oracle import library as ol
from tools import synth_mix as sm

CFG = {"c3": (sm.C3_PLATS, sm.C3_WEIGHTS), "c4": (sm.C4_PLATS, sm.C4_WEIGHTS), "c5": (sm.C5_PLATS, sm.C5_WEIGHTS)}


def _with_ids(pkgs, base):
    for k, pk in enumerate(pkgs):  # every field a driver copies is set, so the copy flags show
        pk["ID"] = f"p{base + k}"
        pk["Identifier"] = {"PURL": f"pkg:x/{base + k}"}
        pk["Layer"] = {"DiffID": f"sha256:{base + k:08x}"}
    return pkgs


def _driver_output(sdb, batch):
    """{package index: [DetectedVulnerability, ...] in the driver's order} from the Python
    oracle drivers, one call per target group."""
    out = collections.defaultdict(list)
    base = 0
    for p, g in batch.groups:
        bucket, kind = sdb.plats[p]
        idx = np.arange(len(g["key"]))
        pkgs = _with_ids(sm.driver_packages(sdb, p, g, idx), base)
        roots = sm.C3_ROOTS.get(kind, [bucket])
        names = {pk["Name"] for pk in pkgs} | {pk.get("SrcName", pk["Name"]) for pk in pkgs}
        if kind == "redhat":
            names |= {od.add_modular_namespace(pk["Name"], pk.get("Modularitylabel", "")) for pk in pkgs}
            recs = od.Records(sdb.records_for({"Red Hat": names, "Red Hat CPE": {"repository", "nvr", "cpe"}}))
            vs = []
            for rel in (7, 8, 9):
                vs += od.driver_detect("redhat", str(rel), None,
                                       [pk for pk, i in zip(pkgs, idx) if int(g["rhrel"][i]) == rel], recs, None)
        else:
            if kind in sm.LANG_OF:
                eco = ol.LANG[sm.LANG_OF[kind]][0]
                names = {ol.normalize_pkg_name(eco, x) for x in names}
            recs = od.Records(sdb.records_for({r: names for r in roots}))
            if kind in sm.LANG_OF:
                vs = ol.detect(recs, sm.LANG_OF[kind], pkgs)
            else:
                fam, fmt = sm.DRIVER_OF[kind]
                vs = od.driver_detect(fam, fmt.format(bucket.split(" ")[-1]), None, pkgs, recs, None)
        for v in vs:
            out[int(v["PkgID"][1:])].append(v)
        base += len(idx)
    return out


@pytest.mark.parametrize("cfg", list(CFG))
def test_checker_equals_oracle_drivers(cfg):
    plats, weights = CFG[cfg]
    sdb = sm.make_mix_db(plats, 700, seed=11)
    batch = sm.make_mix_batch(sdb, 6000, weights, seed=5)
    keys = vr.Keys()
    pkg, rec, installed = vr.expected(sm, sdb, batch, keys, threads=4)
    got = collections.defaultdict(list)
    for p, r in zip(pkg.tolist(), rec.tolist()):
        got[p].append(r)
    want = _driver_output(sdb, batch)
    assert set(got) == set(want)
    n = 0
    for p, vs in want.items():
        exp = []
        for v in vs:
            assert v.get("InstalledVersion", "") == installed[p]
            exp.append(keys(vr.rec_key(*od.record_of(v))))
        assert got[p] == exp, p
        n += len(vs)
    assert n > 2000
    if cfg != "c3":  # merged Red Hat groups of several members are exercised
        assert any(len(v.get("VendorIDs", [])) > 1 for vs in want.values() for v in vs)
