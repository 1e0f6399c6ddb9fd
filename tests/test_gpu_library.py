"""GPU: library detection (pkg/detector/library) through the C-ABI against the reference's
vectors (every compare_test.go KAT, driver_test.go, the lang-pkgs integration goldens) and
against the oracle on random advisories for all six grammars."""
import functools
import glob
import json
import os
import random

import pytest

import golden_tables as gt
from conftest import canon
from test_oracle_library import _KATS, _DRV, _INTEG

pytestmark = pytest.mark.gpu

LANG_OF = {"generic": "gomod", "npm": "npm", "pep440": "pip", "maven": "jar", "gem": "bundler", "bitnami": "bitnami"}
ECO_OF = {"generic": "go", "npm": "npm", "pep440": "pip", "maven": "maven", "gem": "rubygems", "bitnami": "bitnami"}
_ENGINES = {}


def _engine_from_records(key, records):
    import trivy_amd
    if key not in _ENGINES:
        db = trivy_amd.DB()
        db.put_records(records)
        _ENGINES[key] = trivy_amd.Engine(db.finalize(), 0)
    return _ENGINES[key]


def _engine_from_files(paths):
    import trivy_amd
    key = tuple(paths)
    if key not in _ENGINES:
        _ENGINES[key] = trivy_amd.Engine(trivy_amd.load_fixture_files(paths), 0)
    return _ENGINES[key]


def test_comparer_kats():
    """Every compare_test.go case: one advisory per case under its own package."""
    from trivy_amd.detector.library import detect
    recs, pkgs = [], {}
    for i, (cid, g, ver, adv, want) in enumerate(_KATS):
        name = f"kat-{i}"
        recs.append({"path": [ECO_OF[g] + "::KAT", name, "CVE-KAT"], "value": json.dumps(adv)})
        pkgs.setdefault(g, []).append(({"Name": name, "Version": ver, "ID": cid}, want, cid))
    eng = _engine_from_records("kats", recs)
    for g, items in pkgs.items():
        got = detect(eng, LANG_OF[g], [p for p, _, _ in items])
        hit = {v["PkgName"] for v in got}
        for p, want, cid in items:
            assert (p["Name"] in hit) == want, cid


@pytest.mark.parametrize("case", _DRV, ids=[c[0] for c in _DRV])
def test_driver_cases(case):
    from trivy_amd.detector.library import Driver
    from trivy_amd.detector.ospkg import DetectError
    name, fx, lang, pkg, ver, want, err = case
    d = Driver(_engine_from_files(fx), lang)
    if err:
        with pytest.raises(DetectError) as ei:
            d.detect_vulnerabilities("", pkg, ver)
        assert err in str(ei.value)
    else:
        assert canon(d.detect_vulnerabilities("", pkg, ver)) == canon(want), name


@pytest.mark.parametrize("case", _INTEG, ids=[c[0] for c in _INTEG])
def test_integration_goldens(case):
    from trivy_amd.detector.library import detect
    cid, fx, lang, pkgs, want = case
    got = detect(_engine_from_files(fx), lang, pkgs)
    keep = {"VulnerabilityID", "PkgID", "PkgName", "InstalledVersion", "FixedVersion", "PkgPath", "DataSource"}
    assert canon([{k: v for k, v in g.items() if k in keep} for g in got]) == canon(want), cid


def test_detect_errors_and_unsupported():
    from trivy_amd.detector.library import detect, ecosystem
    from trivy_amd.detector.ospkg import DetectError
    fx = [os.path.join(gt.GOLDEN, "fixtures", "library", "invalid-type.json")]
    with pytest.raises(DetectError, match="failed to scan composer vulnerabilities: failed to detect composer "
                                          "vulnerabilities: failed to get composer advisories: failed to unmarshal"):
        detect(_engine_from_files(fx), "composer", [{"Name": "symfony/symfony", "Version": "5.1.5"}])
    assert detect(_engine_from_files(fx), "conda-pkg", [{"Name": "x", "Version": "1"}]) is None
    assert ecosystem("poetry") == "pip" and ecosystem("conda-pkg") is None


@pytest.mark.parametrize("g", list(LANG_OF))
def test_random_parity_vs_oracle(g):
    """Random advisories (2-3 per package, several sources) x random installed versions:
    the GPU result set equals the oracle's library.Detect exactly."""
    import oracle.drivers as od
    import oracle.library as ol
    import test_libver_host as tl
    from trivy_amd.detector.library import detect
    r = random.Random(1000 + len(g))
    eco = ECO_OF[g]
    recs = [{"path": ["data-source", f"{eco}::src{j}"],
             "value": json.dumps({"ID": f"s{j}", "Name": f"Source {j}", "URL": f"https://s{j}"})} for j in range(2)]
    names = [f"pkg{i}" for i in range(300)]
    for name in names:
        for j in range(r.randint(1, 3)):
            adv = {}
            for f in ("VulnerableVersions", "PatchedVersions", "UnaffectedVersions"):
                if r.random() < 0.5:
                    adv[f] = [tl._cons(r, g) for _ in range(r.randint(1, 2))]
            src = f"{eco}::src{r.randint(0, 1)}"
            recs.append({"path": [src, name, f"CVE-{r.randint(0, 3)}"], "value": json.dumps(adv)})
    pkgs = []
    for i in range(3000):
        ver = tl.GENS[g](r)  # Maven: non-transitive shapes included (pairwise AUX_MVN rows)
        pkgs.append({"Name": r.choice(names), "Version": ver, "ID": f"id{i}", "FilePath": f"f{i % 7}"})
    eng = _engine_from_records(f"rand-{g}", recs)
    got = detect(eng, LANG_OF[g], pkgs)
    want = ol.detect(od.Records(recs), LANG_OF[g], pkgs)
    assert len(want) > 100
    assert canon(got) == canon(want)


def test_maven_long_keys_vs_oracle():
    """Maven versions whose keys pass 16 bytes and tie with the bounds' on their heads
    (numeric-bound advisories are key-order intervals over the installed version's numeric
    projection; such a key spills, since a Maven package's tail slot holds its program state):
    the GPU result set equals the oracle's library.Detect."""
    import oracle.drivers as od
    import oracle.library as ol
    from trivy_amd.detector.library import detect
    r = random.Random(77)
    base = ["1.2.3.4.5", "10.20.30.40.50", "1.0.0.0.7", "2023.10.15.1"]
    tail = lambda: "".join(f".{r.choice([0, 1, 2, 9, 10, 99])}" for _ in range(r.randint(1, 3)))  # noqa: E731
    recs = [{"path": ["data-source", "maven::src0"], "value": json.dumps({"ID": "s0", "Name": "S", "URL": "https://s"})}]
    names = [f"long{i}" for i in range(60)]
    for i, name in enumerate(names):
        b = base[i % len(base)]
        for j in range(r.randint(1, 3)):
            lo, hi = sorted([b + tail(), b + tail()],
                            key=functools.cmp_to_key(lambda x, y: ol.MvnVer(x).compare(ol.MvnVer(y))))
            adv = r.choice([{"VulnerableVersions": [f"<{hi}"]}, {"VulnerableVersions": [f">={lo}, <{hi}"]},
                            {"VulnerableVersions": [f"[{lo},{hi}]"]}, {"PatchedVersions": [f">={hi}"]},
                            {"VulnerableVersions": [f"<={hi}"], "PatchedVersions": [f"{lo}"]}])
            recs.append({"path": ["maven::src0", name, f"CVE-{j}"], "value": json.dumps(adv)})
    pkgs = []
    for i in range(4000):
        k = r.randrange(len(names))
        v = base[k % len(base)] + tail() + r.choice(["", "", "-rc1", ".jre", "-sp1", ".0.beta", "-1"])
        pkgs.append({"Name": names[k], "Version": v, "ID": f"id{i}", "FilePath": ""})
    eng = _engine_from_records("maven-long", recs)
    got = detect(eng, "jar", pkgs)
    want = ol.detect(od.Records(recs), "jar", pkgs)
    assert len(want) > 500
    assert canon(got) == canon(want)
