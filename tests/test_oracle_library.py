"""CPU: pins the library oracle (oracle/library.py) to the reference's own vectors:
every compare_test.go table (six comparers) and every driver_test.go case."""
import pytest

import golden_tables as gt
from conftest import canon

import oracle.drivers as od
import oracle.library as ol

COMPARERS = [("compare", "generic"), ("npm", "npm"), ("pep440", "pep440"), ("maven", "maven"),
             ("rubygems", "gem"), ("bitnami", "bitnami")]


def _kats():
    out = []
    for sub, grammar in COMPARERS:
        rel = ("detector__library__compare__compare_test.json" if sub == "compare"
               else f"detector__library__compare__{sub}__compare_test.json")
        for t in gt.load(rel)["tables"]:
            for c in t["cases"]:
                a = c["args"]
                ver = a.get("currentVersion", a.get("ver"))
                out.append((f"{sub}/{c['name']}", grammar, ver, a["advisory"], bool(c.get("want", False))))
    return out


_KATS = _kats()


@pytest.mark.parametrize("case", _KATS, ids=[c[0] for c in _KATS])
def test_comparer_kats(case):
    cid, grammar, ver, adv, want = case
    assert ol.is_vulnerable(grammar, ver, adv) == want, cid


def library_cases():
    out = []
    for c in gt.table("detector__library__driver_test.json", "TestDriver_Detect"):
        fx = [gt.os.path.join(gt.GOLDEN, "fixtures", "library", gt.os.path.basename(f)[:-5] + ".json")
              for f in c.get("fixtures") or []]
        err = c.get("wantErr")
        out.append((c["name"], fx, c["libType"], c["args"]["pkgName"], c["args"]["pkgVer"], c.get("want") or [], err))
    return out


_DRV = library_cases()


@pytest.mark.parametrize("case", _DRV, ids=[c[0] for c in _DRV])
def test_driver_cases(case):
    name, fx, lang, pkg, ver, want, err = case
    db = od.Records.from_files(fx)
    if err:
        with pytest.raises(od.DecodeError) as ei:
            ol.detect_vulnerabilities(db, lang, "", pkg, ver)
        assert err in str(ei.value)
    else:
        assert canon(ol.detect_vulnerabilities(db, lang, "", pkg, ver)) == canon(want), name


def test_create_fixed_versions():
    """driver.go:139-159 (cargo golden: patched constraints joined verbatim)."""
    assert ol.create_fixed_versions({"PatchedVersions": [">= 3.1.0", ">= 2.1.3, < 3.0.0"]}) == \
        ">= 3.1.0, >= 2.1.3, < 3.0.0"
    assert ol.create_fixed_versions({"VulnerableVersions": ["< 1.2", ">= 2.0, < 2.1", "<= 3"]}) == "1.2, 2.1"
    assert ol.create_fixed_versions({"PatchedVersions": ["1", "1", "2"]}) == "1, 2"


def test_unsupported_lang_type():
    assert ol.detect(od.Records([]), "conda-pkg", [{"Name": "x", "Version": "1"}]) is None


def integration_cases():
    import json
    import glob
    with open(gt.os.path.join(gt.GOLDEN, "integration_lib.json"), encoding="utf-8") as f:
        cases = json.load(f)
    fx = sorted(glob.glob(gt.os.path.join(gt.GOLDEN, "fixtures", "integration", "*.json")))
    return [(f"{c['golden']}:{c['target']}", fx, c["type"], c["pkgs"], c["want"]) for c in cases]


_INTEG = integration_cases()


@pytest.mark.parametrize("case", _INTEG, ids=[c[0] for c in _INTEG])
def test_integration_goldens(case):
    """library.Detect over the integration DB reproduces every lang-pkgs golden."""
    cid, fx, lang, pkgs, want = case
    db = od.Records.from_files(fx)
    got = ol.detect(db, lang, pkgs)
    keep = {"VulnerabilityID", "PkgID", "PkgName", "InstalledVersion", "FixedVersion", "PkgPath", "DataSource"}
    assert canon([{k: v for k, v in g.items() if k in keep} for g in got]) == canon(want), cid
