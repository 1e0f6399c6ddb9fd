"""SBOM decode (trivy_amd/sbom.py, mirror of pkg/sbom) pinned by the reference's SBOM
integration tests (integration/sbom_test.go:30-82): the three CycloneDX SBOMs decoded and
run through the detectors must give every golden's detector-produced vulnerabilities.

CPU: decode + the oracle's detectors (oracle/drivers.py, oracle/library.py).
GPU: decode + the product detectors over the C-ABI (the `trivy sbom` path end to end)."""
import datetime
import glob
import json
import os

import pytest

from conftest import canon
from trivy_amd import sbom as ts

HERE = os.path.join(os.path.dirname(__file__), "golden")
CASES = json.load(open(os.path.join(HERE, "sbom_cases.json")))
FX = sorted(glob.glob(os.path.join(HERE, "fixtures", "integration", "*.json")))
KEEP = {"VulnerabilityID", "PkgID", "PkgName", "InstalledVersion", "FixedVersion", "PkgPath", "DataSource"}
# the goldens were produced with a fixed clock (integration tests); detection does not depend on it
NOW = int(datetime.datetime(2021, 8, 25, 12, 20, 30, tzinfo=datetime.timezone.utc).timestamp())


def _decode(case):
    return ts.decode_cyclonedx(open(os.path.join(HERE, "sbom", case["sbom"])).read())


def _check(case, got):
    """got: {(class, type): vulns}.  Every golden Result must match; results the golden
    omits (no vulnerabilities) must be empty."""
    want = {(r["Class"], r["Type"]): r["Vulnerabilities"] for r in case["results"]}
    for key, vulns in got.items():
        sub = canon([{k: v for k, v in g.items() if k in KEEP} for g in vulns])
        assert sub == canon(want.get(key, [])), (case["name"], key)
    for key, vulns in want.items():
        assert key in got or not vulns, (case["name"], key)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_decode_matches_golden_metadata(case):
    d = _decode(case)
    assert d["OS"] == case["os"]
    lang_types = {r["Type"] for r in case["results"] if r["Class"] == "lang-pkgs"}
    assert lang_types <= {a["Type"] for a in d["Applications"]}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_sbom_scan_with_oracle_detectors(case):
    import oracle.drivers as od
    import oracle.library as ol
    d = _decode(case)
    db = od.Records.from_files(FX)
    got = {}
    if d["OS"]:
        got[("os-pkgs", d["OS"]["Family"])] = od.detect(db, d["OS"]["Family"], d["OS"]["Name"], None, d["Packages"],
                                                        NOW)[0]
    for app in d["Applications"]:
        v = ol.detect(db, app["Type"], app["Libraries"])
        if v is not None:
            got.setdefault(("lang-pkgs", app["Type"]), []).extend(v)
    _check(case, got)


def test_decode_rules():
    """decode.go details: rpm version-release split + epoch qualifier, component group in the
    name, app FilePath for non-aggregating types, orphan grouping and order, errors."""
    bom = {"bomFormat": "CycloneDX", "components": [
        {"bom-ref": "os", "type": "operating-system", "name": "alma", "version": "9.2"},
        {"bom-ref": "r1", "type": "library", "name": "z", "purl": "pkg:rpm/alma/z@1.2-3.el9?arch=x86_64&epoch=2"},
        {"bom-ref": "r2", "type": "library", "name": "a", "purl": "pkg:rpm/alma/a@0.1-1.el9"},
        {"bom-ref": "app", "type": "application", "name": "go.sum",
         "properties": [{"name": "aquasecurity:trivy:Type", "value": "gomod"}]},
        {"bom-ref": "g1", "type": "library", "name": "x", "group": "github.com/o", "purl": "pkg:golang/github.com/o/x@1.0.0"},
        {"bom-ref": "m1", "type": "library", "name": "core", "group": "org.a", "purl": "pkg:maven/org.a/core@2.0"},
        {"bom-ref": "n1", "type": "library", "name": "lodash", "purl": "pkg:npm/lodash@4.17.0"},
        {"bom-ref": "u1", "type": "library", "name": "q", "purl": "pkg:generic/q@1"},
        {"bom-ref": "f1", "type": "file", "name": "ignored"}],
        "dependencies": [{"ref": "os", "dependsOn": ["r1"]}, {"ref": "app", "dependsOn": ["g1", "nope"]}]}
    d = ts.decode_cyclonedx(json.dumps(bom))
    assert d["OS"] == {"Family": "alma", "Name": "9.2"}
    assert [(p["Name"], p["Version"], p.get("Release"), p.get("Epoch", 0), p.get("Arch")) for p in d["Packages"]] == [
        ("z", "1.2", "3.el9", 2, "x86_64"), ("a", "0.1", "1.el9", 0, None)]
    assert d["Packages"][0]["SrcName"] == "z" and d["Packages"][0]["SrcEpoch"] == 2
    apps = [(a["Type"], a["FilePath"], [(x["Name"], x["ID"]) for x in a["Libraries"]]) for a in d["Applications"]]
    assert apps == [("gomod", "go.sum", [("github.com/o/x", "github.com/o/x@v1.0.0")]),
                    ("jar", "", [("org.a:core", "org.a:core:2.0")]),
                    ("node-pkg", "", [("lodash", "lodash@4.17.0")])]
    bom["components"].append({"bom-ref": "os2", "type": "operating-system", "name": "x", "version": "1"})
    with pytest.raises(ts.SBOMError, match="multiple OS components are not supported"):
        ts.decode_cyclonedx(json.dumps(bom))
    bom["components"].pop()
    bom["components"].append({"bom-ref": "d1", "type": "library", "name": "d", "purl": "pkg:deb/debian/d@1"})
    with pytest.raises(ts.SBOMError, match="multiple types of OS packages"):
        ts.decode_cyclonedx(json.dumps(bom))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_sbom_scan_on_gpu(case):
    import trivy_amd
    d = _decode(case)
    eng = trivy_amd.Engine(trivy_amd.load_fixture_files(FX), 0)
    got = {}
    for cls, typ, _target, vulns in ts.scan(eng, d, now=NOW):
        got.setdefault((cls, typ), []).extend(vulns)
    _check(case, got)
