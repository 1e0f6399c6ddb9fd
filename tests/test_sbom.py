"""SBOM decode (trivy_amd/sbom.py, mirror of pkg/sbom) pinned by the reference's SBOM
integration tests (integration/sbom_test.go:30-153): the three CycloneDX SBOMs, and the
centos-7 image as an in-toto attestation, SPDX tag-value and SPDX JSON, decoded and run
through the detectors must give every golden's detector-produced vulnerabilities.

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
    return ts.decode(open(os.path.join(HERE, "sbom", case["sbom"])).read())


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


def test_spdx_rules():
    """unmarshal.go details: type by SPDXID prefix, purl only from PACKAGE-MANAGER/purl refs,
    "built package from:" source (rpm epoch:version-release), DESCRIBES skipped, edges only
    between packages, the Trivy-legacy application (path in sourceInfo, type in name),
    multi-line <text> values."""
    tv = """SPDXVersion: SPDX-2.3
SPDXID: SPDXRef-DOCUMENT
Creator: Tool: trivy-0.40
PackageName: alma
SPDXID: SPDXRef-OperatingSystem-1
PackageVersion: 9.2
PackageName: z
SPDXID: SPDXRef-Package-1
PackageVersion: 1.2
PackageSourceInfo: <text>built package from: zsrc 3:1.2-3.el9</text>
ExternalRef: SECURITY cpe23Type cpe:2.3:a:z:z:1.2
ExternalRef: PACKAGE-MANAGER purl pkg:rpm/alma/z@1.2-3.el9?arch=x86_64
PackageAttributionText: <text>PkgID: z@1.2-3.el9.x86_64</text>
PackageName: gomod
SPDXID: SPDXRef-Application-1
PackageSourceInfo: app/go.mod
PackageName: x
SPDXID: SPDXRef-Package-2
PackageVersion: 1.0.0
ExternalRef: PACKAGE-MANAGER purl pkg:golang/github.com/o/x@1.0.0
FileName: app/go.mod
SPDXID: SPDXRef-File-1
Relationship: SPDXRef-DOCUMENT DESCRIBES SPDXRef-OperatingSystem-1
Relationship: SPDXRef-OperatingSystem-1 CONTAINS SPDXRef-Package-1
Relationship: SPDXRef-Application-1 DEPENDS_ON SPDXRef-Package-2
Relationship: SPDXRef-Application-1 CONTAINS SPDXRef-File-1
"""
    d = ts.decode(tv)
    assert d["OS"] == {"Family": "alma", "Name": "9.2"} and d["Root"]["name"] == "alma"
    (z,) = d["Packages"]
    assert (z["Name"], z["Version"], z["Release"], z["ID"]) == ("z", "1.2", "3.el9", "z@1.2-3.el9.x86_64")
    assert (z["SrcName"], z["SrcEpoch"], z["SrcVersion"], z["SrcRelease"]) == ("zsrc", 3, "1.2", "3.el9")
    (app,) = d["Applications"]
    assert app["Type"] == "gomod" and app["FilePath"] == "app/go.mod"
    assert [lib["Name"] for lib in app["Libraries"]] == ["x"]  # pkgName: the SPDX name (no group)
    with pytest.raises(ts.SBOMError):
        ts.decode("not an sbom")
    with pytest.raises(ts.SBOMError):
        ts.decode_intoto('{"payloadType": "text/plain", "payload": ""}')


# pkg/sbom/spdx/unmarshal_test.go:20-338, the fields this decoder produces, transcribed as
# data; the inputs are the reference's spdx/testdata/happy files (tests/golden/sbom/spdx_happy)
_L3 = "sha256:3c79e832b1b4891a1cb4a326ef8524e0bd14a2537150ac0e203a5677176c1ca1"
_YARGS = {"Type": "node-pkg", "FilePath": "", "Libraries": [
    {"ID": "yargs-parser@21.1.1", "Name": "yargs-parser", "Version": "21.1.1",
     "FilePath": "node_modules/yargs-parser/package.json"}]}
SPDX_HAPPY = {
    "bom.json": {"OS": {"Family": "alpine", "Name": "3.16.0"},
                 "Packages": [{"ID": "musl@1.2.3-r0", "Name": "musl", "Version": "1.2.3-r0", "SrcName": "musl",
                               "SrcVersion": "1.2.3-r0",
                               "Layer": "sha256:dd565ff850e7003356e2b252758f9bdc1ff2803f61e995e24c7844f6297f8fc3"}],
                 "Applications": [
                     {"Type": "composer", "FilePath": "app/composer/composer.lock", "Libraries": [
                         {"ID": "pear/log@1.13.1", "Name": "pear/log", "Version": "1.13.1", "Layer": _L3},
                         {"ID": "pear/pear_exception@v1.0.0", "Name": "pear/pear_exception", "Version": "v1.0.0",
                          "Layer": _L3}]},
                     {"Type": "gobinary", "FilePath": "app/gobinary/gobinary", "Libraries": [
                         {"ID": "github.com/package-url/packageurl-go@v0.1.1-0.20220203205134-d70459300c8a",
                          "Name": "github.com/package-url/packageurl-go",
                          "Version": "v0.1.1-0.20220203205134-d70459300c8a", "Layer": _L3}]},
                     {"Type": "jar", "FilePath": "", "Libraries": [
                         {"ID": "org.codehaus.mojo:child-project:1.0", "Name": "org.codehaus.mojo:child-project",
                          "Version": "1.0", "Layer": _L3}]},
                     {"Type": "node-pkg", "FilePath": "", "Libraries": [
                         {"ID": "bootstrap@5.0.2", "Name": "bootstrap", "Version": "5.0.2", "Layer": _L3}]}]},
    "with-hasfiles-bom.json": {"OS": None, "Packages": [], "Applications": [_YARGS]},
    "with-files-in-relationships-bom.json": {"OS": None, "Packages": [], "Applications": [_YARGS]},
    "with-file-as-relationship-parent.json": {"OS": None, "Packages": [], "Applications": []},
    "os-only-bom.json": {"OS": {"Family": "alpine", "Name": "3.16.0"}, "Packages": [], "Applications": []},
    "empty-bom.json": {"OS": None, "Packages": [], "Applications": []},
}
_PKG_KEYS = ("ID", "Name", "Version", "SrcName", "SrcVersion", "FilePath")


def _pkg_view(p):
    v = {k: p[k] for k in _PKG_KEYS if p.get(k)}
    if (p.get("Layer") or {}).get("DiffID"):
        v["Layer"] = p["Layer"]["DiffID"]
    return v


@pytest.mark.parametrize("name", sorted(SPDX_HAPPY))
def test_spdx_unmarshal_happy(name):
    """SPDX JSON decode, incl. file paths from hasFiles / CONTAINS-File relationships
    (unmarshal.go:107-132, 187-195 -> decode.go:224-227), vs unmarshal_test.go."""
    want = SPDX_HAPPY[name]
    d = ts.decode(open(os.path.join(HERE, "sbom", "spdx_happy", name)).read())
    os_ = d["OS"] if d["OS"] and d["OS"].get("Family") else None
    assert os_ == want["OS"]
    assert [_pkg_view(p) for p in d["Packages"]] == want["Packages"]
    got_apps = [{"Type": a["Type"], "FilePath": a["FilePath"], "Libraries": [_pkg_view(x) for x in a["Libraries"]]}
                for a in d["Applications"]]
    assert got_apps == want["Applications"]


def test_decode_malformed_json_is_sbom_error():
    """sbom.go DetectFormat: input that starts like JSON but does not decode is no known
    format - an SBOMError, like every other decode failure."""
    for text in ('{"bomFormat": "CycloneDX", ', "{not json}\n{", "[1, 2]"):
        with pytest.raises(ts.SBOMError, match="failed to detect SBOM format"):
            ts.decode(text)
