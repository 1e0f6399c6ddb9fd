"""The VEX oracle (oracle/vex.py) against TestVEX_Filter (pkg/vex/vex_test.go:66-373) with the
reference's own VEX documents (pkg/vex/testdata, copied as data to tests/golden/vex/)."""
import json
import os

import pytest

from oracle import vex as ov

HERE = os.path.join(os.path.dirname(__file__), "golden", "vex")
TABLE = json.load(open(os.path.join(HERE, "cases.json")))


def load(case):
    rep = case.get("report") or {}
    text = open(os.path.join(HERE, case["file"])).read()
    return ov.VEX.new(text, rep.get("ArtifactType", ""), rep.get("SerialNumber", ""), rep.get("Version", 0))


@pytest.mark.parametrize("case", TABLE["cases"], ids=[c["name"] for c in TABLE["cases"]])
def test_vex_filter_table(case):
    if case.get("wantErr"):
        with pytest.raises(ov.VEXError, match=case["wantErr"]):
            load(case)
        return
    v = load(case)
    vulns = [TABLE["vulns"][k] for k in case["vulns"]]
    root = TABLE["boms"][case["bom"]] if case["bom"] else None
    assert v.filter(vulns, root) == [TABLE["vulns"][k] for k in case["want"]]


def test_cyclonedx_vex_needs_cyclonedx_sbom():
    """vex.go:71-73."""
    with pytest.raises(ov.VEXError, match="CycloneDX VEX can be used with CycloneDX SBOM"):
        ov.VEX.new(open(os.path.join(HERE, "cyclonedx.json")).read(), "container_image")


def test_purl_matches_go_vex_rules():
    """go-vex PurlMatches: versionless p1 matches any version; p1 qualifiers must be in p2 (unpinned
    by reference tests; the go-vex v0.2.5 rules as published)."""
    assert ov.purl_matches("pkg:oci/debian", "pkg:oci/debian@sha256:ab?tag=12")
    assert not ov.purl_matches("pkg:oci/debian@sha256:cd", "pkg:oci/debian@sha256:ab")
    assert not ov.purl_matches("pkg:deb/debian/bash@1?arch=amd64", "pkg:deb/debian/bash@1")
    assert ov.purl_matches("pkg:deb/debian/bash@1?arch=amd64", "pkg:deb/debian/bash@1?arch=amd64&distro=debian-12")
    assert not ov.purl_matches("not a purl", "pkg:deb/debian/bash@1")


def test_openvex_aliases_and_latest_statement():
    doc = {"@context": "https://openvex.dev/ns", "timestamp": "2023-01-16T19:07:16Z", "statements": [
        {"vulnerability": {"name": "GHSA-x", "aliases": ["CVE-1"]}, "products": [{"@id": "pkg:npm/a"}],
         "status": "not_affected", "timestamp": "2023-01-17T00:00:00Z"},
        {"vulnerability": {"name": "CVE-1"}, "products": [{"@id": "pkg:npm/a@1.0.0"}], "status": "affected"}]}
    v = ov.VEX.new(json.dumps(doc))
    vuln = {"VulnerabilityID": "CVE-1", "PkgIdentifier": {"PURL": ov.purl_from_string("pkg:npm/a@1.0.0")}}
    assert v.filter([vuln]) == []  # the later (by timestamp) not_affected statement wins
    vuln2 = dict(vuln, VulnerabilityID="CVE-2")
    assert v.filter([vuln2]) == [vuln2]
    no_purl = {"VulnerabilityID": "CVE-1", "PkgIdentifier": {}}
    assert v.filter([no_purl]) == [no_purl]
