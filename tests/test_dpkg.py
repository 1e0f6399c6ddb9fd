"""dpkg status parsing (trivy_amd/dpkg.py) pinned by Test_dpkgAnalyzer_Analyze
(pkg/fanal/analyzer/pkg/dpkg/dpkg_test.go:17-1470, transcribed to
tests/golden/tables/fanal__analyzer__pkg__dpkg__dpkg_test.json) with the reference's own
status files (testdata/{dpkg,corrupsed,dpkg_apt}, copied as data to tests/golden/dpkg/).
The "happy path with digests" and "info list" cases read other dpkg files (available /
md5sums digests, *.list installed files) that this parser does not cover.

GPU: the parsed Ubuntu 18.04 status file through ospkg.Detect on the GPU equals the
oracle's detection over the same packages."""
import datetime
import glob
import json
import os

import pytest

from conftest import canon
from trivy_amd import dpkg

HERE = os.path.join(os.path.dirname(__file__), "golden")
TABLE = json.load(open(os.path.join(HERE, "tables", "fanal__analyzer__pkg__dpkg__dpkg_test.json")))["tables"][0]
CASES = [c for c in TABLE["cases"] if c["name"] in ("valid", "corrupsed", "only apt")]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_parse_status_reference_cases(case):
    (src, path), = case["testFiles"].items()
    text = open(os.path.join(HERE, "dpkg", os.path.basename(src))).read()
    assert dpkg.parse_status(text, path) == case["want"]["PackageInfos"]


def test_mime_header_rules():
    h = dpkg.read_mime_header("package: a\nDescription: x\n  more\n\ty\nmulti-ARCH: same")
    assert h == {"Package": ["a"], "Description": ["x more y"], "Multi-Arch": ["same"]}
    with pytest.raises(dpkg.MIMEError):
        dpkg.read_mime_header("Package: a\nno colon here")
    with pytest.raises(dpkg.MIMEError):
        dpkg.read_mime_header(" leading: space")
    # a malformed block is skipped, its neighbours survive; deinstalled / purged are dropped
    text = ("Package: a\nVersion: 1.0-1\n\nPackage: b\nbroken line\nVersion: 1\n\n"
            "Package: c\nStatus: deinstall ok config-files\nVersion: 1\n\n"
            "Package: d\nStatus: purge ok not-installed\nVersion: 1\n\n"
            "Package: e\nSource: srce (2:3.0-4)\nVersion: 1:2.0-1\nDepends: a (>= 1) | z, a\n")
    got = dpkg.parse_status(text)[0]["Packages"]
    assert [p["Name"] for p in got] == ["a", "e"]
    e = got[1]
    assert (e["ID"], e["Epoch"], e["Version"], e["Release"]) == ("e@1:2.0-1", 1, "2.0", "1")
    assert (e["SrcName"], e["SrcEpoch"], e["SrcVersion"], e["SrcRelease"]) == ("srce", 2, "3.0", "4")
    assert e["DependsOn"] == ["a@1.0-1"]


@pytest.mark.gpu
def test_parsed_status_detects_like_oracle():
    import oracle.drivers as od
    import trivy_amd
    from trivy_amd.detector.ospkg import detect
    fx = sorted(glob.glob(os.path.join(HERE, "fixtures", "integration", "*.json")))
    pkgs = dpkg.parse_status(open(os.path.join(HERE, "dpkg", "dpkg")).read())[0]["Packages"]
    now = int(datetime.datetime(2021, 8, 25, tzinfo=datetime.timezone.utc).timestamp())
    eng = trivy_amd.Engine(trivy_amd.load_fixture_files(fx), 0)
    for fam, ver in (("ubuntu", "18.04"), ("debian", "10")):
        got, eosl = detect(eng, fam, ver, None, pkgs, now=now)
        want, weosl = od.detect(od.Records.from_files(fx), fam, ver, None, pkgs, now)
        assert canon(got) == canon(want) and eosl == weosl, fam
