"""Alpine installed-database parsing (trivy_amd/apk.py) pinned by TestParseApkInfo
(pkg/fanal/analyzer/pkg/apk/apk_test.go:14-440, transcribed to
tests/golden/tables/fanal__analyzer__pkg__apk__apk_test.json) with the reference's own
database file (testdata/apk, copied as data to tests/golden/apk/installed).  Licenses are
compared before the licensing.Normalize alias step, which this mirror leaves out.

GPU: the parsed packages through ospkg.Detect (alpine 3.10) on the GPU equal the oracle."""
import datetime
import glob
import json
import os

import pytest

from conftest import canon
from trivy_amd import apk

HERE = os.path.join(os.path.dirname(__file__), "golden")
CASE = json.load(open(os.path.join(HERE, "tables", "fanal__analyzer__pkg__apk__apk_test.json")))["tables"][0]["cases"][0]


def _parsed():
    return apk.parse_installed(open(os.path.join(HERE, "apk", "installed")).read())


def test_parse_installed_reference_case():
    infos, files = _parsed()
    got = [{k: v for k, v in p.items() if k != "Licenses"} for p in infos[0]["Packages"]]
    want = [{k: v for k, v in p.items() if k != "Licenses"} for p in CASE["wantPkgs"]]
    assert got == want
    assert files == CASE["wantFiles"]
    # the raw license tokens line up with the normalised ones the reference expects
    assert [len(p.get("Licenses") or []) > 0 for p in infos[0]["Packages"]] == \
        [len(p.get("Licenses") or []) > 0 for p in CASE["wantPkgs"]]


def test_parse_rules():
    text = ("P:a\nV:1.0-r0\np:so:liba.so.1=1 cmd:a\n\nP:b\nV:invalid\n\nP:c\nV:2.0-r1\no:cc\nD:so:liba.so.1 !x a>=1\n"
            "C:Q1ypLbtFv6AH2L0s9uRo6nWbwqUhA=\nF:usr/bin\nR:../bin/c\n\nP:a\nV:9-r0\n")
    (info,), files = apk.parse_installed(text)
    pk = info["Packages"]
    assert [p["ID"] for p in pk] == ["a@1.0-r0", "c@2.0-r1"]  # invalid version dropped, first "a" wins
    assert pk[1]["SrcName"] == "cc" and pk[1]["SrcVersion"] == "2.0-r1"
    assert pk[1]["DependsOn"] == ["a@1.0-r0", "a@9-r0"]  # so:liba.so.1 via provides; "a" via the later block
    assert pk[1]["Digest"].startswith("sha1:") and files == ["usr/bin/c"]


@pytest.mark.gpu
def test_parsed_installed_detects_like_oracle():
    import oracle.drivers as od
    import trivy_amd
    from trivy_amd.detector.ospkg import detect
    fx = sorted(glob.glob(os.path.join(HERE, "fixtures", "integration", "*.json")))
    pkgs = _parsed()[0][0]["Packages"]
    now = int(datetime.datetime(2021, 8, 25, tzinfo=datetime.timezone.utc).timestamp())
    eng = trivy_amd.Engine(trivy_amd.load_fixture_files(fx), 0)
    for ver in ("3.10.2", "3.9.1"):
        got, eosl = detect(eng, "alpine", ver, None, pkgs, now=now)
        want, weosl = od.detect(od.Records.from_files(fx), "alpine", ver, None, pkgs, now)
        assert canon(got) == canon(want) and eosl == weosl, ver
