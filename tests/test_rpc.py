"""Twirp wire format of packages and vulnerabilities (trivy_amd/rpc.py), pinned by the
reference's conversion tests (pkg/rpc/convert_test.go TestConvertToRpcPkgs,
TestConvertFromRpcPkgs, TestConvertToRpcVulns; transcribed as data in
tests/golden/rpc/convert_cases.json).  The expected RPC messages are compared field by
field (protobuf json_format with proto field names); every message also round-trips
through its binary wire encoding.

GPU: a Result carrying the reference's dpkg status packages goes through the GPU detector
and comes back with the same vulnerabilities as the oracle."""
import json
import os

import pytest
from google.protobuf import json_format

from trivy_amd import rpc

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rpc", "convert_cases.json")))


def _msg(m):
    return json_format.MessageToDict(m, preserving_proto_field_name=True)


def _wire(m):
    return type(m).FromString(m.SerializeToString())


@pytest.mark.parametrize("case", CASES["pkgs"], ids=lambda c: c["name"])
def test_to_rpc_pkgs(case):
    (got,) = rpc.to_rpc_pkgs([case["go"]])
    assert _msg(got) == case["rpc"]
    assert _wire(got) == got


@pytest.mark.parametrize("case", CASES["pkgs"], ids=lambda c: c["name"])
def test_from_rpc_pkgs(case):
    m = json_format.ParseDict(case["rpc"], rpc.Package())
    assert rpc.from_rpc_pkgs([_wire(m)]) == [case["go"]]


@pytest.mark.parametrize("case", CASES["vulns"], ids=lambda c: c["name"])
def test_to_rpc_vulns(case):
    (got,) = rpc.to_rpc_vulns([case["go"]])
    assert _msg(got) == case["rpc"]
    assert _wire(got) == got


def test_vulns_round_trip():
    """ConvertFromRPCVulns(ConvertToRPCVulns(v)) keeps every field the wire carries."""
    v = dict(CASES["vulns"][0]["go"], VendorIDs=["RHSA-2019:1"], PkgID="foo@1.2.3", PkgPath="a/b", Status=3,
             SeveritySource="redhat", CweIDs=["CWE-79"], PkgIdentifier={"PURL": "pkg:maven/a/foo@1.2.3"},
             Custom={"x": [1.0, "y"]})
    (back,) = rpc.from_rpc_vulns([_wire(m) for m in rpc.to_rpc_vulns([v])])
    assert back == v
    (inv,) = rpc.from_rpc_vulns(rpc.to_rpc_vulns([CASES["vulns"][1]["go"]]))
    assert inv["Severity"] == "UNKNOWN"  # dbTypes.NewSeverity error -> Severity_UNKNOWN


def test_result_wire():
    raw = rpc.encode_result("debian:12 (debian 12)", "os-pkgs", "debian", [CASES["pkgs"][0]["go"]],
                            [CASES["vulns"][0]["go"]])
    r = rpc.decode_result(raw)
    assert r["Target"] == "debian:12 (debian 12)" and r["Class"] == "os-pkgs" and r["Type"] == "debian"
    assert r["Packages"] == [CASES["pkgs"][0]["go"]] and r["Vulnerabilities"] == [CASES["vulns"][0]["go"]]


@pytest.mark.gpu
def test_detect_scan_result_like_oracle():
    import datetime
    import glob

    import oracle.drivers as od
    import trivy_amd
    from conftest import canon
    from trivy_amd import dpkg
    here = os.path.join(os.path.dirname(__file__), "golden")
    fx = sorted(glob.glob(os.path.join(here, "fixtures", "integration", "*.json")))
    pkgs = dpkg.parse_status(open(os.path.join(here, "dpkg", "dpkg")).read())[0]["Packages"]
    now = int(datetime.datetime(2021, 8, 25, tzinfo=datetime.timezone.utc).timestamp())
    eng = trivy_amd.Engine(trivy_amd.load_fixture_files(fx), 0)
    raw = rpc.encode_result("ubuntu:18.04", "os-pkgs", "ubuntu", pkgs)
    got = rpc.decode_result(rpc.detect_scan_result(eng, raw, "ubuntu", "18.04", now=now))["Vulnerabilities"]
    want, _ = od.detect(od.Records.from_files(fx), "ubuntu", "18.04", None, rpc.from_rpc_pkgs(rpc.to_rpc_pkgs(pkgs)), now)
    assert len(want) > 0
    assert canon(got) == canon(rpc.from_rpc_vulns(rpc.to_rpc_vulns(want)))
