"""GPU: the reference's own driver test tables, through the C-ABI (HIP path only)."""
import pytest

from conftest import load_case_file, parse_now, canon

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("driver", ["debian", "ubuntu"])
def test_driver_cases(engine_factory, driver):
    from trivy_amd.detector.ospkg import Scanner, DetectError
    cf = load_case_file(driver)
    for case in cf["detect"]:
        eng = engine_factory(case["fixtures"])
        sc = Scanner(eng, driver)
        now = parse_now(case["now"]) if "now" in case else None
        if case.get("want_err"):
            with pytest.raises(DetectError) as ei:
                sc.detect(case["os_ver"], case.get("repo"), case["pkgs"], now=now)
            assert case["want_err"] in str(ei.value), case["name"]
        else:
            got = sc.detect(case["os_ver"], case.get("repo"), case["pkgs"], now=now)
            assert canon(got) == canon(case["want"]), case["name"]


def test_ospkg_detect_wraps_and_filters(engine_factory):
    """detect.go:63-82: gpg-pubkey filtered, errors wrapped, unsupported OS."""
    from trivy_amd.detector.ospkg import detect, DetectError, UnsupportedOSError
    eng = engine_factory(["ospkg/debian/debian.json", "ospkg/debian/data-source.json"])
    pkgs = [{"Name": "gpg-pubkey", "Version": "1", "SrcName": "apache2", "SrcVersion": "1.0"},
            {"Name": "htpasswd", "Version": "2.4.24", "SrcName": "apache2", "SrcVersion": "2.4.24"}]
    vulns, eosl = detect(eng, "debian", "9.1", None, pkgs, now=parse_now("2020-01-01T00:00:00Z"))
    assert {v["PkgName"] for v in vulns} == {"htpasswd"}
    assert sorted(v["VulnerabilityID"] for v in vulns) == ["CVE-2020-11985", "CVE-2021-31618"]
    assert eosl is False
    _, eosl = detect(eng, "debian", "9.1", None, pkgs, now=parse_now("2023-01-01T00:00:00Z"))
    assert eosl is True
    with pytest.raises(UnsupportedOSError):
        detect(eng, "plan9", "1", None, pkgs)
    bad = engine_factory(["ospkg/debian/invalid.json", "ospkg/debian/data-source.json"])
    with pytest.raises(DetectError, match="failed detection: failed to get debian advisories: failed to unmarshal"):
        detect(bad, "debian", "9.1", None, pkgs[1:])


def test_debian_parse_error_skips_before_lookup(engine_factory):
    """debian.go:66-70: an unparsable installed version never reaches the (poisoned) bucket."""
    from trivy_amd.detector.ospkg import Scanner
    eng = engine_factory(["ospkg/debian/invalid.json", "ospkg/debian/data-source.json"])
    pkgs = [{"Name": "htpasswd", "Version": "x", "SrcName": "apache2", "SrcVersion": "not-a-version"}]
    assert Scanner(eng, "debian").detect("9.1", None, pkgs) == []


def test_oracle_agrees_on_golden_cases(engine_factory, oracle_built):
    """The Python oracle drivers and the GPU path agree on every golden case."""
    import oracle.drivers as od
    from trivy_amd.detector.ospkg import Scanner
    from conftest import fixture_paths
    for driver in ["debian", "ubuntu"]:
        for case in load_case_file(driver)["detect"]:
            if case.get("want_err"):
                continue
            rec = od.Records.from_files(fixture_paths(case["fixtures"]))
            now = parse_now(case["now"]) if "now" in case else None
            want = (od.debian_detect(rec, case["os_ver"], case["pkgs"]) if driver == "debian"
                    else od.ubuntu_detect(rec, case["os_ver"], case["pkgs"], now))
            got = Scanner(engine_factory(case["fixtures"]), driver).detect(case["os_ver"], None, case["pkgs"], now=now)
            assert canon(got) == canon(want)
