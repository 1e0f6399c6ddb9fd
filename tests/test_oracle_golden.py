"""CPU: pins the oracle to the reference's own test vectors.

The oracle (oracle/*.c + oracle/drivers.py) restates the third-party comparators
and the driver loops; these tests run it over the reference's fixtures and
driver test tables (tests/golden/) and require the exact expected results.
"""
import pytest

from conftest import canon

import oracle.drivers as od


import golden_tables as gt

_DETECT = [c for d in gt.OS_DRIVERS for c in gt.os_detect_cases(d)]
_SUPPORTED = [c for d in gt.OS_DRIVERS for c in gt.os_supported_cases(d)]


@pytest.mark.parametrize("case", _DETECT, ids=[c[0] for c in _DETECT])
def test_oracle_driver_cases(oracle_built, case):
    """Every TestScanner_Detect case of pkg/detector/ospkg/*/*_test.go against the oracle."""
    cid, fixtures, family, os_ver, repo, pkgs, want, want_err, now = case
    db = od.Records.from_files(fixtures)
    if want_err is not None:
        with pytest.raises(od.DecodeError) as ei:
            od.driver_detect(family, os_ver, repo, pkgs, db, now)
        assert want_err in str(ei.value), cid
    else:
        assert canon(od.driver_detect(family, os_ver, repo, pkgs, db, now)) == canon(want), cid


@pytest.mark.parametrize("case", _SUPPORTED, ids=[c[0] for c in _SUPPORTED])
def test_oracle_supported(case):
    cid, family, os_ver, now, want = case
    assert od.is_supported(family, os_ver, now) == want, cid


# dpkg orderings the reference fixtures/tests pin (debian_test.go, ubuntu_test.go,
# integration/testdata/fixtures/db/debian.yaml + debian-*.json.golden)
DEB_PINNED = [
    ("2.4.24", "2.4.25-1", -1),            # debian_test.go happy path: reported
    ("2.4.24", "2.2.22-13", 1),            # CVE-2012-3499 not reported
    ("2.9", "2:2.9-1ubuntu4.3", -1),       # ubuntu_test.go: epoch dominates
    ("2.9", "2.4-0ubuntu10", 1),           # CVE-2016-4476 not reported
]


@pytest.mark.parametrize("a,b,want", DEB_PINNED)
def test_oracle_deb_pinned(oracle_built, a, b, want):
    assert od.deb_cmp(a, b) == want


# Published go-deb-version / dpkg semantics (parity unpinned by reference tests,
# but these are the documented orderings of the algorithm being restated).
DEB_SEMANTICS = [
    ("1.0~rc1", "1.0", -1), ("1.0", "1.0-0", 0), ("1.0", "1.00", 0), ("1.0a", "1.0", 1),
    ("1.0.", "1.0", 1), ("1:0", "0:9", 1), ("1.0-0~", "1.0", -1), ("1.0~~", "1.0~", -1),
    ("1.0+b1", "1.0", 1), ("1.0-1", "1.0-1.1", -1), ("9223372036854775807", "99999999999999999999", 0),
]


@pytest.mark.parametrize("a,b,want", DEB_SEMANTICS)
def test_oracle_deb_semantics(oracle_built, a, b, want):
    assert od.deb_cmp(a, b) == want


@pytest.mark.parametrize("v", ["", "a1", "1.0 ", "-1:1.0", ":1.0", "1.0-a-b!", b"1.0\xff"])
def test_oracle_deb_invalid(oracle_built, v):
    assert not od.deb_valid(v)
