"""CPU: pins the FillInfo oracle (oracle/vulninfo.py) to the reference's own vectors:
every TestClient_FillInfo case (pkg/vulnerability/vulnerability_test.go:17-283) and the
FillInfo fields of every vulnerability in the integration goldens."""
import pytest

import fillinfo_golden as fg
import oracle.vulninfo as vi

_TABLE = fg.table_cases()
_INTEG = fg.integration_cases()


@pytest.mark.parametrize("case", _TABLE, ids=[c[0] for c in _TABLE])
def test_oracle_fillinfo_table(case):
    name, fixtures, vulns, want = case
    got = vi.fill_info(vi.vulnerability_bucket(fg.load_records(fixtures)), vulns)
    assert [fg.norm(v) for v in got] == [fg.norm(v) for v in want], name


def test_oracle_fillinfo_integration():
    bucket = vi.vulnerability_bucket(fg.load_records(fg.integration_fixtures()))
    assert len(_INTEG) >= 100
    for cid, inp, want in _INTEG:
        got = vi.fill_info(bucket, [inp])[0]
        assert fg.got_form(got) == fg.want_form(want), cid


def test_primary_url_rules():
    # vulnerability.go:136-157: ID prefixes first, then source prefixes in order, refs in order
    assert vi.get_primary_url("CVE-2020-1", [], "") == "https://avd.aquasec.com/nvd/cve-2020-1"
    assert vi.get_primary_url("TEMP-1", [], "debian") == "https://security-tracker.debian.org/tracker/TEMP-1"
    refs = ["https://lists.opensuse.org/b", "http://lists.opensuse.org/a"]
    assert vi.get_primary_url("SUSE-SU-1", refs, "suse-cvrf") == "http://lists.opensuse.org/a"
    assert vi.get_primary_url("SUSE-SU-1", refs, "debian") == ""
