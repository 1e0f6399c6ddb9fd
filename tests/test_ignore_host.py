"""Host compile of ignore-file findings for the batch filter (trivy_amd/ignore.py) against
the oracle's IgnoreConfig.MatchVulnerability (oracle/filter.py, pinned by TestFilter)."""
import numpy as np
import pytest

import oracle.filter as of
from tools import synth_vex as sv
from trivy_amd.ignore import split_findings


def test_split_findings_vs_oracle():
    rng = np.random.default_rng(3)
    purls = [sv.purl_of("debian 12", "pkg%d" % (i % 30), "1.%d-1" % (i % 4), "amd64" if i % 3 else None)
             if i % 17 else None for i in range(300)]
    ids = ["CVE-2024-%04d" % k for k in range(20)]
    findings = []
    for k in range(60):
        pu = purls[int(rng.integers(len(purls)))] or "pkg:deb/debian/pkg1@1.1-1"
        base = pu.partition("?")[0]
        pats = [pu, base, base.rpartition("@")[0], base.rpartition("@")[0] + "?arch=amd64"]
        findings.append({"ID": ids[k % 20], "Paths": [], "PURLs": [pats[k % 4]] if k % 5 else [],
                         "ExpiredAt": None, "Statement": ""})
    plain, (pk, pid) = split_findings(findings, purls)
    got = {(i, v) for v in plain for i in range(len(purls))} | set(zip(pk.tolist(), pid))
    ofind = [dict(f, PURLs=[of.purl_from_string(x) for x in f["PURLs"]]) for f in findings]
    want = {(i, v) for i in range(len(purls)) for v in ids
            if of.match_vulnerability(ofind, v, "", "", of.purl_from_string(purls[i]) if purls[i] else None)}
    assert got == want and 0 < len(want) < len(purls) * len(ids)


def test_paths_rejected():
    with pytest.raises(ValueError, match="paths"):
        split_findings([{"ID": "CVE-1", "Paths": ["a/**"], "PURLs": []}], ["pkg:npm/a@1"])
