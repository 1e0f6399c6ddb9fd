"""Seeded synthetic trivy-db bucket "vulnerability" (FillInfo tables) for a set of
vulnerability IDs: VendorSeverity over the sources FillInfo consults (data sources, GHSA,
NVD), DB Severity strings (incl. empty and non-standard ones), References hitting and
missing the primary-URL prefixes (vulnerability.go:15-39), CVSS/CWE/dates as detail.
A small share of records is undecodable (GetVulnerability errors are skipped by FillInfo)."""
import json

import numpy as np

SOURCES = ["nvd", "ghsa", "debian", "ubuntu", "redhat", "amazon", "suse-cvrf", "oracle-oval", "nodejs-security-wg",
           "ruby-advisory-db", "alpine"]
SEVERITIES = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]
REF_HOSTS = ["https://www.debian.org/security/", "http://www.debian.org/x/", "https://usn.ubuntu.com/",
             "https://access.redhat.com/errata/", "https://lists.opensuse.org/a/", "https://linux.oracle.com/errata/",
             "https://www.npmjs.com/advisories/", "https://hackerone.com/reports/", "https://groups.google.com/g/",
             "https://nvd.nist.gov/vuln/detail/", "https://github.com/advisories/", "http://example.com/"]


def vuln_values(ids, seed=11, bad=0.002):
    """[(id bytes, JSON value bytes)] for ids (bytes), deterministic in (ids, seed)."""
    rng = np.random.default_rng(seed)
    out = []
    for vid in ids:
        if rng.random() < bad:
            out.append((vid, b'{"Title":["not","a","string"]}'))
            continue
        d = {"Title": "t-" + vid.decode(), "Description": "synthetic"}
        r = rng.random()
        if r < 0.8:
            d["Severity"] = SEVERITIES[int(rng.integers(0, 5))]
        elif r < 0.9:
            d["Severity"] = "moderate"  # a non-standard DB string is passed through verbatim
        vs = {s: int(rng.integers(0, 5)) for s in SOURCES if rng.random() < 0.35}
        if vs:
            d["VendorSeverity"] = vs
        if rng.random() < 0.6:
            d["CVSS"] = {"nvd": {"V3Vector": "CVSS:3.1/AV:N", "V3Score": round(float(rng.random() * 10), 1)}}
        if rng.random() < 0.5:
            d["CweIDs"] = ["CWE-%d" % int(rng.integers(1, 900))]
        nref = int(rng.integers(0, 4))
        if nref:
            d["References"] = [REF_HOSTS[int(rng.integers(0, len(REF_HOSTS)))] + str(int(rng.integers(0, 1e6)))
                               for _ in range(nref)]
        if rng.random() < 0.7:
            d["PublishedDate"] = "20%02d-0%d-1%dT0%d:00:00Z" % (int(rng.integers(0, 24)), int(rng.integers(1, 9)),
                                                               int(rng.integers(0, 9)), int(rng.integers(0, 9)))
        out.append((vid, json.dumps(d, separators=(",", ":")).encode()))
    return out


def vuln_arena(ids, seed=11):
    """(n, depth=2, arena, off, len) for tvm_db_put_arena: bucket "vulnerability"."""
    from tools.synth import _arena
    items = []
    for vid, val in vuln_values(ids, seed):
        items += [b"vulnerability", vid, val]
    return _arena(items, 2)


def vuln_records(ids, seed=11):
    """The same bucket as fixture-format records (tests/golden/fixtures layout)."""
    return [{"path": ["vulnerability", vid.decode()], "value": val.decode()} for vid, val in vuln_values(ids, seed)]
