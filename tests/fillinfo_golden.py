"""FillInfo golden vectors (test infrastructure): the reference's TestClient_FillInfo
table (pkg/vulnerability/vulnerability_test.go:17-283) and the cases harvested from the
integration goldens (tests/golden/make_fillinfo_cases.py), plus the comparison form."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
VULN_FIELDS = ("Title", "Description", "Severity", "CweIDs", "VendorSeverity", "CVSS", "References",
               "PublishedDate", "LastModifiedDate")


def _unwrap(x):
    if isinstance(x, dict) and x.get("__call__") == "utils.MustTimeParse":
        return x["args"][0]
    return x


def norm(v):
    """DetectedVulnerability dict -> comparison form: the embedded Vulnerability's fields
    and the FillInfo-touched fields, Go zero values dropped at struct level only (a map
    value 0, e.g. VendorSeverity{"nvd": 0}, is kept)."""
    out = {k: v[k] for k in ("VulnerabilityID", "Status", "SeveritySource", "PrimaryURL", "FixedVersion",
                             "DataSource") if v.get(k)}
    emb = v.get("Vulnerability") or {}
    out["Vulnerability"] = {k: _unwrap(emb[k]) for k in VULN_FIELDS if emb.get(k) not in (None, "", [], {})}
    return out


def table_cases():
    """(id, fixture files, input vulns, expected vulns) of TestClient_FillInfo."""
    with open(os.path.join(GOLDEN, "tables", "vulnerability__vulnerability_test.json"), encoding="utf-8") as f:
        t = json.load(f)["tables"][0]
    out = []
    for c in t["cases"]:
        fx = [os.path.join(GOLDEN, "fixtures", "vulnerability", os.path.basename(p)[:-5] + ".json")
              for p in c["fixtures"]]
        out.append((c["name"], fx, c["vulns"], c["expectedVulnerabilities"]))
    return out


def integration_cases():
    """(id, input vuln, want) harvested from integration/testdata/*.json.golden."""
    with open(os.path.join(GOLDEN, "fillinfo_integration.json"), encoding="utf-8") as f:
        cases = json.load(f)
    return [(f"{c['golden']}:{c['input']['VulnerabilityID']}:{i}", c["input"], c["want"])
            for i, c in enumerate(cases)]


def integration_fixtures():
    return [os.path.join(GOLDEN, "fixtures", "integration", "vulnerability.json")]


def want_form(want):
    """The harvested `want` in norm() form (FixedVersion/DataSource/ID come from the input)."""
    out = {k: want[k] for k in ("Status", "SeveritySource", "PrimaryURL") if want.get(k)}
    vul = dict(want.get("Vulnerability") or {})
    if want.get("Severity"):
        vul["Severity"] = want["Severity"]
    out["Vulnerability"] = vul
    return out


def got_form(got):
    """norm() of a FillInfo output as the golden report shows it: result.Filter, which runs
    between FillInfo and the report, turns an empty Severity into UNKNOWN
    (pkg/result/filter.go:114-117)."""
    n = norm(got)
    n["Vulnerability"].setdefault("Severity", "UNKNOWN")
    for k in ("VulnerabilityID", "FixedVersion", "DataSource"):
        n.pop(k, None)
    return n


def load_records(paths):
    recs = []
    for p in paths:
        with open(p, encoding="utf-8") as f:
            recs += json.load(f)
    return recs
