"""CPU: pins the result-filter oracle (oracle/filter.py) to TestFilter
(pkg/result/filter_test.go:19-1040): every case's vulnerability part - severities,
ignore-unfixed statuses, .trivyignore, .trivyignore.yaml (paths, PURLs, expiry), duplicate
handling - with the test's fixed clock (filter_test.go:1008) and the reference's own ignore
files.  Misconfiguration/secret/license filtering, Rego policies and VEX are not part of
this row; cases are compared on their vulnerability lists only."""
import datetime
import json
import os

import pytest

import oracle.filter as of

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NOW = datetime.datetime(2020, 8, 10, 7, 28, 17, 958, tzinfo=datetime.timezone.utc)
IGNORE_FILES = {"testdata/.trivyignore": "trivyignore", "testdata/.trivyignore.yaml": "trivyignore.yaml"}


def _cases():
    with open(os.path.join(GOLDEN, "tables", "result__filter_test.json"), encoding="utf-8") as f:
        cases = json.load(f)["tables"][0]["cases"]
    return [c for c in cases if not c["args"].get("policyFile") and not c["args"].get("vexPath")]


def findings_for(args):
    name = args.get("ignoreFile")
    if not name:
        return []
    with open(os.path.join(GOLDEN, "result_files", IGNORE_FILES[name]), encoding="utf-8") as f:
        text = f.read()
    return of.parse_ignore_yaml(text, NOW) if name.endswith(".yaml") else of.parse_ignore_text(text, NOW)


def _norm(vulns):
    out = []
    for v in vulns or []:
        v = json.loads(json.dumps(v))
        emb = v.get("Vulnerability") or {}
        out.append({k: x for k, x in v.items() if x not in ("", 0, None, {}, [])} | {"Vulnerability": emb})
    return out


_CASES = _cases()


@pytest.mark.parametrize("case", _CASES, ids=[c["name"] for c in _CASES])
def test_oracle_filter_cases(case):
    args = case["args"]
    sev = [of.SEVERITY[s] for s in args.get("severities") or []]
    st = args.get("ignoreStatuses") or []
    findings = findings_for(args)
    want_results = case["want"]["Results"]
    for r, w in zip(args["report"]["Results"], want_results):
        if not r.get("Vulnerabilities"):
            continue
        kept, ignored = of.filter_vulnerabilities(r.get("Target", ""), r["Vulnerabilities"], sev, st, findings)
        assert _norm(kept) == _norm(w.get("Vulnerabilities")), (case["name"], r.get("Target"))
        want_mod = [m for m in w.get("ModifiedFindings") or [] if m.get("Type") in (None, "vulnerability")]
        if want_mod:
            assert [m["Finding"]["VulnerabilityID"] for m in want_mod] == [v["VulnerabilityID"] for v, _ in ignored]
            assert [m.get("Statement", "") for m in want_mod] == [f["Statement"] for _, f in ignored]


def test_doublestar_and_purl():
    assert of.doublestar_match("**/*-lock.json", "foo/package-lock.json")
    assert of.doublestar_match("**/*-lock.json", "package-lock.json")
    assert not of.doublestar_match("bar/package.json", "foo/package-lock.json")
    assert of.doublestar_match("a/{b,c}/d", "a/c/d") and not of.doublestar_match("a/?/d", "a/bc/d")
    p = of.purl_from_string("pkg:golang/github.com/aquasecurity/bar")
    assert of.purl_match(p, {"Type": "golang", "Namespace": "github.com/aquasecurity", "Name": "bar", "Version": "2.3.4"})
    q = of.purl_from_string("pkg:rpm/redhat/curl@7.1?arch=x86_64")
    assert q["Qualifiers"] == {"arch": "x86_64"} and q["Version"] == "7.1"
