"""ORACLE - TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the vulnerability part of the reference's result filter, the
step after FillInfo.  Used only by tests/ as the checker.

Restated from (fwereade/trivy @ 2025-01-14):
  pkg/result/filter.go:100-139   filterVulnerabilities (severity / status / ignore file /
                                 dedup on "vulnID/pkgName/installed/pkgPath")
  pkg/result/filter.go:345-348   shouldOverwrite (the greater FixedVersion string wins)
  pkg/result/filter.go:77        sort.Sort(types.BySeverity(...))
  pkg/types/vulnerability.go:41-58  BySeverity.Less
  pkg/result/ignore.go           IgnoreFinding / IgnoreConfig / ParseIgnoreFile / Prune /
                                 MatchVulnerability / parseIgnore (.trivyignore lines with
                                 exp:YYYY-MM-DD) / parseIgnoreYAML
  pkg/purl/purl.go:249-274       PackageURL.Match
and third-party semantics (absent here; pinned versions from reference go.mod):
  github.com/bmatcuk/doublestar/v4  Match(pattern, path): '/'-separated; '*' any run of
      non-'/' chars, '?' one non-'/' char, '[...]' classes ('!'/'^' negation, ranges),
      '{a,b}' alternatives, '**' as a whole path component matches zero or more
      components, '\\' escapes;
  github.com/package-url/packageurl-go  FromString: "pkg:" type "/" [namespace "/"] name
      ["@" version] ["?" qualifiers] ["#" subpath], type lower-cased, percent-decoding;
  trivy-db types.CompareSeverityString: by SeverityNames index (unknown names = UNKNOWN).

Pinned by TestFilter (pkg/result/filter_test.go:19-1040, transcribed to
tests/golden/tables/result__filter_test.json) - the vulnerability parts of its cases -
with the reference's own ignore files (pkg/result/testdata/.trivyignore{,.yaml}, copied as
data to tests/golden/result_files/).
"""
import datetime
import re
import urllib.parse

import yaml

SEVERITY = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]


# ---- doublestar v4 Match -------------------------------------------------------------------
def _glob_component(pat, s):
    """One path component against one pattern component (no '/')."""
    i = 0
    rx = ""
    while i < len(pat):
        c = pat[i]
        if c == "\\" and i + 1 < len(pat):
            rx += re.escape(pat[i + 1])
            i += 2
        elif c == "*":
            rx += "[^/]*"
            i += 1
        elif c == "?":
            rx += "[^/]"
            i += 1
        elif c == "[":
            j = pat.find("]", i + 2 if i + 1 < len(pat) and pat[i + 1] in "!^" else i + 1)
            if j < 0:
                return None  # invalid pattern: doublestar reports ErrBadPattern (no match)
            body = pat[i + 1:j]
            neg = body[:1] in ("!", "^")
            if neg:
                body = body[1:]
            rx += "[" + ("^" if neg else "") + body.replace("\\", "\\\\") + "]"
            i = j + 1
        elif c == "{":
            j = pat.find("}", i)
            if j < 0:
                return None
            alts = pat[i + 1:j].split(",")
            rx += "(?:" + "|".join(_alt_rx(a) for a in alts) + ")"
            i = j + 1
        else:
            rx += re.escape(c)
            i += 1
    return re.fullmatch(rx, s) is not None


def _alt_rx(a):
    out = ""
    for c in a:
        out += "[^/]*" if c == "*" else "[^/]" if c == "?" else re.escape(c)
    return out


def doublestar_match(pattern, path):
    pp, sp = pattern.split("/"), path.split("/")

    def rec(i, j):
        if i == len(pp):
            return j == len(sp)
        if pp[i] == "**":
            return any(rec(i + 1, k) for k in range(j, len(sp) + 1))
        if j == len(sp):
            return False
        m = _glob_component(pp[i], sp[j])
        return bool(m) and rec(i + 1, j + 1)

    return rec(0, 0)


# ---- package URLs --------------------------------------------------------------------------
def purl_from_string(s):
    if not s.startswith("pkg:"):
        raise ValueError("purl scheme is not \"pkg\": " + s)
    rest = s[4:].lstrip("/")
    subpath = ""
    if "#" in rest:
        rest, subpath = rest.split("#", 1)
        subpath = "/".join(urllib.parse.unquote(x) for x in subpath.strip("/").split("/") if x not in ("", ".", ".."))
    quals = {}
    if "?" in rest:
        rest, q = rest.split("?", 1)
        for kv in q.split("&"):
            if not kv:
                continue
            k, _, v = kv.partition("=")
            if v:
                quals[k.lower()] = urllib.parse.unquote(v)
    typ, _, rest = rest.partition("/")
    if not typ or not rest:
        raise ValueError("purl is missing type or name")
    version = ""
    if "@" in rest:
        rest, version = rest.rsplit("@", 1)
        version = urllib.parse.unquote(version)
    segs = [urllib.parse.unquote(x) for x in rest.strip("/").split("/")]
    name, ns = segs[-1], "/".join(x for x in segs[:-1] if x)
    return {"Type": typ.lower(), "Namespace": ns, "Name": name, "Version": version, "Qualifiers": quals,
            "Subpath": subpath}


def purl_match(p, target):
    """pkg/purl/purl.go:249-274 (target: {Type, Namespace, Name, Version, Qualifiers?, Subpath?})."""
    if target is None:
        return False
    if p["Type"] != target.get("Type", "") or p["Namespace"] != target.get("Namespace", ""):
        return False
    if p["Name"] != target.get("Name", ""):
        return False
    if p["Version"] and p["Version"] != target.get("Version", ""):
        return False
    if p["Subpath"] and p["Subpath"] != target.get("Subpath", ""):
        return False
    tq = target.get("Qualifiers") or {}
    if isinstance(tq, list):
        tq = {q["Key"]: q["Value"] for q in tq}
    return all(k in tq and tq[k] == v for k, v in p["Qualifiers"].items())


# ---- ignore files --------------------------------------------------------------------------
def _date(s):
    return datetime.datetime.strptime(s, "%Y-%m-%d").replace(tzinfo=datetime.timezone.utc)


def parse_ignore_text(text, now):
    """parseIgnore (.trivyignore): one ID per line, '#' comments, optional exp:YYYY-MM-DD;
    expired entries are pruned (Prune, ignore.go).  Returns IgnoreFinding dicts."""
    out = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        fields = line.split()
        exp = None
        if len(fields) > 1:  # getExpirationDate: the first "exp:" field of the line decides
            f = next((x for x in fields if x.startswith("exp:")), None)
            if f is not None:
                try:
                    exp = _date(f[4:])
                except ValueError:
                    continue  # logged and the line skipped
        out.append({"ID": fields[0], "Paths": [], "PURLs": [], "ExpiredAt": exp, "Statement": ""})
    return [f for f in out if f["ExpiredAt"] is None or not f["ExpiredAt"] < now]


def parse_ignore_yaml(text, now):
    doc = yaml.safe_load(text) or {}
    out = []
    for f in doc.get("vulnerabilities") or []:
        exp = f.get("expired_at")
        if isinstance(exp, datetime.date) and not isinstance(exp, datetime.datetime):
            exp = datetime.datetime(exp.year, exp.month, exp.day, tzinfo=datetime.timezone.utc)
        elif isinstance(exp, str):
            exp = _date(exp)
        out.append({"ID": str(f.get("id", "")), "Paths": list(f.get("paths") or []),
                    "PURLs": [purl_from_string(p) for p in f.get("purls") or []], "ExpiredAt": exp,
                    "Statement": f.get("statement", "") or ""})
    return [f for f in out if f["ExpiredAt"] is None or not f["ExpiredAt"] < now]


def match_vulnerability(findings, vuln_id, file_path, pkg_path, purl):
    """IgnoreConfig.MatchVulnerability: the first finding with this ID whose paths match the
    target or the package path and whose PURLs match the package."""
    for p in (file_path, pkg_path):
        for f in findings:
            if f["ID"] != vuln_id:
                continue
            if f["Paths"] and not any(doublestar_match(pat, p) for pat in f["Paths"]):
                continue
            if purl is not None and f["PURLs"] and not any(purl_match(x, purl) for x in f["PURLs"]):
                continue
            return f
    return None


# ---- filterVulnerabilities + BySeverity ------------------------------------------------------
def severity_index(s):
    return SEVERITY.index(s) if s in SEVERITY else 0


def by_severity_key(v):
    """types.BySeverity.Less as a sort key (pkg/types/vulnerability.go:41-58)."""
    sev = (v.get("Vulnerability") or {}).get("Severity", "")
    return (v.get("PkgName", "").encode(), v.get("InstalledVersion", "").encode(), -severity_index(sev),
            v.get("VulnerabilityID", "").encode(), v.get("PkgPath", "").encode())


def filter_vulnerabilities(target, vulns, severities, ignore_statuses=(), findings=()):
    """filter.go:100-139 + the BySeverity sort of FilterResult (:77).  severities: names.
    Returns (kept vulnerabilities in report order or None, ignored [(vuln, finding)])."""
    uniq, order, ignored = {}, [], []
    for v in vulns:
        v = dict(v)
        emb = dict(v.get("Vulnerability") or {})
        if not emb.get("Severity"):
            emb["Severity"] = "UNKNOWN"
        v["Vulnerability"] = emb
        if emb["Severity"] not in severities:
            continue
        if v.get("Status", 0) in ignore_statuses:
            continue
        purl = (v.get("PkgIdentifier") or {}).get("PURL")
        f = match_vulnerability(findings, v.get("VulnerabilityID", ""), target, v.get("PkgPath", ""), purl)
        if f is not None:
            ignored.append((v, f))
            continue
        key = "%s/%s/%s/%s" % (v.get("VulnerabilityID", ""), v.get("PkgName", ""), v.get("InstalledVersion", ""),
                               v.get("PkgPath", ""))
        old = uniq.get(key)
        if old is not None and not old.get("FixedVersion", "").encode() < v.get("FixedVersion", "").encode():
            continue
        if old is None:
            order.append(key)
        uniq[key] = v
    kept = sorted((uniq[k] for k in order), key=by_severity_key)
    return (kept or None), ignored
