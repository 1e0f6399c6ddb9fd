"""ORACLE - TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's VEX filter, the last step of result.Filter
(SURVEY.md §8f rank 2).  Used only by tests/ as the checker; nothing under trivy_amd/
imports it.

Restated from (fwereade/trivy @ 2025-01-14):
  pkg/vex/vex.go:28-106        New (CycloneDX JSON, then OpenVEX, then CSAF; "unable to
                               load VEX"), decodeCycloneDXJSON ("CycloneDX VEX can be used
                               with CycloneDX SBOM")
  pkg/vex/openvex.go:21-54     OpenVEX.Filter / Matches: statements for (vuln, root PURL,
                               [pkg PURL]) first, else (vuln, pkg PURL); the LAST statement
                               after the timestamp sort decides; not_affected/fixed drop
  pkg/vex/cyclonedx.go:48-84   CycloneDX.Filter: the FIRST statement with the vuln ID;
                               BOM-Link affects must name the SBOM's serial/version and
                               match the package (PkgIdentifier.Match)
  pkg/vex/csaf.go:27-138       CSAF.Filter: the FIRST vulnerability with the CVE; product
                               status known_not_affected / fixed, products' helper PURLs
                               and default_component_of / installed_on / installed_with
                               relationships (purl.Match)
  pkg/result/filter.go:38-104  filterByVEX runs after FilterResult (dedup + BySeverity)
  pkg/fanal/types/artifact.go:160-175  PkgIdentifier.Match
and third-party semantics (absent here; pins from reference go.mod):
  github.com/openvex/go-vex v0.2.5 (go.mod:84)  VEX.Matches (statements lacking a
      timestamp take the document's; stable sort by timestamp), Statement.Matches,
      Vulnerability.Matches (name or aliases), Component.Matches (@id equality or
      PurlMatches, identifiers, hashes), PurlMatches (no version in p1 = any version;
      p1's qualifiers must be present with equal values in p2);
  github.com/CycloneDX/cyclonedx-go  ParseBOMLink: urn:cdx:<uuid>/<version>#<ref>;
  github.com/csaf-poc/csaf_distribution/v3  ProductTree.CollectProductIdentificationHelpers
      (full_product_names, branches recursively, relationships' full_product_name).
Pinned by TestVEX_Filter (pkg/vex/vex_test.go:66-373, transcribed to
tests/golden/vex/cases.json) with the reference's own VEX documents (pkg/vex/testdata,
copied as data to tests/golden/vex/).  Unpinned by reference tests (stated choices):
PURL qualifiers compare as a key->value map; Go's random map order between
known_not_affected and fixed in CSAF only changes the ModifiedFinding status, never
whether the finding is dropped.
"""
import datetime
import json
import re
import urllib.parse

from oracle.filter import purl_from_string, purl_match


class VEXError(Exception):
    pass


def _parse_purl(s):
    try:
        return purl_from_string(s)
    except (ValueError, AttributeError):
        return None


def _ts(s):
    """RFC 3339 (nanoseconds allowed) -> integer nanoseconds since the epoch (UTC)."""
    m = re.fullmatch(r"(\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d)(?:\.(\d{1,9}))?(Z|[+-]\d\d:\d\d)", s or "")
    if not m:
        return None
    base = datetime.datetime.strptime(m.group(1), "%Y-%m-%dT%H:%M:%S").replace(tzinfo=datetime.timezone.utc)
    ns = int((m.group(2) or "0").ljust(9, "0"))
    off = 0
    if m.group(3) != "Z":
        sign = 1 if m.group(3)[0] == "+" else -1
        off = sign * (int(m.group(3)[1:3]) * 3600 + int(m.group(3)[4:6]) * 60)
    return (int(base.timestamp()) - off) * 1_000_000_000 + ns


# ---- go-vex v0.2.5 -------------------------------------------------------------------------
def purl_matches(p1s, p2s):
    """go-vex PurlMatches(purl1 general, purl2 specific)."""
    p1, p2 = _parse_purl(p1s), _parse_purl(p2s)
    if p1 is None or p2 is None:
        return False
    if p1["Type"] != p2["Type"] or p1["Namespace"] != p2["Namespace"] or p1["Name"] != p2["Name"]:
        return False
    if p1["Version"] and p1["Version"] != p2["Version"]:
        return False
    return all(k in p2["Qualifiers"] and p2["Qualifiers"][k] == v for k, v in p1["Qualifiers"].items())


def component_matches(c, ident):
    cid = c.get("@id", "") or ""
    if cid and cid == ident:
        return True
    if purl_matches(cid, ident):
        return True
    for t, v in (c.get("identifiers") or {}).items():
        if v == ident or (t == "purl" and purl_matches(v, ident)):
            return True
    return any(h == ident for h in (c.get("hashes") or {}).values())


def statement_matches(st, vuln, product, subcomponents):
    v = st.get("vulnerability") or {}
    if not (v.get("name") == vuln or vuln in (v.get("aliases") or [])):
        return False
    for p in st.get("products") or []:
        if not subcomponents and component_matches(p, product):
            return True
        if not component_matches(p, product):
            continue
        for c in p.get("subcomponents") or []:
            if any(component_matches(c, sc) for sc in subcomponents):
                return True
    return False


def openvex_matches(doc, vuln, product, subcomponents):
    doc_ts = _ts(doc.get("timestamp"))
    out = [st for st in doc.get("statements") or [] if statement_matches(st, vuln, product, subcomponents)]
    key = [(_ts(st["timestamp"]) if st.get("timestamp") else doc_ts) for st in out]
    order = sorted(range(len(out)), key=lambda i: key[i])  # stable
    return [out[i] for i in order]


# ---- CycloneDX BOM-Link ----------------------------------------------------------------------
_BOMLINK = re.compile(r"urn:cdx:([0-9a-f]{8}-[0-9a-f]{4}-[1-5][0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12})/([1-9]\d*)"
                      r"(?:#([0-9a-zA-Z\-._~%!$&'()*+,;=:@/?]+))?")

CDX_STATUS = {"resolved": "fixed", "resolved_with_pedigree": "fixed", "exploitable": "affected",
              "in_triage": "under_investigation", "false_positive": "not_affected", "not_affected": "not_affected"}


def parse_bom_link(s):
    m = _BOMLINK.fullmatch(s or "")
    if not m:
        return None
    return "urn:uuid:" + m.group(1), int(m.group(2)), urllib.parse.unquote(m.group(3) or "")


def pkg_identifier_match(pid, s):
    """PkgIdentifier.Match (artifact.go:160-175): BOMRef or the PURL, PURL strings normalised."""
    parsed = _parse_purl(s) if s.startswith("pkg:") else None
    if pid.get("BOMRef", "") == s:
        return True
    purl = pid.get("PURL")
    if purl is None:
        return False
    if parsed is not None:
        return _purl_key(parsed) == _purl_key(purl)
    return False


def _purl_key(p):
    q = p.get("Qualifiers") or {}
    if isinstance(q, list):
        q = {x["Key"]: x["Value"] for x in q}
    return (p.get("Type", ""), p.get("Namespace", ""), p.get("Name", ""), p.get("Version", ""),
            tuple(sorted(q.items())), p.get("Subpath", ""))


def purl_string(p):
    """A PURL dict -> a string purl_from_string reads back to the same key."""
    q = p.get("Qualifiers") or {}
    if isinstance(q, list):
        q = {x["Key"]: x["Value"] for x in q}
    s = "pkg:" + p["Type"] + "/"
    if p.get("Namespace"):
        s += "/".join(urllib.parse.quote(x, safe="") for x in p["Namespace"].split("/")) + "/"
    s += urllib.parse.quote(p["Name"], safe="")
    if p.get("Version"):
        s += "@" + urllib.parse.quote(p["Version"], safe="")
    if q:
        s += "?" + "&".join(k + "=" + urllib.parse.quote(v, safe="") for k, v in sorted(q.items()))
    if p.get("Subpath"):
        s += "#" + p["Subpath"]
    return s


# ---- CSAF -------------------------------------------------------------------------------------
def csaf_helpers(tree, pid):
    out = []
    for f in (tree or {}).get("full_product_names") or []:
        if f and f.get("product_id") == pid and f.get("product_identification_helper"):
            out.append(f["product_identification_helper"])

    def rec(b):
        if not b:
            return
        f = b.get("product")
        if f and f.get("product_id") == pid and f.get("product_identification_helper"):
            out.append(f["product_identification_helper"])
        for c in b.get("branches") or []:
            rec(c)

    for b in (tree or {}).get("branches") or []:
        rec(b)
    for r in (tree or {}).get("relationships") or []:
        f = (r or {}).get("full_product_name")
        if f and f.get("product_id") == pid and f.get("product_identification_helper"):
            out.append(f["product_identification_helper"])
    return [p for p in (_parse_purl(h["purl"]) for h in out if h.get("purl")) if p is not None]


def csaf_sub_purls(tree, pid):
    out = []
    for r in (tree or {}).get("relationships") or []:
        if r and r.get("category") in ("default_component_of", "installed_on", "installed_with") and \
                (r.get("full_product_name") or {}).get("product_id") == pid:
            out += csaf_helpers(tree, r.get("product_reference"))
    return out


def csaf_status(doc, vuln, purl):
    ps = vuln.get("product_status")
    if purl is None or ps is None:
        return ""
    for status, products in (("not_affected", ps.get("known_not_affected") or []), ("fixed", ps.get("fixed") or [])):
        for prod in products:
            if any(purl_match(p, purl) for p in csaf_helpers(doc.get("product_tree"), prod)):
                return status
            if any(purl_match(p, purl) for p in csaf_sub_purls(doc.get("product_tree"), prod)):
                return status
    return ""


# ---- vex.New + Filter -------------------------------------------------------------------------
class VEX:
    def __init__(self, kind, doc, bom_serial="", bom_version=0):
        self.kind, self.doc, self.serial, self.version = kind, doc, bom_serial, bom_version

    @classmethod
    def new(cls, text, artifact_type="", bom_serial="", bom_version=0):
        """vex.New over the document text; report = (ArtifactType, BOM serial, BOM version)."""
        try:
            doc = json.loads(text)
        except ValueError:
            doc = None
        if isinstance(doc, dict) and doc.get("bomFormat") == "CycloneDX":
            if artifact_type != "cyclonedx":
                raise VEXError("CycloneDX VEX can be used with CycloneDX SBOM")
            return cls("cyclonedx", doc, bom_serial, bom_version)
        if isinstance(doc, dict) and doc.get("@context"):
            return cls("openvex", doc)
        if isinstance(doc, dict) and doc.get("vulnerabilities") is not None:
            return cls("csaf", doc)
        raise VEXError("unable to load VEX")

    def keep(self, vuln, root_purl=None):
        """True when the detected vulnerability survives the filter."""
        pid = vuln.get("PkgIdentifier") or {}
        purl = pid.get("PURL")
        vid = vuln.get("VulnerabilityID", "")
        if self.kind == "openvex":
            if purl is None:
                return True
            ps = purl_string(purl)
            stmts = []
            if root_purl is not None:
                stmts = openvex_matches(self.doc, vid, purl_string(root_purl), [ps])
            if not stmts:
                stmts = openvex_matches(self.doc, vid, ps, [])
            return not (stmts and stmts[-1].get("status") in ("not_affected", "fixed"))
        if self.kind == "cyclonedx":
            st = next((v for v in self.doc.get("vulnerabilities") or [] if v.get("id") == vid), None)
            if st is None:
                return True
            status = CDX_STATUS.get((st.get("analysis") or {}).get("state"), "unknown")
            for a in st.get("affects") or []:
                link = parse_bom_link(a.get("ref"))
                if link is None or link[0] != self.serial or link[1] != self.version:
                    continue
                if pkg_identifier_match(pid, link[2]) and status in ("not_affected", "fixed"):
                    return False
            return True
        found = next((v for v in self.doc.get("vulnerabilities") or [] if v.get("cve") == vid), None)
        if found is None:
            return True
        return csaf_status(self.doc, found, purl) == ""

    def filter(self, vulns, root_purl=None):
        """VEX.Filter over one Result's vulnerabilities (order kept)."""
        return [v for v in vulns if self.keep(v, root_purl)]
