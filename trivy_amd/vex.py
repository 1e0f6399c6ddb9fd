"""VEX documents compiled against a batch (mirror of pkg/vex).

The reference walks every detected vulnerability of every Result and, per vulnerability,
scans the VEX statements (pkg/vex/openvex.go:21-54, cyclonedx.go:48-84, csaf.go:27-138).
Here the document is compiled once per batch on the host into the set of (package,
vulnerability ID) findings it drops: statements are few, and their product PURLs are
resolved through a (type, namespace, name) index of the batch's package PURLs, so the
host cost is O(statements x matching packages), independent of the number of findings.
The per-finding test - is this surviving (package, vulnerability) in the set? - runs on
the GPU inside the batch result filter (filter.hip filter_select, after the dedup, as
filterByVEX runs after FilterResult, pkg/result/filter.go:38-104).

Semantics (same names as the reference):
  VEX.new              vex.New (vex.go:28-61): CycloneDX JSON (needs a CycloneDX SBOM
                       report, :71-73), else OpenVEX (@context), else CSAF (vulnerabilities),
                       else "unable to load VEX";
  OpenVEX              the statements matching (vuln, root PURL, [package PURL]) when the
                       result has a root PURL and any match, else (vuln, package PURL); the
                       last after go-vex's stable timestamp sort decides; not_affected and
                       fixed drop the finding (go-vex v0.2.5 Statement/Component/PurlMatches);
  CycloneDX            the first statement with the vulnerability ID; a BOM-Link affect that
                       names the SBOM's serial number and version and matches the package
                       (PkgIdentifier.Match: BOM ref or PURL) drops it when the analysis
                       state maps to not_affected / fixed;
  CSAF                 the first vulnerability with the CVE; a product in known_not_affected
                       or fixed whose helper PURLs (or default_component_of / installed_on /
                       installed_with sub-products') purl.Match the package drops it.
"""
import datetime
import json
import re
import urllib.parse

import numpy as np


class VEXError(Exception):
    pass


# ---- package URLs (packageurl-go FromString as trivy uses it) ---------------------------------
class PURL:
    __slots__ = ("type", "namespace", "name", "version", "qualifiers", "subpath")

    def __init__(self, type_, namespace, name, version, qualifiers, subpath):
        self.type, self.namespace, self.name = type_, namespace, name
        self.version, self.qualifiers, self.subpath = version, qualifiers, subpath

    @classmethod
    def parse(cls, s):
        """None when s is not a valid package URL."""
        if not isinstance(s, str) or not s.startswith("pkg:"):
            return None
        rest = s[4:].lstrip("/")
        subpath = ""
        if "#" in rest:
            rest, sp = rest.split("#", 1)
            subpath = "/".join(urllib.parse.unquote(x) for x in sp.strip("/").split("/") if x not in ("", ".", ".."))
        quals = {}
        if "?" in rest:
            rest, q = rest.split("?", 1)
            for kv in q.split("&"):
                k, _, v = kv.partition("=")
                if kv and v:
                    quals[k.lower()] = urllib.parse.unquote(v)
        typ, _, rest = rest.partition("/")
        if not typ or not rest:
            return None
        version = ""
        if "@" in rest:
            rest, version = rest.rsplit("@", 1)
            version = urllib.parse.unquote(version)
        segs = [urllib.parse.unquote(x) for x in rest.strip("/").split("/")]
        return cls(typ.lower(), "/".join(x for x in segs[:-1] if x), segs[-1], version, quals, subpath)

    def base(self):
        return self.type, self.namespace, self.name

    def key(self):
        return self.base() + (self.version, tuple(sorted(self.qualifiers.items())), self.subpath)

    def quals_in(self, other):
        return all(other.qualifiers.get(k) == v for k, v in self.qualifiers.items())

    def vex_matches(self, other):
        """go-vex PurlMatches(self general, other specific)."""
        return (self.base() == other.base() and (not self.version or self.version == other.version)
                and self.quals_in(other))

    def trivy_matches(self, other):
        """pkg/purl/purl.go:249-274 PackageURL.Match(self constraint, other target)."""
        return (self.base() == other.base() and (not self.version or self.version == other.version)
                and (not self.subpath or self.subpath == other.subpath) and self.quals_in(other))


def _ts(s):
    """RFC 3339 (nanoseconds allowed) -> integer nanoseconds since the epoch."""
    m = re.fullmatch(r"(\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d)(?:\.(\d{1,9}))?(Z|[+-]\d\d:\d\d)", s or "")
    if not m:
        return None
    t = datetime.datetime.strptime(m.group(1), "%Y-%m-%dT%H:%M:%S").replace(tzinfo=datetime.timezone.utc)
    off = 0 if m.group(3) == "Z" else (1 if m.group(3)[0] == "+" else -1) * (
        int(m.group(3)[1:3]) * 3600 + int(m.group(3)[4:6]) * 60)
    return (int(t.timestamp()) - off) * 10 ** 9 + int((m.group(2) or "0").ljust(9, "0"))


_BOMLINK = re.compile(r"urn:cdx:([0-9a-f]{8}-[0-9a-f]{4}-[1-5][0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12})/([1-9]\d*)"
                      r"(?:#([0-9a-zA-Z\-._~%!$&'()*+,;=:@/?]+))?")
_CDX_DROP = {"resolved", "resolved_with_pedigree", "false_positive", "not_affected"}  # fixed / not_affected


class _Packages:
    """The batch's package identities, indexed for statement resolution."""

    def __init__(self, purls, bom_refs, result_of, roots):
        self.purls = [PURL.parse(p) if p else None for p in purls]
        self.by_base, self.by_key, self.by_ref = {}, {}, {}
        for i, p in enumerate(self.purls):
            if p is not None:
                self.by_base.setdefault(p.base(), []).append(i)
                self.by_key.setdefault(p.key(), []).append(i)
        for i, r in enumerate(bom_refs or ()):
            if r:
                self.by_ref.setdefault(r, []).append(i)
        self.result_of = np.asarray(result_of if result_of is not None else np.zeros(len(purls)), dtype=np.int64)
        self.roots = [PURL.parse(r) if r else None for r in (roots or ())]

    def matching(self, pattern, rule):
        """Indices of packages whose PURL `pattern` (a PURL) matches under `rule`."""
        return [i for i in self.by_base.get(pattern.base(), ()) if rule(pattern, self.purls[i])]


class VEX:
    def __init__(self, kind, doc, bom_serial="", bom_version=0):
        self.kind, self.doc, self.serial, self.version = kind, doc, bom_serial, bom_version

    @classmethod
    def new(cls, text, artifact_type="", bom_serial="", bom_version=0):
        """vex.New over a document's text; (artifact_type, bom_serial, bom_version) are the
        report's ArtifactType and its CycloneDX BOM's serial number / version."""
        try:
            doc = json.loads(text)
        except ValueError:
            doc = None
        if not isinstance(doc, dict):
            raise VEXError("unable to load VEX")
        if doc.get("bomFormat") == "CycloneDX":
            if artifact_type != "cyclonedx":
                raise VEXError("CycloneDX VEX can be used with CycloneDX SBOM")
            return cls("cyclonedx", doc, bom_serial, bom_version)
        if doc.get("@context"):
            return cls("openvex", doc)
        if doc.get("vulnerabilities") is not None:
            return cls("csaf", doc)
        raise VEXError("unable to load VEX")

    # -- compile against a batch --
    def suppressions(self, purls, bom_refs=None, result_of=None, roots=None):
        """(package indices uint32, vulnerability IDs) of the findings this document drops.

        purls[i]: package i's PURL string (None: no PURL, never dropped); bom_refs[i]: its
        CycloneDX bom-ref; result_of[i]: its result; roots[r]: result r's root component
        PURL (the scanned artifact, OpenVEX subcomponent statements) or None."""
        pk = _Packages(purls, bom_refs, result_of, roots)
        drop = getattr(self, "_" + self.kind)(pk)
        items = sorted(drop)
        return np.array([p for p, _ in items], dtype=np.uint32), [v for _, v in items]

    def _openvex(self, pk):
        doc_ts = _ts(self.doc.get("timestamp"))
        # (package, vuln) -> [root-mode statements], [direct statements], as (ts, order, status)
        root_st, direct_st = {}, {}
        for order, st in enumerate(self.doc.get("statements") or []):
            v = st.get("vulnerability") or {}
            vids = {x for x in [v.get("name")] + list(v.get("aliases") or []) if x}
            ts = _ts(st["timestamp"]) if st.get("timestamp") else doc_ts
            rec = (ts if ts is not None else 0, order, st.get("status"))
            for prod in st.get("products") or []:
                for i in self._component_pkgs(prod, pk):
                    for vid in vids:
                        direct_st.setdefault((i, vid), []).append(rec)
                subs = prod.get("subcomponents") or []
                if not subs:
                    continue
                roots = [r for r, root in enumerate(pk.roots) if root is not None and self._component_is(prod, root)]
                if not roots:
                    continue
                in_root = np.isin(pk.result_of, roots)
                for sub in subs:
                    for i in self._component_pkgs(sub, pk):
                        if in_root[i]:
                            for vid in vids:
                                root_st.setdefault((i, vid), []).append(rec)
        out = set()
        for key in set(root_st) | set(direct_st):
            i = key[0]
            if pk.purls[i] is None:
                continue
            root_ok = pk.roots and pk.result_of[i] < len(pk.roots) and pk.roots[pk.result_of[i]] is not None
            recs = root_st.get(key) if root_ok and root_st.get(key) else direct_st.get(key)
            if recs and max(recs, key=lambda r: (r[0], r[1]))[2] in ("not_affected", "fixed"):
                out.add(key)
        return out

    @staticmethod
    def _component_is(comp, purl):
        """go-vex Component.Matches(identifier) for one parsed PURL identifier."""
        cands = [comp.get("@id")] + [v for t, v in (comp.get("identifiers") or {}).items() if t == "purl"]
        for c in cands:
            p = PURL.parse(c) if c else None
            if p is not None and p.vex_matches(purl):
                return True
        return False

    @staticmethod
    def _component_pkgs(comp, pk):
        """Packages the component matches (its @id / purl identifiers as PURL patterns, plus
        string-equal identifiers and hashes of a package PURL's canonical key)."""
        hit = set()
        for c in [comp.get("@id")] + [v for t, v in (comp.get("identifiers") or {}).items() if t == "purl"]:
            p = PURL.parse(c) if c else None
            if p is not None:
                hit.update(pk.matching(p, PURL.vex_matches))
        for v in list((comp.get("identifiers") or {}).values()) + list((comp.get("hashes") or {}).values()):
            p = PURL.parse(v) if v else None
            if p is not None:  # a string equal to a package's PURL string is that PURL
                hit.update(pk.by_key.get(p.key(), ()))
        return hit

    def _cyclonedx(self, pk):
        out, seen = set(), set()
        for v in self.doc.get("vulnerabilities") or []:
            vid = v.get("id")
            if vid in seen:  # lo.Find: only the first statement of an ID is consulted
                continue
            seen.add(vid)
            if (v.get("analysis") or {}).get("state") not in _CDX_DROP:
                continue
            for a in v.get("affects") or []:
                m = _BOMLINK.fullmatch(a.get("ref") or "")
                if not m or "urn:uuid:" + m.group(1) != self.serial or int(m.group(2)) != self.version:
                    continue
                ref = urllib.parse.unquote(m.group(3) or "")
                hit = set(pk.by_ref.get(ref, ()))
                p = PURL.parse(ref) if ref.startswith("pkg:") else None
                if p is not None:
                    hit.update(pk.by_key.get(p.key(), ()))
                out.update((i, vid) for i in hit)
        return out

    def _csaf(self, pk):
        tree = self.doc.get("product_tree") or {}
        out, seen = set(), set()
        for v in self.doc.get("vulnerabilities") or []:
            cve = v.get("cve")
            if cve in seen:
                continue
            seen.add(cve)
            ps = v.get("product_status")
            if ps is None:
                continue
            for prod in (ps.get("known_not_affected") or []) + (ps.get("fixed") or []):
                pats = _csaf_purls(tree, prod)
                for r in tree.get("relationships") or []:
                    if r and r.get("category") in ("default_component_of", "installed_on", "installed_with") and \
                            (r.get("full_product_name") or {}).get("product_id") == prod:
                        pats += _csaf_purls(tree, r.get("product_reference"))
                for p in pats:
                    out.update((i, cve) for i in pk.matching(p, PURL.trivy_matches))
        return out


def _csaf_purls(tree, pid):
    """ProductTree.CollectProductIdentificationHelpers(pid) -> their valid PURLs."""
    helpers = []

    def take(f):
        if f and f.get("product_id") == pid and f.get("product_identification_helper"):
            helpers.append(f["product_identification_helper"])

    for f in tree.get("full_product_names") or []:
        take(f)
    stack = list(reversed(tree.get("branches") or []))
    while stack:
        b = stack.pop()
        if b:
            take(b.get("product"))
            stack.extend(reversed(b.get("branches") or []))
    for r in tree.get("relationships") or []:
        take((r or {}).get("full_product_name"))
    return [p for p in (PURL.parse(h.get("purl")) for h in helpers) if p is not None]
