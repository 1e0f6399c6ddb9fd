"""ORACLE - TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference OS drivers over the raw bucket records
(tests/golden/fixtures format), using the C comparators of liboracle.so.  Used
only by tests/ and __graft_entry__.smoke() as the checker; the product never
imports this.  Small cases only (dict lookups, per-call JSON decode - like the
reference, which decodes every advisory on every Get).

Restated from (fwereade/trivy @ 2025-01-14):
  pkg/detector/ospkg/detect.go:32-82           drivers map, Detect (gpg-pubkey filter, EOSL)
  pkg/detector/ospkg/version/version.go:15-38  Major / Minor / Supported
  pkg/scanner/utils/utils.go:10-29             FormatVersion / FormatSrcVersion
  pkg/detector/ospkg/<os>/<os>.go              every driver's Detect + IsSupportedVersion
and the third-party trivy-db (go.mod:25, absent here) as described in SURVEY.md §8a
a28-a30: GetAdvisories / ForEachAdvisory (data-source join), redhat-oval Get (CPE
resolution through the "Red Hat CPE" bucket, one advisory per (entry, CVE)), rocky Get
(per-arch Entries).
"""
import calendar
import ctypes
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

SEVERITY = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(path)
        for fn in ("orc_deb_cmp_str", "orc_apk_cmp_str", "orc_rpm_cmp_str"):
            f = getattr(L, fn)
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        _LIB = L
    return _LIB


def _b(x):
    return x.encode() if isinstance(x, str) else x


def deb_cmp(a, b):
    """go-deb-version: 2 = a fails to parse, 3 = b fails, else sign(Compare)."""
    a, b = _b(a), _b(b)
    return lib().orc_deb_cmp_str(a, len(a), b, len(b))


def deb_valid(v):
    return deb_cmp(v, "0") != 2


def apk_cmp(a, b):
    """go-apk-version: 2 = a fails to parse, 3 = b fails, else sign(Compare)."""
    a, b = _b(a), _b(b)
    return lib().orc_apk_cmp_str(a, len(a), b, len(b))


def apk_valid(v):
    return apk_cmp(v, "0") != 2


def rpm_cmp(a, b):
    """go-rpm-version Compare (never fails)."""
    a, b = _b(a), _b(b)
    return lib().orc_rpm_cmp_str(a, len(a), b, len(b))


def rpm_string(v):
    """go-rpm-version Version.String(): the epoch is dropped when it is not positive."""
    epoch, rest = 0, v
    if ":" in v:
        e, rest = v.split(":", 1)
        try:
            epoch = int(e) if e.lstrip("+-").isdigit() and e.strip() == e else 0
        except ValueError:
            epoch = 0
        if abs(epoch) > 2 ** 63 - 1:
            epoch = 0
    i = rest.find("-")
    ver, rel = (rest[:i], rest[i + 1:]) if i >= 0 else (rest, "")
    out = f"{epoch}:" if epoch > 0 else ""
    out += ver
    if rel:
        out += "-" + rel
    return out


class DecodeError(Exception):
    pass


_FIELDS = {"vulnerabilityid": ("VulnerabilityID", str), "vendorids": ("VendorIDs", list),
           "arches": ("Arches", list), "status": ("Status", int), "severity": ("Severity", int),
           "fixedversion": ("FixedVersion", str), "affectedversion": ("AffectedVersion", str),
           "vulnerableversions": ("VulnerableVersions", list), "patchedversions": ("PatchedVersions", list),
           "unaffectedversions": ("UnaffectedVersions", list), "datasource": ("DataSource", dict),
           "custom": ("Custom", object), "entries": ("Entries", "entries")}


def _decode_obj(v):
    out = {}
    if v is None:
        return out
    if not isinstance(v, dict):
        raise DecodeError("not an object")
    for k, x in v.items():
        f = _FIELDS.get(k.lower())
        if f is None:
            continue
        name, typ = f
        if x is None:
            out.pop(name, None)
            continue
        if typ is int:
            if isinstance(x, str) and name == "Status":
                x = 0
            elif isinstance(x, bool) or not isinstance(x, int):
                raise DecodeError(f"{name}: not an int")
        elif typ is str and not isinstance(x, str):
            raise DecodeError(f"{name}: not a string")
        elif typ is list:
            if not isinstance(x, list) or any(e is not None and not isinstance(e, str) for e in x):
                raise DecodeError(f"{name}: not []string")
            x = ["" if e is None else e for e in x]
        elif typ is dict and not isinstance(x, dict):
            raise DecodeError(f"{name}: not an object")
        elif typ == "entries":
            if not isinstance(x, list):
                raise DecodeError("Entries: not an array")
            x = [_decode_obj(e) for e in x]
        if name == "Custom":
            x = json.dumps(x, separators=(",", ":"))
        out[name] = x
    return out


def decode_advisory(text):
    """json.Unmarshal into trivy-db types.Advisory (type errors -> DecodeError)."""
    try:
        v = json.loads(text)
    except ValueError as e:
        raise DecodeError(str(e))
    return _decode_obj(v)


def decode_redhat(text):
    """json.Unmarshal into trivy-db redhat-oval Advisory {Entries: [{FixedVersion, Affected,
    Arches, Status, Cves: [{ID, Severity}]}]}."""
    try:
        v = json.loads(text)
    except ValueError as e:
        raise DecodeError(str(e))
    if v is None:
        return []
    if not isinstance(v, dict):
        raise DecodeError("not an object")
    ents = None
    for k, x in v.items():
        if k.lower() == "entries":
            ents = x
    if ents is None:
        return []
    if not isinstance(ents, list):
        raise DecodeError("Entries: not an array")
    out = []
    for e in ents:
        if e is None:
            out.append({"FixedVersion": "", "Affected": [], "Arches": [], "Status": 0, "Cves": []})
            continue
        if not isinstance(e, dict):
            raise DecodeError("entry: not an object")
        d = {"FixedVersion": "", "Affected": [], "Arches": [], "Status": 0, "Cves": []}
        for k, x in e.items():
            kl = k.lower()
            if x is None:
                continue
            if kl == "fixedversion":
                if not isinstance(x, str):
                    raise DecodeError("FixedVersion")
                d["FixedVersion"] = x
            elif kl == "affected":
                if not isinstance(x, list) or any(isinstance(i, bool) or not isinstance(i, int) for i in x):
                    raise DecodeError("Affected")
                d["Affected"] = x
            elif kl == "arches":
                if not isinstance(x, list) or any(i is not None and not isinstance(i, str) for i in x):
                    raise DecodeError("Arches")
                d["Arches"] = ["" if i is None else i for i in x]
            elif kl == "status":
                if isinstance(x, bool) or not isinstance(x, int):
                    raise DecodeError("Status")
                d["Status"] = x
            elif kl == "cves":
                if not isinstance(x, list):
                    raise DecodeError("Cves")
                cves = []
                for c in x:
                    cd = {"ID": "", "Severity": 0}
                    if c is not None:
                        if not isinstance(c, dict):
                            raise DecodeError("cve")
                        for ck, cx in c.items():
                            if cx is None:
                                continue
                            if ck.lower() == "id":
                                if not isinstance(cx, str):
                                    raise DecodeError("cve ID")
                                cd["ID"] = cx
                            elif ck.lower() == "severity":
                                if isinstance(cx, bool) or not isinstance(cx, int):
                                    raise DecodeError("cve Severity")
                                cd["Severity"] = cx
                    cves.append(cd)
                d["Cves"] = cves
        out.append(d)
    return out


class Records:
    """The bucket tree of a set of fixture record files."""

    def __init__(self, records):
        self.tree = {}
        for r in records:
            node = self.tree
            for p in r["path"][:-1]:
                node = node.setdefault(("b", p), {})
            node[("k", r["path"][-1])] = r["value"]

    @classmethod
    def from_files(cls, paths):
        recs = []
        for p in paths:
            with open(p, encoding="utf-8") as f:
                recs += json.load(f)
        return cls(recs)

    def data_source(self, root):
        ds = self.tree.get(("b", "data-source"), {}).get(("k", root))
        if ds is None:
            return None
        d = json.loads(ds) or {}
        out = {k: d[k] for k in ("ID", "Name", "URL") if d.get(k)}
        return out or None

    def raw(self, root, name):
        """(vulnID, value) pairs of bucket root/name in bbolt key order."""
        b = self.tree.get(("b", root), {}).get(("b", name))
        if not b:
            return []
        return [(vid, val) for (kind, vid), val in sorted(b.items(), key=lambda kv: kv[0][1].encode())
                if kind == "k"]

    def get(self, root, name):
        """GetAdvisories(root, name): list of advisories sorted by vulnID, or raises DecodeError."""
        src = self.data_source(root)
        out = []
        for vid, val in self.raw(root, name):
            a = decode_advisory(val)
            a["VulnerabilityID"] = vid
            if src:
                a["DataSource"] = src
            elif "DataSource" in a:
                a["DataSource"] = {k: a["DataSource"][k] for k in ("ID", "Name", "URL") if a["DataSource"].get(k)}
            out.append(a)
        return out

    def get_rocky(self, root, name, arch):
        """trivy-db rocky Get(release, name, arch): per advisory, the Entries whose Arches
        contain arch (FixedVersion/VendorIDs of the entry); an advisory without Entries is
        returned as is."""
        out = []
        for a in self.get(root, name):
            ents = a.pop("Entries", None)
            if not ents:
                out.append(a)
                continue
            for e in ents:
                if arch in (e.get("Arches") or []):
                    out.append(rocky_entry_advisory(a, e))
        return out

    def redhat_cpes(self, content_sets, nvrs):
        """trivy-db RedHatRepoToCPEs / RedHatNVRToCPEs, uniq'ed."""
        cpe = self.tree.get(("b", "Red Hat CPE"), {})
        out = []
        for sub, keys in (("repository", content_sets), ("nvr", nvrs)):
            b = cpe.get(("b", sub), {})
            for k in keys:
                v = b.get(("k", k))
                if v is None:
                    continue
                for i in json.loads(v) or []:
                    if i not in out:
                        out.append(i)
        return out

    def get_redhat(self, name, content_sets, nvrs):
        """trivy-db redhat-oval Get(pkgName, repositories, nvrs)."""
        cpes = set(self.redhat_cpes(content_sets, nvrs))
        out = []
        for vid, val in self.raw("Red Hat", name):
            try:
                entries = decode_redhat(val)
            except DecodeError as e:
                raise DecodeError(f"failed to unmarshal advisory JSON: {e}")
            for e in entries:
                if not any(i in cpes for i in e["Affected"]):
                    continue
                for c in e["Cves"]:
                    out.append(redhat_cve_advisory(vid, e, c))
        return out


def rocky_entry_advisory(a, e):
    """trivy-db rocky Get: advisory a as seen through its arch entry e."""
    b = {k: v for k, v in a.items() if k not in ("FixedVersion", "VendorIDs", "Arches", "Entries")}
    for k in ("FixedVersion", "VendorIDs", "Arches"):
        if e.get(k):
            b[k] = e[k]
    return b


def redhat_cve_advisory(vid, e, c):
    """trivy-db redhat-oval Get: one advisory per (entry e, CVE c) of bucket key vid."""
    a = {"Severity": c["Severity"], "FixedVersion": e["FixedVersion"], "Arches": e["Arches"], "Status": e["Status"]}
    if vid.startswith("CVE-"):
        a["VulnerabilityID"] = vid
    else:
        a["VulnerabilityID"] = c["ID"]
        a["VendorIDs"] = [vid]
    return a


def format_version(epoch, version, release):
    v = version
    if release:
        v = f"{v}-{release}"
    if epoch:
        v = f"{epoch}:{v}"
    return v


def fmt(p):
    return format_version(p.get("Epoch", 0), p.get("Version", ""), p.get("Release", ""))


def fmt_src(p):
    return format_version(p.get("SrcEpoch", 0), p.get("SrcVersion", ""), p.get("SrcRelease", ""))


def major(v):
    return v.split(".", 1)[0]


def minor(v):
    parts = v.split(".", 2)
    return v if len(parts) == 1 else parts[0] + "." + parts[1]


def _eol(y, m, d):
    return calendar.timegm((y, m, d, 23, 59, 59, 0, 0, 0))


def _tab(d):
    return {k: _eol(*v) for k, v in d.items()}


# eolDates of each driver (transcribed data, <os>.go top of file)
UBUNTU_EOL = _tab({
    "4.10": (2006, 4, 30), "5.04": (2006, 10, 31), "5.10": (2007, 4, 13), "6.06": (2011, 6, 1),
    "6.10": (2008, 4, 25), "7.04": (2008, 10, 19), "7.10": (2009, 4, 18), "8.04": (2013, 5, 9),
    "8.10": (2010, 4, 30), "9.04": (2010, 10, 23), "9.10": (2011, 4, 29), "10.04": (2015, 4, 29),
    "10.10": (2012, 4, 10), "11.04": (2012, 10, 28), "11.10": (2013, 5, 9), "12.04": (2019, 4, 26),
    "12.04-ESM": (2019, 4, 28), "12.10": (2014, 5, 16), "13.04": (2014, 1, 27), "13.10": (2014, 7, 17),
    "14.04": (2022, 4, 25), "14.04-ESM": (2024, 4, 25), "14.10": (2015, 7, 23), "15.04": (2016, 1, 23),
    "15.10": (2016, 7, 22), "16.04": (2021, 4, 21), "16.04-ESM": (2026, 4, 29), "16.10": (2017, 7, 20),
    "17.04": (2018, 1, 13), "17.10": (2018, 7, 19), "18.04": (2023, 5, 31), "18.04-ESM": (2028, 3, 31),
    "18.10": (2019, 7, 18), "19.04": (2020, 1, 18), "19.10": (2020, 7, 17), "20.04": (2025, 4, 23),
    "20.10": (2021, 7, 22), "21.04": (2022, 1, 20), "21.10": (2022, 7, 14), "22.04": (2027, 4, 23),
    "22.10": (2023, 7, 20), "23.04": (2024, 1, 20)})
DEBIAN_EOL = _tab({
    "1.1": (1997, 6, 5), "1.2": (1998, 6, 5), "1.3": (1999, 3, 9), "2.0": (2000, 3, 9), "2.1": (2000, 10, 30),
    "2.2": (2003, 7, 30), "3.0": (2006, 6, 30), "3.1": (2008, 3, 30), "4.0": (2010, 2, 15), "5.0": (2012, 2, 6),
    "6.0": (2016, 2, 29), "7": (2018, 5, 31), "8": (2020, 6, 30), "9": (2022, 6, 30), "10": (2024, 6, 30),
    "11": (2026, 8, 14), "12": (2028, 6, 10), "13": (3000, 1, 1)})
ALPINE_EOL = _tab({
    "2.0": (2012, 4, 1), "2.1": (2012, 11, 1), "2.2": (2013, 5, 1), "2.3": (2013, 11, 1), "2.4": (2014, 5, 1),
    "2.5": (2014, 11, 1), "2.6": (2015, 5, 1), "2.7": (2015, 11, 1), "3.0": (2016, 5, 1), "3.1": (2016, 11, 1),
    "3.2": (2017, 5, 1), "3.3": (2017, 11, 1), "3.4": (2018, 5, 1), "3.5": (2018, 11, 1), "3.6": (2019, 5, 1),
    "3.7": (2019, 11, 1), "3.8": (2020, 5, 1), "3.9": (2020, 11, 1), "3.10": (2021, 5, 1), "3.11": (2021, 11, 1),
    "3.12": (2022, 5, 1), "3.13": (2022, 11, 1), "3.14": (2023, 5, 1), "3.15": (2023, 11, 1),
    "3.16": (2024, 5, 23), "3.17": (2024, 11, 22), "3.18": (2025, 5, 9), "3.19": (2025, 11, 1)})
ALPINE_EOL["edge"] = calendar.timegm((9999, 1, 1, 0, 0, 0, 0, 0, 0))
AMAZON_EOL = _tab({"1": (2023, 12, 31), "2": (2025, 6, 30), "2023": (2028, 3, 15)})
REDHAT_EOL = _tab({"4": (2017, 5, 31), "5": (2020, 11, 30), "6": (2024, 6, 30), "7": (3000, 1, 1),
                   "8": (3000, 1, 1), "9": (3000, 1, 1)})
CENTOS_EOL = _tab({"3": (2010, 10, 31), "4": (2012, 2, 29), "5": (2017, 3, 31), "6": (2020, 11, 30),
                   "7": (2024, 6, 30), "8": (2021, 12, 31)})
ALMA_EOL = _tab({"8": (2029, 3, 1), "9": (2032, 5, 31)})
ROCKY_EOL = _tab({"8": (2029, 5, 31), "9": (2032, 5, 31)})
ORACLE_EOL = _tab({"3": (2011, 12, 31), "4": (2013, 12, 31), "5": (2017, 12, 31), "6": (2021, 3, 21),
                   "7": (2024, 7, 23), "8": (2029, 7, 18), "9": (2032, 7, 18)})
PHOTON_EOL = _tab({"1.0": (2022, 2, 28), "2.0": (2022, 12, 31), "3.0": (2024, 6, 30), "4.0": (2025, 12, 31)})
SLES_EOL = _tab({
    "10": (2007, 12, 31), "10.1": (2008, 11, 30), "10.2": (2010, 4, 11), "10.3": (2011, 10, 11),
    "10.4": (2013, 7, 31), "11": (2010, 12, 31), "11.1": (2012, 8, 31), "11.2": (2014, 1, 31),
    "11.3": (2016, 1, 31), "11.4": (2019, 3, 31), "12": (2016, 6, 30), "12.1": (2017, 5, 31),
    "12.2": (2018, 3, 31), "12.3": (2019, 1, 30), "12.4": (2020, 6, 30), "12.5": (2024, 10, 31),
    "15": (2019, 12, 31), "15.1": (2021, 1, 31), "15.2": (2021, 12, 31), "15.3": (2022, 12, 31),
    "15.4": (2023, 12, 31), "15.5": (2028, 12, 31)})
OPENSUSE_EOL = _tab({
    "42.1": (2017, 5, 17), "42.2": (2018, 1, 26), "42.3": (2019, 6, 30), "15.0": (2019, 12, 3),
    "15.1": (2020, 11, 30), "15.2": (2021, 11, 30), "15.3": (2022, 11, 30), "15.4": (2023, 11, 30),
    "15.5": (2024, 12, 31)})


def supported(eol, ver, now):
    """osver.Supported (version.go:31-38)."""
    return ver not in eol or now < eol[ver]


def _base(p, a, installed, fixed=None, pkg_id=True, custom=True):
    d = {"VulnerabilityID": a["VulnerabilityID"]}
    fixed = a.get("FixedVersion") if fixed is None else fixed
    for k_out, val in [("PkgID", p.get("ID") if pkg_id else None), ("PkgName", p.get("Name")),
                       ("PkgIdentifier", p.get("Identifier")), ("InstalledVersion", installed),
                       ("FixedVersion", fixed), ("Layer", p.get("Layer")), ("DataSource", a.get("DataSource")),
                       ("Custom", a.get("Custom") if custom else None)]:
        if val:
            d[k_out] = val
    return d


def _get(db, err, root, name):
    try:
        return db.get(root, name)
    except DecodeError as e:
        raise DecodeError(f"{err}: failed to unmarshal advisory JSON: {e}")


# --------------------------------------------------------------------- dpkg drivers ----
def debian_vuln(p, a):
    """debian.go:78-98: the DetectedVulnerability of package p and advisory a."""
    v = _base(p, a, fmt(p))
    if a.get("VendorIDs"):
        v["VendorIDs"] = a["VendorIDs"]
    if a.get("Status"):
        v["Status"] = a["Status"]
    if a.get("Severity", 0) != 0:
        v["SeveritySource"] = "debian"
        v["Severity"] = SEVERITY[a["Severity"]] if 0 < a["Severity"] < 5 else SEVERITY[0]
    return v


def plain_vuln(p, a):
    """ubuntu.go:99-108, amazon.go:75-83, alpine.go:94-101, wolfi / chainguard: the fields
    _base sets, InstalledVersion = FormatVersion(pkg)."""
    return _base(p, a, fmt(p))


def debian_detect(db, os_ver, repo, pkgs, now=None):
    root = "debian " + major(os_ver)
    out = []
    for p in pkgs:
        src = fmt_src(p)
        if not deb_valid(src):
            continue
        for a in _get(db, "failed to get debian advisories", root, p.get("SrcName", "")):
            v = debian_vuln(p, a)
            fixed = a.get("FixedVersion", "")
            if fixed == "":
                out.append(v)
                continue
            r = deb_cmp(src, fixed)
            if r == 3:
                continue
            if r < 0:
                out.append(v)
    return out


def ubuntu_version_from_eol(os_ver, now, eol):
    if os_ver in eol:
        return os_ver
    ver = os_ver.rstrip("-ESM")
    if ver in eol and now < eol[ver]:
        return ver
    return os_ver


def ubuntu_detect(db, os_ver, repo, pkgs, now):
    out = []
    for p in pkgs:
        os_ver = ubuntu_version_from_eol(os_ver, now, UBUNTU_EOL)
        advs = _get(db, "failed to get Ubuntu advisories", "ubuntu " + os_ver, p.get("SrcName", ""))
        src = fmt_src(p)
        if not deb_valid(src):
            continue
        for a in advs:
            v = plain_vuln(p, a)
            fixed = a.get("FixedVersion", "")
            if fixed == "":
                out.append(v)
                continue
            r = deb_cmp(src, fixed)
            if r == 3:
                continue
            if r < 0:
                out.append(v)
    return out


def amazon_release(os_ver):
    f = os_ver.split()
    v = major(f[0] if f else "")
    return v if v in ("2", "2022", "2023") else "1"


def amazon_detect(db, os_ver, repo, pkgs, now=None):
    v = amazon_release(os_ver)
    out = []
    for p in pkgs:
        advs = _get(db, "failed to get amazon advisories", "amazon linux " + v, p.get("Name", ""))
        inst = fmt(p)
        if inst == "" or not deb_valid(inst):
            continue
        for a in advs:
            r = deb_cmp(inst, a.get("FixedVersion", ""))
            if r == 3:
                continue
            if r < 0:
                out.append(plain_vuln(p, a))
    return out


# ---------------------------------------------------------------------- apk drivers ----
def alpine_repo_release(repo):
    if not repo:
        return ""
    rel = repo.get("Release", "")
    if rel.count(".") > 1:
        rel = rel[:rel.rfind(".")]
    return rel


def alpine_stream(os_ver, repo):
    v = minor(os_ver)
    rr = alpine_repo_release(repo)
    return rr if rr != "" and v != rr else v


def alpine_vulnerable(inst, a):
    aff = a.get("AffectedVersion", "")
    if aff != "":
        if not apk_valid(aff):
            return False
        if apk_cmp(aff, inst) > 0:
            return False
    fixed = a.get("FixedVersion", "")
    if fixed == "":
        return True
    if not apk_valid(fixed):
        return False
    return apk_cmp(inst, fixed) < 0


def alpine_detect(db, os_ver, repo, pkgs, now=None):
    root = "alpine " + alpine_stream(os_ver, repo)
    out = []
    for p in pkgs:
        name = p.get("SrcName") or p.get("Name", "")
        advs = _get(db, "failed to get alpine advisories", root, name)
        src = fmt_src(p)
        if not apk_valid(src):
            continue
        for a in advs:
            if alpine_vulnerable(src, a):
                out.append(plain_vuln(p, a))
    return out


def _apk_stream_detect(root, err):
    def detect(db, os_ver, repo, pkgs, now=None):
        out = []
        for p in pkgs:
            name = p.get("SrcName") or p.get("Name", "")
            advs = _get(db, err, root, name)
            inst = fmt(p)
            if not apk_valid(inst):
                continue
            for a in advs:
                fixed = a.get("FixedVersion", "")
                if apk_valid(fixed) and apk_cmp(inst, fixed) < 0:
                    out.append(plain_vuln(p, a))
        return out
    return detect


wolfi_detect = _apk_stream_detect("wolfi", "failed to get Wolfi advisories")
chainguard_detect = _apk_stream_detect("chainguard", "failed to get Chainguard advisories")


# ---------------------------------------------------------------------- rpm drivers ----
REDHAT_DEFAULT_CONTENT_SETS = {
    "6": ["rhel-6-server-rpms", "rhel-6-server-extras-rpms"],
    "7": ["rhel-7-server-rpms", "rhel-7-server-extras-rpms"],
    "8": ["rhel-8-for-x86_64-baseos-rpms", "rhel-8-for-x86_64-appstream-rpms"],
    "9": ["rhel-9-for-x86_64-baseos-rpms", "rhel-9-for-x86_64-appstream-rpms"],
}


def add_modular_namespace(name, label):
    """redhat.go:207-220 / alma.go: label[:2nd ':'] + '::' + name."""
    count = 0
    for i, ch in enumerate(label):
        if ch == ":":
            count += 1
        if count == 2:
            return label[:i] + "::" + name
    return name


def redhat_detect(db, os_ver, repo, pkgs, now=None):
    os_ver = major(os_ver)
    out = []
    for p in pkgs:
        if p.get("Release", "").endswith(".remi"):
            continue
        name = add_modular_namespace(p.get("Name", ""), p.get("Modularitylabel", ""))
        bi = p.get("BuildInfo")
        if bi is None:
            cs, nvr = REDHAT_DEFAULT_CONTENT_SETS.get(os_ver, []), ""
        else:
            cs, nvr = bi.get("ContentSets") or [], f"{bi.get('Nvr', '')}-{bi.get('Arch', '')}"
        try:
            advs = db.get_redhat(name, cs, [nvr])
        except DecodeError as e:
            raise DecodeError(f"redhat vulnerability detection error: failed to get Red Hat advisories: {e}")
        inst = fmt(p)
        kept = [a for a in advs
                if not (a["Arches"] and p.get("Arch", "") != "noarch" and p.get("Arch", "") not in a["Arches"])
                and (a["FixedVersion"] == "" or rpm_cmp(inst, a["FixedVersion"]) < 0)]
        out += redhat_uniq(p, inst, kept)
    return out


def redhat_uniq(p, inst, advs):
    """redhat.go:146-187 uniqVulns over package p's advisories that passed the arch filter and
    (fixed ones) the version check, in Get order; sorted by VulnerabilityID."""
    uniq = {}
    for a in advs:
        vid = a["VulnerabilityID"]
        v = {"VulnerabilityID": vid, "PkgID": p.get("ID"), "PkgName": p.get("Name"), "InstalledVersion": inst,
             "PkgIdentifier": p.get("Identifier"), "Status": a["Status"], "Layer": p.get("Layer"),
             "SeveritySource": "redhat",
             "Severity": SEVERITY[a["Severity"]] if 0 <= a["Severity"] < 5 else SEVERITY[0]}
        if a["FixedVersion"] == "":
            if vid not in uniq:
                uniq[vid] = v
            continue
        v["VendorIDs"] = a.get("VendorIDs")
        v["FixedVersion"] = rpm_string(a["FixedVersion"])
        if vid in uniq:
            u = uniq[vid]
            u["VendorIDs"] = sorted(set((u.get("VendorIDs") or []) + (v["VendorIDs"] or [])))
            if rpm_cmp(u.get("FixedVersion") or "", a["FixedVersion"]) < 0:
                u["FixedVersion"] = v["FixedVersion"]
        else:
            uniq[vid] = v
    return [{k: x for k, x in v.items() if x not in (None, "", [], 0) or k == "VulnerabilityID"}
            for _, v in sorted(uniq.items())]


def _rpm_simple(root_fn, err, name_fn=lambda p: p.get("Name", ""), inst_fn=fmt, fixed_out="raw",
                skip=lambda p: False, unfixed=False, pkg_id=True, custom=True, getter="get"):
    def vuln(p, a):
        """alma.go:64-71, rocky.go:69-76, oracle.go:70-80, suse.go, photon.go, mariner.go:50-70:
        FixedVersion printed by rpm Version.String() where the driver does."""
        fixed = a.get("FixedVersion", "")
        f = rpm_string(fixed) if fixed_out == "string" and fixed else fixed
        return _base(p, a, fmt(p), fixed=f, pkg_id=pkg_id, custom=custom)

    def detect(db, os_ver, repo, pkgs, now=None):
        root = root_fn(os_ver)
        out = []
        for p in pkgs:
            if skip(p):
                continue
            try:
                if getter == "rocky":
                    advs = db.get_rocky(root, name_fn(p), p.get("Arch", ""))
                else:
                    advs = db.get(root, name_fn(p))
            except DecodeError as e:
                raise DecodeError(f"{err}: failed to unmarshal advisory JSON: {e}")
            cmp_ver = inst_fn(p)
            for a in advs:
                fixed = a.get("FixedVersion", "")
                if unfixed and fixed == "":
                    out.append(vuln(p, a))
                    continue
                if getter == "oracle" and extract_ksplice(fixed) != extract_ksplice(p.get("Release", "")):
                    continue
                if rpm_cmp(cmp_ver, fixed) < 0:
                    out.append(vuln(p, a))
        return out
    detect.vuln = vuln
    return detect


def extract_ksplice(v):
    for s in v.lower().split("."):
        if s.startswith("ksplice"):
            return s
    return ""


alma_detect = _rpm_simple(lambda v: "alma " + major(v), "failed to get AlmaLinux advisories",
                          name_fn=lambda p: add_modular_namespace(p.get("Name", ""), p.get("Modularitylabel", "")),
                          fixed_out="string",
                          skip=lambda p: ".module_el" in p.get("Release", "") and not p.get("Modularitylabel"))
rocky_detect = _rpm_simple(lambda v: "rocky " + major(v), "failed to get Rocky Linux advisories", fixed_out="string",
                           skip=lambda p: bool(p.get("Modularitylabel")), getter="rocky")
oracle_detect = _rpm_simple(lambda v: "Oracle Linux " + major(v), "failed to get Oracle Linux advisory",
                            getter="oracle")
photon_detect = _rpm_simple(lambda v: "Photon OS " + v,
                            "failed to get Photon Linux advisory: failed to get Photon advisories",
                            name_fn=lambda p: p.get("SrcName", ""))
mariner_detect = _rpm_simple(lambda v: "CBL-Mariner " + minor(v), "failed to get CBL-Mariner advisories",
                             name_fn=lambda p: p.get("SrcName", ""), inst_fn=fmt_src, fixed_out="string",
                             unfixed=True, pkg_id=False, custom=False)
sles_detect = _rpm_simple(lambda v: "SUSE Linux Enterprise " + v,
                          "failed to get SUSE advisory: failed to get SUSE advisories")
opensuse_detect = _rpm_simple(lambda v: "openSUSE Leap " + v,
                              "failed to get SUSE advisory: failed to get SUSE advisories")


debian_detect.vuln = debian_vuln
for _d in (ubuntu_detect, amazon_detect, alpine_detect, wolfi_detect, chainguard_detect):
    _d.vuln = plain_vuln


# ----------------------------------------------------------- DetectedVulnerability records ----
# A DetectedVulnerability is a record (the advisory side) plus its package's fields; the
# batch-path checks compare records built here from a driver's own epilogue with a stub package.
COPY_PKG_ID, COPY_PKG_NAME, COPY_IDENTIFIER, COPY_LAYER = 1, 2, 4, 8
_STUB = {"ID": "\x01id", "Name": "\x01name", "Identifier": {"PURL": "\x01purl"}, "Layer": {"DiffID": "\x01layer"},
         "FilePath": "\x01path", "Version": "\x01ver"}
_PKG_FIELDS = {"PkgID": COPY_PKG_ID, "PkgName": COPY_PKG_NAME, "PkgIdentifier": COPY_IDENTIFIER, "Layer": COPY_LAYER}


def record_of(v):
    """(record dict, copy flags) of a DetectedVulnerability built for the stub package: the
    package fields are dropped and remembered as the flags of the ones the driver copied."""
    rec, flags = {}, 0
    for k, x in v.items():
        if k in _PKG_FIELDS:
            flags |= _PKG_FIELDS[k]
        elif k not in ("InstalledVersion", "PkgPath"):
            rec[k] = x
    return rec, flags


def advisory_record(family, a):
    """The record OS driver `family` builds from advisory a (its Get form)."""
    if family in ("redhat", "centos"):
        return redhat_group_record([a])
    return record_of(DRIVERS[family][0].vuln(_STUB, a))


def redhat_group_record(members):
    """The record of one merged Red Hat vulnerability from its members (the advisories that
    entered uniqVulns for one package and VulnerabilityID, Get order)."""
    out = redhat_uniq(_STUB, "", members)
    assert len(out) == 1, "members of one VulnerabilityID"
    return record_of(out[0])


# --------------------------------------------------------------------- dispatcher ----
def _always(ver, now):
    return True


# family (ftypes.OSType) -> (detect, is_supported(os_ver, now))
DRIVERS = {
    "alpine": (alpine_detect, lambda v, now: supported(ALPINE_EOL, minor(v), now)),
    "alma": (alma_detect, lambda v, now: supported(ALMA_EOL, major(v), now)),
    "amazon": (amazon_detect, lambda v, now: supported(AMAZON_EOL, amazon_release(v), now)),
    "cbl-mariner": (mariner_detect, _always),
    "debian": (debian_detect, lambda v, now: supported(DEBIAN_EOL, major(v), now)),
    "ubuntu": (ubuntu_detect, lambda v, now: supported(UBUNTU_EOL, v, now)),
    "redhat": (redhat_detect, lambda v, now: supported(REDHAT_EOL, major(v), now)),
    "centos": (redhat_detect, lambda v, now: supported(CENTOS_EOL, major(v), now)),
    "rocky": (rocky_detect, lambda v, now: supported(ROCKY_EOL, major(v), now)),
    "oracle": (oracle_detect, lambda v, now: supported(ORACLE_EOL, major(v), now)),
    "opensuse.leap": (opensuse_detect, lambda v, now: supported(OPENSUSE_EOL, v, now)),
    "suse linux enterprise server": (sles_detect, lambda v, now: supported(SLES_EOL, v, now)),
    "photon": (photon_detect, lambda v, now: supported(PHOTON_EOL, v, now)),
    "wolfi": (wolfi_detect, _always),
    "chainguard": (chainguard_detect, _always),
}


class UnsupportedOS(Exception):
    pass


def driver_detect(family, os_ver, repo, pkgs, db, now):
    return DRIVERS[family][0](db, os_ver, repo, pkgs, now)


def is_supported(family, os_ver, now):
    return DRIVERS[family][1](os_ver, now)


def detect(db, family, os_name, repo, pkgs, now):
    """ospkg.Detect (detect.go:63-82)."""
    if family not in DRIVERS:
        raise UnsupportedOS("unsupported os")
    eosl = not is_supported(family, os_name, now)
    kept = [p for p in pkgs if p.get("Name") != "gpg-pubkey"]
    try:
        vulns = driver_detect(family, os_name, repo, kept, db, now)
    except DecodeError as e:
        raise DecodeError(f"failed detection: {e}")
    return vulns, eosl
