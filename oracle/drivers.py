"""ORACLE - TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference OS drivers over the raw bucket records
(tests/golden/fixtures format), using the C comparators of liboracle.so.  Used
only by tests/ and __graft_entry__.smoke() as the checker; the product never
imports this.  Small cases only (dict lookups, per-call JSON decode - like the
reference, which decodes every advisory on every Get).

Restated from (fwereade/trivy @ 2025-01-14):
  pkg/detector/ospkg/detect.go:63-82           Detect (gpg-pubkey filter, EOSL)
  pkg/detector/ospkg/debian/debian.go:57-119   Debian Scanner.Detect
  pkg/detector/ospkg/ubuntu/ubuntu.go:79-151   Ubuntu Scanner.Detect + versionFromEolDates
  pkg/detector/ospkg/amazon/amazon.go:43-97    Amazon Scanner.Detect
  pkg/scanner/utils/utils.go:10-29             FormatVersion / FormatSrcVersion
  trivy-db db.Config.GetAdvisories (third party, go.mod:25) as described in SURVEY.md §8a a28
"""
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
        _LIB = ctypes.CDLL(path)
        _LIB.orc_deb_cmp_str.restype = ctypes.c_int
        _LIB.orc_deb_cmp_str.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    return _LIB


def deb_cmp(a, b):
    """go-deb-version: 2 = a fails to parse, 3 = b fails, else sign(Compare)."""
    a = a.encode() if isinstance(a, str) else a
    b = b.encode() if isinstance(b, str) else b
    return lib().orc_deb_cmp_str(a, len(a), b, len(b))


def deb_valid(v):
    return deb_cmp(v, "0") != 2


class DecodeError(Exception):
    pass


_FIELDS = {"vulnerabilityid": ("VulnerabilityID", str), "vendorids": ("VendorIDs", list),
           "arches": ("Arches", list), "status": ("Status", int), "severity": ("Severity", int),
           "fixedversion": ("FixedVersion", str), "affectedversion": ("AffectedVersion", str),
           "vulnerableversions": ("VulnerableVersions", list), "patchedversions": ("PatchedVersions", list),
           "unaffectedversions": ("UnaffectedVersions", list), "datasource": ("DataSource", dict),
           "custom": ("Custom", object)}


def decode_advisory(text):
    """json.Unmarshal into trivy-db types.Advisory (type errors -> DecodeError)."""
    try:
        v = json.loads(text)
    except ValueError as e:
        raise DecodeError(str(e))
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
        if name == "Custom":
            x = json.dumps(x, separators=(",", ":"))
        out[name] = x
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

    def get(self, root, name):
        """GetAdvisories(root, name): list of advisories sorted by vulnID, or raises DecodeError."""
        b = self.tree.get(("b", root), {}).get(("b", name))
        if not b:
            return []
        src = self.data_source(root)
        out = []
        for (kind, vid), val in sorted(b.items(), key=lambda kv: kv[0][1].encode()):
            if kind != "k":
                continue
            a = decode_advisory(val)
            a["VulnerabilityID"] = vid
            if src:
                a["DataSource"] = src
            elif "DataSource" in a:
                a["DataSource"] = {k: a["DataSource"][k] for k in ("ID", "Name", "URL") if a["DataSource"].get(k)}
            out.append(a)
        return out


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


def _base(p, a, installed):
    d = {"VulnerabilityID": a["VulnerabilityID"]}
    for k_out, val in [("PkgID", p.get("ID")), ("PkgName", p.get("Name")), ("PkgIdentifier", p.get("Identifier")),
                       ("InstalledVersion", installed), ("FixedVersion", a.get("FixedVersion")),
                       ("Layer", p.get("Layer")), ("DataSource", a.get("DataSource")), ("Custom", a.get("Custom"))]:
        if val:
            d[k_out] = val
    return d


def debian_detect(db, os_ver, pkgs):
    root = "debian " + major(os_ver)
    out = []
    for p in pkgs:
        src = fmt_src(p)
        if not deb_valid(src):
            continue
        try:
            advs = db.get(root, p.get("SrcName", ""))
        except DecodeError as e:
            raise DecodeError(f"failed to get debian advisories: failed to unmarshal advisory JSON: {e}")
        for a in advs:
            v = _base(p, a, fmt(p))
            if a.get("VendorIDs"):
                v["VendorIDs"] = a["VendorIDs"]
            if a.get("Status"):
                v["Status"] = a["Status"]
            if a.get("Severity", 0) != 0:
                v["SeveritySource"] = "debian"
                v["Severity"] = SEVERITY[a["Severity"]] if 0 < a["Severity"] < 5 else SEVERITY[0]
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


def _eol(y, m, d):
    import calendar
    return calendar.timegm((y, m, d, 23, 59, 59, 0, 0, 0))


# ubuntu.go:19-64 eolDates (transcribed data)
UBUNTU_EOL = {k: _eol(*v) for k, v in {
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
    "22.10": (2023, 7, 20), "23.04": (2024, 1, 20)}.items()}

# debian.go:20-40 eolDates
DEBIAN_EOL = {k: _eol(*v) for k, v in {
    "1.1": (1997, 6, 5), "1.2": (1998, 6, 5), "1.3": (1999, 3, 9), "2.0": (2000, 3, 9), "2.1": (2000, 10, 30),
    "2.2": (2003, 7, 30), "3.0": (2006, 6, 30), "3.1": (2008, 3, 30), "4.0": (2010, 2, 15), "5.0": (2012, 2, 6),
    "6.0": (2016, 2, 29), "7": (2018, 5, 31), "8": (2020, 6, 30), "9": (2022, 6, 30), "10": (2024, 6, 30),
    "11": (2026, 8, 14), "12": (2028, 6, 10), "13": (3000, 1, 1)}.items()}


def supported(eol, ver, now):
    """osver.Supported (version.go:31-38)."""
    return ver not in eol or now < eol[ver]


def ubuntu_version_from_eol(os_ver, now, eol):
    if os_ver in eol:
        return os_ver
    ver = os_ver.rstrip("-ESM")
    if ver in eol and now < eol[ver]:
        return ver
    return os_ver


def ubuntu_detect(db, os_ver, pkgs, now, eol=None):
    eol = UBUNTU_EOL if eol is None else eol
    out = []
    for p in pkgs:
        os_ver = ubuntu_version_from_eol(os_ver, now, eol)
        try:
            advs = db.get("ubuntu " + os_ver, p.get("SrcName", ""))
        except DecodeError as e:
            raise DecodeError(f"failed to get Ubuntu advisories: {e}")
        src = fmt_src(p)
        if not deb_valid(src):
            continue
        for a in advs:
            v = _base(p, a, fmt(p))
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


def amazon_detect(db, os_ver, pkgs):
    f = os_ver.split()
    v = major(f[0] if f else "")
    if v not in ("2", "2022", "2023"):
        v = "1"
    out = []
    for p in pkgs:
        try:
            advs = db.get("amazon linux " + v, p.get("Name", ""))
        except DecodeError as e:
            raise DecodeError(f"failed to get amazon advisories: {e}")
        inst = fmt(p)
        if inst == "" or not deb_valid(inst):
            continue
        for a in advs:
            r = deb_cmp(inst, a.get("FixedVersion", ""))
            if r == 3:
                continue
            if r < 0:
                out.append(_base(p, a, inst))
    return out
