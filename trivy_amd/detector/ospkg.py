"""Mirror of reference pkg/detector/ospkg (detect.go:30-91) over the C-ABI.

Packages and results use the reference's Go field names as dict keys
(ftypes.Package, types.DetectedVulnerability), so tests read like the Go tests.
Only non-zero fields appear in a result dict (Go's zero values omitted).
"""
import ctypes
import time

from .._lib import lib, s, errbuf, Package, Repository, Result, Str
from .._lib import TVM_EUNSUPPORTED_OS, COPY_PKG_ID, COPY_PKG_NAME, COPY_IDENTIFIER, COPY_LAYER


class UnsupportedOSError(Exception):
    """ospkg.ErrUnsupportedOS (detect.go:30)."""


class DetectError(Exception):
    pass


def _pkg_array(pkgs):
    arr = (Package * max(len(pkgs), 1))()
    keep = []
    for i, p in enumerate(pkgs):
        c = arr[i]
        for fld, key in [("id", "ID"), ("name", "Name"), ("version", "Version"), ("release", "Release"),
                         ("arch", "Arch"), ("src_name", "SrcName"), ("src_version", "SrcVersion"),
                         ("src_release", "SrcRelease"), ("modularitylabel", "Modularitylabel"),
                         ("file_path", "FilePath")]:
            st = s(p.get(key, ""))
            keep.append(st)
            setattr(c, fld, st)
        c.epoch = int(p.get("Epoch", 0))
        c.src_epoch = int(p.get("SrcEpoch", 0))
        bi = p.get("BuildInfo")
        if bi is not None:
            c.has_build_info = 1
            cs = bi.get("ContentSets") or []
            csa = (Str * max(len(cs), 1))(*[s(x) for x in cs])
            keep.append(csa)
            c.content_sets = ctypes.cast(csa, ctypes.POINTER(Str))
            c.n_content_sets = len(cs)
            for fld, key in [("nvr", "Nvr"), ("build_arch", "Arch")]:
                st = s(bi.get(key, ""))
                keep.append(st)
                setattr(c, fld, st)
    return arr, keep


def _repo(repo):
    if repo is None:
        return None, None
    r = Repository(s(repo.get("Family", "")), s(repo.get("Release", "")))
    return ctypes.pointer(r), r


def _now(now):
    if now is None:
        return int(time.time())
    if hasattr(now, "timestamp"):
        return int(now.timestamp())
    return int(now)


def _convert(res, pkgs):
    out = []
    for i in range(res.n):
        v = res.vulns[i]
        p = pkgs[v.pkg_index]
        d = {"VulnerabilityID": v.vulnerability_id.decode()}
        if v.n_vendor_ids:
            d["VendorIDs"] = [v.vendor_ids[k].decode() for k in range(v.n_vendor_ids)]
        if v.copy_flags & COPY_PKG_ID and p.get("ID"):
            d["PkgID"] = p["ID"]
        if v.copy_flags & COPY_PKG_NAME and p.get("Name"):
            d["PkgName"] = p["Name"]
        if v.pkg_path:
            d["PkgPath"] = v.pkg_path.decode()
        if v.copy_flags & COPY_IDENTIFIER and p.get("Identifier"):
            d["PkgIdentifier"] = p["Identifier"]
        if v.installed_version:
            d["InstalledVersion"] = v.installed_version.decode()
        if v.fixed_version:
            d["FixedVersion"] = v.fixed_version.decode()
        if v.status:
            d["Status"] = v.status
        if v.copy_flags & COPY_LAYER and p.get("Layer"):
            d["Layer"] = p["Layer"]
        if v.severity_source:
            d["SeveritySource"] = v.severity_source.decode()
        if v.has_data_source:
            d["DataSource"] = {k: val.decode() for k, val in [("ID", v.data_source_id), ("Name", v.data_source_name),
                                                              ("URL", v.data_source_url)] if val}
        if v.custom_json is not None:
            d["Custom"] = v.custom_json.decode()
        if v.severity:
            d["Severity"] = v.severity.decode()
        out.append(d)
    return out


def _call(fn, engine, family, os_ver, repo, pkgs, now):
    arr, keep = _pkg_array(pkgs)
    rp, _r = _repo(repo)
    res = Result()
    e = errbuf()
    rc = fn(engine.h, family.encode(), os_ver.encode(), rp, arr, len(pkgs), _now(now), ctypes.byref(res), e, len(e))
    if rc == TVM_EUNSUPPORTED_OS:
        raise UnsupportedOSError("unsupported os")
    if rc:
        raise DetectError(e.value.decode())
    try:
        return _convert(res, pkgs), bool(res.eosl)
    finally:
        lib().tvm_result_free(ctypes.byref(res))


def detect(engine, os_family, os_name, repo, pkgs, now=None):
    """ospkg.Detect (detect.go:63): returns (vulns, eosl)."""
    return _call(lib().tvm_ospkg_detect, engine, os_family, os_name, repo, pkgs, now)


class Scanner:
    """drivers[family] (detect.go:32-48): Detect + IsSupportedVersion."""

    def __init__(self, engine, family):
        self.engine, self.family = engine, family

    def detect(self, os_ver, repo, pkgs, now=None):
        return _call(lib().tvm_ospkg_driver_detect, self.engine, self.family, os_ver, repo, pkgs, now)[0]

    def is_supported_version(self, os_family, os_ver, now=None):
        r = lib().tvm_ospkg_is_supported(self.family.encode(), os_ver.encode(), _now(now))
        if r < 0:
            raise UnsupportedOSError(self.family)
        return bool(r)


def is_supported_version(family, os_ver, now=None):
    r = lib().tvm_ospkg_is_supported(family.encode(), os_ver.encode(), _now(now))
    if r < 0:
        raise UnsupportedOSError(family)
    return bool(r)
