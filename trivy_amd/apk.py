"""Alpine installed database (lib/apk/db/installed) -> installed packages (mirror of the apk
analyzer; SURVEY.md §8f rank 4, the producer of Alpine package batches for image scans).

Follows pkg/fanal/analyzer/pkg/apk/apk.go:
  :55-124   parseApkInfo: one package per blank-line separated block; P name, V version
            (an invalid apk version is ignored), o origin = source name with the version
            seen so far, A arch, C checksum (Q1 = base64 SHA-1, else MD5), F/R installed
            files (path.Join), p provides and D depends for the dependency graph; a block
            needs a name and a version
  :126-131  trimRequirement (cut at the first '<', '>' or '=')
  :155-170  parseProvides / parseDependencies ('!' conflicts dropped)
  :172-200  consolidateDependencies (provided names -> IDs, sorted, compacted) and
            uniquePkgs (the first package of a name wins)
  :218-236  decodeChecksumLine
License strings (L:) are kept as written: the licensing.Normalize alias table is not on
the vulnerability path.  Version validity is the product's apk grammar (the sort-key
encoder behind tvm_version_key, the same code the GPU match kernel runs).
"""
import base64
import binascii
import posixpath

from ._lib import lib


def apk_valid(v):
    b = v.encode()
    return lib().tvm_version_key(2, b, len(b), None, 0) >= 0


def _path_join(*elems):
    """Go path.Join: the non-empty elements joined with '/', then Clean."""
    parts = [e for e in elems if e]
    if not parts:
        return ""
    return posixpath.normpath("/".join(parts)).replace("//", "/")


def _trim(s):
    i = min((s.find(c) for c in "<>=" if c in s), default=-1)
    return s[:i] if i >= 0 else s


def _checksum(line):
    d, alg = line[2:], "md5"
    if d.startswith("Q1"):
        alg, d = "sha1", d[2:]
    try:
        raw = base64.b64decode(d, validate=True)
    except (binascii.Error, ValueError):
        return ""
    return alg + ":" + raw.hex()


def parse_installed(text, file_path="lib/apk/db/installed"):
    """Returns ([{FilePath, Packages}], system installed files)."""
    pkgs, files, provides = [], [], {}
    pkg, version, cur_dir = {}, "", ""

    def flush():
        if pkg.get("Name") and pkg.get("Version"):
            pkgs.append(pkg)

    for line in text.split("\n"):
        if len(line) < 2:
            flush()
            pkg = {}
            continue
        tag, val = line[:2], line[2:]
        if tag == "P:":
            pkg["Name"] = val
        elif tag == "V:":
            version = val
            if not apk_valid(version):
                continue
            pkg["Version"] = version
        elif tag == "o:":
            pkg["SrcName"], pkg["SrcVersion"] = val, version
        elif tag == "L:":
            pkg["Licenses"] = [x for x in val.split()] or None
        elif tag == "F:":
            cur_dir = val
        elif tag == "R:":
            f = _path_join(cur_dir, val)
            pkg.setdefault("InstalledFiles", []).append(f)
            files.append(f)
        elif tag == "p:":
            for p in val.split():
                provides[_trim(p)] = pkg.get("ID", "")
        elif tag == "D:":
            pkg["DependsOn"] = [_trim(d) for d in val.split() if not d.startswith("!")]
        elif tag == "A:":
            pkg["Arch"] = val
        elif tag == "C:":
            d = _checksum(line)
            if d:
                pkg["Digest"] = d
        if pkg.get("Name") and pkg.get("Version"):
            pkg["ID"] = "%s@%s" % (pkg["Name"], pkg["Version"])
            provides[pkg["Name"]] = pkg["ID"]
    flush()
    seen, uniq = set(), []
    for p in pkgs:  # uniquePkgs
        if p["Name"] not in seen:
            seen.add(p["Name"])
            uniq.append(p)
    for p in uniq:  # consolidateDependencies
        deps = sorted(set(provides[d] for d in p.get("DependsOn") or () if d in provides))
        if deps:
            p["DependsOn"] = deps
        else:
            p.pop("DependsOn", None)
    order = ["ID", "Name", "Version", "SrcName", "SrcVersion", "Licenses", "DependsOn", "Arch", "Digest",
             "InstalledFiles"]
    out = [{k: p[k] for k in order if p.get(k)} for p in uniq]
    return [{"FilePath": file_path, "Packages": out}], files
