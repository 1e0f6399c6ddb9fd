"""dpkg status database -> installed packages (mirror of the dpkg analyzer; SURVEY.md §8f
rank 4, the producer of Debian/Ubuntu package batches for image scans).

Follows pkg/fanal/analyzer/pkg/dpkg:
  scanner.go:13-56     blocks separated by an empty line ("\\n\\n"), each read as a MIME
                       header (net/textproto ReadMIMEHeader: canonical keys, continuation
                       lines folded into the value, a malformed line fails the block)
  dpkg.go:175-209      parseDpkgStatus: packages keyed by ID (a later block with the same
                       ID replaces the earlier), name -> ID for the dependency pass
  dpkg.go:211-268      parseDpkgPkg: "deinstall"/"purge" status or a missing name/version
                       drops the block; Source "name (version)"; the installed and source
                       versions split into epoch / version / revision by go-deb-version (an
                       invalid one drops the package)
  dpkg.go:292-336      parseDepends / trimVersionRequirement / consolidateDependencies
                       (alternatives kept, versions cut, unknown names dropped, IDs sorted)
Version validity is the product's own dpkg grammar (the sort-key encoder behind
tvm_version_key, the same code the GPU match kernel runs).
"""
import re

from ._lib import lib

_SRC = re.compile(r"(?P<name>[^\s]*)( \((?P<version>.*)\))?")
_TOKEN = re.compile(r"[!#$%&'*+\-.^_`|~0-9A-Za-z]+")


class MIMEError(Exception):
    pass


def _canonical_key(k):
    """textproto.CanonicalMIMEHeaderKey."""
    return "-".join(p[:1].upper() + p[1:].lower() for p in k.split("-"))


def read_mime_header(block):
    """{canonical key: [values]} of one block; MIMEError where ReadMIMEHeader fails."""
    lines = block.split("\n")
    if lines and lines[0][:1] in (" ", "\t"):
        raise MIMEError("malformed MIME header initial line: " + lines[0])
    hdr, i = {}, 0
    while i < len(lines):
        line = lines[i].rstrip("\r")
        if line == "":
            break  # the blank line that ends a header
        i += 1
        while i < len(lines) and lines[i][:1] in (" ", "\t"):  # continuation lines
            line = line.rstrip(" \t") + " " + lines[i].strip(" \t\r")
            i += 1
        key, sep, value = line.partition(":")
        if not sep or not _TOKEN.fullmatch(key):
            raise MIMEError("malformed MIME header line: " + line)
        hdr.setdefault(_canonical_key(key), []).append(value.strip(" \t\r"))
    return hdr


def _get(hdr, key):
    v = hdr.get(key)
    return v[0] if v else ""


def deb_valid(v):
    b = v.encode()
    return lib().tvm_version_key(1, b, len(b), None, 0) >= 0


def deb_split(v):
    """go-deb-version Version(): (epoch, upstream version, revision)."""
    v = v.strip()
    epoch = 0
    if ":" in v:
        e, v = v.split(":", 1)
        epoch = int(e)
    ver, sep, rev = v.rpartition("-")
    return (epoch, ver, rev) if sep else (epoch, v, "")


def _depends(s):
    out = []
    for dep in s.split(","):
        for d in dep.split("|"):
            d = d.split("(", 1)[0].strip()
            if d not in out:
                out.append(d)
    return out


def parse_package(hdr):
    """parseDpkgPkg: a package dict (Go zero values omitted) or None."""
    if any(x in ("deinstall", "purge") for x in _get(hdr, "Status").split()):
        return None
    name, version = _get(hdr, "Package"), _get(hdr, "Version")
    if not name or not version:
        return None
    pkg = {"Name": name, "Version": version, "DependsOn": _depends(_get(hdr, "Depends")),
           "Maintainer": _get(hdr, "Maintainer"), "Arch": _get(hdr, "Architecture")}
    src_name = src_ver = ""
    src = _get(hdr, "Source")
    if src:
        m = _SRC.search(src)
        src_name, src_ver = (m.group("name") or "").strip(), (m.group("version") or "").strip()
    src_name = src_name or name
    src_ver = src_ver or version
    if not deb_valid(version):
        return None
    pkg["ID"] = "%s@%s" % (name, version)
    pkg["Epoch"], pkg["Version"], pkg["Release"] = deb_split(version)
    if not deb_valid(src_ver):
        return None
    pkg["SrcName"] = src_name
    pkg["SrcEpoch"], pkg["SrcVersion"], pkg["SrcRelease"] = deb_split(src_ver)
    return pkg


def parse_status(text, file_path="var/lib/dpkg/status"):
    """parseDpkgStatus: [{FilePath, Packages}] with packages in Packages.Less order
    (Name, Version, FilePath), as the reference's test sorts them."""
    pkgs, ids = {}, {}
    pos = 0
    while pos < len(text):
        i = text.find("\n\n", pos)
        block, pos = (text[pos:i], i + 2) if i >= 0 else (text[pos:], len(text))
        try:
            hdr = read_mime_header(block)
        except MIMEError:
            continue  # logged and skipped
        p = parse_package(hdr)
        if p is not None:
            pkgs[p["ID"]] = p
            ids[p["Name"]] = p["ID"]
    out = []
    for p in pkgs.values():
        deps = sorted(ids[d] for d in p["DependsOn"] if d in ids)
        p["DependsOn"] = deps
        out.append({k: v for k, v in p.items() if v not in ("", 0, [], None)})
    out.sort(key=lambda p: (p["Name"].encode(), p["Version"].encode(), p.get("FilePath", "").encode()))
    return [{"FilePath": file_path, "Packages": out}]
