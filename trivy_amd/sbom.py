"""CycloneDX SBOM -> detector input (mirror of pkg/sbom).

The step before the hot path for SBOM scans (`trivy sbom`, C1): the document's components
become the OS package list and the language applications the detectors consume, then
`scan` runs them through the GPU detectors (ospkg.Detect / library.Detect over the
C-ABI).  Host-side JSON work, O(components); it follows:

  pkg/sbom/cyclonedx/unmarshal.go:63-230  parseBOM / parseComponent (supported component
      types, PURL, "aquasecurity:trivy:" properties, metadata component = root,
      dependencies -> relationships between known bom-refs)
  pkg/sbom/io/decode.go:47-380            Decoder.Decode: one OS component at most, apps by
      their Type property (aggregating types carry no FilePath), libraries from their PURL
      (decodeLibrary: class must be OS or language; pkgName: component group/name; PkgID,
      FilePath, Src*, Modularitylabel, layer properties), fillSrcPkg for OS packages,
      the OS's dependencies -> OS packages, each app's dependencies -> its libraries,
      the rest: OS packages (one PURL type only, only when an OS is known) and one
      application per language type; applications sorted by (Type, FilePath)
  pkg/purl/purl.go:130-243                LangType / Class / Package (name from namespace,
      arch / epoch / modularitylabel qualifiers, rpm version-release split)
  pkg/fanal/types/artifact.go:203-211     Packages.Less (Name, Version, FilePath)
"""
import gc
import json
import re
import urllib.parse

NAMESPACE = "aquasecurity:trivy:"
AGGREGATING = {"python-pkg", "conda-pkg", "gemspec", "node-pkg", "jar"}
LANG_OF_PURL = {"composer": "composer", "maven": "jar", "gem": "gemspec", "conda": "conda-pkg",
                "pypi": "python-pkg", "golang": "gobinary", "npm": "node-pkg", "cargo": "cargo", "nuget": "nuget",
                "swift": "swift", "cocoapods": "cocoapods", "hex": "hex", "conan": "conan", "pub": "pub",
                "bitnami": "bitnami"}
K8S_LANG = {"eks": "eks", "gke": "gke", "aks": "aks", "ocp": "ocp", "": "kubernetes"}
OS_PURL_TYPES = {"apk", "deb", "rpm"}
CDX_TYPES = {"container", "application", "library", "operating-system", "platform"}


class SBOMError(Exception):
    pass


def parse_purl(s):
    """packageurl-go FromString: {type, namespace, name, version, qualifiers (ordered), subpath};
    raises SBOMError on a malformed PURL."""
    if not s.startswith("pkg:"):
        raise SBOMError("failed to parse PURL: scheme is not \"pkg\"")
    unq = urllib.parse.unquote if "%" in s else (lambda x: x)  # most PURLs carry no escapes
    rest = s[4:].lstrip("/")
    subpath = ""
    if "#" in rest:
        rest, sp = rest.split("#", 1)
        subpath = "/".join(unq(x) for x in sp.strip("/").split("/") if x not in ("", ".", ".."))
    quals = []
    if "?" in rest:
        rest, q = rest.split("?", 1)
        for kv in q.split("&"):
            k, _, v = kv.partition("=")
            if kv and v:
                quals.append((k.lower(), unq(v)))
    typ, _, rest = rest.partition("/")
    if not typ or not rest:
        raise SBOMError("failed to parse PURL: missing type or name")
    version = ""
    if "@" in rest:
        rest, version = rest.rsplit("@", 1)
        version = unq(version)
    segs = [unq(x) for x in rest.strip("/").split("/")]
    return {"type": typ.lower(), "namespace": "/".join(x for x in segs[:-1] if x), "name": segs[-1],
            "version": version, "qualifiers": quals, "subpath": subpath}


def lang_type(p):
    """purl.go:130-179."""
    if p["type"] == "k8s":
        return K8S_LANG.get(p["namespace"], "")
    return LANG_OF_PURL.get(p["type"], "")


def purl_class(p):
    """purl.go:181-193."""
    if p["type"] in OS_PURL_TYPES:
        return "os-pkgs"
    return "lang-pkgs" if lang_type(p) else ""


def go_atoi(v):
    """strconv.Atoi: an optional sign, then ASCII digits only (no spaces), within int64; None on
    error (parity unpinned: restated from Go's strconv, tests/test_sbom.py)."""
    if not _ATOI.fullmatch(v):
        return None
    x = int(v)
    return x if -(1 << 63) <= x < (1 << 63) else None


_ATOI = re.compile(r"[+-]?[0-9]+")


def _rpm_split(v):
    """go-rpm-version NewVersion (purl.go:238-240): [epoch:]version[-release], the release after
    the FIRST '-' as the comparator splits it (oracle/rpm.c)."""
    if ":" in v:
        v = v.split(":", 1)[1]
    ver, sep, rel = v.partition("-")
    return (ver, rel) if sep else (v, "")


def package_of(p):
    """purl.go:195-243 PackageURL.Package."""
    name = p["name"]
    cls = purl_class(p)
    if p["namespace"] and cls != "os-pkgs":
        name = p["namespace"] + (":" if p["type"] in ("maven", "gradle") else "/") + p["name"]
    if p["subpath"] and p["type"] == "cocoapods":
        name = p["name"] + "/" + p["subpath"]
    pkg = {"Name": name, "Version": p["version"]}
    for k, v in p["qualifiers"]:
        if k == "arch":
            pkg["Arch"] = v
        elif k == "modularitylabel":
            pkg["Modularitylabel"] = v
        elif k == "epoch" and go_atoi(v) is not None:  # purl.go:229-233: an error leaves Epoch as it is
            pkg["Epoch"] = go_atoi(v)
    if p["type"] == "rpm":
        pkg["Version"], pkg["Release"] = _rpm_split(p["version"])
    return pkg


def dependency_id(lang, name, version):
    """pkg/dependency/id.go:9-27: name + "@" + version; "/" for conan, ":" for
    jar/pom/gradle, Go versions get a "v" prefix; an empty version gives the name."""
    if not version:
        return name
    sep = "@"
    if lang == "conan":
        sep = "/"
    elif lang in ("gomod", "gobinary") and not version.startswith("v"):
        version = "v" + version
    elif lang in ("jar", "pom", "gradle"):
        sep = ":"
    return name + sep + version


def _component(c):
    """unmarshal.go parseComponent; None for an unsupported component type."""
    if c.get("type") not in CDX_TYPES:
        return None
    purl = parse_purl(c["purl"]) if c.get("purl") else None
    return {"type": c["type"], "name": c.get("name", ""), "group": c.get("group", ""),
            "version": c.get("version", ""), "bom_ref": c.get("bom-ref", ""), "purl": purl,
            "purl_str": c.get("purl", ""),
            "props": [(pr.get("name", "")[len(NAMESPACE):] if pr.get("name", "").startswith(NAMESPACE)
                       else pr.get("name", ""), pr.get("value", "")) for pr in c.get("properties") or []]}


def _library(c):
    """decode.go decodeLibrary (None: no PURL or an unsupported PURL type)."""
    p = c["purl"]
    if p is None or not purl_class(p):
        return None
    pkg = package_of(p)
    if p["type"] != "cocoapods":
        pkg["Name"] = (c["group"] + (":" if p["type"] in ("maven", "gradle") else "/") + c["name"]
                       if c["group"] else c["name"])
    pkg["ID"] = dependency_id(lang_type(p), pkg["Name"], p["version"])
    for k, v in c["props"]:
        if k == "PkgID":
            pkg["ID"] = v
        elif k == "FilePath":
            pkg["FilePath"] = v
        elif k in ("SrcName", "SrcVersion", "SrcRelease", "Modularitylabel"):
            pkg[k] = v
        elif k == "SrcEpoch":  # decode.go:208-211 strconv.Atoi
            e = go_atoi(v)
            if e is None:
                raise SBOMError("failed to decode components: failed to decode library: invalid src epoch")
            pkg["SrcEpoch"] = e
        elif k == "LayerDigest":
            pkg.setdefault("Layer", {})["Digest"] = v
        elif k == "LayerDiffID":
            pkg.setdefault("Layer", {})["DiffID"] = v
    for f in c.get("files") or []:  # decode.go:224-227: the first file path, unless a property set one
        if f and not pkg.get("FilePath"):
            pkg["FilePath"] = f
    pkg["Identifier"] = {"PURL": c["purl_str"], "BOMRef": c["bom_ref"]}
    pkg["_purl"] = p
    if purl_class(p) == "os-pkgs":  # fillSrcPkg (decode.go:260-279)
        if c.get("src_name") and not pkg.get("SrcName"):  # an SPDX "built package from" source
            pkg["SrcName"] = c["src_name"]
        if c.get("src_version"):  # parseSrcVersion (decode.go:282-301)
            _parse_src_version(pkg, p["type"], c["src_version"])
        if not pkg.get("SrcName"):
            pkg["SrcName"] = pkg["Name"]
        if not pkg.get("SrcVersion"):
            pkg["SrcVersion"] = pkg["Version"]
        if not pkg.get("SrcRelease"):
            pkg["SrcRelease"] = pkg.get("Release", "")
        if not pkg.get("SrcEpoch"):
            pkg["SrcEpoch"] = pkg.get("Epoch", 0)
    return pkg


def _parse_src_version(pkg, typ, ver):
    if typ == "rpm":  # go-rpm-version NewVersion: Atoi(epoch) before the first ':', release after the first '-'
        e, sep, rest = ver.partition(":")
        epoch, v = ((go_atoi(e) or 0), rest) if sep else (0, ver)
        v, _, rel = v.partition("-")
        pkg["SrcEpoch"], pkg["SrcVersion"], pkg["SrcRelease"] = epoch, v, rel
    elif typ == "deb":  # go-deb-version NewVersion; a parse error leaves the package as it is
        from .dpkg import deb_split, deb_valid
        if deb_valid(ver):
            pkg["SrcEpoch"], pkg["SrcVersion"], pkg["SrcRelease"] = deb_split(ver)


def _sort_pkgs(pkgs):
    return sorted(pkgs, key=lambda p: (p["Name"].encode(), p["Version"].encode(), p.get("FilePath", "").encode()))


def decode_cyclonedx(text):
    """CycloneDX JSON -> {"OS": {Family, Name} | None, "Packages": [...], "Applications":
    [{Type, FilePath, Libraries}], "Root": root component or None, "SerialNumber", "Version"}."""
    # the decode allocates several small containers per component and frees none of them:
    # cyclic-GC passes over that growing heap would dominate (2.7x slower at 100k components)
    enabled = gc.isenabled()
    gc.disable()
    try:
        return _decode(text)
    finally:
        if enabled:
            gc.enable()


def _decode(text):
    try:
        bom = json.loads(text)
    except ValueError as e:
        raise SBOMError("failed to decode CycloneDX JSON: %s" % e)
    return _decode_cdx(bom)


def _decode_cdx(bom):
    comps, order = {}, []
    for c in bom.get("components") or []:
        try:
            pc = _component(c)
        except SBOMError:
            continue  # parseComponents logs and skips a component it cannot parse
        if pc is not None:
            comps[pc["bom_ref"]] = pc
            order.append(pc)
    root = None
    mc = (bom.get("metadata") or {}).get("component")
    if mc:
        root = _component(mc)
        if root is None:
            raise SBOMError("failed to parse root component: unsupported component type")
        comps[root["bom_ref"]] = root
        order.append(root)
    rels = {}
    for d in bom.get("dependencies") or []:
        if d.get("ref") in comps:
            rels[id(comps[d["ref"]])] = [comps[x] for x in d.get("dependsOn") or [] if x in comps]
    return _decode_bom_meta(order, root, rels, bom.get("serialNumber", ""), bom.get("version", 0))


def _decode_bom(order, root, rels):
    """io/decode.go Decoder.Decode over the format-neutral BOM: components in document
    order, the root, and relationships {id(parent): [child components]}."""
    return _decode_bom_meta(order, root, rels, "", 0)


def _decode_bom_meta(order, root, rels, serial, version):
    os_c, apps, pkgs = None, {}, {}
    out = {"OS": None, "Packages": [], "Applications": [], "Root": root, "SerialNumber": serial, "Version": version}
    for c in order:
        if c["type"] == "operating-system":
            if os_c is not None:
                raise SBOMError("failed to decode components: multiple OS components are not supported")
            os_c = c
            out["OS"] = {"Family": c["name"], "Name": c["version"]}
            continue
        if c["type"] == "application":
            t = next((v for k, v in c["props"] if k == "Type"), "")
            if t:
                apps[id(c)] = {"Type": t, "FilePath": "" if t in AGGREGATING else c["name"], "Libraries": []}
                continue
        pkg = _library(c)
        if pkg is not None:
            pkgs[id(c)] = pkg
    if os_c is not None:
        os_pkgs = [pkgs.pop(id(d)) for d in rels.get(id(os_c), []) if id(d) in pkgs]
        if os_pkgs:
            out["Packages"] = os_pkgs
    for cid, app in apps.items():
        app["Libraries"] = [pkgs.pop(id(d)) for d in rels.get(cid, []) if id(d) in pkgs]
        out["Applications"].append(app)
    os_rest, lang_rest = {}, {}
    for pkg in pkgs.values():
        p = pkg["_purl"]
        if purl_class(p) == "os-pkgs":
            os_rest.setdefault(p["type"], []).append(pkg)
        else:
            lang_rest.setdefault(lang_type(p), []).append(pkg)
    if len(os_rest) > 1:
        raise SBOMError("failed to aggregate packages: multiple types of OS packages in SBOM are not supported")
    if os_rest and out["OS"] is not None and out["OS"]["Family"]:
        out["Packages"] = out["Packages"] + _sort_pkgs(next(iter(os_rest.values())))
    for t, libs in lang_rest.items():
        out["Applications"].append({"Type": t, "FilePath": "", "Libraries": _sort_pkgs(libs)})
    out["Applications"].sort(key=lambda a: (a["Type"].encode(), a["FilePath"].encode()))
    for p in out["Packages"] + [lib for a in out["Applications"] for lib in a["Libraries"]]:
        p.pop("_purl", None)
    return out


# ---- the native decoder (trivy_amd/csrc/sbom.cpp, tvm_sbom_*) ------------------------------------
_SP_KEYS = [(1, "Arch"), (2, "Epoch"), (4, "Release"), (8, "Modularitylabel"), (16, "FilePath"), (32, "SrcName"),
            (64, "SrcVersion"), (128, "SrcRelease"), (256, "SrcEpoch")]


class NativeSBOM:
    """A CycloneDX document decoded by the library (no Python objects per component): the
    OS, and per target (-1 = the OS packages, 0.. = applications) a tvm_package array the
    detectors take as it is (tvm_ospkg_detect / tvm_library_detect)."""

    def __init__(self, text):
        import ctypes
        from ._lib import lib, errbuf
        data = text.encode() if isinstance(text, str) else bytes(text)
        h, e = ctypes.c_void_p(), errbuf()
        # TVM_SBOM_BORROW: the decode points into `data`, which this object keeps alive
        if lib().tvm_sbom_decode_cyclonedx(data, len(data), 1, ctypes.byref(h), e, len(e)):
            raise SBOMError(e.value.decode())
        self.h, self._data = h, data
        from ._lib import RawStr
        has_os, fam, name, serial = ctypes.c_int32(), RawStr(), RawStr(), RawStr()
        ver, napps = ctypes.c_int64(), ctypes.c_size_t()
        lib().tvm_sbom_info(h, ctypes.byref(has_os), ctypes.byref(fam), ctypes.byref(name), ctypes.byref(serial),
                            ctypes.byref(ver), ctypes.byref(napps))
        self.os = {"Family": fam.bytes().decode(), "Name": name.bytes().decode()} if has_os.value else None
        self.serial, self.version, self.n_apps = serial.bytes().decode(), ver.value, napps.value

    def target(self, app):
        """(Type, FilePath, tvm_package pointer, n) of target `app` (-1: the OS packages)."""
        import ctypes
        from ._lib import lib, RawStr, RawPackage
        t, fp, pk, n = RawStr(), RawStr(), ctypes.POINTER(RawPackage)(), ctypes.c_size_t()
        lib().tvm_sbom_packages(self.h, app, ctypes.byref(t), ctypes.byref(fp), ctypes.byref(pk), ctypes.byref(n))
        return t.bytes().decode(), fp.bytes().decode(), pk, n.value

    def packages(self, app):
        """The packages of target `app` as trivy_amd/sbom.py's dicts (checker / inspection)."""
        import ctypes
        from ._lib import lib, SbomExtra
        _, _, pk, n = self.target(app)
        out = []
        ex = SbomExtra()
        for i in range(n):
            p = pk[i]
            lib().tvm_sbom_package_extra(self.h, app, i, ctypes.byref(ex))
            d = {"Name": p.name.bytes().decode(), "Version": p.version.bytes().decode(), "ID": p.id.bytes().decode()}
            vals = {"Arch": p.arch.bytes().decode(), "Epoch": p.epoch, "Release": p.release.bytes().decode(),
                    "Modularitylabel": p.modularitylabel.bytes().decode(), "FilePath": p.file_path.bytes().decode(),
                    "SrcName": p.src_name.bytes().decode(), "SrcVersion": p.src_version.bytes().decode(),
                    "SrcRelease": p.src_release.bytes().decode(), "SrcEpoch": p.src_epoch}
            for bit, k in _SP_KEYS:
                if ex.present & bit:
                    d[k] = vals[k]
            if ex.present & (512 | 1024):
                d["Layer"] = {}
                if ex.present & 512:
                    d["Layer"]["Digest"] = ex.layer_digest.bytes().decode()
                if ex.present & 1024:
                    d["Layer"]["DiffID"] = ex.layer_diff_id.bytes().decode()
            d["Identifier"] = {"PURL": ex.purl.bytes().decode(), "BOMRef": ex.bom_ref.bytes().decode()}
            out.append(d)
        return out

    def as_dict(self):
        """The decode in trivy_amd/sbom.py's form (without the root component)."""
        apps = []
        for a in range(self.n_apps):
            t, fp, _, _ = self.target(a)
            apps.append({"Type": t, "FilePath": fp, "Libraries": self.packages(a)})
        return {"OS": self.os, "Packages": self.packages(-1), "Applications": apps,
                "SerialNumber": self.serial, "Version": self.version}

    def close(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            from . import _lib
            if _lib._lib is not None:
                _lib._lib.tvm_sbom_free(h)

    def __del__(self):
        self.close()


def decode_cyclonedx_native(text):
    return NativeSBOM(text)


def scan_native(engine, nsbom, artifact_name="", now=None):
    """scan() over a NativeSBOM: the library's tvm_package arrays go to tvm_ospkg_detect /
    tvm_library_detect as they are (no per-package Python objects on the way in)."""
    import ctypes
    from ._lib import lib, errbuf, Package, Result, TVM_EUNSUPPORTED_TYPE
    from .detector.ospkg import _convert, _now, DetectError, UnsupportedOSError
    results = []

    def run(fn, app, *head):
        _, _, pk, n = nsbom.target(app)
        res, e = Result(), errbuf()
        rc = fn(engine.h, *head, ctypes.cast(pk, ctypes.POINTER(Package)), n, *(() if app >= 0 else (_now(now),)),
                ctypes.byref(res), e, len(e))
        if rc == TVM_EUNSUPPORTED_TYPE:
            return None
        if rc == 2 and app < 0:
            raise UnsupportedOSError("unsupported os")
        if rc:
            raise DetectError(e.value.decode())
        try:
            return _convert(res, nsbom.packages(app))
        finally:
            lib().tvm_result_free(ctypes.byref(res))

    if nsbom.os is not None and nsbom.os["Family"]:
        fam, name = nsbom.os["Family"], nsbom.os["Name"]
        vulns = run(lib().tvm_ospkg_detect, -1, fam.encode(), name.encode(), None)
        results.append(("os-pkgs", fam, "%s (%s %s)" % (artifact_name, fam, name), vulns))
    for a in range(nsbom.n_apps):
        t, fp, _, _ = nsbom.target(a)
        vulns = run(lib().tvm_library_detect, a, t.encode())
        if vulns is not None:
            results.append(("lang-pkgs", t, fp, vulns))
    return results


# ---- SPDX (pkg/sbom/spdx/unmarshal.go) and in-toto attestations (pkg/sbom/sbom.go) ----------------
SPDX_PURL_CATEGORIES = {"PACKAGE-MANAGER", "PACKAGE_MANAGER"}  # SPDX 2.3 / 2.2 spelling of the category


def _spdx_id(x):
    """tools-golang ElementID: the identifier without its "SPDXRef-" prefix."""
    return x[len("SPDXRef-"):] if x.startswith("SPDXRef-") else x


def _spdx_components(doc):
    """unmarshal.go: packages -> components (type from the SPDXID prefix, PURL from the
    PACKAGE-MANAGER purl reference, "built package from:" source, attribution texts as
    properties, the Trivy-legacy application form), the DESCRIBES target as root, every
    other relationship between two packages as an edge.  doc: {"creators", "packages":
    [{SPDXID, name, version, sourceInfo, purls: [(category, type, locator)], attributions}],
    "relationships": [(a, type, b)]}."""
    trivy = any(c.startswith("Tool: trivy") for c in doc["creators"])
    # parseFiles (unmarshal.go:107-132): a CONTAINS (or "CONTAIN") relationship from a package
    # to a File element gives the package that file's path (the last such relationship wins)
    files = doc.get("files") or {}
    file_of = {}
    for a, t, b in doc["relationships"]:
        if t in ("CONTAINS", "CONTAIN") and _spdx_id(b).startswith("File") and _spdx_id(b) in files:
            file_of[_spdx_id(a)] = files[_spdx_id(b)]
    root_id = next((_spdx_id(b) for a, t, b in doc["relationships"] if _spdx_id(a) == "DOCUMENT" and t == "DESCRIBES"),
                   None)
    comps, order = {}, []
    root = None
    for sp in doc["packages"]:
        sid = _spdx_id(sp["SPDXID"])
        typ = ("operating-system" if sid.startswith("OperatingSystem") else
               "application" if sid.startswith("Application") else "library")
        c = {"type": typ, "name": sp.get("name", ""), "group": "", "version": sp.get("version", ""), "bom_ref": "",
             "purl": None, "purl_str": "", "props": []}
        for cat, rtype, loc in sp.get("purls") or []:
            if rtype == "purl" and cat in SPDX_PURL_CATEGORIES:
                c["purl"], c["purl_str"] = parse_purl(loc), loc
                break
        src = sp.get("sourceInfo", "")
        if src.startswith("built package from"):
            src = src[len("built package from: "):] if src.startswith("built package from: ") else src
            c["src_name"], _, c["src_version"] = src.partition(" ")
        for at in sp.get("attributions") or []:
            k, sep, v = at.partition(": ")
            if sep:
                c["props"].append((k, v))
        if trivy and typ == "application" and sp.get("sourceInfo"):  # older Trivy: path in sourceInfo, type in name
            c["name"] = sp["sourceInfo"]
            c["props"].append(("Type", sp.get("name", "")))
        if sid in file_of:  # unmarshal.go:187-195: else the package's own first file
            c["files"] = [file_of[sid]]
        elif sp.get("files"):
            c["files"] = [sp["files"][0]]
        comps[sid] = c
        order.append(c)
        if sid == root_id:
            root = c
    rels = {}
    for a, t, b in doc["relationships"]:
        if t in ("DESCRIBES", "DESCRIBE"):
            continue
        ca, cb = comps.get(_spdx_id(a)), comps.get(_spdx_id(b))
        if ca is not None and cb is not None:
            rels.setdefault(id(ca), []).append(cb)
    return order, root, rels


def decode_spdx_json(text):
    """SPDX JSON (spdx/unmarshal.go UnmarshalJSON) -> the same result as decode_cyclonedx."""
    try:
        d = json.loads(text)
    except ValueError as e:
        raise SBOMError("failed to load spdx json: %s" % e)
    doc = {"creators": (d.get("creationInfo") or {}).get("creators") or [], "packages": [], "relationships": [],
           "files": {_spdx_id(f.get("SPDXID", "")): f.get("fileName", "") for f in d.get("files") or []}}
    has_files = []
    for p in d.get("packages") or []:
        # tools-golang turns the deprecated hasFiles into CONTAINS relationships (spdx/tools-golang#201)
        has_files += [(p.get("SPDXID", ""), "CONTAINS", f) for f in p.get("hasFiles") or []]
        doc["packages"].append({
            "SPDXID": p.get("SPDXID", ""), "name": p.get("name", ""), "version": p.get("versionInfo", ""),
            "sourceInfo": p.get("sourceInfo", ""), "attributions": p.get("attributionTexts") or [],
            "purls": [(r.get("referenceCategory", ""), r.get("referenceType", ""), r.get("referenceLocator", ""))
                      for r in p.get("externalRefs") or []]})
    for r in d.get("relationships") or []:
        doc["relationships"].append((r.get("spdxElementId", ""), r.get("relationshipType", ""),
                                     r.get("relatedSpdxElement", "")))
    doc["relationships"] += has_files
    order, root, rels = _spdx_components(doc)
    return _decode_bom(order, root, rels)


def _tv_pairs(text):
    """SPDX tag-value: (tag, value) per line; <text>...</text> values span lines."""
    lines = text.split("\n")
    i = 0
    while i < len(lines):
        line = lines[i].rstrip("\r")
        i += 1
        if not line.strip() or line.lstrip().startswith("#"):
            continue
        tag, sep, val = line.partition(":")
        if not sep:
            raise SBOMError("failed to load tag-value spdx: invalid line %d" % i)
        val = val.strip()
        if val.startswith("<text>"):
            val = val[len("<text>"):]
            while "</text>" not in val and i < len(lines):
                val += "\n" + lines[i].rstrip("\r")
                i += 1
            val = val.split("</text>", 1)[0]
        yield tag.strip(), val


def decode_spdx_tv(text):
    """SPDX tag-value (spdx/unmarshal.go TVDecoder) -> the same result as decode_cyclonedx."""
    doc = {"creators": [], "packages": [], "relationships": [], "files": {}}
    cur = cur_file = last_pkg = None
    for tag, val in _tv_pairs(text):
        if tag == "Creator":
            doc["creators"].append(val)
        elif tag == "PackageName":
            cur = {"SPDXID": "", "name": val, "version": "", "sourceInfo": "", "attributions": [], "purls": [],
                   "files": []}
            doc["packages"].append(cur)
            last_pkg, cur_file = cur, None
        elif tag == "FileName":  # a file section; a file that follows a package is one of its files
            cur, cur_file = None, {"name": val, "id": ""}
            if last_pkg is not None:
                last_pkg["files"].append(val)
        elif tag == "SnippetSPDXID":
            cur = cur_file = None  # a snippet section: its SPDXID is not a package's
        elif tag == "SPDXID" and cur_file is not None and not cur_file["id"]:
            cur_file["id"] = val
            doc["files"][_spdx_id(val)] = cur_file["name"]
        elif tag == "SPDXID" and cur is not None and not cur["SPDXID"]:
            cur["SPDXID"] = val
        elif cur is not None and tag == "PackageVersion":
            cur["version"] = val
        elif cur is not None and tag == "PackageSourceInfo":
            cur["sourceInfo"] = val
        elif cur is not None and tag == "PackageAttributionText":
            cur["attributions"].append(val)
        elif cur is not None and tag == "ExternalRef":
            f = val.split(None, 2)
            if len(f) == 3:
                cur["purls"].append((f[0], f[1], f[2]))
        elif tag == "Relationship":
            f = val.split()
            if len(f) >= 3:
                doc["relationships"].append((f[0], f[1], f[2]))
    order, root, rels = _spdx_components(doc)
    return _decode_bom(order, root, rels)


def decode_intoto(text):
    """An in-toto attestation of a CycloneDX BOM in a DSSE envelope (sbom.go
    decodeAttestCycloneDXJSONFormat + attestation.Statement.UnmarshalJSON): the first line."""
    import base64
    line = text.strip().split("\n", 1)[0]
    try:
        env = json.loads(line)
    except ValueError as e:
        raise SBOMError("failed to decode as a dsse envelope: %s" % e)
    if env.get("payloadType") != "application/vnd.in-toto+json":
        raise SBOMError("invalid attestation payload type: %s" % env.get("payloadType"))
    try:
        st = json.loads(base64.b64decode(env.get("payload", ""), validate=True))
    except (ValueError, TypeError) as e:
        raise SBOMError("failed to decode attestation payload: %s" % e)
    if st.get("predicateType") not in ("https://cyclonedx.org/bom", "https://cyclonedx.org/schema"):
        raise SBOMError("unsupported predicate type: %s" % st.get("predicateType"))
    pred = st.get("predicate")
    if not isinstance(pred, dict):
        raise SBOMError("no predicate")
    if "Data" in pred:  # legacy cosign predicate: {"Data": <BOM>}
        pred = pred["Data"] if isinstance(pred["Data"], dict) else json.loads(pred["Data"])
    return _decode_cdx(pred)


def decode(text):
    """sbom.go DetectFormat + Decode for the formats above."""
    s = text.lstrip()
    if s.startswith("{"):
        try:
            d = json.loads(s.split("\n", 1)[0]) if s.count("\n") and s.split("\n", 1)[0].rstrip().endswith("}") \
                else json.loads(s)
        except ValueError:
            try:
                d = json.loads(s)
            except ValueError:  # sbom.go DetectFormat: undecodable JSON is no known format
                raise SBOMError("failed to detect SBOM format") from None
        if not isinstance(d, dict):
            raise SBOMError("failed to detect SBOM format")
        if d.get("bomFormat") == "CycloneDX":
            return decode_cyclonedx(text)
        if str(d.get("spdxVersion", "")).startswith("SPDX-"):
            return decode_spdx_json(text)
        if "payloadType" in d:
            return decode_intoto(text)
    elif s.startswith("SPDX"):
        return decode_spdx_tv(text)
    raise SBOMError("failed to detect SBOM format")


def scan(engine, sbom, artifact_name="", now=None):
    """The detector part of scanning a decoded SBOM: ospkg.Detect over the OS packages and
    library.Detect per application, on the GPU.  Returns [(class, type, target, vulns)];
    the OS target is "<artifact> (<family> <name>)" as pkg/scanner/local names it."""
    from .detector import library, ospkg
    results = []
    if sbom["OS"] is not None and sbom["OS"]["Family"]:
        fam, name = sbom["OS"]["Family"], sbom["OS"]["Name"]
        vulns, _eosl = ospkg.detect(engine, fam, name, None, sbom["Packages"], now=now)
        results.append(("os-pkgs", fam, "%s (%s %s)" % (artifact_name, fam, name), vulns))
    for app in sbom["Applications"]:
        vulns = library.detect(engine, app["Type"], app["Libraries"])
        if vulns is not None:
            results.append(("lang-pkgs", app["Type"], app["FilePath"], vulns))
    return results
