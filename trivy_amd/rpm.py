"""RPM installed database -> installed packages (mirror of the rpm and rpmqa analyzers;
SURVEY.md §8f rank 4, the producer of Red Hat-family package batches for image scans).

Follows pkg/fanal/analyzer/pkg/rpm/rpm.go:
  :105-193  listPkgs: one Package per PackageInfo - ID name@version-release.arch, arch ""
            -> "None", EpochNum for Epoch and SrcEpoch, the source RPM split by
            splitFileName (an invalid one leaves the Src* fields empty), installed files
            (DirNames[DirIndexes[i]] joined with BaseNames[i]) only for vendor-provided
            packages, MD5 digest from SIGMD5, Requires -> DependsOn through Provides
            (consolidateDependencies :278-295)
  :214-236  splitFileName (yum rpmUtils.miscutils.splitFilename: last '.', then the last
            two '-')
  :238-252  packageProvidedByVendor (vendor prefixes; no vendor: "amzn" in the release)
and pkg/fanal/analyzer/pkg/rpm/rpmqa.go:48-84 (the CBL-Mariner distroless manifest).

The database containers are read by github.com/knqyf263/go-rpmdb (reference go.mod, not in
the reference checkout); its published formats are restated here:
  * the rpm header blob (rpm's headerImport layout): be32 index count, be32 data size,
    16-byte index entries {tag, type, offset, count} (big-endian), then the data store;
  * SQLite (rpm >= 4.16, RHEL 9 / Fedora): table Packages(hnum, blob);
  * Berkeley DB hash (RHEL <= 8, CentOS): hash pages whose values point (H_OFFPAGE) at
    chains of overflow pages holding one header blob each;
  * NDB (SUSE): slot pages {'Slot', pkg index, block offset, block count} pointing at
    16-byte-aligned blobs {'BlbS', pkg index, generation, length, blob}.
The reference checkout holds no rpm database fixture (pkg/fanal/analyzer/pkg/rpm/testdata
is absent), so the container readers are parity-unpinned: tests build databases with the
layouts above and check the round trip.  listPkgs, splitFileName and the rpmqa parser are
pinned by the reference's own tables (rpm_test.go:70-260, rpmqa_test.go:12-75).
"""
import posixpath
import sqlite3
import struct

# rpm tags (rpm lib/rpmtag.h) go-rpmdb's PackageInfo reads
TAG = {
    "NAME": 1000, "VERSION": 1001, "RELEASE": 1002, "EPOCH": 1003, "SUMMARY": 1004, "INSTALLTIME": 1008,
    "SIZE": 1009, "VENDOR": 1011, "LICENSE": 1014, "ARCH": 1022, "SOURCERPM": 1044, "PROVIDENAME": 1047,
    "REQUIRENAME": 1049, "DIRINDEXES": 1116, "BASENAMES": 1117, "DIRNAMES": 1118, "SIGMD5": 261,
    "PGP": 259, "MODULARITYLABEL": 5096, "FILEDIGESTALGO": 5011,
}
# header value types (rpm lib/rpmtypes.h)
T_CHAR, T_INT8, T_INT16, T_INT32, T_INT64, T_STRING, T_BIN, T_STRING_ARRAY, T_I18NSTRING = 1, 2, 3, 4, 5, 6, 7, 8, 9
_REGION_TAGS = (61, 62, 63)  # HEADERSIGNATURES / HEADERIMMUTABLE / HEADERREGIONS: region trailers, skipped

OS_VENDORS = ["Amazon Linux", "Amazon.com", "CentOS", "Fedora Project", "Oracle America", "Red Hat", "AlmaLinux",
              "CloudLinux", "VMware", "SUSE", "openSUSE", "Microsoft Corporation", "Rocky"]


class RpmError(Exception):
    pass


# ---- splitFileName / vendor / listPkgs (rpm.go) ---------------------------------------------------
def split_file_name(filename):
    """(name, version, release); RpmError("unexpected name format") (rpm.go:214-236)."""
    if filename.endswith(".rpm"):
        filename = filename[:-4]
    arch = filename.rfind(".")
    if arch == -1:
        raise RpmError("unexpected name format")
    rel = filename.rfind("-", 0, arch)
    if rel == -1:
        raise RpmError("unexpected name format")
    ver = filename.rfind("-", 0, rel)
    if ver == -1:
        raise RpmError("unexpected name format")
    return filename[:ver], filename[ver + 1:rel], filename[rel + 1:arch]


def provided_by_vendor(info):
    vendor = info.get("Vendor") or ""
    if vendor == "":
        return "amzn" in (info.get("Release") or "")
    return any(vendor.startswith(v) for v in OS_VENDORS)


def _filepath_join(d, b):
    """Go filepath.Join of two elements (Clean of the '/'-joined non-empty parts)."""
    parts = [x for x in (d, b) if x]
    if not parts:
        return ""
    return posixpath.normpath("/".join(parts)).replace("//", "/")


def installed_file_names(info):
    """go-rpmdb PackageInfo.InstalledFileNames."""
    dirs, idx, base = info.get("DirNames") or [], info.get("DirIndexes") or [], info.get("BaseNames") or []
    if not dirs or not idx or not base:
        return []
    if len(idx) != len(base) or len(dirs) > len(base):
        raise RpmError("invalid rpm database")
    out = []
    for i, b in enumerate(base):
        if idx[i] < 0 or idx[i] >= len(dirs):
            raise RpmError("invalid rpm database")
        out.append(_filepath_join(dirs[idx[i]], b))
    return out


def list_pkgs(infos):
    """listPkgs (rpm.go:105-193): (packages, installed files)."""
    pkgs, files_all, provides = [], [], {}
    for info in infos:
        arch = info.get("Arch") or ""
        src_name = src_ver = src_rel = ""
        src = info.get("SourceRpm") or ""
        if src not in ("(none)", ""):
            try:
                src_name, src_ver, src_rel = split_file_name(src)
            except RpmError:
                src_name = src_ver = src_rel = ""
        files = []
        if provided_by_vendor(info):
            files = installed_file_names(info)
        epoch = info.get("Epoch") or 0
        p = {"ID": "%s@%s-%s.%s" % (info.get("Name", ""), info.get("Version", ""), info.get("Release", ""), arch),
             "Name": info.get("Name", ""), "Epoch": epoch, "Version": info.get("Version", ""),
             "Release": info.get("Release", ""), "Arch": arch or "None", "SrcName": src_name, "SrcEpoch": epoch,
             "SrcVersion": src_ver, "SrcRelease": src_rel, "Modularitylabel": info.get("Modularitylabel", ""),
             "Licenses": [info["License"]] if info.get("License") else None,
             "DependsOn": list(info.get("Requires") or []), "Maintainer": info.get("Vendor", ""),
             "Digest": ("md5:" + info["SigMD5"]) if info.get("SigMD5") else "",
             "InstalledFiles": files or None}
        pkgs.append(p)
        files_all += files
        for prov in info.get("Provides") or []:
            provides[prov] = p["ID"]
    for p in pkgs:  # consolidateDependencies (rpm.go:278-295)
        deps = sorted({provides[d] for d in p["DependsOn"] if d in provides and provides[d] != p["ID"]})
        p["DependsOn"] = deps or None
    return pkgs, files_all


def parse_rpmqa_manifest(text):
    """rpmqa.go:48-84: NAME VERSION-RELEASE ... ARCH EPOCHNUM SOURCERPM (tab separated)."""
    pkgs = []
    lines = text.split("\n")
    if lines and lines[-1] == "":  # bufio.Scanner: no token after a final newline
        lines.pop()
    for line in lines:
        line = line[:-1] if line.endswith("\r") else line  # ScanLines drops a trailing \r
        s = line.split("\t")
        if len(s) != 10:
            raise RpmError(f"failed to parse a line ({line})")
        vr = s[1].split("-")
        if len(vr) != 2:
            raise RpmError(f"failed to split a version ({s[1]})")
        try:
            sn, sv, sr = split_file_name(s[9])
        except RpmError as e:
            raise RpmError(f"failed to split source rpm: {e}")
        pkgs.append({"Name": s[0], "Version": vr[0], "Release": vr[1], "Arch": s[7], "SrcName": sn,
                     "SrcVersion": sv, "SrcRelease": sr})
    return pkgs


# ---- the rpm header blob ----------------------------------------------------------------------------
def header_import(blob):
    """{tag: value} of one header blob (strings decoded as UTF-8 with replacement)."""
    if len(blob) < 8:
        raise RpmError("header blob too short")
    il, dl = struct.unpack_from(">ii", blob, 0)
    if il < 0 or dl < 0 or 8 + 16 * il + dl > len(blob):
        raise RpmError("invalid header blob")
    data = blob[8 + 16 * il: 8 + 16 * il + dl]
    out = {}
    for i in range(il):
        tag, typ, off, cnt = struct.unpack_from(">iiii", blob, 8 + 16 * i)
        if tag in _REGION_TAGS:
            continue
        if off < 0 or off > dl:
            raise RpmError("invalid header entry offset")
        out[tag] = _decode_value(data, typ, off, cnt)
    return out


def _decode_value(data, typ, off, cnt):
    if typ in (T_STRING, T_I18NSTRING, T_STRING_ARRAY):
        vals, p = [], off
        n = 1 if typ == T_STRING else cnt
        for _ in range(n):
            e = data.find(b"\0", p)
            if e < 0:
                raise RpmError("unterminated string")
            vals.append(data[p:e].decode("utf-8", "replace"))
            p = e + 1
        return vals[0] if typ == T_STRING else vals
    if typ == T_INT32:
        return list(struct.unpack_from(">%di" % cnt, data, off))
    if typ == T_INT16:
        return list(struct.unpack_from(">%dh" % cnt, data, off))
    if typ == T_INT64:
        return list(struct.unpack_from(">%dq" % cnt, data, off))
    if typ in (T_CHAR, T_INT8):
        return list(data[off:off + cnt])
    if typ == T_BIN:
        return bytes(data[off:off + cnt])
    raise RpmError(f"unknown header type {typ}")


def package_info(hdr):
    """go-rpmdb PackageInfo fields (as listPkgs reads them) from a decoded header."""
    def s(tag):
        v = hdr.get(TAG[tag], "")
        return v[0] if isinstance(v, list) and v else (v if isinstance(v, str) else "")

    def arr(tag):
        v = hdr.get(TAG[tag])
        return list(v) if isinstance(v, list) else []

    epoch = hdr.get(TAG["EPOCH"])
    md5 = hdr.get(TAG["SIGMD5"])
    return {"Name": s("NAME"), "Version": s("VERSION"), "Release": s("RELEASE"),
            "Epoch": epoch[0] if epoch else None, "Arch": s("ARCH"), "SourceRpm": s("SOURCERPM"),
            "Vendor": s("VENDOR"), "License": s("LICENSE"), "Modularitylabel": s("MODULARITYLABEL"),
            "SigMD5": md5.hex() if isinstance(md5, bytes) else "", "DirNames": arr("DIRNAMES"),
            "DirIndexes": arr("DIRINDEXES"), "BaseNames": arr("BASENAMES"), "Provides": arr("PROVIDENAME"),
            "Requires": arr("REQUIRENAME")}


def header_export(fields):
    """Header blob from {tag: (type, value)} (test helper: the layout header_import reads)."""
    index, store = [], b""
    for tag, (typ, val) in sorted(fields.items()):
        align = {T_INT16: 2, T_INT32: 4, T_INT64: 8}.get(typ, 1)
        store += b"\0" * ((-len(store)) % align)
        off = len(store)
        if typ == T_STRING:
            store += val.encode() + b"\0"
            cnt = 1
        elif typ in (T_STRING_ARRAY, T_I18NSTRING):
            store += b"".join(v.encode() + b"\0" for v in val)
            cnt = len(val)
        elif typ == T_INT32:
            store += struct.pack(">%di" % len(val), *val)
            cnt = len(val)
        elif typ == T_INT16:
            store += struct.pack(">%dh" % len(val), *val)
            cnt = len(val)
        elif typ == T_BIN:
            store += val
            cnt = len(val)
        else:
            raise RpmError(f"unsupported type {typ}")
        index.append(struct.pack(">iiii", tag, typ, off, cnt))
    return struct.pack(">ii", len(index), len(store)) + b"".join(index) + store


# ---- database containers (go-rpmdb) -----------------------------------------------------------------
_BDB_HASH_MAGIC = 0x061561
_NDB_MAGIC = int.from_bytes(b"RpmP", "little")
_NDB_SLOT_MAGIC = int.from_bytes(b"Slot", "little")
_NDB_BLOB_MAGIC = int.from_bytes(b"BlbS", "little")
_P_HASH_UNSORTED, _P_OVERFLOW, _P_HASH = 2, 7, 13
_H_OFFPAGE = 3


def detect_format(raw):
    if raw[:16] == b"SQLite format 3\0":
        return "sqlite"
    if len(raw) >= 16 and int.from_bytes(raw[:4], "little") == _NDB_MAGIC:
        return "ndb"
    if len(raw) >= 16:
        for order in ("little", "big"):
            if int.from_bytes(raw[12:16], order) == _BDB_HASH_MAGIC:
                return "bdb"
    raise RpmError("unknown rpm database format")


def _blobs_sqlite(path):
    con = sqlite3.connect("file:%s?mode=ro" % path, uri=True)
    try:
        return [bytes(r[0]) for r in con.execute("SELECT blob FROM Packages ORDER BY hnum")]
    finally:
        con.close()


def _blobs_bdb(raw):
    order = "little" if int.from_bytes(raw[12:16], "little") == _BDB_HASH_MAGIC else "big"
    e = "<" if order == "little" else ">"
    page_size = struct.unpack_from(e + "I", raw, 20)[0]
    last_pgno = struct.unpack_from(e + "I", raw, 32)[0]
    if page_size < 512 or page_size > 65536:
        raise RpmError("invalid bdb page size")

    def page(n):
        b = n * page_size
        if b + page_size > len(raw):
            raise RpmError("bdb page out of range")
        return raw[b:b + page_size]

    out = []
    for n in range(1, last_pgno + 1):
        pg = page(n)
        typ = pg[25]
        if typ not in (_P_HASH, _P_HASH_UNSORTED):
            continue
        entries = struct.unpack_from(e + "H", pg, 20)[0]
        offs = struct.unpack_from(e + "%dH" % entries, pg, 26)
        for i in range(1, entries, 2):  # (key, value) pairs: the values
            o = offs[i]
            if pg[o] != _H_OFFPAGE:
                continue
            pgno, tlen = struct.unpack_from(e + "II", pg, o + 4)
            blob, left = b"", tlen
            while pgno and left > 0:
                ov = page(pgno)
                if ov[25] != _P_OVERFLOW:
                    raise RpmError("bdb overflow chain broken")
                used = struct.unpack_from(e + "H", ov, 22)[0]  # hf_offset: bytes on the page
                chunk = ov[26:26 + min(used, left)]
                blob += chunk
                left -= len(chunk)
                pgno = struct.unpack_from(e + "I", ov, 16)[0]  # next_pgno
            if left:
                raise RpmError("bdb overflow chain short")
            out.append(blob)
    return out


def _blobs_ndb(raw):
    version, generation, slot_npages = struct.unpack_from("<III", raw, 4)
    out = []
    slots_end = slot_npages * 4096
    for o in range(16, min(slots_end, len(raw)), 16):
        magic, pkg, blk_off, blk_cnt = struct.unpack_from("<IIII", raw, o)
        if magic != _NDB_SLOT_MAGIC or pkg == 0:
            continue
        b = blk_off * 16
        bmagic, bpkg, _gen, blen = struct.unpack_from("<IIII", raw, b)
        if bmagic != _NDB_BLOB_MAGIC or bpkg != pkg or b + 16 + blen > len(raw):
            raise RpmError("invalid ndb blob")
        out.append(raw[b + 16:b + 16 + blen])
    return out


def list_packages(path):
    """go-rpmdb rpmdb.Open + ListPackages: PackageInfo dicts of every header in the DB."""
    with open(path, "rb") as f:
        raw = f.read()
    fmt = detect_format(raw)
    blobs = _blobs_sqlite(path) if fmt == "sqlite" else _blobs_bdb(raw) if fmt == "bdb" else _blobs_ndb(raw)
    return [package_info(header_import(b)) for b in blobs]


def analyze(path, file_path="var/lib/rpm/Packages"):
    """rpmPkgAnalyzer.Analyze: ([{FilePath, Packages}], installed files)."""
    try:
        infos = list_packages(path)
    except (RpmError, sqlite3.Error, struct.error) as e:
        raise RpmError(f"failed to parse rpmdb: {e}")
    pkgs, files = list_pkgs(infos)
    return [{"FilePath": file_path, "Packages": pkgs}], files


def required(file_path):
    return file_path in ("usr/lib/sysimage/rpm/Packages", "var/lib/rpm/Packages", "usr/lib/sysimage/rpm/Packages.db",
                         "var/lib/rpm/Packages.db", "usr/lib/sysimage/rpm/rpmdb.sqlite", "var/lib/rpm/rpmdb.sqlite")


__all__ = ["split_file_name", "list_pkgs", "parse_rpmqa_manifest", "header_import", "header_export", "package_info",
           "list_packages", "analyze", "required", "RpmError"]
