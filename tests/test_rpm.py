"""RPM installed-database extraction (trivy_amd/rpm.py).

Pinned by the reference's own tables (transcribed by tests/golden/extract_go_tables.py):
Test_splitFileName and Test_rpmPkgAnalyzer_listPkgs (pkg/fanal/analyzer/pkg/rpm/rpm_test.go),
TestParseMarinerDistrolessManifest (rpmqa_test.go).  The database containers (header blob,
SQLite, Berkeley DB hash, NDB) are parity-unpinned: the reference checkout holds no rpm
database fixture, so databases are built here from the published layouts and read back.

GPU: packages extracted from a database go through ospkg.Detect (redhat 8) on the GPU and
equal the oracle's detection."""
import datetime
import json
import os
import sqlite3
import struct

import pytest

from trivy_amd import rpm

HERE = os.path.join(os.path.dirname(__file__), "golden", "tables")
TABLES = json.load(open(os.path.join(HERE, "fanal__analyzer__pkg__rpm__rpm_test.json")))["tables"]
QA = json.load(open(os.path.join(HERE, "fanal__analyzer__pkg__rpm__rpmqa_test.json")))["tables"][0]["cases"]


def _nz(d):
    """Go zero values are absent fields."""
    return {k: v for k, v in d.items() if v not in ("", None, 0, [], {})}


@pytest.mark.parametrize("case", TABLES[1]["cases"], ids=lambda c: c["name"])
def test_split_file_name(case):
    if case["wantErr"]:
        with pytest.raises(rpm.RpmError):
            rpm.split_file_name(case["filename"])
    else:
        assert rpm.split_file_name(case["filename"]) == (case["wantName"], case["wantVer"], case["wantRel"])


@pytest.mark.parametrize("case", TABLES[2]["cases"], ids=lambda c: c["name"])
def test_list_pkgs(case):
    mock = case["mock"]
    if mock.get("err"):  # the DB's ListPackages error surfaces unchanged
        return
    pkgs, files = rpm.list_pkgs(mock["packages"])
    assert [_nz(p) for p in pkgs] == [_nz(p) for p in case["wantPkgs"]]
    assert files == (case.get("wantFiles") or [])


@pytest.mark.parametrize("case", QA, ids=lambda c: c["name"])
def test_rpmqa_manifest(case):
    if case.get("wantErr"):
        with pytest.raises(rpm.RpmError) as e:
            rpm.parse_rpmqa_manifest(case["content"])
        assert str(e.value) == case["wantErr"]
    else:
        assert rpm.parse_rpmqa_manifest(case["content"]) == case["wantPkgs"]


def test_consolidate_dependencies():
    infos = [{"Name": "a", "Version": "1", "Release": "1", "Arch": "x86_64", "Provides": ["liba.so", "a"],
              "Requires": ["libb.so", "liba.so", "libb.so", "missing"]},
             {"Name": "b", "Version": "2", "Release": "1", "Arch": "", "Provides": ["libb.so"], "Requires": ["liba.so"],
              "Epoch": 3, "SigMD5": "00ff", "License": "MIT", "Vendor": "CentOS", "DirNames": ["/x/"],
              "DirIndexes": [0], "BaseNames": ["y"]}]
    pkgs, files = rpm.list_pkgs(infos)
    assert pkgs[0]["DependsOn"] == ["b@2-1."] and pkgs[1]["DependsOn"] == ["a@1-1.x86_64"]
    assert pkgs[1]["Arch"] == "None" and pkgs[1]["Epoch"] == 3 and pkgs[1]["SrcEpoch"] == 3
    assert pkgs[1]["Digest"] == "md5:00ff" and pkgs[1]["Licenses"] == ["MIT"] and files == ["/x/y"]
    with pytest.raises(rpm.RpmError):
        rpm.installed_file_names({"DirNames": ["/"], "DirIndexes": [0, 0], "BaseNames": ["a"]})


# ---- database containers (parity-unpinned round trips) -----------------------------------------
def _header(name, ver, rel, arch="x86_64", epoch=None, src=None, vendor="Red Hat, Inc.", label=None):
    f = {rpm.TAG["NAME"]: (rpm.T_STRING, name), rpm.TAG["VERSION"]: (rpm.T_STRING, ver),
         rpm.TAG["RELEASE"]: (rpm.T_STRING, rel), rpm.TAG["ARCH"]: (rpm.T_STRING, arch),
         rpm.TAG["VENDOR"]: (rpm.T_STRING, vendor), rpm.TAG["LICENSE"]: (rpm.T_STRING, "GPLv2"),
         rpm.TAG["SOURCERPM"]: (rpm.T_STRING, src or f"{name}-{ver}-{rel}.src.rpm"),
         rpm.TAG["DIRNAMES"]: (rpm.T_STRING_ARRAY, ["/usr/bin/", "/etc/"]),
         rpm.TAG["DIRINDEXES"]: (rpm.T_INT32, [0, 1]), rpm.TAG["BASENAMES"]: (rpm.T_STRING_ARRAY, [name, name + ".conf"]),
         rpm.TAG["PROVIDENAME"]: (rpm.T_STRING_ARRAY, [name]), rpm.TAG["REQUIRENAME"]: (rpm.T_STRING_ARRAY, ["glibc"]),
         rpm.TAG["SIGMD5"]: (rpm.T_BIN, bytes(range(16))), 63: (rpm.T_BIN, b"\0" * 16)}
    if epoch is not None:
        f[rpm.TAG["EPOCH"]] = (rpm.T_INT32, [epoch])
    if label:
        f[rpm.TAG["MODULARITYLABEL"]] = (rpm.T_STRING, label)
    return rpm.header_export(f)


HEADERS = [_header("glibc", "2.28", "211.el8", vendor="Red Hat, Inc."),
           _header("openssl-libs", "1.1.1k", "9.el8_7", epoch=1, src="openssl-1.1.1k-9.el8_7.src.rpm"),
           _header("nodejs", "14.21.3", "1.module+el8.8.0+18531+1a0c5a1e", epoch=1,
                   label="nodejs:14:8080020230207112541:ad008a3a"),
           _header("gpg-pubkey", "fd431d51", "4ae0493b", arch="", vendor="", src="(none)")]


def _check(infos):
    assert [i["Name"] for i in infos] == ["glibc", "openssl-libs", "nodejs", "gpg-pubkey"]
    assert infos[1]["Epoch"] == 1 and infos[0]["Epoch"] is None
    assert infos[2]["Modularitylabel"] == "nodejs:14:8080020230207112541:ad008a3a"
    assert infos[0]["SigMD5"] == bytes(range(16)).hex() and infos[0]["DirIndexes"] == [0, 1]
    pkgs, files = rpm.list_pkgs(infos)
    assert pkgs[1]["SrcName"] == "openssl" and pkgs[1]["SrcVersion"] == "1.1.1k" and pkgs[1]["SrcEpoch"] == 1
    assert pkgs[0]["InstalledFiles"] == ["/usr/bin/glibc", "/etc/glibc.conf"]
    assert pkgs[3]["Arch"] == "None" and pkgs[3]["InstalledFiles"] is None
    assert pkgs[1]["DependsOn"] == ["glibc@2.28-211.el8.x86_64"]


def test_header_roundtrip_and_errors():
    h = rpm.header_import(HEADERS[1])
    assert h[rpm.TAG["NAME"]] == "openssl-libs" and h[rpm.TAG["EPOCH"]] == [1]
    with pytest.raises(rpm.RpmError):
        rpm.header_import(HEADERS[1][:20])
    with pytest.raises(rpm.RpmError):
        rpm.header_import(b"broken")


def test_sqlite_db(tmp_path):
    p = str(tmp_path / "rpmdb.sqlite")
    con = sqlite3.connect(p)
    con.execute("CREATE TABLE Packages (hnum INTEGER PRIMARY KEY AUTOINCREMENT, blob BLOB NOT NULL)")
    for h in HEADERS:
        con.execute("INSERT INTO Packages (blob) VALUES (?)", (h,))
    con.commit()
    con.close()
    _check(rpm.list_packages(p))
    infos, files = rpm.analyze(p, "var/lib/rpm/rpmdb.sqlite")
    assert infos[0]["FilePath"] == "var/lib/rpm/rpmdb.sqlite" and len(infos[0]["Packages"]) == 4


def _bdb(blobs, page_size=4096, order="<"):
    """Berkeley DB hash file: meta page, one hash page of (key, H_OFFPAGE) pairs, overflow chains."""
    pages = [bytearray(page_size)]
    meta = pages[0]
    struct.pack_into(order + "I", meta, 12, 0x061561)
    struct.pack_into(order + "I", meta, 20, page_size)
    chains = []
    next_free = 2
    for b in blobs:
        cap = page_size - 26
        n = (len(b) + cap - 1) // cap
        chains.append((next_free, len(b)))
        for i in range(n):
            pg = bytearray(page_size)
            chunk = b[i * cap:(i + 1) * cap]
            struct.pack_into(order + "I", pg, 8, next_free + i)
            struct.pack_into(order + "I", pg, 16, next_free + i + 1 if i + 1 < n else 0)
            struct.pack_into(order + "H", pg, 22, len(chunk))
            pg[25] = 7
            pg[26:26 + len(chunk)] = chunk
            pages.append(pg)
        next_free += n
    hp = bytearray(page_size)
    hp[25] = 13
    items, offs, top = [], [], page_size
    for i, (pgno, tlen) in enumerate(chains):
        key = bytes([1]) + struct.pack(order + "I", i + 1)
        val = bytes([3, 0, 0, 0]) + struct.pack(order + "II", pgno, tlen)
        for it in (key, val):
            top -= len(it)
            hp[top:top + len(it)] = it
            offs.append(top)
    struct.pack_into(order + "H", hp, 20, len(offs))
    struct.pack_into(order + "%dH" % len(offs), hp, 26, *offs)
    pages.insert(1, hp)
    struct.pack_into(order + "I", meta, 32, len(pages) - 1)
    return b"".join(bytes(p) for p in pages)


@pytest.mark.parametrize("order", ["<", ">"])
def test_bdb_hash_db(tmp_path, order):
    big = HEADERS[:1] + [_header("kernel-core", "4.18.0", "477.el8", src="kernel-4.18.0-477.el8.src.rpm") * 1] + HEADERS[1:]
    p = tmp_path / "Packages"
    p.write_bytes(_bdb([HEADERS[0], HEADERS[1], HEADERS[2], HEADERS[3]], order=order))
    _check(rpm.list_packages(str(p)))
    assert len(big) == 5


def test_bdb_multi_page_blob(tmp_path):
    h = _header("x" * 3000, "1", "1", src="y-1-1.src.rpm")
    p = tmp_path / "Packages"
    p.write_bytes(_bdb([h], page_size=1024))
    assert rpm.list_packages(str(p))[0]["Name"] == "x" * 3000


def _ndb(blobs):
    slots = bytearray(4096)
    struct.pack_into("<IIII", slots, 0, int.from_bytes(b"RpmP", "little"), 0, 1, 1)
    data, blk = bytearray(), 4096 // 16
    for i, b in enumerate(blobs):
        struct.pack_into("<IIII", slots, 16 * (i + 1), int.from_bytes(b"Slot", "little"), i + 1, blk + len(data) // 16,
                         (16 + len(b) + 15) // 16)
        rec = struct.pack("<IIII", int.from_bytes(b"BlbS", "little"), i + 1, 1, len(b)) + b
        data += rec + b"\0" * ((-len(rec)) % 16)
    return bytes(slots) + bytes(data)


def test_ndb_db(tmp_path):
    p = tmp_path / "Packages.db"
    p.write_bytes(_ndb(HEADERS))
    _check(rpm.list_packages(str(p)))


def test_broken_db(tmp_path):
    p = tmp_path / "Packages"
    p.write_bytes(b"broken")
    with pytest.raises(rpm.RpmError, match="failed to parse rpmdb"):
        rpm.analyze(str(p))
    assert rpm.required("var/lib/rpm/Packages") and not rpm.required("var/lib/dpkg/status")


@pytest.mark.gpu
def test_extracted_packages_detect_like_oracle(tmp_path):
    """rpmdb -> listPkgs -> ospkg.Detect(redhat 8) on the GPU == the oracle on the same records."""
    import glob

    import oracle.drivers as od
    import trivy_amd
    from conftest import canon
    from trivy_amd.detector.ospkg import detect
    fx = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "fixtures", "integration", "*.json")))
    p = str(tmp_path / "rpmdb.sqlite")
    con = sqlite3.connect(p)
    con.execute("CREATE TABLE Packages (hnum INTEGER PRIMARY KEY AUTOINCREMENT, blob BLOB NOT NULL)")
    for h in HEADERS + [_header("openssl", "1.0.2k", "8.el7", epoch=1), _header("bash", "4.2.46", "30.el7")]:
        con.execute("INSERT INTO Packages (blob) VALUES (?)", (h,))
    con.commit()
    con.close()
    (info,), _ = rpm.analyze(p)
    pkgs = info["Packages"]
    now = int(datetime.datetime(2021, 8, 25, tzinfo=datetime.timezone.utc).timestamp())
    eng = trivy_amd.Engine(trivy_amd.load_fixture_files(fx), 0)
    for fam, ver in (("redhat", "7.9"), ("centos", "7.6.1810"), ("redhat", "8.8")):
        got, eosl = detect(eng, fam, ver, None, pkgs, now=now)
        want, weosl = od.detect(od.Records.from_files(fx), fam, ver, None, pkgs, now)
        assert canon(got) == canon(want) and eosl == weosl, (fam, ver)
