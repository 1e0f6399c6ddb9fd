"""CPU: the read-only bbolt walker (trivy_amd/csrc/bbolt.cpp; tvm_bbolt_walk / tvm_db_put_bbolt)
- on the reference's own bolt files (copied as data into tests/golden/bbolt/): fanal.db /
  broken-image.db hold exactly what pkg/fanal/cache/fs_test.go expects of them
  (TestFSCache_GetBlob: the blob's JSON; TestFSCache_MissingBlobs: which artifact / blob keys
  exist), new.db holds the trivy/metadata/data record pkg/rpc/server/listen_test.go installs;
- on trivy-db-shaped files written from the repo's bolt fixtures (tools/bolt_write.py, with
  branch pages, inline buckets and overflow pages): the walk returns every record, and a DB
  loaded from the file equals the DB loaded record by record;
- malformed files fail with an error, never a hang or a read out of bounds."""
import glob
import json
import os
import struct

import pytest

from tools import bolt_write
from trivy_amd.db import DB, bbolt_records

HERE = os.path.dirname(os.path.abspath(__file__))
BOLT = os.path.join(HERE, "golden", "bbolt")


def _read(name):
    with open(os.path.join(BOLT, name), "rb") as f:
        return f.read()


def test_reference_fanal_cache_files():
    recs = dict(bbolt_records(_read("fanal.db")))
    image = b"sha256:58701fd185bda36cab0557bb6438661831267aa4a9e0b54211c4d5317a48aff4"
    layer = b"sha256:24df0d4e20c0f42d3703bf1f1db2bdd77346c7956f74f423603d651e8e5ae8a7"
    # TestFSCache_GetBlob happy path: the blob decodes to {SchemaVersion 2, OS alpine 3.10}
    blob = json.loads(recs[(b"blob", layer + b"/11101")])
    assert blob == {"SchemaVersion": 2, "OS": {"Family": "alpine", "Name": "3.10"}}
    # TestFSCache_MissingBlobs: the image /1 and layer 24df.../11101 exist, the others do not
    assert (b"artifact", image + b"/1") in recs and (b"artifact", image + b"/2") not in recs
    for missing in (b"sha256:dffd9992ca398466a663c87c92cfea2a2db0ae0cf33fcb99da60eec52addbfc5/11101",
                    b"sha256:dab15cac9ebd43beceeeda3ce95c574d6714ed3d3969071caead678c065813ec/11101",
                    layer + b"/11102"):
        assert (b"blob", missing) not in recs
    assert json.loads(recs[(b"artifact", image + b"/1")])["SchemaVersion"] == 1
    broken = dict(bbolt_records(_read("broken-image.db")))
    assert broken[(b"artifact", image)] == b"broken"  # "broken-image": the artifact JSON is invalid
    assert json.loads(broken[(b"blob", layer)])["SchemaVersion"] == 100


def test_reference_trivy_metadata_file():
    recs = bbolt_records(_read("new.db"))
    assert [p for p, _ in recs] == [(b"trivy", b"metadata", b"data")]  # nested bucket
    meta = json.loads(recs[0][1])
    assert meta["Version"] == 1 and meta["NextUpdate"].startswith("3000-01-01")


def _fixture_records():
    out = {}
    for f in sorted(glob.glob(os.path.join(HERE, "golden", "fixtures", "**", "*.json"), recursive=True)):
        for r in json.load(open(f, encoding="utf-8")):
            out[tuple(p.encode() for p in r["path"])] = r["value"].encode()
    return sorted(out.items())


@pytest.mark.parametrize("per_leaf,inline", [(64, True), (5, False), (3, True)])
def test_trivy_db_shaped_round_trip(per_leaf, inline):
    recs = _fixture_records()
    assert len(recs) > 200
    img = bolt_write.write(recs, per_leaf=per_leaf, inline=inline)
    got = bbolt_records(img)
    assert got == recs  # every record, in bucket / key order
    a, b = DB(), DB()
    a.put_bbolt(img)
    b.put_records({"path": [x.decode() for x in p], "value": v.decode()} for p, v in recs)
    assert a.finalize().stats() == b.finalize().stats()


def test_overflow_pages_and_large_values():
    recs = [((b"debian 12", b"pkg%03d" % i, b"CVE-2024-%04d" % i), b'{"FixedVersion":"1.%d"}' % i + b" " * (i * 97))
            for i in range(120)]
    img = bolt_write.write(recs, per_leaf=200)  # one leaf page far larger than 4 KiB
    assert bbolt_records(img) == sorted(recs)


def test_malformed_files_fail_cleanly():
    img = bolt_write.write(_fixture_records()[:50], per_leaf=4)
    with pytest.raises(ValueError, match="meta"):
        bbolt_records(b"not a bolt file" * 10)
    bad = bytearray(img)
    bad[16 + 20] ^= 1  # root pgid of meta 0 ...
    bad[4096 + 16 + 20] ^= 1  # ... and of meta 1: both checksums fail
    with pytest.raises(ValueError, match="meta"):
        bbolt_records(bytes(bad))
    with pytest.raises(ValueError):
        bbolt_records(img[: len(img) - 4096])  # a page cut off
    # a branch page whose child is itself: bounded by the nesting limit, not a hang
    loop = bytearray(img)
    root = struct.unpack_from("<Q", loop, 16 + 16)[0]
    struct.pack_into("<QHHI", loop, root * 4096, root, 0x01, 1, 0)
    struct.pack_into("<IIQ", loop, root * 4096 + 16, 16, 1, root)
    with pytest.raises(ValueError):
        bbolt_records(bytes(loop))


def test_page_referenced_twice_is_refused():
    """A crafted branch whose elements all name one child would be walked count^depth times
    (a denial of service on an untrusted trivy.db): every page may be reached once."""
    img = bytearray(bolt_write.write(_fixture_records()[:50], per_leaf=4))
    root = struct.unpack_from("<Q", img, 16 + 16)[0]
    leaf = next(p for p in range(3, len(img) // 4096)
                if p != root and struct.unpack_from("<H", img, p * 4096 + 8)[0] == 0x02)
    n = 200
    struct.pack_into("<QHHI", img, root * 4096, root, 0x01, n, 0)
    for i in range(n):  # zero-length keys, every element naming the same leaf page
        struct.pack_into("<IIQ", img, root * 4096 + 16 + 16 * i, 16 * (n - i), 0, leaf)
    with pytest.raises(ValueError, match="twice"):
        bbolt_records(bytes(img))
