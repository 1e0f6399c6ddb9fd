#!/usr/bin/env python3
"""Test infrastructure: writes a bbolt file image from (bucket path..., key) -> value records,
so the read-only walker (trivy_amd/csrc/bbolt.cpp) can be checked on trivy-db-shaped files
(the reference only ships small bolt files: pkg/fanal/cache/testdata/*.db,
pkg/rpc/server/testdata/new.db).  Restates the published on-disk format: two meta pages
(FNV-1a 64 checksums), a freelist page, then every bucket's pages - leaf pages (a bucket
larger than `per_leaf` records is split under a branch page), nested buckets as 16-byte
headers {root pgid, sequence}, small record-only buckets inline (root 0, their leaf page
inside the value) when `inline` is set, overflow pages for pages larger than the page size."""
import struct

PSZ = 4096
MAGIC = 0xED0CDAED
BRANCH, LEAF, META, FREELIST = 0x01, 0x02, 0x04, 0x10
BUCKET_LEAF = 0x01


def fnv1a64(b):
    h = 0xCBF29CE484222325
    for x in b:
        h = ((h ^ x) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def tree(records):
    """records: iterable of (path tuple of bytes, value bytes) -> nested dicts."""
    root = {}
    for path, value in records:
        d = root
        for b in path[:-1]:
            d = d.setdefault(b, {})
        d[path[-1]] = value
    return root


class Writer:
    def __init__(self, per_leaf=64, inline=True):
        self.pages = {}  # pgid -> bytes (whole page run, padded)
        self.next = 3    # 0, 1 meta; 2 freelist
        self.per_leaf = per_leaf
        self.inline = inline

    def _page_bytes(self, pgid, flags, elems):
        """elems: [(16-byte element sans pos patched, key, value)] -> page image (no padding)."""
        count = len(elems)
        hdr_end = 16 + 16 * count
        body = bytearray()
        table = bytearray()
        for i, (kind, a, k, v) in enumerate(elems):
            pos = hdr_end + len(body) - (16 + 16 * i)  # relative to the element itself
            if flags & LEAF:
                table += struct.pack("<IIII", a, pos, len(k), len(v))
            else:
                table += struct.pack("<IIQ", pos, len(k), a)
            body += k + v
        return bytearray(struct.pack("<QHHI", pgid, flags, count, 0)) + table + body

    def _alloc(self, img):
        n = (len(img) + PSZ - 1) // PSZ
        pgid = self.next
        self.next += n
        struct.pack_into("<Q", img, 0, pgid)
        struct.pack_into("<I", img, 12, n - 1)
        self.pages[pgid] = bytes(img) + b"\0" * (n * PSZ - len(img))
        return pgid

    def bucket(self, d):
        """Writes bucket d; returns its 16-byte header value (root pgid or inline page)."""
        items = sorted(d.items())
        elems = []
        for k, v in items:
            if isinstance(v, dict):
                elems.append((0, BUCKET_LEAF, k, self.bucket(v)))
            else:
                elems.append((0, 0, k, v))
        if (self.inline and items and all(not isinstance(v, dict) for _, v in items)
                and len(items) <= 4 and sum(len(k) + len(v) for k, v in items) < PSZ // 8):
            return struct.pack("<QQ", 0, 0) + bytes(self._page_bytes(0, LEAF, [(0, f, k, v) for _, f, k, v in elems]))
        leaves = [elems[i:i + self.per_leaf] for i in range(0, len(elems), self.per_leaf)] or [[]]
        ids = [self._alloc(self._page_bytes(0, LEAF, [(0, f, k, v) for _, f, k, v in part])) for part in leaves]
        if len(ids) == 1:
            return struct.pack("<QQ", ids[0], 0)
        branch = [(0, pid, part[0][2], b"") for pid, part in zip(ids, leaves)]
        return struct.pack("<QQ", self._alloc(self._page_bytes(0, BRANCH, branch)), 0)

    def image(self, records):
        root_hdr = self.bucket(tree(records))
        root = struct.unpack_from("<Q", root_hdr)[0]
        if root == 0:  # the root bucket is never inline: give it a page of its own
            self.inline, self.next = False, 3
            self.pages = {}
            root = struct.unpack_from("<Q", self.bucket(tree(records)))[0]
        out = bytearray(self.next * PSZ)
        for txid, m in ((0, 0), (1, 1)):
            meta = struct.pack("<IIIIQQQQQ", MAGIC, 2, PSZ, 0, root, 0, 2, self.next, txid)
            meta += struct.pack("<Q", fnv1a64(meta))
            out[m * PSZ:m * PSZ + 16] = struct.pack("<QHHI", m, META, 0, 0)
            out[m * PSZ + 16:m * PSZ + 16 + len(meta)] = meta
        out[2 * PSZ:2 * PSZ + 16] = struct.pack("<QHHI", 2, FREELIST, 0, 0)
        for pgid, img in self.pages.items():
            out[pgid * PSZ:pgid * PSZ + len(img)] = img
        return bytes(out)


def write(records, per_leaf=64, inline=True):
    return Writer(per_leaf, inline).image(records)
