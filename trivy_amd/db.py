"""Advisory DB intake and device engine (wrappers of tvm_db_* / tvm_engine_*).

Replaces trivy-db's db.Init (reference pkg/commands/artifact/run.go:311): the
bucket tree is handed over record by record - (bucket path..., key) -> JSON
value, what a bbolt walk or bolt-fixtures (pkg/dbtest/db.go:17-36) produces -
then flattened once and uploaded to HBM.
"""
import ctypes
import json

from . import _lib
from ._lib import lib, s, errbuf, Str


class DB:
    def __init__(self):
        self.h = lib().tvm_db_new()
        self._finalized = False

    def put(self, path, value):
        arr = (Str * len(path))(*[s(p) for p in path])
        v = value.encode() if isinstance(value, str) else value
        rc = lib().tvm_db_put(self.h, arr, len(path), v, len(v))
        if rc:
            raise ValueError(f"tvm_db_put failed ({rc})")

    def put_records(self, records):
        """records: iterable of {"path": [...], "value": "<json>"} (tests/golden/fixtures format)."""
        by_depth = {}
        for r in records:
            by_depth.setdefault(len(r["path"]), []).append(r)
        for depth, recs in by_depth.items():
            keep = []
            paths = (Str * (len(recs) * depth))()
            vals = (Str * len(recs))()
            for i, r in enumerate(recs):
                for j, p in enumerate(r["path"]):
                    b = p.encode()
                    keep.append(b)
                    paths[i * depth + j] = Str(b, len(b))
                v = r["value"].encode()
                keep.append(v)
                vals[i] = Str(v, len(v))
            rc = lib().tvm_db_put_many(self.h, len(recs), ctypes.cast(paths, ctypes.c_void_p), depth,
                                       ctypes.cast(vals, ctypes.c_void_p))
            if rc:
                raise ValueError(f"tvm_db_put_many failed ({rc})")

    def put_bbolt(self, data):
        """Every record of a bbolt file image (trivy.db) - tvm_db_put_bbolt."""
        e = errbuf()
        rc = lib().tvm_db_put_bbolt(self.h, data, len(data), e, len(e))
        if rc:
            raise ValueError(e.value.decode())

    def put_arena(self, n, depth, arena, off, lens):
        """n records of `depth` path components + value, packed in one arena (record r's
        strings are items r*(depth+1) .. r*(depth+1)+depth; off u64 / lens u32 per item)."""
        rc = lib().tvm_db_put_arena(self.h, n, depth, arena, off.ctypes.data, lens.ctypes.data)
        if rc:
            raise ValueError(f"tvm_db_put_arena failed ({rc})")

    def finalize(self):
        e = errbuf()
        rc = lib().tvm_db_finalize(self.h, e, len(e))
        if rc:
            raise ValueError(e.value.decode())
        self._finalized = True
        return self

    def stats(self):
        out = (ctypes.c_uint64 * 5)()
        lib().tvm_db_stats(self.h, out)
        return dict(zip(["platforms", "keys", "advisories", "rows", "key_bytes"], list(out)))

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h and _lib._lib is not None:
            _lib._lib.tvm_db_free(h)


class _RawStr(ctypes.Structure):  # tvm_str with the pointer kept raw (keys may hold any byte)
    _fields_ = [("p", ctypes.c_void_p), ("n", ctypes.c_size_t)]


BBOLT_VISIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(_RawStr), ctypes.c_size_t,
                               ctypes.c_void_p, ctypes.c_size_t)


def bbolt_records(data):
    """[(path tuple of bytes (buckets..., key), value bytes)] of a bbolt file image, in the
    walk's (bucket, key) order (tvm_bbolt_walk)."""
    out = []

    def visit(_ctx, path, depth, value, vlen):
        out.append((tuple(ctypes.string_at(path[i].p, path[i].n) for i in range(depth)),
                    ctypes.string_at(value, vlen) if vlen else b""))
        return 0
    cb = BBOLT_VISIT(visit)
    e = errbuf()
    rc = lib().tvm_bbolt_walk(data, len(data), ctypes.cast(cb, ctypes.c_void_p), None, e, len(e))
    if rc:
        raise ValueError(e.value.decode())
    return out


def load_fixture_files(paths):
    """Build + finalize a DB from tests/golden/fixtures JSON files (dbtest.InitDB analogue)."""
    db = DB()
    for p in paths:
        with open(p, encoding="utf-8") as f:
            db.put_records(json.load(f))
    return db.finalize()


class Engine:
    """Device-resident tables on one HIP device (fails loudly without a GPU)."""

    def __init__(self, db, device=0):
        if not db._finalized:
            db.finalize()
        e = errbuf()
        self.db = db  # the engine references the DB's host tables
        self.h = lib().tvm_engine_open(db.h, device, e, len(e))
        if not self.h:
            raise RuntimeError(f"tvm_engine_open: {e.value.decode()}")

    def swap(self, db):
        if not db._finalized:
            db.finalize()
        e = errbuf()
        rc = lib().tvm_engine_swap(self.h, db.h, e, len(e))
        if rc:
            raise RuntimeError(e.value.decode())
        self.db = db

    def verify(self):
        """Raises when a device table no longer equals its host image."""
        e = errbuf()
        if lib().tvm_engine_verify(self.h, e, len(e)):
            raise RuntimeError(e.value.decode())

    def table_bytes(self):
        return lib().tvm_engine_table_bytes(self.h)

    def close(self):
        h, self.h = getattr(self, "h", None), None
        if h and _lib._lib is not None:
            _lib._lib.tvm_engine_close(h)

    def __del__(self):
        self.close()
