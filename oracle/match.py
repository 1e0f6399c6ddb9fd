"""ORACLE - TEST INFRASTRUCTURE ONLY: ctypes front end of oracle/match.c (orc_match).

Feeds the raw synthetic strings (tools/synth.py) to the C restatement and returns the
(package, advisory) pairs; used by tests/ (parity) and bench.py (cpu_baseline leg).
"""
import ctypes
import os

import numpy as np

from .drivers import lib as _lib

ORC_DRV_DEBIAN, ORC_DRV_UBUNTU = 1, 2

_I32, _I64, _U64, _U32, _U8 = (ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64),
                               ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint8))


class OrcDB(ctypes.Structure):
    _fields_ = [("n_keys", ctypes.c_int32), ("key_plat", _I32), ("key_name_arena", ctypes.c_char_p),
                ("key_name_off", _U64), ("key_name_len", _U32), ("key_poisoned", _U8), ("key_adv_begin", _I64),
                ("adv_fixed_arena", ctypes.c_char_p), ("adv_fixed_off", _U64), ("adv_fixed_len", _U32),
                ("n_plat", ctypes.c_int32), ("plat_driver", _I32)]


class OrcBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("plat", _I32), ("name_arena", ctypes.c_char_p), ("name_off", _U64),
                ("name_len", _U32), ("ver_arena", ctypes.c_char_p), ("ver_off", _U64), ("ver_len", _U32)]


def _arena(items):
    lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
    off = np.zeros(len(items), dtype=np.uint64)
    if len(items):
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return b"".join(items), off, lens


def _p(a, t):
    return a.ctypes.data_as(t)


def driver_of(root):
    return ORC_DRV_DEBIAN if root.startswith("debian") else ORC_DRV_UBUNTU


class Prepared:
    """Oracle-side copies of a synthetic DB + batch (the product never sees these)."""

    def __init__(self, sdb, batch, poisoned=()):
        self.keep = []
        kn, koff, klen = _arena(sdb.key_names)
        fx, foff, flen = _arena(sdb.adv_fixed)
        self.key_plat = np.ascontiguousarray(sdb.key_plat, dtype=np.int32)
        self.poison = np.zeros(len(sdb.key_names), dtype=np.uint8)
        self.poison[list(poisoned)] = 1
        self.adv_begin = np.ascontiguousarray(sdb.adv_begin, dtype=np.int64)
        self.plat_drv = np.array([driver_of(p) for p in sdb.platforms], dtype=np.int32)
        self.keep += [kn, koff, klen, fx, foff, flen]
        self.db = OrcDB(len(sdb.key_names), _p(self.key_plat, _I32), kn, _p(koff, _U64), _p(klen, _U32),
                        _p(self.poison, _U8), _p(self.adv_begin, _I64), fx, _p(foff, _U64), _p(flen, _U32),
                        len(sdb.platforms), _p(self.plat_drv, _I32))
        nm, noff, nlen = _arena(batch.names)
        vr, voff, vlen = _arena(batch.versions)
        self.plat = np.ascontiguousarray(batch.plat, dtype=np.int32)
        self.keep += [nm, noff, nlen, vr, voff, vlen]
        self.batch = OrcBatch(len(batch.names), _p(self.plat, _I32), nm, _p(noff, _U64), _p(nlen, _U32),
                              vr, _p(voff, _U64), _p(vlen, _U32))


def match(prep, n_threads=1, cap=None):
    """Returns (pkg array, adv array) or raises with the first poisoned package index.  The
    output buffers live in prep and are reused (fresh arrays per call cost page faults that
    serialise the threads); the returned arrays are views into them."""
    L = _lib()
    L.orc_match.restype = ctypes.c_int64
    L.orc_match.argtypes = [ctypes.POINTER(OrcDB), ctypes.POINTER(OrcBatch), ctypes.c_int, _I64, _I64,
                            ctypes.c_int64]
    out = getattr(prep, "_out", None)
    if out is None or (cap and len(out[0]) < cap):
        c = cap or max(16, prep.batch.n * 8)
        out = prep._out = (np.zeros(c, dtype=np.int64), np.zeros(c, dtype=np.int64))
    while True:
        pk, ad = out
        n = L.orc_match(ctypes.byref(prep.db), ctypes.byref(prep.batch), n_threads, _p(pk, _I64), _p(ad, _I64), len(pk))
        if n < 0:
            raise PoisonedKey(-1 - n)
        if n <= len(pk):
            return pk[:n].copy(), ad[:n].copy()
        out = prep._out = (np.zeros(int(n), dtype=np.int64), np.zeros(int(n), dtype=np.int64))


class PoisonedKey(Exception):
    def __init__(self, pkg):
        super().__init__(f"package {pkg} hits an undecodable advisory")
        self.pkg = pkg
