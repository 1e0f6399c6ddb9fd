"""The drop-in path under concurrency (include/trivy_amd.h tvm_engine_swap /
tvm_engine_dropin_stats; engine.hip "drop-in path").

The reference serves concurrent Detect calls (pkg/rpc/server/server.go:45, the k8s
scanner's worker pool pkg/k8s/scanner/scanner.go:141) and hot-swaps its DB
(pkg/rpc/server/listen.go:154-190).  Here: threads call tvm_ospkg_driver_detect through
ctypes (the GIL is released during the call) on many targets at once while another thread
swaps the engine between two DBs.  Every result must equal the serial result of the same
call on one of the two DBs - never a mix - and concurrent calls must share launches."""
import ctypes
import random
import threading

import numpy as np
import pytest

import trivy_amd
from trivy_amd import _lib as L
from trivy_amd._lib import lib
from trivy_amd.detector import ospkg as osp
from tools.synth import make_db, make_batch

pytestmark = pytest.mark.gpu

PLATS = ["debian 12", "ubuntu 22.04"]


def _db(seed):
    sdb = make_db(PLATS, 1500, seed=seed)
    db = trivy_amd.DB()
    for n, depth, arena, off, lens in (sdb.records_arena(), sdb.source_arena()):
        db.put_arena(n, depth, arena, off, lens)
    return sdb, db.finalize()


def _targets(sdb, n_targets=48):
    batch = make_batch(sdb, n_targets, 120, [1, 1], seed=11)
    out = []
    for p, b0, b1 in batch.targets:
        fam, ver = ("debian", "12") if PLATS[p].startswith("debian") else ("ubuntu", "22.04")
        pk = [{"Name": batch.names[i].decode(), "SrcName": batch.names[i].decode(),
               "Version": batch.versions[i].decode(), "SrcVersion": batch.versions[i].decode()}
              for i in range(b0, b1)]
        arr, keep = osp._pkg_array(pk)
        out.append((fam, ver, pk, arr, keep))
    return out


def _call(eng, t):
    fam, ver, pk, arr, _keep = t
    res, ebuf = L.Result(), L.errbuf()
    rc = lib().tvm_ospkg_driver_detect(eng.h, fam.encode(), ver.encode(), None, arr, len(pk), 1700000000,
                                       ctypes.byref(res), ebuf, len(ebuf))
    if rc:
        raise RuntimeError(ebuf.value.decode())
    try:
        got = sorted((v["VulnerabilityID"], v.get("PkgName", ""), v.get("InstalledVersion", ""),
                      v.get("FixedVersion", "")) for v in osp._convert(res, pk))
    finally:
        lib().tvm_result_free(ctypes.byref(res))
    return got


def _stats(eng):
    out = (ctypes.c_uint64 * 3)()
    assert lib().tvm_engine_dropin_stats(eng.h, out) == 0
    return tuple(out)


def test_concurrent_calls_coalesce_and_match_serial():
    sdb, db = _db(7)
    eng = trivy_amd.Engine(db, 0)
    ts = _targets(sdb)
    serial = [_call(eng, t) for t in ts]
    assert sum(len(x) for x in serial) > 100
    l0, c0, _ = _stats(eng)
    errors, results = [], {}

    def worker(w):
        rnd = random.Random(w)
        try:
            for _ in range(60):
                k = rnd.randrange(len(ts))
                results.setdefault(k, []).append(_call(eng, ts[k]))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for k, rs in results.items():
        for r in rs:
            assert r == serial[k], k
    launches, calls, merged = (a - b for a, b in zip(_stats(eng), (l0, c0, 0)))
    assert calls == 8 * 60
    assert launches < calls and merged > 0, (launches, calls, merged)


def test_swap_under_load_never_mixes():
    sdb1, db1 = _db(7)
    sdb2, db2 = _db(8)
    eng = trivy_amd.Engine(db1, 0)
    ts = _targets(sdb1)
    want1 = [_call(eng, t) for t in ts]
    eng.swap(db2)
    want2 = [_call(eng, t) for t in ts]
    assert want1 != want2
    eng.swap(db1)
    stop, errors, seen = threading.Event(), [], [0, 0]

    def worker(w):
        rnd = random.Random(100 + w)
        try:
            while not stop.is_set():
                k = rnd.randrange(len(ts))
                r = _call(eng, ts[k])
                if r == want1[k]:
                    seen[0] += 1
                elif r == want2[k]:
                    seen[1] += 1
                else:
                    raise AssertionError(f"target {k}: result of neither DB")
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(w,)) for w in range(6)]
    for t in th:
        t.start()
    for i in range(8):
        eng.swap(db2 if i % 2 == 0 else db1)
    stop.set()
    for t in th:
        t.join()
    assert not errors, errors
    assert seen[0] + seen[1] > 0
