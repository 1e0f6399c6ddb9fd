"""GPU: bit-exact (package, advisory) match sets against the oracle on seeded synthetic
workloads, through the C-ABI batch interface (the same path bench.py times)."""
import ctypes

import numpy as np
import pytest

from tools.synth import make_db, make_batch
from oracle import match as om

pytestmark = pytest.mark.gpu


def build_engine(sdb, poison=()):
    import trivy_amd
    from trivy_amd._lib import lib
    db = trivy_amd.DB()
    for n, depth, arena, off, lens in (sdb.records_arena(poison), sdb.source_arena()):
        rc = lib().tvm_db_put_arena(db.h, n, depth, arena, off.ctypes.data, lens.ctypes.data)
        assert rc == 0
    db.finalize()
    return trivy_amd.Engine(db, 0)


def run_batch(eng, sdb, batch, cap=None):
    """Runs one match pass; with cap=None the match buffer is re-sized to the exact total."""
    if cap is None:
        r = _run_batch(eng, sdb, batch, max(1024, 8 * len(batch)))
        if r[0] is not None:
            return r
        cap = r[3]
    return _run_batch(eng, sdb, batch, cap, strict=True)


def _run_batch(eng, sdb, batch, cap, strict=False):
    from trivy_amd._lib import lib, errbuf
    L = lib()
    b = L.tvm_batch_new()
    try:
        arena, noff, nlen, voff, vlen = batch.arena()
        for p, b0, b1 in batch.targets:
            first = L.tvm_batch_add_many(b, eng.h, sdb.platforms[p].encode(), b1 - b0, arena,
                                         noff[b0:].ctypes.data, nlen[b0:].ctypes.data,
                                         voff[b0:].ctypes.data, vlen[b0:].ctypes.data)
            assert first == b0
        e = errbuf()
        assert L.tvm_batch_upload(eng.h, b, cap, e, len(e)) == 0, e.value
        assert L.tvm_match_launch(eng.h, b, e, len(e)) == 0, e.value
        assert L.tvm_engine_sync(eng.h, e, len(e)) == 0, e.value
        n, errp, bits = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_uint64()
        assert L.tvm_match_status(eng.h, b, ctypes.byref(n), ctypes.byref(errp), ctypes.byref(bits)) == 0
        assert bits.value == 0
        out = np.zeros(2 * max(n.value, 1), dtype=np.uint32)
        got = ctypes.c_uint64()
        rc = L.tvm_match_fetch(eng.h, b, out.ctypes.data, n.value, ctypes.byref(got))
        if n.value > cap:
            assert rc != 0 and got.value == 0  # overflow is reported, never silently truncated
            return None, None, errp.value, n.value
        assert rc == 0
        pairs = out[:2 * got.value].reshape(-1, 2)
        return pairs[:, 0].astype(np.int64), pairs[:, 1].astype(np.int64), errp.value, n.value
    finally:
        L.tvm_batch_free(b)


PLATS = ["debian 11", "debian 12", "ubuntu 22.04", "ubuntu 24.04"]


@pytest.fixture(scope="module")
def world():
    sdb = make_db(PLATS, 4000, seed=11)
    return sdb, build_engine(sdb)


@pytest.mark.parametrize("seed,targets,per,long_frac", [(1, 200, 400, 0.0), (2, 50, 1000, 0.05), (3, 1, 7, 0.0)])
def test_parity_vs_oracle(world, oracle_built, seed, targets, per, long_frac):
    sdb, eng = world
    batch = make_batch(sdb, targets, per, [3, 3, 2, 2], seed=seed, long_versions=long_frac, invalid=0.01)
    pk, ad, errp, total = run_batch(eng, sdb, batch)
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=8)
    assert errp == -1
    assert total == len(opk)
    # engine output is in (package, advisory) order, as is the oracle's
    assert np.array_equal(pk, opk) and np.array_equal(ad, oad)


def test_output_buffer_too_small_reports_total(world):
    sdb, eng = world
    batch = make_batch(sdb, 20, 200, [1, 1, 1, 1], seed=5)
    pk, ad, errp, total = run_batch(eng, sdb, batch, cap=10)
    assert total > 10 and pk is None


def test_heavy_key_overflows_lds_buffer(oracle_built):
    """One key with 5000 advisories requested by every package: tiles exceed the LDS match buffer."""
    sdb = make_db(["debian 12"], 50, seed=3, unfixed=0.9)
    k = sdb.key_names.index(b"linux")
    from tools.synth import SynthBatch
    n = 700
    batch = SynthBatch(np.zeros(n, dtype=np.int32), [b"linux"] * n, [b"1.0-1"] * n, [(0, 0, n)])
    eng = build_engine(sdb)
    pk, ad, errp, total = run_batch(eng, sdb, batch, cap=n * 5000)
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=8)
    assert total == len(opk) and np.array_equal(pk, opk) and np.array_equal(ad, oad)
    assert total > 2048 * 2


def test_poisoned_key_first_package(oracle_built):
    sdb = make_db(["debian 12", "ubuntu 22.04"], 300, seed=4)
    poison = [int(sdb.plat_keys[0][5]), int(sdb.plat_keys[1][7])]
    eng = build_engine(sdb, poison)
    batch = make_batch(sdb, 30, 300, [1, 1], seed=9, miss=0.0)
    _, _, errp, _ = run_batch(eng, sdb, batch)
    with pytest.raises(om.PoisonedKey) as ei:
        om.match(om.Prepared(sdb, batch, poisoned=poison), n_threads=1)
    assert errp == ei.value.pkg


def test_empty_batch(world):
    sdb, eng = world
    from tools.synth import SynthBatch
    pk, ad, errp, total = run_batch(eng, sdb, SynthBatch(np.zeros(0, dtype=np.int32), [], [], []))
    assert total == 0 and errp == -1


def variants(grammar_set=1):
    """Indices of the non-ablation match-kernel variants (engine.hip kVariants) built for the
    grammar set (bit 0 dpkg-only, 1 OS grammars, 2 any, 3 GM_LEAN: library grammars without Maven / RubyGems)."""
    from trivy_amd._lib import lib
    out, v = [], 0
    while lib().tvm_variant_name(v):
        if not lib().tvm_variant_name(v).decode().startswith(("ablate", "diag")) and \
                lib().tvm_variant_grammar_sets(v) & grammar_set:
            out.append(v)
        v += 1
    return out


def test_every_variant_matches_oracle(world, oracle_built):
    """Every tile/LDS-budget variant (10% long versions: keys spill past the LDS slot)."""
    from trivy_amd._lib import lib
    sdb, eng = world
    batch = make_batch(sdb, 40, 500, [3, 3, 2, 2], seed=21, long_versions=0.1, invalid=0.01)
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=8)
    vs = variants()
    assert len(vs) >= 5
    try:
        for v in vs:
            lib().tvm_engine_set_variant(eng.h, v)
            pk, ad, errp, total = run_batch(eng, sdb, batch)
            assert errp == -1 and total == len(opk), lib().tvm_variant_name(v)
            assert np.array_equal(pk, opk) and np.array_equal(ad, oad), lib().tvm_variant_name(v)
    finally:
        lib().tvm_engine_set_variant(eng.h, 0)
