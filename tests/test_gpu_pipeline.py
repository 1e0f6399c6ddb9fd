"""GPU: the end-to-end pipelined pass (tvm_pipeline_*: chunked H2D of a host batch, match,
order_kernel, D2H of the per-package advisory lists as CSR) gives exactly the oracle's
(package, advisory) pairs, for chunk sizes that do and do not divide the batch, and
reports overflow / poisoned keys like the device-resident path."""
import numpy as np
import pytest

from oracle import match as om
from tools.synth import make_db, make_batch

pytestmark = pytest.mark.gpu


def _fill(eng, sdb, batch):
    from trivy_amd.batch import MatchBatch
    mb = MatchBatch(eng)
    arena, noff, nlen, voff, vlen = batch.arena()
    for p, b0, b1 in batch.targets:
        mb.add_arena(sdb.platforms[p], b1 - b0, arena, noff[b0:], nlen[b0:], voff[b0:], vlen[b0:])
    return mb


def _pairs_of(adv, row_end):
    counts = np.diff(np.concatenate([[0], row_end.astype(np.int64)]))
    return np.repeat(np.arange(len(row_end), dtype=np.uint32), counts), adv


@pytest.fixture(scope="module")
def world():
    from test_gpu_parity import build_engine
    sdb = make_db(["debian 11", "debian 12", "ubuntu 22.04"], 3000, seed=11)
    return sdb, build_engine(sdb)


@pytest.mark.parametrize("chunk", [256, 1000, 4096, 1 << 19])
def test_pipeline_matches_oracle(world, chunk, oracle_built):
    sdb, eng = world
    batch = make_batch(sdb, 37, 333, [2, 2, 1], seed=chunk)  # 12321 packages: ragged last tile
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=8)
    mb = _fill(eng, sdb, batch).pipeline_prepare(match_cap=len(opk) + 5, chunk_packages=chunk)
    for _ in range(2):  # a second pass over the same pinned batch gives the same lists
        total, errp, ms = mb.pipeline_run()
        assert errp == -1 and total == len(opk) and ms > 0
        adv, rend = mb.pipeline_csr()
        pk, ad = _pairs_of(adv, rend)
        assert np.array_equal(pk, opk) and np.array_equal(ad, oad)
    st = mb.pipeline_stats()
    assert st["chunks"] == -(-len(batch) // (-(-chunk // 256) * 256)) and st["h2d_bytes"] > 0
    assert st["d2h_bytes"] == 4 * (len(batch) + len(opk))
    mb.close()


def test_pipeline_overflow_then_exact(world, oracle_built):
    sdb, eng = world
    batch = make_batch(sdb, 5, 400, [1, 1, 1], seed=3)
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=8)
    mb = _fill(eng, sdb, batch).pipeline_prepare(match_cap=max(1, len(opk) // 3), chunk_packages=512)
    with pytest.raises(OverflowError) as ei:
        mb.pipeline_run()
    assert ei.value.args[0] == len(opk)  # the exact total is reported, nothing silently cut
    mb.pipeline_prepare(match_cap=len(opk), chunk_packages=512)
    total, errp, _ = mb.pipeline_run()
    pk, ad = _pairs_of(*mb.pipeline_csr())
    assert total == len(opk) and np.array_equal(pk, opk) and np.array_equal(ad, oad)
    mb.close()


def test_pipeline_poisoned_and_empty(oracle_built):
    from test_gpu_parity import build_engine
    from trivy_amd.batch import MatchBatch
    sdb = make_db(["debian 12", "ubuntu 22.04"], 300, seed=4)
    poison = [int(sdb.plat_keys[0][5]), int(sdb.plat_keys[1][7])]
    eng = build_engine(sdb, poison)
    batch = make_batch(sdb, 30, 300, [1, 1], seed=9, miss=0.0)
    mb = _fill(eng, sdb, batch).pipeline_prepare(match_cap=64 * len(batch), chunk_packages=700)
    _, errp, _ = mb.pipeline_run()
    with pytest.raises(om.PoisonedKey) as ei:
        om.match(om.Prepared(sdb, batch, poisoned=poison), n_threads=1)
    assert errp == ei.value.pkg
    mb.close()
    empty = MatchBatch(eng).pipeline_prepare(chunk_packages=256)
    assert empty.pipeline_run()[:2] == (0, -1)
    empty.close()
