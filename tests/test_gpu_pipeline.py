"""GPU: the end-to-end pipelined pass (tvm_pipeline_*: chunked H2D of a host batch - its
transport form, rebuilt in HBM by unpack_kernel, or its raw arrays - match, the result move
of the per-package advisory lists into host memory as CSR) gives exactly the oracle's
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


def _chunks(nt, ct):
    """The chunk count prepare() lays out (pipeline.hip): batches of 3+ chunks begin and end
    with a quarter chunk, whole chunks in between while more than a chunk and a quarter remain."""
    if nt == 0:
        return 1
    q = max(1, ct // 4)
    if nt < 3 * ct:
        return -(-nt // ct)
    bounds, t = [0, q], q
    while nt - t > ct + q:
        t += ct
        bounds.append(t)
    if nt - t > q:
        bounds.append(nt - q)
    bounds.append(nt)
    return len(bounds) - 1


@pytest.mark.parametrize("raw,adv32", [(False, False), (True, False), (False, True)])
@pytest.mark.parametrize("chunk", [256, 1000, 4096, 1 << 19])
def test_pipeline_matches_oracle(world, chunk, raw, adv32, oracle_built):
    sdb, eng = world
    batch = make_batch(sdb, 37, 333, [2, 2, 1], seed=chunk)  # 12321 packages: ragged last tile
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=8)
    mb = _fill(eng, sdb, batch).pipeline_prepare(match_cap=len(opk) + 5, chunk_packages=chunk, raw=raw, adv32=adv32)
    for _ in range(2):  # a second pass over the same pinned batch gives the same lists
        total, errp, ms = mb.pipeline_run()
        assert errp == -1 and total == len(opk) and ms > 0
        adv, rend = mb.pipeline_csr()
        pk, ad = _pairs_of(adv[:total], rend[:len(batch)])
        assert np.array_equal(pk, opk) and np.array_equal(ad, oad)
        araw, width = mb.pipeline_csr_raw()  # the bytes as they crossed the link
        assert width == (4 if adv32 else 3) and np.array_equal(araw, oad)
        vs = mb.vulns(pipeline=True)  # the DetectedVulnerability set straight from the result as it arrived
        assert np.array_equal(vs.pkg, opk) and np.array_equal(vs.rec, oad)
        vs.close()
    st = mb.pipeline_stats()
    ct, nt = -(-chunk // 256), -(-len(batch) // 256)  # tiles per chunk, tiles
    assert st["chunks"] == _chunks(nt, ct) and st["h2d_bytes"] > 0
    assert st["d2h_bytes"] == 4 * len(batch) + (4 if adv32 else 3) * len(opk)
    assert st["transport_form"] == (not raw)
    mb.close()


def test_pipeline_heavy_lists(oracle_built):
    """Per-package lists of 255 advisories and more ("linux" packages at the lowest version
    match every advisory of the heaviest key) beside ordinary packages; equal to the oracle."""
    from test_gpu_parity import build_engine
    from tools.synth import SynthBatch
    sdb = make_db(["debian 12"], 400, seed=21, max_adv=700)
    eng = build_engine(sdb)
    base = make_batch(sdb, 4, 300, [1], seed=2)
    names, vers = list(base.names), list(base.versions)
    for i in range(5, len(names), 97):
        names[i], vers[i] = b"linux", b"0.1"
    batch = SynthBatch(base.plat, names, vers, list(base.targets))
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=4)
    assert np.bincount(opk).max() >= 255
    mb = _fill(eng, sdb, batch).pipeline_prepare(match_cap=len(opk) + 1, chunk_packages=512)
    total, errp, _ = mb.pipeline_run()
    pk, ad = _pairs_of(*mb.pipeline_csr())
    assert total == len(opk) and np.array_equal(pk[:len(opk)], opk) and np.array_equal(ad[:len(opk)], oad)
    mb.close()


def test_pipeline_transport_form_edges(oracle_built):
    """The transport form against the oracle where it differs from the raw arrays: empty
    versions, names repeated across chunks (referenced back into earlier chunks' strings),
    a version equal to a name; and a string of 256 bytes, which has no transport form (the
    batch goes raw)."""
    from test_gpu_parity import build_engine
    from tools.synth import SynthBatch
    sdb = make_db(["debian 12", "ubuntu 22.04"], 500, seed=8)
    eng = build_engine(sdb)
    base = make_batch(sdb, 12, 300, [1, 1], seed=4)
    names, vers = list(base.names), list(base.versions)
    for i in range(0, len(names), 7):
        vers[i] = b""
    for i in range(3, len(names), 11):
        vers[i] = names[i]
    for long_one in (False, True):
        v2 = list(vers)
        if long_one:
            v2[100] = b"1." + b"9" * 254
        plat = [p for p, b0, b1 in base.targets]
        targets = list(base.targets)
        batch = SynthBatch(base.plat, names, v2, targets)
        opk, oad = om.match(om.Prepared(sdb, batch), n_threads=4)
        mb = _fill(eng, sdb, batch).pipeline_prepare(match_cap=len(opk) + 1, chunk_packages=512)
        assert mb.pipeline_stats()["transport_form"] == (not long_one)
        total, errp, _ = mb.pipeline_run()
        pk, ad = _pairs_of(*mb.pipeline_csr())
        assert total == len(opk) and np.array_equal(pk, opk) and np.array_equal(ad, oad), (long_one, plat[:3])
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


def test_concurrent_batches_keep_their_scratch():
    """Every batch owns its kernel scratch (installed keys over 32 bytes, Maven parses): a
    pipelined pass on its own streams and device-resident launches of other batches at the
    same time, from three threads, give each batch its serial result."""
    import threading

    import trivy_amd
    from tools import synth_mix as sm
    from trivy_amd.batch import MatchBatch
    sdb = sm.make_mix_db([("maven::", "maven"), ("npm::", "npm")], 1500, seed=3)
    eng = trivy_amd.Engine(sdb.put(trivy_amd.DB()).finalize(), 0)
    groups = [sm.make_mix_batch(sdb, 40_000, [3, 1], seed=s) for s in (1, 2, 3)]
    for g in groups:  # long versions: keys beyond 32 bytes take the scratch too
        for _, cols in g.groups:
            cols["ver"] = np.where(np.arange(len(cols["ver"])) % 5 == 0,
                                   np.char.add(cols["ver"], b".1.2.3.4.5.6.7.8.9.10.11.12.13"), cols["ver"])

    def make(g):
        mb = MatchBatch(eng)
        sm.add_to(mb, sdb, g)
        return mb
    serial = []
    for g in groups:
        mb = make(g)
        mb.run()
        serial.append(mb.pairs())
        mb.close()
    assert all(len(s) > 5000 for s in serial)
    pipe = make(groups[0]).pipeline_prepare(match_cap=len(serial[0]), chunk_packages=4096)
    dev = [make(g).upload(len(s)) for g, s in zip(groups[1:], serial[1:])]
    bad = []

    def run_pipe():
        for _ in range(6):
            total, errp, _ = pipe.pipeline_run()
            pk, ad = _pairs_of(*pipe.pipeline_csr())
            if not (total == len(serial[0]) and np.array_equal(np.stack([pk, ad], 1), serial[0])):
                bad.append("pipeline")

    def run_dev(k):
        for _ in range(6):
            dev[k].launch()
            if not np.array_equal(dev[k].pairs(), serial[k + 1]):
                bad.append(f"batch {k + 1}")
    ths = [threading.Thread(target=run_pipe)] + [threading.Thread(target=run_dev, args=(k,)) for k in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not bad, bad[:5]
    for mb in [pipe] + dev:
        mb.close()


def test_batches_refused_after_swap(oracle_built):
    """A batch resolves its platforms against the tables it was built on: after
    tvm_engine_swap its pipeline pass and its launches are refused (not run on mixed
    tables), freeing it touches nothing of the swapped-out engine, and a batch rebuilt on
    the new tables matches like the oracle."""
    import trivy_amd
    from test_gpu_parity import build_engine
    sdb = make_db(["debian 12", "ubuntu 22.04"], 400, seed=5)
    sdb2 = make_db(["debian 11", "debian 12", "ubuntu 22.04"], 500, seed=6)
    eng = build_engine(sdb)
    batch = make_batch(sdb, 6, 300, [1, 1], seed=2)
    pipe = _fill(eng, sdb, batch).pipeline_prepare(match_cap=1 << 17, chunk_packages=512)
    assert pipe.pipeline_run()[1] == -1
    dev = _fill(eng, sdb, batch)
    dev.run()
    eng2 = build_engine(sdb2)  # only for its DB handle
    eng.swap(eng2.db)
    with pytest.raises(RuntimeError, match="rebuild"):
        pipe.pipeline_run()
    with pytest.raises(RuntimeError, match="rebuild"):
        dev.launch()
    with pytest.raises(RuntimeError):
        dev.upload()
    pipe.close()
    dev.close()
    batch2 = make_batch(sdb2, 6, 300, [1, 1, 1], seed=3)
    fresh = _fill(eng, sdb2, batch2)
    total, errp, _ = fresh.run()
    opk, oad = om.match(om.Prepared(sdb2, batch2), n_threads=4)
    got = fresh.pairs()
    assert errp == -1 and np.array_equal(got[:, 0], opk) and np.array_equal(got[:, 1], oad)
    fresh.close()
