"""CPU: the multi-GPU layer (trivy_amd/dist.py) with world_size 2 over gloo.

The GPU runs use the same code with the RCCL ("nccl") backend, one process per GPU; here
each rank's match step is the oracle (oracle/match.c) on its shard of ONE global batch, and
the gathered lists must equal the single-process match of the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from trivy_amd import dist as td


def test_shard_covers_everything():
    for n in (0, 1, 7, 4_000_000):
        for ws in (1, 2, 3, 8):
            spans = [td.shard(n, r, ws) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(e - b for b, e in spans) - min(e - b for b, e in spans) <= 1


def test_balanced_shards_follow_weights():
    w = np.ones(1000)
    w[10] = 5000  # a Zipf-heavy package
    b = td.balanced_shards(w, 4)
    assert b[0] == 0 and b[-1] == 1000 and b == sorted(b)
    assert b[1] <= 11  # the heavy package closes the first shard on its own
    assert td.balanced_shards([], 3) == [0, 0, 0, 0]


def test_target_shards_keep_targets_whole():
    tb = [0, 3, 10, 11, 40]
    w = np.ones(50)
    w[12] = 100.0
    b = td.target_shards(tb, 50, w, 3)
    assert b[0] == 0 and b[-1] == 50 and all(x in tb + [50] for x in b) and b == sorted(b)
    assert td.target_shards([], 0, [], 2) == [0, 0, 0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch():
    from tools.synth import make_db, make_batch
    sdb = make_db(["debian 12", "ubuntu 22.04"], 800, seed=21)
    batch = make_batch(sdb, 23, 97, [1, 1], seed=22)
    return sdb, batch


def _rows(sdb, batch):
    """Predicted work per package: advisories of its key (the host pre-probe) + 1."""
    cnt = {}
    for k, name in enumerate(sdb.key_names):
        cnt[(int(sdb.key_plat[k]), name)] = int(sdb.adv_begin[k + 1] - sdb.adv_begin[k])
    return np.array([cnt.get((int(p), n), 0) + 1 for p, n in zip(batch.plat, batch.names)], dtype=np.float64)


def _csr(pk, ad, n):
    """(advisories, row ends) of n packages from (package, advisory)-ordered pairs."""
    row_end = np.cumsum(np.bincount(np.asarray(pk, dtype=np.int64), minlength=n)[:n])
    return np.asarray(ad, dtype=np.int32), row_end.astype(np.int32)


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from oracle import match as om
        from tools.synth import SynthBatch
        sdb, batch = _global_batch()
        bounds = td.target_shards([b0 for _, b0, _ in batch.targets], len(batch), _rows(sdb, batch), ws)
        b, e = bounds[rank], bounds[rank + 1]
        sub = SynthBatch(batch.plat[b:e], batch.names[b:e], batch.versions[b:e], [])
        pk, ad = om.match(om.Prepared(sdb, sub), n_threads=2)
        pkg = torch.tensor(np.asarray(pk, dtype=np.int64) + b, dtype=torch.int32)
        adv = torch.tensor(np.asarray(ad, dtype=np.int64), dtype=torch.int32)
        parts = td.MatchGather("cpu")(pkg, adv, len(pk))
        # the ordered form: every rank's CSR (offsets from its shard's first package)
        ca, cr = _csr(np.asarray(pk), ad, e - b)
        g = td.CSRGather("cpu")(torch.from_numpy(ca), torch.from_numpy(cr), len(ca), e - b)
        csr = None if g is None else (g[0].tolist(), g[1].tolist())
        wall = td.timed(lambda: None, steps=3, warmup=1)
        m = td.max_over_ranks(float(rank + 1))
        merged = None
        if parts is not None:
            merged = (torch.cat([p for p, _ in parts]).tolist(), torch.cat([a for _, a in parts]).tolist())
        q.put((rank, merged, wall >= 0, m, (b, e), csr))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_sharded_match_gathers_to_single_rank_result(oracle_built):
    from oracle import match as om
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {r: (m, ok, mx, span, csr) for r, m, ok, mx, span, csr in (q.get(timeout=100) for _ in ps)}
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    merged, ok, mx, span0, csr = out[0]
    assert ok and mx == 2.0 and out[1][2] == 2.0 and out[1][0] is None
    assert span0[0] == 0 and span0[1] == out[1][3][0] and 0 < span0[1]  # both ranks got work
    sdb, batch = _global_batch()
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=2)
    assert merged[0] == [int(x) for x in opk] and merged[1] == [int(x) for x in oad]
    # the ordered gather: the root holds the whole batch's per-package lists in batch order,
    # equal to the oracle's CSR without any sort
    assert out[1][4] is None
    ca, cr = _csr(opk, oad, len(batch))
    assert csr[0] == ca.tolist() and csr[1] == cr.tolist()


def _overflow_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        g = td.CSRGather("cpu")
        g.MAX_MATCHES = 5  # stand-in for 2^31: 3 + 3 matches overflow it
        adv = torch.arange(3, dtype=torch.int32)
        try:
            g(adv, torch.tensor([1, 3], dtype=torch.int32), 3, 2)
            q.put((rank, "returned"))
        except ValueError:
            q.put((rank, "raised"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_csr_gather_overflow_raises_on_every_rank():
    """An oversized gather fails on every rank before any send (no rank left blocked)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_overflow_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=100) for _ in ps)
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert out == {0: "raised", 1: "raised"}
