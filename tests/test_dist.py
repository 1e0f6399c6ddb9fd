"""CPU: the multi-GPU layer (trivy_amd/dist.py) with world_size 2 over gloo.

The GPU runs use the same code with the RCCL ("nccl") backend, one process per GPU."""
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        b, e = td.shard(10, rank, ws)
        # rank r matches packages [b, e); rank 1 has one more match than rank 0
        local = torch.tensor([[i - b, 100 + i] for i in range(b, e)] + ([[0, 7]] if rank == 1 else []),
                             dtype=torch.int64)
        merged = td.gather_pairs(local, b)
        wall = td.timed(lambda: None, steps=3, warmup=1)
        m = td.max_over_ranks(float(rank + 1))
        q.put((rank, None if merged is None else merged.tolist(), wall >= 0, m))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gather_and_max_over_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict((r, (m, ok, mx)) for r, m, ok, mx in (q.get(timeout=100) for _ in ps))
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    merged, ok, mx = out[0]
    assert ok and mx == 2.0 and out[1][2] == 2.0
    assert out[1][0] is None
    assert merged == [[i, 100 + i] for i in range(5)] + [[i, 100 + i] for i in range(5, 10)] + [[5, 7]]
