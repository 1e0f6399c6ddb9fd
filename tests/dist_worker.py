#!/usr/bin/env python3
"""TEST HELPER (not collected by pytest): two-rank check of the sharded match + gather on ONE
GPU (ranks share the device, gloo collectives through host memory).  One global batch,
shards on target boundaries balanced by predicted rows; every rank matches its shard through
the product engine, the order kernel turns its matches into per-package lists (CSR), and
the CSR gather brings them to rank 0 in global batch order.  Rank 0 compares them, with no
sort, with the oracle's match of the whole batch (oracle/match.c), and the raw pair gather
with the oracle as a multiset.  Run by tests/test_gpu_dist.py under torch.distributed.run."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import trivy_amd
    from trivy_amd import dist as td
    from trivy_amd._lib import lib
    from trivy_amd.batch import MatchBatch
    from tools.synth import make_db, make_batch
    from oracle import match as om
    dist.init_process_group("gloo")
    rank, ws = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    sdb = make_db(["debian 12", "ubuntu 22.04", "ubuntu 24.04"], 4000, seed=31)
    batch = make_batch(sdb, 301, 211, [2, 1, 1], seed=32)
    db = trivy_amd.DB()
    for n, depth, arena, off, lens in (sdb.records_arena(), sdb.source_arena()):
        db.put_arena(n, depth, arena, off, lens)
    eng = trivy_amd.Engine(db.finalize(), 0)
    arena, noff, nlen, voff, vlen = batch.arena()
    rows = np.zeros(len(batch), dtype=np.uint32)
    for p, b0, b1 in batch.targets:
        lib().tvm_db_rows_many(db.h, sdb.platforms[p].encode(), b1 - b0, arena, noff[b0:].ctypes.data,
                               nlen[b0:].ctypes.data, rows[b0:].ctypes.data)
    bounds = td.target_shards([b0 for _, b0, _ in batch.targets], len(batch), rows + 1.0, ws)
    sb, se = bounds[rank], bounds[rank + 1]

    def fill(mb, b, e):
        for p, b0, b1 in batch.targets:
            if b0 >= b and b1 <= e:
                mb.add_arena(sdb.platforms[p], b1 - b0, arena, noff[b0:], nlen[b0:], voff[b0:], vlen[b0:])
        return mb

    mb = fill(MatchBatch(eng), sb, se).set_package_base(sb)
    total, errp, bits = mb.run()
    assert errp == -1 and bits == 0
    cols = [torch.empty(max(total, 1), dtype=torch.int32, device="cuda:0") for _ in range(2)]
    mb.upload_into(*cols).launch()
    assert mb.status()[0] == total
    parts = td.MatchGather("cpu")(cols[0][:total].cpu(), cols[1][:total].cpu(), total)
    csr_adv = torch.empty(max(total, 1), dtype=torch.int32, device="cuda:0")
    row_end = torch.empty(max(se - sb, 1), dtype=torch.int32, device="cuda:0")
    assert mb.order_into(csr_adv, row_end) == total
    g = td.CSRGather("cpu")(csr_adv[:total].cpu(), row_end[:se - sb].cpu(), total, se - sb)
    if rank == 0:
        opk, oad = om.match(om.Prepared(sdb, batch), n_threads=4)
        # ordered CSR in global batch order, compared as is
        want_end = np.cumsum(np.bincount(opk, minlength=len(batch)))
        assert np.array_equal(g[0].numpy().view(np.uint32), oad.astype(np.uint32)), "CSR advisories"
        assert np.array_equal(g[1].numpy().astype(np.int64), want_end), "CSR row ends"
        # raw pairs: each rank's list is in tile order, so compare as a (package, advisory) set
        merged = np.stack([torch.cat([p for p, _ in parts]).numpy().view(np.uint32),
                           torch.cat([a for _, a in parts]).numpy().view(np.uint32)], axis=1)
        got = merged[np.lexsort((merged[:, 1], merged[:, 0]))]
        assert np.array_equal(got, np.stack([opk, oad], axis=1).astype(np.uint32)), (got.shape, len(opk))
        print(f"DIST OK {ws} ranks, shards {bounds}, {len(opk)} matches (CSR and pairs equal the oracle)", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
