#!/usr/bin/env python3
"""Two-rank check of the sharded match + gather on ONE GPU (ranks share the device, gloo
collectives through host memory): one global batch, shards on target boundaries balanced by
predicted rows, every rank matches its shard with global package indices, the exact-size
gather brings every rank's list to rank 0, which compares it with a single-rank match of
the whole batch.  Run by tests/test_gpu_dist.py under torch.distributed.run."""
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
    if rank == 0:
        merged = np.stack([torch.cat([p for p, _ in parts]).numpy().view(np.uint32),
                           torch.cat([a for _, a in parts]).numpy().view(np.uint32)], axis=1)
        full = fill(MatchBatch(eng), 0, len(batch))
        full.run()
        ref = full.pairs()
        # each rank's list is in tile order, shards in rank order: compare as (package, advisory) sets
        got = merged[np.lexsort((merged[:, 1], merged[:, 0]))]
        assert got.shape == ref.shape and np.array_equal(got, ref), (got.shape, ref.shape)
        print(f"DIST OK {ws} ranks, shards {bounds}, {len(ref)} matches", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
