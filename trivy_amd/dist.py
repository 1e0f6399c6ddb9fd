"""Node-level sharding of package batches over GPUs.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, "gloo" on CPU for
tests).  Packages are independent, so the batch is split into contiguous shards - by
package count, or by predicted pair count (Σ advisories per package, from a host-side
pre-probe) so a Zipf-heavy key does not leave one GPU behind - and each rank matches its
shard against its own replica of the advisory tables: no collective on the data path.
Match lists stay on their GPU; `gather_pairs` brings them to one rank when a caller needs
the merged set (sizes all-gathered first, then one gather of the variable-length lists).
"""
import time

import numpy as np
import torch
import torch.distributed as dist


def world():
    """(rank, world_size) of the current process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard(n, rank, world_size):
    """Contiguous [begin, end) of n packages for `rank` (sizes differ by at most one)."""
    q, r = divmod(n, world_size)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def balanced_shards(weights, world_size):
    """Contiguous shard boundaries (world_size + 1 entries) with near-equal Σ weights."""
    w = np.asarray(weights, dtype=np.float64)
    if len(w) == 0:
        return [0] * (world_size + 1)
    c = np.cumsum(w)
    total = c[-1]
    bounds = [0]
    for k in range(1, world_size):
        bounds.append(int(np.searchsorted(c, total * k / world_size, side="left")) + 1)
    bounds.append(len(w))
    for k in range(1, len(bounds)):
        bounds[k] = min(max(bounds[k], bounds[k - 1]), len(w))
    return bounds


def max_over_ranks(x, device="cpu"):
    """The maximum of a float over all ranks (the job's wall time is its slowest rank)."""
    if world()[1] == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(step, steps, warmup, sync=lambda: None, device="cpu"):
    """Runs `warmup` untimed steps, then `steps` steps bracketed by barrier + sync on both
    sides; returns the wall seconds of the timed region, maximum over ranks."""
    for _ in range(warmup):
        step()
    if world()[1] > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world()[1] > 1:
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, device)


def gather_pairs(pairs, pkg_offset, dst=0):
    """Gathers every rank's (package, advisory) pairs to rank `dst`.

    pairs: int64 tensor [m, 2] of this rank's matches with shard-local package indices;
    pkg_offset: this rank's first global package index.  Returns the merged [M, 2] tensor
    in global package order on `dst`, None elsewhere."""
    rank, ws = world()
    local = pairs.to(torch.int64).clone()
    if local.numel():
        local[:, 0] += pkg_offset
    if ws == 1:
        return local
    dev = local.device
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    cap = max(max(sizes), 1)
    buf = torch.zeros((cap, 2), dtype=torch.int64, device=dev)
    buf[:local.shape[0]] = local
    if rank == dst:
        parts = [torch.zeros((cap, 2), dtype=torch.int64, device=dev) for _ in range(ws)]
        dist.gather(buf, gather_list=parts, dst=dst)
        return torch.cat([p[:s] for p, s in zip(parts, sizes)])
    dist.gather(buf, dst=dst)
    return None
