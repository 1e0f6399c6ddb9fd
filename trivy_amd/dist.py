"""Node-level sharding of one package batch over GPUs.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, "gloo" on CPU for
tests).  The advisory tables are replicated on every GPU; ONE global batch is cut into
contiguous shards on target (result) boundaries - so a result is never split across ranks
and result.Filter's per-result dedup / order stays valid - balanced by predicted work: the
Σ advisory rows of each target from a host-side pre-probe of the DB index
(tvm_db_rows_many), not by package count, so a Zipf-heavy key ("linux") does not leave one
GPU behind.  Each rank matches its shard; the match lists then come to one rank through an
exact-size gather (all-gather of the per-rank counts, then one point-to-point receive per
rank into the root's buffer, no padding): 8 bytes per match (package u32, advisory u32).
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
    """Contiguous [begin, end) of n items for `rank` (sizes differ by at most one)."""
    q, r = divmod(n, world_size)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def balanced_shards(weights, world_size):
    """Contiguous boundaries (world_size + 1 entries) over len(weights) items with near-equal
    Σ weights; every boundary falls between items."""
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


def target_shards(target_begin, n_packages, pkg_weights, world_size):
    """Shards of a batch on target boundaries.  target_begin: first package of every target
    (ascending); pkg_weights: predicted work per package (e.g. rows + 1).  Returns
    world_size + 1 package boundaries."""
    tb = np.asarray(list(target_begin) + [n_packages], dtype=np.int64)
    csum = np.concatenate([[0.0], np.cumsum(np.asarray(pkg_weights, dtype=np.float64))])
    tw = csum[tb[1:]] - csum[tb[:-1]]
    tbounds = balanced_shards(tw, world_size)
    return [int(tb[t]) for t in tbounds]


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


class MatchGather:
    """Exact-size gather of every rank's match columns to `root`.

    pkg / adv: this rank's uint32 columns as int32 tensors (their first n entries are the
    matches; package indices already global).  The root keeps one receive buffer per rank
    sized by the largest count seen (grown on demand), so a steady-state gather allocates
    nothing."""

    def __init__(self, device, root=0):
        self.device = device
        self.root = root
        self.bufs = {}

    def __call__(self, pkg, adv, n):
        rank, ws = world()
        if ws == 1:
            return [(pkg[:n], adv[:n])]
        cnt = torch.tensor([n], dtype=torch.int64, device=self.device)
        counts = [torch.zeros_like(cnt) for _ in range(ws)]
        dist.all_gather(counts, cnt)
        counts = [int(c.item()) for c in counts]
        if rank != self.root:
            if n:
                ops = [dist.P2POp(dist.isend, pkg[:n].contiguous(), self.root),
                       dist.P2POp(dist.isend, adv[:n].contiguous(), self.root)]
                for r in dist.batch_isend_irecv(ops):
                    r.wait()
            return None
        ops, parts = [], []
        for r in range(ws):
            if r == rank:
                parts.append((pkg[:n], adv[:n]))
                continue
            c = counts[r]
            bp, ba = self.bufs.get(r, (None, None))
            if bp is None or bp.numel() < c:
                bp = torch.empty(max(c, 1), dtype=torch.int32, device=self.device)
                ba = torch.empty(max(c, 1), dtype=torch.int32, device=self.device)
                self.bufs[r] = (bp, ba)
            parts.append((bp[:c], ba[:c]))
            if c:
                ops += [dist.P2POp(dist.irecv, bp[:c], r), dist.P2POp(dist.irecv, ba[:c], r)]
        if ops:
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        return parts
