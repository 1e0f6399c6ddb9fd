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


class CSRGather:
    """Exact-size gather of every rank's ORDERED per-package advisory lists to `root`, which
    ends up holding the whole batch's lists in global batch order with no host sort.

    Each rank hands its shard's CSR (MatchBatch.order_into: csr_adv = the advisory indices in
    (package, advisory) order, row_end[i] = end of the shard's i-th package's list, offsets
    from 0) as int32 tensors.  Shards are contiguous package ranges in rank order, so the root
    receives rank r's advisories straight into its slice of one global array and its row ends
    into the next package slice, then adds the advisories of ranks < r to those row ends: 4 B
    per match + 4 B per package over the wire, one device-side add, no reordering.  Buffers
    only grow, so a steady-state gather allocates nothing."""

    MAX_MATCHES = 1 << 31  # row ends are int32

    def __init__(self, device, root=0):
        self.device = device
        self.root = root
        self.adv = None
        self.row_end = None

    def _grow(self, n_adv, n_pkg):
        if self.adv is None or self.adv.numel() < n_adv:
            self.adv = torch.empty(max(n_adv, 1), dtype=torch.int32, device=self.device)
        if self.row_end is None or self.row_end.numel() < n_pkg:
            self.row_end = torch.empty(max(n_pkg, 1), dtype=torch.int32, device=self.device)

    def __call__(self, csr_adv, row_end, n_matches, n_pkgs):
        """Returns (adv, row_end) of the whole batch on the root, None elsewhere."""
        rank, ws = world()
        if ws == 1:
            return csr_adv[:n_matches], row_end[:n_pkgs]
        cnt = torch.tensor([n_matches, n_pkgs], dtype=torch.int64, device=self.device)
        counts = [torch.zeros_like(cnt) for _ in range(ws)]
        dist.all_gather(counts, cnt)
        counts = [(int(c[0].item()), int(c[1].item())) for c in counts]
        t_adv = sum(c[0] for c in counts)
        t_pkg = sum(c[1] for c in counts)
        # checked on every rank before any send: a root-only check would leave the senders
        # blocked in isend
        if t_adv >= self.MAX_MATCHES:
            raise ValueError("row ends are 32-bit: gather below 2^31 matches at a time")
        if rank != self.root:
            ops = []
            if n_matches:
                ops.append(dist.P2POp(dist.isend, csr_adv[:n_matches].contiguous(), self.root))
            if n_pkgs:
                ops.append(dist.P2POp(dist.isend, row_end[:n_pkgs].contiguous(), self.root))
            if ops:
                for r in dist.batch_isend_irecv(ops):
                    r.wait()
            return None
        self._grow(t_adv, t_pkg)
        ops, a0, p0, fix = [], 0, 0, []
        for r, (na, npk) in enumerate(counts):
            dst_a, dst_p = self.adv[a0:a0 + na], self.row_end[p0:p0 + npk]
            if r == rank:
                dst_a.copy_(csr_adv[:na])
                dst_p.copy_(row_end[:npk])
            else:
                if na:
                    ops.append(dist.P2POp(dist.irecv, dst_a, r))
                if npk:
                    ops.append(dist.P2POp(dist.irecv, dst_p, r))
            if a0 and npk:
                fix.append((dst_p, a0))
            a0 += na
            p0 += npk
        if ops:
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        for dst_p, off in fix:
            dst_p.add_(off)
        return self.adv[:t_adv], self.row_end[:t_pkg]


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
