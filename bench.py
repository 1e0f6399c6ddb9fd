#!/usr/bin/env python3
"""Benchmark: packages matched/sec (node) on BASELINE.json config C2 (dpkg, ~4M packages).

BASELINE.json metric: "packages matched/sec (node) at 1/2/4/8 GPUs; probe HBM GB/s vs peak".
Workload (configs[1], the default): 10k synthetic Debian/Ubuntu image SBOMs x 400 packages
= 4M packages, Debian:Ubuntu 60:40 (debian 11/12, ubuntu 20.04/22.04/24.04), against a
seeded synthetic trivy-db of 5 x 30k package keys (~1.7M advisories, heavy-tailed, 15 %
unfixed).  The pinned trivy-db cannot be fetched offline, hence synthetic data
(tools/synth.py).  --config c3 / c4 / c5: the language-package, mixed OS+language and
RHEL-family/Alpine workloads (tools/synth_mix.py) - extra measurements, not the headline.

One step = one pass of the hot path over a batch resident in HBM: the match kernels (probe +
interval sweep).  With N > 1 GPUs (one process per GPU; `python bench.py --gpus N` starts the N
ranks itself) every rank matches its own batch of the config against its replica of the
tables: packages are independent, so the step has no collective (weak scaling, value = N x
packages x steps / max-over-ranks wall time).  --gather instead cuts ONE global batch into
contiguous shards on target boundaries (balanced by predicted advisory rows) and adds the
per-rank order kernel (per-package lists, CSR) and the exact-size gather of those lists to rank
0 over RCCL to the step (strong scaling).

Also reported (rank 0): roofline of the match kernels (algorithmic bytes per launch / HIP
event time, vs the 8 TB/s HBM peak), the end-to-end pipelined pass over PCIe
(end_to_end: host batch -> GPU -> per-package advisory lists on the host, N = 1), the
FillInfo and result.Filter legs behind the match, and the oracle CPU baseline on a
bounded sample (N = 1).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PLATS = ["debian 11", "debian 12", "ubuntu 20.04", "ubuntu 22.04", "ubuntu 24.04"]
WEIGHTS = [30, 30, 13, 13, 14]  # Debian:Ubuntu 60:40


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


# ---- workloads ------------------------------------------------------------------------------
# Every workload is ONE global batch (identical on every rank) cut into targets (SBOMs /
# lockfiles): targets() = first package of each target; fill(mb, b, e) adds packages [b, e)
# (whole targets) to a MatchBatch; rows(db) = predicted advisory rows per package.
class C2:
    """dpkg fleet (tools/synth.py); the oracle C port (oracle/match.c) is the CPU baseline."""

    def __init__(self, args):
        from tools.synth import make_db, make_batch
        self.sdb = make_db(PLATS, args.keys_per_plat)
        self.batch = make_batch(self.sdb, args.targets, args.pkgs_per_target, WEIGHTS, seed=2)
        self.name = f"c2-dpkg-{args.targets}x{args.pkgs_per_target}"
        self.n = len(self.batch)
        self.n_adv = self.sdb.n_adv
        self.n_keys = len(self.sdb.key_names)
        self.plats = PLATS
        self.has_vulns = False
        self._arena = None

    def load(self, db, vulns=True):
        from tools.synth_vuln import vuln_arena
        parts = [self.sdb.records_arena(detail=vulns), self.sdb.source_arena()]
        if vulns:  # bucket "vulnerability" for the FillInfo leg (tools/synth_vuln.py)
            parts.append(vuln_arena(self.sdb.vuln_ids()))
        self.has_vulns = vulns
        for n, depth, arena, off, lens in parts:
            db.put_arena(n, depth, arena, off, lens)

    def arena(self):
        if self._arena is None:
            self._arena = self.batch.arena()
        return self._arena

    def targets(self):
        return [b0 for _, b0, _ in self.batch.targets]

    def rows(self, db):
        from trivy_amd._lib import lib
        arena, noff, nlen, _, _ = self.arena()
        out = np.zeros(self.n, dtype=np.uint32)
        for p, b0, b1 in self.batch.targets:
            lib().tvm_db_rows_many(db.h, self.sdb.platforms[p].encode(), b1 - b0, arena, noff[b0:].ctypes.data,
                                   nlen[b0:].ctypes.data, out[b0:].ctypes.data)
        return out

    build_how = "tvm_batch_add_targets: one C-ABI call for every target of the batch (per target its bucket)"

    def fill(self, mb, b=0, e=None):
        """Packages [b, e) (whole targets), one Result per target, in one tvm_batch_add_targets call."""
        e = self.n if e is None else e
        arena, noff, nlen, voff, vlen = self.arena()
        sel = [(p, b0, b1) for p, b0, b1 in self.batch.targets if b0 >= b and b1 <= e]
        if not sel:
            return
        lo, hi = sel[0][1], sel[-1][2]
        ends = np.array([b1 - lo for _, _, b1 in sel], dtype=np.uint64)
        mb.add_targets([self.sdb.platforms[p] for p, _, _ in sel], ends, arena, noff[lo:hi], nlen[lo:hi], voff[lo:hi],
                       vlen[lo:hi])

    def vuln_ids(self):
        return self.sdb.vuln_ids()

    def adv_vuln_id(self, db, a):
        return self.sdb.adv_vid[a]

    def cpu_baseline(self, budget_s, threads):
        from oracle import match as om
        from tools.synth import SynthBatch
        batch = self.batch
        n = min(self.n, 500_000)
        sub = SynthBatch(batch.plat[:n], batch.names[:n], batch.versions[:n], [])
        prep = om.Prepared(self.sdb, sub)
        rates = {}
        for t in sorted({1, threads}):
            done, dt, t0 = 0, 0.0, time.perf_counter()
            while dt < budget_s / 2:  # whole passes over the sample until half the budget is spent
                om.match(prep, n_threads=t)
                done += n
                dt = time.perf_counter() - t0
            rates[t] = done / dt
        return {"value": rates[threads], "unit": "packages/s", "cores": threads, "kind": "port",
                "value_1thread": rates[1], "cpu_model": cpu_model(),
                "sample": f"passes over the first {n} packages of the same batch, oracle/match.c orc_match (C, "
                          f"pthreads) with {threads} threads (this host's CPU share) and with 1 thread, "
                          f"~{budget_s / 2:.0f}s each"}


class Mix:
    """C3 (language packages), C5 (rpm + apk) and C4 (mixed OS + language) batches of
    tools/synth_mix.py; a group (one platform's packages) is cut into targets of
    `per_target` packages.  CPU baseline: the C port of the driver loops (oracle/mixmatch.c) on a
    bounded sample batch, at 1 and N threads."""

    per_target = 400
    build_how = ("tvm_batch_add_targets_attrs: one C-ABI call for every target of the batch (per target its bucket "
                 "and attribute flags; arch / ksplice / CPE-set columns per package; CPE sets registered per batch)")

    def __init__(self, args, which):
        from tools import synth_mix as sm
        self.sm = sm
        plats, weights, kpp, n = {
            "c3": (sm.C3_PLATS, sm.C3_WEIGHTS, 25_000, 1_000_000),
            "c4": (sm.C4_PLATS, sm.C4_WEIGHTS, 20_000, 100_000_000),
            "c5": (sm.C5_PLATS, sm.C5_WEIGHTS, 12_000, 20_000_000)}[which]
        n = args.packages or n
        if os.environ.get("TVM_BENCH_WEIGHTS"):  # measurement only: another platform mix (named in the workload)
            weights = [float(x) for x in os.environ["TVM_BENCH_WEIGHTS"].split(",")]
        self.which, self.kpp = which, kpp
        self.sdb = sm.make_mix_db(plats, kpp)
        self.batch = sm.make_mix_batch(self.sdb, n, weights, seed=2)
        kind = {"c3": "lang", "c4": "os+lang", "c5": "rpm-apk"}[which]
        self.name = f"{which}-{kind}-{n}" + (f"-w{os.environ['TVM_BENCH_WEIGHTS']}" if os.environ.get("TVM_BENCH_WEIGHTS") else "") \
            + (f"-mvnpre{os.environ['TVM_SYNTH_MAVEN_PRE']}" if os.environ.get("TVM_SYNTH_MAVEN_PRE") else "")
        self.n = len(self.batch)
        self.n_adv = self.sdb.n_adv
        self.n_keys = len(self.sdb.keys)
        self.plats = [b for b, _ in plats]
        self.has_vulns = False
        self.starts = []
        o = 0
        for _, g in self.batch.groups:
            self.starts.append(o)
            o += len(g["key"])

    def load(self, db, vulns=False):
        self.sdb.put(db)
        if vulns:  # bucket "vulnerability" over every advisory's VulnerabilityID (FillInfo / Filter / VEX legs)
            from tools.synth_vuln import vuln_arena
            self._vids = self.sm.MixDB.vuln_ids_of(self.sdb)
            db.put_arena(*vuln_arena(self._vids))
        self.has_vulns = vulns

    def vuln_ids(self):
        return self._vids

    def adv_vuln_id(self, db, a):
        from trivy_amd.batch import advisory_vuln_id
        return advisory_vuln_id(db, a)

    def targets(self):
        out = []
        for s, (_, g) in zip(self.starts, self.batch.groups):
            out += list(range(s, s + len(g["key"]), self.per_target))
        return out

    def rows(self, db):
        from trivy_amd._lib import lib
        from trivy_amd.batch import arena_of
        out = np.zeros(self.n, dtype=np.uint32)
        for s, (p, g) in zip(self.starts, self.batch.groups):
            bucket, kind = self.sdb.plats[p]
            if kind in self.sm.LANG_OF:
                out[s:s + len(g["key"])] = 1  # language buckets span several roots: count packages
                continue
            arena, ((off, ln),) = arena_of(g["name"])
            lib().tvm_db_rows_many(db.h, bucket.encode(), len(ln), arena, off.ctypes.data, ln.ctypes.data,
                                   out[s:].ctypes.data)
        return out

    def fill(self, mb, b=0, e=None):
        """Packages [b, e) (whole targets) in one tvm_batch_add_targets_attrs call: one Result
        (result.Filter's scope: its dedup and order) per target of per_target packages, as the
        images / lockfiles of a fleet arrive.  The columns (one arena) are built once per
        workload (tools/synth_mix.py BulkCols), as a caller's decoder would hand them over."""
        if getattr(self, "_bulk", None) is None:
            self._bulk = self.sm.BulkCols(self.sdb, self.batch, self.per_target)
        self._bulk.add(mb, b, self.n if e is None else e)

    def cpu_baseline(self, budget_s, threads):
        """The native C port of the driver loops (oracle/mixmatch.c + oracle/libcmp.c, pinned by
        tests/test_cport.py to oracle/drivers.py + oracle/library.py and the reference's
        compare_test.go tables) over a bounded sample batch of the same DB and generator, at
        1 thread and at `threads` threads.  The advisories of the sample's keys are decoded once
        beforehand (oracle/mix_c.py), which makes this a conservative - fast - baseline: the
        reference decodes them per call."""
        from oracle import mix_c
        n = {"c3": 200_000, "c4": 200_000, "c5": 200_000}[self.which]
        sb = self.sm.make_mix_batch(self.sdb, n, {"c3": self.sm.C3_WEIGHTS, "c4": self.sm.C4_WEIGHTS,
                                                  "c5": self.sm.C5_WEIGHTS}[self.which], seed=1000)
        prep = mix_c.Prepared(self.sm, self.sdb, [(p, g, list(range(len(g["key"])))) for p, g in sb.groups])
        rates = {}
        for t in sorted({1, threads}):
            done, dt, t0 = 0, 0.0, time.perf_counter()
            while dt < budget_s / 2:
                mix_c.match(prep, n_threads=t)
                done += prep.n
                dt = time.perf_counter() - t0
            rates[t] = done / dt
        return {"value": rates[threads], "unit": "packages/s", "cores": threads, "kind": "port",
                "value_1thread": rates[1], "cpu_model": cpu_model(),
                "sample": f"passes over a seeded {prep.n}-package sample batch of the same DB and generator, "
                          f"oracle/mixmatch.c orc_mix_match (C, pthreads; advisories decoded once beforehand) with "
                          f"{threads} threads (this host's CPU share) and with 1 thread, ~{budget_s / 2:.0f}s each"}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def kernel_source_hash():
    """sha1 over the sources the match kernels are compiled from (their headers + kern_*.hip) and the
    table builder whose layout they read (db.cpp / db.h: slot load, row packing): ties a committed PMC
    summary to the build it was measured on."""
    import glob
    import hashlib
    h = hashlib.sha1()
    csrc = os.path.join(ROOT, "trivy_amd", "csrc")
    # the match kernels' translation units and the headers they include (Makefile HDRS_KERN)
    kern_hdrs = ["common.h", "engine.h", "libver.h", "verkey.h", "unicode_tab.h", "match_kernel.h", "match_variants.h",
                 "db.h", "db.cpp"]
    for f in sorted([os.path.join(csrc, h) for h in kern_hdrs] + glob.glob(os.path.join(csrc, "kern_*.hip"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(config, workload, variant, src_hash):
    """HBM bytes (raw FETCH_SIZE + WRITE_SIZE) of one full-grid launch of the match kernel from
    the committed rocprofv3 summary of this config (tools/pmc_summary.py --json), or the reason
    it cannot be used: a summary of another workload, kernel variant or kernel source is refused."""
    p = os.path.join(ROOT, "profiles", f"pmc_summary_{config}.json")
    if not os.path.exists(p):
        return None, f"no profiles/pmc_summary_{config}.json"
    with open(p) as f:
        d = json.load(f)
    for k, want in (("workload", workload), ("kernel_variant", variant), ("kernel_source", src_hash)):
        if d.get(k) != want:
            return None, f"profiles/pmc_summary_{config}.json is for {k}={d.get(k)!r}, this run is {want!r}"
    sized = d.get("hbm_bytes_sized")
    return (sized if sized else d["hbm_bytes_per_launch"]), {
        "kernel": d["kernel"], "grid": d["grid"], "fetch_bytes_raw": d["fetch_bytes_raw"],
        "fetch_bytes_sized": d.get("fetch_bytes_sized"), "write_bytes": d["write_bytes"],
        "hbm_bytes_raw": d["hbm_bytes_per_launch"], "rdreq": d.get("rdreq"),
        "traffic_is": ("corrected: read bytes by request size (128 R_128B + 64 R_64B + 32 R_32B) + WRITE_SIZE"
                       if sized else "raw FETCH_SIZE + WRITE_SIZE (no request-size pass in the summary)"),
        "avg_ns_full_grid": d["avg_ns_full_grid"], "source": f"profiles/pmc_summary_{config}.json", "note": d["note"]}


def launch_ranks(n):
    """N ranks of this script through torch.distributed.run on one node (127.0.0.1, a free
    port), one per GPU; returns the launcher's exit status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL / tensor sharing need dmabuf IPC on this host
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment, N > 1 launches N ranks "
                         "through torch.distributed.run itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2")
    ap.add_argument("--keys-per-plat", type=int, default=30000)
    ap.add_argument("--targets", type=int, default=10000)
    ap.add_argument("--pkgs-per-target", type=int, default=400)
    ap.add_argument("--packages", type=int, default=0, help="c3/c4/c5: packages of the global batch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: OMP_NUM_THREADS, else os.cpu_count()")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-fill", action="store_true", help="c2: skip the FillInfo / Filter legs")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end pipelined pass")
    ap.add_argument("--chunk", type=int, default=1 << 20, help="end-to-end pass: packages per pipeline chunk")
    ap.add_argument("--no-dropin", action="store_true",
                    help="c2: skip the C1-shaped leg (100-package requests through the per-target driver path)")
    ap.add_argument("--variant", type=int, default=None, help="match-path variant (tvm_engine_set_variant)")
    ap.add_argument("--sweep", type=int, default=0,
                    help="time every match-path variant over N interleaved rounds (stderr table) first")
    ap.add_argument("--gather", action="store_true",
                    help="strong scaling: ONE global batch sharded across the ranks on target boundaries, each "
                         "rank's per-package lists gathered to rank 0 over RCCL inside the timed step (default: "
                         "weak scaling, every rank matches its own batch of the config, no collective in the step)")
    ap.add_argument("--dump-csr", default=None,
                    help="rank 0 writes the whole batch's per-package advisory lists (CSR, as gathered) to this "
                         ".npz after the timed region (checked against the oracle by tests/test_gpu_bench_dist.py)")
    args = ap.parse_args()

    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: start the N ranks here, before this process touches a GPU
        # (no torch import yet), and hand back rank 0's line and the launcher's exit status
        return launch_ranks(args.gpus)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if args.gpus is not None and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    local = int(os.environ.get("LOCAL_RANK", 0))
    # torch first: libtrivy_amd.so and torch's bundled HIP runtime share the SONAME
    # libamdhip64.so.7, so the library then binds to torch's runtime (ROCm 7.0 in this image)
    # rather than /opt/rocm's 7.2 it was built with; the line records which one ran
    # (config.hip_runtime).  Loading the library first does not work: torch's HIP initialisation
    # then fails on the box and no device is visible to either (measured)
    import torch
    import torch.distributed as dist
    import trivy_amd
    # TVM_BENCH_BACKEND=gloo rehearses the N>1 path on a box with fewer GPUs than ranks
    # (ranks then share devices round-robin, the gather goes through host memory); the
    # scaling runs use RCCL, one rank per GPU
    backend = os.environ.get("TVM_BENCH_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend)
    if torch.cuda.is_available():
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
    gdev = f"cuda:{local}"
    cdev = gdev if backend == "nccl" else "cpu"  # where collectives run

    from trivy_amd import dist as td
    from trivy_amd._lib import lib
    from trivy_amd.batch import MatchBatch
    t0 = time.perf_counter()
    wl = C2(args) if args.config == "c2" else Mix(args, args.config)
    db = trivy_amd.DB()
    wl.load(db, vulns=args.config in ("c2", "c4", "c5") and not args.no_fill)
    eng = trivy_amd.Engine(db.finalize(), local)
    log(rank, f"[bench] {wl.name}: db {wl.n_keys} keys, {wl.n_adv} advisories, tables "
              f"{eng.table_bytes()/1e6:.1f} MB ({time.perf_counter()-t0:.1f}s)")

    rows = wl.rows(db)
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)

    def measure(strong, primary):
        """One scaling mode: weak (every rank matches its own batch of the config, no
        collective) or strong (ONE global batch sharded on target boundaries by predicted rows,
        per-rank order kernel + CSR gather to rank 0 inside the timed step)."""
        t0 = time.perf_counter()
        if strong:
            bounds = td.target_shards(wl.targets(), wl.n, rows.astype(np.float64) + 1.0, world)
        else:
            bounds = [0] * (rank + 1) + [wl.n] * (world - rank)
        sb, se = bounds[rank], bounds[rank + 1]
        mb = MatchBatch(eng)
        wl.fill(mb, sb, se)
        mb.set_package_base(sb)
        n_local = len(mb)
        assert n_local == se - sb
        total, errp, bits = mb.run()
        if bits or errp != -1:
            raise RuntimeError(f"engine error bits={bits} poisoned_pkg={errp}")
        gather, csr = None, None
        if world > 1 and strong:  # the order kernel writes this rank's per-package lists (CSR) into the tensors the gather sends
            csr = (torch.empty(max(total, 1), dtype=torch.int32, device=gdev),
                   torch.empty(max(n_local, 1), dtype=torch.int32, device=gdev))
            gather = td.CSRGather(cdev)
        log(rank, f"[bench] {'strong' if strong else 'weak'}: shard {sb}..{se} of {wl.n}: {n_local} packages, "
                  f"{total} matches, {int(rows[sb:se].sum())} predicted rows ({time.perf_counter()-t0:.1f}s)")

        if primary and args.sweep and rank == 0:
            names, v = [], 0
            while lib().tvm_variant_name(v):
                names.append(lib().tvm_variant_name(v).decode())
                v += 1
            times = {n: [] for n in names}
            for _ in range(args.sweep):
                for v, n in enumerate(names):
                    lib().tvm_engine_set_variant(eng.h, v)
                    try:
                        mb.launch(2)
                    except RuntimeError as e:  # a variant not built for this batch's grammar set
                        if "is not built" not in str(e):
                            raise
                        times.pop(n, None)
                        continue
                    times[n].append(mb.time(10))
                    if not n.startswith("diag") and mb.status() != (total, -1, 0):
                        raise RuntimeError(f"variant {n} disagrees on the match count")
            for n in names:
                if n not in times:
                    continue
                t = sorted(times[n])
                log(rank, f"[sweep] {n:>16}: median {t[len(t)//2]:.4f} ms  min {t[0]:.4f} ms per pass")
        lib().tvm_engine_set_variant(eng.h, args.variant if args.variant is not None else 0)
        if primary and args.sweep:
            mb.launch(1)  # the diagnostics left wrong counts behind

        def do_gather():
            mb.order_into(*csr)  # per-package lists in batch order on this rank's GPU (synchronised)
            if backend == "nccl":
                return gather(csr[0], csr[1], total, n_local)
            # gloo rehearsal: through host memory
            return gather(csr[0][:total].cpu(), csr[1][:n_local].cpu(), total, n_local)

        # ---- timed region: match pass (+ gather to rank 0) -----------------------------------
        def step():
            # passes queue back to back on the engine stream (each a full pass over the resident
            # batch, its list overwriting the last one's); the timed region's closing sync waits
            # for the last; the strong step's order kernel + gather are stream-ordered behind it
            mb.launch(1, sync=False)
            if gather is not None:
                do_gather()

        def step_sync():  # the engine stream (libtrivy_amd's HIP runtime), then torch's
            mb.launch(0, sync=True)
            sync()

        wall = td.timed(step, steps=args.steps, warmup=args.warmup, sync=step_sync, device=cdev)
        if mb.status() != (total, -1, 0):
            raise RuntimeError("timed passes disagree with the first pass")
        n_job = wl.n * (1 if strong else world)  # packages all ranks match per step
        out = {"mb": mb, "total": total, "n_local": n_local, "sb": sb, "se": se, "wall": wall, "n_job": n_job,
               "value": n_job * args.steps / wall, "gather_ms": None}
        if gather is not None:
            sync()
            g0 = time.perf_counter()
            for _ in range(args.steps):
                do_gather()
            sync()
            out["gather_ms"] = td.max_over_ranks(time.perf_counter() - g0, cdev) * 1e3 / args.steps
        if args.dump_csr:  # the lists as the timed step leaves them at rank 0, for the parity test
            adv = rend = None
            if gather is not None:
                got = do_gather()
                if rank == 0:
                    adv, rend = (t.cpu().numpy().astype(np.uint32) for t in got)
            else:
                pr = mb.pairs()
                adv = pr[:, 1].astype(np.uint32)
                rend = np.cumsum(np.bincount(pr[:, 0] - sb, minlength=n_local)).astype(np.uint32)
            if rank == 0:
                path = args.dump_csr if primary else args.dump_csr.replace(".npz", "_strong.npz")
                np.savez(path, adv=adv, row_end=rend, n_gpus=world)
        return out

    main_run = measure(args.gather, True)
    mb, total, n_local, sb = main_run["mb"], main_run["total"], main_run["n_local"], main_run["sb"]
    wall, n_job, value, gather_ms = main_run["wall"], main_run["n_job"], main_run["value"], main_run["gather_ms"]
    vname = lib().tvm_variant_name(lib().tvm_engine_last_variant(eng.h)).decode()
    # kernel-only time of this rank's pass (HIP events on the engine stream) for the roofline
    kernel_ms = mb.time(args.steps)
    alg_bytes = mb.algorithmic_bytes()
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
    # the batch's DetectedVulnerability set (tvm_match_vulns: the drivers' epilogues over every
    # match; Red Hat batches merged per CVE on the device first), host time of the export
    vulns = None
    if rank == 0:
        t_v = time.perf_counter()
        vs = mb.vulns()  # the first export builds the per-advisory records (once per DB)
        first_ms = (time.perf_counter() - t_v) * 1e3
        vs.close()
        vms = []
        for _ in range(3):
            mb.launch(1)
            vs = mb.vulns()
            vms.append(vs.ms)
            n_v, n_grp = len(vs), vs.n_grp_recs
            vs.close()
        vulns = {"ms": sorted(vms)[1], "detected_vulnerabilities": n_v, "merged_group_records": n_grp,
                 "first_call_ms": first_ms,
                 "is": "tvm_match_vulns after a device-resident pass: (Red Hat per-CVE merge, group records of "
                       "several members flagged, scanned and gathered on the device,) the per-package record lists "
                       "written into pinned host memory by the result move (3-byte indices), the merged groups' "
                       "records on the host threads; per-advisory records built once per DB on the first call "
                       "(first_call_ms)"}
        mb.launch(1)
    strong = None
    if world > 1 and not args.gather:  # north_star's multi-GPU path: one global batch, lists gathered at rank 0
        sr = measure(True, False)
        strong = {"packages_per_s": sr["value"], "ms_per_step": sr["wall"] * 1e3 / args.steps,
                  "gather_ms": sr["gather_ms"], "packages": wl.n, "packages_rank0": sr["n_local"],
                  "matches_rank0": sr["total"],
                  "step": "match pass of this rank's shard + order kernel + exact-size CSR gather to rank 0 (RCCL) "
                          "in global batch order"}
        sr["mb"].close()

    # ---- end-to-end pipelined pass over PCIe (N = 1) -------------------------------------------
    # the host batch in, the DetectedVulnerability set out and consumed: one pipelined pass
    # (upload, match, per-package lists in pinned host memory) + tvm_pipeline_vulns over the
    # result as it arrived (Red Hat batches: the per-CVE merge and the export over the pass's
    # list, still in HBM) + tvm_vuln_set_walk, a native consumer that decodes every record
    # index and reads its record and its package's InstalledVersion (INTEGRATION.md §3's loop)
    e2e = None

    def vulns_and_consume(m):
        vs = m.vulns(pipeline=True)
        t_c = time.perf_counter()
        n_w, dig = vs.walk()
        c_ms = (time.perf_counter() - t_c) * 1e3
        if n_w != len(vs):
            raise RuntimeError("the consumer walked another number of DetectedVulnerabilities than the set holds")
        out = (vs.ms, c_ms, len(vs), vs.n_grp_recs)
        vs.close()
        return out

    if world == 1 and not args.no_e2e and rank == 0:
        mp = MatchBatch(eng)
        wl.fill(mp)
        mp.pipeline_prepare(match_cap=total, chunk_packages=args.chunk)
        for _ in range(max(1, args.warmup)):
            mp.pipeline_run()
            vulns_and_consume(mp)
        npass = max(3, args.steps // 4)
        runs = []
        for _ in range(npass):
            got, ep, m = mp.pipeline_run()
            if got != total or ep != -1:
                raise RuntimeError("end-to-end pass disagrees with the device-resident pass")
            v_ms, c_ms, n_dv, n_grp = vulns_and_consume(mp)
            runs.append((m + v_ms + c_ms, m, v_ms, c_ms))
        runs.sort(key=lambda r: r[0])
        both, med, v_ms, c_ms = runs[len(runs) // 2]
        st = mp.pipeline_stats()
        e2e = {"packages_per_s": wl.n / (both / 1e3), "ms": both, "pass_ms": med, "vulns_ms": v_ms,
               "consume_ms": c_ms, "pass_packages_per_s": wl.n / (med / 1e3), "passes": npass,
               "detected_vulnerabilities": n_dv, "merged_group_records": n_grp,
               "result_form": "CSR, 3-byte advisory indices + row ends in pinned host memory",
               "h2d_bytes": st["h2d_bytes"], "d2h_bytes": st["d2h_bytes"], "chunks": st["chunks"],
               "pcie_GBs": (st["h2d_bytes"] + st["d2h_bytes"]) / (med / 1e3) / 1e9,
               "transport_form": st["transport_form"], "prepare_encode_ms": st["encode_ms"],
               "inside": "H2D of the batch from pinned host memory (its transport form: each distinct name / "
                         "version string once + per-package references, one DMA per chunk) + the kernel that "
                         "rebuilds each chunk in HBM + match kernels + the per-package advisory lists (CSR) "
                         "written into pinned host memory by the next launch's first workgroups (pass_ms) + "
                         "tvm_pipeline_vulns, the DetectedVulnerability set (vulns_ms: the lists as they arrived; "
                         "batches with Red Hat packages: the per-CVE merge + export over the pass's list in HBM and "
                         "the merged groups' records) + tvm_vuln_set_walk on the host threads, every "
                         "DetectedVulnerability's record index decoded, its record and its package's "
                         "InstalledVersion read (consume_ms)",
               "prepare_ms": st["prepare_ms"],
               "outside": "prepare (once per batch: sizing, building the transport form on the host threads "
                          "(prepare_encode_ms); the batch is re-run, see fresh_batch for batches seen once)"}
        mp.close()

    # ---- fresh batches: each batch built, prepared and matched once (a fleet scan's steady state) ----
    fresh = None
    if world == 1 and not args.no_e2e and rank == 0:
        runs = []
        for _ in range(6):  # the first warms the block cache (pool.h); the median of the rest is reported
            tb = time.perf_counter()
            mf = MatchBatch(eng)
            wl.fill(mf)
            tp = time.perf_counter()
            mf.pipeline_prepare(match_cap=total, chunk_packages=args.chunk, raw=True)
            tr = time.perf_counter()
            got, ep, _ = mf.pipeline_run()  # the result: the CSR in pinned host memory (3-byte indices)
            te = time.perf_counter()
            if got != total or ep != -1:
                raise RuntimeError("fresh-batch pass disagrees with the device-resident pass")
            v_ms, c_ms, _, _ = vulns_and_consume(mf)
            st = mf.pipeline_stats()
            runs.append({"build_ms": (tp - tb) * 1e3, "prepare_ms": (tr - tp) * 1e3, "pass_ms": (te - tr) * 1e3,
                         "vulns_ms": v_ms, "consume_ms": c_ms, "h2d_bytes": st["h2d_bytes"],
                         "d2h_bytes": st["d2h_bytes"]})
            mf.close()
        steady = sorted(runs[1:], key=lambda r: r["prepare_ms"] + r["pass_ms"] + r["vulns_ms"] + r["consume_ms"])
        med = steady[len(steady) // 2]
        inner = med["prepare_ms"] + med["pass_ms"] + med["vulns_ms"] + med["consume_ms"]
        fresh = dict(med, packages_per_s=wl.n / (inner / 1e3),
                     packages_per_s_with_build=wl.n / ((inner + med["build_ms"]) / 1e3), batches=len(runs),
                     form="raw (pinned staging copy on the host threads; no per-batch string dedup)",
                     inside="prepare (freeze, size, pinned staging copy, buffers from the block cache) + one "
                            "pipelined pass (upload, match, per-package advisory lists back in pinned host memory "
                            "as the CSR: 3-byte indices + row ends) + tvm_pipeline_vulns (vulns_ms) + "
                            "tvm_vuln_set_walk (consume_ms)",
                     build=wl.build_how,
                     outside="build_ms (in packages_per_s_with_build only): the caller adding the batch's packages")

    fill = None
    if rank == 0 and wl.has_vulns and world == 1:
        # Red Hat batches: the driver's per-CVE merge (redhat.go:146-187) on the device, then
        # FillInfo and result.Filter over the MERGED list - the reference's order of work
        mb.launch(1)
        merge_ms = None
        if "Red Hat" in wl.plats:
            merge_ms = mb.redhat_merge_time(args.steps)
        # FillInfo (vulnerability.go:60-157) fused behind the match list: timed apart, on the
        # same stream, over the same device-resident match list (DESIGN.md "FillInfo")
        fill_ms = mb.fill_time(args.steps)
        fill_bytes = mb.fill_algorithmic_bytes()
        fill_gbs = fill_bytes / (fill_ms / 1e3) / 1e9
        n_list = mb.status()[0]  # the merged list's length when the batch has Red Hat packages
        fill = {"kernel_ms": fill_ms, "matches_per_s": total / (fill_ms / 1e3), "pairs_filled": n_list,
                "algorithmic_bytes_per_launch": fill_bytes, "achieved_GBs": fill_gbs,
                "frac": fill_gbs / HBM_PEAK_GBS, "db_vulnerabilities": len(wl.vuln_ids())}
        # result.Filter (filter.go:60-139) behind FillInfo: default options (every severity),
        # per result dedup + BySeverity order; wall time per call incl. its one sync
        mb.fill()
        fopts = mb.filter_opts()
        kept = mb.filter(fopts)
        filt_ms = mb.filter_time(fopts, max(3, args.steps // 4))
        fill["result_filter"] = {"ms": filt_ms, "kept": kept, "matches_per_s": total / (filt_ms / 1e3)}
        if merge_ms is not None:
            fill["redhat_merge"] = {"kernel_ms": merge_ms, "raw_pairs": total, "merged_pairs": n_list,
                                    "note": "FillInfo / result.Filter above run over the merged list"}
        # + a VEX document's suppressions (filterByVEX, filter.go:38-104): 1% of the findings,
        # sampled from the match list, as the host compile (trivy_amd/vex.py) would emit them
        pr = mb.pairs()
        pick = np.random.default_rng(5).choice(len(pr), size=max(1, len(pr) // 100), replace=False)
        vex = (pr[pick, 0] - sb, [wl.adv_vuln_id(db, a) for a in pr[pick, 1].tolist()])
        vopts = mb.filter_opts(vex=vex)
        vkept = mb.filter(vopts)
        vex_ms = mb.filter_time(vopts, max(3, args.steps // 4))
        fill["result_filter"]["vex"] = {"suppressions": len(pick), "ms": vex_ms, "kept": vkept,
                                        "matches_per_s": total / (vex_ms / 1e3)}

    dropin = None
    if not args.no_dropin and args.config == "c2" and rank == 0 and world == 1:
        # C1-shaped request through the drop-in per-target path (debian Scanner.Detect,
        # debian.go:57-119): 100 packages of one Debian 12 image, through the C-ABI alone
        import ctypes
        from trivy_amd import _lib as L
        from trivy_amd.detector import ospkg as osp
        p12 = wl.plats.index("debian 12")
        b0, b1 = next((b0, b1) for p, b0, b1 in wl.batch.targets if p == p12 and b1 - b0 >= 100)
        pk = [{"Name": wl.batch.names[i].decode(), "SrcName": wl.batch.names[i].decode(),
               "Version": wl.batch.versions[i].decode(), "SrcVersion": wl.batch.versions[i].decode()}
              for i in range(b0, b0 + 100)]
        arr, _keep = osp._pkg_array(pk)
        res, ebuf, now = L.Result(), L.errbuf(), osp._now(None)
        n_calls, found, lat = 400, 0, []
        for _ in range(n_calls):
            t_c = time.perf_counter()
            if lib().tvm_ospkg_driver_detect(eng.h, b"debian", b"12", None, arr, len(pk), now, ctypes.byref(res), ebuf,
                                             len(ebuf)):
                raise RuntimeError(ebuf.value.decode())
            found = res.n
            lib().tvm_result_free(ctypes.byref(res))
            lat.append((time.perf_counter() - t_c) * 1e3)
        lat = sorted(lat[20:])  # the first calls grow the drop-in buffers
        c_ms = sum(lat) / len(lat)
        # the same call from 8 threads at once (a twirp server / k8s worker pool): the engine
        # coalesces the queued calls into shared launches (tvm_engine_dropin_stats)
        import threading
        st0 = (ctypes.c_uint64 * 3)()
        lib().tvm_engine_dropin_stats(eng.h, st0)
        n_thr, per_thr, fails = 8, 200, []

        def caller():
            r2, e2 = L.Result(), L.errbuf()
            for _ in range(per_thr):
                if lib().tvm_ospkg_driver_detect(eng.h, b"debian", b"12", None, arr, len(pk), now, ctypes.byref(r2),
                                                 e2, len(e2)):
                    fails.append(e2.value.decode())
                    return
                if r2.n != found:
                    fails.append(f"{r2.n} != {found} vulnerabilities")
                lib().tvm_result_free(ctypes.byref(r2))
        ths = [threading.Thread(target=caller) for _ in range(n_thr)]
        t_c = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        conc_s = time.perf_counter() - t_c
        if fails:
            raise RuntimeError(f"concurrent drop-in calls: {fails[:3]}")
        st1 = (ctypes.c_uint64 * 3)()
        lib().tvm_engine_dropin_stats(eng.h, st1)
        dropin = {"workload": "c1-shaped: 100 debian-12 packages per call (tvm_ospkg_driver_detect: debian "
                              "Scanner.Detect, debian.go:57-119)", "c_abi_ms_per_call": c_ms,
                  "p50_ms": lat[len(lat) // 2], "p99_ms": lat[int(len(lat) * 0.99)],
                  "vulnerabilities_per_call": found,
                  "concurrent": {"threads": n_thr, "calls": n_thr * per_thr,
                                 "calls_per_s": n_thr * per_thr / conc_s, "launches": st1[0] - st0[0],
                                 "calls_sharing_a_launch": st1[2] - st0[2]}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # the box's CPU share: OMP_NUM_THREADS is set to it there (os.cpu_count() shows the
        # whole machine, whose other cores belong to other jobs)
        threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", 0) or 0) or os.cpu_count() or 1
        cpu = wl.cpu_baseline(args.cpu_seconds, threads)

    src_hash = kernel_source_hash()
    traffic, traffic_src = pmc_traffic(args.config, wl.name, vname, src_hash)
    if rank == 0:
        if args.gather:
            par = f"dp{world}: tables replicated, one global batch sharded x{world} on target boundaries by predicted rows"
            if world > 1:
                par += (", per-rank order kernel (per-package lists, CSR) + exact-size CSR gather to rank 0 in "
                        "global batch order inside the timed step")
        else:
            par = (f"dp{world}: tables replicated, every rank matches its own {wl.n}-package batch of the config "
                   "(packages are independent: no collective in the step)")
        line = {
            "metric": "packages matched/sec (node)",
            "value": value,
            "unit": "packages/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if args.gather else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded trivy-db + SBOM batch, tools/synth.py / tools/synth_mix.py)",
            "config": {"workload": wl.name, "packages": wl.n, "packages_per_step": n_job, "packages_rank0": n_local,
                       "matches_rank0": total,
                       "kernel_variant": vname, "kernel_source": src_hash, "db_keys": wl.n_keys, "db_advisories": wl.n_adv,
                       "platforms": wl.plats, "parallelism": par, "hip_runtime": trivy_amd.runtime_info()},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_from": traffic_src,
                         "algorithmic_bytes_per_launch": alg_bytes, "kernel_ms": kernel_ms,
                         "achieved_is": "algorithmic bytes (SURVEY §8d, no cache-reuse credit) / kernel time"},
            "cpu_baseline": cpu,
        }
        if gather_ms is not None:
            line["gather_ms"] = gather_ms
        if strong is not None:
            line["strong"] = strong
        if vulns is not None:
            line["vulns"] = vulns
        if e2e is not None:
            line["end_to_end"] = e2e
        if fresh is not None:
            line["fresh_batch"] = fresh
        if fill is not None:
            line["fill_info"] = fill
        if dropin is not None:
            line["dropin_latency"] = dropin
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
