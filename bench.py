#!/usr/bin/env python3
"""Benchmark: packages matched/sec on BASELINE.json config C2 (dpkg, ~4M packages).

BASELINE.json metric: "packages matched/sec (node) at 1/2/4/8 GPUs; probe HBM GB/s vs peak".
Workload (config[1]): 10k synthetic Debian/Ubuntu image SBOMs x 400 packages = 4M packages,
Debian:Ubuntu 60:40 (debian 11/12, ubuntu 20.04/22.04/24.04), against a seeded synthetic
trivy-db of 5 x 30k package keys (~1.7M advisories, heavy-tailed, 15% unfixed).  The pinned
trivy-db cannot be fetched offline, hence synthetic data (tools/synth.py).

One step = one pass of the match kernel over the whole device-resident batch: packages
(descriptors + name/version bytes) in HBM -> (package, advisory) match list in HBM.
Weak scaling: every rank matches its own 4M-package batch against its own replica of the
tables; no collective on the data path.  value = all ranks' packages x steps / max wall.

Also reported: roofline (algorithmic bytes per launch / HIP-event launch time, vs the
8 TB/s HBM peak), the oracle CPU baseline on a bounded sample (rank 0, N=1 only), and
traffic from the committed rocprofv3 PMC summary when one matches this config.
"""
import argparse
import ctypes
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


def build_engine(sdb, device):
    import trivy_amd
    from trivy_amd._lib import lib
    db = trivy_amd.DB()
    for n, depth, arena, off, lens in (sdb.records_arena(), sdb.source_arena()):
        if lib().tvm_db_put_arena(db.h, n, depth, arena, off.ctypes.data, lens.ctypes.data):
            raise RuntimeError("tvm_db_put_arena failed")
    db.finalize()
    return trivy_amd.Engine(db, device)


def upload_batch(eng, sdb, batch, cap):
    from trivy_amd._lib import lib, errbuf
    L = lib()
    b = L.tvm_batch_new()
    arena, noff, nlen, voff, vlen = batch.arena()
    for p, b0, b1 in batch.targets:
        L.tvm_batch_add_many(b, eng.h, sdb.platforms[p].encode(), b1 - b0, arena, noff[b0:].ctypes.data,
                             nlen[b0:].ctypes.data, voff[b0:].ctypes.data, vlen[b0:].ctypes.data)
    e = errbuf()
    if L.tvm_batch_upload(eng.h, b, cap, e, len(e)):
        raise RuntimeError(e.value.decode())
    return b


def status(eng, b):
    from trivy_amd._lib import lib
    n, errp, bits = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_uint64()
    lib().tvm_match_status(eng.h, b, ctypes.byref(n), ctypes.byref(errp), ctypes.byref(bits))
    return n.value, errp.value, bits.value


def launch(eng, b, k=1):
    from trivy_amd._lib import lib, errbuf
    e = errbuf()
    for _ in range(k):
        if lib().tvm_match_launch(eng.h, b, e, len(e)):
            raise RuntimeError(e.value.decode())
    if lib().tvm_engine_sync(eng.h, e, len(e)):
        raise RuntimeError(e.value.decode())


def cpu_baseline(sdb, batch, budget_s, threads):
    """Oracle (C restatement of the reference loops, 'port') on a bounded sample."""
    from oracle import match as om
    from tools.synth import SynthBatch
    n_total = len(batch)
    n = min(n_total, 200_000)
    while True:
        sub = SynthBatch(batch.plat[:n], batch.names[:n], batch.versions[:n], [])
        prep = om.Prepared(sdb, sub)
        t = time.perf_counter()
        om.match(prep, n_threads=threads)
        dt = time.perf_counter() - t
        if dt >= budget_s * 0.5 or n == n_total:
            return n / dt, n, dt
        n = min(n_total, int(n * max(2.0, budget_s / max(dt, 1e-3))))


def pmc_traffic(cfg_name):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, when it matches."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    if d.get("workload") != cfg_name:
        return None
    return d.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--keys-per-plat", type=int, default=30000)
    ap.add_argument("--targets", type=int, default=10000)
    ap.add_argument("--pkgs-per-target", type=int, default=400)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify the bench batch against the oracle")
    ap.add_argument("--gather", action="store_true",
                    help="after the timed region, gather all match lists to rank 0 (RCCL), reported apart")
    ap.add_argument("--variant", type=int, default=None, help="match-kernel variant (tvm_engine_set_variant)")
    ap.add_argument("--sweep", type=int, default=0,
                    help="time every kernel variant over N interleaved rounds (stderr table) before the bench")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)

    from tools.synth import make_db, make_batch
    t0 = time.perf_counter()
    sdb = make_db(PLATS, args.keys_per_plat)
    eng = build_engine(sdb, local)
    log(rank, f"[bench] db: {len(sdb.key_names)} keys, {sdb.n_adv} advisories, tables {eng.table_bytes()/1e6:.1f} MB "
              f"({time.perf_counter()-t0:.1f}s)")
    t0 = time.perf_counter()
    batch = make_batch(sdb, args.targets, args.pkgs_per_target, WEIGHTS, seed=2 + 1000 * rank)
    n_pkgs = len(batch)
    b = upload_batch(eng, sdb, batch, cap=8 * n_pkgs)
    launch(eng, b)
    total, errp, bits = status(eng, b)
    if total > 8 * n_pkgs:  # size the match buffer exactly, once
        from trivy_amd._lib import lib
        lib().tvm_batch_free(b)
        b = upload_batch(eng, sdb, batch, cap=total)
        launch(eng, b)
        total, errp, bits = status(eng, b)
    if bits or errp != -1:
        raise RuntimeError(f"engine error bits={bits} poisoned_pkg={errp}")
    log(rank, f"[bench] batch: {n_pkgs} packages, {total} matches ({time.perf_counter()-t0:.1f}s)")

    if args.check and rank == 0:
        from oracle import match as om
        from trivy_amd._lib import lib
        out = np.zeros(2 * total, dtype=np.uint32)
        got = ctypes.c_uint64()
        if lib().tvm_match_fetch(eng.h, b, out.ctypes.data, total, ctypes.byref(got)):
            raise RuntimeError("tvm_match_fetch failed")
        opk, oad = om.match(om.Prepared(sdb, batch), n_threads=args.cpu_threads)
        pr = out.reshape(-1, 2)
        ok = np.array_equal(pr[:, 0], opk) and np.array_equal(pr[:, 1], oad)
        log(rank, f"[bench] check vs oracle: {'OK' if ok else 'MISMATCH'}")
        if not ok:
            raise SystemExit(1)

    # ---- warmup + timed region -------------------------------------------------------------
    from trivy_amd._lib import lib, errbuf
    if args.sweep and rank == 0:
        names, v = [], 0
        while lib().tvm_variant_name(v):
            names.append(lib().tvm_variant_name(v).decode())
            v += 1
        times = {n: [] for n in names}
        for _ in range(args.sweep):
            for v, n in enumerate(names):
                lib().tvm_engine_set_variant(eng.h, v)
                launch(eng, b, 2)
                ms = ctypes.c_double()
                e = errbuf()
                lib().tvm_match_time(eng.h, b, 10, ctypes.byref(ms), e, len(e))
                times[n].append(ms.value / 10)
                if not n.startswith("ablate") and status(eng, b) != (total, -1, 0):
                    raise RuntimeError(f"variant {n} disagrees on the match count")
        for n in names:
            t = sorted(times[n])
            log(rank, f"[sweep] {n:>16}: median {t[len(t)//2]:.4f} ms  min {t[0]:.4f} ms per pass")
    lib().tvm_engine_set_variant(eng.h, args.variant if args.variant is not None else 0)
    launch(eng, b, args.warmup)

    from trivy_amd import dist as td
    ms = ctypes.c_double()
    e = errbuf()

    def timed_region():
        if lib().tvm_match_time(eng.h, b, args.steps, ctypes.byref(ms), e, len(e)):
            raise RuntimeError(e.value.decode())

    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    dev = f"cuda:{local}" if torch.cuda.is_available() else "cpu"
    wall = td.timed(timed_region, steps=1, warmup=0, sync=sync, device=dev)
    total2, errp2, bits2 = status(eng, b)
    if (total2, errp2, bits2) != (total, -1, 0):
        raise RuntimeError("timed launches disagree with the first pass")

    gather = None
    if args.gather:  # optional RCCL gather of every rank's match list to rank 0, timed apart
        pairs = torch.empty((total, 2), dtype=torch.int32, device=dev)
        got = ctypes.c_uint64()
        if lib().tvm_match_copy_device(eng.h, b, pairs.data_ptr(), total, ctypes.byref(got)) or got.value != total:
            raise RuntimeError("tvm_match_copy_device failed")
        g0 = time.perf_counter()
        merged = td.gather_pairs(pairs, rank * n_pkgs)
        sync()
        g_wall = td.max_over_ranks(time.perf_counter() - g0, dev)
        gather = {"ms": g_wall * 1e3, "pairs_on_root": None if merged is None else int(merged.shape[0]),
                  "bytes_per_rank": total * 16}

    value = world * n_pkgs * args.steps / wall
    launch_s = ms.value / 1e3 / args.steps
    alg_bytes = lib().tvm_match_algorithmic_bytes(eng.h, b)
    achieved = alg_bytes / launch_s / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        rate, n_sample, dt = cpu_baseline(sdb, batch, args.cpu_seconds, args.cpu_threads)
        cpu = {"value": rate, "unit": "packages/s", "cores": args.cpu_threads, "kind": "port",
               "sample": f"first {n_sample} packages of the same batch, oracle/match.c orc_match with "
                         f"{args.cpu_threads} threads, {dt:.1f}s"}

    cfg_name = f"c2-dpkg-{args.targets}x{args.pkgs_per_target}"
    traffic = pmc_traffic(cfg_name)
    if rank == 0:
        line = {
            "metric": "packages matched/sec (node)",
            "value": value,
            "unit": "packages/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded trivy-db + SBOM batch, tools/synth.py)",
            "config": {"workload": cfg_name, "packages_per_gpu": n_pkgs, "matches_per_gpu": total,
                       "kernel_variant": lib().tvm_variant_name(lib().tvm_engine_set_variant(eng.h, -1)).decode(),
                       "db_keys": len(sdb.key_names), "db_advisories": sdb.n_adv,
                       "platforms": PLATS, "parallelism": f"replicated tables, batch sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "algorithmic_bytes_per_launch": alg_bytes,
                         "kernel_ms": launch_s * 1e3},
            "cpu_baseline": cpu,
        }
        if gather is not None:
            line["gather"] = gather
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
