#!/usr/bin/env python3
"""Benchmark: packages matched/sec on BASELINE.json config C2 (dpkg, ~4M packages).

BASELINE.json metric: "packages matched/sec (node) at 1/2/4/8 GPUs; probe HBM GB/s vs peak".
Workload (config[1], the default): 10k synthetic Debian/Ubuntu image SBOMs x 400 packages =
4M packages, Debian:Ubuntu 60:40 (debian 11/12, ubuntu 20.04/22.04/24.04), against a seeded
synthetic trivy-db of 5 x 30k package keys (~1.7M advisories, heavy-tailed, 15% unfixed).
The pinned trivy-db cannot be fetched offline, hence synthetic data (tools/synth.py).
--config c3 / c5 run the language-package (1M npm/pip/maven/go) and RHEL-family/Alpine
(rpm + apk) mixes of tools/synth_mix.py instead - extra measurements, not the headline.

One step = one pass of the match kernel over the whole device-resident batch: packages
(descriptors + name/version bytes) in HBM -> (package, advisory) match list in HBM.
Weak scaling: every rank matches its own batch against its own replica of the tables; no
collective on the data path.  value = all ranks' packages x steps / max-over-ranks wall.
--gather additionally gathers every rank's match list to rank 0 over RCCL after the timed
region and reports that time apart.

Also reported: roofline (algorithmic bytes per launch / HIP-event launch time, vs the
8 TB/s HBM peak), the oracle CPU baseline on a bounded sample (rank 0, N=1 only), and
traffic from the committed rocprofv3 PMC summary when one matches this config.
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


# ---- workloads ----------------------------------------------------------------------------
class C2:
    """dpkg fleet (tools/synth.py); the oracle C port (oracle/match.c) is the CPU baseline."""

    def __init__(self, args, rank):
        from tools.synth import make_db, make_batch
        self.sdb = make_db(PLATS, args.keys_per_plat)
        self.batch = make_batch(self.sdb, args.targets, args.pkgs_per_target, WEIGHTS, seed=2 + 1000 * rank)
        self.name = f"c2-dpkg-{args.targets}x{args.pkgs_per_target}"
        self.n_adv = self.sdb.n_adv
        self.n_keys = len(self.sdb.key_names)
        self.plats = PLATS

    def load(self, db, vulns=True):
        from tools.synth_vuln import vuln_arena
        parts = [self.sdb.records_arena(detail=vulns), self.sdb.source_arena()]
        if vulns:  # bucket "vulnerability" for the FillInfo leg (tools/synth_vuln.py)
            parts.append(vuln_arena(self.sdb.vuln_ids()))
        self.has_vulns = vulns
        for n, depth, arena, off, lens in parts:
            db.put_arena(n, depth, arena, off, lens)

    def fill(self, mb):
        arena, noff, nlen, voff, vlen = self.batch.arena()
        for p, b0, b1 in self.batch.targets:
            mb.add_arena(self.sdb.platforms[p], b1 - b0, arena, noff[b0:], nlen[b0:], voff[b0:], vlen[b0:])

    def cpu_baseline(self, budget_s, threads):
        from oracle import match as om
        from tools.synth import SynthBatch
        batch = self.batch
        n_total = len(batch)
        n = min(n_total, 200_000)
        while True:
            sub = SynthBatch(batch.plat[:n], batch.names[:n], batch.versions[:n], [])
            prep = om.Prepared(self.sdb, sub)
            t = time.perf_counter()
            om.match(prep, n_threads=threads)
            dt = time.perf_counter() - t
            if dt >= budget_s * 0.5 or n == n_total:
                return {"value": n / dt, "unit": "packages/s", "cores": threads, "kind": "port",
                        "sample": f"first {n} packages of the same batch, oracle/match.c orc_match with "
                                  f"{threads} threads, {dt:.1f}s"}
            n = min(n_total, int(n * max(2.0, budget_s / max(dt, 1e-3))))


class Mix:
    """C3 (language packages) / C5 (rpm + apk) mixes of tools/synth_mix.py; the CPU baseline
    is the Python oracle drivers on a bounded sample (1 core)."""

    def __init__(self, args, rank, which):
        from tools import synth_mix as sm
        self.sm = sm
        plats, self.weights, kpp, n = {
            "c3": (sm.C3_PLATS, sm.C3_WEIGHTS, 25_000, 1_000_000),
            "c5": (sm.C5_PLATS, sm.C5_WEIGHTS, 12_000, 20_000_000)}[which]
        n = args.packages or n
        self.sdb = sm.make_mix_db(plats, kpp)
        self.batch = sm.make_mix_batch(self.sdb, n, self.weights, seed=2 + 1000 * rank)
        self.name = f"{which}-{'lang' if which == 'c3' else 'rpm-apk'}-{n}"
        self.n_adv = self.sdb.n_adv
        self.n_keys = len(self.sdb.keys)
        self.plats = [b for b, _ in plats]

    def load(self, db):
        self.sdb.put(db)

    def fill(self, mb):
        self.sm.add_to(mb, self.sdb, self.batch)

    def cpu_baseline(self, budget_s, threads):
        import oracle.drivers as od
        import oracle.library as ol
        sm = self.sm
        per, n_done, dt = 200, 0, 0.0
        while dt < budget_s:
            for p, g in self.batch.groups:
                bucket, kind = self.sdb.plats[p]
                idx = np.arange(min(per, len(g["key"])))
                pkgs = sm.driver_packages(self.sdb, p, g, idx)
                roots = sm.C3_ROOTS.get(kind, [bucket])
                recs = od.Records(self.sdb.records_for({r: {x["Name"] for x in pkgs} for r in roots}))
                t = time.perf_counter()
                if kind in sm.LANG_OF:
                    ol.detect(recs, sm.LANG_OF[kind], pkgs)
                else:
                    fam, fmt = sm.DRIVER_OF[kind]
                    od.driver_detect(fam, fmt.format(bucket.split(" ")[-1]), None, pkgs, recs, None)
                dt += time.perf_counter() - t
                n_done += len(idx)
            per *= 2
        return {"value": n_done / dt, "unit": "packages/s", "cores": 1, "kind": "port",
                "sample": f"{n_done} packages (first rows of every platform group), oracle/drivers.py + "
                          f"oracle/library.py per-driver Detect, 1 thread, {dt:.1f}s (Python)"}


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
    ap.add_argument("--config", choices=["c2", "c3", "c5"], default="c2")
    ap.add_argument("--keys-per-plat", type=int, default=30000)
    ap.add_argument("--targets", type=int, default=10000)
    ap.add_argument("--pkgs-per-target", type=int, default=400)
    ap.add_argument("--packages", type=int, default=0, help="c3/c5: packages per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-fill", action="store_true", help="c2: skip the FillInfo leg (no vulnerability bucket)")
    ap.add_argument("--dropin", action="store_true",
                    help="c2: also time 100-package requests through the per-target driver path (off by default: "
                         "its many tiny match launches would mix into a kernel-trace average of this command)")
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
    # TVM_BENCH_BACKEND=gloo rehearses the N>1 path on a box with fewer GPUs than ranks
    # (ranks then share devices round-robin); the scaling runs use RCCL, one rank per GPU
    backend = os.environ.get("TVM_BENCH_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend)
    if torch.cuda.is_available():
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)

    import trivy_amd
    from trivy_amd import dist as td
    from trivy_amd._lib import lib
    from trivy_amd.batch import MatchBatch
    t0 = time.perf_counter()
    wl = C2(args, rank) if args.config == "c2" else Mix(args, rank, args.config)
    db = trivy_amd.DB()
    if args.config == "c2":
        wl.load(db, vulns=not args.no_fill)
    else:
        wl.load(db)
    eng = trivy_amd.Engine(db.finalize(), local)
    log(rank, f"[bench] {wl.name}: db {wl.n_keys} keys, {wl.n_adv} advisories, tables "
              f"{eng.table_bytes()/1e6:.1f} MB ({time.perf_counter()-t0:.1f}s)")
    t0 = time.perf_counter()
    mb = MatchBatch(eng)
    wl.fill(mb)
    n_pkgs = len(mb)
    total, errp, bits = mb.run()
    if bits or errp != -1:
        raise RuntimeError(f"engine error bits={bits} poisoned_pkg={errp}")
    log(rank, f"[bench] batch: {n_pkgs} packages, {total} matches ({time.perf_counter()-t0:.1f}s)")

    # ---- warmup + timed region -------------------------------------------------------------
    if args.sweep and rank == 0:
        names, v = [], 0
        while lib().tvm_variant_name(v):
            names.append(lib().tvm_variant_name(v).decode())
            v += 1
        times = {n: [] for n in names}
        for _ in range(args.sweep):
            for v, n in enumerate(names):
                lib().tvm_engine_set_variant(eng.h, v)
                mb.launch(2)
                times[n].append(mb.time(10))
                if not n.startswith("ablate") and mb.status() != (total, -1, 0):
                    raise RuntimeError(f"variant {n} disagrees on the match count")
        for n in names:
            t = sorted(times[n])
            log(rank, f"[sweep] {n:>16}: median {t[len(t)//2]:.4f} ms  min {t[0]:.4f} ms per pass")
    lib().tvm_engine_set_variant(eng.h, args.variant if args.variant is not None else 0)
    mb.launch(args.warmup)

    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    dev = f"cuda:{local}" if torch.cuda.is_available() and backend == "nccl" else "cpu"  # where max-over-ranks reduces
    launch_ms = []
    wall = td.timed(lambda: launch_ms.append(mb.time(args.steps)), steps=1, warmup=0, sync=sync, device=dev)
    vname = lib().tvm_variant_name(lib().tvm_engine_last_variant(eng.h)).decode()
    if mb.status() != (total, -1, 0) and not vname.startswith("ablate"):  # ablations are wrong by design
        raise RuntimeError("timed launches disagree with the first pass")

    gather = None
    if args.gather:  # optional RCCL gather of every rank's match list to rank 0, timed apart
        import ctypes
        pairs = torch.empty((total, 2), dtype=torch.int32, device=f"cuda:{local}")
        got = ctypes.c_uint64()
        if lib().tvm_match_copy_device(eng.h, mb.h, pairs.data_ptr(), total, ctypes.byref(got)) or got.value != total:
            raise RuntimeError("tvm_match_copy_device failed")
        g0 = time.perf_counter()
        merged = td.gather_pairs(pairs, rank * n_pkgs)
        sync()
        g_wall = td.max_over_ranks(time.perf_counter() - g0, dev)
        gather = {"ms": g_wall * 1e3, "pairs_on_root": None if merged is None else int(merged.shape[0]),
                  "bytes_per_rank": total * 16}

    value = world * n_pkgs * args.steps / wall
    launch_s = launch_ms[0] / 1e3
    alg_bytes = mb.algorithmic_bytes()
    achieved = alg_bytes / launch_s / 1e9

    fill = None
    if getattr(wl, "has_vulns", False):
        # FillInfo (vulnerability.go:60-157) fused behind the match list: timed apart, on the
        # same stream, over the same device-resident pairs (DESIGN.md "FillInfo")
        mb.launch(1)
        fill_ms = mb.fill_time(args.steps)
        fill_bytes = mb.fill_algorithmic_bytes()
        fill_gbs = fill_bytes / (fill_ms / 1e3) / 1e9
        fill = {"kernel_ms": fill_ms, "matches_per_s": total / (fill_ms / 1e3),
                "algorithmic_bytes_per_launch": fill_bytes, "achieved_GBs": fill_gbs,
                "frac": fill_gbs / HBM_PEAK_GBS, "db_vulnerabilities": len(wl.sdb.vuln_ids())}
        # result.Filter (filter.go:60-139) behind FillInfo: default options (every severity),
        # per result dedup + BySeverity order; wall time per call incl. its one sync
        mb.fill()
        fopts = mb.filter_opts()
        kept = mb.filter(fopts)
        filt_ms = mb.filter_time(fopts, max(3, args.steps // 4))
        fill["result_filter"] = {"ms": filt_ms, "kept": kept, "matches_per_s": total / (filt_ms / 1e3)}
        # + a VEX document's suppressions (filterByVEX, filter.go:38-104): 1% of the findings,
        # sampled from the match list, as the host compile (trivy_amd/vex.py) would emit them
        pr = mb.pairs()
        pick = np.random.default_rng(5).choice(len(pr), size=max(1, len(pr) // 100), replace=False)
        vex = (pr[pick, 0], [wl.sdb.adv_vid[a] for a in pr[pick, 1].tolist()])
        vopts = mb.filter_opts(vex=vex)
        vkept = mb.filter(vopts)
        vex_ms = mb.filter_time(vopts, max(3, args.steps // 4))
        fill["result_filter"]["vex"] = {"suppressions": len(pick), "ms": vex_ms, "kept": vkept,
                                        "matches_per_s": total / (vex_ms / 1e3)}

    dropin = None
    if args.dropin and args.config == "c2" and rank == 0:
        # C1-shaped request through the drop-in per-target path (debian Scanner.Detect,
        # debian.go:57-119): 100 packages of one Debian 12 image, host prologue + one launch +
        # sync + host epilogue per call - the latency a single `trivy image` scan sees
        from trivy_amd.detector.ospkg import Scanner
        p12 = wl.plats.index("debian 12")
        b0, b1 = next((b0, b1) for p, b0, b1 in wl.batch.targets if p == p12 and b1 - b0 >= 100)
        pk = [{"Name": wl.batch.names[i].decode(), "SrcName": wl.batch.names[i].decode(),
               "Version": wl.batch.versions[i].decode(), "SrcVersion": wl.batch.versions[i].decode()}
              for i in range(b0, b0 + 100)]
        sc = Scanner(eng, "debian")
        found = sc.detect("12", None, pk)
        t_d = time.perf_counter()
        n_calls = 200
        for _ in range(n_calls):
            sc.detect("12", None, pk)
        d_ms = (time.perf_counter() - t_d) * 1e3 / n_calls
        # the same call at the C-ABI alone (what a cgo caller pays): no Python result objects
        import ctypes
        from trivy_amd import _lib as L
        from trivy_amd.detector import ospkg as osp
        arr, _keep = osp._pkg_array(pk)
        res, ebuf, now = L.Result(), L.errbuf(), osp._now(None)
        t_c = time.perf_counter()
        for _ in range(n_calls):
            if lib().tvm_ospkg_driver_detect(eng.h, b"debian", b"12", None, arr, len(pk), now, ctypes.byref(res), ebuf,
                                             len(ebuf)):
                raise RuntimeError(ebuf.value.decode())
            lib().tvm_result_free(ctypes.byref(res))
        c_ms = (time.perf_counter() - t_c) * 1e3 / n_calls
        dropin = {"workload": "c1-shaped: 100 debian-12 packages per call", "ms_per_call": d_ms,
                  "c_abi_ms_per_call": c_ms, "vulnerabilities_per_call": len(found),
                  "packages_per_s": 100 / (d_ms / 1e3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = wl.cpu_baseline(args.cpu_seconds, args.cpu_threads)

    traffic = pmc_traffic(wl.name)
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
            "data": "synthetic (seeded trivy-db + SBOM batch, tools/synth.py / tools/synth_mix.py)",
            "config": {"workload": wl.name, "packages_per_gpu": n_pkgs, "matches_per_gpu": total,
                       "kernel_variant": vname,
                       "db_keys": wl.n_keys, "db_advisories": wl.n_adv,
                       "platforms": wl.plats, "parallelism": f"replicated tables, batch sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "algorithmic_bytes_per_launch": alg_bytes,
                         "kernel_ms": launch_s * 1e3},
            "cpu_baseline": cpu,
        }
        if gather is not None:
            line["gather"] = gather
        if fill is not None:
            line["fill_info"] = fill
        if dropin is not None:
            line["dropin_latency"] = dropin
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
