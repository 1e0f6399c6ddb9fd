"""Batch matching: many targets' packages in one device pass (wrappers of tvm_batch_* /
tvm_match_*).

The reference matches package by package inside each driver's Detect loop
(pkg/detector/ospkg/*/*.go, pkg/detector/library/detect.go:29-60); a scan server sees
thousands of targets at once, so this layer coalesces them: every package is added with
its platform bucket (the string a driver would pass to Get: "debian 12", "alma 9",
"npm::", ...), an already-formatted version and, for the rpm drivers that filter on them,
its arch / ksplice attributes; one launch returns every (package, advisory) pair.
"""
import ctypes
import time

import numpy as np

from . import _lib
from ._lib import lib, errbuf

ATTR_ARCH, ATTR_KSPLICE, ATTR_CPESET = 1, 2, 4


def _packed(col):
    """(bytes, lens u32) of a byte-string column (list or numpy 'S' array, no NUL bytes)."""
    a = col if isinstance(col, np.ndarray) and col.dtype.kind == "S" else np.array(list(col), dtype="S")
    n, w = len(a), a.dtype.itemsize
    if n == 0 or w == 0:
        return b"", np.zeros(n, dtype=np.uint32)
    lens = np.char.str_len(a).astype(np.uint32)
    mat = np.ascontiguousarray(a).view(np.uint8).reshape(n, w)
    return mat[np.arange(w, dtype=np.uint32)[None, :] < lens[:, None]].tobytes(), lens


def arena_of(*columns):
    """Packs byte-string columns into one arena, column after column:
    (arena, [(off u64, len u32) per column])."""
    parts, cols, base = [], [], 0
    for c in columns:
        data, lens = _packed(c)
        off = np.zeros(len(lens), dtype=np.uint64)
        if len(lens):
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        cols.append((off + np.uint64(base), lens))
        parts.append(data)
        base += len(data)
    return b"".join(parts), cols


class MatchBatch:
    """One device batch on `engine`; fail-loud (RuntimeError) on every C-ABI error."""

    def __init__(self, engine):
        self.engine = engine
        self.h = lib().tvm_batch_new()
        self.total = None

    def add_many(self, bucket, names, versions, arches=None, ksplice=False, cpe_sets=None):
        """Adds len(names) packages of one platform bucket; returns the first index.
        cpe_sets: per package a cpe_set() id (Red Hat)."""
        if not len(names):
            return len(self)
        from ._lib import AttrCols
        cols = [names, versions] + ([arches] if arches is not None else [])
        arena, c = arena_of(*cols)
        flags = (ATTR_ARCH if arches is not None else 0) | (ATTR_KSPLICE if ksplice else 0)
        ao, al = c[2] if arches is not None else (None, None)
        cs = None
        if cpe_sets is not None:
            flags |= ATTR_CPESET
            cs = np.ascontiguousarray(cpe_sets, dtype=np.uint32)
        attrs = AttrCols(ao.ctypes.data if ao is not None else None, al.ctypes.data if al is not None else None,
                         cs.ctypes.data if cs is not None else None)
        first = lib().tvm_batch_add_many_attrs(
            self.h, self.engine.h, bucket.encode(), len(names), arena, c[0][0].ctypes.data, c[0][1].ctypes.data,
            c[1][0].ctypes.data, c[1][1].ctypes.data, ctypes.byref(attrs), flags)
        if first < 0:
            raise RuntimeError("tvm_batch_add_many_attrs rejected the packages")
        return first

    def cpe_set(self, content_sets, nvr=""):
        """Registers a Red Hat (content sets, NVR) CPE set (redhat.go:112-120); returns its id."""
        from ._lib import Str, s
        keep = [s(x) for x in content_sets]
        arr = (Str * max(len(keep), 1))(*keep)
        i = lib().tvm_batch_cpe_set(self.h, self.engine.h, arr, len(keep), s(nvr))
        if i < 0:
            raise RuntimeError("tvm_batch_cpe_set failed")
        return i

    def redhat_result(self, pkgs):
        """The Red Hat driver's epilogue for the batch's Red Hat packages (GPU per-CVE merge,
        tvm_match_redhat_result); pkgs: the package dicts in batch order (Name, ID, ...)."""
        from ._lib import Result
        from .detector.ospkg import _convert
        res, e = Result(), errbuf()
        self._check(lib().tvm_match_redhat_result(self.engine.h, self.h, ctypes.byref(res), e, len(e)), e,
                    "tvm_match_redhat_result")
        try:
            return _convert(res, pkgs)
        finally:
            lib().tvm_result_free(ctypes.byref(res))

    def redhat_merge(self):
        """Enqueue the per-CVE merge on the device (tvm_match_redhat_merge): from now until
        the next launch the batch's match list - pairs(), fill(), filter() - is the merged
        one (Red Hat packages: one pair per (package, VulnerabilityID))."""
        e = errbuf()
        self._check(lib().tvm_match_redhat_merge(self.engine.h, self.h, e, len(e)), e, "tvm_match_redhat_merge")
        return self

    def redhat_merge_time(self, steps):
        """ms per merge over `steps` back-to-back merges (HIP events on the engine stream)."""
        ms = ctypes.c_double()
        e = errbuf()
        self._check(lib().tvm_match_redhat_merge_time(self.engine.h, self.h, steps, ctypes.byref(ms), e, len(e)), e,
                    "tvm_match_redhat_merge_time")
        return ms.value / steps

    def redhat_vulns(self, pairs, pkgs):
        """The merged Red Hat DetectedVulnerabilities of the given merged-list pairs (e.g.
        filtered_pairs()), in that order; pairs of other drivers are skipped."""
        from ._lib import Result
        from .detector.ospkg import _convert
        pr = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1, 2)
        res, e = Result(), errbuf()
        self._check(lib().tvm_match_redhat_vulns(self.engine.h, self.h, pr.ctypes.data if len(pr) else None, len(pr),
                                                 ctypes.byref(res), e, len(e)), e, "tvm_match_redhat_vulns")
        try:
            return _convert(res, pkgs)
        finally:
            lib().tvm_result_free(ctypes.byref(res))

    def add_arena(self, bucket, n, arena, name_off, name_len, ver_off, ver_len):
        """Adds n packages whose name/version bytes already sit in one arena (u64 offsets,
        u32 lengths as numpy arrays); returns the first index."""
        first = lib().tvm_batch_add_many(self.h, self.engine.h, bucket.encode(), n, arena, name_off.ctypes.data,
                                         name_len.ctypes.data, ver_off.ctypes.data, ver_len.ctypes.data)
        if first < 0:
            raise RuntimeError("tvm_batch_add_many rejected the packages")
        return first

    def add_targets(self, buckets, target_end, arena, name_off, name_len, ver_off, ver_len, flags=None,
                    arch_off=None, arch_len=None, cpe_sets=None):
        """Many targets in one call (tvm_batch_add_targets): target t = packages
        [target_end[t-1], target_end[t]) of the arena columns under buckets[t].  flags: per target
        ATTR_* bits, with the per-package attribute columns (arch strings in the arena, cpe_set()
        ids) - tvm_batch_add_targets_attrs."""
        from ._lib import AttrCols, Str
        bl = [b.encode() if isinstance(b, str) else bytes(b) for b in buckets]
        arr = (Str * max(len(bl), 1))(*[Str(b, len(b)) for b in bl])
        te = np.ascontiguousarray(target_end, dtype=np.uint64)
        cols = [np.ascontiguousarray(c, dtype=t) for c, t in ((name_off, np.uint64), (name_len, np.uint32),
                                                              (ver_off, np.uint64), (ver_len, np.uint32))]
        if flags is None:
            first = lib().tvm_batch_add_targets(self.h, self.engine.h, len(bl), arr, te.ctypes.data, arena,
                                                *[c.ctypes.data for c in cols])
        else:
            fl = np.ascontiguousarray(flags, dtype=np.uint32)
            ao = None if arch_off is None else np.ascontiguousarray(arch_off, dtype=np.uint64)
            al = None if arch_len is None else np.ascontiguousarray(arch_len, dtype=np.uint32)
            cs = None if cpe_sets is None else np.ascontiguousarray(cpe_sets, dtype=np.uint32)
            attrs = AttrCols(ao.ctypes.data if ao is not None else None, al.ctypes.data if al is not None else None,
                             cs.ctypes.data if cs is not None else None)
            first = lib().tvm_batch_add_targets_attrs(self.h, self.engine.h, len(bl), arr, fl.ctypes.data,
                                                      te.ctypes.data, arena, *[c.ctypes.data for c in cols],
                                                      ctypes.byref(attrs))
        if first < 0:
            raise RuntimeError("tvm_batch_add_targets rejected the targets")
        return first

    def __len__(self):
        return lib().tvm_batch_size(self.h)

    def _check(self, rc, e, what):
        if rc:
            raise RuntimeError(f"{what}: {e.value.decode()}")

    def upload(self, match_cap=None):
        e = errbuf()
        cap = match_cap if match_cap is not None else max(1024, 8 * len(self))
        self._check(lib().tvm_batch_upload(self.engine.h, self.h, cap, e, len(e)), e, "tvm_batch_upload")
        self.cap = cap
        return self

    def set_package_base(self, base):
        """Every match reports package index base + i (a shard of a global batch)."""
        if lib().tvm_batch_set_package_base(self.h, base):
            raise RuntimeError("tvm_batch_set_package_base")
        return self

    def upload_into(self, pkg, adv):
        """Upload, with the match columns written into caller device buffers (torch int32
        tensors on the engine's GPU, same length = the match capacity)."""
        e = errbuf()
        cap = pkg.numel()
        if adv.numel() != cap or pkg.dtype.itemsize != 4 or adv.dtype.itemsize != 4:
            raise ValueError("two 4-byte columns of equal length")
        self._check(lib().tvm_batch_upload_into(self.engine.h, self.h, pkg.data_ptr(), adv.data_ptr(), cap, e, len(e)),
                    e, "tvm_batch_upload_into")
        self.cap = cap
        self._cols = (pkg, adv)
        return self

    def order_into(self, csr_adv, row_end):
        """The last pass's per-package advisory lists as CSR, written by the order kernel into
        caller device buffers (int32 torch tensors on the engine's GPU: csr_adv >= the match
        count, row_end = one entry per package of this batch); returns the match count."""
        if row_end.numel() < len(self) or csr_adv.dtype.itemsize != 4 or row_end.dtype.itemsize != 4:
            raise ValueError("row_end needs one 4-byte entry per package, csr_adv 4-byte entries")
        e, n = errbuf(), ctypes.c_uint64()
        self._check(lib().tvm_match_order_into(self.engine.h, self.h, csr_adv.data_ptr(), row_end.data_ptr(),
                                               csr_adv.numel(), ctypes.byref(n), e, len(e)), e, "tvm_match_order_into")
        return n.value

    def launch(self, k=1, sync=True):
        e = errbuf()
        for _ in range(k):
            self._check(lib().tvm_match_launch(self.engine.h, self.h, e, len(e)), e, "tvm_match_launch")
        if sync:
            self._check(lib().tvm_engine_sync(self.engine.h, e, len(e)), e, "tvm_engine_sync")
        return self

    def status(self):
        """(n_matches, first poisoned package or -1, error bits)."""
        n, errp, bits = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_uint64()
        rc = lib().tvm_match_status(self.engine.h, self.h, ctypes.byref(n), ctypes.byref(errp), ctypes.byref(bits))
        if rc:
            raise RuntimeError(f"tvm_match_status failed ({rc})")
        return n.value, errp.value, bits.value

    def run(self):
        """Upload (sizing the match buffer exactly after a first pass if needed) + one pass."""
        self.upload().launch()
        total, errp, bits = self.status()
        if total > self.cap:
            self.upload(total).launch()
            total, errp, bits = self.status()
        self.total = total
        return total, errp, bits

    def pairs(self):
        """All (package, advisory) pairs as uint32 [n, 2], in (package, advisory) order."""
        total = self.status()[0]
        out = np.zeros((total, 2), dtype=np.uint32)
        got = ctypes.c_uint64()
        if lib().tvm_match_fetch(self.engine.h, self.h, out.ctypes.data, total, ctypes.byref(got)):
            raise RuntimeError("tvm_match_fetch failed (match buffer overflow?)")
        return out[:got.value]

    def time(self, steps):
        """ms per pass over `steps` back-to-back launches (HIP events on the engine stream)."""
        ms = ctypes.c_double()
        e = errbuf()
        self._check(lib().tvm_match_time(self.engine.h, self.h, steps, ctypes.byref(ms), e, len(e)), e,
                    "tvm_match_time")
        return ms.value / steps

    def algorithmic_bytes(self):
        return lib().tvm_match_algorithmic_bytes(self.engine.h, self.h)

    # ---- end-to-end pipelined pass (tvm_pipeline_*) ----
    def pipeline_prepare(self, match_cap=None, chunk_packages=1 << 19, raw=False, adv32=False):
        """Pins the batch and sizes the pipeline (host batch -> GPU -> host CSR).  raw: upload
        the batch's own arrays instead of its transport form (TVM_PIPE_RAW); adv32: 4-byte
        advisory indices in the result even when 3 bytes hold them (TVM_PIPE_ADV32)."""
        e = errbuf()
        cap = match_cap if match_cap is not None else max(1024, 8 * len(self))
        flags = (1 if raw else 0) | (2 if adv32 else 0)
        self._check(lib().tvm_pipeline_prepare(self.engine.h, self.h, cap, chunk_packages, flags, e, len(e)), e,
                    "tvm_pipeline_prepare")
        self.pipe_cap = cap
        return self

    def pipeline_run(self):
        """One end-to-end pass: (matches, first poisoned package or -1, wall ms)."""
        e = errbuf()
        n, errp, ms = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_double()
        rc = lib().tvm_pipeline_run(self.engine.h, self.h, ctypes.byref(n), ctypes.byref(errp), ctypes.byref(ms), e,
                                    len(e))
        if rc and n.value > self.pipe_cap:
            raise OverflowError(n.value)
        self._check(rc, e, "tvm_pipeline_run")
        return n.value, errp.value, ms.value

    def pipeline_csr(self):
        """(adv uint32[matches], row_end uint32[packages]) of the last pass (copies)."""
        adv, rend, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        if lib().tvm_pipeline_result(self.h, ctypes.byref(adv), ctypes.byref(rend), ctypes.byref(n)):
            raise RuntimeError("tvm_pipeline_result: no valid pass")
        m = len(self)
        a = np.ctypeslib.as_array((ctypes.c_uint32 * max(n.value, 1)).from_address(adv.value))[:n.value].copy() \
            if n.value else np.zeros(0, np.uint32)
        r = np.ctypeslib.as_array((ctypes.c_uint32 * max(m, 1)).from_address(rend.value))[:m].copy() \
            if m else np.zeros(0, np.uint32)
        return a, r

    def pipeline_csr_raw(self):
        """(adv uint32[matches] decoded from the bytes as they arrived, width 3 or 4) of the last
        pass - tvm_pipeline_result_raw."""
        adv, rend, n, w = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint32()
        if lib().tvm_pipeline_result_raw(self.h, ctypes.byref(adv), ctypes.byref(w), ctypes.byref(rend), ctypes.byref(n)):
            raise RuntimeError("tvm_pipeline_result_raw: no valid pass")
        k, width = n.value, w.value
        if not k:
            return np.zeros(0, np.uint32), width
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * (k * width)).from_address(adv.value)).reshape(k, width)
        out = np.zeros(k, np.uint32)
        for j in range(width):
            out |= raw[:, j].astype(np.uint32) << (8 * j)
        return out, width

    def pipeline_decode_ms(self):
        """tvm_pipeline_result's host time for the last pass (the 3-byte indices widened into
        the 4-byte CSR; once per pass), ms."""
        adv, rend, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        t0 = time.perf_counter()
        if lib().tvm_pipeline_result(self.h, ctypes.byref(adv), ctypes.byref(rend), ctypes.byref(n)):
            raise RuntimeError("tvm_pipeline_result: no valid pass")
        return (time.perf_counter() - t0) * 1e3

    def pipeline_stats(self):
        out = (ctypes.c_uint64 * 5)()
        if lib().tvm_pipeline_stats(self.h, out):
            raise RuntimeError("tvm_pipeline_stats")
        enc, prep = ctypes.c_uint64(), ctypes.c_uint64()
        lib().tvm_pipeline_times(self.h, ctypes.byref(enc), ctypes.byref(prep))
        return {"h2d_bytes": out[0], "d2h_bytes": out[1], "chunks": out[2], "transport_form": bool(out[3]),
                "encode_ms": out[4] / 1e3, "prepare_ms": prep.value / 1e3}

    # ---- FillInfo fused behind the match list (tvm_match_fill*) ----
    def fill(self, sync=True):
        """Enqueue FillInfo over the device match list (after launch())."""
        e = errbuf()
        self._check(lib().tvm_match_fill(self.engine.h, self.h, e, len(e)), e, "tvm_match_fill")
        if sync:
            self._check(lib().tvm_engine_sync(self.engine.h, e, len(e)), e, "tvm_engine_sync")
        return self

    def fill_decisions(self):
        """uint32 [n, 4] per pair in pairs() order: {record or 0xFFFFFFFF, status,
        severity code | source id << 16, URL kind << 28 | reference index}."""
        total = self.status()[0]
        out = np.zeros((total, 4), dtype=np.uint32)
        got = ctypes.c_uint64()
        if lib().tvm_match_fill_fetch(self.engine.h, self.h, out.ctypes.data, total, ctypes.byref(got)):
            raise RuntimeError("tvm_match_fill_fetch failed")
        return out[:got.value]

    def fill_time(self, steps):
        ms = ctypes.c_double()
        e = errbuf()
        self._check(lib().tvm_match_fill_time(self.engine.h, self.h, steps, ctypes.byref(ms), e, len(e)), e,
                    "tvm_match_fill_time")
        return ms.value / steps

    def fill_algorithmic_bytes(self):
        return lib().tvm_match_fill_algorithmic_bytes(self.engine.h, self.h)

    # ---- result.Filter per result (tvm_match_filter*) ----
    def set_report(self, first, names=None, versions=None, paths=None):
        """DetectedVulnerability PkgName / InstalledVersion / PkgPath of packages [first,
        first + n) where they differ from the batch (name, version) / "" (tvm_batch_set_report)."""
        from ._lib import Str
        cols, keep = [], []
        n = None
        for col in (names, versions, paths):
            if col is None:
                cols.append(None)
                continue
            blobs = [x.encode() if isinstance(x, str) else bytes(x) for x in col]
            if n is not None and len(blobs) != n:
                raise ValueError("report columns differ in length")
            n = len(blobs)
            arr = (Str * max(n, 1))(*[Str(b, len(b)) for b in blobs])
            keep.append((blobs, arr))
            cols.append(arr)
        if n is None:
            return
        if lib().tvm_batch_set_report(self.h, first, n, *cols):
            raise ValueError("tvm_batch_set_report: bad range")

    def vuln_ranks(self, str_array, n):
        """tvm_vuln_rank_many over a Str array (uint32, 0xFFFFFFFF = unknown ID)."""
        r = np.zeros(max(n, 1), dtype=np.uint32)
        if lib().tvm_vuln_rank_many(self.engine.h, str_array, n, r.ctypes.data):
            raise RuntimeError("tvm_vuln_rank_many failed")
        return r

    def filter_opts(self, severities=("UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"), ignore_statuses=(),
                    ignore_ids=(), ignore=None, vex=None):
        """FilterOption's vulnerability part.  ignore: trivy_amd.ignore.IgnoreRules compiled
        for this batch; ignore_ids: shorthand for a plain .trivyignore (IDs in file order);
        vex: (package indices, IDs) from trivy_amd.vex.VEX.suppressions (None: no VEX
        document)."""
        from ._lib import FilterOpts, IgnoreRulesC, Str
        from .ignore import plain_rules
        names = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]
        strs = lambda xs: (lambda bl: (bl, (Str * max(len(bl), 1))(*[Str(b, len(b)) for b in bl])))(  # noqa: E731
            [i.encode() if isinstance(i, str) else bytes(i) for i in xs])
        ptr = lambda a: a.ctypes.data if a is not None and len(a) else None  # noqa: E731
        keep = []
        if ignore is None and ignore_ids:
            ignore = plain_rules(list(ignore_ids), 0)
        rc = None
        if ignore is not None:
            (aid, aprec), (ppk, pid, pprec), (ccl, cid, cprec), pcls = ignore.arrays()
            ids = strs(ignore.ids)
            ranks = self.vuln_ranks(ids[1], len(ids[0]))  # once per compile, not per filter call
            keep.append(ranks)
            rc = IgnoreRulesC(ids[1], len(ids[0]), ranks.ctypes.data, ptr(aid), ptr(aprec), len(aid), ptr(ppk), ptr(pid), ptr(pprec),
                              len(ppk), ptr(pcls), ptr(ccl), ptr(cid), ptr(cprec), len(ccl))
            keep += [ids, aid, aprec, ppk, pid, pprec, ccl, cid, cprec, pcls, rc]
        uniq = {}
        vpk, vidx = np.zeros(0, dtype=np.uint32), np.zeros(0, dtype=np.uint32)
        if vex is not None:
            vpk = np.ascontiguousarray(vex[0], dtype=np.uint32)
            if len(vpk) != len(vex[1]):
                raise ValueError("one vulnerability ID per package index")
            vidx = np.array([uniq.setdefault(i, len(uniq)) for i in vex[1]], dtype=np.uint32)
        vids = strs(list(uniq))
        vranks = self.vuln_ranks(vids[1], len(vids[0]))
        o = FilterOpts(sum(1 << names.index(x) for x in severities), sum(1 << s for s in ignore_statuses),
                       ctypes.pointer(rc) if rc is not None else None, ptr(vpk), ptr(vidx), len(vpk), vids[1],
                       len(vids[0]), vranks.ctypes.data)
        o._keep = (keep, vpk, vidx, vids, vranks)
        return o

    def filter(self, opts):
        """filterVulnerabilities + BySeverity (+ VEX) for every result (after launch() +
        fill()); returns the number of surviving vulnerabilities (self.n_ignored: the
        ignored findings)."""
        e = errbuf()
        n, ni = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(lib().tvm_match_filter(self.engine.h, self.h, ctypes.byref(opts), ctypes.byref(n),
                                           ctypes.byref(ni), e, len(e)), e, "tvm_match_filter")
        self.n_ignored = ni.value
        return n.value

    def filtered_pairs(self, n):
        out = np.zeros((n, 2), dtype=np.uint32)
        got = ctypes.c_uint64()
        if lib().tvm_match_filter_fetch(self.engine.h, self.h, out.ctypes.data, n, ctypes.byref(got)):
            raise RuntimeError("tvm_match_filter_fetch failed")
        return out[:got.value]

    def ignored_findings(self):
        """ModifiedFindings of the last filter(): (n, 3) uint32 {package, advisory, finding
        index} in detection order."""
        n = getattr(self, "n_ignored", 0)
        out = np.zeros((n, 3), dtype=np.uint32)
        got = ctypes.c_uint64()
        if lib().tvm_match_filter_ignored(self.engine.h, self.h, out.ctypes.data, n, ctypes.byref(got)):
            raise RuntimeError("tvm_match_filter_ignored failed")
        return out[:got.value]

    def filter_time(self, opts, steps):
        ms = ctypes.c_double()
        e = errbuf()
        self._check(lib().tvm_match_filter_time(self.engine.h, self.h, ctypes.byref(opts), steps, ctypes.byref(ms), e,
                                                len(e)), e, "tvm_match_filter_time")
        return ms.value / steps

    # ---- DetectedVulnerability sets (tvm_match_vulns / tvm_pipeline_vulns) ----
    def vulns(self, pipeline=False):
        """The batch's DetectedVulnerability set (the drivers' epilogues over every match):
        a VulnSet with pkg / rec columns and the records (after launch(), or after
        pipeline_run() with pipeline=True)."""
        from ._lib import VulnSet as CSet
        vs, e = CSet(), errbuf()
        fn = lib().tvm_pipeline_vulns if pipeline else lib().tvm_match_vulns
        t0 = time.perf_counter()
        self._check(fn(self.engine.h, self.h, ctypes.byref(vs), e, len(e)), e,
                    "tvm_pipeline_vulns" if pipeline else "tvm_match_vulns")
        ms = (time.perf_counter() - t0) * 1e3
        return VulnSet(self, vs, ms)

    def report(self, first=0, n=None):
        """(names, installed versions, paths) of packages [first, first + n) as the export pairs
        them with records (tvm_batch_report_get): names None where the caller's Name applies."""
        from ._lib import RawStr
        n = len(self) - first if n is None else n
        cols = [(RawStr * max(n, 1))() for _ in range(3)]
        if lib().tvm_batch_report_get(self.h, first, n, *cols):
            raise ValueError("tvm_batch_report_get: bad range")
        names = [(c.bytes().decode() if c.p else None) for c in cols[0][:n]]
        return names, [c.bytes().decode() for c in cols[1][:n]], [c.bytes().decode() for c in cols[2][:n]]

    def close(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            if _lib._lib is not None:
                _lib._lib.tvm_batch_free(h)

    def __del__(self):
        self.close()


def vuln_record(v):
    """A tvm_vuln record (the advisory side of a DetectedVulnerability) as a dict of the
    DetectedVulnerability fields it sets, plus "_copy" = its copy flags."""
    d = {"VulnerabilityID": v.vulnerability_id.decode(), "_copy": v.copy_flags}
    if v.n_vendor_ids:
        d["VendorIDs"] = [v.vendor_ids[k].decode() for k in range(v.n_vendor_ids)]
    if v.fixed_version:
        d["FixedVersion"] = v.fixed_version.decode()
    if v.status:
        d["Status"] = v.status
    if v.severity_source:
        d["SeveritySource"] = v.severity_source.decode()
    if v.severity:
        d["Severity"] = v.severity.decode()
    if v.has_data_source:
        d["DataSource"] = {k: val.decode() for k, val in [("ID", v.data_source_id), ("Name", v.data_source_name),
                                                          ("URL", v.data_source_url)] if val}
    if v.custom_json is not None:
        d["Custom"] = v.custom_json.decode()
    return d


class VulnSet:
    """tvm_vuln_set: per-package lists (CSR) of record indices; DetectedVulnerability i = record
    rec[i] + package pkg[i] (the columns are expanded here, numpy)."""

    def __init__(self, batch, cset, ms):
        self.batch, self._c, self.ms = batch, cset, ms
        n, npk, w = cset.n, cset.n_pkgs, cset.rec_width
        self.row_end = np.ctypeslib.as_array(cset.row_end, shape=(npk,)).copy() if npk else np.zeros(0, np.uint32)
        counts = np.diff(np.concatenate([[0], self.row_end.astype(np.int64)]))
        self.pkg = np.repeat(np.arange(npk, dtype=np.uint32) + np.uint32(cset.first_pkg), counts)
        if n:
            raw = np.ctypeslib.as_array((ctypes.c_uint8 * (n * w)).from_address(cset.rec)).reshape(n, w)
            self.rec = np.zeros(n, np.uint32)
            for j in range(w):
                self.rec |= raw[:, j].astype(np.uint32) << np.uint32(8 * j)
        else:
            self.rec = np.zeros(0, np.uint32)
        self.rec_width = w
        self.n_adv_recs, self.n_grp_recs = cset.n_adv_recs, cset.n_grp_recs
        self._recs = {}

    def __len__(self):
        return len(self.pkg)

    def record(self, r):
        """Record r as a dict (vuln_record)."""
        r = int(r)
        d = self._recs.get(r)
        if d is None:
            c = self._c
            d = vuln_record(c.adv_recs[r] if r < c.n_adv_recs else c.grp_recs[r - c.n_adv_recs])
            self._recs[r] = d
        return d

    def dicts(self, pkgs=None, report=None):
        """DetectedVulnerability dicts (small sets): pkgs maps a package index as the set
        reports it (self.pkg: first_pkg + batch index, tvm_batch_set_package_base) to the
        caller's package dict (ID, Name, Identifier, Layer copied per the record's flags);
        report = MatchBatch.report() columns of the whole batch (batch indices from 0:
        InstalledVersion, PkgPath, PkgName overrides)."""
        from ._lib import COPY_IDENTIFIER, COPY_LAYER, COPY_PKG_ID, COPY_PKG_NAME
        names, vers, paths = report if report is not None else self.batch.report()
        base = int(self._c.first_pkg) if self._c is not None else 0
        out = []
        for p, r in zip(self.pkg.tolist(), self.rec.tolist()):
            d = dict(self.record(r))
            fl = d.pop("_copy")
            pk = (pkgs or {}).get(p, {})
            p -= base  # the report columns are indexed from the batch's first package
            if fl & COPY_PKG_ID and pk.get("ID"):
                d["PkgID"] = pk["ID"]
            name = names[p] if names[p] is not None else (pk.get("Name") if fl & COPY_PKG_NAME else None)
            if name:
                d["PkgName"] = name
            if paths[p]:
                d["PkgPath"] = paths[p]
            if fl & COPY_IDENTIFIER and pk.get("Identifier"):
                d["PkgIdentifier"] = pk["Identifier"]
            if vers[p]:
                d["InstalledVersion"] = vers[p]
            if fl & COPY_LAYER and pk.get("Layer"):
                d["Layer"] = pk["Layer"]
            out.append(d)
        return out

    def walk(self):
        """tvm_vuln_set_walk: (DetectedVulnerabilities walked, digest) - a native consumer that
        decodes every record index and reads its record and its package's InstalledVersion."""
        n, d = ctypes.c_uint64(), ctypes.c_uint64()
        if lib().tvm_vuln_set_walk(ctypes.byref(self._c), self.batch.h, ctypes.byref(n), ctypes.byref(d)):
            raise RuntimeError("tvm_vuln_set_walk rejected the set")
        return n.value, d.value

    def digest(self, report=None):
        """The walk's digest recomputed here (numpy) from the columns and the records."""
        names, vers, _ = report if report is not None else self.batch.report()
        M = np.uint64(0xFFFFFFFFFFFFFFFF)
        base = int(self._c.first_pkg)
        vlen = np.array([len(v.encode()) for v in vers], dtype=np.uint64)
        uniq, inv = np.unique(self.rec, return_inverse=True)
        fl = np.zeros(len(uniq), np.uint64)
        for k, r in enumerate(uniq.tolist()):
            d = self.record(r)
            fl[k] = ((d.get("Status", 0) & 0xFF) << 32 | (len(d.get("VendorIDs", [])) & 0xFF) << 24
                     | (1 << 8 if "DataSource" in d else 0) | (d["_copy"] & 0xFF))
        with np.errstate(over="ignore"):
            p = self.pkg.astype(np.uint64)
            h = (p * np.uint64(0x9E3779B97F4A7C15) + self.rec.astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)
                 + (vlen[(p - np.uint64(base)).astype(np.int64)] << np.uint64(40)) + fl[inv]) & M
            for c in (0xff51afd7ed558ccd, 0xc4ceb9fe1a85ec53):
                h ^= h >> np.uint64(33)
                h *= np.uint64(c)
            h ^= h >> np.uint64(33)
            return int(h.sum(dtype=np.uint64))

    def close(self):
        if self._c is not None and self._c.priv:
            lib().tvm_vuln_set_free(ctypes.byref(self._c))
        self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def advisory_vuln_id(db, adv):
    p = lib().tvm_db_advisory_vuln_id(db.h, adv)
    return p.decode() if p else None
