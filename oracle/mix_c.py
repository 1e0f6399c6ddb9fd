"""ORACLE - TEST INFRASTRUCTURE ONLY: ctypes front end of oracle/mixmatch.c (orc_mix_match),
the native CPU baseline of the mixed workloads (BASELINE C3 / C4 / C5).

Prepared(sdb, sample) digests a sample of a tools/synth_mix.py batch the way the reference
drivers see it: each package becomes (platform, the driver's lookup name, the version string
the driver compares, arch, Red Hat CPE set, skip), and the advisories of every looked-up key
are decoded ONCE with the oracle's own decoders (oracle/drivers.py Records / decode_redhat,
oracle/library.py get_advisories_prefix) into flat entries.  match() then runs the C driver
loops.  Used by bench.py's cpu_baseline leg and tests/test_cport.py (which checks the result
against oracle/drivers.py + oracle/library.py on the same sample); the product never sees
this.
"""
import ctypes

import numpy as np

from . import drivers as od
from . import library as ol
from .drivers import lib as _lib

MX = {"debian": 1, "ubuntu": 2, "alpine": 3, "alma": 4, "rocky": 5, "oracle": 6, "redhat": 7}
MX_LIB = 8
GRAMMAR = {"generic": 1, "npm": 2, "pep440": 3, "maven": 4}
HAS_VULN, HAS_SECURE, ALWAYS = 1, 2, 4

_I32, _I64, _U64, _U32, _U8 = (ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64),
                               ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint8))


class OrcMixDB(ctypes.Structure):
    _fields_ = [("n_plat", ctypes.c_int32), ("plat_driver", _I32), ("plat_grammar", _I32), ("n_keys", ctypes.c_int32),
                ("key_plat", _I32), ("key_name_arena", ctypes.c_char_p), ("key_name_off", _U64),
                ("key_name_len", _U32), ("key_begin", _I64), ("arena", ctypes.c_char_p),
                ("fixed_off", _U64), ("fixed_len", _U32), ("aff_off", _U64), ("aff_len", _U32),
                ("vul_off", _U64), ("vul_len", _U32), ("sec_off", _U64), ("sec_len", _U32), ("lib_flags", _U32),
                ("vid", _I32), ("ids_begin", _I64), ("n_arch", _I32), ("ids", _I32)]


class OrcMixBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("plat", _I32), ("name_arena", ctypes.c_char_p), ("name_off", _U64),
                ("name_len", _U32), ("ver_arena", ctypes.c_char_p), ("ver_off", _U64), ("ver_len", _U32),
                ("arch", _I32), ("noarch_id", ctypes.c_int32), ("skip", _U8), ("cpe_begin", _I64), ("cpe_ids", _I32)]


class _Arena:
    def __init__(self):
        self.parts, self.n = [], 0

    def put(self, s):
        b = s.encode() if isinstance(s, str) else s
        off = self.n
        self.parts.append(b)
        self.n += len(b)
        return off, len(b)

    def bytes(self):
        return b"".join(self.parts)


def _p(a, t):
    return a.ctypes.data_as(t)


def _driver_view(kind, p):
    """(lookup name, compared version, skip) of driver package p (the oracle's driver code)."""
    if kind in ("debian", "ubuntu"):
        return p.get("SrcName", ""), od.fmt_src(p), False
    if kind == "alpine":
        return p.get("SrcName") or p.get("Name", ""), od.fmt_src(p), False
    label = p.get("Modularitylabel", "")
    if kind == "alma":
        return (od.add_modular_namespace(p.get("Name", ""), label), od.fmt(p),
                ".module_el" in p.get("Release", "") and not label)
    if kind == "rocky":
        return p.get("Name", ""), od.fmt(p), bool(label)
    if kind == "oracle":
        return p.get("Name", ""), od.fmt(p), False
    if kind == "redhat":
        return od.add_modular_namespace(p.get("Name", ""), label), od.fmt(p), p.get("Release", "").endswith(".remi")
    raise ValueError(kind)


def _fmt_cols(epoch, version, release):
    """format_version (drivers.py) over columns: version, "-release" when set, "epoch:" when set."""
    v = np.where(release != b"", np.char.add(np.char.add(version, b"-"), release), version)
    return np.where(epoch != 0, np.char.add(np.char.add(epoch.astype("S"), b":"), v), v)


def _per_unique(col, fn):
    """fn over the distinct values of a bytes column, mapped back to every row."""
    uniq, inv = np.unique(col, return_inverse=True)
    return np.array([fn(u) for u in uniq.tolist()] or [b""], dtype=object)[inv]


def _columnar_views(sm, sdb, p, g, idx, aid):
    """The per-package fields Prepared's scalar loop takes from driver_packages + _driver_view,
    over whole columns (numpy), for batches too large for a Python loop per package:
    (lookup names, compared versions, installed versions, arch ids, skip, CPE-combination
    representative rows).  Pinned to the scalar loop by tests/test_cport.py."""
    bucket, kind = sdb.plats[p]
    take = lambda c: g[c][idx]  # noqa: E731
    n = len(idx)
    if kind in sm.LANG_OF:
        eco = ol.LANG[sm.LANG_OF[kind]][0]
        ver = take("ver")
        nm = _per_unique(take("name"), lambda b: ol.normalize_pkg_name(eco, b.decode()).encode())
        return nm, ver, ver, np.full(n, -1, np.int32), np.zeros(n, np.uint8), None
    name = take("pname") if kind == "redhat" else take("name")
    ver = _fmt_cols(take("epoch"), take("version"), take("rel"))
    label = take("label") if kind == "redhat" else np.full(n, b"", dtype="S1")
    skip = np.zeros(n, np.uint8)
    if kind in ("alma", "redhat"):
        if kind == "redhat":
            lab_u, lab_inv = np.unique(label, return_inverse=True)
            ns = [b"" if not lb else od.add_modular_namespace("", lb.decode()).encode() for lb in lab_u.tolist()]
            nm = np.char.add(np.array(ns, dtype="S")[lab_inv], name)
            skip = np.char.endswith(take("rel"), b".remi").astype(np.uint8)
        else:  # alma packages here carry no Modularitylabel
            nm = name
            skip = (np.char.find(take("rel"), b".module_el") >= 0).astype(np.uint8)
    else:  # debian / ubuntu (SrcName = Name), alpine, rocky (no label), oracle
        nm = name
    arches = np.full(n, -1, np.int32)
    if "arch" in g:
        au, ainv = np.unique(take("arch"), return_inverse=True)
        arches = np.array([aid(a.decode()) if a else -1 for a in au.tolist()], np.int32)[ainv]
    combo = None
    if kind == "redhat":  # one (content sets, NVR) per (release, BuildInfo NVR)
        key = np.char.add(np.char.add(take("rhrel").astype("S"), b"|"), np.where(take("bi"), take("nvr"), b""))
        _, combo_first, combo_inv = np.unique(key, return_index=True, return_inverse=True)
        combo = (idx[combo_first], combo_inv)
    return nm, ver, ver, arches, skip, combo


class _Decoded:
    """A bytes column read as str per element (Prepared.installed in the columnar form)."""

    def __init__(self, col):
        self.col = col

    def __len__(self):
        return len(self.col)

    def __getitem__(self, i):
        return self.col[i].decode()


class Prepared:
    """Oracle-side digest of a sample: sample = [(platform index p, group g, row indices)] of a
    tools/synth_mix.py MixBatch over MixDB sdb.  columnar: the per-package fields come from
    _columnar_views (whole-batch checks at 10-20M packages); the default scalar form builds
    every package's driver dict (oracle/drivers.py) and is the one the C port is pinned to."""

    def __init__(self, sm, sdb, sample, columnar=False):
        if columnar:
            self._init_columnar(sm, sdb, sample)
            return
        self.pkgs = []  # (plat, driver package dict) in sample order
        self.installed = []  # per package: the InstalledVersion its driver reports
        self.plat_family = []  # per platform: the OS driver family, or None for a language bucket
        plat_drv, plat_gram = [], []
        for bucket, kind in sdb.plats:
            if kind in sm.LANG_OF:
                plat_drv.append(MX_LIB)
                plat_gram.append(GRAMMAR[ol.LANG[sm.LANG_OF[kind]][1]])
                self.plat_family.append(None)
            else:
                plat_drv.append(MX[sm.DRIVER_OF[kind][0]])
                plat_gram.append(0)
                self.plat_family.append(sm.DRIVER_OF[kind][0])
        arch_id = {}

        def aid(a):
            return arch_id.setdefault(a, len(arch_id))
        noarch = aid("noarch")
        names, vers, plats, arches, skip, cpes = [], [], [], [], [], [[]]
        want = {}  # (plat, lookup name) -> None (the keys the sample looks up)
        for p, g, idx in sample:
            bucket, kind = sdb.plats[p]
            dp = sm.driver_packages(sdb, p, g, idx)
            if kind in sm.LANG_OF:
                eco = ol.LANG[sm.LANG_OF[kind]][0]
            for pk, i in zip(dp, idx):
                if kind == "redhat":  # the release the driver is called with (one per image)
                    pk["_rel"] = int(g["rhrel"][i])
                self.pkgs.append((p, pk))
                self.installed.append(pk.get("Version", "") if kind in sm.LANG_OF else od.fmt(pk))
                if kind in sm.LANG_OF:
                    nm, ver, sk = ol.normalize_pkg_name(eco, pk.get("Name", "")), pk.get("Version", ""), False
                else:
                    nm, ver, sk = _driver_view(kind, pk)
                names.append(nm)
                vers.append(ver)
                plats.append(p)
                arches.append(aid(pk["Arch"]) if pk.get("Arch") else -1)
                skip.append(1 if sk else 0)
                cpes.append([])
                want[(p, nm)] = None
        self.plat_of = np.array(plats, dtype=np.int64)
        recs = self._records(sm, sdb, want)
        cpe_of = {}  # (content sets, nvr) -> the CPE set (one per image, not per package)
        for i, (p, pk) in enumerate(self.pkgs):
            if sdb.plats[p][1] == "redhat":
                cpes[i + 1] = self._cpe_set(recs, cpe_of, pk)
        names = [x.encode() for x in names]
        vers = [x.encode() for x in vers]
        self._finish(sm, sdb, recs, want, aid, noarch, plat_drv, plat_gram, names, vers, plats, arches, skip, cpes)

    def _init_columnar(self, sm, sdb, sample):
        self.pkgs = None
        plat_drv, plat_gram = [], []
        self.plat_family = []
        for bucket, kind in sdb.plats:
            if kind in sm.LANG_OF:
                plat_drv.append(MX_LIB)
                plat_gram.append(GRAMMAR[ol.LANG[sm.LANG_OF[kind]][1]])
                self.plat_family.append(None)
            else:
                plat_drv.append(MX[sm.DRIVER_OF[kind][0]])
                plat_gram.append(0)
                self.plat_family.append(sm.DRIVER_OF[kind][0])
        arch_id = {}

        def aid(a):
            return arch_id.setdefault(a, len(arch_id))
        noarch = aid("noarch")
        cols = []
        want = {}
        for p, g, idx in sample:
            nm, ver, inst, arches, skip, combo = _columnar_views(sm, sdb, p, g, np.asarray(idx), aid)
            cols.append((p, g, nm, ver, inst, arches, skip, combo))
            for u in np.unique(nm).tolist():
                want[(p, u.decode())] = None
        recs = self._records(sm, sdb, want)
        cpe_of = {}
        cpes = [[]]
        for p, g, nm, ver, inst, arches, skip, combo in cols:
            if combo is None:
                cpes += [[]] * len(nm)
                continue
            first_rows, inv = combo
            sets = []
            for r in first_rows.tolist():  # the scalar form's own package dict, one per combination
                pk = sm.driver_packages(sdb, p, g, [r])[0]
                pk["_rel"] = int(g["rhrel"][r])
                sets.append(self._cpe_set(recs, cpe_of, pk))
            cpes += [sets[c] for c in inv.tolist()]
        cat = lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt)  # noqa: E731
        names = cat([c[2].astype("S") for c in cols], "S1")
        vers = cat([c[3] for c in cols], "S1")
        plats = cat([np.full(len(c[2]), c[0], np.int32) for c in cols], np.int32)
        self.plat_of = plats.astype(np.int64)
        self.installed = _Decoded(cat([c[4] for c in cols], "S1"))
        self._finish(sm, sdb, recs, want, aid, noarch, plat_drv, plat_gram, names, vers, plats,
                     cat([c[5] for c in cols], np.int32), cat([c[6] for c in cols], np.uint8), cpes)

    @staticmethod
    def _records(sm, sdb, want):
        # Red Hat CPE sets need the "Red Hat CPE" buckets: one Records over every record the
        # sample's keys touch (+ data sources)
        by_root = {}
        for p, nm in want:
            bucket, kind = sdb.plats[p]
            roots = sm.C3_ROOTS.get(kind, [bucket])
            for r in roots:
                by_root.setdefault(r, set()).add(nm)
        by_root["Red Hat CPE"] = {"repository", "nvr", "cpe"}
        return od.Records(sdb.records_for(by_root))

    @staticmethod
    def _cpe_set(recs, cpe_of, pk):
        """The CPE set of a Red Hat package (redhat.go:112-120), cached per (content sets, NVR)."""
        bi = pk.get("BuildInfo")
        cs, nvr = ((od.REDHAT_DEFAULT_CONTENT_SETS.get(str(pk["_rel"]), []), "")
                   if bi is None else (bi.get("ContentSets") or [], f"{bi.get('Nvr', '')}-{bi.get('Arch', '')}"))
        k = (tuple(cs), nvr)
        if k not in cpe_of:
            cpe_of[k] = recs.redhat_cpes(cs, [nvr])
        return cpe_of[k]

    def _finish(self, sm, sdb, recs, want, aid, noarch, plat_drv, plat_gram, names, vers, plats, arches, skip, cpes):
        # entries per wanted key
        ar = _Arena()
        vids = set()
        keys = []  # (plat, name, [entry dicts])
        for (p, nm) in sorted(want, key=lambda x: (x[0], x[1].encode())):
            bucket, kind = sdb.plats[p]
            ents = []
            if kind in sm.LANG_OF:
                eco = ol.LANG[sm.LANG_OF[kind]][0]
                for a in ol.get_advisories_prefix(recs, eco + "::", nm):
                    vul = a.get("VulnerableVersions") or []
                    sec = (a.get("PatchedVersions") or []) + (a.get("UnaffectedVersions") or [])
                    fl = (HAS_VULN if vul else 0) | (HAS_SECURE if sec else 0)
                    if any(v == "" for v in vul + (a.get("PatchedVersions") or [])):
                        fl |= ALWAYS
                    ents.append({"vid": a["VulnerabilityID"], "vul": " || ".join(vul), "sec": " || ".join(sec),
                                 "flags": fl, "adv": a})
            elif kind == "redhat":
                for vid, val in recs.raw("Red Hat", nm):
                    for e in od.decode_redhat(val):
                        for c in e["Cves"]:
                            ents.append({"vid": vid if vid.startswith("CVE-") else c["ID"], "fixed": e["FixedVersion"],
                                         "arches": e["Arches"], "cpes": e["Affected"],
                                         "adv": od.redhat_cve_advisory(vid, e, c)})
            else:
                for a in recs.get(bucket, nm):
                    if kind == "rocky" and a.get("Entries"):
                        for e in a["Entries"]:
                            ents.append({"vid": a["VulnerabilityID"], "fixed": e.get("FixedVersion", ""),
                                         "arches": e.get("Arches") or [], "adv": od.rocky_entry_advisory(a, e)})
                        continue
                    ents.append({"vid": a["VulnerabilityID"], "fixed": a.get("FixedVersion", ""),
                                 "aff": a.get("AffectedVersion", ""), "arches": None, "adv": a})
            for e in ents:
                vids.add(e["vid"])
            keys.append((p, nm, ents))
        vid_of = {v: i for i, v in enumerate(sorted(vids, key=str.encode))}
        self.vid_names = sorted(vids, key=str.encode)
        kn = _Arena()
        key_plat, key_off, key_len, key_begin = [], [], [], [0]
        cols = {c: [] for c in ("fixed_off", "fixed_len", "aff_off", "aff_len", "vul_off", "vul_len", "sec_off",
                                "sec_len", "flags", "vid", "n_arch")}
        ids, ids_begin = [], [0]
        self.entries = []
        for p, nm, ents in keys:
            o, n = kn.put(nm)
            key_plat.append(p)
            key_off.append(o)
            key_len.append(n)
            for e in ents:
                self.entries.append(e)
                for k in ("fixed", "aff", "vul", "sec"):
                    o, n = ar.put(e.get(k) or "")
                    cols[k + "_off"].append(o)
                    cols[k + "_len"].append(n)
                cols["flags"].append(e.get("flags", 0))
                cols["vid"].append(vid_of[e["vid"]])
                arch_list = e.get("arches")
                cols["n_arch"].append(-1 if arch_list is None else len(arch_list))
                ids += [aid(a) for a in (arch_list or [])] + list(e.get("cpes") or [])
                ids_begin.append(len(ids))
            key_begin.append(len(self.entries))
        self.keep = []

        def arr(x, dt):
            a = np.ascontiguousarray(np.asarray(x, dtype=dt))
            self.keep.append(a)
            return a
        self.plat_drv, self.plat_gram = arr(plat_drv, np.int32), arr(plat_gram, np.int32)
        kna, ara = kn.bytes(), ar.bytes()
        self.keep += [kna, ara]
        c = {k: arr(v, np.uint64 if k.endswith("_off") else np.uint32 if k.endswith("_len") or k == "flags" else np.int32)
             for k, v in cols.items()}
        self.db = OrcMixDB(len(plat_drv), _p(self.plat_drv, _I32), _p(self.plat_gram, _I32), len(keys),
                           _p(arr(key_plat, np.int32), _I32), kna, _p(arr(key_off, np.uint64), _U64),
                           _p(arr(key_len, np.uint32), _U32), _p(arr(key_begin, np.int64), _I64), ara,
                           _p(c["fixed_off"], _U64), _p(c["fixed_len"], _U32), _p(c["aff_off"], _U64),
                           _p(c["aff_len"], _U32), _p(c["vul_off"], _U64), _p(c["vul_len"], _U32),
                           _p(c["sec_off"], _U64), _p(c["sec_len"], _U32), _p(c["flags"], _U32), _p(c["vid"], _I32),
                           _p(arr(ids_begin, np.int64), _I64), _p(c["n_arch"], _I32), _p(arr(ids or [0], np.int32), _I32))
        def packed(bs):
            if isinstance(bs, np.ndarray):  # a bytes column: lengths and the arena without a loop
                ln = np.char.str_len(bs).astype(np.uint32) if len(bs) else np.zeros(0, np.uint32)
                off = np.zeros(len(bs), dtype=np.uint64)
                if len(bs):
                    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
                return b"".join(bs.tolist()), off, ln
            ln = np.fromiter((len(x) for x in bs), dtype=np.uint32, count=len(bs))
            off = np.zeros(len(bs), dtype=np.uint64)
            if len(bs):
                off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
            return b"".join(bs), off, ln
        nab, no, nl = packed(names)
        vab, vo, vl = packed(vers)
        self.keep += [nab, vab]
        cb = np.cumsum([0] + [len(x) for x in cpes[1:]]).astype(np.int64)
        cid = [x for s in cpes[1:] for x in s] or [0]
        self.batch = OrcMixBatch(len(names), _p(arr(plats, np.int32), _I32), nab, _p(arr(no, np.uint64), _U64),
                                 _p(arr(nl, np.uint32), _U32), vab, _p(arr(vo, np.uint64), _U64),
                                 _p(arr(vl, np.uint32), _U32), _p(arr(arches, np.int32), _I32), noarch,
                                 _p(arr(skip, np.uint8), _U8), _p(arr(cb, np.int64), _I64), _p(arr(cid, np.int32), _I32))
        self.n = len(names)


def match(prep, n_threads=1, members=False):
    """(package index array, entry index array) in per-package driver output order.  The
    output buffers live in prep and are reused (fresh arrays per call cost page faults that
    serialise the threads).  members: after each Red Hat group's entry come its members as
    -(entry + 1) (ORC_MIX_MEMBERS)."""
    L = _lib()
    L.orc_mix_match_ex.restype = ctypes.c_int64
    L.orc_mix_match_ex.argtypes = [ctypes.POINTER(OrcMixDB), ctypes.POINTER(OrcMixBatch), ctypes.c_int, _I64, _I64,
                                   ctypes.c_int64, ctypes.c_int]
    while True:
        out = getattr(prep, "_out", None)
        if out is None:
            cap = max(1024, prep.n * 8)
            out = prep._out = (np.zeros(cap, dtype=np.int64), np.zeros(cap, dtype=np.int64))
        pk, en = out
        n = L.orc_mix_match_ex(ctypes.byref(prep.db), ctypes.byref(prep.batch), n_threads, _p(pk, _I64),
                               _p(en, _I64), len(pk), 1 if members else 0)
        if n <= len(pk):
            return pk[:n], en[:n]
        prep._out = (np.zeros(int(n), dtype=np.int64), np.zeros(int(n), dtype=np.int64))
