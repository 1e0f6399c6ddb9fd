"""Seeded synthetic DBs + batches for the rpm/apk (BASELINE.json C5) and language-package
(C3) workloads.

Like tools/synth.py (the dpkg C2 workload), the pinned trivy-db cannot be fetched offline,
so the advisory tables are generated with the value formats the drivers read (plain
FixedVersion for alma/oracle/alpine, arch Entries for rocky, Vulnerable/Patched constraint
lists for GHSA-style language buckets) and heavy-tailed advisories per package.  Every
generated package keeps its structured fields, so the same package can be handed to the
batch API (bucket + formatted version + attributes) and, for a sample, to the per-driver
APIs and to the oracle (tests/test_gpu_mix.py).
"""
import json
import os

import numpy as np

from tools.synth import _SYL, _counts

# (batch bucket, kind, DB roots) - OS buckets are their own root; language buckets scan
# every root with the "eco::" prefix (pkg/detector/library/driver.go:124-131)
C5_PLATS = [("Oracle Linux 8", "oracle"), ("Oracle Linux 9", "oracle"), ("Red Hat", "redhat"), ("alma 8", "alma"),
            ("alma 9", "alma"), ("alpine 3.19", "alpine"), ("alpine 3.20", "alpine"), ("rocky 8", "rocky"),
            ("rocky 9", "rocky")]
C5_WEIGHTS = [5, 5, 30, 8, 8, 15, 15, 7, 7]  # RHEL family 70 (Red Hat 30) / Alpine 30
C3_PLATS = [("go::", "go"), ("maven::", "maven"), ("npm::", "npm"), ("pip::", "pip")]
C3_WEIGHTS = [15, 20, 40, 25]
# C4 (BASELINE config 4): one mixed batch, OS packages 60 % / language packages 40 %: the
# dpkg fleet (Debian / Ubuntu), the Red Hat family (Red Hat with CPE sets and modular keys,
# Oracle with ksplice, alma, rocky arch entries), Alpine, and the four lockfile ecosystems
C4_PLATS = [("Oracle Linux 9", "oracle"), ("Red Hat", "redhat"), ("alma 9", "alma"), ("alpine 3.20", "alpine"),
            ("debian 12", "debian"), ("rocky 9", "rocky"), ("ubuntu 22.04", "ubuntu")] + C3_PLATS
C4_WEIGHTS = [4, 12, 6, 8, 14, 6, 10] + [6, 8, 16, 10]
C3_ROOTS = {"go": ["go::GitHub Security Advisory Go", "go::The Go Vulnerability Database"],
            "maven": ["maven::GitHub Security Advisory Maven"], "npm": ["npm::GitHub Security Advisory npm"],
            "pip": ["pip::GitHub Security Advisory pip"]}
DRIVER_OF = {"alma": ("alma", "{}"), "rocky": ("rocky", "{}"), "oracle": ("oracle", "{}"),
             "alpine": ("alpine", "{}.1"), "redhat": ("redhat", "{}"), "debian": ("debian", "{}"),
             "ubuntu": ("ubuntu", "{}")}
DPKG = ("debian", "ubuntu")
# Red Hat (one "Red Hat" bucket for every release; the CPE sets pick the release):
# CPE indices per release and the repositories / NVRs the "Red Hat CPE" buckets map to them
RH_CPES = {7: [0, 1], 8: [2, 3], 9: [4, 5]}
RH_CPE_NAMES = ["cpe:/o:redhat:enterprise_linux:7::server", "cpe:/o:redhat:enterprise_linux:7::client",
                "cpe:/a:redhat:enterprise_linux:8::appstream", "cpe:/o:redhat:enterprise_linux:8::baseos",
                "cpe:/a:redhat:enterprise_linux:9::appstream", "cpe:/o:redhat:enterprise_linux:9::baseos"]
RH_DEFAULT_CS = {7: ["rhel-7-server-rpms", "rhel-7-server-extras-rpms"],
                 8: ["rhel-8-for-x86_64-baseos-rpms", "rhel-8-for-x86_64-appstream-rpms"],
                 9: ["rhel-9-for-x86_64-baseos-rpms", "rhel-9-for-x86_64-appstream-rpms"]}
RH_REPOS = {"rhel-7-server-rpms": [0], "rhel-7-server-extras-rpms": [0, 1],
            "rhel-8-for-x86_64-baseos-rpms": [3], "rhel-8-for-x86_64-appstream-rpms": [2],
            "rhel-9-for-x86_64-baseos-rpms": [5], "rhel-9-for-x86_64-appstream-rpms": [4]}
RH_NVRS = {f"ubi{r}-container-{r}.{k}-{k + 1}-x86_64": RH_CPES[r] for r in (7, 8, 9) for k in range(4)}
LANG_OF = {"go": "gomod", "maven": "jar", "npm": "npm", "pip": "pip"}
ARCHES = [b"x86_64", b"aarch64", b"noarch", b"i686"]


def _os_ver(bucket):
    return bucket.split(" ")[-1]


class MixDB:
    """records: list of (path tuple of str, value str) in bbolt byte order per root."""

    def __init__(self, plats, keys, key_plat, key_base, records, sources):
        self.plats = plats          # [(bucket, kind)]
        self.keys = keys            # [bytes] package names, contiguous per platform
        self.key_plat = key_plat    # np.int32
        self.key_base = key_base    # np.int64 [n_keys, 3]: major, minor, flag (epoch / ksplice / scope)
        self.records = records
        self.sources = sources
        self.plat_keys = [np.nonzero(key_plat == p)[0] for p in range(len(plats))]
        self.n_adv = len(records)

    def put(self, db):
        """Loads the records into a trivy_amd.DB through tvm_db_put_arena."""
        from trivy_amd.batch import arena_of
        for depth, recs in ((3, self.records), (2, self.sources)):
            cols = list(zip(*[tuple(p.encode() for p in path) + (v.encode(),) for path, v in recs]))
            arena, c = arena_of(*cols)
            # tvm_db_put_arena wants the items of one record adjacent: interleave the columns
            off = np.stack([o for o, _ in c], axis=1).reshape(-1)
            lens = np.stack([n for _, n in c], axis=1).reshape(-1)
            db.put_arena(len(recs), depth, arena, np.ascontiguousarray(off), np.ascontiguousarray(lens))
        return db

    @staticmethod
    def vuln_ids_of(mdb):
        """Distinct VulnerabilityIDs the drivers report (Red Hat: the entries' CVE IDs, else
        the bucket key), in byte order - the keys of the "vulnerability" bucket."""
        ids = set()
        for path, v in mdb.records:
            if path[0] == "Red Hat":
                for e in json.loads(v).get("Entries", []):
                    for c in e.get("Cves", []):
                        ids.add(c.get("ID") or path[2])
            elif path[0] != "Red Hat CPE":
                ids.add(path[2])
        return sorted((i.encode() for i in ids))

    def records_for(self, names_by_root):
        """Fixture-format records of the given (root -> names) buckets + data sources."""
        out = [{"path": list(p), "value": v} for p, v in self.sources]
        for path, v in self.records:
            if path[1] in names_by_root.get(path[0], ()):
                out.append({"path": list(path), "value": v})
        return out


def _names(rng, kind, n):
    syl = rng.integers(0, len(_SYL), size=(n, 3))
    out = []
    for i, (a, b, c) in enumerate(syl):
        s = (_SYL[a] + _SYL[b]).decode()
        if kind == "npm":
            out.append(f"@{_SYL[c].decode()}/{s}{i}" if i % 5 == 0 else f"{s}-{i}")
        elif kind == "pip":
            out.append(f"{s}-{_SYL[c].decode()}{i}")
        elif kind == "maven":
            out.append(f"org.{_SYL[c].decode()}:{s}{i}")
        elif kind == "go":
            out.append(f"github.com/{_SYL[c].decode()}/{s}{i}")
        else:
            out.append(f"{s}{_SYL[c].decode()}{i}")
    return sorted(set(out), key=str.encode)


def _rpm(ep, ma, mi, p, r, el, ksplice):
    v = f"{ma}.{mi}.{p}-{r}.el{el}" if not ksplice else f"{ma}.{mi}.{p}-{r}.0.1.ksplice{ksplice}.el{el}"
    return f"{ep}:{v}" if ep else v


def _lib_adv(rng, kind, ma, mi, f):
    lo = f"{ma}.{mi}.0" if rng.random() < 0.6 else f"{ma}.0.0"
    hi = f"{ma}.{mi}.{f}"
    sep = " " if kind == "npm" else ", "
    x = rng.random()
    if x < 0.55:
        vul = [f">={lo}{sep}<{hi}"]
    elif x < 0.85:
        vul = [f"<{hi}"]
    else:
        vul = [f">={lo}{sep}<{hi}", f">={ma + 1}.0.0{sep}<{ma + 1}.{mi}.{f}"]
    adv = {"VulnerableVersions": vul}
    if rng.random() < 0.6:
        adv["PatchedVersions"] = [f">={hi}" if kind != "pip" or rng.random() < 0.5 else hi]
    if rng.random() < 0.1:
        adv = {"PatchedVersions": [f">={hi}"]}
    return adv


def _deb(ep, ma, mi, p, r, ubuntu, tilde):
    v = f"{ma}.{mi}.{p}" + ("~rc1" if tilde else "") + "-" + (f"{r}ubuntu0.{r % 7}" if ubuntu else
                                                             (f"{r}+deb12u{r % 5}" if r % 3 == 0 else f"{r}"))
    return f"{ep}:{v}" if ep else v


def make_mix_db(plats, keys_per_plat, seed=0x5EED, mean_adv=6, max_adv=400):
    rng = np.random.default_rng(seed)
    keys, key_plat, key_base, records, sources = [], [], [], [], []
    for p, (bucket, kind) in enumerate(plats):
        names = _names(rng, kind, keys_per_plat)
        cnt = _counts(rng, len(names), mean_adv, max_adv)
        roots = C3_ROOTS.get(kind, [bucket])
        for r in roots:
            sources.append((("data-source", r), json.dumps({"ID": kind, "Name": f"{r} source", "URL": f"https://{kind}"})))
        el = _os_ver(bucket).split(".")[0]
        by_root = {r: [] for r in roots}
        if kind == "redhat":  # 5 % modular keys: "module:stream::name" (redhat.go:207-220)
            names = sorted(set(names) | {f"{n}:{1 + i % 3}.{i % 5}::{n}" for i, n in enumerate(names) if i % 20 == 7},
                           key=str.encode)
            cnt = _counts(rng, len(names), mean_adv, max_adv)
            for r, cps in RH_REPOS.items():
                records.append((("Red Hat CPE", "repository", r), json.dumps(cps)))
            for r, cps in RH_NVRS.items():
                records.append((("Red Hat CPE", "nvr", r), json.dumps(cps)))
            for i, c in enumerate(RH_CPE_NAMES):
                records.append((("Red Hat CPE", "cpe", str(i)), json.dumps(c)))
        for i, name in enumerate(names):
            ma, mi = int(rng.integers(0, 12)), int(rng.integers(0, 20))
            flag = int(rng.random() < 0.05) * int(rng.integers(1, 3))  # rpm epoch / oracle ksplice
            keys.append(name.encode())
            key_plat.append(p)
            key_base.append((ma, mi, flag))
            for j in range(int(cnt[i])):
                f = int(rng.integers(0, 40))
                r = int(rng.integers(1, 9))
                if kind in DPKG:  # debian.go / ubuntu.go: unfixed (15 %) reported; Debian severity
                    fx = "" if rng.random() < 0.15 else _deb(flag, ma, mi, f, r, kind == "ubuntu", rng.random() < 0.03)
                    val = {"FixedVersion": fx}
                    if rng.random() < 0.25:
                        val.update({"Severity": int(rng.integers(1, 5)), "Status": int(rng.integers(0, 8))})
                elif kind == "alpine":
                    val = {"FixedVersion": f"{ma}.{mi}.{f}-r{r}" if rng.random() > 0.01 else "0"}
                elif kind == "alma":
                    val = {"FixedVersion": _rpm(flag, ma, mi, f, r, el, 0)}
                elif kind == "oracle":
                    ks = flag if rng.random() < 0.5 else 0
                    val = {"FixedVersion": _rpm(0, ma, mi, f, r, el, ks)}
                elif kind == "redhat":
                    rel = int(rng.choice([7, 8, 9]))
                    ent = {"Affected": RH_CPES[rel]}
                    if rng.random() < 0.1:
                        ent["Arches"] = ["x86_64"] if rng.random() < 0.5 else ["aarch64", "x86_64"]
                    pool = max(2, int(cnt[i]) // 2)  # CVEs repeat across a package's advisories: merges
                    cve = f"CVE-{2016 + (i + j) % 8}-{20000 + (i * 7 + j % pool) % 9000}"
                    if rng.random() < 0.25:  # unfixed, keyed by its CVE
                        vid = cve
                        ent.update({"Cves": [{"Severity": int(rng.integers(0, 5))}], "FixedVersion": "",
                                    "Status": int(rng.choice([3, 5, 6]))})
                    else:
                        vid = f"RHSA-{2015 + j % 9}:{1000 + (i * 13 + j) % 9000}"
                        cves = [{"ID": cve, "Severity": int(rng.integers(0, 5))}]
                        if rng.random() < 0.3:
                            cves.append({"ID": f"CVE-{2016 + (i + j + 1) % 8}-{20000 + (i * 7 + (j + 1) % pool) % 9000}",
                                         "Severity": int(rng.integers(0, 5))})
                        ent.update({"Cves": cves, "FixedVersion": _rpm(flag, ma, mi, f, r, f"{rel}_{r % 3}", 0)})
                    val = {"Entries": [ent]}
                elif kind == "rocky":
                    ents = [{"FixedVersion": _rpm(flag, ma, mi, f, r, el, 0), "Arches": ["aarch64", "x86_64"]}]
                    if rng.random() < 0.3:
                        ents.append({"FixedVersion": _rpm(flag, ma, mi, f + 1, r, el, 0), "Arches": ["noarch"]})
                    val = {"Entries": ents}
                else:
                    val = _lib_adv(rng, kind, ma, mi, f)
                if kind != "redhat":
                    vid = f"CVE-{2010 + (j * 31 + i) % 15}-{10000 + j}"
                root = roots[0] if len(roots) == 1 or rng.random() < 0.7 else roots[1]
                by_root[root].append(((root, name, vid), json.dumps(val)))
                if len(roots) > 1 and rng.random() < 0.1:  # the same ID in the other source too
                    other = roots[1] if root == roots[0] else roots[0]
                    by_root[other].append(((other, name, vid), json.dumps(_lib_adv(rng, kind, ma, mi, f))))
        for r in roots:
            seen = {}
            for path, v in by_root[r]:
                seen[path] = v
            records += sorted(seen.items(), key=lambda kv: tuple(x.encode() for x in kv[0]))
    sources.sort(key=lambda kv: kv[0][1].encode())
    return MixDB(plats, keys, np.array(key_plat, dtype=np.int32), np.array(key_base, dtype=np.int64),
                 records, sources)


def _cat(*parts):
    out = parts[0]
    for p in parts[1:]:
        out = np.char.add(out, p)
    return out


def _s(a):
    return np.asarray(a).astype("S")


class MixBatch:
    """Per platform: key index, structured version fields, and the batch-API columns."""

    def __init__(self, groups):
        self.groups = groups  # [(plat, dict of columns)]

    def __len__(self):
        return sum(len(g["key"]) for _, g in self.groups)


def make_mix_batch(db, n, weights, seed, miss=0.25, zipf=2.5):
    rng = np.random.default_rng(seed)
    w = np.asarray(weights, dtype=np.float64)
    counts = rng.multinomial(n, w / w.sum())
    groups = []
    for p, (bucket, kind) in enumerate(db.plats):
        m = int(counts[p])
        ks = db.plat_keys[p]
        if m == 0 or len(ks) == 0:
            continue
        K = len(ks)
        rank = np.minimum((K * rng.random(m) ** zipf).astype(np.int64), K - 1)
        key = ks[(rank * 7919 + p * 1000003) % K]
        base = db.key_base[key]
        ma, mi, flag = base[:, 0], base[:, 1], base[:, 2]
        patch = rng.integers(0, 40, m)
        rel = rng.integers(1, 9, m)
        names = np.array(db.keys, dtype=object)[key].astype("S")
        missing = rng.random(m) < miss
        names = np.where(missing, _cat(b"absent-", _s(np.arange(m))), names)
        mmp = _cat(_s(ma), b".", _s(mi), b".", _s(patch))
        g = {"key": np.where(missing, -1, key), "name": names}
        el = _os_ver(bucket).split(".")[0].encode()
        if kind == "redhat":
            # one RHEL release per image (target of 400 packages): it picks the default
            # content sets; 20 % of images carry BuildInfo (content sets + container NVR)
            nt = (m + 399) // 400
            rel_t = rng.choice([7, 8, 9], nt)
            bi_t = rng.random(nt) < 0.2
            nvr_t = np.array([f"ubi{r}-container-{r}.{k}-{k + 1}" for r, k in zip(rel_t, rng.integers(0, 4, nt))],
                             dtype="S")
            t = np.arange(m) // 400
            keyname = np.array(db.keys, dtype=object)[key].astype("S")
            modular = np.char.find(keyname, b"::") >= 0
            plain = np.array([k.split(b"::")[-1] for k in keyname], dtype="S")
            g["pname"] = np.where(missing, names, plain)
            g["label"] = np.where(modular & ~missing,
                                  _cat(np.array([k.split(b"::")[0] for k in keyname], dtype="S"), b":20210101:abcdef12"),
                                  b"")
            g["rhrel"] = rel_t[t]
            g["bi"] = bi_t[t]
            g["nvr"] = nvr_t[t]
            relv = _cat(_s(rel), b".el", _s(rel_t[t]), b"_", _s(rel % 3))
            epoch = np.where(rng.random(m) < 0.9, flag, 0)
            g["version"], g["rel"], g["epoch"] = mmp, relv, epoch
            full = _cat(mmp, b"-", relv)
            g["ver"] = np.where(epoch > 0, _cat(_s(epoch), b":", full), full)
            g["arch"] = np.array(ARCHES, dtype="S")[rng.choice(4, m, p=[0.6, 0.15, 0.2, 0.05])]
        elif kind in DPKG:  # SrcVersion / SrcRelease / SrcEpoch formatted as utils.FormatSrcVersion
            up = np.where(rng.random(m) < 0.03, _cat(mmp, b"~rc1"), mmp)
            if kind == "ubuntu":
                relv = _cat(_s(rel), b"ubuntu0.", _s(rel % 7))
            else:
                relv = np.where(rel % 3 == 0, _cat(_s(rel), b"+deb12u", _s(rel % 5)), _s(rel))
            epoch = np.where(rng.random(m) < 0.9, flag, 0)
            g["version"], g["rel"], g["epoch"] = up, relv, epoch
            full = _cat(up, b"-", relv)
            g["ver"] = np.where(epoch > 0, _cat(_s(epoch), b":", full), full)
        elif kind == "alpine":
            g["ver"] = _cat(mmp, b"-r", _s(rel))
            g["rel"] = np.full(m, b"", dtype="S1")
            g["epoch"] = np.zeros(m, dtype=np.int64)
            g["version"] = g["ver"]
        else:
            if kind == "oracle":
                ks = np.where((flag > 0) & (rng.random(m) < 0.5), flag, 0)
                relv = np.where(ks > 0, _cat(_s(rel), b".0.1.ksplice", _s(ks), b".el", el), _cat(_s(rel), b".el", el))
                epoch = np.zeros(m, dtype=np.int64)
            else:
                relv = _cat(_s(rel), b".el", el)
                epoch = np.where(rng.random(m) < 0.9, flag, 0)
            g["version"], g["rel"], g["epoch"] = mmp, relv, epoch
            full = _cat(mmp, b"-", relv)
            g["ver"] = np.where(epoch > 0, _cat(_s(epoch), b":", full), full)
            if kind == "rocky":
                g["arch"] = np.array(ARCHES, dtype="S")[rng.choice(4, m, p=[0.6, 0.25, 0.1, 0.05])]
        if kind in LANG_OF:
            v = mmp
            pre = rng.random(m)
            if kind == "npm":
                v = np.where(pre < 0.03, _cat(v, b"-beta.", _s(rel)), v)
            elif kind == "pip":
                v = np.where(pre < 0.03, _cat(v, b"rc", _s(rel)), np.where(pre < 0.05, _cat(v, b".post1"), v))
            elif kind == "maven":  # TVM_SYNTH_MAVEN_PRE: another "-rcN" share (measurement only)
                v = np.where(pre < float(os.environ.get("TVM_SYNTH_MAVEN_PRE", "0.03")), _cat(v, b"-rc", _s(rel)), v)
            elif kind == "go":
                v = np.where(pre < 0.5, _cat(b"v", v), v)
            g["ver"] = g["version"] = v
        groups.append((p, g))
    return MixBatch(groups)


def rh_cpe_key(g, i):
    """(content sets, NVR) of Red Hat package i (redhat.go:112-120)."""
    r = int(g["rhrel"][i])
    if g["bi"][i]:
        return tuple(RH_DEFAULT_CS[r]), g["nvr"][i].decode() + "-x86_64"
    return tuple(RH_DEFAULT_CS[r]), ""


def add_slice(mb, db, p, g, lo, hi):
    """Adds rows [lo, hi) of group g (platform p) to a MatchBatch; returns the first index."""
    bucket, kind = db.plats[p]
    arches = g["arch"][lo:hi] if "arch" in g else None
    if kind != "redhat":
        return mb.add_many(bucket, g["name"][lo:hi], g["ver"][lo:hi], arches=arches, ksplice=(kind == "oracle"))
    ids, sets = np.zeros(hi - lo, dtype=np.uint32), {}
    for i in range(lo, hi):
        k = rh_cpe_key(g, i)
        if k not in sets:
            sets[k] = mb.cpe_set(list(k[0]), k[1])
        ids[i - lo] = sets[k]
    return mb.add_many(bucket, g["name"][lo:hi], g["ver"][lo:hi], arches=arches, cpe_sets=ids)


def add_to(mb, db, batch):
    """Adds every group to a trivy_amd.batch.MatchBatch; returns [(plat, first index)]."""
    return [(p, add_slice(mb, db, p, g, 0, len(g["key"]))) for p, g in batch.groups]


def driver_packages(db, p, g, idx):
    """The packages at rows idx of group g as the drivers' package dicts (ftypes.Package)."""
    bucket, kind = db.plats[p]
    pk = []
    for i in idx:
        name = g["name"][i].decode()
        if kind in LANG_OF:
            pk.append({"Name": name, "Version": g["ver"][i].decode(), "ID": f"p{i}"})
            continue
        if kind == "redhat":
            name = g["pname"][i].decode()
        d = {"ID": f"p{i}", "Name": name, "Version": g["version"][i].decode(), "Release": g["rel"][i].decode(),
             "Epoch": int(g["epoch"][i]), "SrcName": name, "SrcVersion": g["version"][i].decode(),
             "SrcRelease": g["rel"][i].decode(), "SrcEpoch": int(g["epoch"][i])}
        if "arch" in g:
            d["Arch"] = g["arch"][i].decode()
        if kind == "redhat":
            if g["label"][i]:
                d["Modularitylabel"] = g["label"][i].decode()
            if g["bi"][i]:
                cs, nvr = rh_cpe_key(g, i)
                d["BuildInfo"] = {"ContentSets": list(cs), "Nvr": g["nvr"][i].decode(), "Arch": "x86_64"}
        pk.append(d)
    return pk


class BulkCols:
    """A MixBatch's columns in the form tvm_batch_add_targets_attrs takes them, built once per
    batch: one arena (names, versions, arches), targets of `per_target` packages cut from each
    group (images / lockfiles), per target its bucket and attribute flags (arch for Red Hat /
    Oracle / Rocky, ksplice for Oracle, the CPE set for Red Hat), and per Red Hat package the
    index of its (content sets, NVR) combination (registered per batch: cpe_set ids are
    per-batch).  Package order = add_to's."""

    def __init__(self, db, batch, per_target=400):
        from trivy_amd.batch import ATTR_ARCH, ATTR_CPESET, ATTR_KSPLICE, arena_of
        names, vers, arches = [], [], []
        buckets, flags, ends = [], [], []
        combo = []  # per package: (content sets, NVR) combination index, -1 = none
        self.combos = {}
        o = 0
        for p, g in batch.groups:
            bucket, kind = db.plats[p]
            m = len(g["key"])
            names.append(g["name"])
            vers.append(g["ver"])
            arches.append(g["arch"] if "arch" in g else np.full(m, b"", dtype="S1"))
            f = (ATTR_ARCH if "arch" in g else 0) | (ATTR_KSPLICE if kind == "oracle" else 0) | \
                (ATTR_CPESET if kind == "redhat" else 0)
            cidx = np.full(m, -1, dtype=np.int64)
            if kind == "redhat":
                # (release, NVR when BuildInfo) -> combination index, vectorised over the group
                _, first_i, inv = np.unique(np.char.add(np.char.add(g["rhrel"].astype("S"), b"|"),
                                                        np.where(g["bi"], g["nvr"], b"")), return_index=True,
                                            return_inverse=True)
                for i in first_i.tolist():
                    self.combos.setdefault(rh_cpe_key(g, i), len(self.combos))
                cidx = np.array([self.combos[rh_cpe_key(g, i)] for i in first_i.tolist()], dtype=np.int64)[inv]
            combo.append(cidx)
            for t0 in range(0, m, per_target):
                buckets.append(bucket)
                flags.append(f)
                ends.append(o + min(m, t0 + per_target))
            o += m
        self.n = o
        self.buckets, self.flags = buckets, np.array(flags, dtype=np.uint32)
        self.ends = np.array(ends, dtype=np.uint64)
        self.combo = np.concatenate(combo) if combo else np.zeros(0, np.int64)
        cat = lambda xs: np.concatenate(xs) if xs else np.zeros(0, dtype="S1")  # noqa: E731
        self.arena, ((self.noff, self.nlen), (self.voff, self.vlen), (self.aoff, self.alen)) = \
            arena_of(cat(names), cat(vers), cat(arches))

    def add(self, mb, lo=0, hi=None):
        """Adds the whole targets inside packages [lo, hi) to a MatchBatch in one call; returns
        the first index."""
        hi = self.n if hi is None else hi
        starts = np.concatenate([[0], self.ends[:-1]]).astype(np.int64)
        sel = np.nonzero((starts >= lo) & (self.ends.astype(np.int64) <= hi))[0]
        if not len(sel):
            return len(mb)
        a, z = int(starts[sel[0]]), int(self.ends[sel[-1]])
        ids = {}
        cs = self.combo[a:z]
        sets = np.zeros(z - a, dtype=np.uint32)
        if (cs >= 0).any():
            inv = {v: k for k, v in self.combos.items()}
            for c in np.unique(cs[cs >= 0]).tolist():
                k = inv[c]
                ids[c] = mb.cpe_set(list(k[0]), k[1])
            lut = np.zeros(len(self.combos), dtype=np.uint32)
            for c, i in ids.items():
                lut[c] = i
            sets = np.where(cs >= 0, lut[np.maximum(cs, 0)], 0).astype(np.uint32)
        return mb.add_targets([self.buckets[t] for t in sel.tolist()], self.ends[sel] - np.uint64(a), self.arena,
                              self.noff[a:z], self.nlen[a:z], self.voff[a:z], self.vlen[a:z],
                              flags=self.flags[sel], arch_off=self.aoff[a:z], arch_len=self.alen[a:z], cpe_sets=sets)

