"""Seeded synthetic trivy-db + package batches (bench and large parity tests).

The pinned trivy-db (ghcr.io/aquasecurity/trivy-db:2) cannot be fetched offline
(SURVEY.md §7 hard part 6), so throughput is measured on a generated DB with the
distributions of SURVEY.md §8d, and parity at scale is checked against the oracle
on the same generated data.

Everything is emitted pre-sorted in bbolt byte order (platform buckets, package
buckets, vulnerability IDs), so the engine's global advisory index equals the CSR
index here - tests can compare (package, advisory) pairs directly.
"""
import numpy as np

SEED_DB = 0x7157DB

DEBIAN_DS = b'{"ID":"debian","Name":"Debian Security Tracker","URL":"https://salsa.debian.org/security-tracker-team/security-tracker"}'
UBUNTU_DS = b'{"ID":"ubuntu","Name":"Ubuntu CVE Tracker","URL":"https://git.launchpad.net/ubuntu-cve-tracker"}'
AMAZON_DS = b'{"ID":"amazon","Name":"Amazon Linux Security Center","URL":"https://alas.aws.amazon.com/"}'

_SYL = [b"lib", b"py", b"gnu", b"x", b"ssl", b"core", b"util", b"net", b"font", b"perl", b"gtk", b"qt", b"db",
        b"cups", b"krb", b"sql", b"z", b"bz", b"xml", b"curl", b"dev", b"data", b"doc", b"common", b"bin"]


def _counts(rng, n, mean, cap):
    """Heavy-tailed advisories-per-key with the requested mean (Pareto tail, >= 1)."""
    c = 1 + np.floor(rng.pareto(1.6, n) * (mean - 1) * 0.6)
    c = np.minimum(c, cap).astype(np.int64)
    c = np.maximum(c, 1)
    return c


class SynthDB:
    """platforms: list of root bucket names (sorted).  CSR: key -> advisories."""

    def __init__(self, platforms, key_plat, key_names, adv_begin, adv_vid, adv_fixed, key_base):
        self.platforms = platforms
        self.key_plat = key_plat
        self.key_names = key_names
        self.adv_begin = adv_begin
        self.adv_vid = adv_vid
        self.adv_fixed = adv_fixed
        self.key_base = key_base
        self.plat_keys = [np.nonzero(key_plat == p)[0] for p in range(len(platforms))]

    @property
    def n_adv(self):
        return int(self.adv_begin[-1])

    @staticmethod
    def adv_detail(a):
        """(Status, Severity) of advisory a when records carry detail (deterministic)."""
        return (a % 8 if a % 3 == 0 else 0), (a % 5 if a % 4 == 0 else 0)

    def records_arena(self, poison_keys=(), detail=False):
        """(n, depth=3, arena, off, len) for tvm_db_put_arena, plus data-source records.
        detail=True adds adv_detail()'s Status/Severity to the advisory values."""
        items = []
        poison = set(int(k) for k in poison_keys)
        for k in range(len(self.key_names)):
            root = self.platforms[self.key_plat[k]].encode()
            name = self.key_names[k]
            for a in range(self.adv_begin[k], self.adv_begin[k + 1]):
                val = b'{"FixedVersion":"' + self.adv_fixed[a] + b'"}'
                if detail:
                    st, sev = self.adv_detail(a)
                    val = val[:-1] + b',"Status":%d,"Severity":%d}' % (st, sev)
                if k in poison and a == self.adv_begin[k]:
                    val = b'{"FixedVersion":["bad"]}'
                items += [root, name, self.adv_vid[a], val]
        return _arena(items, 3)

    def source_arena(self):
        items = []
        for p in self.platforms:
            ds = DEBIAN_DS if p.startswith("debian") else UBUNTU_DS if p.startswith("ubuntu") else AMAZON_DS
            items += [b"data-source", p.encode(), ds]
        return _arena(items, 2)

    def vuln_ids(self):
        """Distinct vulnerability IDs of the DB, in bbolt byte order."""
        return sorted(set(self.adv_vid))


def _arena(items, depth):
    lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
    off = np.zeros(len(items), dtype=np.uint64)
    if len(items):
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return len(items) // (depth + 1), depth, b"".join(items), off, lens


def _deb_version(epoch, major, minor, patch, rev, ubuntu, tilde, dfsg):
    v = b"%d.%d.%d" % (major, minor, patch)
    if tilde:
        v += b"~rc%d" % tilde
    if dfsg:
        v += b"+dfsg"
    v += (b"-%dubuntu0.%d" % (rev, rev % 7)) if ubuntu else (b"-%d+deb12u%d" % (rev, rev % 5) if rev % 3 == 0 else b"-%d" % rev)
    if epoch:
        v = b"%d:" % epoch + v
    return v


def make_db(platforms, keys_per_plat, seed=SEED_DB, mean_adv=12, max_adv=5000, unfixed=0.15):
    """dpkg-family DB (debian/ubuntu/amazon buckets)."""
    rng = np.random.default_rng(seed)
    platforms = sorted(platforms)
    key_plat, key_names, counts, bases = [], [], [], []
    for p, root in enumerate(platforms):
        n = keys_per_plat
        syl = rng.integers(0, len(_SYL), size=(n, 2))
        names = sorted({_SYL[a] + _SYL[b] + b"%d" % i for i, (a, b) in enumerate(syl)} | {b"linux"})
        c = _counts(rng, len(names), mean_adv, max_adv)
        c[names.index(b"linux")] = max_adv  # the heavy key of every real distro
        key_plat += [p] * len(names)
        key_names += names
        counts.append(c)
        for _ in names:
            bases.append((int(rng.random() < 0.05) * int(rng.integers(1, 4)), int(rng.integers(0, 20)),
                          int(rng.integers(0, 30)), int(rng.random() < 0.1), root.startswith("ubuntu")))
    counts = np.concatenate(counts)
    adv_begin = np.zeros(len(key_names) + 1, dtype=np.int64)
    adv_begin[1:] = np.cumsum(counts)
    n_adv = int(adv_begin[-1])
    patch = rng.integers(0, 40, n_adv)
    rev = rng.integers(1, 9, n_adv)
    tilde = (rng.random(n_adv) < 0.03) * rng.integers(1, 4, n_adv)
    is_unfixed = rng.random(n_adv) < unfixed
    adv_vid, adv_fixed = [], []
    for k in range(len(key_names)):
        b, e = int(adv_begin[k]), int(adv_begin[k + 1])
        ep, ma, mi, dfsg, ubu = bases[k]
        ids = sorted(b"CVE-%d-%d" % (2000 + (j * 7919 + k) % 25, 1000 + j) for j in range(e - b))
        adv_vid += ids
        for a in range(b, e):
            adv_fixed.append(b"" if is_unfixed[a] else
                             _deb_version(ep, ma, mi, int(patch[a]), int(rev[a]), ubu, int(tilde[a]), dfsg))
    return SynthDB(platforms, np.array(key_plat, dtype=np.int32), key_names, adv_begin, adv_vid, adv_fixed, bases)


class SynthBatch:
    def __init__(self, plat, names, versions, target_bounds):
        self.plat = plat            # np.int32 per package (-1 absent bucket)
        self.names = names          # list[bytes]
        self.versions = versions    # list[bytes]
        self.targets = target_bounds  # [(plat, begin, end)] one entry per SBOM/target

    def __len__(self):
        return len(self.names)

    def arena(self):
        """arena bytes + name/version offsets and lengths (interleaved name, version)."""
        items = [x for pair in zip(self.names, self.versions) for x in pair]
        lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
        off = np.zeros(len(items), dtype=np.uint64)
        if len(items):
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        return b"".join(items), off[0::2].copy(), lens[0::2].copy(), off[1::2].copy(), lens[1::2].copy()


def make_batch(db, n_targets, pkgs_per_target, plat_weights, seed, miss=0.25, zipf=2.5, invalid=0.002,
               long_versions=0.0):
    """SBOM-like batch: each target draws one platform, then packages over its keys (numpy-vectorised)."""
    rng = np.random.default_rng(seed)
    w = np.asarray(plat_weights, dtype=np.float64)
    w = w / w.sum()
    t_plat = rng.choice(len(db.platforms), size=n_targets, p=w)
    n = n_targets * pkgs_per_target
    plat = np.repeat(t_plat, pkgs_per_target).astype(np.int32)
    start = np.array([int(k[0]) if len(k) else 0 for k in db.plat_keys], dtype=np.int64)
    K = np.array([len(k) for k in db.plat_keys], dtype=np.int64)[plat]
    # popularity skew without a single dominant key: P(rank < r) = (r / K) ** (1 / zipf)
    rank = np.minimum((K * rng.random(n) ** zipf).astype(np.int64), K - 1)
    local = (rank * 7919 + (plat.astype(np.int64) * 1000003) % K) % K
    kidx = start[plat] + local  # keys of one platform are contiguous (make_db emits them per platform)
    missing = rng.random(n) < miss
    patch = rng.integers(0, 40, n)
    rev = rng.integers(1, 9, n)
    bad = rng.random(n) < invalid
    longv = rng.random(n) < long_versions
    base = np.array(db.key_base, dtype=np.int64)  # (ep, major, minor, dfsg, ubuntu) per key
    kb = base[kidx]
    prefix = np.array([(b"%d:" % e if e else b"") + b"%d.%d." % (ma, mi) for e, ma, mi, _, _ in db.key_base],
                      dtype=object)[kidx].astype("S")
    v = np.char.add(prefix, patch.astype("S"))
    v = np.char.add(v, np.where(kb[:, 3] == 1, b"+dfsg", b"").astype("S"))
    v = np.char.add(np.char.add(v, b"-"), rev.astype("S"))
    deb_tail = np.where(rev % 3 == 0, np.char.add(b"+deb12u", (rev % 5).astype("S")), b"")
    ubu_tail = np.char.add(b"ubuntu0.", (rev % 7).astype("S"))
    v = np.char.add(v, np.where(kb[:, 4] == 1, ubu_tail, deb_tail).astype("S"))
    v = np.where(bad, np.char.add(b"x", v), v)  # upstream must start with a digit: parse error
    if long_versions:
        v = np.where(longv, np.char.add(v, b"+" + b".".join(b"%d" % j for j in range(30))), v)
    names = np.array(db.key_names, dtype=object)[kidx]
    miss_idx = np.nonzero(missing)[0]
    names[miss_idx] = [b"absent-%d" % i for i in miss_idx]
    targets = [(int(t_plat[t]), t * pkgs_per_target, (t + 1) * pkgs_per_target) for t in range(n_targets)]
    return SynthBatch(plat, names.tolist(), v.tolist(), targets)
