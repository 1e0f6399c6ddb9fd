"""GPU: FillInfo (vulnerability.go:60-157) through the C-ABI, bit-exact against the
reference's own vectors and against the oracle (oracle/vulninfo.py):

* every TestClient_FillInfo case (vulnerability_test.go:17-283);
* the FillInfo fields of every vulnerability of the integration goldens, in one launch;
* seeded random DBs/inputs covering every branch (unknown IDs, undecodable records,
  vendor/GHSA/NVD/DB severity, package-specific severities, all URL rules, long IDs);
* the batch path: FillInfo fused behind a device-resident match list, per pair against
  the oracle applied to the driver's DetectedVulnerability for that pair.
"""
import json

import numpy as np
import pytest

import fillinfo_golden as fg
import oracle.vulninfo as vi

pytestmark = pytest.mark.gpu

_TABLE = fg.table_cases()


def _engine(records):
    import trivy_amd
    db = trivy_amd.DB()
    db.put_records(records)
    return trivy_amd.Engine(db, 0)


@pytest.mark.parametrize("case", _TABLE, ids=[c[0] for c in _TABLE])
def test_fillinfo_table(case):
    from trivy_amd.vulnerability import Client
    name, fixtures, vulns, want = case
    got = Client(_engine(fg.load_records(fixtures))).fill_info(vulns)
    assert [fg.norm(v) for v in got] == [fg.norm(v) for v in want], name


def test_fillinfo_integration_goldens():
    from trivy_amd.vulnerability import Client
    cases = fg.integration_cases()
    got = Client(_engine(fg.load_records(fg.integration_fixtures()))).fill_info([c[1] for c in cases])
    assert len(got) == len(cases) >= 100
    for (cid, _inp, want), g in zip(cases, got):
        assert fg.got_form(g) == fg.want_form(want), cid


def _random_case(seed, n_vulns=400, n_items=3000):
    from tools.synth_vuln import SOURCES, vuln_values
    rng = np.random.default_rng(seed)
    prefixes = ["CVE-2021-", "GHSA-", "RUSTSEC-2020-", "TEMP-000", "ALAS-2023-", "DSA-", "USN-", "SUSE-SU-", "ELSA-",
                "NSWG-ECO-", "OSVDB-", "cve-"]
    ids = []
    for i in range(n_vulns):
        p = prefixes[int(rng.integers(0, len(prefixes)))]
        ids.append((p + str(i) + ("-" + "x" * int(rng.integers(20, 40)) if i % 37 == 0 else "")).encode())
    ids = sorted(set(ids))
    recs = [{"path": ["vulnerability", k.decode()], "value": v.decode()} for k, v in vuln_values(ids, seed)]
    unknown = [b"CVE-1999-%d" % i for i in range(20)] + [b"", b"GHSA-unknown"]
    pool = ids + unknown
    items = []
    for _ in range(n_items):
        v = {"VulnerabilityID": pool[int(rng.integers(0, len(pool)))].decode()}
        r = rng.random()
        if r < 0.8:
            v["DataSource"] = {"ID": SOURCES[int(rng.integers(0, len(SOURCES)))] if r < 0.75 else "other",
                               "Name": "n"}
        if rng.random() < 0.5:
            v["FixedVersion"] = "1.2.%d" % int(rng.integers(0, 9))
        if rng.random() < 0.3:
            v["Status"] = int(rng.integers(0, 8))
        if rng.random() < 0.15:
            v["SeveritySource"] = ["debian", "redhat", "nvd"][int(rng.integers(0, 3))]
            v["Vulnerability"] = {"Severity": ["LOW", "HIGH", "CRITICAL", "bogus", ""][int(rng.integers(0, 5))]}
        items.append(v)
    return recs, items


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fillinfo_random_vs_oracle(seed):
    from trivy_amd.vulnerability import Client
    recs, items = _random_case(seed)
    got = Client(_engine(recs)).fill_info(items)
    want = vi.fill_info(vi.vulnerability_bucket(recs), items)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert fg.norm(g) == fg.norm(w), (i, items[i])


def test_fillinfo_empty_and_no_bucket():
    from trivy_amd.vulnerability import Client
    c = Client(_engine([{"path": ["data-source", "x"], "value": "{}"}]))
    assert c.fill_info([]) == []
    got = c.fill_info([{"VulnerabilityID": "CVE-1-1", "FixedVersion": "1"}, {"VulnerabilityID": "X", "Status": 5}])
    assert got == [{"VulnerabilityID": "CVE-1-1", "FixedVersion": "1", "Status": 3},
                   {"VulnerabilityID": "X", "Status": 5}]


def test_match_fill_batch_vs_oracle():
    """Batch path: match kernel -> fill kernel on the same stream; every pair's decision
    equals the oracle's FillInfo of that pair's debian/ubuntu DetectedVulnerability."""
    import trivy_amd
    from trivy_amd._lib import lib
    from trivy_amd.batch import MatchBatch
    from tools.synth import DEBIAN_DS, UBUNTU_DS, make_batch, make_db
    from tools.synth_vuln import vuln_arena, vuln_values

    sdb = make_db(["debian 12", "ubuntu 22.04"], 1500, seed=5)
    ids = sdb.vuln_ids()
    db = trivy_amd.DB()
    for n, depth, arena, off, lens in (sdb.records_arena(detail=True), sdb.source_arena(), vuln_arena(ids, 5)):
        assert lib().tvm_db_put_arena(db.h, n, depth, arena, off.ctypes.data, lens.ctypes.data) == 0
    eng = trivy_amd.Engine(db, 0)
    batch = make_batch(sdb, 12, 300, [1, 1], seed=5)
    mb = MatchBatch(eng)
    arena, noff, nlen, voff, vlen = batch.arena()
    for p, b0, b1 in batch.targets:
        mb.add_arena(sdb.platforms[p], b1 - b0, arena, noff[b0:], nlen[b0:], voff[b0:], vlen[b0:])
    total, errp, _ = mb.run()
    assert errp == -1 and total > 1000
    pairs = mb.pairs()
    dec = mb.fill().fill_decisions()
    assert dec.shape == (len(pairs), 4)

    bucket = {k.decode(): v.decode() for k, v in vuln_values(ids, 5)}
    rec_of = {k.decode(): i for i, k in enumerate(ids)}
    ds_of = {p: json.loads((DEBIAN_DS if p.startswith("debian") else UBUNTU_DS).decode()) for p in sdb.platforms}
    pkg_plat = np.zeros(len(batch), dtype=np.int64)
    for p, b0, b1 in batch.targets:
        pkg_plat[b0:b1] = p
    names = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]
    for (pk, adv), d in zip(pairs.tolist(), dec.tolist()):
        plat = sdb.platforms[pkg_plat[pk]]
        vid = sdb.adv_vid[adv].decode()
        v = {"VulnerabilityID": vid, "DataSource": ds_of[plat]}
        if sdb.adv_fixed[adv]:
            v["FixedVersion"] = sdb.adv_fixed[adv].decode()
        if plat.startswith("debian"):  # debian.go:89-98
            st, sev = sdb.adv_detail(adv)
            if st:
                v["Status"] = st
            if sev:
                v["SeveritySource"] = "debian"
                v["Vulnerability"] = {"Severity": names[sev]}
        w = vi.fill_info(bucket, [v])[0]
        assert d[1] == w["Status"], (pk, adv)
        try:
            found = vid in bucket and vi.decode_vulnerability(bucket[vid]) is not None
        except vi.DecodeError:
            found = False
        if not found:
            assert d[0] == 0xFFFFFFFF, (pk, adv)  # GetVulnerability error: skipped
            continue
        assert d[0] == rec_of[vid]
        code, src = d[2] & 0xFFFF, d[2] >> 16
        sev = (v["Vulnerability"]["Severity"] if code == 0xFFFD else
               json.loads(bucket[vid]).get("Severity", "") if code == 0xFFFE else
               names[code] if code < 5 else "UNKNOWN")
        assert sev == w["Vulnerability"].get("Severity", ""), (pk, adv, d)
        ssrc = v.get("SeveritySource", "") if code == 0xFFFD else lib().tvm_fill_source_name(eng.h, src).decode()
        assert ssrc == w.get("SeveritySource", ""), (pk, adv, d)
        assert d[3] >> 28 == 1 and w["PrimaryURL"] == "https://avd.aquasec.com/nvd/" + vid.lower()
    mb.close()


def _filter_fixture(seed=9, copies=0):
    """A multi-result batch with repeated (name, version) packages inside results, FillInfo
    run, plus the oracle's view of every result's DetectedVulnerability list.  copies: every
    result also ends with that many more copies of its first three packages (duplicated
    lockfile rows: dedup groups of hundreds of packages)."""
    import trivy_amd
    from trivy_amd._lib import lib
    from trivy_amd.batch import MatchBatch
    from tools.synth import DEBIAN_DS, UBUNTU_DS, SynthBatch, make_batch, make_db
    from tools.synth_vuln import vuln_arena, vuln_values

    sdb = make_db(["debian 12", "ubuntu 22.04"], 800, seed=seed)
    ids = sdb.vuln_ids()
    db = trivy_amd.DB()
    for n, depth, arena, off, lens in (sdb.records_arena(detail=True), sdb.source_arena(), vuln_arena(ids, seed)):
        assert lib().tvm_db_put_arena(db.h, n, depth, arena, off.ctypes.data, lens.ctypes.data) == 0
    eng = trivy_amd.Engine(db, 0)
    b0 = make_batch(sdb, 30, 120, [1, 1], seed=seed)
    # duplicate a quarter of every result's packages (same name and version) at its end
    plat, names, vers, targets = [], [], [], []
    for p, s, e in b0.targets:
        idx = list(range(s, e)) + list(range(s, e, 4)) + [s + (k % 3) for k in range(copies)]
        start = len(names)
        for i in idx:
            plat.append(p)
            names.append(b0.names[i])
            vers.append(b0.versions[i])
        targets.append((p, start, len(names)))
    batch = SynthBatch(np.array(plat, dtype=np.int32), names, vers, targets)
    mb = MatchBatch(eng)
    arena, noff, nlen, voff, vlen = batch.arena()
    for p, s, e in batch.targets:
        mb.add_arena(sdb.platforms[p], e - s, arena, noff[s:], nlen[s:], voff[s:], vlen[s:])
    mb.result_bounds = [(s, e) for _, s, e in batch.targets]
    total, errp, _ = mb.run()
    assert errp == -1 and total > 1000
    pairs = mb.pairs()
    mb.fill()
    bucket = {k.decode(): v.decode() for k, v in vuln_values(ids, seed)}
    names5 = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]
    ds_of = {p: json.loads((DEBIAN_DS if p.startswith("debian") else UBUNTU_DS).decode()) for p in sdb.platforms}
    by_target = [[] for _ in batch.targets]
    tgt_of = np.zeros(len(batch), dtype=np.int64)
    for t, (_, s, e) in enumerate(batch.targets):
        tgt_of[s:e] = t
    for pk, adv in pairs.tolist():  # detection order: package, then advisory
        t = tgt_of[pk]
        plat = sdb.platforms[batch.targets[t][0]]
        v = {"VulnerabilityID": sdb.adv_vid[adv].decode(), "PkgName": batch.names[pk].decode(),
             "InstalledVersion": batch.versions[pk].decode(), "DataSource": ds_of[plat], "_pair": (pk, adv)}
        if sdb.adv_fixed[adv]:
            v["FixedVersion"] = sdb.adv_fixed[adv].decode()
        if plat.startswith("debian"):
            st, sev = sdb.adv_detail(adv)
            if st:
                v["Status"] = st
            if sev:
                v["SeveritySource"] = "debian"
                v["Vulnerability"] = {"Severity": names5[sev]}
        by_target[t].append(v)
    return mb, bucket, by_target, sdb


@pytest.mark.parametrize("opts", [
    dict(severities=("UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL")),
    dict(severities=("HIGH", "CRITICAL"), ignore_statuses=(5, 7)),
    dict(severities=("LOW", "MEDIUM", "HIGH"), ignore_statuses=(2,), ignore_ids=("__first3__",)),
])
def test_match_filter_batch_vs_oracle(opts):
    """Batch result.Filter on the GPU (severity, status, ignore IDs, dedup keeping the
    greater FixedVersion, BySeverity order) equals oracle/filter.py per result, in order."""
    import oracle.filter as of
    mb, bucket, by_target, sdb = _filter_fixture()
    opts = dict(opts)
    if opts.get("ignore_ids") == ("__first3__",):
        opts["ignore_ids"] = tuple(v["VulnerabilityID"] for v in by_target[0][:3]) + ("CVE-0000-none",)
    n = mb.filter(mb.filter_opts(**opts))
    got = mb.filtered_pairs(n).tolist()
    findings = [{"ID": i, "Paths": [], "PURLs": [], "ExpiredAt": None, "Statement": ""}
                for i in opts.get("ignore_ids", ())]
    want, want_ign = [], []
    for vulns in by_target:
        filled = vi.fill_info(bucket, [{k: x for k, x in v.items() if k != "_pair"} for v in vulns])
        for f, v in zip(filled, vulns):
            f["_pair"] = v["_pair"]
        kept, ign = of.filter_vulnerabilities("", filled, list(opts["severities"]), opts.get("ignore_statuses", ()),
                                              findings)
        want += kept or []
        want_ign += [list(v["_pair"]) + [findings.index(f)] for v, f in ign]
    assert len(got) == len(want), (len(got), len(want))
    # exact pairs: the dedup winner is the reference's first-seen package
    assert got == [list(w["_pair"]) for w in want]
    assert mb.ignored_findings().tolist() == want_ign and (not findings or want_ign)
    mb.close()


def test_match_filter_many_duplicates_vs_oracle():
    """Dedup groups of ~170 packages per result (500 extra copies of three packages): the
    kept pairs equal oracle/filter.py, and a call stays fast - a repeating package's pair scans
    the other packages of its dedup key until one beats it, and copies with the same list are
    beaten by the first copy (filter.hip beaten_by; O(K M log M) for K copies of M pairs)."""
    import time

    import oracle.filter as of
    mb, bucket, by_target, sdb = _filter_fixture(seed=4, copies=500)
    opts = mb.filter_opts()
    n = mb.filter(opts)
    got = mb.filtered_pairs(n).tolist()
    want = []
    for vulns in by_target:
        filled = vi.fill_info(bucket, [{k: x for k, x in v.items() if k != "_pair"} for v in vulns])
        for f, v in zip(filled, vulns):
            f["_pair"] = v["_pair"]
        kept, _ = of.filter_vulnerabilities("", filled, ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"])
        want += kept or []
    assert got == [list(w["_pair"]) for w in want] and len(got) > 1000
    t0 = time.perf_counter()
    ms = mb.filter_time(opts, 5)
    assert ms < 50 and time.perf_counter() - t0 < 5, ms
    mb.close()


@pytest.mark.parametrize("kind", ["openvex", "cyclonedx", "csaf"])
def test_match_filter_batch_vex_vs_oracle(kind):
    """Batch result.Filter + the VEX filter (pkg/result/filter.go:38-104 filterByVEX after
    FilterResult): the document is compiled on the host (trivy_amd/vex.py) into (package,
    vulnerability) suppressions, the survivors are tested on the GPU (filter_select), and the
    result equals oracle/filter.py then oracle/vex.py per result, in order."""
    import oracle.filter as of
    import oracle.vex as ov
    from tools import synth_vex as sv
    from trivy_amd.vex import VEX
    mb, bucket, by_target, sdb = _filter_fixture()
    # package identities: the OS PURL of (platform, name, version); one root image per result
    n_pkgs = len(mb)
    purls, refs, result_of = [None] * n_pkgs, [""] * n_pkgs, np.zeros(n_pkgs, dtype=np.int64)
    roots = [sv.root_of(t) if t % 4 else None for t in range(len(by_target))]
    findings = []
    for t, vulns in enumerate(by_target):
        plat = "debian 12" if vulns and vulns[0]["DataSource"]["ID"] == "debian" else "ubuntu 22.04"
        for v in vulns:
            pk = v["_pair"][0]
            purls[pk] = sv.purl_of(plat, v["PkgName"], v["InstalledVersion"], "amd64" if len(v["PkgName"]) % 3 else None)
            refs[pk] = "ref-%d-%s-%s" % (t, v["PkgName"], v["InstalledVersion"])
            result_of[pk] = t
            findings.append((pk, v["VulnerabilityID"]))
    rng = np.random.default_rng(11)
    text = {"openvex": lambda: sv.openvex(rng, findings, purls, len(roots), n_stmts=400),
            "cyclonedx": lambda: sv.cyclonedx(rng, findings, purls, refs, n_vulns=300),
            "csaf": lambda: sv.csaf(rng, findings, purls, n_vulns=300)}[kind]()
    at = "cyclonedx" if kind == "cyclonedx" else ""
    sup = VEX.new(text, at, sv.SERIAL, 1).suppressions(purls, refs, result_of, roots)
    opts = dict(severities=("UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"))
    o2 = mb.filter_opts(vex=sup, **opts)
    o2.vex_id_ranks = None  # the C-ABI ranks the ID strings itself
    n2 = mb.filter(o2)
    n = mb.filter(mb.filter_opts(vex=sup, **opts))
    assert n == n2
    got = mb.filtered_pairs(n).tolist()
    oracle_vex = ov.VEX.new(text, at, sv.SERIAL, 1)
    want, dropped = [], 0
    for t, vulns in enumerate(by_target):
        filled = vi.fill_info(bucket, [{k: x for k, x in v.items() if k != "_pair"} for v in vulns])
        for f, v in zip(filled, vulns):
            f["_pair"] = v["_pair"]
            pk = v["_pair"][0]
            f["PkgIdentifier"] = {"PURL": ov.purl_from_string(purls[pk]), "BOMRef": refs[pk]}
        kept, _ = of.filter_vulnerabilities("", filled, list(opts["severities"]))
        after = oracle_vex.filter(kept or [], ov.purl_from_string(roots[t]) if roots[t] else None)
        dropped += len(kept or []) - len(after)
        want += after
    assert dropped > 0
    assert len(got) == len(want), (len(got), len(want))
    assert got == [list(w["_pair"]) for w in want]
    # a statement naming a package the batch does not have is refused (checked on the device)
    bad = (np.concatenate([np.asarray(sup[0], dtype=np.uint32), [len(mb)]]), list(sup[1]) + [sup[1][0]])
    with pytest.raises(RuntimeError, match="out of range"):
        mb.filter(mb.filter_opts(vex=bad, **opts))
    assert mb.filter(mb.filter_opts(vex=sup, **opts)) == n
    mb.close()


def test_match_filter_batch_ignore_purls_vs_oracle():
    """Ignore-file findings scoped by PURL (ignore.go MatchVulnerability, before the dedup,
    filter.go:117-122) on the GPU batch filter: plain IDs + PURL-scoped findings (versioned,
    versionless, qualifier-scoped) equal oracle/filter.py per result."""
    import oracle.filter as of
    from tools import synth_vex as sv
    from trivy_amd.ignore import compile_rules
    mb, bucket, by_target, sdb = _filter_fixture()
    purls = [None] * len(mb)
    for vulns in by_target:
        plat = "debian 12" if vulns and vulns[0]["DataSource"]["ID"] == "debian" else "ubuntu 22.04"
        for v in vulns:
            # every 7th package has no PURL: PURL-scoped findings match it (matchPURL)
            purls[v["_pair"][0]] = None if v["_pair"][0] % 7 == 0 else sv.purl_of(
                plat, v["PkgName"], v["InstalledVersion"], "amd64" if len(v["PkgName"]) % 3 else None)
    rng = np.random.default_rng(21)
    flat = [v for vulns in by_target for v in vulns]
    findings = []
    for k in range(120):
        v = flat[rng.integers(len(flat))]
        pu = purls[v["_pair"][0]] or "pkg:deb/debian/%s@%s" % (v["PkgName"], v["InstalledVersion"])
        base, _, q = pu.partition("?")
        pat = [pu, base, base.rpartition("@")[0], base.rpartition("@")[0] + "?arch=amd64"][k % 4]
        findings.append({"ID": v["VulnerabilityID"], "Paths": [], "PURLs": [pat], "ExpiredAt": None, "Statement": ""})
    findings.append({"ID": flat[0]["VulnerabilityID"], "Paths": [], "PURLs": [], "ExpiredAt": None, "Statement": ""})
    rules = compile_rules(findings, purls)
    assert rules.pkg_class is not None and len(rules.cls[0]) > 0  # PURL-less packages: class rules
    opts = dict(severities=("UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"))
    n = mb.filter(mb.filter_opts(ignore=rules, **opts))
    got = mb.filtered_pairs(n).tolist()
    ofind = [dict(f, PURLs=[of.purl_from_string(x) for x in f["PURLs"]]) for f in findings]
    want, want_ign = [], []
    for vulns in by_target:
        filled = vi.fill_info(bucket, [{k: x for k, x in v.items() if k != "_pair"} for v in vulns])
        for f, v in zip(filled, vulns):
            f["_pair"] = v["_pair"]
            pu = purls[v["_pair"][0]]
            f["PkgIdentifier"] = {"PURL": of.purl_from_string(pu) if pu else None}
        kept, ig = of.filter_vulnerabilities("", filled, list(opts["severities"]), (), ofind)
        want_ign += [list(v["_pair"]) + [ofind.index(f)] for v, f in ig]
        want += kept or []
    assert want_ign
    assert got == [list(w["_pair"]) for w in want]
    assert mb.ignored_findings().tolist() == want_ign
    bad = mb.filter_opts(**opts)
    bad.severity_mask |= 1 << 5  # SeverityNames has 5 entries: higher bits are rejected
    with pytest.raises(RuntimeError, match="severity_mask"):
        mb.filter(bad)
    mb.close()


def test_match_filter_batch_report_paths_vs_oracle():
    """The dedup key and BySeverity on report identities (tvm_batch_set_report): packages that
    match under different source names but report one (PkgName, InstalledVersion) dedup
    across packages with DIFFERENT FixedVersions (the greater wins, ties the first seen);
    PkgPath splits dedup groups and breaks BySeverity ties; path-scoped ignore findings
    (Target / PkgPath globs, pass order) and ModifiedFindings - all vs oracle/filter.py."""
    import oracle.filter as of
    from trivy_amd.ignore import compile_rules
    mb, bucket, by_target, sdb = _filter_fixture(seed=13)
    n_pkgs = len(mb)
    key_of = {bytes(k): i for i, k in enumerate(sdb.key_names)}
    rname, rver, rpath = [None] * n_pkgs, [None] * n_pkgs, [""] * n_pkgs
    pkg_name, pkg_ver = {}, {}
    for vulns in by_target:
        for v in vulns:
            pkg_name[v["_pair"][0]], pkg_ver[v["_pair"][0]] = v["PkgName"], v["InstalledVersion"]
    for pk in range(n_pkgs):
        nm, ver = pkg_name.get(pk), pkg_ver.get(pk)
        if nm is None:
            nm, ver = "none%d" % pk, "0"
        k = key_of.get(nm.encode(), pk)
        # keys 25 apart share CVE IDs (tools/synth.py): one binary name per residue class
        rname[pk] = "bin-%d" % (k % 25) if k % 3 else nm
        rver[pk] = "1.0" if k % 2 else ver
        rpath[pk] = "" if pk % 4 else "opt/app%d/lib.jar" % (pk % 3)
    mb.set_report(0, rname, rver, rpath)
    targets = ["img%d/layer%d" % (t, t % 3) for t in range(len(by_target))]
    res = [(targets[t], s, e) for t, (s, e) in enumerate(mb.result_bounds)]
    rng = np.random.default_rng(5)
    flat = [v for vulns in by_target for v in vulns]
    globs = ["**", "img1/**", "img*/layer2", "opt/app1/*.jar", "opt/**", "nomatch/**"]
    findings = []
    for k in range(80):
        v = flat[int(rng.integers(len(flat)))]
        f = {"ID": v["VulnerabilityID"], "Paths": [], "PURLs": [], "ExpiredAt": None, "Statement": "st%d" % k}
        if k % 2:
            f["Paths"] = [globs[int(rng.integers(len(globs)))]]
        findings.append(f)
    rules = compile_rules(findings, [None] * n_pkgs, res, rpath)
    opts = dict(severities=("UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"))
    n = mb.filter(mb.filter_opts(ignore=rules, **opts))
    got = mb.filtered_pairs(n).tolist()
    want, want_ign, cross = [], [], 0
    for t, vulns in enumerate(by_target):
        filled = vi.fill_info(bucket, [{k: x for k, x in v.items() if k != "_pair"} for v in vulns])
        for f, v in zip(filled, vulns):
            pk = v["_pair"][0]
            f["_pair"] = v["_pair"]
            f["PkgName"], f["InstalledVersion"], f["PkgPath"] = rname[pk], rver[pk], rpath[pk]
            if not rpath[pk]:
                f.pop("PkgPath")
        kept, ig = of.filter_vulnerabilities(targets[t], filled, list(opts["severities"]), (), findings)
        want_ign += [list(v["_pair"]) + [findings.index(f)] for v, f in ig]
        want += kept or []
        seen = {}
        for f in filled:  # dedup keys held by two packages with different FixedVersions
            key = (f["VulnerabilityID"], f["PkgName"], f["InstalledVersion"], f.get("PkgPath", ""))
            seen.setdefault(key, set()).add((f["_pair"][0], f.get("FixedVersion", "")))
        cross += sum(1 for s in seen.values() if len({x[0] for x in s}) > 1 and len({x[1] for x in s}) > 1)
    assert cross > 0 and want_ign
    assert len(got) == len(want), (len(got), len(want))
    assert got == [list(w["_pair"]) for w in want]
    assert mb.ignored_findings().tolist() == want_ign
    mb.close()
