"""GPU: the Red Hat chain composed on the device in the reference's order of work - the
driver's per-CVE merge (pkg/detector/ospkg/redhat/redhat.go:146-187) -> FillInfo
(pkg/vulnerability/vulnerability.go:60-157) -> result.Filter (pkg/result/filter.go:60-139)
(+ a VEX suppression list, filter.go:38-104).

A C5-shaped batch (RHEL family + Alpine: Red Hat with CPE sets, modular keys and RHSA
advisories naming several CVEs) is matched, merged, filled and filtered without leaving the
GPU (tvm_match_launch -> tvm_match_redhat_merge -> tvm_match_fill -> tvm_match_filter).  Each
result's survivors - order, (package, VulnerabilityID), FillInfo Status, and for Red Hat the
merged FixedVersion and VendorIDs - equal the oracle chain oracle/drivers.py ->
oracle/vulninfo.py -> oracle/filter.py on the same packages."""
import collections

import numpy as np
import pytest

from tools import synth_mix as sm

pytestmark = pytest.mark.gpu

_STATE = {}


def _setup():
    if _STATE:
        return _STATE
    import oracle.drivers as od
    import trivy_amd
    from tools.synth_vuln import vuln_arena, vuln_values
    from trivy_amd.batch import MatchBatch
    sdb = sm.make_mix_db(sm.C5_PLATS, 1500, seed=0xC5C5)
    db = sdb.put(trivy_amd.DB())
    ids = sm.MixDB.vuln_ids_of(sdb)
    db.put_arena(*vuln_arena(ids))
    db.finalize()
    eng = trivy_amd.Engine(db, 0)
    batch = sm.make_mix_batch(sdb, 24_000, sm.C5_WEIGHTS, seed=31)
    mb = MatchBatch(eng)
    firsts = sm.add_to(mb, sdb, batch)
    for (p, g), (_, first) in zip(batch.groups, firsts):
        if sdb.plats[p][1] == "redhat":  # DetectedVulnerability.PkgName = pkg.Name, not the modular lookup name
            mb.set_report(first, names=[x.decode() for x in g["pname"]])
    total, errp, bits = mb.run()
    assert errp == -1 and bits == 0 and total > 10_000
    raw = len(mb.pairs())
    mb.redhat_merge()
    merged_pairs = mb.pairs()
    mb.fill()
    # the oracle's detection output per result (one result per platform group), in the
    # drivers' order: package by package, each package's vulnerabilities as Detect returns them
    bucket = {k.decode(): v.decode() for k, v in vuln_values(ids)}
    names = collections.defaultdict(set)
    for p, g in batch.groups:
        names[sdb.plats[p][0]] |= {x.decode() for x in g["name"]}
    names["Red Hat CPE"] = {"repository", "nvr", "cpe"}
    recs = od.Records(sdb.records_for(names))
    results, pkgs_of = [], {}
    for (p, g), (_, first) in zip(batch.groups, firsts):
        bucket_name, kind = sdb.plats[p]
        pkgs = sm.driver_packages(sdb, p, g, np.arange(len(g["key"])))
        for i, pk in enumerate(pkgs):
            pkgs_of[first + i] = pk
        if kind == "redhat":
            vulns = []
            for rel in (7, 8, 9):
                sub = [pk for pk, r in zip(pkgs, g["rhrel"]) if int(r) == rel]
                vulns += od.driver_detect("redhat", str(rel), None, sub, recs, None)
            vulns.sort(key=lambda v: int(v["PkgID"][1:]))  # stable: each package's list stays in ID order
        else:
            fam, fmt = sm.DRIVER_OF[kind]
            vulns = od.driver_detect(fam, fmt.format(bucket_name.split(" ")[-1]), None, pkgs, recs, None)
        results.append((first, kind, vulns))
    _STATE.update(mb=mb, results=results, bucket=bucket, pkgs_of=pkgs_of, raw=raw, merged_pairs=merged_pairs,
                  firsts=firsts)
    return _STATE


def _oracle_kept(st, severities, ignore_statuses, vex=frozenset()):
    import oracle.filter as of
    import oracle.vulninfo as vi
    want = []
    for first, kind, vulns in st["results"]:
        # the drivers' dicts carry the embedded Vulnerability.Severity flattened (its JSON form)
        vulns = [dict({k: x for k, x in v.items() if k != "Severity"},
                      **({"Vulnerability": {"Severity": v["Severity"]}} if "Severity" in v else {})) for v in vulns]
        filled = vi.fill_info(st["bucket"], vulns)
        kept, _ = of.filter_vulnerabilities("", filled, list(severities), ignore_statuses)
        for v in kept or []:
            key = (first + int(v["PkgID"][1:]), v["VulnerabilityID"])
            if key not in vex:  # filterByVEX runs on the survivors (filter.go:38-104)
                want.append((key, kind, v))
    return want


@pytest.mark.parametrize("opts", [
    dict(severities=("UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL")),
    dict(severities=("LOW", "MEDIUM", "HIGH"), ignore_statuses=(3,)),
    dict(severities=("UNKNOWN", "MEDIUM", "CRITICAL"), ignore_statuses=(2, 5), vex=True),
])
def test_redhat_chain_vs_oracle(opts):
    from trivy_amd.batch import advisory_vuln_id
    st = _setup()
    mb = st["mb"]
    db = mb.engine.db
    opts = dict(opts)
    use_vex = opts.pop("vex", False)
    sev, ign = opts["severities"], opts.get("ignore_statuses", ())
    sup = set()
    vex = None
    if use_vex:  # a VEX document's (package, vulnerability) suppressions: every 9th survivor
        base = _oracle_kept(st, sev, ign)
        sup = {k for j, (k, _, _) in enumerate(base) if j % 9 == 4}
        vex = ([k[0] for k in sorted(sup)], [k[1] for k in sorted(sup)])
    n = mb.filter(mb.filter_opts(vex=vex, **opts))
    got = mb.filtered_pairs(n)
    want = _oracle_kept(st, sev, ign, frozenset(sup))
    got_keys = [(int(p), advisory_vuln_id(db, int(a))) for p, a in got.tolist()]
    # per result (one per platform group): counts, then the first differing position
    bounds = [f for f, _, _ in st["results"]] + [1 << 40]
    res_of = lambda p: int(np.searchsorted(bounds, p, side="right")) - 1  # noqa: E731
    for r, (first, kind, _) in enumerate(st["results"]):
        g = [k for k in got_keys if res_of(k[0]) == r]
        w = [x for x in want if res_of(x[0][0]) == r]
        if len(g) != len(w) or any(a != b[0] for a, b in zip(g, w)):
            i = next((i for i, (a, b) in enumerate(zip(g, w)) if a != b[0]), min(len(g), len(w)))
            ctx = lambda x: (x[0], x[2].get("PkgName"), x[2].get("InstalledVersion"),  # noqa: E731
                             (x[2].get("Vulnerability") or {}).get("Severity"), x[2].get("FixedVersion"), x[2].get("Status"))
            pytest.fail(f"result {r} ({kind}): got {len(g)}, want {len(w)}; first difference at {i}: "
                        f"got {g[max(0, i - 2):i + 3]} want {[ctx(x) for x in w[max(0, i - 2):i + 3]]}", pytrace=False)
    assert len(got_keys) == len(want)

    # FillInfo Status of every survivor (a merged entry: Fixed when any member is fixed)
    dec = {(int(p), int(a)): d for (p, a), d in zip(st["merged_pairs"].tolist(), mb.fill_decisions().tolist())}
    st_got = [dec[(int(p), int(a))][1] for p, a in got.tolist()]
    st_bad = [(i, st_got[i], w[2]["Status"], w[0]) for i, w in enumerate(want) if st_got[i] != w[2]["Status"]]
    assert not st_bad, (len(st_bad), st_bad[:5])
    # the merged Red Hat fields of the survivors
    rh = [(i, w) for i, w in enumerate(want) if w[1] == "redhat"]
    assert len(rh) > (50 if 3 in ign else 300)
    vulns = mb.redhat_vulns(got[[i for i, _ in rh]], st["pkgs_of"])
    assert len(vulns) == len(rh)
    for v, (_, (_, _, w)) in zip(vulns, rh):
        assert v["VulnerabilityID"] == w["VulnerabilityID"]
        assert v.get("FixedVersion", "") == w.get("FixedVersion", "")
        assert v.get("VendorIDs", []) == w.get("VendorIDs", [])
    if 3 not in ign:  # fixed survivors: some merged entries union several RHSA VendorIDs
        assert any(len(w.get("VendorIDs", [])) > 1 for _, (_, _, w) in rh)


def test_redhat_merge_shrinks_only_redhat():
    """The merge keeps every other driver's pair and replaces a Red Hat package's members of
    one CVE by one entry; the merged list is in (package, VulnerabilityID) order."""
    from trivy_amd.batch import advisory_vuln_id
    st = _setup()
    mb = st["mb"]
    mp = st["merged_pairs"]
    assert len(mp) < st["raw"]
    assert np.all(np.diff(mp[:, 0].astype(np.int64)) >= 0)
    rh_pk = set()
    for (first, kind, vulns), (g_p, g_first) in zip(st["results"], st["firsts"]):
        if kind == "redhat":
            rh_pk |= {first + int(v["PkgID"][1:]) for v in vulns}
    seen = set()
    for p, a in mp.tolist():
        if p in rh_pk:  # one entry per (package, VulnerabilityID) of a Red Hat package
            key = (p, advisory_vuln_id(mb.engine.db, int(a)))
            assert key not in seen
            seen.add(key)
    # every driver's Detect output has exactly one entry per merged-list pair
    assert len(mp) == sum(len(vulns) for _, _, vulns in st["results"])
