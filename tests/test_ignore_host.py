"""Host compile of ignore-file findings for the batch filter (trivy_amd/ignore.py) against
the oracle's IgnoreConfig.MatchVulnerability (oracle/filter.py, pinned by TestFilter), and
the product doublestar matcher (trivy_amd/glob.py) against the oracle's."""
import numpy as np
import pytest

import oracle.filter as of
from tools import synth_vex as sv
from trivy_amd import glob
from trivy_amd.ignore import PASS_PKGPATH, compile_rules, plain_rules


def _evaluate(rules, n, ids):
    """The GPU's rule lookup restated: per (package, ID) the smallest precedence."""
    (aid, aprec), (ppk, pid, pprec), (ccl, cid, cprec), pcls = rules.arrays()
    names = rules.ids
    best = {}

    def put(i, v, prec):
        k = (i, names[v])
        best[k] = min(best.get(k, 1 << 40), int(prec))

    for v, p in zip(aid.tolist(), aprec.tolist()):
        for i in range(n):
            put(i, v, p)
    for i, v, p in zip(ppk.tolist(), pid.tolist(), pprec.tolist()):
        put(i, v, p)
    for c, v, p in zip(ccl.tolist(), cid.tolist(), cprec.tolist()):
        for i in range(n):
            if pcls[i] == c:
                put(i, v, p)
    return best


def _fixture(seed, with_paths):
    rng = np.random.default_rng(seed)
    n = 300
    purls = [sv.purl_of("debian 12", "pkg%d" % (i % 30), "1.%d-1" % (i % 4), "amd64" if i % 3 else None)
             if i % 17 else None for i in range(n)]
    paths = ["" if i % 5 else "usr/lib/app%d/pkg%d.jar" % (i % 3, i % 30) for i in range(n)]
    results = [("img%d:layer/%s" % (t, "var/lib/dpkg" if t % 2 else "app"), t * 50, t * 50 + 50) for t in range(6)]
    ids = ["CVE-2024-%04d" % k for k in range(20)]
    globs = ["**", "img1*/**", "**/app", "usr/lib/app1/*.jar", "usr/**/pkg1?.jar", "{img2,img4}:layer/app",
             "img[0-2]:layer/**", "nomatch"]
    findings = []
    for k in range(90):
        pu = purls[int(rng.integers(n))] or "pkg:deb/debian/pkg1@1.1-1"
        base = pu.partition("?")[0]
        pats = [pu, base, base.rpartition("@")[0], base.rpartition("@")[0] + "?arch=amd64"]
        f = {"ID": ids[k % 20], "Paths": [], "PURLs": [pats[k % 4]] if k % 5 else [], "ExpiredAt": None,
             "Statement": "s%d" % k}
        if with_paths and k % 3 == 0:
            f["Paths"] = [globs[int(rng.integers(len(globs)))] for _ in range(1 + k % 2)]
        findings.append(f)
    return purls, paths, results, ids, findings


@pytest.mark.parametrize("with_paths", [False, True])
def test_compile_rules_vs_oracle(with_paths):
    purls, paths, results, ids, findings = _fixture(3 + with_paths, with_paths)
    n = len(purls)
    rules = compile_rules(findings, purls, results, paths if with_paths else None)
    best = _evaluate(rules, n, ids)
    ofind = [dict(f, PURLs=[of.purl_from_string(x) for x in f["PURLs"]]) for f in findings]
    target = {}
    for t, b, e in results:
        for i in range(b, e):
            target[i] = t
    hits = 0
    for i in range(n):
        for v in ids:
            w = of.match_vulnerability(ofind, v, target[i] if with_paths else "", paths[i] if with_paths else "",
                                       of.purl_from_string(purls[i]) if purls[i] else None)
            got = best.get((i, v))
            if w is None:
                assert got is None, (i, v, got)
            else:
                hits += 1
                assert got is not None and (got & ~PASS_PKGPATH) == ofind.index(w), (i, v, got, ofind.index(w))
    assert 0 < hits < n * len(ids)
    # rules never grow as findings x packages
    assert len(rules) < 4 * len(findings) * (1 + len(set(zip(paths, [p is None for p in purls]))))


def test_purl_less_packages_use_classes():
    """a PURL-scoped finding on N PURL-less packages is one class rule, not N pairs."""
    purls = [None] * 10000 + ["pkg:deb/debian/a@1"]
    rules = compile_rules([{"ID": "CVE-1", "Paths": [], "PURLs": ["pkg:deb/debian/a"]}], purls)
    assert len(rules.cls[0]) == 1 and len(rules.pkg[0]) == 1 and rules.pkg_class is not None


def test_plain_rules_first_wins():
    r = plain_rules(["CVE-1", "CVE-2", "CVE-1"], 5)
    best = _evaluate(r, 5, ["CVE-1", "CVE-2"])
    assert best[(0, "CVE-1")] == 0 and best[(4, "CVE-2")] == 1


def test_paths_need_results():
    with pytest.raises(ValueError, match="Target"):
        compile_rules([{"ID": "CVE-1", "Paths": ["a/**"], "PURLs": []}], ["pkg:npm/a@1"])


@pytest.mark.parametrize("pat,path", [
    ("**", ""), ("**", "a/b/c"), ("a/**", "a"), ("a/**", "a/b"), ("a/**/b", "a/b"), ("a/**/b", "a/x/y/b"),
    ("a/*/b", "a/x/b"), ("a/*/b", "a/x/y/b"), ("*.jar", "x.jar"), ("*.jar", "d/x.jar"), ("?x", "ax"), ("?x", "x"),
    ("[a-c]x", "bx"), ("[!a-c]x", "bx"), ("[^a-c]x", "dx"), ("{foo,bar}/z", "bar/z"), ("{foo,ba*}/z", "baz/z"),
    ("\\*x", "*x"), ("\\*x", "ax"), ("", ""), ("a", ""), ("usr/**/*.jar", "usr/lib/a/b.jar"), ("[a", "[a"),
    ("/abs/**", "/abs/x"), ("**/app", "img1:layer/app"),
])
def test_glob_vs_oracle(pat, path):
    assert glob.match(pat, path) == bool(of.doublestar_match(pat, path)), (pat, path)
