"""CPU: the library sort keys (trivy_amd/csrc/libver.h, host build) and the load-time
constraint compiler (libdb.cpp) against the pairwise oracle (oracle/library.py).

The same encoders run on the GPU for installed versions; the compiler's interval rows are
what the kernel tests.  Both are checked here on random versions / advisories drawn from
realistic grammars, plus every comparer KAT of the reference."""
import ctypes
import functools
import json
import random
import re
import zlib

import pytest

import oracle.library as ol
from trivy_amd._lib import lib

GRAMMAR = {"generic": 4, "npm": 5, "pep440": 6, "maven": 7, "gem": 8, "bitnami": 9}
PARSERS = {"generic": ol.GenVer, "npm": ol.NpmVer, "pep440": ol.PepVer, "maven": ol.MvnVer, "gem": ol.GemVer,
           "bitnami": lambda s: ol.GenVer(s, True)}
_BUF = ctypes.create_string_buffer(1 << 16)


def key(g, v):
    b = v.encode()
    n = lib().tvm_version_key(GRAMMAR[g], b, len(b), _BUF, len(_BUF))
    return None if n < 0 else _BUF.raw[:n]


def cls(g, v):
    b = v.encode()
    return lib().tvm_version_class(GRAMMAR[g], b, len(b))


def host_vuln(g, ver, adv):
    b, j = ver.encode(), json.dumps(adv).encode()
    return lib().tvm_lib_is_vulnerable_host(GRAMMAR[g], b, len(b), j, len(j))


# ---------------------------------------------------------------- version generators ----
def _num(r):
    return str(r.choice([0, 0, 1, 1, 2, 3, 5, 9, 10, 12, 99, 100, 2023]))


def gen_generic(r):
    v = ".".join(_num(r) for _ in range(r.randint(1, 4)))
    if r.random() < 0.1:
        v = "v" + v
    x = r.random()
    if x < 0.3:
        v += "-" + ".".join(r.choice(["alpha", "beta", "rc", "1", "2", "0", "x-y", "rc1", "a"])
                            for _ in range(r.randint(1, 3)))
    elif x < 0.35:
        v += r.choice(["beta", "rc1", "alpha.1"])
    if r.random() < 0.1:
        v += "+" + r.choice(["build.1", "incompatible", "meta"])
    return v


def gen_bitnami(r):
    v = ".".join(_num(r) for _ in range(r.randint(1, 3)))
    x = r.random()
    if x < 0.4:
        v += "-" + _num(r)
    elif x < 0.5:
        v += "-" + r.choice(["beta", "rc.1"])
    return v


def gen_npm(r):
    v = ".".join(_num(r) for _ in range(3))
    if r.random() < 0.35:
        v += "-" + ".".join(r.choice(["alpha", "beta", "rc", "0", "1", "2", "10", "x"]) for _ in range(r.randint(1, 3)))
    if r.random() < 0.05:
        v += "+build"
    return v


def gen_pep(r):
    v = ".".join(_num(r) for _ in range(r.randint(1, 4)))
    if r.random() < 0.05:
        v = "1!" + v
    if r.random() < 0.3:
        v += r.choice(["a", "b", "rc", ".alpha", "-beta", "c", "pre"]) + r.choice(["", "0", "1", "2"])
    if r.random() < 0.2:
        v += r.choice([".post", "-", ".post1", "post2", ".rev"]) + r.choice(["1", "2", ""]) if r.random() < 0.5 \
            else ".post" + _num(r)
    if r.random() < 0.2:
        v += ".dev" + r.choice(["", "0", "1", "3"])
    if r.random() < 0.15:
        v += "+" + ".".join(r.choice(["ubuntu", "1", "2", "abc", "01"]) for _ in range(r.randint(1, 2)))
    return v


def gen_maven(r):
    parts = [_num(r) for _ in range(r.randint(1, 4))]
    v = ".".join(parts)
    x = r.random()
    if x < 0.15:
        v += "-" + r.choice(["SNAPSHOT", "alpha", "beta-1", "rc1", "RC2", "jre", "android", "Final", "GA", "sp1",
                             "M1", "a1", "b2"])
    elif x < 0.3:
        v += "." + r.choice(["Final", "RELEASE", "RC1", "M1", "v20210516", "jre"])
    elif x < 0.35:
        v += r.choice(["a1", "b1", "rc1", "m2"])
    elif x < 0.45:  # ComparableVersion's non-transitive corners: zeros / qualifiers vs sub-lists
        v += r.choice([".0.rc", ".0.beta", ".0.alpha1", ".jre", ".sp", ".foo", "-x", "-sp", "-1", "-0", "--1", ".0-rc1",
                       "-jre7", ".0.0-1"])
    return v


def gen_gem(r):
    v = ".".join(_num(r) for _ in range(r.randint(1, 4)))
    x = r.random()
    if x < 0.2:
        v += "." + r.choice(["pre", "a", "beta", "rc1", "b2"])
    elif x < 0.3:
        v += r.choice(["a", "b1", "rc"])
    elif x < 0.4:
        v += "-" + r.choice(["java", "x86-mingw32", "1"])
    return v


GENS = {"generic": gen_generic, "npm": gen_npm, "pep440": gen_pep, "maven": gen_maven, "gem": gen_gem,
        "bitnami": gen_bitnami}


_MVN_NUMERIC = re.compile(r"^[0-9]{1,9}(\.[0-9]{1,9})*$")


@pytest.mark.parametrize("g", list(GRAMMAR))
def test_key_order_matches_oracle(g):
    """Maven: ComparableVersion is not an order, and the product's Maven key
    is the installed version's numeric projection (libver.h mvn_numeric_projection), which
    only ever meets numeric bounds: pairs with a numeric side are checked (every installed
    shape against numeric bounds, the non-transitive corners included); advisories with
    other bounds are pairwise programs (the IsVulnerable fuzz below)."""
    r = random.Random(zlib.crc32(g.encode()))
    bad, n = [], 0
    for _ in range(20000):
        a, b = GENS[g](r), GENS[g](r)
        try:
            va, vb = PARSERS[g](a), PARSERS[g](b)
        except ol.VersionError:
            continue
        ka, kb = key(g, a), key(g, b)
        assert ka is not None and kb is not None, (a, b)
        if g == "maven" and not (_MVN_NUMERIC.match(a) or _MVN_NUMERIC.match(b)):
            continue
        n += 1
        want = va.compare(vb)
        got = (ka > kb) - (ka < kb)
        if got != want:
            bad.append((a, b, want, got))
    assert n > 5000
    assert not bad, bad[:10]


def _mvn_any(r):
    """Arbitrary ComparableVersion shapes: int / zero / qualifier items joined by '.', '-' or
    nothing (digit <-> letter transitions open sub-lists), empty items included."""
    items = ["0", "00", "1", "2", "10", "007", "alpha", "a", "b", "m", "rc", "cr", "snapshot", "ga", "final",
             "release", "sp", "jre", "x", "", "RC", "Final", "SNAPSHOT", "GA", "M", "x_y", "b+1"]
    v = r.choice(["0", "1", "2", "10", "1.0", "alpha", "rc", "sp", "RELEASE"])
    for _ in range(r.randint(0, 5)):
        v += r.choice([".", "-", "", "."]) + r.choice(items)
    return v


def _mvn_numeric_bound(r):
    return ".".join(r.choice(["0", "0", "1", "2", "10", "007", "999999999"]) for _ in range(r.randint(1, 5)))


def test_maven_projection_against_numeric_bounds():
    """compare(V, B) for any installed V and numeric B is the key order of V's numeric
    projection against B's key (libver.h mvn_numeric_projection): 60k pairs of arbitrary
    shapes, the non-transitive ones of DESIGN.md §2.2 among them, against the oracle's
    ComparableVersion."""
    r = random.Random(355)
    bad, n = [], 0
    for _ in range(60000):
        a, b = _mvn_any(r), _mvn_numeric_bound(r)
        try:
            va, vb = ol.MvnVer(a), ol.MvnVer(b)
        except ol.VersionError:
            assert key("maven", a) is None, a
            continue
        ka, kb = key("maven", a), key("maven", b)
        assert ka is not None and kb is not None, (a, b)
        n += 1
        want = va.compare(vb)
        if (ka > kb) - (ka < kb) != want:
            bad.append((a, b, want))
    assert n > 40000
    assert not bad, bad[:10]
    assert cls("maven", "1.0-rc1") == 0 and cls("maven", "1.2.3") == 0  # one class
    for _ in range(5000):  # numeric texts: surrounding blanks are trimmed before the parse
        b = _mvn_numeric_bound(r)
        assert key("maven", b) == key("maven", " " + b), b


@pytest.mark.parametrize("g,v", [("generic", "1.2..4"), ("npm", "1.2"), ("npm", "1.2..4"), ("pep440", "1.2..4"),
                                 ("gem", "1.2..4"), ("maven", "<1.0\\.0"), ("generic", "*"), ("pep440", "1.0+")])
def test_invalid_versions(g, v):
    assert key(g, v) is None
    with pytest.raises(ol.VersionError):
        PARSERS[g](v)


def test_classes():
    assert cls("npm", "1.2.3") == 0 and cls("npm", "1.2.3-rc.1") == 1
    assert cls("pep440", "1.0") == 0 and cls("pep440", "1.0+local") == 1
    assert cls("pep440", "1.0a1") == 2 and cls("pep440", "1.0.dev1") == 2 and cls("pep440", "1.0.post1") == 4
    assert cls("pep440", "1.0.post1.dev2+x") == 7


# ------------------------------------------------------------------- compiled rows -----
def _cons(r, g):
    """A random constraint string in the grammar's syntax."""
    v = lambda: GENS[g](r).split("+")[0]  # noqa: E731
    if g == "maven" and r.random() < 0.3:
        lo, hi = sorted([v(), v()], key=functools.cmp_to_key(lambda x, y: ol.MvnVer(x).compare(ol.MvnVer(y))))
        return r.choice([f"[{lo},{hi})", f"(,{hi}]", f"[{lo},)", f"[{lo}]", f"({lo},{hi}),[{hi},)"])
    ops = {"generic": ["<", "<=", ">", ">=", "=", "!=", "~>", "^", "~"], "bitnami": ["<", "<=", ">", ">=", "="],
           "npm": ["<", "<=", ">", ">=", "", "^", "~"], "pep440": ["<", "<=", ">", ">=", "==", "!=", "~="],
           "maven": ["<", "<=", ">", ">=", "="], "gem": ["<", "<=", ">", ">=", "=", "!=", "~>"]}[g]
    parts = []
    for _ in range(r.randint(1, 2)):
        op = r.choice(ops)
        ver = v()
        if g == "npm" and r.random() < 0.15:
            ver = r.choice(["1.x", "2.0.x", "*", "1", "0.2"])
        if g == "pep440" and op in ("==", "!=") and r.random() < 0.2:
            ver = ".".join(ver.split(".")[:2]).split("a")[0].split("b")[0].split("rc")[0] + ".*"
        parts.append(f"{op}{' ' if r.random() < 0.3 else ''}{ver}")
    sep = {"npm": " ", "gem": ", "}.get(g, r.choice([", ", " "]))
    return sep.join(parts)


@pytest.mark.parametrize("g", list(GRAMMAR))
def test_compiled_rows_match_oracle(g):
    """libdb.cpp's interval compilation of IsVulnerable (Maven: the pairwise program) == the
    oracle's direct evaluation, the non-transitive Maven shapes included."""
    r = random.Random(17 + len(g))
    bad, checked = [], 0
    for _ in range(2500):
        adv = {}
        for f in ("VulnerableVersions", "PatchedVersions", "UnaffectedVersions"):
            if r.random() < 0.5:
                adv[f] = [_cons(r, g) for _ in range(r.randint(1, 2))]
        for _ in range(4):
            ver = GENS[g](r)
            want = ol.is_vulnerable(g, ver, adv)
            got = host_vuln(g, ver, adv)
            checked += 1
            if got != int(want):
                bad.append((ver, adv, want, got))
    assert checked > 5000
    assert not bad, bad[:5]


@pytest.mark.parametrize("g", list(GRAMMAR) + ["deb", "apk", "rpm"])
def test_encoders_never_read_past_the_version(g):
    """The GPU encodes versions in place inside a packed arena: the bytes after a version
    are arbitrary (stale digits included) and must never change its key."""
    gid = {"deb": 1, "apk": 2, "rpm": 3}.get(g) or GRAMMAR[g]
    gen = GENS.get(g) or (lambda r: ".".join(_num(r) for _ in range(r.randint(1, 4))) + r.choice(["", "-1", "-r2"]))
    r = random.Random(5)
    for _ in range(3000):
        v = gen(r).encode()
        for tail in (b"1234", b".5-r9", b"a1", b"\x00", b"+x", b"~1"):
            buf = ctypes.create_string_buffer(v + tail, len(v) + len(tail))
            n1 = lib().tvm_version_key(gid, buf, len(v), _BUF, len(_BUF))
            k1 = _BUF.raw[:n1] if n1 >= 0 else None
            b2 = v
            n2 = lib().tvm_version_key(gid, b2, len(b2), _BUF, len(_BUF))
            k2 = _BUF.raw[:n2] if n2 >= 0 else None
            assert k1 == k2, (g, v, tail)


@pytest.mark.parametrize("ver,adv", [
    ("1.0.rc", {"VulnerableVersions": ["<1-x"]}),          # int 0 > list, though 1.0.rc < 1 < 1-x
    ("1-x", {"VulnerableVersions": [">1.0.rc"]}),
    ("99.jre", {"VulnerableVersions": ["<99-rc1"]}),       # string < list
    ("99-rc1", {"PatchedVersions": ["99.jre"]}),
    ("1.0.beta", {"VulnerableVersions": ["[1-sp,2)"]}),
    ("2.0.0", {"VulnerableVersions": ["(,2.0-1]"]}),
    ("release", {"VulnerableVersions": [">ga.milestone"]}),  # flat lists too: "" item vs end of list
    ("0.beta.alpha", {"VulnerableVersions": [">sp.m..alpha.milestone"]}),
    ("m", {"PatchedVersions": [">=0.beta.00.milestone.rc"]}),
])
def test_maven_non_transitive_pairs_exact(ver, adv):
    """The shapes where ComparableVersion is not an order evaluate exactly
    as the oracle's pairwise IsVulnerable (host run of the kernel's program evaluator)."""
    assert host_vuln("maven", ver, adv) == int(ol.is_vulnerable("maven", ver, adv))


def test_maven_rows_equal_pairwise_program():
    """tvm_lib_is_vulnerable_host mirrors the device rows (numeric-bound advisories: key-order
    intervals over the installed version's numeric projection); with TVM_ISVULN_PAIRWISE it runs
    ComparableVersion's pairwise program for every advisory.  The two agree on random shapes
    against numeric-bound advisories, and the pairwise form agrees with the oracle, so the
    projection rows are checked against an independent evaluator, not against themselves."""
    import random

    import oracle.library as ol
    r = random.Random(17)
    n = 0
    for _ in range(3000):
        b1, b2 = sorted([".".join(str(r.randint(0, 12)) for _ in range(r.randint(1, 4))) for _ in range(2)])
        adv = {"VulnerableVersions": [f">= {b1}, < {b2}"], "PatchedVersions": [b2]}
        v = gen_maven(r)
        rows = host_vuln("maven", v, adv)
        b, j = v.encode(), json.dumps(adv).encode()
        pair = lib().tvm_lib_is_vulnerable_host(GRAMMAR["maven"] | 0x100, b, len(b), j, len(j))
        want = ol.is_vulnerable("maven", v, adv)
        assert rows == pair == int(want), (v, adv, rows, pair, want)
        n += 1
    assert n > 2000

