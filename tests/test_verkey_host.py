"""CPU: the version sort-key encoder (trivy_amd/csrc/verkey.h, host build) against the oracle.

The same encoder source runs on the GPU for installed versions; here its host
build must order every pair of versions exactly as the restated comparator does
(and agree on which strings fail to parse).
"""
import ctypes
import random

import pytest

import oracle.drivers as od
from trivy_amd._lib import lib

_BUF = ctypes.create_string_buffer(8192)


def key(grammar, v):
    b = v.encode() if isinstance(v, str) else v
    n = lib().tvm_version_key(grammar, b, len(b), _BUF, len(_BUF))
    return None if n < 0 else _BUF.raw[:n]


ATOMS = [b"0", b"1", b"2", b"9", b"00", b"10", b"010", b".", b"-", b"+", b"~", b":", b"_", b"a", b"b", b"z",
         b"A", b"Z", b"r", b"rc", b"ubuntu", b"deb", b"dfsg", b"\xc3\xa9", b"\xd7", b"\xff", b"\xe2\x82\xac",
         b"99999999999999999999", b"18446744073709551616", b"9223372036854775807", b" ", b"!"]


def _gen(rng):
    s = b"".join(rng.choice(ATOMS) for _ in range(rng.randint(0, 8)))
    if rng.random() < 0.6:
        s = rng.choice([b"1", b"2", b"0", b"10"]) + s
    if rng.random() < 0.2:
        s = rng.choice([b"1:", b"0:", b"-1:", b"+2:", b":", b"a:", b"-0:"]) + s
    return s


def test_deb_key_matches_oracle(oracle_built):
    rng = random.Random(1234)
    bad = []
    for _ in range(60000):
        a, b = _gen(rng), _gen(rng)
        r = od.deb_cmp(a, b)
        ka, kb = key(1, a), key(1, b)
        if r == 2:
            assert ka is None, a
            continue
        assert ka is not None, a
        if r == 3:
            assert kb is None, b
            continue
        assert kb is not None, b
        got = (ka > kb) - (ka < kb)
        if got != r:
            bad.append((a, b, r, got))
    assert not bad, bad[:10]


@pytest.mark.parametrize("v", ["2.4.25-1", "2:2.9-1ubuntu4.3", "1.0~rc1+dfsg-3", "0", "1:1", "7.88.1-10+deb12u5"])
def test_deb_key_length_bound(v):
    k = key(1, v)
    assert k is not None and len(k) <= 2 * len(v) + 12


APK_ATOMS = [b"0", b"1", b"2", b"9", b"00", b"01", b"10", b"010", b".", b"_", b"-r", b"-r1", b"-r10", b"-", b"a",
             b"b", b"z", b"_alpha", b"_beta", b"_pre", b"_rc", b"_cvs", b"_svn", b"_git", b"_hg", b"_p", b"_x",
             b"A", b"~", b"99999999999"]


def _gen_apk(rng):
    s = b"".join(rng.choice(APK_ATOMS) for _ in range(rng.randint(0, 7)))
    if rng.random() < 0.7:
        s = rng.choice([b"1", b"2", b"0", b"10", b"1.0", b"0.1.0"]) + s
    return s


def test_apk_key_matches_oracle(oracle_built):
    """go-apk-version order (oracle/apk.c) == byte order of the apk sort keys (grammar 2)."""
    rng = random.Random(99)
    bad, n_valid = [], 0
    for _ in range(60000):
        a, b = _gen_apk(rng), _gen_apk(rng)
        r = od.apk_cmp(a, b)
        ka, kb = key(2, a), key(2, b)
        if r == 2:
            assert ka is None, a
            continue
        assert ka is not None, a
        if r == 3:
            assert kb is None, b
            continue
        assert kb is not None, b
        n_valid += 1
        got = (ka > kb) - (ka < kb)
        if got != r:
            bad.append((a, b, r, got))
        assert len(ka) <= 4 * len(a) + 16
    assert not bad, bad[:10]
    assert n_valid > 10000


# apk orderings pinned by the reference tests (alpine_test.go, wolfi_test.go, chainguard_test.go)
APK_PINNED = [("1.6-r0", "1.6-r1", -1), ("1.6_rc1-r0", "1.6-r0", -1), ("0.1.0_alpha", "0.1.0_alpha2", -1),
              ("0.1.0_alpha", "0.1.0_alpha_pre2", 1), ("2.6.4", "2.8.4-r0", -1)]


@pytest.mark.parametrize("a,b,want", APK_PINNED)
def test_apk_pinned(oracle_built, a, b, want):
    assert od.apk_cmp(a, b) == want
    ka, kb = key(2, a), key(2, b)
    assert (ka > kb) - (ka < kb) == want


RPM_ATOMS = [b"0", b"1", b"2", b"9", b"00", b"01", b"10", b"010", b".", b"_", b"-", b"+", b"~", b"^", b":", b"a",
             b"b", b"Z", b"el", b"el7", b"module", b"ksplice1", b"99999999999999999999999", b"\xc3\xa9", b" "]


def _gen_rpm(rng):
    s = b"".join(rng.choice(RPM_ATOMS) for _ in range(rng.randint(0, 8)))
    if rng.random() < 0.2:
        s = rng.choice([b"1:", b"0:", b"-1:", b"+2:", b":", b"a:", b"99999999999999999999:"]) + s
    return s


def test_rpm_key_matches_oracle(oracle_built):
    """go-rpm-version order (oracle/rpm.c) == byte order of the rpm sort keys (grammar 3)."""
    rng = random.Random(7)
    bad = []
    for _ in range(60000):
        a, b = _gen_rpm(rng), _gen_rpm(rng)
        r = od.rpm_cmp(a, b)
        ka, kb = key(3, a), key(3, b)
        assert ka is not None and kb is not None
        got = (ka > kb) - (ka < kb)
        if got != r:
            bad.append((a, b, r, got))
        assert len(ka) <= 3 * len(a) + 16
    assert not bad, bad[:10]


RPM_PINNED = [("3.10.0-326.36-3.el7", "0:3.10.0-327.36.3.el7", -1), ("2:7.4.160-1.el7", "2:7.4.160-6.el7_6", -1),
              ("7.29.0-59.0.1.el7_9.1", "7.29.0-59.0.1.el7_9.1", 0), ("1.0~rc1", "1.0", -1), ("1.0", "", 1)]


@pytest.mark.parametrize("a,b,want", RPM_PINNED)
def test_rpm_pinned(oracle_built, a, b, want):
    assert od.rpm_cmp(a, b) == want
    ka, kb = key(3, a), key(3, b)
    assert (ka > kb) - (ka < kb) == want
