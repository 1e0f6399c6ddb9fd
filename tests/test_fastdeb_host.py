"""CPU: the match kernel's lane-serial dpkg key builder (verkey.h deb_fast_key, the code the
kernel runs, built for the host) equals the generic dpkg encoder (deb_encode, itself checked
against the independent comparator oracle/deb.c) on every version it accepts, at every
dword alignment; versions it hands back (FAST_FALLBACK) are the rare shapes the generic
encoder keeps: non-ASCII bytes, signed / long / empty epochs, digit runs over 9 significant
digits, keys over 39 bytes."""
import ctypes
import random

import pytest

from trivy_amd._lib import lib

_BUF = ctypes.create_string_buffer(1 << 12)
_OUT = ctypes.create_string_buffer(64)


def generic(v):
    n = lib().tvm_version_key(1, v, len(v), _BUF, len(_BUF))
    return None if n < 0 else _BUF.raw[:n]


def fast(v, shift):
    n = lib().tvm_deb_fast_key_host(v, len(v), shift, _OUT, len(_OUT))
    if n == -2:
        return "fallback"
    return None if n < 0 else _OUT.raw[:n]


def check(v):
    want = generic(v)
    for sh in range(4):
        got = fast(v, sh)
        if got == "fallback":
            return "fallback"
        assert got == want, (v, sh, got, want)
    return "ok" if want is not None else "invalid"


FIXED = [b"", b"0", b"1", b"1.0", b"1:1.0", b"0:1.0-1", b"1.0-", b"-1", b"1-", b"a1.0", b"1.0~rc1-1", b"1.0+dfsg-1ubuntu0.1",
         b"2:1.2.3-4+deb12u1", b"1:2:3-4", b"1:2-3:4", b"1.2-3-4", b"10:1", b"123456789:1", b"1234567890:1",
         b"+1:1.0", b"-1:1.0", b":1.0", b"1::2", b"1.0-a:b", b"1.0_1", b"1.0 1", b"1.0\x00", b"1.\xc3\xa9",
         b"999999999", b"1000000000", b"0000000001234", b"00000000000000000000", b"4294967295",
         b"1.0-0", b"1.0-00", b"1.0-ubuntu", b"7.25.12-4", b"12.13.4-3+deb12u3", b"1~", b"1~~a", b"1.a.b.c.d.e.f.g.h.i",
         b"1.2.3.4.5.6.7.8.9.10.11.12-13.14.15", b"5:1.0", b"1:", b"1:-", b"1.0-1.0-1.0"]


def test_fixed_cases():
    seen = {check(v) for v in FIXED}
    assert {"ok", "invalid", "fallback"} <= seen


def test_synthetic_c2_versions_never_fall_back():
    """The C2 bench batch's versions all take the fast path (no divergent fallback lanes)."""
    from tools.synth import make_db, make_batch
    sdb = make_db(["debian 12", "ubuntu 22.04"], 2000, seed=7)
    batch = make_batch(sdb, 40, 200, [3, 2], seed=7)
    stats = {}
    for v in batch.versions:
        r = check(v)
        stats[r] = stats.get(r, 0) + 1
    assert stats.get("fallback", 0) == 0, stats
    assert stats["ok"] > 0.99 * len(batch.versions) - 100


@pytest.mark.parametrize("seed", range(4))
def test_random_versions(seed):
    rnd = random.Random(seed)
    alpha = b"0123456789" * 4 + b".+-:~_abzAZ" + b"-:.~" * 2 + b"!/ \xe9"
    stats = {}
    for _ in range(4000):
        n = rnd.randint(0, 28)
        v = bytes(rnd.choice(alpha) for _ in range(n))
        if rnd.random() < 0.5 and v:  # mostly well-formed: start with a digit
            v = b"%d" % rnd.randint(0, 99) + v
        r = check(v)
        stats[r] = stats.get(r, 0) + 1
    assert stats.get("ok", 0) > 500 and stats.get("invalid", 0) > 100, stats
