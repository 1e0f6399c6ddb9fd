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
