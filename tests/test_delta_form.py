"""The delta result form (trivy_amd/csrc/delta_form.h): the host decoder behind
tvm_pipeline_result (tvm_delta_decode) against the Python restatement tests/delta_ref.py on
CSRs that exercise every rule - packages without matches, lists of 255 or more (the count
escape), differences of 0, of more than 255 and negative ones (the index escape), empty
tiles, a ragged last tile - and its refusal of inconsistent streams.  The GPU side (the
result move writing the form) is tests/test_gpu_pipeline.py."""
import ctypes

import numpy as np
import pytest

import delta_ref as dr
from trivy_amd._lib import errbuf, lib


def _native_decode(stream, info, n):
    nt = len(info)
    adv = np.zeros(max(n, 1), np.uint32)
    rend = np.zeros(max(nt * 256, 1), np.uint32)
    e = errbuf()
    ti = np.ascontiguousarray(info, np.uint32)
    rc = lib().tvm_delta_decode(stream.ctypes.data, len(stream), ti.ctypes.data, nt, n, adv.ctypes.data,
                                rend.ctypes.data, e, len(e))
    if rc:
        raise ValueError(e.value.decode())
    return adv[:n], rend[:nt * 256]


def _csr(rng, n_pkgs, kind):
    counts = rng.choice([0, 0, 1, 2, 3, 7, 20], size=n_pkgs)
    if kind == "heavy":
        counts[rng.integers(0, n_pkgs, 3)] = [255, 300, 4571][:min(3, n_pkgs)]
    if kind == "empty_tiles":
        counts[256:768] = 0
    lists = []
    for c in counts:
        a = int(rng.integers(0, 1 << 24))
        x = []
        for _ in range(int(c)):
            x.append(a)
            step = rng.choice([1, 1, 2, 5, 46, 255, 256, 100000, -3, 0])
            a = int((a + step) % (1 << 24))
        lists.append(x)
    adv = np.array([v for x in lists for v in x], np.uint32)
    return adv, np.cumsum([len(x) for x in lists]).astype(np.uint32)


@pytest.mark.parametrize("kind,n_pkgs", [("plain", 1000), ("heavy", 700), ("empty_tiles", 1100), ("plain", 256),
                                         ("plain", 1)])
def test_native_decode_equals_reference(kind, n_pkgs):
    rng = np.random.default_rng(n_pkgs)
    adv, rend = _csr(rng, n_pkgs, kind)
    nt = -(-n_pkgs // 256)
    stream, info = dr.encode(adv, rend, nt, cap=len(adv) + 3)
    a, r = _native_decode(stream, info, len(adv))
    ra, rr = dr.decode(stream, info)
    assert np.array_equal(a, adv) and np.array_equal(ra, adv)
    assert np.array_equal(r[:n_pkgs], rend) and np.array_equal(rr, r)
    assert np.all(r[n_pkgs:] == (rend[-1] if len(rend) else 0))
    # the form's size: the heavy lists pay their 4-byte counts, the rest ~1-4 bytes a match
    assert info[:, 1].sum() <= 256 * nt + 4 * len(adv) + 4 * 3


def test_native_decode_refuses_inconsistent_streams():
    rng = np.random.default_rng(3)
    adv, rend = _csr(rng, 600, "plain")
    stream, info = dr.encode(adv, rend, 3, cap=len(adv))
    bad = info.copy()
    bad[1, 0] += 1  # counts no longer add up to the total
    with pytest.raises(ValueError, match="add up"):
        _native_decode(stream, bad, len(adv))
    bad = info.copy()
    bad[0, 1] -= 1  # a stream cut short
    with pytest.raises(ValueError, match="inconsistent"):
        _native_decode(stream, bad, len(adv))
    s2 = stream.copy()
    s2[dr.region(0, 0)] ^= 1  # a count byte changed
    with pytest.raises(ValueError):
        _native_decode(s2, info, len(adv))


def test_region_matches_reference():
    for t, b in [(0, 0), (1, 7), (5, 1000), (70000, 3 << 30)]:
        assert lib().tvm_delta_region(t, b) == dr.region(t, b)


# ---- the byte form (trivy_amd/csrc/byte_form.h, TVM_PIPE_BYTE) ----------------------------

@pytest.mark.parametrize("kind,n_pkgs", [("plain", 1000), ("heavy", 700), ("empty_tiles", 1100), ("plain", 1)])
def test_byte_form_native_decode_equals_reference(kind, n_pkgs):
    import byte_ref as br
    rng = np.random.default_rng(n_pkgs + 7)
    adv, rend = _csr(rng, n_pkgs, kind)
    nt = -(-n_pkgs // 256)
    b, hi, wide, n_esc = br.encode(adv, rend, nt)
    rpad = np.zeros(nt * 256, np.uint32)
    rpad[:len(rend)] = rend
    rpad[len(rend):] = rend[-1] if len(rend) else 0
    assert np.array_equal(br.decode(b, hi, wide, rpad, len(adv)), adv)
    out = np.zeros(max(len(adv), 1), np.uint32)
    bb = np.concatenate([b, np.zeros(16, np.uint8)])
    esc = lib().tvm_byte_decode(bb.ctypes.data, hi.ctypes.data, np.ascontiguousarray(wide).ctypes.data,
                                rpad.ctypes.data, nt, out.ctypes.data)
    assert esc == n_esc and (n_pkgs < 10 or n_esc > 0)
    assert np.array_equal(out[:len(adv)], adv)
