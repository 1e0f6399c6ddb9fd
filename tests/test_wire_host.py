"""CPU: the batch's transport form (trivy_amd/csrc/wire.cpp, what a pipelined pass sends over
PCIe) decodes back to exactly the batch - every package's platform, name and version - for
ragged batches, empty strings, strings shared between names and versions and across chunks;
it is byte-identical for 1 and many host threads; every string crosses once (references
point back to the first occurrence); batches with a 256-byte string or more than 255
platforms have no transport form.  Decoding here is the host restatement of unpack_kernel."""
import ctypes

import numpy as np
import pytest

from trivy_amd._lib import lib
from trivy_amd.batch import arena_of


def encode(plat, names, vers, chunk, threads):
    arena, [(no, nl), (vo, vl)] = arena_of(names, vers)
    plat = np.asarray(plat, dtype=np.uint32)
    args = (len(plat), plat.ctypes.data, arena, no.ctypes.data, nl.ctypes.data, vo.ctypes.data, vl.ctypes.data,
            chunk, threads)
    nb, nc, npl = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
    assert lib().tvm_wire_encode(*args, None, 0, ctypes.byref(nb), None, 0, ctypes.byref(nc), None, 0,
                                 ctypes.byref(npl)) == 0
    if nb.value == 0:
        return None
    out = np.zeros(nb.value, dtype=np.uint8)
    ch = np.zeros((nc.value, 10), dtype=np.uint64)
    pt = np.zeros(max(npl.value, 1), dtype=np.uint32)
    assert lib().tvm_wire_encode(*args, out.ctypes.data, len(out), ctypes.byref(nb), ch.ctypes.data, nc.value,
                                 ctypes.byref(nc), pt.ctypes.data, len(pt), ctypes.byref(npl)) == 0
    return out, ch, pt[:npl.value]


def decode(wire, chunks, ptab):
    """unpack_kernel's rebuild, on the host: per package (platform id, name, version)."""
    out = []
    for off, nbytes, o_n, o_v, o_l, o_p, o_t, o_a, m, groups in chunks.astype(np.int64):
        nref = wire[o_n:o_n + 4 * m].view(np.uint32)
        vref = wire[o_v:o_v + 4 * m].view(np.uint32)
        lens = wire[o_l:o_l + 2 * m].view(np.uint16)
        pl = wire[o_p:o_p + m]
        for i in range(m):
            nl, vl = int(lens[i]) & 255, int(lens[i]) >> 8
            out.append((int(ptab[pl[i]]), bytes(wire[nref[i]:nref[i] + nl]), bytes(wire[vref[i]:vref[i] + vl])))
            # a reference never points past its own chunk (it is a first occurrence in this or an earlier chunk)
            assert nref[i] + nl <= off + nbytes and vref[i] + vl <= off + nbytes
    return out


def _batch(n, seed):
    rng = np.random.default_rng(seed)
    pool = [b"pkg%d" % i for i in range(n // 7 + 3)]
    vpool = [b"%d.%d-%d" % (rng.integers(0, 9), rng.integers(0, 30), rng.integers(0, 5)) for _ in range(n // 11 + 3)]
    names = [pool[int(rng.zipf(1.3)) % len(pool)] for _ in range(n)]
    vers = [vpool[int(rng.integers(0, len(vpool)))] for _ in range(n)]
    for i in range(0, n, 13):
        vers[i] = b""
    for i in range(5, n, 17):
        vers[i] = names[i]  # a version equal to a name: one string, referenced twice
    for i in range(9, n, 29):
        names[i] = b""
    plat = [[3, 7, 0xFFFFFFFF, 1][(i // 300) % 4] for i in range(n)]
    return plat, names, vers


@pytest.mark.parametrize("n,chunk", [(1, 256), (700, 256), (12321, 1000), (40000, 1 << 20), (70001, 8192)])
def test_round_trip_and_thread_invariance(n, chunk):
    plat, names, vers = _batch(n, n)
    one = encode(plat, names, vers, chunk, 1)
    many = encode(plat, names, vers, chunk, 8)
    assert one is not None
    assert np.array_equal(one[1], many[1]) and np.array_equal(one[2], many[2])
    w1, wm = one[0], many[0]
    got = decode(*one)
    assert got == list(zip(plat, names, vers))
    assert decode(*many) == got
    # the string sections agree byte for byte (pads aside): every chunk's sections
    for off, nbytes, o_n, o_v, o_l, o_p, o_t, o_a, m, groups in one[1].astype(np.int64):
        for a, ln in ((o_n, 4 * m), (o_v, 4 * m), (o_l, 2 * m), (o_p, m), (o_t, 8 * (groups + 1))):
            assert np.array_equal(w1[a:a + ln], wm[a:a + ln])
    # each distinct non-empty string crosses once
    distinct = {s for s in names + vers if s}
    heap = sum(int(c[1]) for c in one[1])
    assert heap >= sum(len(s) for s in distinct)
    refs = set()
    for off, nbytes, o_n, o_v, o_l, o_p, o_t, o_a, m, groups in one[1].astype(np.int64):
        lens = w1[o_l:o_l + 2 * m].view(np.uint16)
        for r, ln in zip(w1[o_n:o_n + 4 * m].view(np.uint32), lens & 255):
            if ln:
                refs.add(int(r))
        for r, ln in zip(w1[o_v:o_v + 4 * m].view(np.uint32), lens >> 8):
            if ln:
                refs.add(int(r))
    assert len(refs) == len(distinct)


def test_no_transport_form():
    plat, names, vers = _batch(500, 3)
    vers[100] = b"1." + b"9" * 254  # 256 bytes
    assert encode(plat, names, vers, 256, 4) is None
    plat2 = list(range(300))  # 300 platforms
    assert encode(plat2, [b"a"] * 300, [b"1"] * 300, 256, 4) is None
    assert encode(plat2[:255], [b"a"] * 255, [b"1"] * 255, 256, 4) is not None
