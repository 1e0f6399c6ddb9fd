"""A plain-numpy restatement of the pipeline's byte result form (trivy_amd/csrc/byte_form.h)
for the tests: the arrays the GPU result move writes for a CSR, and their decode."""
import numpy as np

TILE = 256


def encode(adv, row_end, n_tiles):
    """(bytes uint8[n], hi uint16[n_tiles * 256], wide uint32[n], escapes) of a CSR (row_end per
    package, padded to whole tiles by repeating the last value)."""
    adv = np.asarray(adv, np.int64)
    n = len(adv)
    rend = np.zeros(n_tiles * TILE, np.int64)
    rend[:len(row_end)] = row_end
    rend[len(row_end):] = row_end[-1] if len(row_end) else 0
    start = np.concatenate([[0], rend[:-1]])
    pkg = np.repeat(np.arange(n_tiles * TILE), rend - start)
    first = np.ones(n, bool)
    first[1:] = pkg[1:] != pkg[:-1]
    d = np.zeros(n, np.int64)
    d[1:] = adv[1:] - adv[:-1]
    esc = ~first & ((d < 1) | (d > 254))
    b = np.where(first, adv & 0xFF, np.where(esc, 0xFF, d)).astype(np.uint8)
    hi = np.zeros(n_tiles * TILE, np.uint16)
    hi[pkg[first]] = (adv[first] >> 8).astype(np.uint16)
    wide = np.zeros(n, np.uint32)
    wide[esc] = adv[esc]
    return b, hi, wide, int(esc.sum())


def decode(b, hi, wide, row_end, n):
    """The advisory indices (pure Python loop: small inputs)."""
    out = np.zeros(n, np.uint32)
    prev = 0
    for p, e in enumerate(row_end.tolist()):
        a = 0
        for i in range(prev, e):
            if i == prev:
                a = (int(hi[p]) << 8) | int(b[i])
            elif b[i] == 0xFF:
                a = int(wide[i])
            else:
                a += int(b[i])
            out[i] = a
        prev = e
    return out
