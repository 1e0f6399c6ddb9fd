"""A plain-Python restatement of the pipeline's delta result form (trivy_amd/csrc/delta_form.h)
for the tests: encode the per-package advisory lists of a batch the way the GPU result move
does, and decode streams the way the host does.  Small inputs only (pure-Python loops)."""
import numpy as np

TILE = 256


def region(t, b):
    """Byte offset of tile t's stream, b = the CSR position of its first match (engine.h)."""
    return ((288 * t + 5 * b) >> 4) << 4


def stream_bytes(n_tiles, cap):
    return 288 * n_tiles + 5 * cap + 64


def encode_tile(lists):
    """The stream of one tile: lists = 256 lists of advisory indices (< 2^24)."""
    out = bytearray(min(len(x), 255) for x in lists)
    for x in lists:
        if not x:
            continue
        if len(x) >= 255:
            out += int(len(x)).to_bytes(4, "little")
        out += int(x[0]).to_bytes(3, "little")
        for prev, a in zip(x, x[1:]):
            d = (a - prev) & 0xFFFFFFFF
            if 1 <= d <= 255:
                out.append(d)
            else:
                out.append(0)
                out += int(a).to_bytes(3, "little")
    return bytes(out)


def encode(adv, row_end, n_tiles, cap):
    """(stream uint8, tile_info uint32[n_tiles, 2]) for a CSR (row_end per package, padded to
    whole tiles by the caller or not)."""
    rend = np.zeros(n_tiles * TILE, np.int64)
    rend[:len(row_end)] = row_end
    rend[len(row_end):] = row_end[-1] if len(row_end) else 0
    stream = np.zeros(stream_bytes(n_tiles, cap), np.uint8)
    info = np.zeros((n_tiles, 2), np.uint32)
    b = 0
    for t in range(n_tiles):
        lists = []
        for p in range(t * TILE, (t + 1) * TILE):
            lo = rend[p - 1] if p else 0
            lists.append([int(v) for v in adv[lo:rend[p]]])
        count = sum(len(x) for x in lists)
        info[t, 0] = count
        if count:
            s = encode_tile(lists)
            r = region(t, b)
            stream[r:r + len(s)] = np.frombuffer(s, np.uint8)
            info[t, 1] = len(s)
        b += count
    return stream, info


def decode(stream, info):
    """(adv, row_end[n_tiles * 256]) of the streams."""
    adv, rend, b = [], [], 0
    for t, (count, nbytes) in enumerate(info.tolist()):
        if count == 0:
            rend += [b] * TILE
            continue
        s = bytes(stream[region(t, b):region(t, b) + nbytes])
        q = TILE
        for p in range(TILE):
            k = s[p]
            if k == 255:
                k = int.from_bytes(s[q:q + 4], "little")
                q += 4
            if k:
                a = int.from_bytes(s[q:q + 3], "little")
                q += 3
                adv.append(a)
                for _ in range(k - 1):
                    d = s[q]
                    q += 1
                    if d:
                        a += d
                    else:
                        a = int.from_bytes(s[q:q + 3], "little")
                        q += 3
                    adv.append(a)
            rend.append(len(adv))
        assert q == nbytes and len(adv) == b + count
        b += count
    return np.array(adv, np.uint32), np.array(rend, np.uint32)
