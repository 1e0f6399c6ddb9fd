// Host decode of the delta result form (delta_form.h).
#include "delta_form.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

#include "engine.h"
#include "host_par.h"

namespace tvm {

namespace {

// Leading non-zero bytes of q[0, n): 8 bytes per step (the lowest set bit of the SWAR
// zero-byte mask is exact).
inline uint64_t nonzero_prefix(const uint8_t* q, uint64_t n) {
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, q + i, 8);
    const uint64_t z = (w - 0x0101010101010101ull) & ~w & 0x8080808080808080ull;
    if (z) return i + (uint64_t(__builtin_ctzll(z)) >> 3);
  }
  while (i < n && q[i]) i++;
  return i;
}

inline uint32_t le24(const uint8_t* q) { return uint32_t(q[0]) | uint32_t(q[1]) << 8 | uint32_t(q[2]) << 16; }

}  // namespace

// The common tile (no list of 255 or more): the row ends from the count bytes, then ONE loop
// over the tile's entries in which nothing branches on the data - an entry is a package's
// first (3 bytes), a one-byte difference, or an escape (0 + 3 bytes), picked with selects -
// because a loop per package mispredicted its trip count and its empty packages about
// twice per package (3.6 ns per entry at 5 entries per package).
static bool decode_tile_flat(const uint8_t* h, const uint8_t* end, uint64_t pos0, uint64_t count, uint32_t* adv,
                             uint32_t* re) {
  uint32_t first[kTile + 1];
  uint32_t nf = 0, pos = 0;
  for (int p = 0; p < kTile; p++) {
    const uint32_t k = h[p];
    first[nf] = pos;
    nf += k != 0;
    pos += k;
    re[p] = uint32_t(pos0) + pos;
  }
  if (pos != count) return false;
  first[nf] = 0xFFFFFFFFu;
  const uint8_t* q = h + kTile;
  uint32_t* o = adv + pos0;
  uint32_t a = 0, f = 0, next = first[0];
  for (uint32_t e = 0; e < pos; e++) {
    uint32_t w;
    std::memcpy(&w, q, 4);
    const bool is_first = e == next;
    f += is_first;
    next = first[f];
    const uint32_t x = w & 0xFFu;
    const bool esc = !is_first && x == 0;
    a = is_first ? (w & 0xFFFFFFu) : (esc ? (w >> 8) : a + x);
    q += is_first ? 3 : (esc ? 4 : 1);
    o[e] = a;
  }
  return q == end;
}

bool delta_decode_tile(const uint8_t* stream, uint64_t stream_bytes, uint32_t t, uint64_t pos0, uint2 info,
                       uint32_t* adv, uint32_t* row_end) {
  const uint64_t count = info.x, bytes = info.y;
  uint32_t* re = row_end + size_t(t) * kTile;
  if (count == 0) {
    for (int p = 0; p < kTile; p++) re[p] = uint32_t(pos0);
    return true;
  }
  const uint64_t r = delta_region(t, pos0);
  if (bytes < kTile || r + bytes > stream_bytes) return false;
  {
    // the flat loop reads at most 4 bytes a match (+ 1 ahead) and trusts the count bytes: a
    // tile with a 255 count, or whose reads could leave the buffer, takes the loop below
    bool ext = false;
    for (int p = 0; p < kTile; p++) ext |= stream[r + p] == 255;
    if (!ext && r + kTile + 4 * count + 4 <= stream_bytes)
      return decode_tile_flat(stream + r, stream + r + bytes, pos0, count, adv, re);
  }
  const uint8_t* h = stream + r;
  const uint8_t* q = h + kTile;
  const uint8_t* end = h + bytes;
  uint32_t* o = adv + pos0;
  uint32_t* const o_end = adv + pos0 + count;
  for (int p = 0; p < kTile; p++) {
    uint64_t k = h[p];
    if (k == 255) {
      if (end - q < 4) return false;
      k = le24(q) | uint32_t(q[3]) << 24;
      q += 4;
    }
    if (k) {
      if (uint64_t(o_end - o) < k || end - q < 3) return false;
      uint32_t a = le24(q);
      q += 3;
      *o++ = a;
      // the rest: runs of one-byte differences (a branch-free running sum), each ended by an
      // escape (0 + 3 bytes) or by the list's end
      uint64_t left = k - 1;
      while (left) {
        const uint64_t f = nonzero_prefix(q, std::min<uint64_t>(left, uint64_t(end - q)));
        for (uint64_t i = 0; i < f; i++) {
          a += q[i];
          o[i] = a;
        }
        o += f;
        q += f;
        left -= f;
        if (!left) break;
        if (end - q < 4 || *q != 0) return false;
        a = le24(q + 1);
        q += 4;
        *o++ = a;
        left--;
      }
    }
    re[p] = uint32_t(o - adv);
  }
  return o == o_end && q == end;
}

bool delta_decode(const uint8_t* stream, uint64_t stream_bytes, const uint2* tile_info, uint32_t n_tiles,
                  uint64_t total, uint32_t* adv, uint32_t* row_end, std::string& err) {
  std::vector<uint64_t> b(size_t(n_tiles) + 1, 0);
  for (uint32_t t = 0; t < n_tiles; t++) b[t + 1] = b[t] + tile_info[t].x;
  if (b[n_tiles] != total) {
    err = "delta form: the tiles' counts do not add up to the pass's matches";
    return false;
  }
  std::atomic<bool> bad{false};
  range_for(n_tiles, 64, [&](size_t t0, size_t t1) {
    for (size_t t = t0; t < t1 && !bad.load(std::memory_order_relaxed); t++)
      if (!delta_decode_tile(stream, stream_bytes, uint32_t(t), b[t], tile_info[t], adv, row_end)) bad = true;
  });
  if (bad) {
    err = "delta form: a tile's stream is inconsistent with its count";
    return false;
  }
  return true;
}

}  // namespace tvm
