// Parallel host encoder of the batch's transport form (wire.h).
#include "wire.h"

#include "host_par.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <thread>

namespace tvm {

namespace {

constexpr int kShardBits = 8;          // 256 dedup shards, each a private open-addressing table
constexpr uint32_t kBlock = 1u << 14;  // packages per layout / emit block
constexpr uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

// 64-bit string hash, 8 bytes per step (multiply / xor-shift mixing).  Only a sharding and
// probing hint: equal strings are decided by length + bytes.
inline uint64_t str_hash(const uint8_t* p, uint32_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t(n) * 0xC2B2AE3D27D4EB4Full);
  uint32_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t w;
    std::memcpy(&w, p + k, 8);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  if (k < n) {
    uint64_t w = 0;
    std::memcpy(&w, p + k, n - k);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  h ^= h >> 29;
  h *= 0xC4CEB9FE1A85EC53ull;
  return h ^ (h >> 32);
}

// TVM_WIRE_TRACE=1 (measurement only): per-phase host times on stderr
struct PhaseClock {
  bool on = std::getenv("TVM_WIRE_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "wire %-8s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

}  // namespace

void WireEncoder::clear() {
  wc_.clear();
  blocks_.clear();
  total_ = 0;
  hb_ = nullptr;
}

bool WireEncoder::plan(const HostBatch& hb, const std::vector<uint64_t>& toff, const std::vector<uint32_t>& bounds,
                       int threads, std::string& err) {
  clear();
  err.clear();
  PhaseClock clk;
  const size_t n = hb.pk.size();
  if (n == 0 || n >= (1ull << 31)) return false;
  hb_ = &hb;
  toff_ = &toff;
  bounds_ = bounds;
  const int T = std::max(1, std::min<int>(threads, int((n + 4095) / 4096)));
  threads_ = std::max(1, threads);
  auto range = [&](int t, size_t total) { return std::make_pair(total * size_t(t) / size_t(T), total * size_t(t + 1) / size_t(T)); };

  // 0. lengths fit a byte; platforms in first-occurrence order (a thread's range, ranges in order)
  std::vector<std::vector<uint32_t>> plats(static_cast<size_t>(T));
  std::vector<uint8_t> too_long(static_cast<size_t>(T), 0);
  run_threads(T, [&](int t) {
    auto [a, b] = range(t, n);
    uint32_t last = 0xFFFFFFFEu;
    auto& seen = plats[size_t(t)];
    for (size_t i = a; i < b; i++) {
      const uint2 d = hb.pk[i];
      if ((d.y & 0xFFFFu) > 255 || (d.y >> 16) > 255) {
        too_long[size_t(t)] = 1;
        return;
      }
      if (d.x != last) {
        last = d.x;
        if (std::find(seen.begin(), seen.end(), d.x) == seen.end()) {
          if (seen.size() > 255) return;  // more than 255 on one thread alone: no form either way
          seen.push_back(d.x);
        }
      }
    }
  });
  ptab_.clear();
  uint32_t max_plat = 0;
  for (int t = 0; t < T; t++) {
    if (too_long[size_t(t)]) return false;
    for (uint32_t p : plats[size_t(t)])
      if (std::find(ptab_.begin(), ptab_.end(), p) == ptab_.end()) {
        if (ptab_.size() == 255) return false;
        ptab_.push_back(p);
        if (p != 0xFFFFFFFFu) max_plat = std::max(max_plat, p);
      }
  }
  pidx_of_.assign(size_t(max_plat) + 1, 0);
  for (size_t k = 0; k < ptab_.size(); k++) {
    if (ptab_[k] == 0xFFFFFFFFu) pidx_absent_ = uint8_t(k);
    else pidx_of_[ptab_[k]] = uint8_t(k);
  }

  clk.lap("scan");
  // 1. per package its arena offset; per non-empty string its hash, bucketed by shard
  //    (thread-major, so a shard's strings come in string-id order)
  off_.resize(n);
  first_.resize(2 * n);
  std::vector<uint64_t> hash(2 * n);
  constexpr size_t S = size_t(1) << kShardBits;
  std::vector<std::vector<std::vector<uint32_t>>> bucket(static_cast<size_t>(T), std::vector<std::vector<uint32_t>>(S));
  const size_t n_groups = (n + kGroup - 1) / kGroup;
  const uint8_t* ar = hb.arena.data();
  run_threads(T, [&](int t) {
    auto [g0, g1] = range(t, n_groups);
    auto& bk = bucket[size_t(t)];
    for (auto& v : bk) v.reserve(2 * (g1 - g0) * kGroup / S + 16);
    for (size_t g = g0; g < g1; g++) {
      uint64_t o = toff[g];
      const size_t i1 = std::min(n, (g + 1) * kGroup);
      for (size_t i = g * kGroup; i < i1; i++) {
        off_[i] = o;
        const uint32_t nl = hb.pk[i].y & 0xFFFFu, vl = hb.pk[i].y >> 16;
        const uint32_t s0 = uint32_t(2 * i);
        first_[s0] = s0;
        first_[s0 + 1] = s0 + 1;
        if (nl) {
          const uint64_t h = str_hash(ar + o, nl);
          hash[s0] = h;
          bk[h >> (64 - kShardBits)].push_back(s0);
        }
        if (vl) {
          const uint64_t h = str_hash(ar + o + nl, vl);
          hash[s0 + 1] = h;
          bk[h >> (64 - kShardBits)].push_back(s0 + 1);
        }
        o += nl + vl;
      }
    }
  });

  clk.lap("hash");
  // 2. dedup per shard: the first string with these bytes (lowest id) is the occurrence the
  //    others refer to
  auto str_of = [&](uint32_t sid, uint32_t& len) -> const uint8_t* {
    const size_t i = sid >> 1;
    const uint32_t nl = hb.pk[i].y & 0xFFFFu;
    len = (sid & 1) ? (hb.pk[i].y >> 16) : nl;
    return ar + off_[i] + ((sid & 1) ? nl : 0);
  };
  dynamic_for(threads_, S, [&](size_t s) {
    size_t cnt = 0;
    for (int t = 0; t < T; t++) cnt += bucket[size_t(t)][s].size();
    if (!cnt) return;
    size_t cap = 16;
    while (cap < 2 * cnt) cap <<= 1;
    struct E {
      uint64_t h;
      uint32_t sid;  // + 1 (0 = empty)
      uint32_t len;
    };
    std::vector<E> tab(cap, E{0, 0, 0});
    for (int t = 0; t < T; t++)
      for (uint32_t sid : bucket[size_t(t)][s]) {
        const uint64_t h = hash[sid];
        uint32_t len;
        const uint8_t* p = str_of(sid, len);
        for (size_t k = size_t(h) & (cap - 1);; k = (k + 1) & (cap - 1)) {
          E& e = tab[k];
          if (e.sid == 0) {
            e = E{h, sid + 1, len};
            break;
          }
          if (e.h == h && e.len == len) {
            uint32_t l2;
            const uint8_t* q = str_of(e.sid - 1, l2);
            if (std::memcmp(p, q, len) == 0) {
              first_[sid] = e.sid - 1;
              break;
            }
          }
        }
      }
  });

  clk.lap("dedup");
  // 3. layout: per block the bytes of the strings it sees first; per chunk its sections, then
  //    its blocks' strings in package order
  const uint32_t nc = uint32_t(bounds.size() - 1);
  for (uint32_t c = 0; c < nc; c++) {
    const size_t p0 = std::min<size_t>(size_t(bounds[c]) * kTile, n), p1 = std::min<size_t>(size_t(bounds[c + 1]) * kTile, n);
    for (size_t a = p0; a < p1; a += kBlock)
      blocks_.push_back(Block{uint32_t(a), uint32_t(std::min<size_t>(p1, a + kBlock)), c, 0, 0});
  }
  dynamic_for(threads_, blocks_.size(), [&](size_t k) {
    Block& b = blocks_[k];
    uint64_t bytes = 0;
    for (size_t i = b.p0; i < b.p1; i++) {
      const uint32_t nl = hb.pk[i].y & 0xFFFFu, vl = hb.pk[i].y >> 16;
      if (nl && first_[2 * i] == 2 * i) bytes += nl;
      if (vl && first_[2 * i + 1] == 2 * i + 1) bytes += vl;
    }
    b.bytes = bytes;
  });
  const bool has_attr = !hb.attr.empty();
  uint64_t pos = 0;
  size_t bi = 0;
  for (uint32_t c = 0; c < nc; c++) {
    WireChunk w;
    const size_t p0 = std::min<size_t>(size_t(bounds[c]) * kTile, n), p1 = std::min<size_t>(size_t(bounds[c + 1]) * kTile, n);
    w.m = uint32_t(p1 - p0);
    w.groups = (bounds[c + 1] - bounds[c]) * kGroupsPerTile;
    w.off = pos;
    w.o_nref = pos;
    w.o_vref = align16(w.o_nref + 4ull * w.m);
    w.o_lens = align16(w.o_vref + 4ull * w.m);
    w.o_plat = align16(w.o_lens + 2ull * w.m);
    w.o_toff = align16(w.o_plat + w.m);
    w.o_attr = align16(w.o_toff + 8ull * (w.groups + 1));
    uint64_t heap = align16(w.o_attr + (has_attr ? 8ull * w.m : 0));
    for (; bi < blocks_.size() && blocks_[bi].chunk == c; bi++) {
      blocks_[bi].heap = heap;
      heap += blocks_[bi].bytes;
    }
    pos = align16(heap);
    w.bytes = pos - w.off;
    wc_.push_back(w);
  }
  if (pos >= (1ull << 32)) {  // references are 32-bit
    clear();
    return false;
  }
  total_ = pos;
  clk.lap("layout");
  return true;
}

void WireEncoder::emit(uint8_t* wire) {
  const HostBatch& hb = *hb_;
  const uint8_t* ar = hb.arena.data();
  PhaseClock clk;
  ref_.resize(first_.size());
  // strings first seen in each block, at the block's heap offset; their references
  dynamic_for(threads_, blocks_.size(), [&](size_t k) {
    const Block& b = blocks_[k];
    uint64_t h = b.heap;
    for (size_t i = b.p0; i < b.p1; i++) {
      const uint32_t nl = hb.pk[i].y & 0xFFFFu, vl = hb.pk[i].y >> 16;
      const uint32_t s0 = uint32_t(2 * i);
      if (nl && first_[s0] == s0) {
        std::memcpy(wire + h, ar + off_[i], nl);
        ref_[s0] = uint32_t(h);
        h += nl;
      }
      if (vl && first_[s0 + 1] == s0 + 1) {
        std::memcpy(wire + h, ar + off_[i] + nl, vl);
        ref_[s0 + 1] = uint32_t(h);
        h += vl;
      }
    }
  });
  clk.lap("strings");
  // per package: references, lengths, platform index; per chunk: group offsets, attributes
  dynamic_for(threads_, blocks_.size(), [&](size_t k) {
    const Block& b = blocks_[k];
    const WireChunk& w = wc_[b.chunk];
    const size_t cp0 = size_t(bounds_[b.chunk]) * kTile;
    auto* nref = reinterpret_cast<uint32_t*>(wire + w.o_nref);
    auto* vref = reinterpret_cast<uint32_t*>(wire + w.o_vref);
    auto* lens = reinterpret_cast<uint16_t*>(wire + w.o_lens);
    uint8_t* pl = wire + w.o_plat;
    for (size_t i = b.p0; i < b.p1; i++) {
      const uint32_t nl = hb.pk[i].y & 0xFFFFu, vl = hb.pk[i].y >> 16;
      const size_t li = i - cp0;
      nref[li] = nl ? ref_[first_[2 * i]] : 0;
      vref[li] = vl ? ref_[first_[2 * i + 1]] : 0;
      lens[li] = uint16_t(nl | (vl << 8));
      pl[li] = pidx(hb.pk[i].x);
    }
  });
  const bool has_attr = !hb.attr.empty();
  dynamic_for(threads_, wc_.size(), [&](size_t c) {
    const WireChunk& w = wc_[c];
    std::memcpy(wire + w.o_toff, toff_->data() + size_t(bounds_[c]) * kGroupsPerTile, 8ull * (w.groups + 1));
    if (has_attr) std::memcpy(wire + w.o_attr, hb.attr.data() + size_t(bounds_[c]) * kTile, 8ull * w.m);
  });
  clk.lap("refs");
}

}  // namespace tvm
