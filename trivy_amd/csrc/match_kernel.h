// The fused match kernel (gfx950 / CDNA4), as templates.
//
// Replaces the per-package loops of the reference drivers (e.g.
// pkg/detector/ospkg/debian/debian.go:65-117, ubuntu/ubuntu.go:86-126,
// library/driver.go:111-137) with one launch over a whole batch of packages from
// many targets.  One workgroup owns a tile of T consecutive packages (one per lane):
//
//   0. stage: the tile's name/version bytes (one contiguous arena window) are copied
//      into LDS with coalesced 16-byte loads, so the byte-serial hashing/parsing below
//      runs on LDS latency instead of global latency;
//   1. probe+encode (lane per package): hash (platform, name), linear-probe the
//      open-addressing index (slot hash and value loaded together), verify the name
//      bytes, and encode the installed version into its sort key in LDS (verkey.h, the
//      same code the flattener ran on the advisory side at load time);
//   2. block exclusive scan of the per-package row counts (wave shuffles + LDS);
//   3. pair sweep: the tile's (package, row) pairs are dealt T at a time to the lanes
//      (binary search of the LDS scan maps pair -> package); each pair is one interval
//      test against a 32-byte row whose first 16 key bytes are inline, so most pairs
//      cost one row load; the next chunk's row is loaded before the current one is
//      tested (software pipelining); a Zipf-heavy key makes its tile loop longer, never
//      a single lane;
//   4. ballot/popcount compaction into an LDS match buffer, then one atomic reservation
//      per tile and a tile directory entry: the per-package advisory lists come out in
//      (package, row) order within each tile segment with no inter-tile waiting.
//
// All arithmetic is integer/byte; the kernel is bound by memory latency/traffic
// (rows, keys, descriptors, strings), never by ALU.
//
// The templates are instantiated in kern_*.hip, one translation unit per grammar set
// (libver.h GM_*) and variant list (match_variants.h), so the build compiles them in
// parallel; engine.hip only holds the launch tables.
#pragma once
#include "engine.h"
#include "libver.h"

namespace tvm {

struct MatchArgs {
  DevDB db;
  const uint4* desc;
  const uint8_t* arena;
  const uint2* attr;       // per-package attributes, nullptr when no row of the DB filters
  const uint32_t* cpe_bits;
  uint32_t cpe_words;
  uint32_t n_cpe_sets;
  uint32_t n;
  uint32_t n_tiles;
  uint2* out;
  uint64_t out_cap;
  TileDir* dir;
  unsigned long long* ctl;  // [0] total, [1] n - first poisoned, [2] spill used, [3] err bits, [4] ticket, [5] tile size
  uint64_t* spill;
  uint64_t spill_cap;
  uint64_t* kbuf;  // KG variants: installed-key slots in global memory, KW words per package
};

using LaunchFn = void (*)(uint32_t n_tiles, hipStream_t st, const MatchArgs& a);

namespace {

enum : uint32_t { KI_VALID = 1u << 31, KI_SPILL = 1u << 30, KI_LEN = 0x3FFFu, KI_CLS_SHIFT = 26, KI_CLS_MASK = 7u };

// FILT: the batch's grammar set has rows with per-package predicates (RowAux); dpkg-only
// batches (GM_DEB) never do, so their tiles carry no package attributes (2 KB less LDS per
// block = one more resident workgroup per CU).
template <int T, int KW, int MB, bool KG, bool FILT>
struct TileShared {
  uint64_t key[KG ? 1 : T * KW];  // installed keys (KG: in global memory instead)
  union {
    uint2 mbuf[MB];           // phase 3: compacted matches
    uint4 stage[MB / 2];      // phase 0/1: the tile's name/version bytes
  };
  uint32_t scan[T + 1];       // exclusive scan of row counts
  uint32_t rbeg[T];           // first row per package
  uint32_t kinfo[T];          // key length | flags
  uint32_t koff[T];           // spill word offset when KI_SPILL
  uint2 pattr[FILT ? T : 1];  // package attributes (filtered rows only)
  uint32_t wsum[T / 64];
  uint32_t tile;
  uint32_t span_lo, span_hi;  // arena window of the tile's strings
  unsigned long long base;
};

__device__ __forceinline__ bool name_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

// key_hash (common.h) fused with packing the name's first kSlotNameWords*8 bytes into
// words (memory order, zero padded), so the slot's inline name is verified with word
// compares.  Registers only (an if-chain, no dynamically indexed array).
__device__ __forceinline__ uint64_t hash_pack(uint32_t plat, const uint8_t* s, uint32_t n,
                                              uint64_t (&w)[kSlotNameWords]) {
  static_assert(kSlotNameWords == 5, "hash_pack fills exactly five words");
  uint64_t h = key_hash_seed(plat), cur = 0;
  w[0] = w[1] = w[2] = w[3] = w[4] = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    h = key_hash_step(h, c);
    cur |= uint64_t(c) << (8 * (i & 7));
    if ((i & 7) == 7 || i + 1 == n) {  // a word is complete (or the name ends)
      const uint32_t k = i >> 3;
      if (k == 0) w[0] = cur;
      else if (k == 1) w[1] = cur;
      else if (k == 2) w[2] = cur;
      else if (k == 3) w[3] = cur;
      else if (k == 4) w[4] = cur;
      cur = 0;
    }
  }
  return key_hash_fin(h);
}

// Name check against a slot (its first 40 bytes inline, loaded with the hash); names
// longer than 40 bytes finish bytewise against the name arena.
__device__ __forceinline__ bool name_eq_slot(const uint64_t (&w)[kSlotNameWords], const uint4 q1, const uint4 q2,
                                             const uint4 q3, const uint8_t* name, const uint8_t* arena, uint32_t n) {
  const uint64_t y0 = q1.z | (uint64_t(q1.w) << 32), y1 = q2.x | (uint64_t(q2.y) << 32),
                 y2 = q2.z | (uint64_t(q2.w) << 32), y3 = q3.x | (uint64_t(q3.y) << 32),
                 y4 = q3.z | (uint64_t(q3.w) << 32);
  bool eq = w[0] == y0;  // zero padded on both sides, so a short name compares whole words
  eq &= w[1] == y1;
  eq &= w[2] == y2;
  eq &= w[3] == y3;
  eq &= w[4] == y4;
  if (eq && n > 8 * kSlotNameWords) {
    const uint8_t* full = arena + q1.y;
    for (uint32_t i = 8 * kSlotNameWords; eq && i < n; i++) eq = full[i] == name[i];
  }
  return eq;
}

// Block-wide exclusive scan of v over T lanes; returns the block total.
template <int T, class S>
__device__ __forceinline__ uint32_t block_scan(S& s, uint32_t v, uint32_t tid) {
  constexpr int W = T / 64;
  const uint32_t lane = tid & 63, wave = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= uint32_t(d)) x += y;
  }
  if (lane == 63) s.wsum[wave] = x;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < W; w++) {
    uint32_t t = s.wsum[w];
    off += (uint32_t(w) < wave) ? t : 0;
    tot += t;
  }
  s.scan[tid] = off + x - v;
  if (tid == 0) s.scan[T] = tot;
  __syncthreads();
  return tot;
}

// Package of pair j: the last q with scan[q] <= j (its count is > 0 since j < scan[q + 1]).
template <int T, class S>
__device__ __forceinline__ uint32_t pair_pkg(const S& s, uint32_t j) {
  uint32_t lo = 0, hi = T;  // invariant: scan[lo] <= j < scan[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s.scan[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Per-package predicates of a ROW_FILTER row (common.h RowAux).
__device__ __forceinline__ bool aux_pass(const MatchArgs& a, uint32_t ridx, uint2 pa, uint32_t ki) {
  const RowAux x = a.db.aux[ridx];
  const uint32_t* ids = a.db.aux_ids + x.list_off;
  if (x.kind & (AUX_ARCH_RH | AUX_ARCH_IN)) {
    bool ok = (x.kind & AUX_ARCH_RH) && (x.n_arch == 0 || (pa.x & PA_NOARCH));
    const uint32_t arch = pa.x & PA_ARCH_MASK;
    for (uint32_t i = 0; i < x.n_arch && !ok; i++) ok = ids[i] == arch;
    if (!ok) return false;
  }
  if (x.kind & AUX_CPE) {
    if (pa.y >= a.n_cpe_sets) return false;
    const uint32_t* set = a.cpe_bits + size_t(pa.y) * a.cpe_words;
    bool ok = false;
    for (uint32_t i = 0; i < x.n_cpe && !ok; i++) {
      const uint32_t c = ids[x.n_arch + i];
      ok = (c >> 5) < a.cpe_words && ((set[c >> 5] >> (c & 31)) & 1u);
    }
    if (!ok) return false;
  }
  if ((x.kind & AUX_TAG) && x.tag != pa.y) return false;
  if ((x.kind & AUX_CLASS) && !((x.tag >> ((ki >> KI_CLS_SHIFT) & KI_CLS_MASK)) & 1u)) return false;
  return true;
}

// The installed key's first two words are kept big-endian and zero-masked beyond the key
// length (be_head, applied once per package in phase 1), like Row::hi_pre*, so an interval
// bound test is two u64 compares; only 16-byte ties with both keys longer read the tails
// (memory-order words from word 2 on).
__device__ __forceinline__ uint64_t be_word(uint64_t w, uint32_t bytes) {  // bytes in [1, 8]
  if (bytes < 8) w &= (1ull << (8 * bytes)) - 1ull;
  return __builtin_bswap64(w);
}
__device__ __forceinline__ void be_head(uint64_t* k, uint32_t n) {
  const uint64_t w0 = n ? be_word(k[0], n < 8 ? n : 8) : 0ull;
  const uint64_t w1 = n > 8 ? be_word(k[1], n < 16 ? n - 8 : 8) : 0ull;
  k[0] = w0;
  k[1] = w1;
}
// sign(installed key - bound): a0/a1 the installed BE head, b0/b1 the bound's BE head.
__device__ __forceinline__ int cmp_be(uint64_t a0, uint64_t a1, const uint64_t* a, uint32_t na, uint64_t b0,
                                      uint64_t b1, const uint64_t* b, uint32_t nb) {
  if (a0 != b0) return a0 < b0 ? -1 : 1;
  if (a1 != b1) return a1 < b1 ? -1 : 1;
  if (na <= 16 || nb <= 16) return (na > nb) - (na < nb);
  return key_cmp(a + 2, na - 16, b + 2, nb - 16);
}

// Installed key of tile package q: the global spill area for long keys, else its slot
// (LDS, or global memory for KG variants).
template <int T, int KW, bool KG, class S>
__device__ __forceinline__ const uint64_t* key_ptr(const MatchArgs& a, const S& s, uint32_t q) {
  if (s.kinfo[q] & KI_SPILL) return a.spill + s.koff[q];
  if constexpr (KG) return a.kbuf + size_t(s.tile * T + q) * KW;
  else return &s.key[q * KW];
}

// Interval test of package q's installed key (k; first two words k0, k1 already loaded)
// against one row (global index ridx).
template <bool FILT, class S>
__device__ __forceinline__ bool eval_row(const MatchArgs& a, const S& s, uint32_t q, const Row& row, uint32_t ridx,
                                         const uint64_t* k, uint64_t k0, uint64_t k1) {
  if constexpr (FILT) {
    if ((row.adv & ROW_FILTER) && !aux_pass(a, ridx, s.pattr[q], s.kinfo[q])) return false;
  }
  if (row.adv & ROW_ALWAYS) return true;
  const uint32_t ki = s.kinfo[q];
  if (!(ki & KI_VALID)) return false;
  const uint32_t kl = ki & KI_LEN;
  bool m = true;
  if (!(row.hi_len & KEY_INF)) {
    const int c = cmp_be(k0, k1, k, kl, row.hi_pre0, row.hi_pre1, a.db.key_words + row.hi_off,
                         row.hi_len & KEY_LEN_MASK);
    m = (row.hi_len & KEY_INCL) ? c <= 0 : c < 0;
  }
  if (m && !(row.lo_len & KEY_INF)) {  // rare (library / rpm ranges): the bound's head from the arena
    const uint64_t* lw = a.db.key_words + row.lo_off;
    const uint32_t nl = row.lo_len & KEY_LEN_MASK;
    const uint64_t l0 = nl ? be_word(lw[0], nl < 8 ? nl : 8) : 0ull;
    const uint64_t l1 = nl > 8 ? be_word(lw[1], nl < 16 ? nl - 8 : 8) : 0ull;
    const int c = cmp_be(k0, k1, k, kl, l0, l1, lw, nl);
    m = (row.lo_len & KEY_INCL) ? c >= 0 : c > 0;
  }
  return m;
}

// One sweep over the tile's pairs.  DIRECT=false: compact into LDS (count all, store the
// first MB).  DIRECT=true: store straight to out[base + position].
// AB (ablation, diagnostics only): 2 = load rows but skip the key compare.
template <int T, int KW, int MB, bool KG, bool FILT, bool DIRECT, int AB = 0>
__device__ __forceinline__ uint32_t sweep(const MatchArgs& a, TileShared<T, KW, MB, KG, FILT>& s, uint32_t total_pairs,
                                          uint32_t tid, unsigned long long base) {
  constexpr int W = T / 64;
  const uint32_t lane = tid & 63, wave = tid >> 6;
  uint32_t nm = 0;
  uint32_t j = tid, q = 0, ridx = 0;
  Row row{};
  const uint64_t* kp = nullptr;
  uint64_t k0 = 0, k1 = 0;  // KG: the key's first words travel with the row load
  if (j < total_pairs) {
    q = pair_pkg<T>(s, j);
    ridx = s.rbeg[q] + (j - s.scan[q]);
    row = a.db.rows[ridx];
    kp = key_ptr<T, KW, KG>(a, s, q);
    if (KG) k0 = kp[0], k1 = kp[1];
  }
  for (uint32_t b0 = 0; b0 < total_pairs; b0 += T) {
    // issue the next chunk's row load before testing this chunk's pair
    const uint32_t jn = j + T;
    uint32_t qn = 0, ridxn = 0;
    Row rown{};
    const uint64_t* kpn = nullptr;
    uint64_t k0n = 0, k1n = 0;
    if (jn < total_pairs) {
      qn = pair_pkg<T>(s, jn);
      ridxn = s.rbeg[qn] + (jn - s.scan[qn]);
      rown = a.db.rows[ridxn];
      kpn = key_ptr<T, KW, KG>(a, s, qn);
      if (KG) k0n = kpn[0], k1n = kpn[1];
    }
    if (!KG && j < total_pairs) {
      if (s.kinfo[q] & KI_SPILL) k0 = kp[0], k1 = kp[1];
      else k0 = s.key[q * KW], k1 = s.key[q * KW + 1];  // LDS loads, not flat ones
    }
    const bool m = (j < total_pairs) && (AB == 2 ? (row.adv & 7u) == 0 : eval_row<FILT>(a, s, q, row, ridx, kp, k0, k1));
    const unsigned long long bal = __ballot(m);
    const uint32_t lane_off = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) s.wsum[wave] = uint32_t(__popcll(bal));
    __syncthreads();
    uint32_t woff = 0, ctot = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint32_t t = s.wsum[w];
      woff += (uint32_t(w) < wave) ? t : 0;
      ctot += t;
    }
    const uint32_t pos = nm + woff + lane_off;
    if (m) {
      const uint2 rec = make_uint2(s.tile * T + q, row.adv & ROW_ADV_MASK);
      if (DIRECT) {
        if (base + pos < a.out_cap) a.out[base + pos] = rec;
      } else if (pos < uint32_t(MB)) {
        s.mbuf[pos] = rec;
      }
    }
    nm += ctot;
    __syncthreads();
    j = jn;
    q = qn;
    ridx = ridxn;
    row = rown;
    kp = kpn;
    k0 = k0n;
    k1 = k1n;
  }
  return nm;
}

// Phase 1 for one package: encode the installed version into its key slot and probe the
// index.  Instantiated separately for LDS-staged and global string pointers so the staged
// case compiles to LDS loads rather than generic (flat) ones.
template <int T, int KW, int MB, bool KG, bool FILT, uint32_t GM, int AB>
__device__ __forceinline__ void probe_encode(const MatchArgs& a, TileShared<T, KW, MB, KG, FILT>& s, uint32_t tid,
                                             uint32_t p, const uint4 d, const uint8_t* name, const uint8_t* ver,
                                             uint32_t& cnt, uint32_t& rbeg, uint32_t& kinfo, uint32_t& koff) {
  const PlatInfo pi = a.db.plats[d.x];
  const uint32_t nlen = d.w & 0xFFFFu, vlen = d.w >> 16;
  // installed version -> sort key: one optimistic pass into the LDS slot; a key longer
  // than the slot is re-encoded into the global spill area
  bool valid = AB == 4;
  if (AB != 4) {
    uint64_t* slot;
    if constexpr (KG) slot = a.kbuf + size_t(p) * KW;
    else slot = &s.key[tid * KW];
    CapWordSink cs(slot, KW * 8);
    uint32_t cls = 0;
    valid = encode_version_gm<GM>(pi.cmp, ver, vlen, cs, cls);
    cs.flush();
    if (valid && cs.n > uint32_t(KW * 8)) {
      const uint32_t need = (cs.n + 7) / 8;
      const unsigned long long o = atomicAdd(&a.ctl[2], (unsigned long long)need);
      if (o + need > a.spill_cap) {
        atomicOr(&a.ctl[3], (unsigned long long)ERR_SPILL);
        valid = false;
      } else {
        WordSink ws(a.spill + o);
        uint32_t cls2 = 0;
        encode_version_gm<GM>(pi.cmp, ver, vlen, ws, cls2);
        ws.flush();
        koff = uint32_t(o);
        kinfo |= KI_SPILL;
      }
    }
    kinfo |= (cs.n & KI_LEN) | (valid ? KI_VALID : 0u) | ((cls & KI_CLS_MASK) << KI_CLS_SHIFT);
    if (valid) be_head((kinfo & KI_SPILL) ? a.spill + koff : slot, cs.n);
  }
  // parse-first drivers (debian.go:66-70) skip an unparsable package before the lookup
  if (AB != 3 && (valid || (pi.flags & PLAT_LOOKUP_FIRST))) {
    uint64_t nw[kSlotNameWords];
    const uint64_t h = hash_pack(d.x, name, nlen, nw);
    for (uint64_t i = h & a.db.slot_mask;; i = (i + 1) & a.db.slot_mask) {
      // the whole 64-B slot in one round trip: hash, rows, inline name
      const uint4* sp = reinterpret_cast<const uint4*>(a.db.slots + i);
      const uint4 q0 = sp[0], q1 = sp[1], q2 = sp[2], q3 = sp[3];
      const uint64_t sh = q0.x | (uint64_t(q0.y) << 32);
      if (sh == 0) break;
      if (sh != h) continue;
      if ((q1.x & SLOT_LEN_MASK) != nlen || !name_eq_slot(nw, q1, q2, q3, name, a.db.name_arena, nlen)) continue;
      if (q1.x & SLOT_POISONED) {
        atomicMax(&a.ctl[1], (unsigned long long)(a.n - p));
      } else if (valid) {
        cnt = q0.w;
        rbeg = q0.z;
      }
      break;
    }
  }
}

// AB (ablation, diagnostics only): 0 = full kernel, 1 = stage+probe+encode+scan only,
// 2 = no key compare, 3 = stage+encode+scan (no probe), 4 = stage+probe+scan (no encode).  Ablation variants produce wrong match lists by construction.
template <int T, int KW, int MB, bool KG, uint32_t GM, int AB = 0>
__global__ __launch_bounds__(T) void match_kernel(MatchArgs a) {
  constexpr bool FILT = GM != GM_DEB;
  __shared__ TileShared<T, KW, MB, KG, FILT> s;
  constexpr uint32_t kStageBytes = MB * 8;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) {
    s.tile = blockIdx.x;  // segments are placed through the tile directory: any order works
    s.span_lo = 0xFFFFFFFFu;
    s.span_hi = 0;
    if (blockIdx.x == 0) a.ctl[5] = T;
  }
  __syncthreads();
  const uint32_t tile = s.tile;
  const uint32_t p = tile * T + tid;

  // ---- 0. stage the tile's name/version bytes in LDS (coalesced 16-byte loads) ---------
  uint4 d = make_uint4(0xFFFFFFFFu, 0, 0, 0);
  if (p < a.n) d = a.desc[p];
  {
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    if (p < a.n) {
      lo = d.y < d.z ? d.y : d.z;
      const uint32_t e1 = d.y + (d.w & 0xFFFFu), e2 = d.z + (d.w >> 16);
      hi = e1 > e2 ? e1 : e2;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
      lo = l2 < lo ? l2 : lo;
      hi = h2 > hi ? h2 : hi;
    }
    if ((tid & 63) == 0) {
      atomicMin(&s.span_lo, lo);
      atomicMax(&s.span_hi, hi);
    }
  }
  __syncthreads();
  const uint32_t base16 = s.span_lo & ~15u;
  const bool staged = s.span_hi > base16 && s.span_hi - base16 <= kStageBytes;
  if (staged) {
    const uint32_t nv = (s.span_hi - base16 + 15) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(a.arena + base16);
    for (uint32_t i = tid; i < nv; i += T) s.stage[i] = src[i];
  }
  __syncthreads();
  // Rebase offsets as integers: an LDS pointer minus a large arena offset would wrap the
  // 32-bit LDS address before its conversion to a flat pointer.
  const uint8_t* stage_bytes = reinterpret_cast<const uint8_t*>(s.stage);

  // ---- 1. probe + encode -------------------------------------------------------------
  uint32_t cnt = 0, rbeg = 0, kinfo = 0, koff = 0;
  if (p < a.n && d.x < a.db.n_plats) {
    if (staged)
      probe_encode<T, KW, MB, KG, FILT, GM, AB>(a, s, tid, p, d, stage_bytes + (d.y - base16), stage_bytes + (d.z - base16),
                                          cnt, rbeg, kinfo, koff);
    else
      probe_encode<T, KW, MB, KG, FILT, GM, AB>(a, s, tid, p, d, a.arena + d.y, a.arena + d.z, cnt, rbeg, kinfo, koff);
  }
  s.rbeg[tid] = rbeg;
  s.kinfo[tid] = kinfo;
  s.koff[tid] = koff;
  if constexpr (FILT) s.pattr[tid] = (a.attr && p < a.n) ? a.attr[p] : make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu);

  // ---- 2. scan of row counts ------------------------------------------------------------
  const uint32_t total_pairs = block_scan<T>(s, cnt, tid);

  // ---- 3+4. pair sweep with LDS compaction -----------------------------------------------
  const uint32_t nm = (AB == 1 || AB >= 3) ? (total_pairs & 1u) : sweep<T, KW, MB, KG, FILT, false, AB>(a, s, total_pairs, tid, 0);

  // ---- reserve the tile's output segment (one atomic per tile, no inter-tile waiting) -----
  if (tid == 0) {
    const unsigned long long base = nm ? atomicAdd(&a.ctl[0], (unsigned long long)nm) : 0ull;
    TileDir e;
    e.base = base;
    e.count = nm;
    e.pad = 0;
    a.dir[tile] = e;
    s.base = base;
  }
  __syncthreads();
  const unsigned long long base = s.base;

  // ---- 5. store the tile's matches -------------------------------------------------------
  if (nm <= uint32_t(MB)) {
    for (uint32_t i = tid; i < nm; i += T)
      if (base + i < a.out_cap) a.out[base + i] = s.mbuf[i];
  } else {
    sweep<T, KW, MB, KG, FILT, true, AB>(a, s, total_pairs, tid, base);  // rare: more matches than the LDS buffer
  }
}

template <int T, int KW, int MB, bool KG, uint32_t GM, int AB>
void launch_one(uint32_t n_tiles, hipStream_t st, const MatchArgs& a) {
  hipLaunchKernelGGL((match_kernel<T, KW, MB, KG, GM, AB>), dim3(n_tiles), dim3(T), 0, st, a);
}

}  // namespace
}  // namespace tvm
