// The match path on gfx950 (CDNA4): two kernels per batch (or per pipeline chunk).
//
// Replaces the per-package loops of the reference drivers (e.g.
// pkg/detector/ospkg/debian/debian.go:65-117, ubuntu/ubuntu.go:86-126,
// library/driver.go:111-137) with two launches over a whole batch of packages from many
// targets.  Both kernels tile the batch into T = 256 consecutive packages per workgroup.
//
//   probe_kernel  (lane per package; no barrier after the staging step)
//     0. the tile's packages are {plat, name_len | ver_len << 16} with their name and
//        version bytes back to back in the arena from tile_off[t]: a block scan of the
//        lengths gives every lane its string offsets, and the tile's byte window is staged
//        into LDS with coalesced 16-byte loads;
//     1. the installed version is encoded into its sort key (verkey.h / libver.h: the same
//        code the flattener ran over the advisory bounds at load time); the first 16 key
//        bytes stay in registers (big-endian, ready for two u64 compares), bytes 16..31 go
//        to a per-package tail slot, longer keys to the spill area;
//     2. the name is read as words (aligned LDS dwords + v_alignbyte), hashed word by word
//        and probed in the open-addressing index (one 64-B slot = hash, rows, first 40 name
//        bytes), so a probe is one memory round trip;
//     3. out: per package {k0, k1} and {row_begin, row_count, key info, spill offset}.
//   sweep_kernel
//     0. the tile's package records are read (coalesced) into LDS; a block scan of the
//        row counts over the packages that have rows (ballot-compacted) spans the tile's
//        (package, row) pair space, and a byte map pair -> package is filled in LDS;
//     1. rounds of K x 256 pairs: pair j = b0 + k * 256 + lane, so a wave's lanes read
//        consecutive 32-B rows (coalesced) and every lane has K row loads in flight before
//        it tests any;
//     2. per pair one interval test (two u64 compares on the inline 16-byte bound head,
//        the key tails only on a 16-byte tie); compaction in pair order by one wave ballot
//        per sub-round and one barrier per round, into an LDS buffer;
//     3. one atomic reservation per tile places its segment; the tile directory (base,
//        count) gives the global (package, advisory) order without inter-tile waiting.
//   The two kernels of consecutive chunks of a pass run on two streams (engine.hip), so one
//   chunk's probe overlaps the previous chunk's sweep on the same CUs: both are latency-bound.
//
// All arithmetic is integer/byte work bound by memory traffic and latency: no MFMA.
// Templates are instantiated per grammar set (libver.h GM_*) in kern_*.hip.
#pragma once
#include "engine.h"
#include "libver.h"
#include "match_variants.h"

namespace tvm {

constexpr uint32_t kStage = 12288;  // LDS bytes for a tile's strings (larger windows read global memory)
constexpr uint32_t kKeyWords = 4;   // key bytes kept per package (head 16 in registers, tail 16 in a slot)
constexpr uint32_t kMapCap = 4096;  // LDS byte map pair -> package: one entry per pair up to this many pairs,
                                    // one per 2^shift pairs above (map_shift, map_rank)

struct ProbeArgs {
  DevDB db;
  const uint2* pk;           // chunk-relative: {plat, name_len | ver_len << 16}
  const uint64_t* tile_off;  // chunk-relative: arena offset of each 64-package group (+1)
  const uint8_t* arena;
  uint32_t n;                // packages in this launch
  uint32_t p0;               // batch index of the launch's first package
  uint32_t n_total;          // packages in the whole batch (poisoned-package encoding)
  PkgRec* rec;               // chunk-relative
  uint4* tail;               // chunk-relative
  unsigned long long* ctl;   // [1] n_total - first poisoned, [2] spill words used, [3] error bits
  uint64_t* spill;
  uint64_t spill_cap;
};

struct SweepArgs {
  DevDB db;
  const PkgRec* rec;         // chunk-relative
  const uint4* tail;
  const uint64_t* spill;
  const uint8_t* arena;      // the batch's name/version bytes (Maven rows re-read the installed text)
  const uint2* attr;         // per-package attributes (chunk-relative), nullptr when no row filters
  const uint32_t* cpe_bits;
  uint32_t cpe_words;
  uint32_t n_cpe_sets;
  uint32_t n;
  uint32_t p0;
  uint32_t out_base;         // added to every output package index (a shard's first global package)
  uint32_t n_tiles;          // tiles in this launch
  uint32_t t0;               // batch index of the launch's first tile
  TileDir* dir;              // batch-indexed tile directory (tile t0 + i)
  uint32_t* out_pkg;
  uint32_t* out_adv;
  uint64_t out_cap;
  unsigned long long* ctl;   // [0] total matches (reservation counter)
};

struct FusedArgs {
  ProbeArgs pa;
  SweepArgs sa;
  CopyOutArgs co;       // end-to-end pipeline: the previous chunk's result move ...
  uint32_t n_copy = 0;  // ... by workgroups [0, n_copy) of this launch (0: none)
  const uint32_t* tile_map = nullptr;  // workgroup -> tile (DevBatch::tile_map; no result move)
  unsigned long long* ctl_zero = nullptr;  // device-resident pass: the control block to zero for the next
};

using ProbeFn = void (*)(uint32_t n_tiles, hipStream_t st, const ProbeArgs& a);
using SweepFn = void (*)(uint32_t n_tiles, hipStream_t st, const SweepArgs& a);
using FusedFn = void (*)(uint32_t n_tiles, hipStream_t st, const FusedArgs& a);

namespace {

// KI_MVN: a Maven package whose key has program rows (the sweep defers those pairs)
// KI_H24: a dpkg-grammar package (its rows carry 24-byte key heads, Row::hi_pre2)
enum : uint32_t { KI_VALID = 1u << 31, KI_SPILL = 1u << 30, KI_MVN = 1u << 29, KI_H24 = 1u << 25, KI_LEN = 0x3FFFu,
                  KI_CLS_SHIFT = 26, KI_CLS_MASK = 7u };

// Block-wide exclusive scan of v over T lanes (wave shuffles + one LDS exchange); returns
// the block total.  `wsum` holds T/64 words; two barriers.
template <int T>
__device__ __forceinline__ uint32_t block_exscan(uint32_t* wsum, uint32_t v, uint32_t tid, uint32_t& excl) {
  constexpr int W = T / 64;
  const uint32_t lane = tid & 63, wave = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= uint32_t(d)) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const uint32_t t = wsum[w];
    off += (uint32_t(w) < wave) ? t : 0;
    tot += t;
  }
  excl = off + x - v;
  __syncthreads();
  return tot;
}

// ---- probe_kernel helpers ---------------------------------------------------------------

// Sort-key sink: key bytes 0..15 accumulate in two registers, bytes 16..31 go to the
// package's tail slot; every byte is counted, so one pass both encodes a typical key and
// sizes a long one (which is then re-encoded into the spill area).
struct HeadSink {
  uint64_t* tail;
  uint64_t acc = 0, w0 = 0, w1 = 0, w2 = 0;
  uint32_t n = 0;
  __device__ explicit HeadSink(uint64_t* t) : tail(t) {}
  __device__ __forceinline__ void word(uint32_t w) {
    if (w == 0) w0 = acc;
    else if (w == 1) w1 = acc;
    else if (w < kKeyWords) tail[w - 2] = acc;
    if (w == 2) w2 = acc;
  }
  __device__ __forceinline__ void put(uint8_t b) {
    acc |= uint64_t(b) << (8 * (n & 7));
    if ((n & 7) == 7) {
      word(n >> 3);
      acc = 0;
    }
    n++;
  }
  __device__ __forceinline__ void flush() {
    if (n & 7) word(n >> 3);
  }
};

__device__ __forceinline__ uint64_t be_word(uint64_t w, uint32_t bytes) {  // bytes in [1, 8]
  if (bytes < 8) w &= (1ull << (8 * bytes)) - 1ull;
  return __builtin_bswap64(w);
}

// Name bytes -> words.  `s` may sit at any byte offset; the bytes are read as aligned
// dwords and funnel-shifted (v_alignbyte), so an 8-byte word costs three dword loads
// instead of eight byte loads.  Word i is zero past the name's end.
template <class P>
__device__ __forceinline__ uint64_t name_word(const P* base, uint32_t sh, uint32_t i, uint32_t n) {
  const uint32_t d0 = base[2 * i], d1 = base[2 * i + 1], d2 = base[2 * i + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh), hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
  uint64_t w = uint64_t(lo) | (uint64_t(hi) << 32);
  const uint32_t left = n - 8 * i;  // > 0
  if (left < 8) w &= (1ull << (8 * left)) - 1ull;
  return w;
}

// Hash of (plat, name) from the name's bytes, word by word.
template <class P>
__device__ __forceinline__ uint64_t name_hash(uint32_t plat, const uint8_t* s, uint32_t n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(s);
  const P* base = reinterpret_cast<const P*>(a & ~uintptr_t(3));
  const uint32_t sh = uint32_t(a & 3);
  uint64_t h = key_hash_seed2(plat, n);
  for (uint32_t i = 0; 8 * i < n; i++) h = key_hash_word(h, name_word(base, sh, i, n));
  return key_hash_fin(h);
}

// Name check against a slot (first 40 bytes inline, loaded with the hash; the name's words
// are re-read, which is cheaper than keeping five words live across the probe); longer
// names finish bytewise against the name arena.
template <class P>
__device__ __forceinline__ bool name_eq_slot(const uint8_t* s, uint32_t n, const uint4 q1, const uint4 q2,
                                             const uint4 q3, const uint8_t* arena) {
  static_assert(kSlotNameWords == 5, "five inline name words");
  const uintptr_t a = reinterpret_cast<uintptr_t>(s);
  const P* base = reinterpret_cast<const P*>(a & ~uintptr_t(3));
  const uint32_t sh = uint32_t(a & 3);
  const uint64_t y[kSlotNameWords] = {q1.z | (uint64_t(q1.w) << 32), q2.x | (uint64_t(q2.y) << 32),
                                      q2.z | (uint64_t(q2.w) << 32), q3.x | (uint64_t(q3.y) << 32),
                                      q3.z | (uint64_t(q3.w) << 32)};
  bool eq = true;
#pragma unroll
  for (uint32_t i = 0; i < kSlotNameWords; i++) eq &= (8 * i < n ? name_word(base, sh, i, n) : 0ull) == y[i];
  if (eq && n > 8 * kSlotNameWords) {
    const uint8_t* full = arena + q1.y;
    for (uint32_t i = 8 * kSlotNameWords; eq && i < n; i++) eq = full[i] == s[i];
  }
  return eq;
}

// Index probe of one package given its key state (shared by the fast and generic paths).
// h: the name's hash; start / found: the first slot of its chain whose fingerprint is the
// name's (fp_chain), if any; q0 / q0n: the first 16 bytes of that slot and (has_q0n) of the
// slot after it, loaded early so the round trips overlap the encoder.
template <class P>
__device__ __forceinline__ void probe_lookup(const ProbeArgs& a, uint32_t p, uint32_t plat, const PlatInfo& pi,
                                            uint32_t nlen, const uint8_t* name, bool valid, uint64_t h,
                                            uint64_t start, bool found, uint4 q0, uint4 q0n, bool has_q0n,
                                            uint32_t& rbeg, uint32_t& cnt, uint32_t* sflags = nullptr,
                                            uint32_t cls = 0);

__device__ __forceinline__ uint4 slot_head(const ProbeArgs& a, uint64_t i) {
  return reinterpret_cast<const uint4*>(a.db.slots + (i & a.db.slot_mask))[0];
}

// The first slot of h's linear-probing chain whose fingerprint is h's (DB::slot_fp), or false
// at the chain's end: slots with another fingerprint cannot hold the name, so they are passed
// over without reading their 64 B, and an absent name (a quarter of the synthetic batches)
// reads one byte from an L2-resident array instead of a 128-B line.
__device__ __forceinline__ bool fp_chain(const ProbeArgs& a, uint64_t h, uint64_t& i) {
  i = h & a.db.slot_mask;
#ifdef TVM_EXP_NOFP  // measurement only (make exp): no fingerprint walk, every chain from its home slot
  return true;
#else
  const uint8_t want = slot_fp_of(h);
  for (;;) {
    const uint8_t f = a.db.slot_fp[i];
    if (f == 0) return false;
    if (f == want) return true;
    i = (i + 1) & a.db.slot_mask;
  }
#endif
}

// One package: encode, hash, probe.  P = uint32_t in the LDS or global address space of s.
// kb / tab: the lane's LDS key buffer and the dpkg code table (nullptr: generic encoder only).
template <uint32_t GM, class P, int DIAG = 0>
__device__ __forceinline__ void probe_one(const ProbeArgs& a, uint32_t p, uint32_t plat, uint32_t nlen, uint32_t vlen,
                                          const uint8_t* name, const uint8_t* ver, uint64_t vglob, PkgRec& r,
                                          uint8_t* kb = nullptr, const uint8_t* tab = nullptr) {
  const PlatInfo pi = a.db.plats[plat];
  // the hash and the fingerprint walk come before the encoder; the dpkg-only kernels load the
  // slot heads before it too, the other grammar sets after it (their encoders' registers: held
  // across them, the heads made the all-grammar kernel spill)
  constexpr bool kPre = GM == GM_DEB;
  uint64_t h = 0, start = 0;
  bool found = false;
  uint4 q0 = make_uint4(0, 0, 0, 0), q0n = q0;
  bool has_q0n = false;
  if (!(DIAG & 2)) {
    h = name_hash<P>(plat, name, nlen);
    found = fp_chain(a, h, start);
  }
  auto heads = [&]() {
    if ((DIAG & 2) || !found) return;
    q0 = slot_head(a, start);
    // the next slot's head too, but only from the same 128-B line (an even slot index: every
    // L2 miss is a 128-B request, so it costs no request of its own); at slot load <= 1/8 a
    // second slot is rarely probed, and fetching the next line for the odd slots cost C2 a
    // random request per second package (0.393 -> 0.386 ms, profiles/r06/q0n)
    if constexpr (kPre) {
      has_q0n = !(start & 1);
      if (has_q0n) q0n = slot_head(a, start + 1);
    }
  };
  if constexpr (kPre) heads();
  if (!(DIAG & 1) && kb && ((GM >> CMP_DEB) & 1u) && pi.cmp == CMP_DEB) {
    uint32_t kl = 0;
    const uint32_t st = deb_fast_key(ver, vlen, kb, tab, kl);
    if (st != FAST_FALLBACK) {
      const bool valid = st == FAST_OK;
      const uint32_t* kw = reinterpret_cast<const uint32_t*>(kb);
      uint32_t kinfo = (valid ? (kl & KI_LEN) | KI_VALID : 0u) | KI_H24, koff = 0;
      r.k0 = r.k1 = r.k2 = 0;
      if (valid) {
        const uint64_t m0 = uint64_t(kw[0]) | (uint64_t(kw[1]) << 32), m1 = uint64_t(kw[2]) | (uint64_t(kw[3]) << 32);
        r.k0 = be_word(m0, kl < 8 ? kl : 8);
        r.k1 = kl > 8 ? be_word(m1, kl < 16 ? kl - 8 : 8) : 0ull;
        r.k2 = kl > 16 ? be_word(uint64_t(kw[4]) | (uint64_t(kw[5]) << 32), kl < 24 ? kl - 16 : 8) : 0ull;
        static_assert(kFastKeyCap <= kKeyWords * 8, "fast keys fit head + tail slot");
        // dpkg-only kernels compare 24-byte heads (bytes 16..23 in r.k2), so their tail slot is
        // read only past a 24-byte tie (bytes 24..31) or by a lower bound, which takes bytes
        // 16..23 from k2 (eval_row): a key of 17..24 bytes writes nothing (C2: ~49 MB of tail
        // stores per pass).  Other grammar sets keep it: their split-form sweeps compare 16.
        if (kl > (GM == GM_DEB ? 24u : 16u)) a.tail[p] = make_uint4(kw[4], kw[5], kw[6], kw[7]);
      }
      uint32_t cnt = 0, rbeg = 0;
      if constexpr (!kPre) heads();
      if (!(DIAG & 2)) probe_lookup<P>(a, p, plat, pi, nlen, name, (kinfo & KI_VALID) != 0, h, start, found, q0, q0n, has_q0n,
                                          rbeg, cnt);
      r.meta = make_uint4(rbeg, cnt, kinfo, koff);
      return;
    }
  }
  uint64_t* tslot = reinterpret_cast<uint64_t*>(a.tail + p);
  HeadSink hs(tslot);
  uint32_t cls = 0;
  bool valid = true;
  if (DIAG & 1) {
    hs.n = vlen;
    hs.w0 = vlen;
  } else {
    valid = encode_version_gm<GM>(pi.cmp, ver, vlen, hs, cls);
  }
  hs.flush();
  uint32_t kinfo = 0, koff = 0;
  // long key: the whole key again into the spill area.  A Maven package's tail slot holds its
  // program state (below), so its keys spill from 17 bytes on (Engine::scratch_words)
  const bool mvn_pkg = ((GM >> CMP_MAVEN) & 1u) && pi.cmp == CMP_MAVEN;
  if (valid && hs.n > (mvn_pkg ? 16u : kKeyWords * 8)) {
    const uint32_t need = (hs.n + 7) / 8;
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
  uint32_t cnt = 0, rbeg = 0, sflags = 0;
  if constexpr (!kPre) heads();
  if (!(DIAG & 2)) probe_lookup<P>(a, p, plat, pi, nlen, name, valid, h, start, found, q0, q0n, has_q0n, rbeg, cnt,
                                   &sflags, cls);
  if (((GM >> CMP_MAVEN) & 1u) && pi.cmp == CMP_MAVEN) {
    // Maven rows compare parses, not keys (AUX_MVN): the installed version's parse, packed
    // into the batch scratch, and its text location take the tail slot - only when the key
    // has a program row that admits the version's class (SLOT_MVN_C0 / C1: most numeric
    // versions meet hybrid advisories only, whose program rows reject them by class)
    uint32_t off = 0, nt = 0;
    if (valid && (sflags & (cls == 1 ? SLOT_MVN_C1 : SLOT_MVN_C0))) {
      MvnParse mp;
      if (mvn_parse(ver, vlen, mp)) {
        const uint32_t need = (kMvnPackedWords * mp.n + 1) / 2;
        const unsigned long long o = atomicAdd(&a.ctl[2], (unsigned long long)need);
        if (o + need > a.spill_cap) {  // the pass fails (ERR_SPILL); the package keeps no rows
          atomicOr(&a.ctl[3], (unsigned long long)ERR_SPILL);
          valid = false;
          cnt = rbeg = 0;
        } else {
          mvn_pack(mp, ver, reinterpret_cast<uint32_t*>(a.spill + o));
          off = uint32_t(o);
          nt = uint32_t(mp.n);
        }
      }
    }
    a.tail[p] = make_uint4(off, nt | (vlen << 16), uint32_t(vglob), uint32_t(vglob >> 32));
  }
  const uint32_t kl = hs.n;
  kinfo |= (kl & KI_LEN) | (valid ? KI_VALID : 0u) | ((cls & KI_CLS_MASK) << KI_CLS_SHIFT);
  if (pi.cmp == CMP_DEB) kinfo |= KI_H24;
  // only a key with program rows can defer a pair (numeric-bound advisories are intervals)
  if (((GM >> CMP_MAVEN) & 1u) && pi.cmp == CMP_MAVEN && (sflags & (SLOT_MVN_C0 | SLOT_MVN_C1))) kinfo |= KI_MVN;
  r.k0 = valid && kl ? be_word(hs.w0, kl < 8 ? kl : 8) : 0ull;
  r.k1 = valid && kl > 8 ? be_word(hs.w1, kl < 16 ? kl - 8 : 8) : 0ull;
  r.k2 = valid && kl > 16 ? be_word(hs.w2, kl < 24 ? kl - 16 : 8) : 0ull;
  r.meta = make_uint4(rbeg, cnt, kinfo, koff);
}

template <class P>
__device__ __forceinline__ void probe_lookup(const ProbeArgs& a, uint32_t p, uint32_t plat, const PlatInfo& pi,
                                            uint32_t nlen, const uint8_t* name, bool valid, uint64_t h,
                                            uint64_t start, bool found, uint4 q0, uint4 q0n, bool has_q0n,
                                            uint32_t& rbeg, uint32_t& cnt, uint32_t* sflags, uint32_t cls) {
  // parse-first drivers (debian.go:66-70) skip an unparsable package before the lookup;
  // lookup-first drivers (ubuntu.go:86-92) probe first, so a poisoned key still raises
  if (found && (valid || (pi.flags & PLAT_LOOKUP_FIRST))) {
    uint32_t step = 0;
    for (uint64_t i = start;; i = (i + 1) & a.db.slot_mask, step++) {
      const uint4* sp = reinterpret_cast<const uint4*>(a.db.slots + i);
      if (step == 1 && has_q0n) q0 = q0n;
      else if (step > 0) q0 = sp[0];
      const uint4 q1 = sp[1], q2 = sp[2], q3 = sp[3];  // the rest of the 64-B slot
      const uint64_t sh = q0.x | (uint64_t(q0.y) << 32);
      if (sh == 0) break;
      if (sh != h) continue;
      if ((q1.x & SLOT_LEN_MASK) != nlen || !name_eq_slot<P>(name, nlen, q1, q2, q3, a.db.name_arena)) continue;
      if (q1.x & SLOT_POISONED) {
        atomicMax(&a.ctl[1], (unsigned long long)(a.n_total - (a.p0 + p)));
      } else if (valid) {
        const uint2 rr = slot_rows(q1.x, q0.z, q0.w, cls);  // a split key: the list of the version's class
        rbeg = rr.x;
        cnt = rr.y;
        if (sflags) *sflags = q1.x & (SLOT_MVN_C0 | SLOT_MVN_C1);
      }
      break;
    }
  }
}

// A tile's string window (nv 16-byte words, nv <= kStage / 16) into LDS, plus two zero
// words: every lane issues its (at most kStage / 16 / kTile) loads before storing any.
template <uint32_t STG = kStage>
__device__ __forceinline__ void stage_window(uint4* buf, const uint8_t* src8, uint32_t nv, uint32_t tid) {
  constexpr uint32_t SV = (STG / 16 + kTile - 1) / kTile;
  const uint4* src = reinterpret_cast<const uint4*>(src8);
  if (nv) {
    uint4 v[SV];
#pragma unroll
    for (uint32_t k = 0; k < SV; k++) v[k] = src[min(tid + k * kTile, nv - 1)];
#pragma unroll
    for (uint32_t k = 0; k < SV; k++)
      if (tid + k * kTile < nv) buf[tid + k * kTile] = v[k];
  }
  if (tid < 2) buf[nv + tid] = make_uint4(0, 0, 0, 0);
}

// Per-wave staging (fused_kernel SEG bit 1): wave w stages its own 64-package group's window
// (tile_off[g] .. tile_off[g + 1], at most kStage / 4 bytes) into its quarter of the buffer,
// with a wave scan of the lengths - no workgroup barrier before the probe.
__device__ __forceinline__ uint32_t wave_exscan(uint32_t v, uint32_t lane) {
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= uint32_t(d)) x += y;
  }
  return x - v;
}

template <uint32_t STG = kStage>
__device__ __forceinline__ void stage_window_wave(uint4* buf, const uint8_t* src8, uint32_t nv, uint32_t lane) {
  constexpr uint32_t SV = (STG / 4 / 16 + 63) / 64;
  const uint4* src = reinterpret_cast<const uint4*>(src8);
  if (nv) {
    uint4 v[SV];
#pragma unroll
    for (uint32_t k = 0; k < SV; k++) v[k] = src[min(lane + k * 64, nv - 1)];
#pragma unroll
    for (uint32_t k = 0; k < SV; k++)
      if (lane + k * 64 < nv) buf[lane + k * 64] = v[k];
  }
  if (lane < 2) buf[nv + lane] = make_uint4(0, 0, 0, 0);
}

template <uint32_t GM, int DIAG = 0>
__global__ __launch_bounds__(kTile) void probe_kernel(ProbeArgs a) {
  __shared__ uint4 stage[kStage / 16 + 2];  // +2: the dword reads of a name's last word run past its end
  __shared__ uint32_t wsum[kTile / 64];
  __shared__ uint32_t kbuf[kTile * kFastKeyStride / 4];  // per-lane dpkg key (deb_fast_key)
  __shared__ uint8_t tab[128];
  const uint32_t tid = threadIdx.x, t = blockIdx.x;
  if (tid < 128) tab[tid] = deb_fast_code(tid);
  const uint32_t p = t * kTile + tid;
  uint2 d = make_uint2(0xFFFFFFFFu, 0);
  if (p < a.n) d = a.pk[p];
  const uint64_t w0 = a.tile_off[t * kGroupsPerTile], w1 = a.tile_off[(t + 1) * kGroupsPerTile];
  const uint32_t nlen = d.y & 0xFFFFu, vlen = d.y >> 16;
  uint32_t off = 0;
  block_exscan<kTile>(wsum, nlen + vlen, tid, off);
  const uint64_t base16 = w0 & ~uint64_t(15);
  const bool staged = w1 - base16 <= kStage;
  if (staged) stage_window(stage, a.arena + base16, uint32_t((w1 - base16 + 15) / 16), tid);
  __syncthreads();
  PkgRec r;
  r.meta = make_uint4(0, 0, 0, 0);
  r.k0 = r.k1 = r.k2 = 0;
  if (p < a.n && d.x < a.db.n_plats) {
    if (staged) {
      const uint8_t* sb = reinterpret_cast<const uint8_t*>(stage) + uint32_t(w0 - base16) + off;
      probe_one<GM, uint32_t, DIAG>(a, p, d.x, nlen, vlen, sb, sb + nlen, w0 + off + nlen, r,
                                    reinterpret_cast<uint8_t*>(kbuf) + tid * kFastKeyStride, tab);
    } else {
      const uint8_t* gb = a.arena + w0 + off;
      probe_one<GM, uint32_t, DIAG>(a, p, d.x, nlen, vlen, gb, gb + nlen, w0 + off + nlen, r);
    }
  }
  if (p < a.n) a.rec[p] = r;
}

// ---- sweep_kernel helpers ---------------------------------------------------------------

template <int FILT>
struct SweepShared {
  uint64_t k0[kTile], k1[kTile], k2[FILT < 2 ? kTile : 1];  // key heads by tile package
  uint32_t kinfo[kTile];
  uint32_t koff[kTile];           // spill word offset of a long key (KI_SPILL)
  uint2 pattr[FILT ? kTile : 1];
  uint32_t nz_scan[kTile + 1];    // pair offset of the r-th package that has rows (+ total)
  uint32_t nz_rd[kTile];          // its row_begin - pair offset
  uint32_t nz_q[kTile];           // its tile package index
  uint32_t wsum[2][kTile / 64];
  uint32_t wsum2[2][8 * (kTile / 64)];  // per round: K sub-rounds x wave match counts
  uint32_t tile;
  unsigned long long base;
};

// log2 of the pairs per map entry: 0 up to kMapCap pairs (an entry per pair), else the
// smallest power of two that fits the tile's pairs into kMapCap entries.
__device__ __forceinline__ uint32_t map_shift(uint32_t total) {
  uint32_t sh = 0;
  while ((total + (1u << sh) - 1) >> sh > kMapCap) sh++;
  return sh;
}

// Per-package predicates of a ROW_FILTER row (common.h RowAux); p = the package's index
// in the launch (its tail slot holds a Maven package's text location, probe_one).
// FILT (the sweep's template flag): 0 no row filters, 1 filters without Maven programs (the OS
// grammar set, whose rows never carry AUX_MVN: keeps the program evaluator's registers out of
// that kernel), 2 all filters.
// DEFER: a Maven program is not run here but reported (2) for the round's compacted
// evaluation (sweep_programs); else 0 / 1 = the predicates fail / hold.
template <int FILT>
__device__ __forceinline__ bool mvn_pair(const SweepArgs& a, const uint32_t* ids, uint32_t p) {
  // the installed parse packed by probe_one, the program's packed bounds
  const uint4 t = a.tail[p];
  const MvnPackedView V{reinterpret_cast<const uint32_t*>(a.spill + t.x), int(t.y & 0xFFFFu),
                        a.arena + (uint64_t(t.z) | (uint64_t(t.w) << 32))};
  return mvn_program_eval(ids, V);
}

// The predicates an rpm row carries inline (common.h ROW_INLINE): no load but the package's
// CPE-set word.
__device__ __forceinline__ uint32_t inline_pass(const SweepArgs& a, const Row& row, uint2 pa) {
  const uint32_t kind = row.lo_len & 15u, na = (row.lo_len >> 4) & 3u, nc = (row.lo_len >> 6) & 3u;
  if (kind & AUX_TAG) return row.off.lo_off == pa.y ? 1u : 0u;
  const uint32_t w[2] = {row.off.lo_off, row.off.hi_off};
  auto id = [&](uint32_t i) { return (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu; };
  if (kind & (AUX_ARCH_RH | AUX_ARCH_IN)) {
    bool ok = (kind & AUX_ARCH_RH) && (na == 0 || (pa.x & PA_NOARCH));
    const uint32_t arch = pa.x & PA_ARCH_MASK;
    for (uint32_t i = 0; i < na; i++) ok |= id(i) == arch;
    if (!ok) return 0;
  }
  if (kind & AUX_CPE) {
    if (pa.y >= a.n_cpe_sets) return 0;
    const uint32_t* set = a.cpe_bits + size_t(pa.y) * a.cpe_words;
    bool ok = false;
    for (uint32_t i = 0; i < nc; i++) {
      const uint32_t c = id(na + i);
      ok |= (c >> 5) < a.cpe_words && ((set[c >> 5] >> (c & 31)) & 1u);
    }
    if (!ok) return 0;
  }
  return 1;
}

template <int FILT, bool DEFER = false>
__device__ __forceinline__ uint32_t aux_pass(const SweepArgs& a, uint32_t ridx, uint2 pa, uint32_t ki, uint32_t p) {
#ifdef TVM_EXP_NOAUX  // measurement only (make exp): every row filter passes - wrong lists by design
  if (FILT < 2) return 1;
#endif
  const RowAux x = a.db.aux[ridx];
  const uint32_t* ids = a.db.aux_ids + x.list_off;
  // the class first: a Maven hybrid program row is rejected for numeric versions before its
  // program would run
  if ((x.kind & AUX_CLASS) && !((x.tag >> ((ki >> KI_CLS_SHIFT) & KI_CLS_MASK)) & 1u)) return 0;
  if (FILT >= 2 && (x.kind & AUX_MVN)) {
    if constexpr (DEFER) return 2;
    return mvn_pair<FILT>(a, ids, p) ? 1u : 0u;
  }
  if (x.kind & (AUX_ARCH_RH | AUX_ARCH_IN)) {
    bool ok = (x.kind & AUX_ARCH_RH) && (x.n_arch == 0 || (pa.x & PA_NOARCH));
    const uint32_t arch = pa.x & PA_ARCH_MASK;
    for (uint32_t i = 0; i < x.n_arch && !ok; i++) ok = ids[i] == arch;
    if (!ok) return 0;
  }
  if (x.kind & AUX_CPE) {
    if (pa.y >= a.n_cpe_sets) return 0;
    const uint32_t* set = a.cpe_bits + size_t(pa.y) * a.cpe_words;
    bool ok = false;
    for (uint32_t i = 0; i < x.n_cpe && !ok; i++) {
      const uint32_t c = ids[x.n_arch + i];
      ok = (c >> 5) < a.cpe_words && ((set[c >> 5] >> (c & 31)) & 1u);
    }
    if (!ok) return 0;
  }
  if ((x.kind & AUX_TAG) && x.tag != pa.y) return 0;
  return 1;
}

// sign(installed key - bound) on the big-endian heads; the tails (memory-order words from
// byte 16 on) only on a 16-byte tie with both keys longer.
__device__ __forceinline__ int cmp_be(uint64_t a0, uint64_t a1, const uint64_t* atail, uint32_t na, uint64_t b0,
                                      uint64_t b1, const uint64_t* btail, uint32_t nb) {
  if (a0 != b0) return a0 < b0 ? -1 : 1;
  if (a1 != b1) return a1 < b1 ? -1 : 1;
  if (na <= 16 || nb <= 16) return (na > nb) - (na < nb);
  return key_cmp(atail, na - 16, btail, nb - 16);
}

// sign(installed - bound) from the big-endian heads alone (hl = 16 or 24 bytes; a 16-byte head
// passes a2 = b2 = 0), branch-free: valid unless both heads tie and both keys are longer than
// the head (`tie`: the key tails).
__device__ __forceinline__ int cmp_head(uint64_t a0, uint64_t a1, uint64_t a2, uint32_t na, uint64_t b0, uint64_t b1,
                                        uint64_t b2, uint32_t nb, uint32_t hl, bool& tie) {
  const bool eq0 = a0 == b0, eq1 = eq0 && a1 == b1, eq = eq1 && a2 == b2;
  const bool lt = a0 < b0 || (eq0 && a1 < b1) || (eq1 && a2 < b2);
  tie = eq && na > hl && nb > hl;
  const int byl = (na > nb) - (na < nb);
  return eq ? byl : (lt ? -1 : 1);
}

// Interval test of tile package q's installed key against one row (global index ridx).
// The common case (a bound decided by the inline 24-byte heads) runs without branches;
// a 24-byte tie reads the key tails, a lower bound (library / rpm ranges) its key head.
// dpkg-grammar packages (FILT 0 kernels: all of them; else KI_H24) compare 24-byte heads and
// find their rows' offsets in DB::row_off on the rare path that needs them; the other
// grammars 16-byte heads with the offsets inline.
template <int FILT, bool DEFER = false, class S>
__device__ __forceinline__ uint32_t eval_row(const SweepArgs& a, const S& s, uint32_t q, uint32_t p, const Row& row,
                                             uint32_t ridx) {
  const uint32_t ki = s.kinfo[q];
  const uint32_t kl = ki & KI_LEN;
  // h24: the row keeps its offsets in DB::row_off; c24: this kernel compares its 24-byte head
  // (the all-grammar kernel, at its register cap, compares 16 bytes for every grammar)
  const bool h24 = FILT == 0 || (ki & KI_H24), c24 = FILT < 2 && h24;
  const uint64_t k0 = s.k0[q], k1 = s.k1[q], k2 = c24 ? s.k2[q] : 0ull;
  const uint32_t nh = row.hi_len & KEY_LEN_MASK, hl = c24 ? 24u : 16u;
  bool tie = false;
  int c = cmp_head(k0, k1, k2, kl, row.hi_pre0, row.hi_pre1, c24 ? row.hi_pre2 : 0ull, nh, hl, tie);
  const bool hi_inf = (row.hi_len & KEY_INF) != 0;
  if (tie && !hi_inf) {  // rare: same head, both keys longer
    const uint64_t* ktail =
        (ki & KI_SPILL) ? a.spill + s.koff[q] + 2 : reinterpret_cast<const uint64_t*>(a.tail + p);
    const uint32_t w = hl / 8;
    const uint32_t hi_off = (h24 || (row.adv & ROW_INLINE)) ? a.db.row_off[ridx].hi_off : row.off.hi_off;
    c = key_cmp(ktail + (w - 2), kl - hl, a.db.key_words + hi_off + w, nh - hl);
  }
  bool m = hi_inf || ((row.hi_len & KEY_INCL) ? c <= 0 : c < 0);
  if (!(row.lo_len & KEY_INF) && m) {  // rare (library / rpm ranges): the bound's head from the arena
    // a 24-byte-head package of at most 24 key bytes wrote no tail slot (probe_one): its bytes
    // 16..23 come from k2, back in memory order
    const uint64_t t24[2] = {__builtin_bswap64(c24 ? k2 : 0ull), 0ull};
    const uint64_t* ktail = (ki & KI_SPILL) ? a.spill + s.koff[q] + 2
                            : (c24 && kl <= 24) ? t24
                                                : reinterpret_cast<const uint64_t*>(a.tail + p);
    const uint64_t* lw = a.db.key_words + (h24 ? a.db.row_off[ridx].lo_off : row.off.lo_off);
    const uint32_t nl = row.lo_len & KEY_LEN_MASK;
    const uint64_t l0 = nl ? be_word(lw[0], nl < 8 ? nl : 8) : 0ull;
    const uint64_t l1 = nl > 8 ? be_word(lw[1], nl < 16 ? nl - 8 : 8) : 0ull;
    const int cl = cmp_be(k0, k1, ktail, kl, l0, l1, lw + 2, nl);
    m = (row.lo_len & KEY_INCL) ? cl >= 0 : cl > 0;
  }
  m = m && (ki & KI_VALID);
  m = m || (row.adv & ROW_ALWAYS);
  if constexpr (FILT) {
    if (m && (row.adv & ROW_FILTER))
      return (row.adv & ROW_INLINE) ? inline_pass(a, row, s.pattr[q]) : aux_pass<FILT, DEFER>(a, ridx, s.pattr[q], ki, p);
  }
  return m ? 1u : 0u;
}

// The Maven programs of a sweep round, run compacted (FILT >= 2, tiles with Maven packages):
// the lanes' deferred pairs (pend: bit k = sub-round k) are queued in LDS and every lane of
// the workgroup takes one, so a program occupies all 64 lanes of a wave instead of one (a
// round had its few program pairs spread over the waves, each wave waiting on its own:
// Maven-only 1M packages took 0.62 ms with 3 % non-numeric versions, 0.34 ms with none).
// Returns the lane's pass bits; q.res holds 4 bits per lane (K <= 4).
struct DeferQ {
  uint32_t* j;    // queued pair indices (cap of them; more are run in batches)
  uint32_t* res;  // kTile / 8 words
  uint32_t cap;
};

template <int K, int FILT>
__device__ __forceinline__ uint32_t sweep_programs(const SweepArgs& a, const SweepShared<FILT>& s, const uint8_t* map,
                                                   uint32_t nnz, uint32_t total, uint32_t b0, uint32_t pend,
                                                   uint32_t tid, const DeferQ& q, uint32_t* ws) {
  static_assert(K <= 4, "4 result bits per lane");
  uint32_t excl;
  const uint32_t n = block_exscan<kTile>(ws, uint32_t(__popc(pend)), tid, excl);
  if (n == 0) return 0;
  if (tid < kTile / 8) q.res[tid] = 0;
  const uint32_t shift = map_shift(total);
  const uint32_t pbase = s.tile * kTile;
  for (uint32_t q0 = 0; q0 < n; q0 += q.cap) {
    uint32_t o = excl;
#pragma unroll
    for (int k = 0; k < K; k++)
      if ((pend >> k) & 1u) {
        if (o >= q0 && o < q0 + q.cap) q.j[o - q0] = b0 + k * kTile + tid;
        o++;
      }
    __syncthreads();
    const uint32_t m = min(q.cap, n - q0);
    for (uint32_t e = tid; e < m; e += kTile) {
      const uint32_t j = q.j[e];
      const uint32_t r = map_rank(s, map, shift, j);
      const uint32_t ridx = j + s.nz_rd[r];
      if (mvn_pair<FILT>(a, a.db.aux_ids + a.db.aux[ridx].list_off, pbase + s.nz_q[r])) {
        const uint32_t owner = (j - b0) % kTile, kk = (j - b0) / kTile;
        atomicOr(&q.res[owner >> 3], 1u << ((owner & 7) * 4 + kk));
      }
    }
    __syncthreads();
  }
  return (q.res[tid >> 3] >> ((tid & 7) * 4)) & 0xFu;
}

// Tile package (nz rank) of pair j from the map: its entry, or (shift > 0) its bucket's entry
// advanced over the packages that start inside the bucket before j (a tile has at most 256
// packages over at least 4096 buckets: rarely a step).  Tiles above kMapCap pairs were a
// binary search per pair before, and they are the grid's heaviest tiles (C2: 2.6 % of the
// tiles, 6 % of the pairs).
template <int FILT>
__device__ __forceinline__ uint32_t map_rank(const SweepShared<FILT>& s, const uint8_t* map, uint32_t shift, uint32_t j) {
  if (shift == 0) return map[j];
  uint32_t r = map[j >> shift];
  while (s.nz_scan[r + 1] <= j) r++;
  return r;
}

// Tile package (nz rank) of pair j by binary search of the nz scan.
template <int FILT>
__device__ __forceinline__ uint32_t pair_rank(const SweepShared<FILT>& s, uint32_t nnz, uint32_t j) {
  uint32_t lo = 0, hi = nnz;  // last r with nz_scan[r] <= j
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s.nz_scan[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One sweep over the tile's pairs in rounds of K x T: pair j = b0 + k * T + tid, so the 64
// lanes of a wave read consecutive rows (coalesced) and every lane has K row loads in
// flight before it tests any.  Pair -> package comes from the LDS byte map (one read).
// Matches are placed in pair order - sub-round by sub-round, a wave ballot per sub-round and
// one barrier per round for the wave totals - into the LDS buffer while it has room
// (pass 1, which also counts matches per package), or straight to the output at base +
// position (DIRECT: pass 2, for a tile with more matches than the buffer).
template <int K, int MB, int FILT, bool DIRECT>
__device__ __forceinline__ uint32_t sweep(const SweepArgs& a, SweepShared<FILT>& s, uint32_t* madv, uint8_t* mq,
                                          const uint8_t* map, uint32_t nnz, uint32_t total, uint32_t tid,
                                          unsigned long long base, bool mvn, const DeferQ& dq) {
  constexpr int W = kTile / 64;
  const uint32_t lane = tid & 63, wave = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const uint32_t pbase = s.tile * kTile;
  const uint32_t shift = map_shift(total);
  uint32_t nm = 0, round = 0;
  for (uint32_t b0 = 0; b0 < total; b0 += kTile * K, round++) {
    // every lane issues its K row loads back to back, unconditionally (pairs past the end
    // re-read the tile's last pair), so the K loads are in flight together and the lane
    // waits once; a load under a branch would be waited for before the next one issues
    Row row[K];
    uint32_t qq[K], rid[K];
#pragma unroll
    for (int k = 0; k < K; k++) rid[k] = map_rank(s, map, shift, min(b0 + k * kTile + tid, total - 1));
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t r = rid[k];
      qq[k] = s.nz_q[r];
      rid[k] = min(b0 + k * kTile + tid, total - 1) + s.nz_rd[r];
    }
#pragma unroll
    for (int k = 0; k < K; k++) row[k] = a.db.rows[rid[k]];
    uint32_t mask = 0, pend = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t e = eval_row<FILT, (FILT >= 2)>(a, s, qq[k], pbase + qq[k], row[k], rid[k]);
      const bool in = b0 + k * kTile + tid < total;
      mask |= (e == 1 && in) ? 1u << k : 0u;
      pend |= (e == 2 && in) ? 1u << k : 0u;
    }
    if constexpr (FILT >= 2) {
      if (mvn) mask |= sweep_programs<K, FILT>(a, s, map, nnz, total, b0, pend, tid, dq, s.wsum[0]);
    }
    uint32_t* ws = s.wsum2[round & 1];
    unsigned long long bal[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      bal[k] = __ballot((mask >> k) & 1u);
      if (lane == 0) ws[k * W + wave] = uint32_t(__popcll(bal[k]));
    }
    __syncthreads();
    uint32_t acc = nm;
#pragma unroll
    for (int k = 0; k < K; k++) {
      uint32_t woff = 0, tk = 0;
#pragma unroll
      for (int w = 0; w < W; w++) {
        const uint32_t t = ws[k * W + w];
        woff += (uint32_t(w) < wave) ? t : 0;
        tk += t;
      }
      if ((mask >> k) & 1u) {
        const uint32_t pos = acc + woff + uint32_t(__popcll(bal[k] & lt));
        const uint32_t adv = row[k].adv & ROW_ADV_MASK;
        if (DIRECT) {
          if (base + pos < a.out_cap) {
            a.out_pkg[base + pos] = a.out_base + a.p0 + pbase + qq[k];
            a.out_adv[base + pos] = adv;
          }
        } else {
          if (pos < uint32_t(MB)) {
            madv[pos] = adv;
            mq[pos] = uint8_t(qq[k]);
          }
        }
      }
      acc += tk;
    }
    nm = acc;
  }
  return nm;
}

// SEG form of the sweep: wave w takes the contiguous pairs [s0, s1) of the tile (a quarter,
// in 64-pair units) in rounds of K x 64 and compacts its matches into its own quarter of the
// LDS buffer, so no round waits on the other waves (the shared form needs a workgroup
// barrier per round to place matches across waves); the waves' counts are combined once,
// after the sweep.  DIRECT: the wave's re-sweep straight to the output (base = its offset).
template <int K, int MBW, int FILT, bool DIRECT>
__device__ __forceinline__ uint32_t sweep_seg(const SweepArgs& a, const SweepShared<FILT>& s, uint32_t* madv,
                                              uint8_t* mq, const uint8_t* map, uint32_t nnz, uint32_t total,
                                              uint32_t s0, uint32_t s1, uint32_t lane, unsigned long long base) {
  const unsigned long long lt = (1ull << lane) - 1ull;
  const uint32_t pbase = s.tile * kTile;
  const uint32_t shift = map_shift(total);
  uint32_t nm = 0;
  for (uint32_t b0 = s0; b0 < s1; b0 += 64 * K) {
    Row row[K];
    uint32_t qq[K], rid[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t j = min(b0 + k * 64 + lane, s1 - 1);
      rid[k] = map_rank(s, map, shift, j);
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t r = rid[k];
      qq[k] = s.nz_q[r];
      rid[k] = min(b0 + k * 64 + lane, s1 - 1) + s.nz_rd[r];
    }
#pragma unroll
    for (int k = 0; k < K; k++) row[k] = a.db.rows[rid[k]];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const bool m = eval_row<FILT>(a, s, qq[k], pbase + qq[k], row[k], rid[k]) != 0 && b0 + k * 64 + lane < s1;
      const unsigned long long bal = __ballot(m);
      if (m) {
        const uint32_t pos = nm + uint32_t(__popcll(bal & lt));
        const uint32_t adv = row[k].adv & ROW_ADV_MASK;
        if (DIRECT) {
          if (base + pos < a.out_cap) {
            a.out_pkg[base + pos] = a.out_base + a.p0 + pbase + qq[k];
            a.out_adv[base + pos] = adv;
          }
        } else if (pos < uint32_t(MBW)) {
          madv[pos] = adv;
          mq[pos] = uint8_t(qq[k]);
        }
      }
      nm += uint32_t(__popcll(bal));
    }
  }
  return nm;
}

// The sweep of tile t (packages t * 256 ..) given each lane's package record r.
template <int K, int MB, int FILT, int SEG = 0>
__device__ __forceinline__ void sweep_tile(const SweepArgs& a, SweepShared<FILT>& s, uint32_t* madv, uint8_t* mq,
                                           uint8_t* map, uint32_t t, uint32_t tid, const PkgRec& r,
                                           const DeferQ& dq = DeferQ{nullptr, nullptr, 0}) {
  const uint32_t lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s.tile = t;
  const uint32_t p = t * kTile + tid;
  s.k0[tid] = r.k0;
  s.k1[tid] = r.k1;
  if constexpr (FILT < 2) s.k2[tid] = r.k2;
  s.kinfo[tid] = r.meta.z;
  s.koff[tid] = r.meta.w;
  if constexpr (FILT) s.pattr[tid] = (a.attr && p < a.n) ? a.attr[p] : make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu);
  // compact the packages that have rows (ballot) and scan their row counts
  const uint32_t cnt = r.meta.y;
  const unsigned long long bal = __ballot(cnt != 0);
  const uint32_t lrank = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) s.wsum[1][wave] = uint32_t(__popcll(bal));
  uint32_t excl = 0;
  const uint32_t total = block_exscan<kTile>(s.wsum[0], cnt, tid, excl);  // its barriers publish wsum[1]
  uint32_t nrank = lrank, nnz = 0;
#pragma unroll
  for (int w = 0; w < kTile / 64; w++) {
    const uint32_t c = s.wsum[1][w];
    nrank += (uint32_t(w) < wave) ? c : 0;
    nnz += c;
  }
  if (cnt) {
    s.nz_scan[nrank] = excl;
    s.nz_rd[nrank] = r.meta.x - excl;
    s.nz_q[nrank] = tid;
  }
  if (tid == 0) s.nz_scan[nnz] = total;
  __syncthreads();
  {  // pair (bucket of 2^shift pairs) -> nz rank map: every lane fills a contiguous run of it
    const uint32_t shift = map_shift(total), nb = (total + (1u << shift) - 1) >> shift;
    const uint32_t per = (nb + kTile - 1) / kTile;
    uint32_t b = tid * per;
    const uint32_t be = min(b + per, nb);
    if (b < be) {
      uint32_t rr = pair_rank(s, nnz, b << shift);
      for (; b < be; b++) {
        while (s.nz_scan[rr + 1] <= (b << shift)) rr++;
        map[b] = uint8_t(rr);
      }
    }
    __syncthreads();
  }

  if constexpr (SEG != 0) {
    constexpr int MBW = MB / 4;
    const uint32_t seg = ((total + 4 * 64 - 1) / (4 * 64)) * 64;  // a wave's share, whole 64-pair units
    const uint32_t s0 = min(total, wave * seg), s1 = min(total, s0 + seg);
    uint32_t* madv_w = madv + wave * MBW;
    uint8_t* mq_w = mq + wave * MBW;
    const uint32_t nmw = sweep_seg<K, MBW, FILT, false>(a, s, madv_w, mq_w, map, nnz, total, s0, s1, lane, 0);
    if (lane == 0) s.wsum[0][wave] = nmw;  // the row-count scan is done with wsum[0]
    __syncthreads();
    uint32_t woff = 0, nm = 0;
#pragma unroll
    for (int w = 0; w < kTile / 64; w++) {
      const uint32_t c = s.wsum[0][w];
      woff += (uint32_t(w) < wave) ? c : 0;
      nm += c;
    }
    if (tid == 0) {
      s.base = nm ? atomicAdd(&a.ctl[0], (unsigned long long)nm) : 0ull;
      TileDir e;
      e.base = s.base;
      e.count = nm;
      e.pad = 0;
      a.dir[a.t0 + t] = e;
    }
    __syncthreads();
    const unsigned long long base = s.base + woff;
    if (nmw <= uint32_t(MBW)) {
      const uint32_t pb = a.out_base + a.p0 + t * kTile;
      for (uint32_t i = lane; i < nmw; i += 64) {
        if (base + i < a.out_cap) {
          a.out_pkg[base + i] = pb + mq_w[i];
          a.out_adv[base + i] = madv_w[i];
        }
      }
    } else {
      sweep_seg<K, MBW, FILT, true>(a, s, madv_w, mq_w, map, nnz, total, s0, s1, lane, base);  // rare
    }
    return;
  }
  // a tile with Maven packages runs its rounds' Maven programs compacted (sweep_programs)
  const bool mvn = FILT >= 2 && dq.cap && __syncthreads_or((r.meta.z & KI_MVN) != 0);
  const uint32_t nm = sweep<K, MB, FILT, false>(a, s, madv, mq, map, nnz, total, tid, 0, mvn, dq);

  // the tile's output segment: one atomic reservation, no waiting on other tiles; the
  // tile directory gives the global (package, advisory) order
  if (tid == 0) {
    s.base = nm ? atomicAdd(&a.ctl[0], (unsigned long long)nm) : 0ull;
    TileDir e;
    e.base = s.base;
    e.count = nm;
    e.pad = 0;
    a.dir[a.t0 + t] = e;
  }
  __syncthreads();
  const unsigned long long base = s.base;
  if (nm <= uint32_t(MB)) {
    const uint32_t pb = a.out_base + a.p0 + t * kTile;
    for (uint32_t i = tid; i < nm; i += kTile) {
      if (base + i < a.out_cap) {
        a.out_pkg[base + i] = pb + mq[i];
        a.out_adv[base + i] = madv[i];
      }
    }
  } else {
    sweep<K, MB, FILT, true>(a, s, madv, mq, map, nnz, total, tid, base, mvn, dq);  // rare: more matches than the buffer
  }
}

template <int K, int MB, int FILT>
__global__ __launch_bounds__(kTile) void sweep_kernel(SweepArgs a) {
  __shared__ SweepShared<FILT> s;
  __shared__ uint32_t madv[MB];
  __shared__ uint8_t mq[MB];
  __shared__ uint8_t map[kMapCap];  // pair -> nz rank of its package
  constexpr uint32_t kQ = FILT >= 2 ? 512 : 1;
  __shared__ uint32_t dqj[kQ], dqres[FILT >= 2 ? kTile / 8 : 1];
  const uint32_t tid = threadIdx.x, t = blockIdx.x;
  const uint32_t p = t * kTile + tid;
  PkgRec r;
  r.meta = make_uint4(0, 0, 0, 0);
  r.k0 = r.k1 = r.k2 = 0;
  if (p < a.n) r = a.rec[p];
  sweep_tile<K, MB, FILT>(a, s, madv, mq, map, t, tid, r, DeferQ{dqj, dqres, FILT >= 2 ? kQ : 0u});
}

// Probe and sweep of one tile in one workgroup (the record stays in registers/LDS): tiles
// of one CU sit in different phases, so one tile's probe latency overlaps another's sweep.
// DIAG (measurement only, wrong match lists by construction; "diag_*" variants): bit 0 skips
// the version encoder, bit 1 the index probe, bit 2 the sweep.
// STG: LDS bytes for the tile's string window (smaller: more tiles resident per CU, more
// windows read from global memory instead).
// MOVE: the launch carries the previous pipeline chunk's result move (fa.n_copy workgroups).
// Device-resident launches instantiate without it: copy_out_tiles inlined into the match
// kernel cost registers (44 -> 52 VGPRs) and ~10 % of C2's time even where it never ran.
template <uint32_t GM, int K, int MB, int FILT, int DIAG = 0, int WPE = 1, int SEG = 0, uint32_t STG = kStage,
          bool MOVE = false>
__global__ __launch_bounds__(kTile, WPE) void fused_kernel(FusedArgs fa) {
  constexpr uint32_t kStageVec = STG / 16 + 8;  // + two zero words per wave window (per-wave staging)
  constexpr uint32_t kMbufVec = (MB * 5 + 15) / 16;
  __shared__ uint4 buf[kStageVec > kMbufVec ? kStageVec : kMbufVec];  // strings (probe), then matches (sweep)
  // the probe's per-lane dpkg keys + code table share LDS with the sweep's state (the scan
  // below is done with s.wsum before the table is written)
  struct SweepPart {
    SweepShared<FILT> s;
    uint8_t map[kMapCap];
  };
  struct ProbePart {
    uint32_t kbuf[kTile * kFastKeyStride / 4];
    uint8_t tab[128];
  };
  static_assert(sizeof(ProbePart) <= sizeof(SweepPart), "the probe's LDS fits in the sweep's");
  __shared__ union {
    SweepPart sw;
    ProbePart pr;
  } u;
  SweepShared<FILT>& s = u.sw.s;
  uint8_t* map = u.sw.map;
  const ProbeArgs& a = fa.pa;
  if constexpr (MOVE) {
    if (blockIdx.x < fa.n_copy) {  // pipeline: the previous chunk's result move, dispatched first so the link writes overlap the tiles
      static_assert(sizeof(buf) >= kCopyLdsWords * 4, "the result move borrows the staging buffer");
      __builtin_amdgcn_s_setprio(3);  // its waves issue ahead of the match waves sharing the CU: the link is the bound
      copy_out_tiles(fa.co, blockIdx.x, fa.n_copy, reinterpret_cast<uint32_t*>(buf));
      return;
    }
  }
  const uint32_t tid = threadIdx.x;
  if (!MOVE && fa.ctl_zero && blockIdx.x == 0 && tid < 8) fa.ctl_zero[tid] = 0ull;  // the next pass's counters
  const uint32_t t = MOVE ? blockIdx.x - fa.n_copy : (fa.tile_map ? fa.tile_map[blockIdx.x] : blockIdx.x);
  const uint32_t p = t * kTile + tid;
  uint2 d = make_uint2(0xFFFFFFFFu, 0);
  if (p < a.n) d = a.pk[p];
  constexpr bool kWaveStage = (SEG & 2) != 0;
  const uint32_t g = t * kGroupsPerTile + (kWaveStage ? (tid >> 6) : 0u);  // the window's first group
  const uint64_t w0 = a.tile_off[g], w1 = a.tile_off[kWaveStage ? g + 1 : (t + 1) * kGroupsPerTile];  // before the scan's barriers
  const uint32_t nlen = d.y & 0xFFFFu, vlen = d.y >> 16;
  uint32_t off = 0;
  uint4* sbuf = buf;  // this lane's staging window
  const uint64_t base16 = w0 & ~uint64_t(15);
  bool staged;
  if constexpr (kWaveStage) {
    off = wave_exscan(nlen + vlen, tid & 63);
    sbuf = buf + (tid >> 6) * (STG / 4 / 16 + 2);
    staged = w1 - base16 <= STG / 4;
    if (staged) stage_window_wave<STG>(sbuf, a.arena + base16, uint32_t((w1 - base16 + 15) / 16), tid & 63);
    if (tid < 128) u.pr.tab[tid] = deb_fast_code(tid);
    __syncthreads();  // the code table (one wave's LDS traffic alone is ordered)
  } else {
    block_exscan<kTile>(s.wsum[0], nlen + vlen, tid, off);
    staged = w1 - base16 <= STG;
    if (staged) stage_window<STG>(buf, a.arena + base16, uint32_t((w1 - base16 + 15) / 16), tid);
    if (tid < 128) u.pr.tab[tid] = deb_fast_code(tid);
    __syncthreads();
  }
  PkgRec r;
  r.meta = make_uint4(0, 0, 0, 0);
  r.k0 = r.k1 = r.k2 = 0;
  if (p < a.n && d.x < a.db.n_plats) {
    if (staged) {
      const uint8_t* sb = reinterpret_cast<const uint8_t*>(sbuf) + uint32_t(w0 - base16) + off;
      probe_one<GM, uint32_t, DIAG & 3>(a, p, d.x, nlen, vlen, sb, sb + nlen, w0 + off + nlen, r,
                                        reinterpret_cast<uint8_t*>(u.pr.kbuf) + tid * kFastKeyStride, u.pr.tab);
    } else {
      const uint8_t* gb = a.arena + w0 + off;
      probe_one<GM, uint32_t, DIAG & 3>(a, p, d.x, nlen, vlen, gb, gb + nlen, w0 + off + nlen, r);
    }
  }
  if (DIAG & 4) r.meta.y = 0;  // no rows: the sweep does nothing
  __syncthreads();  // the strings are dead: buf becomes the match buffer
  uint32_t* madv = reinterpret_cast<uint32_t*>(buf);
  // the Maven program queue takes the rest of buf behind the match buffer (FILT >= 2)
  constexpr uint32_t kBufWords = sizeof(buf) / 4, kMbWords = (uint32_t(MB) * 5 + 3) / 4;
  constexpr uint32_t kQ = kBufWords > kMbWords + kTile / 8 + 16 ? kBufWords - kMbWords - kTile / 8 : 0;
  static_assert(FILT < 2 || kQ >= 16, "no room for the Maven program queue");
  const DeferQ dq{madv + kMbWords + kTile / 8, madv + kMbWords, FILT >= 2 ? kQ : 0u};
  sweep_tile<K, MB, FILT, SEG>(fa.sa, s, madv, reinterpret_cast<uint8_t*>(madv + MB), map, t, tid, r, dq);
}

template <uint32_t GM, int DIAG = 0>
void launch_probe(uint32_t n_tiles, hipStream_t st, const ProbeArgs& a) {
  hipLaunchKernelGGL((probe_kernel<GM, DIAG>), dim3(n_tiles), dim3(kTile), 0, st, a);
}

template <int K, int MB, int FILT>
void launch_sweep(uint32_t n_tiles, hipStream_t st, const SweepArgs& a) {
  hipLaunchKernelGGL((sweep_kernel<K, MB, FILT>), dim3(n_tiles), dim3(kTile), 0, st, a);
}

template <uint32_t GM, int K, int MB, int FILT, int DIAG = 0, int WPE = 1, int SEG = 0, uint32_t STG = kStage>
void launch_fused(uint32_t n_tiles, hipStream_t st, const FusedArgs& a) {
  if (a.n_copy)
    hipLaunchKernelGGL((fused_kernel<GM, K, MB, FILT, DIAG, WPE, SEG, STG, true>), dim3(n_tiles + a.n_copy), dim3(kTile), 0,
                       st, a);
  else
    hipLaunchKernelGGL((fused_kernel<GM, K, MB, FILT, DIAG, WPE, SEG, STG, false>), dim3(n_tiles), dim3(kTile), 0, st, a);
}

// Table entry of variant (F, K, MB) for grammar set GM / row-filter level FILT
// (match_variants.h: F = 0 split, 1-3 fused, 4 fused with per-wave sweep segments, 5 also
// per-wave staging, 11-15 fused measurement builds).
template <uint32_t GM, int FILT, int F, int K, int MB>
constexpr FusedFn fused_entry() {
  if constexpr (F == 0) return nullptr;
  else if constexpr (F == 4) return &launch_fused<GM, K, MB, FILT, 0, 1, 1>;
  else if constexpr (F == 5) return &launch_fused<GM, K, MB, FILT, 0, 1, 3>;
  else if constexpr (F == 6) return &launch_fused<GM, K, MB, FILT, 0, 6, 3>;
  // the all-grammar K <= 2 kernels are held at 5 waves per SIMD (96 VGPRs): the Maven program
  // queue (sweep_programs) took them to 97 and 4 waves
  else return &launch_fused<GM, K, MB, FILT, (F >= 10 ? F - 10 : 0), (FILT >= 2 && K <= 2 && F == 1) ? 5 : TVM_FUSED_WPE(F)>;
}

}  // namespace
}  // namespace tvm
