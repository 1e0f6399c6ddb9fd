// Device engine: HBM-resident advisory tables + the match path (gfx950).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <memory>
#include <cstdint>
#include <mutex>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "common.h"

namespace tvm {

class DB;

constexpr int kTile = 256;   // packages per tile (workgroup) of the match kernels
constexpr int kGroup = 64;   // packages per offset group (one wavefront); tile_off is per group
constexpr int kGroupsPerTile = kTile / kGroup;

// Device view of the flattened tables (db.h device images).
struct DevDB {
  const Slot* slots = nullptr;
  const uint8_t* slot_fp = nullptr;  // DB::slot_fp
  uint64_t slot_mask = 0;
  const uint8_t* name_arena = nullptr;
  const Row* rows = nullptr;
  const RowOff* row_off = nullptr;  // parallel to rows
  const uint64_t* key_words = nullptr;
  const PlatInfo* plats = nullptr;
  uint32_t n_plats = 0;
  const RowAux* aux = nullptr;
  const uint32_t* aux_ids = nullptr;
};

// Vector storage whose growth leaves new elements default-initialised (plain data: untouched)
// rather than zeroed: the bulk adds (tvm_batch_add_targets) size the batch arrays once and fill
// them on the host threads, so no serial zero fill runs first and every page is first touched
// by the thread that writes it.
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using BulkVec = std::vector<T, NoInitAlloc<T>>;

// A package batch.  pk[i] = {plat, name_len | ver_len << 16}; the name and version bytes
// of every package sit back to back in `arena`, package after package, so offsets are
// implicit: tile_off[g] is the arena offset of package g * kGroup (the kernels scan the
// lengths within a 64-package group, one wavefront).  plat = 0xFFFFFFFF when the bucket is absent.  Lengths
// saturate at 0xFFFF (the stored bytes are cut to match).  Optional per-package attributes
// (common.h PA_*), present when the batch touches rows with filters: attr[i] = {arch id |
// PA_NOARCH, ksplice tag or CPE-set id}; CPE set s is the bitset cpe_bits[s * cpe_words ..
// +cpe_words) over CPE indices.
struct HostBatch {
  BulkVec<uint2> pk;
  BulkVec<uint8_t> arena;
  BulkVec<uint64_t> tile_off;
  BulkVec<uint2> attr;
  std::vector<uint32_t> cpe_bits;
  uint32_t cpe_words = 0;
  void add(uint32_t plat, std::string_view name, std::string_view ver);
  void add(uint32_t plat, std::string_view name, std::string_view ver, uint2 a);
  size_t size() const { return pk.size(); }
  uint32_t n_tiles() const { return uint32_t((pk.size() + kTile - 1) / kTile); }
  uint32_t n_groups() const { return uint32_t((pk.size() + kGroup - 1) / kGroup); }
  // arena offset of package i's name (O(kTile) per call); all of them at once
  uint64_t name_off(size_t i) const;
  void name_offsets(std::vector<uint64_t>& off) const;
  std::string_view name(size_t i) const;
  std::string_view version(size_t i) const;
  void clear();
};

// Per-package record handed from probe_kernel to sweep_kernel (match_kernel.h):
// meta = {row_begin, row_count, key info, spill word offset}; k0/k1 = the installed key's
// first 16 bytes as big-endian words.
struct PkgRec {
  uint4 meta;
  uint64_t k0, k1, k2;  // the installed key's first 24 bytes, big-endian (rows compare 24-byte heads)
};

struct DevBatch {
  uint2* pk = nullptr;
  uint64_t* tile_off = nullptr;
  uint8_t* arena = nullptr;
  uint2* attr = nullptr;
  uint32_t* cpe_bits = nullptr;
  uint32_t cpe_words = 0;
  uint32_t n_cpe_sets = 0;
  uint32_t n = 0;
  uint32_t n_tiles = 0;
  uint64_t arena_bytes = 0;
  uint64_t spill_words = 0;  // scratch for installed keys longer than 32 bytes
  uint32_t gm = 0;           // grammar bits (1 << Cmp) of the batch's platforms (libver.h GM_*)
  uint32_t pkg_base = 0;     // added to the package index of every match (multi-GPU shards)
  uint64_t* spill = nullptr;  // the batch's own long-key / Maven-parse scratch (never shared between batches)
  uint64_t spill_cap = 0;
  // launch order of the tiles (device-resident launches of batches with library grammars:
  // the heaviest tiles first, so the launch does not end on a tail of Maven-program tiles);
  // nullptr = tile order
  uint32_t* tile_map = nullptr;
  // batches of the all-grammar set: the first n_lean_tiles entries of tile_map are the tiles
  // without Maven / RubyGems packages, matched by the GM_LEAN kernel in a launch of their own
  // (Engine::launch); the rest take the all-grammar kernel
  uint32_t n_lean_tiles = 0;
  // probe -> sweep hand-off (device only)
  PkgRec* rec = nullptr;
  uint4* tail = nullptr;  // key bytes 16..31 per package
};

// Device-side results of one match pass: the per-package advisory lists as two columns
// (pkg[i], adv[i]).  Tile t (packages [256t, 256t+256)) owns the segment
// [dir[t].base, dir[t].base + dir[t].count), in (package, advisory) order; segments are
// placed by one atomic reservation per tile, so the global order is read through the
// directory.
struct TileDir {
  unsigned long long base;
  uint32_t count;
  uint32_t pad;
};
struct DevMatches {
  uint32_t* pkg = nullptr;
  uint32_t* adv = nullptr;
  uint64_t cap = 0;  // capacity in matches
  TileDir* dir = nullptr;
  uint32_t dir_cap = 0;
  // control block (device): [0] total matches (reservation counter), [1] n - first
  // poisoned pkg (0 = none), [2] spill words used, [3] error bits
  unsigned long long* ctl = nullptr;
  // device-resident launches alternate between two control blocks: a launch counts into
  // ctl_next (zeroed by the launch before) and zeroes the block it leaves behind, so a pass
  // is one kernel, no memset (Engine::launch); ctl_mem = the allocation
  unsigned long long* ctl_next = nullptr;
  unsigned long long* ctl_mem = nullptr;
};
// ERR_BOUNDS: a result move or an unpack found an index beyond the buffer it was sized for
// (the store is dropped and the pass fails; never expected: a guard, not a code path)
enum : uint32_t { ERR_SPILL = 1, ERR_TILES = 2, ERR_BOUNDS = 8 };  // 4 is redhat.h ERR_RH_ORDER

// The end-to-end pipeline's result move for one chunk (tiles [t0, t1)): the chunk's match
// segments, straight from the tile directory, become the per-package advisory lists (CSR)
// in the pinned host result - no CSR in HBM, no separate order kernel.  A tile's segment is
// already in package order (the match kernels compact in lane order), so the move only
// places it: tile t's lists start at chunk_base[c] + the counts of the chunk's tiles before
// t, and its 256 row ends are that base + the inclusive scan of its per-package counts.
// Stores into host memory are 16-byte kernel stores (55 GB/s; a DMA device-to-host copy
// runs at 28.6 GB/s, profiles/r03/pcie_probe.txt), so each segment is realigned in registers to
// the destination's 16-byte units.  Run by the first workgroups of the next chunk's match
// launch (Engine::launch_tiles), so the link writes overlap that chunk's matching, or by
// copy_out_kernel for the last chunk.  chunk_base[0] = 0 is set by the host; the move of
// chunk c writes chunk_base[c + 1].
struct CopyOutArgs {
  const TileDir* dir = nullptr;       // the chunk's match list
  const uint32_t* pkg = nullptr;
  const uint32_t* adv = nullptr;
  uint32_t* row_end_h = nullptr;      // device addresses of the pinned host result (16-B aligned,
  uint32_t* adv_h = nullptr;          // row ends padded to whole tiles, advisories to whole units)
  unsigned long long* chunk_base = nullptr;
  uint32_t c = 0;                     // chunk index
  uint32_t t0 = 0, t1 = 0;            // the chunk's tiles
  uint32_t pkg_base = 0;              // subtracted from the match list's package indices
  uint64_t cap = 0;                   // match / result capacity (an overflowed pass moves no advisories)
  uint32_t packed = 0;                // 1: advisories as 3-byte little-endian indices (the DB has < 2^24)
  uint64_t adv_units = 0;             // 16-byte units of adv_h
  uint64_t row_end_units = 0;         // 16-byte units of row_end_h
  unsigned long long* ctl = nullptr;  // the pass's control block: ctl[3] |= ERR_BOUNDS on a guard hit
};
constexpr uint32_t kCopyRunMax = kTile;  // tiles per prefix segment of the wave-per-tile move
// copy_out_tiles' LDS: the run's tile offsets + a 256-entry count array per wave
constexpr uint32_t kCopyLdsWords = 2 * kCopyRunMax + 8 + (kTile / 64) * kTile;
constexpr uint32_t kCopyWorkgroups = 256;      // workgroups of a result move

// Exclusive block scan of v; tot = the block's sum.  red: kTile / 64 words of LDS.
__device__ __forceinline__ uint32_t copy_block_scan(uint32_t v, uint32_t* red, uint32_t tid, uint32_t& tot) {
  const uint32_t lane = tid & 63, wave = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= uint32_t(o)) x += y;
  }
  __syncthreads();  // red is free
  if (lane == 63) red[wave] = x;
  __syncthreads();
  uint32_t pre = 0;
  tot = 0;
#pragma unroll
  for (int w = 0; w < kTile / 64; w++) {
    const uint32_t r = red[w];
    pre += uint32_t(w) < wave ? r : 0u;
    tot += r;
  }
  return pre + x - v;
}

__device__ __forceinline__ uint32_t copy_block_sum(uint32_t v, uint32_t* red, uint32_t tid) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (int w = 0; w < kTile / 64; w++) s += red[w];
  return s;
}

// One tile's CSR move by one wave (lane of 64): its per-package counts in the wave's own LDS
// array (no workgroup barrier: one wave's LDS operations are ordered), the 256 row ends
// from a wave scan (4 packages a lane, one 16-byte store each), then the segment realigned to
// the destination's 16-byte units (3- or 4-byte indices).  b = the tile's first CSR position.
__device__ __forceinline__ void copy_out_tile_wave(const CopyOutArgs& a, uint32_t t, uint64_t b, uint32_t lane,
                                                   uint32_t* cw) {
  const TileDir d = a.dir[t];
  const bool fits = d.base + d.count <= a.cap && b + d.count <= a.cap;
  const uint32_t p_first = t * kTile;
  reinterpret_cast<uint4*>(cw)[lane] = make_uint4(0, 0, 0, 0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (fits)
    for (uint32_t i0 = 0; i0 < d.count; i0 += 4 * 64) {  // four loads in flight per lane
      uint32_t q[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t i = i0 + u * 64 + lane;
        q[u] = i < d.count ? a.pkg[d.base + i] - a.pkg_base - p_first : kTile;
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (q[u] < kTile) atomicAdd(&cw[q[u]], 1u);
    }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint4 c4 = reinterpret_cast<const uint4*>(cw)[lane];
  const uint32_t s0 = c4.x, s1 = s0 + c4.y, s2 = s1 + c4.z, s3 = s2 + c4.w;
  uint32_t x = s3;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= uint32_t(o)) x += y;
  }
  const uint32_t e = uint32_t(b) + x - s3;  // row ends are 32-bit
  if (p_first / 4 + lane < a.row_end_units)
    reinterpret_cast<uint4*>(a.row_end_h)[p_first / 4 + lane] = make_uint4(e + s0, e + s1, e + s2, e + s3);
  else
    atomicOr(a.ctl + 3, (unsigned long long)ERR_BOUNDS);
  if (a.packed) {  // 3 bytes per advisory: destination bytes [3b, 3(b + count)) in 16-byte units
    const uint64_t B0 = 3 * b, B1 = 3 * (b + d.count), U0 = B0 >> 4;
    uint64_t nu = fits && d.count ? ((B1 + 15) >> 4) - U0 : 0;
    if (nu && U0 + nu > a.adv_units) {  // guard: never expected
      if (lane == 0) atomicOr(a.ctl + 3, (unsigned long long)ERR_BOUNDS);
      nu = 0;
    }
    uint8_t* dst = reinterpret_cast<uint8_t*>(a.adv_h);
    constexpr int kP = 2;
    for (uint64_t j0 = 0; j0 < nu; j0 += uint64_t(kP) * 64) {
      uint32_t id[kP][6];
#pragma unroll
      for (int k = 0; k < kP; k++) {
        const uint64_t j = j0 + uint64_t(k) * 64 + lane, g0 = ((U0 + j) * 16) / 3;
#pragma unroll
        for (int tt = 0; tt < 6; tt++) {
          const int64_t i = int64_t(g0 + tt) - int64_t(b);  // segment index of the unit's tt-th advisory
          id[k][tt] = (j < nu && i >= 0 && i < int64_t(d.count)) ? a.adv[d.base + uint64_t(i)] : 0u;
        }
      }
#pragma unroll
      for (int k = 0; k < kP; k++) {
        const uint64_t j = j0 + uint64_t(k) * 64 + lane;
        if (j >= nu) continue;
        const uint64_t G0 = (U0 + j) * 16, g0 = G0 / 3;
        const uint32_t r = uint32_t(G0 - g0 * 3);  // byte of advisory g0 the unit starts at
        uint32_t wv[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const uint32_t tt = (r + q) / 3, kb = (r + q) % 3;
          wv[q >> 2] |= ((id[k][tt] >> (8 * kb)) & 0xFFu) << (8 * (q & 3));
        }
        if (G0 >= B0 && G0 + 16 <= B1) {
          reinterpret_cast<uint4*>(dst)[U0 + j] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        } else {  // a unit shared with a neighbour tile: its own bytes only
#pragma unroll
          for (int q = 0; q < 16; q++)
            if (G0 + q >= B0 && G0 + q < B1) dst[G0 + q] = uint8_t(wv[q >> 2] >> (8 * (q & 3)));
        }
      }
    }
    return;
  }
  const uint64_t u0 = b >> 2;
  uint64_t nu = fits && d.count ? ((b + d.count + 3) >> 2) - u0 : 0;
  if (nu && u0 + nu > a.adv_units) {  // guard: never expected
    if (lane == 0) atomicOr(a.ctl + 3, (unsigned long long)ERR_BOUNDS);
    nu = 0;
  }
  const uint32_t sh = uint32_t(b & 3);
  constexpr int kU = 4;
  for (uint64_t j0 = 0; j0 < nu; j0 += uint64_t(kU) * 64) {
    uint32_t v[kU][4];
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const uint64_t j = j0 + uint64_t(k) * 64 + lane;
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const int64_t i = int64_t(j * 4 + w) - int64_t(sh);  // segment index of the unit's word w
        v[k][w] = (j < nu && i >= 0 && i < int64_t(d.count)) ? a.adv[d.base + uint64_t(i)] : 0u;
      }
    }
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const uint64_t j = j0 + uint64_t(k) * 64 + lane;
      if (j >= nu) continue;
      const int64_t i0 = int64_t(j * 4) - int64_t(sh);
      if (i0 >= 0 && i0 + 4 <= int64_t(d.count)) {
        reinterpret_cast<uint4*>(a.adv_h)[u0 + j] = make_uint4(v[k][0], v[k][1], v[k][2], v[k][3]);
      } else {  // the segment's first or last unit, shared with a neighbour tile: its own words only
#pragma unroll
        for (int w = 0; w < 4; w++)
          if (i0 + w >= 0 && i0 + w < int64_t(d.count)) a.adv_h[(u0 + j) * 4 + w] = v[k][w];
      }
    }
  }
}

// Workgroup `wg` of `n_wg` moves a contiguous run of the chunk's tiles: the CSR offsets of
// the run's tiles from one block scan per 256 tiles, then each wave moves every fourth tile
// on its own (round 4: a workgroup per tile in turn waited on its count pass, scan and move
// one tile at a time; the kernel trace showed each 1M-package chunk's move taking ~450 us
// beside 180 us of matching).
__device__ __forceinline__ void copy_out_tiles(const CopyOutArgs& a, uint32_t wg, uint32_t n_wg, uint32_t* lds) {
  unsigned long long* pre = reinterpret_cast<unsigned long long*>(lds);  // kCopyRunMax offsets
  uint32_t* red = lds + 2 * kCopyRunMax;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t* cw = red + 8 + wave * kTile;
  const uint32_t nt = a.t1 - a.t0;
  const uint32_t r0 = a.t0 + uint32_t(uint64_t(nt) * wg / n_wg), r1 = a.t0 + uint32_t(uint64_t(nt) * (wg + 1) / n_wg);
  uint32_t before = 0;  // counts of the chunk's tiles before the run (a pass's total fits 32 bits: cap < 2^32)
  for (uint32_t u = a.t0 + tid; u < r0; u += kTile) before += a.dir[u].count;
  unsigned long long b = a.chunk_base[a.c] + copy_block_sum(before, red, tid);
  for (uint32_t s0 = r0; s0 < r1; s0 += kCopyRunMax) {
    const uint32_t s1 = min(r1, s0 + kCopyRunMax);
    uint32_t tot;
    const uint32_t ex = copy_block_scan(s0 + tid < s1 ? a.dir[s0 + tid].count : 0u, red, tid, tot);
    pre[tid] = b + ex;
    __syncthreads();
    for (uint32_t t = s0 + wave; t < s1; t += kTile / 64) copy_out_tile_wave(a, t, pre[t - s0], lane, cw);
    b += tot;
    __syncthreads();  // pre is rewritten by the next segment
  }
  if (wg == n_wg - 1 && tid == 0) a.chunk_base[a.c + 1] = b;
}

class Engine {
 public:
  ~Engine();
  static Engine* open(const DB& db, int device, std::string& err);
  int device() const { return dev_; }
  hipStream_t stream() const { return stream_; }
  uint64_t table_bytes() const { return table_bytes_; }

  // Device-resident batch management.  alloc_batch sizes the device buffers without
  // copying (the pipelined path copies chunk by chunk); upload = alloc + copy.
  // pooled: the buffers come from / go back to the process-wide block cache (pool.h; the
  // pipeline's per-batch buffers), else plain hipMalloc / hipFree
  bool alloc_batch(const HostBatch& hb, DevBatch& b, std::string& err, bool pooled = false);
  bool upload(const HostBatch& hb, DevBatch& b, std::string& err);
  uint32_t grammar_set(const HostBatch& hb) const;
  uint64_t scratch_words(const HostBatch& hb) const;
  // Frees a batch's / a match list's device buffers (device = the GPU they live on; no
  // engine state is touched, so a batch outlives a hot swap of the engine's tables).
  static void free_batch(int device, DevBatch& b, bool pooled = false);
  bool alloc_matches(uint64_t cap, uint32_t n_pkgs, DevMatches& m, std::string& err, bool pooled = false);
  static void free_matches(int device, DevMatches& m, bool pooled = false);

  // Enqueues one match pass (probe + sweep over every tile) on `stream`; no host sync.
  // Moves m.ctl to the other control block (DevMatches::ctl_next).
  bool launch(const DevBatch& b, DevMatches& m, hipStream_t stream, std::string& err);
  // The pass over tiles [t_begin, t_end) only: probe on `probe_st`, sweep on `sweep_st`
  // behind event `ev` (the caller zeroes m.ctl once before the first chunk).
  // co: a previous chunk's result move, run by extra workgroups of this launch (fused
  // variants) or by its own kernel ahead of it (split variants).
  // tmap / tmap_n / gm: (fused variants, whole batch) the launch's grid is tmap_n workgroups
  // over the tiles tmap lists, with the kernel of grammar set gm
  bool launch_tiles(const DevBatch& b, const DevMatches& m, uint32_t t_begin, uint32_t t_end, hipStream_t probe_st,
                    hipStream_t sweep_st, hipEvent_t ev, std::string& err, const CopyOutArgs* co = nullptr,
                    unsigned long long* ctl_zero = nullptr, const uint32_t* tmap = nullptr, uint32_t tmap_n = 0,
                    uint32_t gm = 0);

  // After the pass: the match list as {package, advisory} pairs in (package, advisory) order.
  static bool fetch_ordered(const DevMatches& m, uint32_t n_pkgs, uint64_t total, std::vector<uint2>& out,
                            hipStream_t st, std::string& err);

  // The drop-in path (one driver Detect call): upload, match, download. out = pairs;
  // err_pkg = first poisoned package or -1.  Thread-safe: concurrent calls are coalesced
  // into one launch (the caller that finds no launch running leads and serves every call
  // queued meanwhile) over pooled device buffers and pinned staging - no per-call
  // allocation (engine.hip "drop-in path").
  bool match_host(const HostBatch& hb, std::vector<uint2>& out, int64_t& err_pkg, std::string& err);
  // Drop-in counters: {launches, calls served, calls that shared a launch}.
  void dropin_stats(uint64_t out[3]);

  const DB& db() const { return *db_; }
  const PlatInfo* device_plats() const { return d_.plats; }

  // Sweep-kernel variant (pairs per lane / LDS buffer); returns the previous one.  Default
  // 0 = "auto", overridable with the TVM_VARIANT environment variable at open().
  int set_variant(int v);
  int last_launched() const { return last_launched_; }
  bool verify(std::string& err);
  int variant() const { return variant_; }

 private:
  int dev_ = 0;
  int variant_ = 0;
  std::atomic<int> last_launched_{-1};
  hipStream_t stream_ = nullptr;
  const DB* db_ = nullptr;
  DevDB d_;
  std::vector<void*> allocs_;
  uint64_t table_bytes_ = 0;
  struct Dropin;
  struct DropinReq;
  std::unique_ptr<Dropin> dropin_;
  std::mutex dropin_init_mu_;
  Dropin* dropin(std::string& err);
  bool dropin_run(Dropin& d, DropinReq* const* reqs, size_t n, std::string& err);
};

// Kernel variants: count and names (engine.hip; 0 = "auto").
int num_variants();
const char* variant_name(int v);
int variant_grammar_sets(int v);  // bit 0 dpkg-only, 1 OS grammars, 2 all grammars
int resolve_variant(int v, uint32_t gm);

}  // namespace tvm
