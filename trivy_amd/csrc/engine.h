// Device engine: HBM-resident advisory tables + the match path (gfx950).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <memory>
#include <cstdint>
#include <mutex>
#include <string>
#include <string_view>
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
  uint64_t slot_mask = 0;
  const uint8_t* name_arena = nullptr;
  const Row* rows = nullptr;
  const uint64_t* key_words = nullptr;
  const PlatInfo* plats = nullptr;
  uint32_t n_plats = 0;
  const RowAux* aux = nullptr;
  const uint32_t* aux_ids = nullptr;
};

// A package batch.  pk[i] = {plat, name_len | ver_len << 16}; the name and version bytes
// of every package sit back to back in `arena`, package after package, so offsets are
// implicit: tile_off[g] is the arena offset of package g * kGroup (the kernels scan the
// lengths within a 64-package group, one wavefront).  plat = 0xFFFFFFFF when the bucket is absent.  Lengths
// saturate at 0xFFFF (the stored bytes are cut to match).  Optional per-package attributes
// (common.h PA_*), present when the batch touches rows with filters: attr[i] = {arch id |
// PA_NOARCH, ksplice tag or CPE-set id}; CPE set s is the bitset cpe_bits[s * cpe_words ..
// +cpe_words) over CPE indices.
struct HostBatch {
  std::vector<uint2> pk;
  std::vector<uint8_t> arena;
  std::vector<uint64_t> tile_off;
  std::vector<uint2> attr;
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
  uint64_t k0, k1;
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
};
enum : uint32_t { ERR_SPILL = 1, ERR_TILES = 2 };

// The end-to-end pipeline's result move for one chunk (packages [p0, p1)): the chunk's
// per-package advisory lists (device CSR from order_kernel) into the pinned host result
// through 16-byte kernel stores (kernel stores into host memory: 55 GB/s; a DMA
// device-to-host copy: 28.6 GB/s; profiles/r03/pcie_probe.txt).  The chunk's advisory range
// is read from the device row ends, so the host never waits per chunk.  Run by extra
// workgroups of the next chunk's match launch (Engine::launch_tiles), so the link writes
// overlap that chunk's matching, or by copy_out_kernel for the last chunk.
struct CopyOutArgs {
  const uint32_t* row_end = nullptr;  // device CSR
  const uint32_t* csr_adv = nullptr;
  uint4* row_end_h = nullptr;         // device addresses of the pinned host result (16-B aligned, padded)
  uint4* adv_h = nullptr;
  uint32_t p0 = 0, p1 = 0;            // p0 a multiple of 4, p1 > p0
  uint64_t cap = 0;                   // advisory capacity (an overflowed pass's range is cut to it)
};

// Whole 16-byte units are moved: the words before the chunk's range are the previous chunk's
// (final) and those after it are rewritten by the next chunk's move, which runs later.
__device__ __forceinline__ void copy_out_range(const CopyOutArgs& a, uint64_t tid, uint64_t stride) {
  const uint64_t s0 = a.p0 ? a.row_end[a.p0 - 1] : 0, e0 = a.row_end[a.p1 - 1];
  const uint64_t e = e0 < a.cap ? e0 : a.cap, s = s0 < e ? s0 : e;
  const uint64_t u0 = s / 4, nu = (e + 3) / 4 - u0;                    // advisory units
  const uint64_t r0 = a.p0 / 4, nr = (uint64_t(a.p1) + 3) / 4 - r0;    // row-end units
  const uint4* csr = reinterpret_cast<const uint4*>(a.csr_adv);
  const uint4* re = reinterpret_cast<const uint4*>(a.row_end);
  for (uint64_t i = tid; i < nu + nr; i += stride) {
    if (i < nu) a.adv_h[u0 + i] = csr[u0 + i];
    else a.row_end_h[r0 + (i - nu)] = re[r0 + (i - nu)];
  }
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
  bool alloc_batch(const HostBatch& hb, DevBatch& b, std::string& err);
  bool upload(const HostBatch& hb, DevBatch& b, std::string& err);
  uint32_t grammar_set(const HostBatch& hb) const;
  uint64_t scratch_words(const HostBatch& hb) const;
  // Frees a batch's / a match list's device buffers (device = the GPU they live on; no
  // engine state is touched, so a batch outlives a hot swap of the engine's tables).
  static void free_batch(int device, DevBatch& b);
  bool alloc_matches(uint64_t cap, uint32_t n_pkgs, DevMatches& m, std::string& err);
  static void free_matches(int device, DevMatches& m);

  // Enqueues one match pass (probe + sweep over every tile) on `stream`; no host sync.
  bool launch(const DevBatch& b, const DevMatches& m, hipStream_t stream, std::string& err);
  // The pass over tiles [t_begin, t_end) only: probe on `probe_st`, sweep on `sweep_st`
  // behind event `ev` (the caller zeroes m.ctl once before the first chunk).
  // co: a previous chunk's result move, run by extra workgroups of this launch (fused
  // variants) or by its own kernel ahead of it (split variants).
  bool launch_tiles(const DevBatch& b, const DevMatches& m, uint32_t t_begin, uint32_t t_end, hipStream_t probe_st,
                    hipStream_t sweep_st, hipEvent_t ev, std::string& err, const CopyOutArgs* co = nullptr);

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
int resolve_variant(int v, uint32_t gm);

}  // namespace tvm
