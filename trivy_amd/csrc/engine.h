// Device engine: HBM-resident advisory tables + the match kernel (gfx950).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace tvm {

class DB;

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

// A package batch in SoA-of-descriptors form.  desc[i] = {plat, name_off, ver_off,
// name_len | ver_len << 16} into `arena`; plat = 0xFFFFFFFF when the bucket is absent.
// Optional per-package attributes (common.h PA_*), present when the batch touches rows
// with filters: attr[i] = {arch id | PA_NOARCH, ksplice tag or CPE-set id}; CPE set s is
// the bitset cpe_bits[s * cpe_words .. +cpe_words) over CPE indices.
struct HostBatch {
  std::vector<uint4> desc;
  std::vector<uint8_t> arena;
  std::vector<uint2> attr;
  std::vector<uint32_t> cpe_bits;
  uint32_t cpe_words = 0;
  void add(uint32_t plat, std::string_view name, std::string_view ver);
  void add(uint32_t plat, std::string_view name, std::string_view ver, uint2 a);
};

struct DevBatch {
  uint4* desc = nullptr;
  uint8_t* arena = nullptr;
  uint2* attr = nullptr;
  uint32_t* cpe_bits = nullptr;
  uint32_t cpe_words = 0;
  uint32_t n_cpe_sets = 0;
  uint32_t n = 0;
  uint64_t arena_bytes = 0;
  uint64_t spill_words = 0;  // scratch needed for installed keys longer than the LDS slot
  uint32_t gm = 0;           // grammar bits (1 << Cmp) of the batch's platforms (libver.h GM_*)
};

// Device-side results of one match launch: the per-package advisory lists.
// Tile t (packages [256t, 256t+256)) owns the segment pairs[dir[t].base .. + dir[t].count),
// ordered by (package, advisory); segments are placed by one atomic reservation per
// tile, so the global (package, advisory) order is read through the directory.
struct TileDir {
  unsigned long long base;
  uint32_t count;
  uint32_t pad;
};
struct DevMatches {
  uint2* pairs = nullptr;          // {pkg index, advisory index}
  uint64_t cap = 0;                // capacity in pairs
  TileDir* dir = nullptr;          // one entry per tile
  uint32_t dir_cap = 0;
  // control block (device): [0] total matches (reservation counter), [1] n - first
  // poisoned pkg (0 = none), [2] spill words used, [3] error bits, [4] tile ticket
  unsigned long long* ctl = nullptr;
};
enum : uint32_t { ERR_SPILL = 1, ERR_TILES = 2 };

class Engine {
 public:
  ~Engine();
  static Engine* open(const DB& db, int device, std::string& err);
  int device() const { return dev_; }
  hipStream_t stream() const { return stream_; }
  uint64_t table_bytes() const { return table_bytes_; }

  // Device-resident batch management.
  bool upload(const HostBatch& hb, DevBatch& db, std::string& err);
  uint32_t grammar_set(const HostBatch& hb) const;
  void free_batch(DevBatch& db);
  bool alloc_matches(uint64_t cap, uint32_t n_pkgs, DevMatches& m, std::string& err);
  void free_matches(DevMatches& m);

  // Enqueues one match pass on `stream` (no host synchronisation).
  bool launch(const DevBatch& b, const DevMatches& m, hipStream_t stream, std::string& err);

  // After the pass: copies the match lists to host in (package, advisory) order.
  // Returns false when the device buffer was too small (total > m.cap).
  static bool fetch_ordered(const DevMatches& m, uint32_t n_pkgs, uint64_t total, std::vector<uint2>& out,
                            std::string& err);

  // Convenience: upload, match, download. out = pairs; err_pkg = first poisoned package or -1.
  bool match_host(const HostBatch& hb, std::vector<uint2>& out, int64_t& err_pkg, std::string& err);

  const DB& db() const { return *db_; }

  // Kernel variant (tile size / LDS budget); returns the previous one.  Default 0 =
  // "auto" (the tuned variant for the batch's grammar set), overridable with the
  // TVM_VARIANT environment variable at open().
  int set_variant(int v);
  // Variant index of the most recent launch (auto resolved), -1 before the first.
  int last_launched() const { return last_launched_; }
  // Integrity check: the device tables still equal the host images (bytes compared).
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
  // per-launch scratch
  uint64_t* spill_ = nullptr;
  uint64_t spill_cap_ = 0;
  std::mutex call_mu_;  // serialises host-synchronous calls sharing the scratch buffers
  bool ensure_scratch(uint64_t spill_words, std::string& err);
};

// Kernel variants: count and names (engine.hip; 0 = "auto").
int num_variants();
const char* variant_name(int v);
// The variant "auto" (0) resolves to for a batch of grammar bits gm; other v unchanged.
int resolve_variant(int v, uint32_t gm);

}  // namespace tvm
