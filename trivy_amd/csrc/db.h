// Load-time flattener: trivy-db bucket tree -> columnar tables for HBM.
//
// Replaces the per-call trivy-db lookups of the reference (db.Config.GetAdvisories /
// <os>.VulnSrc.Get, called from pkg/detector/ospkg/*/ *.go and
// pkg/detector/library/driver.go:114) with one pass at load time, at the point where
// the reference opens the DB (pkg/commands/artifact/run.go:311 db.Init).
//
// Input: the bucket tree as (path..., key) -> JSON value records, exactly what a bbolt
// walk (or bolt-fixtures YAML) produces.  Output: the device images below.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace tvm {

struct DataSource {
  std::string id, name, url;
  bool empty() const { return id.empty() && name.empty() && url.empty(); }
};

// One advisory as the reference driver sees it after trivy-db's Get: trivy-db
// pkg/types.Advisory for most sources; for Red Hat one record per (entry, CVE) of the
// redhat-oval value, for Rocky one per arch entry.
struct Advisory {
  std::string vuln_id;                 // from the bucket key (or the CVE of a Red Hat entry)
  std::vector<std::string> vendor_ids;
  std::vector<std::string> arches;
  int64_t status = 0;
  int64_t severity = 0;
  std::string fixed, affected;
  std::vector<std::string> vulnerable, patched, unaffected;
  int32_t data_source = -1;            // index into DB::sources, -1 = nil
  std::string custom;                  // raw JSON text of Custom, "" = nil
  bool has_inline_source = false;      // DataSource present in the value JSON itself
  DataSource inline_source;
  std::vector<Advisory> entries;       // Rocky: per-arch entries (types.Advisory.Entries)
  std::vector<int64_t> cpes;           // Red Hat: the entry's affected CPE indices
  bool arch_entry = false;             // Rocky: expanded from an arch entry (arch must be listed)
  std::string lib_fixed;               // library: createFixedVersions (driver.go:139-159)
};

// Library ecosystems: trivy-db bucket prefix (ecosystem) and the grammar its comparer
// uses (driver.go:25-93); CMP_NONE when no LangType maps to it.
uint8_t ecosystem_grammar(std::string_view eco);
// createFixedVersions (driver.go:139-159).
std::string create_fixed_versions(const Advisory& a);

// Decodes one advisory value (Go json.Unmarshal into types.Advisory).
bool decode_advisory(std::string_view json, Advisory& a, std::string& err);

struct Bucket {
  std::map<std::string, Bucket> sub;        // nested buckets (byte order = bbolt order)
  std::map<std::string, std::string> kv;    // key -> JSON value
};

struct Platform {
  std::string name;   // root bucket name
  uint8_t drv = DRV_NONE;
  uint8_t cmp = CMP_NONE;
  uint32_t flags = 0;
};

struct Key {
  uint32_t plat;
  std::string name;
  std::vector<uint32_t> advs;  // advisory indices, bbolt key (vulnID) order
  bool poisoned = false;
  std::string err;
};

class DB {
 public:
  // ---- intake (before finalize) ----
  void put(const std::vector<std::string>& path, std::string_view value);
  // Decode + flatten; false on a structural error.
  bool finalize(std::string& err);

  // ---- flattened host view ----
  std::vector<Platform> plats;
  std::vector<Key> keys;
  std::vector<Advisory> advs;
  std::vector<DataSource> sources;
  int32_t find_plat(std::string_view root) const;
  // Host-side lookup of a key index (used by drivers for error text); -1 if absent.
  int32_t find_key(uint32_t plat, std::string_view name) const;
  // Interval rows of key (plat, name) in the device tables (0: no key) - the host pre-probe of
  // a package's work (multi-GPU shard balance, heavy-first tile order).
  uint32_t key_rows(uint32_t plat, std::string_view name) const;

  // Red Hat CPE resolution (trivy-db RedHatRepoToCPEs / RedHatNVRToCPEs): the unique CPE
  // indices of content sets + NVRs, in first-seen order.
  std::vector<int64_t> redhat_cpes(const std::vector<std::string_view>& repos,
                                   const std::vector<std::string_view>& nvrs) const;
  uint32_t n_cpe = 0;  // 1 + the largest CPE index anywhere (bitset width)
  // Arch / ksplice dictionaries for package attributes (PA_* in common.h).
  uint32_t arch_id(std::string_view arch) const;    // PA_ARCH_NONE when no advisory lists it
  uint32_t ksplice_id(std::string_view tag) const;  // 0 for "", 0xFFFFFFFF when unknown

  // ---- device images ----
  std::vector<uint64_t> slot_hash;
  std::vector<SlotVal> slot_val;
  std::vector<Slot> slots;          // device probe table (common.h Slot), same positions
  std::vector<uint8_t> slot_fp;     // device: per slot slot_fp_of(hash), 0 = empty (common.h)
  std::vector<uint32_t> slot_key;   // host only: slot -> Key index
  std::vector<uint8_t> name_arena;
  std::vector<Row> rows;
  std::vector<RowOff> row_off;  // parallel to rows (the dpkg grammar's rows keep their offsets here only)
  std::vector<RowAux> aux;          // parallel to rows (read only for ROW_FILTER rows)
  std::vector<uint32_t> aux_ids;
  std::vector<uint64_t> key_words;
  std::vector<PlatInfo> plat_info;
  uint64_t slot_mask = 0;
  uint64_t n_rows_total = 0;
  bool has_filters = false;

  const Bucket& tree() const { return root_; }

 private:
  Bucket root_;
  std::unordered_map<std::string, uint32_t> plat_by_name_;
  std::unordered_map<std::string, uint32_t> key_dedup_;  // encoded key bytes -> word offset
  std::unordered_map<std::string, std::vector<int64_t>> rh_repo_, rh_nvr_;
  std::unordered_map<std::string, uint32_t> arch_ids_, ksplice_ids_;
  uint32_t intern_key(const std::vector<uint8_t>& k);
  uint32_t intern_arch(const std::string& a);
  void flatten_os(uint32_t plat, const Bucket& b, int32_t ds);
  void flatten_library(uint32_t plat, const std::vector<std::pair<const Bucket*, int32_t>>& roots);
  bool compile_rows(const Platform& P, const Advisory& a, uint32_t ai, std::vector<uint8_t>& kb);
  static constexpr uint32_t kRowSplit = 1u << 31;  // split_by_class's mark on a packed count
  static constexpr uint32_t kRowsPerLine = 4;       // 32-B rows per 128-B line (a key's run starts on one)
  void split_by_class(const Platform& P, uint32_t row_begin, uint32_t& row_count);
  void build_index();
};

// Classifies a root bucket name into a driver family (OS buckets only).
bool classify_os_bucket(std::string_view root, uint8_t& drv, uint8_t& cmp, uint32_t& flags);

// oracle.go:101-109 extractKsplice: the lower-cased dot-segment starting "ksplice", or "".
std::string extract_ksplice(std::string_view v);

}  // namespace tvm
