// Vulnerability-detail join (FillInfo) on the GPU: load-time tables + kernel interface.
//
// Replaces the per-match work of the reference's pkg/vulnerability/vulnerability.go:
//   :60-109   Client.FillInfo   - status rule, trivy-db GetVulnerability(vulnID) (a bbolt
//                                 lookup + JSON decode per detected vulnerability), the
//                                 detector's package-specific severity override
//   :111-134  getVendorSeverity - data source -> GHSA (for GHSA- IDs) -> NVD -> DB severity
//   :136-157  getPrimaryURL     - ID-prefix URLs, else the first reference matching the
//                                 data source's prefixes (:15-39)
//
// At load time bucket "vulnerability" is decoded once (json.Unmarshal into trivy-db
// types.Vulnerability semantics) into a hash index on the vulnerability ID, one 16-B
// record per vulnerability and a small entry list per vulnerability holding its
// VendorSeverity pairs and, for IDs without a URL prefix rule, the reference index the
// primary-URL rule picks for each data source that has prefixes.  The kernel then does,
// per detected vulnerability, one hash probe + record + entry scan and writes a 16-B
// decision; strings (detail JSON, URLs) are rebuilt on the host from the decision.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace tvm {

class DB;
struct Advisory;

// Decision codes written by the kernel.
enum : uint32_t {
  FILL_NOT_FOUND = 0xFFFFFFFFu,  // out.x: GetVulnerability failed (missing key or decode error)
  SEV_KEEP = 0xFFFDu,            // severity = the detector's (package-specific) severity
  SEV_RAW = 0xFFFEu,             // severity = the DB's Vulnerability.Severity string verbatim
  SEV_OOR = 0xFFFFu,             // a VendorSeverity value outside SeverityNames (reported as UNKNOWN)
  SRC_NONE = 0xFFFFu,            // severity source ""
  URL_NONE = 0, URL_CVE = 1, URL_RUSTSEC = 2, URL_GHSA = 3, URL_TEMP = 4, URL_REF = 5,
  URL_KIND_SHIFT = 28, URL_REF_MASK = 0x0FFFFFFFu,
  // item flags (FillItem.z bits 8..15)
  FI_FIXED = 1u << 8,            // FixedVersion != ""
  FI_SEV_SRC = 1u << 9,          // the detector set SeveritySource
  // entry word: kind (bit 31) | source id (bits 16..30) | value (bits 0..15)
  ENT_URL = 1u << 31,
};

// Per-item input (16 B): x = vuln-ID offset into the item arena, y = ID length | source
// id << 16, z = status | FI_* flags, w = resolved vulnerability record or FILL_NOT_FOUND
// (batch path; the drop-in path probes and ignores w).
// Per-item output (16 B): x = record index or FILL_NOT_FOUND, y = status,
// z = severity code (0..4 = SeverityNames, SEV_*) | severity source id << 16,
// w = URL kind << 28 | reference index.
// Record (16 B): x = first entry, y = entry count, z = DB severity code (0..4 or
// SEV_RAW), w = REC_BAD | ID-prefix URL kind << REC_URL_SHIFT.
enum : uint32_t { REC_BAD = 1, REC_URL_SHIFT = 4 };

// Host view of one decoded vulnerability (trivy-db types.Vulnerability).
struct VulnDetail {
  std::string id;
  std::string severity;                                  // Vulnerability.Severity
  std::vector<std::pair<std::string, int64_t>> vendor;   // VendorSeverity, key order
  std::vector<std::string> refs;                         // References
  std::string detail_json;                               // canonical JSON of the whole record
  bool bad = false;                                      // GetVulnerability would fail
};

class VulnTable {
 public:
  // Decodes bucket "vulnerability" of the DB's tree and builds the device images.
  void build(const DB& db);
  bool built() const { return built_; }

  // Source-ID dictionary (VendorSeverity keys, primary-URL sources, data sources).
  uint32_t source_id(std::string_view s) const;  // SRC_NONE when unknown
  const std::string& source_name(uint32_t id) const {
    static const std::string none;
    return id < src_names_.size() ? src_names_[id] : none;
  }
  uint32_t ghsa_id() const { return ghsa_; }
  uint32_t nvd_id() const { return nvd_; }
  int32_t find(std::string_view vuln_id) const;  // host lookup, -1 when absent

  // Host rebuild of the strings behind a kernel decision (record rec):
  //   the Vulnerability JSON with Severity = severity and VendorSeverity plus, when
  //   extra_src is non-empty, VendorSeverity[extra_src] = extra_val (vulnerability.go:95-101);
  std::string vulnerability_json(uint32_t rec, std::string_view severity, std::string_view extra_src,
                                 int64_t extra_val) const;
  //   PrimaryURL from the URL word (kind << 28 | reference index) and the vulnerability ID.
  std::string primary_url(uint32_t rec, uint32_t url_word) const;
  //   Severity string of a severity code (0..4, SEV_RAW, SEV_OOR; SEV_KEEP is the caller's).
  const std::string& severity_string(uint32_t rec, uint32_t code) const;

  std::vector<VulnDetail> vulns;

  // ---- device images ----
  std::vector<uint64_t> slot_hash;   // 0 = empty; key_hash(kVulnSeed, id)
  std::vector<uint4> slot_val;       // {id_off, id_len, record, 0}
  std::vector<uint8_t> id_arena;     // 8-B aligned IDs, zero padded (+4 zero words)
  std::vector<uint4> recs;           // {entry_off, entry_n, db severity code, REC_BAD | url kind}
  std::vector<uint32_t> ents;        // ENT_* words
  uint64_t slot_mask = 0;

  // Batch path: per advisory of the DB, the FillInfo input its detector output carries
  // (uint4 as the item layout: record in w, source in y >> 16, the detector's
  // package-specific severity index in y & 0xFF (0xFF = none)).
  std::vector<uint4> adv_items;
  // Batch filter (result.Filter): per advisory {rank of its vulnerability ID among all
  // advisory IDs, rank of its output FixedVersion among all output FixedVersions}, both
  // in byte order (Go string order), and the ID -> rank map for ignore files.
  std::vector<uint2> adv_rank;
  uint32_t vuln_rank(std::string_view id) const;  // 0xFFFFFFFF when no advisory has it
  uint32_t n_vuln_ranks() const { return uint32_t(rank_names_.size()); }

 private:
  bool built_ = false;
  std::unordered_map<std::string, uint32_t> src_ids_;
  std::vector<std::string> src_names_;
  std::unordered_map<std::string_view, int32_t> by_id_;
  std::vector<std::string> rank_names_;                      // owns the keys of vuln_rank_
  std::unordered_map<std::string_view, uint32_t> vuln_rank_;  // no allocation per lookup
  uint32_t ghsa_ = SRC_NONE, nvd_ = SRC_NONE;
  uint32_t intern_source(const std::string& s);
};

constexpr uint32_t kVulnSeed = 0x7F11A0u;  // key_hash seed of the vulnerability-ID index

// The FillInfo inputs a detector's output for (package, advisory a of a platform of
// driver family drv) carries (drivers.cpp; the fields each driver's Detect copies).
struct DetFill {
  int32_t data_source = -1;       // index into DB::sources, -1 = nil
  int64_t status = 0;
  bool fixed = false;             // FixedVersion != ""
  const char* severity_source = nullptr;
  const char* severity = nullptr;
  std::string fixed_version;      // the output FixedVersion
};
void detector_fill_fields(uint8_t drv, const Advisory& a, DetFill& f);

// Severity names (trivy-db SeverityNames) and NewSeverity.
const char* fill_severity_name(int64_t s);
int64_t fill_new_severity(std::string_view s);

// Device side (fill.hip).
struct FillDev {
  const uint64_t* slot_hash;
  const uint4* slot_val;
  uint64_t slot_mask;
  const uint8_t* id_arena;
  const uint4* recs;
  const uint32_t* ents;
  const uint4* adv_items;
  const uint2* adv_rank;
  uint32_t n_advs;
  uint32_t ghsa, nvd;
};
// Severity index of a batch pair after FillInfo, as filterVulnerabilities reads it (0..4;
// 5 = a DB string outside SeverityNames, which no severity filter passes).  d = the fill
// decision, it = the advisory's item.
__host__ __device__ inline uint32_t fill_pair_severity(uint4 d, uint4 it) {
  const uint32_t det = it.y & 0xFFu;  // the detector's package-specific severity (0xFF none)
  if (d.x == FILL_NOT_FOUND) return (it.z & FI_SEV_SRC) && det < 5 ? det : 0u;  // unchanged; "" -> UNKNOWN
  const uint32_t code = d.z & 0xFFFFu;
  if (code < 5) return code;
  if (code == SEV_KEEP) return det < 5 ? det : 0u;
  if (code == SEV_RAW) return 5u;
  return 0u;  // SEV_OOR prints UNKNOWN
}

class FillEngine {
 public:
  ~FillEngine();
  static FillEngine* open(const VulnTable& t, int device, std::string& err);
  // Drop-in path: items (vuln IDs in `arena`) -> decisions, host in / host out.
  bool run_host(const std::vector<uint4>& items, const std::vector<uint8_t>& arena, std::vector<uint4>& out,
                std::string& err);
  // Batch path: decisions for the device match pairs {pkg, adv} (resolved records), on
  // `stream`; the pair count is read from n_dev on the device (at most cap pairs).
  // side (optional): per pair the filter's hand-off word {vulnerability-ID rank, severity
  // index | status << 8} (filter.hip reads it instead of the 16-B decision).
  // base (optional, merged Red Hat lists): per pair the member that supplies Status /
  // Severity; adv then only decides FixedVersion != "".
  bool launch_pairs(const uint32_t* adv, const uint32_t* base, const unsigned long long* n_dev, uint64_t cap,
                    uint4* out, uint2* side, hipStream_t stream, std::string& err);
  uint64_t table_bytes() const { return table_bytes_; }
  const VulnTable& table() const { return *t_; }
  // Algorithmic HBM bytes of one batch-path launch over these pairs (host copy).
  uint64_t pair_bytes(const std::vector<uint32_t>& adv, const std::vector<uint32_t>& base) const;
  const FillDev& dev() const { return *d_; }
  int device() const { return dev_; }

 private:
  int dev_ = 0;
  const VulnTable* t_ = nullptr;
  FillDev* d_ = nullptr;
  std::vector<void*> allocs_;
  uint64_t table_bytes_ = 0;
  hipStream_t stream_ = nullptr;
};

// result.Filter over a batch's device match list (filter.hip).
// Per package, fixed once per batch (host): the report order of the packages and the groups
// the filter compares them in.
struct FilterPackages {
  std::vector<uint32_t> perm;          // packages by (result, PkgName, InstalledVersion, PkgPath, index)
  std::vector<uint32_t> grp_b, grp_e;  // per package: perm range of its (result, PkgName, InstalledVersion)
  std::vector<uint32_t> dkey;          // per package: id of its (result, PkgName, InstalledVersion, PkgPath)
  std::vector<uint32_t> prank;         // per package: rank of its PkgPath inside its group
  std::vector<uint8_t> dup;            // per package: another package shares its dkey
};

// Host-compiled rules of one call, as the caller's arrays: list k holds n entries (subject
// = package or class, index into its ID-rank table, precedence); the device builds the
// hash-set keys tag << 62 | subject << 32 | vulnerability rank (subject < 2^30) and
// inserts them, keeping the smallest precedence per key.
enum : uint64_t { RULE_ALL = 0, RULE_PKG = 1, RULE_CLS = 2, RULE_VEX = 3 };
struct RuleList {
  uint64_t tag = 0;
  const uint32_t* subject = nullptr;  // nullptr: subject 0 (RULE_ALL)
  const uint32_t* id = nullptr;
  const uint32_t* prec = nullptr;     // nullptr: 0 (VEX)
  uint64_t n = 0;
  int table = 0;                      // 0: ignore-file ID ranks, 1: VEX ID ranks
};
struct FilterRules {
  RuleList lists[4];
  int n_lists = 0;
  std::vector<uint32_t> rank[2];     // ID index -> vulnerability rank (0xFFFFFFFF unknown)
  const uint32_t* pkg_class = nullptr;  // per package (nullptr: no class rules)
  uint32_t kinds = 0;                // bit k: some rule of tag k
  uint64_t size() const {
    uint64_t t = 0;
    for (int k = 0; k < n_lists; k++) t += lists[k].n;
    return t;
  }
};

class BatchFilter {
 public:
  ~BatchFilter();
  bool set_packages(const FilterPackages& fp, std::string& err);
  bool has_packages() const { return n_pkgs_ != 0; }
  void reset_packages() { n_pkgs_ = 0; }
  // Filters the n device pairs (with their FillInfo decisions) on `st`; synchronises once, at
  // the end, to learn the counts.
  bool run(const FillDev& t, const uint32_t* pkg, const uint32_t* adv, const uint2* side, uint64_t n,
           const FilterRules& rules, uint32_t n_ranks, uint32_t sev_mask, uint32_t status_mask, hipStream_t st,
           std::string& err);
  uint64_t survivors() const { return survivors_; }
  uint64_t ignored() const { return ignored_; }
  // The surviving {package, advisory} pairs in report order.
  bool fetch(std::vector<uint2>& out, hipStream_t st, std::string& err);
  // The ignored {package, advisory, precedence} in detection order.
  bool fetch_ignored(std::vector<uint32_t>& out3, hipStream_t st, std::string& err);

 private:
  enum { kBufs = 29 };
  void* bufs_[kBufs] = {};
  uint64_t caps_[kBufs] = {};
  uint64_t n_ = 0, survivors_ = 0, ignored_ = 0, n_pkgs_ = 0;
  void* pin_ = nullptr;  // pinned staging of the per-call rule upload
  uint64_t pin_cap_ = 0;
  bool grow(int i, uint64_t need, std::string& err);
};

}  // namespace tvm
