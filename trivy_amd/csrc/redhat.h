// Red Hat per-CVE merge of a batch's match list on the device (redhat.hip;
// pkg/detector/ospkg/redhat/redhat.go:146-187).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "common.h"
#include "engine.h"

namespace tvm {

constexpr uint32_t RH_NONE = 0xFFFFFFFFu;

// One merged vulnerability of one package: the group of the package's matches that share a
// VulnerabilityID.  base = the first member (Get order: Status, Severity, Custom); best =
// the member with the greatest fixed version (RH_NONE: all unfixed); members = positions
// [start, start + len) of the raw match list (contrib[i] = advisory at raw position i).
struct RhRec {
  uint32_t pkg, base, best, start, len;
  uint32_t pad[3];
};

// The merged match list, device resident, in the layout of DevMatches (tile directory +
// columns + control block) so that FillInfo, result.Filter and the ordered fetch read it
// like a raw list.  Per entry: pkg, adv = the representative advisory (best when a member
// is fixed, else base: its FixedVersion is the merged FixedVersion), base = the first
// member, grp = {raw position of the first member, member count}.  Pairs of packages of
// other drivers pass through as groups of one (adv = base).
struct RhMerged {
  DevMatches m;          // m.pkg / m.adv / m.dir / m.ctl ([0] entries, [3] error bits)
  uint32_t* base = nullptr;
  uint2* grp = nullptr;
  uint64_t cap = 0;
};
enum : uint32_t { ERR_RH_ORDER = 4 };  // a Red Hat package's IDs were not grouped (load-time order broken)

struct RhInputs {
  const uint2* pk;                  // device batch packages
  const PlatInfo* plats;
  uint32_t n_plats;
  const DevMatches* raw;            // the match kernel's list
  uint32_t n_tiles;
  uint32_t n;                       // packages in the batch (tile t = packages [256 t, 256 t + 256))
  uint32_t pkg_base;
  const uint2* rk;                  // per advisory {vulnerability-ID rank, rpm order rank of FixedVersion (RH_NONE = unfixed)}
};

class RedHatMerge {
 public:
  ~RedHatMerge();
  // Enqueues the merge on `st` (no host synchronisation); the result stays in merged().
  bool launch(const RhInputs& in, hipStream_t st, std::string& err);
  const RhMerged& merged() const { return out_; }
  // Which of the batch's tiles hold Red Hat packages (flags[t] = 1), computed on the host
  // once per upload (the caller holds the packages' platforms): the merge's kernels give those
  // tiles a workgroup each and pass the others' pairs through a wave per tile.
  bool set_tiles(const std::vector<uint8_t>& flags, std::string& err);
  bool tiles_known() const { return tiles_known_; }
  void forget_tiles() { tiles_known_ = false; }  // the batch's packages changed (a new upload)
  // After launch: the merged list in (package, VulnerabilityID) order as host columns
  // (pkg, adv, base, grp) and the raw list's advisory column in raw positions (contrib);
  // synchronises `st`.  grp is defined for the entries of Red Hat packages (the groups).
  bool fetch(const RhInputs& in, std::vector<uint32_t>& pkg, std::vector<uint32_t>& adv, std::vector<uint32_t>& base,
             std::vector<uint2>& grp, std::vector<uint32_t>& contrib, hipStream_t st, std::string& err);

 private:
  int dev_ = -1;
  RhMerged out_;
  uint32_t* counts_ = nullptr;            // per tile: merged entries (rh_count_kernel)
  unsigned long long* bases_ = nullptr;   // per tile: output base (exclusive scan of counts_)
  // the batch's tiles (set_tiles): per tile 1 = holds Red Hat packages, and their list
  uint8_t* flags_ = nullptr;
  uint32_t* rh_list_ = nullptr;
  uint32_t n_rh_ = 0;
  size_t flags_cap_ = 0;
  int tiles_dev_ = -1;
  bool tiles_known_ = false;
  void* scan_tmp_ = nullptr;              // the scan's temporary storage
  size_t scan_tmp_bytes_ = 0;
  void release();
};

}  // namespace tvm
