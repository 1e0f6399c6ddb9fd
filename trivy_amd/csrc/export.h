// DetectedVulnerability sets of a batch (export.hip; the C-ABI's tvm_match_vulns).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "common.h"
#include "engine.h"

namespace tvm {

// A device match list in the tile-directory layout (DevMatches: dir, pkg, adv, ctl), the
// batch's raw one or the Red Hat-merged one (rh = true: base / grp columns and the raw list's
// advisory column, which holds the groups' members).
struct ExportList {
  DevMatches list;
  uint64_t total = 0;
  uint32_t n_tiles = 0;
  uint32_t pkg_base = 0;
  bool rh = false;
  const uint32_t* base = nullptr;  // merged: the first member of each entry
  const uint2* grp = nullptr;      // merged: {raw position of the first member, member count}
  const uint32_t* raw_adv = nullptr;
  uint64_t raw_cap = 0;
  const uint2* pk = nullptr;       // the batch's package words (platform per package)
  const PlatInfo* plats = nullptr;
  uint32_t n_plats = 0;
};

// The set as it arrives in pinned host memory: per package (tile-padded) its row end, per
// match its record index as `width` (3 or 4) little-endian bytes - the advisory, or n_adv + k
// for the k-th Red Hat group of several members, groups[k] = {merged position, package, first
// member, representative} with its members at members[moff[k] .. moff[k + 1]).
struct VulnExport {
  uint32_t* row_end_h = nullptr;
  uint8_t* rec_h = nullptr;
  uint32_t width = 4;
  uint64_t n = 0;
  uint32_t n_groups = 0;
  std::vector<uint4> groups;
  std::vector<uint32_t> moff;
  std::vector<uint32_t> members;
  uint32_t* moff_h(uint32_t n_groups) {
    moff.assign(size_t(n_groups) + 1, 0);
    return moff.data();
  }
  ~VulnExport();
};

// Enqueues and runs the export of a completed pass's list on stream `st` (synchronised).
bool export_vulns(int dev, hipStream_t st, const ExportList& in, uint32_t n_adv, VulnExport& out, std::string& err);

}  // namespace tvm
