// Red Hat per-CVE merge of a batch's match list (redhat.hip; redhat.go:146-187).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

namespace tvm {

constexpr uint32_t RH_NONE = 0xFFFFFFFFu;

// One merged vulnerability of one package: the group of the package's matches that share a
// VulnerabilityID.  base = the first member (Get order: Status, Severity, Custom); best =
// the member with the greatest fixed version (RH_NONE: all unfixed); members = sorted
// positions [start, start + len) of the contrib array.
struct RhRec {
  uint32_t pkg, base, best, start, len;
  uint32_t pad[3];
};

struct RhInputs {
  const uint2* pk;                  // device batch packages
  const PlatInfo* plats;
  uint32_t n_plats;
  const uint32_t* pkg;              // device match columns
  const uint32_t* adv;
  const unsigned long long* n_dev;  // device match count
  uint64_t n_matches;               // host copy (the buffers' valid length)
  uint32_t pkg_base;
  const uint2* adv_rank;            // FillDev::adv_rank (.x vulnerability-ID rank)
  const uint32_t* fixed_rank;       // per advisory: rpm order rank of FixedVersion, RH_NONE = unfixed
};

class RedHatMerge {
 public:
  ~RedHatMerge();
  // records in (package, VulnerabilityID) order; contrib[i] = advisory at sorted position i
  bool run(const RhInputs& in, std::vector<RhRec>& recs, std::vector<uint32_t>& contrib, hipStream_t st,
           std::string& err);

 private:
  void* bufs_[10] = {};
  size_t caps_[10] = {};
  bool grow(int i, size_t need, std::string& err);
};

}  // namespace tvm
