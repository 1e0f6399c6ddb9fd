// Red Hat per-CVE merge over a batch's match list on the GPU (gfx950): the batch form of
// the uniqVulns loop of pkg/detector/ospkg/redhat/redhat.go:146-187.
//
// For one package the reference walks its advisories in trivy-db Get order and keys them by
// VulnerabilityID: an unfixed advisory enters only if the ID is new (first seen wins); a
// fixed one (installed < fixed) enters, or merges into the existing entry - VendorIDs
// unioned (ustrings.Unique), FixedVersion raised to the greater rpm version - and the
// result is sorted by VulnerabilityID.  Here, over every (package, advisory) pair of the
// batch's Red Hat packages at once:
//   rh_keys    key = package << 32 | vulnerability-ID rank (byte order = Go string order);
//              pairs of other drivers get the all-ones key (they sort last, no group);
//   radix sort (hipcub, stable: equal keys keep the match list's per-package Get order);
//   rh_heads   a group starts where the key changes;
//   select     group heads in order (hipcub DeviceSelect::Flagged);
//   rh_records per group: the first member (Status / Severity / Custom), the member with the
//              greatest fixed version (rpm order rank computed at load time; ties keep the
//              first, as LessThan does), the members' range (the host unions their VendorIDs).
// Integer / byte work bound by memory traffic: no MFMA.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <string>

#include "redhat.h"

namespace tvm {

namespace {

constexpr int kBlock = 256;
constexpr unsigned long long kNone = ~0ull;

struct MergeArgs {
  const uint2* pk;             // batch packages {plat, lengths}
  const PlatInfo* plats;
  uint32_t n_plats;
  const uint32_t* pkg;         // match columns
  const uint32_t* adv;
  const unsigned long long* n_dev;  // match count (device)
  uint64_t cap;
  uint32_t pkg_base;
  const uint2* adv_rank;       // .x = vulnerability-ID rank
  const uint32_t* fixed_rank;  // rpm order rank of the advisory's fixed version, kNoFix = unfixed
  unsigned long long* keys;
  uint32_t* idx;
  const unsigned long long* skeys;
  const uint32_t* sidx;
  uint8_t* flags;
  const uint32_t* heads;
  const uint32_t* n_heads;
  RhRec* recs;
  uint32_t* contrib;           // advisory of every sorted position
};

__global__ __launch_bounds__(kBlock) void rh_keys(MergeArgs a) {
  const uint64_t n = *a.n_dev < a.cap ? *a.n_dev : a.cap;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.cap; i += stride) {
    unsigned long long k = kNone;
    if (i < n) {
      const uint32_t p = a.pkg[i], ad = a.adv[i];
      const uint32_t plat = a.pk[p - a.pkg_base].x;
      if (plat < a.n_plats && a.plats[plat].drv == DRV_REDHAT) k = (uint64_t(p) << 32) | a.adv_rank[ad].x;
    }
    a.keys[i] = k;
    a.idx[i] = uint32_t(i);
  }
}

__global__ __launch_bounds__(kBlock) void rh_heads(MergeArgs a) {
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.cap; i += stride) {
    const unsigned long long k = a.skeys[i];
    a.flags[i] = k != kNone && (i == 0 || a.skeys[i - 1] != k);
    a.contrib[i] = a.adv[a.sidx[i]];
  }
}

__global__ __launch_bounds__(kBlock) void rh_records(MergeArgs a) {
  const uint32_t nh = *a.n_heads;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t h = uint64_t(blockIdx.x) * kBlock + threadIdx.x; h < nh; h += stride) {
    const uint32_t s = a.heads[h];
    const unsigned long long k = a.skeys[s];
    const uint32_t base = a.contrib[s];
    uint32_t best = RH_NONE, best_r = 0, j = s;
    for (; j < a.cap && a.skeys[j] == k; j++) {
      const uint32_t ad = a.contrib[j];
      const uint32_t r = a.fixed_rank[ad];
      if (r != RH_NONE && (best == RH_NONE || r > best_r)) {
        best = ad;
        best_r = r;
      }
    }
    RhRec o;
    o.pkg = uint32_t(k >> 32);
    o.base = base;
    o.best = best;
    o.start = s;
    o.len = j - s;
    o.pad[0] = o.pad[1] = o.pad[2] = 0;
    a.recs[h] = o;
  }
}

bool ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

}  // namespace

RedHatMerge::~RedHatMerge() {
  for (void* p : bufs_)
    if (p) (void)hipFree(p);
}

bool RedHatMerge::grow(int i, size_t need, std::string& err) {
  if (caps_[i] >= need) return true;
  if (bufs_[i]) (void)hipFree(bufs_[i]);
  bufs_[i] = nullptr;
  caps_[i] = 0;
  if (!ok(hipMalloc(&bufs_[i], std::max<size_t>(need, 1)), "hipMalloc(redhat merge)", err)) return false;
  caps_[i] = need;
  return true;
}

bool RedHatMerge::run(const RhInputs& in, std::vector<RhRec>& recs, std::vector<uint32_t>& contrib, hipStream_t st,
                      std::string& err) {
  recs.clear();
  contrib.clear();
  const uint64_t cap = in.n_matches;
  if (cap == 0) return true;
  if (cap > 0x7FFFFFFFull) {
    err = "redhat merge: too many matches";
    return false;
  }
  size_t sort_bytes = 0, sel_bytes = 0;
  if (!ok(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, static_cast<unsigned long long*>(nullptr),
                                             static_cast<unsigned long long*>(nullptr), static_cast<uint32_t*>(nullptr),
                                             static_cast<uint32_t*>(nullptr), int(cap), 0, 64, st),
          "hipcub sort sizing", err) ||
      !ok(hipcub::DeviceSelect::Flagged(nullptr, sel_bytes, hipcub::CountingInputIterator<uint32_t>(0),
                                        static_cast<const uint8_t*>(nullptr), static_cast<uint32_t*>(nullptr),
                                        static_cast<uint32_t*>(nullptr), int(cap), st),
          "hipcub select sizing", err))
    return false;
  // 0 keys, 1 idx, 2 sorted keys, 3 sorted idx, 4 flags, 5 heads, 6 head count, 7 records, 8 contrib, 9 temp
  if (!grow(0, cap * 8, err) || !grow(1, cap * 4, err) || !grow(2, cap * 8, err) || !grow(3, cap * 4, err) ||
      !grow(4, cap, err) || !grow(5, cap * 4, err) || !grow(6, 4, err) || !grow(7, cap * sizeof(RhRec), err) ||
      !grow(8, cap * 4, err) || !grow(9, std::max(sort_bytes, sel_bytes), err))
    return false;
  MergeArgs a{};
  a.pk = in.pk;
  a.plats = in.plats;
  a.n_plats = in.n_plats;
  a.pkg = in.pkg;
  a.adv = in.adv;
  a.n_dev = in.n_dev;
  a.cap = cap;
  a.pkg_base = in.pkg_base;
  a.adv_rank = in.adv_rank;
  a.fixed_rank = in.fixed_rank;
  a.keys = static_cast<unsigned long long*>(bufs_[0]);
  a.idx = static_cast<uint32_t*>(bufs_[1]);
  a.skeys = static_cast<unsigned long long*>(bufs_[2]);
  a.sidx = static_cast<uint32_t*>(bufs_[3]);
  a.flags = static_cast<uint8_t*>(bufs_[4]);
  a.heads = static_cast<uint32_t*>(bufs_[5]);
  a.n_heads = static_cast<uint32_t*>(bufs_[6]);
  a.recs = static_cast<RhRec*>(bufs_[7]);
  a.contrib = static_cast<uint32_t*>(bufs_[8]);
  const uint32_t blocks = uint32_t(std::min<uint64_t>((cap + kBlock - 1) / kBlock, 256ull * 32));
  hipLaunchKernelGGL(rh_keys, dim3(blocks), dim3(kBlock), 0, st, a);
  if (!ok(hipGetLastError(), "rh_keys", err) ||
      !ok(hipcub::DeviceRadixSort::SortPairs(bufs_[9], sort_bytes, a.keys, static_cast<unsigned long long*>(bufs_[2]),
                                             a.idx, static_cast<uint32_t*>(bufs_[3]), int(cap), 0, 64, st),
          "hipcub sort", err))
    return false;
  hipLaunchKernelGGL(rh_heads, dim3(blocks), dim3(kBlock), 0, st, a);
  if (!ok(hipGetLastError(), "rh_heads", err) ||
      !ok(hipcub::DeviceSelect::Flagged(bufs_[9], sel_bytes, hipcub::CountingInputIterator<uint32_t>(0), a.flags,
                                        static_cast<uint32_t*>(bufs_[5]), static_cast<uint32_t*>(bufs_[6]), int(cap),
                                        st),
          "hipcub select", err))
    return false;
  hipLaunchKernelGGL(rh_records, dim3(blocks), dim3(kBlock), 0, st, a);
  uint32_t nh = 0;
  if (!ok(hipGetLastError(), "rh_records", err) ||
      !ok(hipMemcpyAsync(&nh, bufs_[6], 4, hipMemcpyDeviceToHost, st), "D2H head count", err) ||
      !ok(hipStreamSynchronize(st), "redhat merge", err))
    return false;
  recs.resize(nh);
  contrib.resize(cap);
  return (!nh || ok(hipMemcpyAsync(recs.data(), bufs_[7], nh * sizeof(RhRec), hipMemcpyDeviceToHost, st),
                    "D2H records", err)) &&
         ok(hipMemcpyAsync(contrib.data(), bufs_[8], cap * 4, hipMemcpyDeviceToHost, st), "D2H contrib", err) &&
         ok(hipStreamSynchronize(st), "redhat merge", err);
}

}  // namespace tvm
