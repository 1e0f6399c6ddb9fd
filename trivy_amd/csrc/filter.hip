// result.Filter for a batch of results on the GPU (gfx950): the vulnerability part of
// pkg/result/filter.go:60-139 over a batch's device match list, after FillInfo.
//
// Reference semantics per Result (= one tvm_batch_add* call):
//   filter.go:104-114   drop by severity ("" counts as UNKNOWN) and by ignored status;
//   filter.go:117-122   drop vulnerabilities whose ID the ignore file lists;
//   filter.go:124-130   dedup on "vulnID/pkgName/installed/pkgPath": the greater
//                       FixedVersion string wins (shouldOverwrite, :345-348), ties keep
//                       the first seen;
//   filter.go:77        sort.Sort(types.BySeverity) (pkg/types/vulnerability.go:41-58):
//                       PkgName, InstalledVersion, severity descending, VulnerabilityID,
//                       PkgPath.
// All strings are replaced by ranks fixed before the launch: the vulnerability ID and
// output FixedVersion of every advisory (load time, vulninfo.cpp) and the (name, version)
// of every package within its result (host, once per batch).  Then:
//   filter_count_dup  pairs of packages whose (result, name, version) repeats (sizes the
//                  dedup table for them alone; one host synchronisation);
//   filter_mark    per pair: severity/status/ignore test; duplicates (packages whose
//                  (result, name, version) repeats) race into an open-addressing table
//                  with one 64-bit atomicMax of (FixedVersion rank, -package) per key;
//   filter_select  losers drop out; then the VEX filter (filter.go:51-53, after dedup):
//                  a survivor whose (package, vulnerability rank) the host-compiled VEX
//                  suppression list holds (binary search) drops out too; survivors keep
//                  the BySeverity sort key
//                  (package rank << (b + 3) | (4 - severity) << b | vulnerability rank,
//                  b = bits of the DB's vulnerability-rank count);
//   radix sort     hipcub DeviceRadixSort over (key, pair index), dropped pairs last;
//   filter_gather  the surviving {package, advisory} pairs in report order.
// Integer work bound by HBM traffic (pairs, decisions, ranks); no MFMA.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "vulninfo.h"

namespace tvm {

namespace {

constexpr int kFilterBlock = 256;
constexpr unsigned long long kEmpty = ~0ull;  // sort key of a dropped pair

struct FilterArgs {
  FillDev t;
  const uint32_t* pkg;  // the ordered match list (package, advisory columns)
  const uint32_t* adv;
  const uint4* fill;
  uint64_t n;
  const uint32_t* pkg_rank;     // per package: rank of (result, name, version) in the batch
  const uint8_t* pkg_dup;       // per package: its (result, name, version) repeats
  const uint32_t* ignore;       // sorted vulnerability ranks of the ignore file
  uint32_t n_ignore;
  const unsigned long long* vex;  // sorted (package << 32 | tag << 31 | vulnerability rank):
                                  // tag 0 VEX suppression, tag 1 ignore-file pair
  uint32_t n_vex;
  uint32_t sev_mask, status_mask;
  uint32_t id_bits;             // sort key: package rank << (id_bits + 3) | (4 - severity) << id_bits | ID rank
  unsigned long long* table;    // {key, value} pairs, 2^k entries (dup pairs only)
  uint64_t table_mask;
  unsigned long long* sort_key;
  unsigned long long* mine;     // dup pairs: the table slot filter_mark put the pair's key in
  uint32_t* idx;
  unsigned long long* count;
};

__device__ __forceinline__ uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h;
}

// Severity index of a pair after FillInfo (0..4; 5 = a string outside SeverityNames).
__device__ __forceinline__ uint32_t pair_severity(const FillDev& t, uint4 d, uint4 it) {
  const uint32_t det = it.y & 0xFFu;  // the detector's package-specific severity (0xFF none)
  if (d.x == FILL_NOT_FOUND) return (it.z & FI_SEV_SRC) && det < 5 ? det : 0u;  // unchanged; "" -> UNKNOWN
  const uint32_t code = d.z & 0xFFFFu;
  if (code < 5) return code;
  if (code == SEV_KEEP) return det < 5 ? det : 0u;
  if (code == SEV_RAW) return 5u;  // a DB string that is not a severity name never passes
  return 0u;                       // SEV_OOR prints UNKNOWN
}

__global__ __launch_bounds__(kFilterBlock) void filter_mark(FilterArgs a) {
  const uint64_t stride = uint64_t(gridDim.x) * kFilterBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kFilterBlock + threadIdx.x; i < a.n; i += stride) {
    const uint2 p = make_uint2(a.pkg[i], a.adv[i]);
    const uint4 d = a.fill[i];
    const uint4 it = a.t.adv_items[p.y];
    const uint2 rk = a.t.adv_rank[p.y];
    const uint32_t sev = pair_severity(a.t, d, it);
    bool keep = ((a.sev_mask >> sev) & 1u) && !((a.status_mask >> (d.y & 31u)) & 1u);
    if (keep && a.n_ignore) {  // binary search of the ignore file's vulnerability ranks
      uint32_t lo = 0, hi = a.n_ignore;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.ignore[mid] < rk.x) lo = mid + 1;
        else hi = mid;
      }
      keep = !(lo < a.n_ignore && a.ignore[lo] == rk.x);
    }
    if (keep && a.n_vex) {  // ignore findings scoped by PURL: tagged keys, before the dedup
      const unsigned long long key = (uint64_t(p.x) << 32) | 0x80000000ull | rk.x;
      uint32_t lo = 0, hi = a.n_vex;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.vex[mid] < key) lo = mid + 1;
        else hi = mid;
      }
      keep = !(lo < a.n_vex && a.vex[lo] == key);
    }
    const unsigned long long key = (uint64_t(a.pkg_rank[p.x]) << 32) | rk.x;
    const unsigned long long val = (uint64_t(rk.y) << 32) | (0xFFFFFFFFu - p.x);
    a.idx[i] = uint32_t(i);
    a.sort_key[i] = keep ? (uint64_t(a.pkg_rank[p.x]) << (a.id_bits + 3)) | (uint64_t(4u - sev) << a.id_bits) | rk.x
                         : kEmpty;
    if (keep && a.pkg_dup[p.x]) {  // table entries: {key + 1 (0 = empty), max value}, zeroed
      for (uint64_t s = mix64(key) & a.table_mask;; s = (s + 1) & a.table_mask) {
        const unsigned long long prev = atomicCAS(&a.table[2 * s], 0ull, key + 1);
        if (prev == 0ull || prev == key + 1) {
          atomicMax(&a.table[2 * s + 1], val);
          a.mine[i] = s;  // filter_select reads the winner straight from this slot
          break;
        }
      }
    }
  }
}

__global__ __launch_bounds__(kFilterBlock) void filter_select(FilterArgs a) {
  __shared__ uint32_t wsum[kFilterBlock / 64];
  const uint64_t stride = uint64_t(gridDim.x) * kFilterBlock;
  uint32_t live_n = 0;  // survivors seen by this lane; one counter atomic per block at the end
  for (uint64_t i = uint64_t(blockIdx.x) * kFilterBlock + threadIdx.x; i < a.n; i += stride) {
    bool live = a.sort_key[i] != kEmpty;
    const uint2 p = make_uint2(a.pkg[i], a.adv[i]);
    if (live && a.pkg_dup[p.x]) {  // the slot filter_mark inserted this pair's key into
      const unsigned long long own = (uint64_t(a.t.adv_rank[p.y].y) << 32) | (0xFFFFFFFFu - p.x);
      if (a.table[2 * a.mine[i] + 1] != own) {
        a.sort_key[i] = kEmpty;  // another duplicate won (greater FixedVersion, or first seen)
        live = false;
      }
    }
    if (live && a.n_vex) {  // VEX: openvex.go:35-40 / cyclonedx.go:56-60 / csaf.go:36-40 drop it
      const unsigned long long key = (uint64_t(p.x) << 32) | a.t.adv_rank[p.y].x;
      uint32_t lo = 0, hi = a.n_vex;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.vex[mid] < key) lo = mid + 1;
        else hi = mid;
      }
      if (lo < a.n_vex && a.vex[lo] == key) {
        a.sort_key[i] = kEmpty;
        live = false;
      }
    }
    live_n += live ? 1u : 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) live_n += __shfl_xor(live_n, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = live_n;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kFilterBlock / 64; w++) t += wsum[w];
    if (t) atomicAdd(a.count, (unsigned long long)t);
  }
}

// Pairs whose package's (result, name, version) repeats: the only ones that enter the dedup
// table, so the table is sized (and cleared) for them alone.
__global__ __launch_bounds__(kFilterBlock) void filter_count_dup(const uint32_t* pkg, const uint8_t* pkg_dup,
                                                                 uint64_t n, unsigned long long* count) {
  __shared__ uint32_t wsum[kFilterBlock / 64];
  const uint64_t stride = uint64_t(gridDim.x) * kFilterBlock;
  uint32_t c = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kFilterBlock + threadIdx.x; i < n; i += stride) c += pkg_dup[pkg[i]];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kFilterBlock / 64; w++) t += wsum[w];
    if (t) atomicAdd(count, (unsigned long long)t);
  }
}

__global__ __launch_bounds__(kFilterBlock) void filter_gather(const uint32_t* pkg, const uint32_t* adv,
                                                              const uint32_t* idx, uint64_t n, uint2* out) {
  const uint64_t i = uint64_t(blockIdx.x) * kFilterBlock + threadIdx.x;
  if (i < n) out[i] = make_uint2(pkg[idx[i]], adv[idx[i]]);
}

bool ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

}  // namespace

BatchFilter::~BatchFilter() {
  for (void* p : bufs_)
    if (p) (void)hipFree(p);
}

bool BatchFilter::grow(void*& p, uint64_t& cap, uint64_t need, std::string& err) {
  if (cap >= need) return true;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  if (!ok(hipMalloc(&p, std::max<uint64_t>(need, 1)), "hipMalloc(filter)", err)) return false;
  cap = need;
  return true;
}

bool BatchFilter::set_packages(const std::vector<uint32_t>& pkg_rank, const std::vector<uint8_t>& pkg_dup,
                               std::string& err) {
  any_dup_ = std::any_of(pkg_dup.begin(), pkg_dup.end(), [](uint8_t x) { return x != 0; });
  n_pkgs_ = pkg_rank.size();
  return grow(bufs_[0], caps_[0], pkg_rank.size() * 4, err) && grow(bufs_[1], caps_[1], pkg_dup.size(), err) &&
         (pkg_rank.empty() || ok(hipMemcpy(bufs_[0], pkg_rank.data(), pkg_rank.size() * 4, hipMemcpyHostToDevice),
                                 "hipMemcpy(pkg ranks)", err)) &&
         (pkg_dup.empty() ||
          ok(hipMemcpy(bufs_[1], pkg_dup.data(), pkg_dup.size(), hipMemcpyHostToDevice), "hipMemcpy(pkg dup)", err));
}

bool BatchFilter::run(const FillDev& t, const uint32_t* pkg, const uint32_t* adv, const uint4* fill, uint64_t n,
                      const std::vector<uint32_t>& ignore, const std::vector<uint64_t>& vex, uint32_t n_ranks,
                      uint32_t sev_mask, uint32_t status_mask, hipStream_t st, std::string& err) {
  n_ = n;
  survivors_ = 0;
  if (n == 0) return true;
  if (n > 0xFFFFFFFFull || vex.size() > 0xFFFFFFFFull) {
    err = "filter: too many pairs";
    return false;
  }
  const uint32_t blocks = uint32_t(std::min<uint64_t>((n + kFilterBlock - 1) / kFilterBlock, 256ull * 64));
  uint64_t tcap = 0;  // dedup table: 2^k >= 2 x the pairs that can enter it (load <= 0.5, probes end)
  if (any_dup_) {
    unsigned long long dup_n = 0;
    if (!grow(bufs_[10], caps_[10], 8, err) || !ok(hipMemsetAsync(bufs_[10], 0, 8, st), "memset(dup count)", err))
      return false;
    hipLaunchKernelGGL(filter_count_dup, dim3(blocks), dim3(kFilterBlock), 0, st, pkg,
                       static_cast<const uint8_t*>(bufs_[1]), n, static_cast<unsigned long long*>(bufs_[10]));
    if (!ok(hipGetLastError(), "filter_count_dup", err) ||
        !ok(hipMemcpyAsync(&dup_n, bufs_[10], 8, hipMemcpyDeviceToHost, st), "D2H dup count", err) ||
        !ok(hipStreamSynchronize(st), "filter sync", err))
      return false;
    if (dup_n) {
      tcap = 16;
      while (tcap < 2 * dup_n) tcap <<= 1;
    }
  }
  // sort only the key bits in use: package rank (< 2^pkg_bits, never all ones) << (id_bits
  // + 3) | severity | ID rank (< 2^id_bits); a dropped pair's all-ones key stays the largest
  uint32_t id_bits = 1;
  while (id_bits < 32 && (uint64_t(1) << id_bits) < n_ranks) id_bits++;
  int pkg_bits = 1;
  while (pkg_bits < 32 && (uint64_t(1) << pkg_bits) <= n_pkgs_) pkg_bits++;
  const int end_bit = int(id_bits) + 3 + pkg_bits;
  if (end_bit > 64) {
    err = "filter: sort key wider than 64 bits";
    return false;
  }
  size_t sort_bytes = 0;
  if (!ok(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, static_cast<unsigned long long*>(nullptr),
                                             static_cast<unsigned long long*>(nullptr), static_cast<uint32_t*>(nullptr),
                                             static_cast<uint32_t*>(nullptr), int(n), 0, end_bit, st),
          "hipcub sort sizing", err))
    return false;
  // 2 ignore, 3 table, 4 sort keys in, 5 sort keys out, 6 mine, 7 idx in, 8 idx out, 9 temp, 10 count,
  // 11 out pairs, 12 VEX suppressions
  if (!grow(bufs_[2], caps_[2], std::max<size_t>(ignore.size(), 1) * 4, err) ||
      !grow(bufs_[3], caps_[3], std::max<uint64_t>(tcap, 1) * 16, err) || !grow(bufs_[4], caps_[4], n * 8, err) ||
      !grow(bufs_[5], caps_[5], n * 8, err) || !grow(bufs_[6], caps_[6], n * 8, err) ||
      !grow(bufs_[7], caps_[7], n * 4, err) || !grow(bufs_[8], caps_[8], n * 4, err) ||
      !grow(bufs_[9], caps_[9], sort_bytes, err) || !grow(bufs_[10], caps_[10], 8, err) ||
      !grow(bufs_[11], caps_[11], n * 8, err) || !grow(bufs_[12], caps_[12], std::max<size_t>(vex.size(), 1) * 8, err))
    return false;
  if (!vex.empty()) {  // unsorted keys in (bufs_[5], free until the main sort) -> sorted in bufs_[12]
    size_t vb = 0;
    if (!ok(hipcub::DeviceRadixSort::SortKeys(nullptr, vb, static_cast<unsigned long long*>(nullptr),
                                              static_cast<unsigned long long*>(nullptr), int(vex.size()), 0, 64, st),
            "hipcub vex sort sizing", err) ||
        !grow(bufs_[9], caps_[9], std::max(sort_bytes, vb), err) ||
        !grow(bufs_[5], caps_[5], std::max<uint64_t>(n, vex.size()) * 8, err) ||
        !ok(hipMemcpyAsync(bufs_[5], vex.data(), vex.size() * 8, hipMemcpyHostToDevice, st), "H2D vex", err) ||
        !ok(hipcub::DeviceRadixSort::SortKeys(bufs_[9], vb, static_cast<unsigned long long*>(bufs_[5]),
                                              static_cast<unsigned long long*>(bufs_[12]), int(vex.size()), 0, 64, st),
            "hipcub vex sort", err))
      return false;
  }
  if (!ignore.empty() &&
      !ok(hipMemcpyAsync(bufs_[2], ignore.data(), ignore.size() * 4, hipMemcpyHostToDevice, st), "H2D ignore", err))
    return false;
  if (tcap && !ok(hipMemsetAsync(bufs_[3], 0, tcap * 16, st), "memset(filter table)", err)) return false;
  if (!ok(hipMemsetAsync(bufs_[10], 0, 8, st), "memset(count)", err)) return false;
  FilterArgs a{};
  a.t = t;
  a.pkg = pkg;
  a.adv = adv;
  a.fill = fill;
  a.n = n;
  a.pkg_rank = static_cast<const uint32_t*>(bufs_[0]);
  a.pkg_dup = static_cast<const uint8_t*>(bufs_[1]);
  a.ignore = static_cast<const uint32_t*>(bufs_[2]);
  a.n_ignore = uint32_t(ignore.size());
  a.vex = static_cast<const unsigned long long*>(bufs_[12]);
  a.n_vex = uint32_t(vex.size());
  a.sev_mask = sev_mask;
  a.id_bits = id_bits;
  a.status_mask = status_mask;
  a.table = static_cast<unsigned long long*>(bufs_[3]);
  a.table_mask = tcap ? tcap - 1 : 0;
  a.sort_key = static_cast<unsigned long long*>(bufs_[4]);
  a.mine = static_cast<unsigned long long*>(bufs_[6]);
  a.idx = static_cast<uint32_t*>(bufs_[7]);
  a.count = static_cast<unsigned long long*>(bufs_[10]);
  hipLaunchKernelGGL(filter_mark, dim3(blocks), dim3(kFilterBlock), 0, st, a);
  hipLaunchKernelGGL(filter_select, dim3(blocks), dim3(kFilterBlock), 0, st, a);
  if (!ok(hipGetLastError(), "filter launch", err)) return false;
  if (!ok(hipcub::DeviceRadixSort::SortPairs(bufs_[9], sort_bytes, a.sort_key,
                                             static_cast<unsigned long long*>(bufs_[5]), a.idx,
                                             static_cast<uint32_t*>(bufs_[8]), int(n), 0, end_bit, st),
          "hipcub sort", err))
    return false;
  unsigned long long cnt = 0;
  if (!ok(hipMemcpyAsync(&cnt, bufs_[10], 8, hipMemcpyDeviceToHost, st), "D2H count", err) ||
      !ok(hipStreamSynchronize(st), "filter sync", err))
    return false;
  survivors_ = cnt;
  if (cnt) {
    hipLaunchKernelGGL(filter_gather, dim3(uint32_t((cnt + kFilterBlock - 1) / kFilterBlock)), dim3(kFilterBlock), 0,
                       st, pkg, adv, static_cast<const uint32_t*>(bufs_[8]), uint64_t(cnt),
                       static_cast<uint2*>(bufs_[11]));
    if (!ok(hipGetLastError(), "filter gather", err)) return false;
  }
  return true;
}

bool BatchFilter::fetch(std::vector<uint2>& out, hipStream_t st, std::string& err) {
  out.assign(survivors_, make_uint2(0, 0));
  if (!survivors_) return true;
  return ok(hipMemcpyAsync(out.data(), bufs_[11], survivors_ * 8, hipMemcpyDeviceToHost, st), "D2H filtered", err) &&
         ok(hipStreamSynchronize(st), "filter sync", err);
}

}  // namespace tvm
