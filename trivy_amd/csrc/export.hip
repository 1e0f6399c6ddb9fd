// The batch path's DetectedVulnerability set on the device (export.h): a batch's match list
// (raw, or Red Hat-merged) turned into per-package record lists in pinned host memory.
//
// The records of a DetectedVulnerability are one per DB advisory (its driver's epilogue,
// drivers.h advisory_templates) except for Red Hat groups of several advisories merged per
// VulnerabilityID (redhat.go:146-187), which need a record of their own (the VendorIDs union,
// the greatest FixedVersion).  So the device writes, per match, its record index - the
// advisory, or n_adv + k for the k-th multi-member Red Hat group - and the host only builds the
// k group records from their members, which the device gathers into a compact list.  The
// per-package lists reach the host through the result move of the pipelined pass (engine.h
// copy_out_tiles: kernel stores into pinned memory, 3-byte record indices when they fit).
#include "export.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "pipeline.h"
#include "pool.h"

namespace tvm {

namespace {

constexpr int kBlock = 256;

bool ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

// flag[i] = 1: merged entry i is a Red Hat group of several members (its own record)
__global__ __launch_bounds__(kBlock) void rh_flag_kernel(const uint32_t* pkg, const uint2* grp, const uint2* pk,
                                                         const PlatInfo* plats, uint32_t n_plats, uint32_t pkg_base,
                                                         uint64_t n, uint32_t* flag) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t plat = pk[pkg[i] - pkg_base].x;
    flag[i] = plat < n_plats && plats[plat].drv == DRV_REDHAT && grp[i].y > 1u ? 1u : 0u;
  }
}

// rec[i] = the entry's advisory, or n_adv + k for the k-th flagged entry (k = the exclusive
// scan of the flags), whose {position, package, first member, representative} and member
// range go to the compact group list
__global__ __launch_bounds__(kBlock) void rh_rec_kernel(const uint32_t* pkg, const uint32_t* adv, const uint32_t* base,
                                                        const uint2* grp, const uint32_t* flag, const uint32_t* k_of,
                                                        uint64_t n, uint32_t n_adv, uint32_t* rec, uint4* groups,
                                                        uint2* ranges) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock) {
    if (flag[i]) {
      const uint32_t k = k_of[i];
      rec[i] = n_adv + k;
      groups[k] = make_uint4(uint32_t(i), pkg[i], base[i], adv[i]);
      ranges[k] = grp[i];  // {raw position of the first member, member count}
    } else {
      rec[i] = adv[i];
    }
  }
}

// The members of every flagged group (advisories at raw positions [start, start + len)) at
// their group's offset (exclusive scan of the counts)
__global__ __launch_bounds__(kBlock) void rh_members_kernel(const uint2* ranges, const uint32_t* moff, uint32_t n_groups,
                                                            const uint32_t* raw_adv, uint64_t raw_cap, uint32_t* members) {
  for (uint64_t k = uint64_t(blockIdx.x) * kBlock + threadIdx.x; k < n_groups; k += uint64_t(gridDim.x) * kBlock) {
    const uint2 r = ranges[k];
    const uint32_t o = moff[k];
    for (uint32_t m = 0; m < r.y; m++) members[o + m] = uint64_t(r.x) + m < raw_cap ? raw_adv[r.x + m] : 0xFFFFFFFFu;
  }
}

struct LenOf {
  const uint2* r;
  __host__ __device__ uint32_t operator()(uint32_t k) const { return r[k].y; }
};

// Device blocks of one export call, back to the pool on every exit.
struct Blocks {
  int dev;
  std::vector<void*> v;
  ~Blocks() {
    for (void* p : v) pool_device_put(dev, p);
  }
  template <class T>
  T* get(size_t count, const char* what, std::string& err) {
    void* p = pool_device_get(dev, std::max<size_t>(count, 1) * sizeof(T), what, err);
    if (p) v.push_back(p);
    return static_cast<T*>(p);
  }
};

}  // namespace

VulnExport::~VulnExport() {
  pool_host_put(row_end_h);
  pool_host_put(rec_h);
}

bool export_vulns(int dev, hipStream_t st, const ExportList& in, uint32_t n_adv, VulnExport& out, std::string& err) {
  Blocks blocks{dev, {}};
  (void)hipSetDevice(dev);
  const uint64_t n = in.total;
  uint32_t n_groups = 0;
  const uint32_t* rec_dev = in.list.adv;
  uint4* g_dev = nullptr;
  uint32_t *moff_dev = nullptr, *mem_dev = nullptr;
  uint64_t n_members = 0;
  const uint32_t grid = uint32_t(std::min<uint64_t>((n + kBlock - 1) / kBlock, 8192));
  if (in.rh && n) {  // Red Hat groups of several members: their own records
    uint32_t* flag = blocks.get<uint32_t>(n + 1, "hipMalloc(export flags)", err);
    uint32_t* k_of = flag ? blocks.get<uint32_t>(n + 1, "hipMalloc(export scan)", err) : nullptr;
    uint32_t* rec = k_of ? blocks.get<uint32_t>(n, "hipMalloc(export records)", err) : nullptr;
    if (!rec) return false;
    hipLaunchKernelGGL(rh_flag_kernel, dim3(grid), dim3(kBlock), 0, st, in.list.pkg, in.grp, in.pk, in.plats,
                       in.n_plats, in.pkg_base, n, flag);
    size_t tmp_bytes = 0;
    if (!ok(hipMemsetAsync(flag + n, 0, 4, st), "memset(export flags)", err) ||
        !ok(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, flag, k_of, int(n + 1), st), "hipcub scan", err))
      return false;
    void* tmp = blocks.get<uint8_t>(tmp_bytes, "hipMalloc(export scan temp)", err);
    uint32_t ng = 0;
    if (!tmp || !ok(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, flag, k_of, int(n + 1), st), "hipcub scan", err) ||
        !ok(hipMemcpyAsync(&ng, k_of + n, 4, hipMemcpyDeviceToHost, st), "D2H group count", err) ||
        !ok(hipStreamSynchronize(st), "export", err))
      return false;
    n_groups = ng;
    g_dev = blocks.get<uint4>(n_groups, "hipMalloc(export groups)", err);
    uint2* ranges = g_dev ? blocks.get<uint2>(n_groups, "hipMalloc(export ranges)", err) : nullptr;
    moff_dev = ranges ? blocks.get<uint32_t>(size_t(n_groups) + 1, "hipMalloc(export member offsets)", err) : nullptr;
    if (!moff_dev) return false;
    hipLaunchKernelGGL(rh_rec_kernel, dim3(grid), dim3(kBlock), 0, st, in.list.pkg, in.list.adv, in.base, in.grp, flag,
                       k_of, n, n_adv, rec, g_dev, ranges);
    rec_dev = rec;
    if (n_groups) {
      using Count = hipcub::CountingInputIterator<uint32_t>;
      using Lens = hipcub::TransformInputIterator<uint32_t, LenOf, Count>;
      size_t tb = 0;
      uint32_t last[2] = {0, 0};
      if (!ok(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, Lens(Count(0), LenOf{ranges}), moff_dev, int(n_groups), st),
              "hipcub scan", err))
        return false;
      void* t2 = blocks.get<uint8_t>(tb, "hipMalloc(export scan temp)", err);
      if (!t2 ||
          !ok(hipcub::DeviceScan::ExclusiveSum(t2, tb, Lens(Count(0), LenOf{ranges}), moff_dev, int(n_groups), st),
              "hipcub scan", err) ||
          !ok(hipMemcpyAsync(&last[0], moff_dev + n_groups - 1, 4, hipMemcpyDeviceToHost, st), "D2H members", err) ||
          !ok(hipMemcpyAsync(&last[1], &ranges[n_groups - 1].y, 4, hipMemcpyDeviceToHost, st), "D2H members", err) ||
          !ok(hipStreamSynchronize(st), "export", err))
        return false;
      n_members = uint64_t(last[0]) + last[1];
      mem_dev = blocks.get<uint32_t>(n_members, "hipMalloc(export members)", err);
      if (!mem_dev) return false;
      hipLaunchKernelGGL(rh_members_kernel, dim3(uint32_t(std::min<uint64_t>((n_groups + kBlock - 1) / kBlock, 4096))),
                         dim3(kBlock), 0, st, ranges, moff_dev, n_groups, in.raw_adv, in.raw_cap, mem_dev);
    }
    if (!ok(hipGetLastError(), "export kernels", err)) return false;
  }
  // the per-package record lists into pinned host memory (the pipelined pass's result move)
  const uint64_t recs = uint64_t(n_adv) + n_groups;
  out.width = recs < (1ull << 24) ? 3u : 4u;
  const size_t n4 = (size_t(in.n_tiles) * kTile + 3) & ~size_t(3), cap4 = (std::max<uint64_t>(n, 1) + 3) & ~uint64_t(3);
  std::string e2;
  out.row_end_h = static_cast<uint32_t*>(pool_host_get(std::max<size_t>(n4, 4) * 4, "hipHostMalloc(export rows)", err));
  out.rec_h = out.row_end_h ? static_cast<uint8_t*>(pool_host_get(cap4 * 4, "hipHostMalloc(export records)", err)) : nullptr;
  unsigned long long* cb = blocks.get<unsigned long long>(2, "hipMalloc(export chunk base)", err);
  if (!out.rec_h || !cb) return false;
  void *row_d = nullptr, *rec_d = nullptr;
  if (!ok(hipHostGetDevicePointer(&row_d, out.row_end_h, 0), "hipHostGetDevicePointer(rows)", err) ||
      !ok(hipHostGetDevicePointer(&rec_d, out.rec_h, 0), "hipHostGetDevicePointer(records)", err) ||
      !ok(hipMemsetAsync(cb, 0, 16, st), "memset(chunk base)", err))
    return false;
  CopyOutArgs ca;
  ca.dir = in.list.dir;
  ca.pkg = in.list.pkg;
  ca.adv = rec_dev;
  ca.row_end_h = static_cast<uint32_t*>(row_d);
  ca.adv_h = static_cast<uint32_t*>(rec_d);
  ca.chunk_base = cb;
  ca.c = 0;
  ca.t0 = 0;
  ca.t1 = in.n_tiles;
  ca.pkg_base = in.pkg_base;
  ca.cap = in.list.cap;
  ca.packed = out.width == 3 ? 1u : 0u;
  ca.adv_units = cap4 / 4;
  ca.row_end_units = std::max<size_t>(n4, 4) / 4;
  ca.ctl = in.list.ctl;
  if (in.n_tiles) launch_copy_out(st, ca);
  out.groups.resize(n_groups);
  out.members.resize(n_members);
  uint32_t* moff_h = out.moff_h(n_groups);
  unsigned long long ctl3 = 0;
  if (!ok(hipGetLastError(), "export copy-out", err) ||
      (n_groups && !ok(hipMemcpyAsync(out.groups.data(), g_dev, n_groups * sizeof(uint4), hipMemcpyDeviceToHost, st),
                       "D2H groups", err)) ||
      (n_groups && !ok(hipMemcpyAsync(moff_h, moff_dev, n_groups * 4, hipMemcpyDeviceToHost, st),
                       "D2H member offsets", err)) ||
      (n_members && !ok(hipMemcpyAsync(out.members.data(), mem_dev, n_members * 4, hipMemcpyDeviceToHost, st),
                        "D2H members", err)) ||
      !ok(hipMemcpyAsync(&ctl3, in.list.ctl + 3, 8, hipMemcpyDeviceToHost, st), "D2H ctl", err) ||
      !ok(hipStreamSynchronize(st), "export", err))
    return false;
  if (ctl3) {
    err = "export: result move error bits " + std::to_string(ctl3);
    return false;
  }
  out.n = n;
  out.n_groups = n_groups;
  out.moff.back() = uint32_t(n_members);
  return true;
}

}  // namespace tvm
