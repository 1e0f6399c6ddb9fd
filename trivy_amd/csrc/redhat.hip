// Red Hat per-CVE merge over a batch's match list on the GPU (gfx950): the batch form of
// the uniqVulns loop of pkg/detector/ospkg/redhat/redhat.go:146-187.
//
// For one package the reference walks its advisories in trivy-db Get order and keys them by
// VulnerabilityID: an unfixed advisory enters only if the ID is new (first seen wins); a
// fixed one (installed < fixed) enters, or merges into the existing entry - VendorIDs
// unioned (ustrings.Unique), FixedVersion raised to the greater rpm version - and the
// result is sorted by VulnerabilityID.
//
// The flattener numbers each Red Hat key's advisories in (VulnerabilityID, Get order)
// order (db.cpp flatten_os), and the match kernel emits a package's matches in advisory
// order, so a package's members of one CVE are adjacent and in Get order, and the CVEs
// ascend.  The merge is therefore one pass per tile segment, no sort:
//   count   a pair heads a group unless it is a Red Hat pair continuing its predecessor's
//           (package, ID-rank); per tile its group count (a tile without Red Hat
//           packages: its pair count, no reads of the pairs);
//   scan    the tiles' output bases (rocPRIM device scan);
//   emit    a wave per tile: ballot prefix of the head flags; each head lane walks its group (a few pairs) for
//           the member with the greatest fixed version (rpm-order rank computed at load
//           time; ties keep the first, as LessThan does) and writes {pkg, representative,
//           base, raw range}.
// Integer work bound by memory traffic (about 8 B read + 20 B written per pair); no MFMA.
#include <algorithm>
#include <string>

#include <rocprim/device/device_scan.hpp>

#include "redhat.h"

namespace tvm {

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr uint32_t kNoKey = 0xFFFFFFFFu;

struct MergeArgs {
  const TileDir* dir;
  const uint32_t* pkg;         // raw match columns
  const uint32_t* adv;
  const uint2* pk;             // batch packages {plat, lengths}
  const PlatInfo* plats;
  uint32_t n_plats;
  uint32_t pkg_base;
  uint32_t n;                  // packages in the batch
  const uint2* rk;             // {vulnerability-ID rank, fixed-version rank (RH_NONE = unfixed)}
  uint64_t raw_cap;
  TileDir* mdir;
  uint32_t* mpkg;
  uint32_t* madv;
  uint32_t* mbase;
  uint2* mgrp;
  uint64_t mcap;
  unsigned long long* mctl;
};

// Group key of raw position i: the vulnerability-ID rank of a Red Hat pair, kNoKey else.
__device__ __forceinline__ uint32_t group_key(const MergeArgs& a, uint32_t p, uint32_t ad) {
  const uint32_t plat = a.pk[p - a.pkg_base].x;
  const bool rh = plat < a.n_plats && a.plats[plat].drv == DRV_REDHAT;
  return rh ? a.rk[ad].x : kNoKey;
}

// Per package of tile t: 1 = a Red Hat package (its pairs' group keys are their ID ranks);
// one wave fills its own 256 flags (4 a lane) in LDS.
__device__ __forceinline__ void tile_redhat_flags(const MergeArgs& a, uint32_t t, uint32_t lane, uint8_t* rhp) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t p = t * kBlock + lane * 4 + k;
    const uint32_t plat = p < a.n ? a.pk[p].x : 0xFFFFFFFFu;
    rhp[lane * 4 + k] = plat < a.n_plats && a.plats[plat].drv == DRV_REDHAT;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// The lane's pair of chunk c (64 pairs) of a tile segment [b0, b0 + cnt): package p,
// advisory ad, its group key (the ID rank for a Red Hat package, kNoKey else) and, for a
// Red Hat pair, its fixed-version rank (fr) - one gather for both.
__device__ __forceinline__ uint32_t chunk_key(const MergeArgs& a, uint64_t b0, uint32_t c, uint32_t cnt, uint32_t t,
                                              uint32_t lane, const uint8_t* rhp, uint32_t& p, uint32_t& ad,
                                              uint32_t& fr) {
  fr = RH_NONE;
  if (c + lane >= cnt) return kNoKey;
  p = a.pkg[b0 + c + lane];
  ad = a.adv[b0 + c + lane];
  if (!rhp[(p - a.pkg_base - t * kBlock) & (kBlock - 1)]) return kNoKey;
  const uint2 r = a.rk[ad];
  fr = r.y;
  return r.x;
}

// The (package, key) of the pair before the lane's, by shuffle; lane 0 takes the previous
// chunk's last pair (prev_*, advanced here to this chunk's last), so each pair's key is
// gathered once.  left = pairs of the segment from this chunk on.
__device__ __forceinline__ void pair_before(uint32_t lane, uint32_t p, uint32_t k, uint32_t& prev_p, uint32_t& prev_k,
                                            uint32_t left, uint32_t& pp, uint32_t& kp) {
  const uint32_t up = __shfl_up(p, 1, 64), uk = __shfl_up(k, 1, 64);
  pp = lane ? up : prev_p;
  kp = lane ? uk : prev_k;
  const int last = int((left < 64u ? left : 64u) - 1);
  prev_p = __shfl(p, last, 64);
  prev_k = __shfl(k, last, 64);
}

// Pass 1: the merged entry count of every tile into counts[t].  The tiles' output bases then
// come from a scan (rocPRIM), not from an atomic reservation per tile: 78k same-address
// atomics serialised the round-3 kernel (C5: 0.95 ms, SQ_WAIT_ANY / SQ_WAVE_CYCLES = 0.95).
// Workgroups [0, nb_rh) take the tiles that hold Red Hat packages, one wave each (rh_list;
// the groups of their segments, 64 pairs a step, no workgroup barrier); the rest one lane per
// tile for all others, whose pairs are groups of one (a workgroup per such tile spent its
// time being dispatched).
__global__ __launch_bounds__(kBlock) void rh_count_kernel(MergeArgs a, uint32_t* counts, const uint8_t* rh_flags,
                                                          const uint32_t* rh_list, uint32_t n_rh, uint32_t n_tiles) {
  __shared__ uint8_t rhp_all[kWaves][kBlock];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t nb_rh = (n_rh + kWaves - 1) / kWaves;
  if (blockIdx.x >= nb_rh) {
    const uint32_t t = (blockIdx.x - nb_rh) * kBlock + tid;
    if (t >= n_tiles || rh_flags[t]) return;
    const TileDir d = a.dir[t];
    const bool fits = d.base + d.count <= a.raw_cap;
    counts[t] = fits ? d.count : 0u;
    if (!fits) atomicOr(a.mctl + 3, 1ull);  // an overflowed match list: nothing valid to merge
    return;
  }
  const uint32_t r = blockIdx.x * kWaves + wave;
  if (r >= n_rh) return;  // wave-uniform; no workgroup barrier follows
  const uint32_t t = rh_list[r];
  uint8_t* rhp = rhp_all[wave];
  tile_redhat_flags(a, t, lane, rhp);
  const TileDir d = a.dir[t];
  const uint64_t b0 = d.base;
  const uint32_t cnt = d.count;
  if (b0 + cnt > a.raw_cap) {
    if (lane == 0) {
      counts[t] = 0;
      atomicOr(a.mctl + 3, 1ull);
    }
    return;
  }
  uint32_t heads = 0, prev_p = 0xFFFFFFFFu, prev_k = kNoKey;
  bool order_bad = false;
  for (uint32_t c = 0; c < cnt; c += 64) {
    const bool v = c + lane < cnt;
    uint32_t p = 0xFFFFFFFFu, ad = 0, fr;
    const uint32_t k = chunk_key(a, b0, c, cnt, t, lane, rhp, p, ad, fr);
    uint32_t pp, kp;
    pair_before(lane, p, k, prev_p, prev_k, cnt - c, pp, kp);
    bool h = false;
    if (v) {
      const bool cont = k != kNoKey && pp == p;
      h = !(cont && kp == k);
      order_bad |= cont && kp > k;
    }
    heads += uint32_t(__popcll(__ballot(h)));
  }
  if (__ballot(order_bad) && lane == 0) atomicOr(a.mctl + 3, (unsigned long long)ERR_RH_ORDER);
  if (lane == 0) counts[t] = heads;
}

// The tiles' output bases: an exclusive scan of the counts (rocPRIM's single-pass decoupled
// look-back scan, RedHatMerge::launch).

// Pass 2: each tile writes its merged entries at its base, one wave per tile.  Workgroups
// [0, nb_rh): the Red Hat tiles, one entry per group (the member with the greatest fixed
// version; ties keep the first, as LessThan does) and its member range (grp), which only the
// host's Red Hat vulnerability build reads (rh_vulns, for Red Hat packages).  The rest: a
// coalesced copy (pairs pass through as groups of one: 8 bytes in, 12 out per pair).  The
// tile directory entry and, at the last tile, the merged total go with the tile.
__global__ __launch_bounds__(kBlock) void rh_emit_kernel(MergeArgs a, const uint32_t* counts,
                                                         const unsigned long long* bases, const uint8_t* rh_flags,
                                                         const uint32_t* rh_list, uint32_t n_rh, uint32_t n_tiles) {
  __shared__ uint8_t rhp_all[kWaves][kBlock];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t nb_rh = (n_rh + kWaves - 1) / kWaves;
  if (blockIdx.x >= nb_rh) {
    const uint32_t t = (blockIdx.x - nb_rh) * kWaves + wave;
    if (t >= n_tiles || rh_flags[t]) return;
    const TileDir d = a.dir[t];
    const uint64_t b0 = d.base;
    const uint32_t cnt = d.count;
    const unsigned long long o0 = bases[t];
    const uint32_t heads = counts[t];
    const bool fits = b0 + cnt <= a.raw_cap && o0 + heads <= a.mcap;
    if (lane == 0) {
      a.mdir[t] = TileDir{o0, fits ? heads : 0u, 0};
      if (t + 1 == n_tiles) a.mctl[0] = o0 + heads;  // the merged total
    }
    if (!fits) return;
    constexpr int kU = 4;  // loads of four pairs in flight per lane before the stores
    for (uint32_t c = 0; c < cnt; c += kU * 64) {
      uint32_t pp[kU], aa[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t i = c + u * 64 + lane;
        pp[u] = i < cnt ? a.pkg[b0 + i] : 0u;
        aa[u] = i < cnt ? a.adv[b0 + i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t i = c + u * 64 + lane;
        if (i < cnt) {
          a.mpkg[o0 + i] = pp[u];
          a.madv[o0 + i] = aa[u];
          a.mbase[o0 + i] = aa[u];
        }
      }
    }
    return;
  }
  const uint32_t r = blockIdx.x * kWaves + wave;
  if (r >= n_rh) return;
  const uint32_t t = rh_list[r];
  uint8_t* rhp = rhp_all[wave];
  tile_redhat_flags(a, t, lane, rhp);
  const TileDir d = a.dir[t];
  const uint64_t b0 = d.base;
  const uint32_t cnt = d.count;
  const unsigned long long o0 = bases[t];
  const uint32_t heads = counts[t];
  const bool fits = b0 + cnt <= a.raw_cap && o0 + heads <= a.mcap;
  if (lane == 0) {
    a.mdir[t] = TileDir{o0, fits ? heads : 0u, 0};
    if (t + 1 == n_tiles) a.mctl[0] = o0 + heads;
  }
  if (!fits) return;  // cannot happen (merged <= raw); the counts tell the host
  const unsigned long long lt = (1ull << lane) - 1ull;
  uint32_t done = 0, prev_p = 0xFFFFFFFFu, prev_k = kNoKey;
  for (uint32_t c = 0; c < cnt; c += 64) {
    const bool v = c + lane < cnt;
    const uint64_t i = b0 + c + lane;
    uint32_t p = 0xFFFFFFFFu, ad = 0, fr;
    const uint32_t k = chunk_key(a, b0, c, cnt, t, lane, rhp, p, ad, fr);
    uint32_t pp, kp;
    pair_before(lane, p, k, prev_p, prev_k, cnt - c, pp, kp);
    const bool h = v && (k == kNoKey || pp != p || kp != k);
    const unsigned long long bal = __ballot(h);
    if (h) {
      uint32_t best = RH_NONE, best_r = 0, len = 1;
      if (k != kNoKey) {
        if (fr != RH_NONE) best = ad, best_r = fr;
        for (uint64_t j = i + 1; j < b0 + cnt && a.pkg[j] == p; j++) {
          const uint32_t aj = a.adv[j];
          const uint2 rj = a.rk[aj];
          if (rj.x != k) break;
          if (rj.y != RH_NONE && (best == RH_NONE || rj.y > best_r)) best = aj, best_r = rj.y;
          len++;
        }
      }
      const uint64_t o = o0 + done + uint32_t(__popcll(bal & lt));
      a.mpkg[o] = p;
      a.madv[o] = best != RH_NONE ? best : ad;
      a.mbase[o] = ad;
      a.mgrp[o] = make_uint2(uint32_t(i), len);
    }
    done += uint32_t(__popcll(bal));
  }
}

bool ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

}  // namespace

void RedHatMerge::release() {
  if (dev_ < 0) return;
  (void)hipSetDevice(dev_);
  Engine::free_matches(dev_, out_.m);
  if (out_.base) (void)hipFree(out_.base);
  if (out_.grp) (void)hipFree(out_.grp);
  for (void* x : {static_cast<void*>(counts_), static_cast<void*>(bases_), scan_tmp_})
    if (x) (void)hipFree(x);
  counts_ = nullptr;
  bases_ = nullptr;
  scan_tmp_ = nullptr;
  scan_tmp_bytes_ = 0;
  out_ = RhMerged{};
}

RedHatMerge::~RedHatMerge() {
  release();
  if (tiles_dev_ >= 0) {
    (void)hipSetDevice(tiles_dev_);
    if (flags_) (void)hipFree(flags_);
    if (rh_list_) (void)hipFree(rh_list_);
  }
}

bool RedHatMerge::set_tiles(const std::vector<uint8_t>& flags, std::string& err) {
  int dev = 0;
  if (!ok(hipGetDevice(&dev), "hipGetDevice", err)) return false;
  std::vector<uint32_t> list;
  for (uint32_t t = 0; t < flags.size(); t++)
    if (flags[t]) list.push_back(t);
  if (flags.size() > flags_cap_ || dev != tiles_dev_) {
    if (tiles_dev_ >= 0) {
      (void)hipSetDevice(tiles_dev_);
      if (flags_) (void)hipFree(flags_);
      if (rh_list_) (void)hipFree(rh_list_);
      (void)hipSetDevice(dev);
    }
    flags_ = nullptr;
    rh_list_ = nullptr;
    flags_cap_ = 0;
    tiles_dev_ = dev;
    void *f = nullptr, *l = nullptr;
    const size_t cap = std::max<size_t>(flags.size(), 1);
    if (!ok(hipMalloc(&f, cap), "hipMalloc(merge flags)", err) || !ok(hipMalloc(&l, cap * 4), "hipMalloc(merge list)", err)) {
      if (f) (void)hipFree(f);
      return false;
    }
    flags_ = static_cast<uint8_t*>(f);
    rh_list_ = static_cast<uint32_t*>(l);
    flags_cap_ = cap;
  }
  if ((!flags.empty() && !ok(hipMemcpy(flags_, flags.data(), flags.size(), hipMemcpyHostToDevice), "H2D merge flags", err)) ||
      (!list.empty() && !ok(hipMemcpy(rh_list_, list.data(), list.size() * 4, hipMemcpyHostToDevice), "H2D merge list", err)))
    return false;
  n_rh_ = uint32_t(list.size());
  tiles_known_ = true;
  return true;
}

bool RedHatMerge::launch(const RhInputs& in, hipStream_t st, std::string& err) {
  const DevMatches& raw = *in.raw;
  int dev = 0;
  if (!ok(hipGetDevice(&dev), "hipGetDevice", err)) return false;
  if (out_.cap < raw.cap || out_.m.dir_cap < in.n_tiles || dev != dev_) {
    release();
    dev_ = dev;
    const uint64_t cap = raw.cap;
    const uint32_t nt = std::max<uint32_t>(in.n_tiles, 1);
    void *p = nullptr, *q = nullptr, *r = nullptr, *s = nullptr, *t = nullptr, *c = nullptr, *u = nullptr, *v = nullptr;
    const bool good = ok(hipMalloc(&p, cap * 4), "hipMalloc(merged)", err) &&
                      ok(hipMalloc(&q, cap * 4), "hipMalloc(merged)", err) &&
                      ok(hipMalloc(&r, cap * 4), "hipMalloc(merged)", err) &&
                      ok(hipMalloc(&s, cap * 8), "hipMalloc(merged)", err) &&
                      ok(hipMalloc(&t, nt * sizeof(TileDir)), "hipMalloc(merged dir)", err) &&
                      ok(hipMalloc(&c, 64), "hipMalloc(merged ctl)", err) &&
                      ok(hipMalloc(&u, nt * 4), "hipMalloc(merge counts)", err) &&
                      ok(hipMalloc(&v, nt * 8), "hipMalloc(merge bases)", err);
    counts_ = static_cast<uint32_t*>(u);
    bases_ = static_cast<unsigned long long*>(v);
    out_.m.pkg = static_cast<uint32_t*>(p);
    out_.m.adv = static_cast<uint32_t*>(q);
    out_.base = static_cast<uint32_t*>(r);
    out_.grp = static_cast<uint2*>(s);
    out_.m.dir = static_cast<TileDir*>(t);
    out_.m.ctl = static_cast<unsigned long long*>(c);
    out_.m.cap = out_.cap = cap;
    out_.m.dir_cap = nt;
    if (!good) {
      release();
      return false;
    }
  }
  if (!ok(hipMemsetAsync(out_.m.ctl, 0, 64, st), "memset(merged ctl)", err)) return false;
  if (in.n_tiles == 0) return true;
  MergeArgs a{};
  a.dir = raw.dir;
  a.pkg = raw.pkg;
  a.adv = raw.adv;
  a.pk = in.pk;
  a.plats = in.plats;
  a.n_plats = in.n_plats;
  a.pkg_base = in.pkg_base;
  a.n = in.n;
  a.rk = in.rk;
  a.raw_cap = raw.cap;
  a.mdir = out_.m.dir;
  a.mpkg = out_.m.pkg;
  a.madv = out_.m.adv;
  a.mbase = out_.base;
  a.mgrp = out_.grp;
  a.mcap = out_.cap;
  a.mctl = out_.m.ctl;
  if (!tiles_known_) {
    err = "redhat merge: the batch's Red Hat tiles are not set (set_tiles)";
    return false;
  }
  const uint32_t nb_rh = (n_rh_ + kWaves - 1) / kWaves;  // a wave per Red Hat tile
  const uint32_t g_count = nb_rh + (in.n_tiles + kBlock - 1) / kBlock, g_emit = nb_rh + (in.n_tiles + kWaves - 1) / kWaves;
  hipLaunchKernelGGL(rh_count_kernel, dim3(g_count), dim3(kBlock), 0, st, a, counts_, flags_, rh_list_, n_rh_,
                     in.n_tiles);
  if (!ok(hipGetLastError(), "rh_count_kernel", err)) return false;
  size_t need = 0;
  if (!ok(rocprim::exclusive_scan(nullptr, need, counts_, bases_, 0ull, in.n_tiles,
                                  rocprim::plus<unsigned long long>(), st),
          "rocprim scan (size)", err))
    return false;
  if (need > scan_tmp_bytes_) {
    if (scan_tmp_) (void)hipFree(scan_tmp_);
    scan_tmp_ = nullptr;
    scan_tmp_bytes_ = 0;
    if (!ok(hipMalloc(&scan_tmp_, need), "hipMalloc(merge scan)", err)) return false;
    scan_tmp_bytes_ = need;
  }
  if (!ok(rocprim::exclusive_scan(scan_tmp_, need, counts_, bases_, 0ull, in.n_tiles,
                                  rocprim::plus<unsigned long long>(), st),
          "rocprim scan", err))
    return false;
  hipLaunchKernelGGL(rh_emit_kernel, dim3(g_emit), dim3(kBlock), 0, st, a, counts_, bases_, flags_, rh_list_, n_rh_,
                     in.n_tiles);
  return ok(hipGetLastError(), "rh_emit_kernel", err);
}

bool RedHatMerge::fetch(const RhInputs& in, std::vector<uint32_t>& pkg, std::vector<uint32_t>& adv,
                        std::vector<uint32_t>& base, std::vector<uint2>& grp, std::vector<uint32_t>& contrib,
                        hipStream_t st, std::string& err) {
  pkg.clear();
  adv.clear();
  base.clear();
  grp.clear();
  contrib.clear();
  unsigned long long ctl[8] = {}, rctl[8] = {};
  if (!ok(hipMemcpyAsync(ctl, out_.m.ctl, sizeof ctl, hipMemcpyDeviceToHost, st), "D2H merged ctl", err) ||
      !ok(hipMemcpyAsync(rctl, in.raw->ctl, sizeof rctl, hipMemcpyDeviceToHost, st), "D2H ctl", err) ||
      !ok(hipStreamSynchronize(st), "redhat merge", err))
    return false;
  if (ctl[3] & ERR_RH_ORDER) {
    err = "redhat merge: a Red Hat package's advisories are not grouped by VulnerabilityID";
    return false;
  }
  if (ctl[3] || rctl[0] > in.raw->cap || ctl[0] > out_.cap) {
    err = "redhat merge: the match buffer overflowed";
    return false;
  }
  const uint64_t n = ctl[0], nr = rctl[0];
  std::vector<TileDir> dir(in.n_tiles);
  std::vector<uint32_t> p(n), a(n), b(n);
  std::vector<uint2> g(n);
  contrib.resize(nr);
  if ((in.n_tiles && !ok(hipMemcpyAsync(dir.data(), out_.m.dir, in.n_tiles * sizeof(TileDir), hipMemcpyDeviceToHost, st),
                         "D2H merged dir", err)) ||
      (n && (!ok(hipMemcpyAsync(p.data(), out_.m.pkg, n * 4, hipMemcpyDeviceToHost, st), "D2H merged", err) ||
             !ok(hipMemcpyAsync(a.data(), out_.m.adv, n * 4, hipMemcpyDeviceToHost, st), "D2H merged", err) ||
             !ok(hipMemcpyAsync(b.data(), out_.base, n * 4, hipMemcpyDeviceToHost, st), "D2H merged", err) ||
             !ok(hipMemcpyAsync(g.data(), out_.grp, n * 8, hipMemcpyDeviceToHost, st), "D2H merged", err))) ||
      (nr && !ok(hipMemcpyAsync(contrib.data(), in.raw->adv, nr * 4, hipMemcpyDeviceToHost, st), "D2H contrib", err)) ||
      !ok(hipStreamSynchronize(st), "redhat merge", err))
    return false;
  pkg.reserve(n);
  adv.reserve(n);
  base.reserve(n);
  grp.reserve(n);
  for (const TileDir& d : dir)
    for (uint64_t i = d.base; i < d.base + d.count; i++) {
      pkg.push_back(p[i]);
      adv.push_back(a[i]);
      base.push_back(b[i]);
      grp.push_back(g[i]);
    }
  return true;
}

}  // namespace tvm
