// FillInfo decisions on the GPU (gfx950): the vulnerability-detail join of
// pkg/vulnerability/vulnerability.go:60-157 for a whole batch of detected
// vulnerabilities in one launch (tables and codes: vulninfo.h).
//
// One lane per detected vulnerability, 256 per workgroup:
//   drop-in path  (ITEMS): hash the vulnerability ID (FNV-1a + fmix64, common.h) from the
//                 item arena, linear-probe the ID index (slot hash and value loaded
//                 together), verify the ID with word compares against the 8-B aligned ID
//                 arena -> record;
//   batch path    (PAIRS): the match kernel's {package, advisory} pair -> the advisory's
//                 load-time resolved FillInfo input -> record (no strings at all);
// then both: status rule, one pass over the record's entry words (VendorSeverity pairs
// and per-source primary-URL picks) selecting data source -> GHSA -> NVD -> DB severity,
// and the URL kind.  Integer/byte work bound by memory latency; no MFMA.
#include "vulninfo.h"

#include <algorithm>

#include "common.h"

namespace tvm {

namespace {

constexpr int kFillTile = 256;

struct FillArgs {
  FillDev t;
  const uint4* items;    // ITEMS
  const uint8_t* arena;  // ITEMS: vulnerability-ID bytes
  const uint32_t* adv;   // PAIRS: the ordered match list's advisory column
  const uint32_t* base;  // PAIRS (merged Red Hat lists): the member whose Status / Severity the entry keeps
  const unsigned long long* n_dev;  // PAIRS: match count written by the match kernel
  uint64_t n;            // ITEMS: item count; PAIRS: pair-buffer capacity
  uint4* out;
  uint2* side;           // PAIRS (optional): the filter's hand-off word per pair
};

__device__ __forceinline__ uint32_t probe_id(const FillDev& t, const uint8_t* id, uint32_t n) {
  static_assert(kNameWords == 4, "the ID is packed into exactly four words");
  uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, cur = 0;  // first 32 bytes, memory order, zero padded
  uint64_t h = key_hash_seed(kVulnSeed);
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = id[i];
    h = key_hash_step(h, c);
    cur |= uint64_t(c) << (8 * (i & 7));
    if ((i & 7) == 7 || i + 1 == n) {  // registers only: no dynamically indexed array
      const uint32_t k = i >> 3;
      if (k == 0) w0 = cur;
      else if (k == 1) w1 = cur;
      else if (k == 2) w2 = cur;
      else if (k == 3) w3 = cur;
      cur = 0;
    }
  }
  h = key_hash_fin(h);
  for (uint64_t s = h & t.slot_mask;; s = (s + 1) & t.slot_mask) {
    const uint64_t sh = t.slot_hash[s];
    const uint4 sv = t.slot_val[s];
    if (sh == 0) return FILL_NOT_FOUND;
    if (sh != h || sv.y != n) continue;
    const uint64_t* y = reinterpret_cast<const uint64_t*>(t.id_arena + sv.x);
    const uint64_t y0 = y[0], y1 = y[1], y2 = y[2], y3 = y[3];  // one round trip (arena is padded)
    bool eq = n == 0 || y0 == w0;
    if (n > 8) eq &= y1 == w1;
    if (n > 16) eq &= y2 == w2;
    if (n > 24) eq &= y3 == w3;
    for (uint32_t i = 8 * kNameWords; eq && i < n; i++) eq = t.id_arena[sv.x + i] == id[i];
    if (eq) return sv.z;
  }
}

// r = t.recs[rec] (loaded by the caller, so a batch of pairs has its record loads in flight
// together); ignored when rec is FILL_NOT_FOUND
__device__ __forceinline__ uint4 decide_r(const FillDev& t, uint4 item, uint32_t rec, uint4 r) {
  // vulnerability.go:64-68: the status rule runs before the lookup
  uint32_t status = item.z & 0xFFu;
  if (item.z & FI_FIXED) status = 3;       // StatusFixed
  else if (status == 0) status = 2;        // StatusAffected
  uint4 o = make_uint4(FILL_NOT_FOUND, status, 0u | (SRC_NONE << 16), URL_NONE);
  if (rec == FILL_NOT_FOUND) return o;
  if (r.w & REC_BAD) return o;             // GetVulnerability decode error: logged, skipped
  o.x = rec;
  const uint32_t src = item.y >> 16;
  const uint32_t url_kind = (r.w >> REC_URL_SHIFT) & 0xFu;
  uint32_t v_src = 0xFFFFFFFFu, v_ghsa = 0xFFFFFFFFu, v_nvd = 0xFFFFFFFFu, ref = 0xFFFFFFFFu;
  // entries four at a time: the four loads are in flight together (an entry list is a few words)
  for (uint32_t i0 = 0; i0 < r.y; i0 += 4) {
    uint32_t ev[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) ev[u] = i0 + u < r.y ? t.ents[r.x + i0 + u] : 0u;
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      if (i0 + u >= r.y) break;
      const uint32_t e = ev[u];
      const uint32_t s = (e >> 16) & 0x7FFFu, v = e & 0xFFFFu;
      if (e & ENT_URL) {
        if (s == src) ref = v;
      } else {
        if (s == src) v_src = v;
        if (s == t.ghsa) v_ghsa = v;
        if (s == t.nvd) v_nvd = v;
      }
    }
  }
  uint32_t sev, ssrc = SRC_NONE;
  if (item.z & FI_SEV_SRC) sev = SEV_KEEP;                       // :90-101 package-specific
  else if (v_src != 0xFFFFFFFFu) sev = v_src, ssrc = src;        // :112-114
  else if (url_kind == URL_GHSA && v_ghsa != 0xFFFFFFFFu) sev = v_ghsa, ssrc = t.ghsa;  // :117-121
  else if (v_nvd != 0xFFFFFFFFu) sev = v_nvd, ssrc = t.nvd;      // :124-126
  else sev = r.z;                                                // :128-133
  o.z = sev | (ssrc << 16);
  if (url_kind != URL_NONE) o.w = url_kind << URL_KIND_SHIFT;    // :137-146
  else if (ref != 0xFFFFFFFFu) o.w = (URL_REF << URL_KIND_SHIFT) | ref;  // :148-155
  return o;
}

__device__ __forceinline__ uint4 decide(const FillDev& t, uint4 item, uint32_t rec) {
  return decide_r(t, item, rec, rec == FILL_NOT_FOUND ? make_uint4(0, 0, 0, 0) : t.recs[rec]);
}

// Drop-in path: one lane per item.
__global__ __launch_bounds__(kFillTile) void fill_items_kernel(FillArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * kFillTile + threadIdx.x;
  if (i >= a.n) return;
  const uint4 item = a.items[i];
  a.out[i] = decide(a.t, item, probe_id(a.t, a.arena + item.x, item.y & 0xFFFFu));
}

// Batch path: grid-stride over the match kernel's pair buffer; the pair count is read on
// the device (no host round trip between the two launches).
// kU pairs per lane per step, each level of the pair -> advisory item -> record chain loaded
// for all of them before the next level is used (the chain is latency-bound: one pair per
// lane kept one gather in flight).
constexpr int kFillU = 8;
__global__ __launch_bounds__(kFillTile) void fill_pairs_kernel(FillArgs a) {
  const uint64_t n = *a.n_dev < a.n ? *a.n_dev : a.n;
  const uint64_t stride = uint64_t(gridDim.x) * kFillTile * kFillU;
  for (uint64_t i0 = uint64_t(blockIdx.x) * kFillTile * kFillU + threadIdx.x; i0 < n; i0 += stride) {
    uint32_t adv[kFillU], rank[kFillU];
    uint4 item[kFillU], r[kFillU];
#pragma unroll
    for (int k = 0; k < kFillU; k++) {
      const uint64_t i = i0 + uint64_t(k) * kFillTile;
      adv[k] = i < n ? a.adv[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < kFillU; k++) {
      const bool known = adv[k] < a.t.n_advs;
      item[k] = known ? a.t.adv_items[adv[k]] : make_uint4(0, SRC_NONE << 16, 0, FILL_NOT_FOUND);
      rank[k] = (a.side && known) ? a.t.adv_rank[adv[k]].x : 0xFFFFFFFFu;
    }
    if (a.base) {  // merged Red Hat entry: FixedVersion of adv (the representative), the rest of base
#pragma unroll
      for (int k = 0; k < kFillU; k++) {
        const uint64_t i = i0 + uint64_t(k) * kFillTile;
        const uint32_t b = i < n ? a.base[i] : adv[k];
        if (b != adv[k] && b < a.t.n_advs) {
          const uint32_t fixed = item[k].z & FI_FIXED;
          item[k] = a.t.adv_items[b];
          item[k].z = (item[k].z & ~FI_FIXED) | fixed;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kFillU; k++)
      r[k] = item[k].w != FILL_NOT_FOUND ? a.t.recs[item[k].w] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < kFillU; k++) {
      const uint64_t i = i0 + uint64_t(k) * kFillTile;
      if (i >= n) break;
      const uint4 o = decide_r(a.t, item[k], item[k].w, r[k]);
      a.out[i] = o;
      if (a.side)  // result.Filter reads this word, not the decision (filter.hip filter_mark)
        a.side[i] = make_uint2(rank[k], fill_pair_severity(o, item[k]) | ((o.y & 31u) << 8));
    }
  }
}

bool hip_ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

template <class T>
bool upload(const std::vector<T>& v, const T** dst, std::vector<void*>& allocs, uint64_t& bytes, std::string& err) {
  const size_t n = std::max<size_t>(v.size(), 1) * sizeof(T);
  void* p = nullptr;
  if (!hip_ok(hipMalloc(&p, n), "hipMalloc(fill tables)", err)) return false;
  allocs.push_back(p);
  if (!v.empty() && !hip_ok(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy(fill)", err))
    return false;
  bytes += n;
  *dst = static_cast<const T*>(p);
  return true;
}

}  // namespace

FillEngine::~FillEngine() {
  (void)hipSetDevice(dev_);
  for (void* p : allocs_) (void)hipFree(p);
  if (stream_) (void)hipStreamDestroy(stream_);
  delete d_;
}

FillEngine* FillEngine::open(const VulnTable& t, int device, std::string& err) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    err = "no HIP device available (trivy_amd requires an MI355X / gfx950 GPU)";
    return nullptr;
  }
  auto* f = new FillEngine();
  f->dev_ = device;
  f->t_ = &t;
  f->d_ = new FillDev();
  FillDev& d = *f->d_;
  d.slot_mask = t.slot_mask;
  d.n_advs = uint32_t(t.adv_items.size());
  d.ghsa = t.ghsa_id();
  d.nvd = t.nvd_id();
  bool ok = hip_ok(hipSetDevice(device), "hipSetDevice", err) &&
            hip_ok(hipStreamCreateWithFlags(&f->stream_, hipStreamNonBlocking), "hipStreamCreate", err) &&
            upload(t.slot_hash, &d.slot_hash, f->allocs_, f->table_bytes_, err) &&
            upload(t.slot_val, &d.slot_val, f->allocs_, f->table_bytes_, err) &&
            upload(t.id_arena, &d.id_arena, f->allocs_, f->table_bytes_, err) &&
            upload(t.recs, &d.recs, f->allocs_, f->table_bytes_, err) &&
            upload(t.ents, &d.ents, f->allocs_, f->table_bytes_, err) &&
            upload(t.adv_items, &d.adv_items, f->allocs_, f->table_bytes_, err) &&
            upload(t.adv_rank, &d.adv_rank, f->allocs_, f->table_bytes_, err);
  if (!ok) {
    delete f;
    return nullptr;
  }
  return f;
}

bool FillEngine::run_host(const std::vector<uint4>& items, const std::vector<uint8_t>& arena, std::vector<uint4>& out,
                          std::string& err) {
  out.assign(items.size(), make_uint4(0, 0, 0, 0));
  if (items.empty()) return true;
  for (const uint4& it : items)  // the kernel reads [x, x + len) of the arena
    if (uint64_t(it.x) + (it.y & 0xFFFFu) > arena.size()) {
      err = "fill: item outside the ID arena";
      return false;
    }
  if (!hip_ok(hipSetDevice(dev_), "hipSetDevice", err)) return false;
  void *di = nullptr, *da = nullptr, *dout = nullptr;
  const size_t ni = items.size() * sizeof(uint4), na = std::max<size_t>(arena.size(), 1);
  bool ok = hip_ok(hipMallocAsync(&di, ni, stream_), "hipMalloc(fill items)", err) &&
            hip_ok(hipMallocAsync(&da, na, stream_), "hipMalloc(fill arena)", err) &&
            hip_ok(hipMallocAsync(&dout, ni, stream_), "hipMalloc(fill out)", err) &&
            hip_ok(hipMemcpyAsync(di, items.data(), ni, hipMemcpyHostToDevice, stream_), "hipMemcpy(fill items)", err) &&
            (arena.empty() ||
             hip_ok(hipMemcpyAsync(da, arena.data(), arena.size(), hipMemcpyHostToDevice, stream_), "hipMemcpy(arena)", err));
  if (ok) {
    FillArgs a{};
    a.t = *d_;
    a.items = static_cast<const uint4*>(di);
    a.arena = static_cast<const uint8_t*>(da);
    a.n = items.size();
    a.out = static_cast<uint4*>(dout);
    const uint32_t blocks = uint32_t((items.size() + kFillTile - 1) / kFillTile);
    hipLaunchKernelGGL(fill_items_kernel, dim3(blocks), dim3(kFillTile), 0, stream_, a);
    ok = hip_ok(hipGetLastError(), "fill_kernel launch", err) &&
         hip_ok(hipMemcpyAsync(out.data(), dout, ni, hipMemcpyDeviceToHost, stream_), "hipMemcpy(fill out)", err);
  }
  for (void* p : {di, da, dout})
    if (p) (void)hipFreeAsync(p, stream_);
  return hip_ok(hipStreamSynchronize(stream_), "fill sync", err) && ok;
}

bool FillEngine::launch_pairs(const uint32_t* adv, const uint32_t* base, const unsigned long long* n_dev, uint64_t cap,
                              uint4* out, uint2* side, hipStream_t stream, std::string& err) {
  if (cap == 0) return true;
  FillArgs a{};
  a.t = *d_;
  a.adv = adv;
  a.base = base;
  a.n_dev = n_dev;
  a.n = cap;
  a.out = out;
  a.side = side;
  // enough waves to cover the chip many times over, capped so the stride loop does the rest
  const uint64_t blocks = std::min<uint64_t>((cap + kFillTile * kFillU - 1) / (kFillTile * kFillU), 256ull * 32);
  hipLaunchKernelGGL(fill_pairs_kernel, dim3(uint32_t(blocks)), dim3(kFillTile), 0, stream, a);
  return hip_ok(hipGetLastError(), "fill_kernel launch", err);
}

uint64_t FillEngine::pair_bytes(const std::vector<uint32_t>& adv, const std::vector<uint32_t>& base) const {
  // per pair: its advisory index (4) + the advisory's item (16) + the record (16) + its
  // entry words (4 each) + the decision (16) + the side word (8); merged lists: + the
  // base index (4) and, where it differs, the base's item (16); no cache-reuse credit
  uint64_t b = 0;
  for (size_t i = 0; i < adv.size(); i++) {
    uint32_t a = adv[i];
    b += 4 + 16 + 16 + 8;
    if (!base.empty()) {
      b += 4;
      if (base[i] != a) b += 16, a = base[i];
    }
    if (a < t_->adv_items.size()) {
      const uint32_t rec = t_->adv_items[a].w;
      if (rec != FILL_NOT_FOUND) b += 16 + 4ull * t_->recs[rec].y;
    }
  }
  return b;
}

}  // namespace tvm
