// End-to-end pipelined match pass (pipeline.h): the batch's DMA upload, the match kernels
// and the order kernel's direct writes of the result into host memory overlap chunk by chunk.  Every buffer is sized once in prepare(); a pass
// allocates nothing.
#include "pipeline.h"

#include <algorithm>
#include <cstring>

namespace tvm {

namespace {

bool ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

}  // namespace

Pipeline::~Pipeline() { release(); }

void Pipeline::release() {
  if (dev_ < 0) return;
  (void)hipSetDevice(dev_);
  if (s_k_) (void)hipStreamSynchronize(s_k_);
  if (s_h2d_) (void)hipStreamSynchronize(s_h2d_);
  Engine::free_batch(dev_, db_);
  Engine::free_matches(dev_, m_);
  for (void* p : {static_cast<void*>(csr_adv_d_), static_cast<void*>(row_end_d_), static_cast<void*>(status_d_),
                  static_cast<void*>(tickets_d_)})
    if (p) (void)hipFree(p);
  for (void* p : {static_cast<void*>(adv_h_), static_cast<void*>(row_end_h_), static_cast<void*>(ctl_h_)})
    if (p) (void)hipHostFree(p);
  for (void* p : registered_) (void)hipHostUnregister(p);
  registered_.clear();
  for (hipEvent_t e : ev_h_) (void)hipEventDestroy(e);
  ev_h_.clear();
  for (hipStream_t s : {s_h2d_, s_k_})
    if (s) (void)hipStreamDestroy(s);
  s_h2d_ = s_k_ = nullptr;
  adv_hd_ = row_end_hd_ = nullptr;
  csr_adv_d_ = row_end_d_ = nullptr;
  status_d_ = tickets_d_ = nullptr;
  adv_h_ = row_end_h_ = nullptr;
  ctl_h_ = nullptr;
  prepared_ = false;
  dev_ = -1;
}

bool Pipeline::prepare(Engine& eng, const HostBatch& hb, uint64_t match_cap, uint32_t chunk_packages,
                       std::string& err) {
  release();

  dev_ = eng.device();
  (void)hipSetDevice(dev_);
  const uint32_t n_tiles = hb.n_tiles();
  const uint32_t chunk_tiles = std::max<uint32_t>(1, (chunk_packages + kTile - 1) / kTile);
  bounds_.clear();
  for (uint32_t t = 0; t < n_tiles; t += chunk_tiles) bounds_.push_back(t);
  bounds_.push_back(n_tiles);
  if (n_tiles == 0) bounds_ = {0, 0};
  const uint32_t nc = uint32_t(bounds_.size() - 1);
  toff_ = hb.tile_off;  // per 64-package group, + the arena end, padded to whole tiles
  toff_.resize(size_t(n_tiles) * kGroupsPerTile + 1, hb.arena.size());
  cap_ = std::max<uint64_t>(match_cap, 1);
  if (cap_ >= (1ull << 32)) {
    err = "pipeline: row ends are 32-bit; split the batch below 2^32 matches";
    return false;
  }
  ev_h_.resize(nc);
  for (hipEvent_t& e : ev_h_)
    if (!ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate", err)) return false;
  if (!ok(hipStreamCreateWithFlags(&s_h2d_, hipStreamNonBlocking), "hipStreamCreate", err) ||
      !ok(hipStreamCreateWithFlags(&s_k_, hipStreamNonBlocking), "hipStreamCreate", err))
    return false;
  // pin the caller's host arrays in place: the copies are DMA from them, no staging memcpy
  auto reg = [&](const void* p, size_t bytes) {
    if (!bytes) return true;
    if (!ok(hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault), "hipHostRegister", err)) return false;
    registered_.push_back(const_cast<void*>(p));
    return true;
  };
  if (!reg(hb.pk.data(), hb.pk.size() * sizeof(uint2)) || !reg(hb.arena.data(), hb.arena.size()) ||
      !reg(toff_.data(), toff_.size() * 8) || !reg(hb.attr.data(), hb.attr.size() * sizeof(uint2)))
    return false;
  if (!eng.alloc_batch(hb, db_, err) || !eng.alloc_matches(cap_, db_.n, m_, err)) return false;
  if (!hb.cpe_bits.empty() && hb.cpe_words) {  // CPE sets: small, copied once here
    void* p = nullptr;
    if (!ok(hipMalloc(&p, hb.cpe_bits.size() * 4), "hipMalloc(cpe sets)", err) ||
        !ok(hipMemcpy(p, hb.cpe_bits.data(), hb.cpe_bits.size() * 4, hipMemcpyHostToDevice), "H2D cpe", err))
      return false;
    db_.cpe_bits = static_cast<uint32_t*>(p);
    db_.cpe_words = hb.cpe_words;
    db_.n_cpe_sets = uint32_t(hb.cpe_bits.size() / hb.cpe_words);
  }
  const size_t n = std::max<size_t>(hb.pk.size(), 1);
  // CSR buffers padded to whole 16-byte units (the result move copies units)
  const size_t cap4 = (cap_ + 3) & ~size_t(3), n4 = (size_t(n_tiles) * kTile + 3) & ~size_t(3);
  void* p = nullptr;
  if (!ok(hipMalloc(&p, cap4 * 4), "hipMalloc(csr)", err)) return false;
  csr_adv_d_ = static_cast<uint32_t*>(p);
  if (!ok(hipMalloc(&p, std::max<size_t>(n4, 4) * 4), "hipMalloc(row ends)", err)) return false;
  row_end_d_ = static_cast<uint32_t*>(p);
  if (!ok(hipMalloc(&p, std::max<size_t>(n_tiles, 1) * 8), "hipMalloc(status)", err)) return false;
  status_d_ = static_cast<unsigned long long*>(p);
  if (!ok(hipMalloc(&p, std::max<size_t>(nc, 1) * 8), "hipMalloc(tickets)", err)) return false;
  tickets_d_ = static_cast<unsigned long long*>(p);
  // the result lives in pinned host memory that the result move writes directly over PCIe
  // (measured, profiles/r03/pcie_probe.txt: kernel stores to host memory 55 GB/s, a DMA
  // device-to-host copy 28.6 GB/s; the DMA engine then only carries the batch upward)
  if (!ok(hipHostMalloc(&p, cap4 * 4, hipHostMallocDefault), "hipHostMalloc(adv)", err)) return false;
  adv_h_ = static_cast<uint32_t*>(p);
  if (!ok(hipHostMalloc(&p, std::max<size_t>(n4, 4) * 4, hipHostMallocDefault), "hipHostMalloc(row ends)", err)) return false;
  row_end_h_ = static_cast<uint32_t*>(p);
  if (!ok(hipHostGetDevicePointer(&p, adv_h_, 0), "hipHostGetDevicePointer(adv)", err)) return false;
  adv_hd_ = static_cast<uint32_t*>(p);
  if (!ok(hipHostGetDevicePointer(&p, row_end_h_, 0), "hipHostGetDevicePointer(row ends)", err)) return false;
  row_end_hd_ = static_cast<uint32_t*>(p);
  if (!ok(hipHostMalloc(&p, 64, hipHostMallocDefault), "hipHostMalloc(ctl)", err)) return false;
  ctl_h_ = static_cast<unsigned long long*>(p);
  prepared_ = true;
  return true;
}

bool Pipeline::run(Engine& eng, const HostBatch& hb, uint64_t& total, int64_t& err_pkg, uint64_t& err_bits,
                   std::string& err) {
  total = 0;
  err_pkg = -1;
  err_bits = 0;
  h2d_ = d2h_ = 0;
  if (!prepared_ || db_.n != hb.pk.size()) {
    err = "pipeline: prepare() the batch first";
    return false;
  }
  (void)hipSetDevice(dev_);
  const uint32_t nc = chunks();
  const uint32_t n = db_.n;
  if (!ok(hipMemsetAsync(m_.ctl, 0, 64, s_k_), "memset(ctl)", err) ||
      !ok(hipMemsetAsync(status_d_, 0, std::max<size_t>(db_.n_tiles, 1) * 8, s_k_), "memset(status)", err) ||
      !ok(hipMemsetAsync(tickets_d_, 0, std::max<size_t>(nc, 1) * 8, s_k_), "memset(tickets)", err))
    return false;
  // Per chunk: its upload on the copy stream; behind it, on the kernel stream, one match
  // launch whose first workgroups move the previous chunk's result out, then the order
  // kernel.  All work is queued up front (measured: the calls never block); the host waits
  // once, at the end.
  auto copy_args = [&](uint32_t c) {
    CopyOutArgs ca;
    ca.row_end = row_end_d_;
    ca.csr_adv = csr_adv_d_;
    ca.row_end_h = reinterpret_cast<uint4*>(row_end_hd_);
    ca.adv_h = reinterpret_cast<uint4*>(adv_hd_);
    ca.p0 = bounds_[c] * kTile;
    ca.p1 = std::min<uint32_t>(bounds_[c + 1] * kTile, n);
    ca.cap = cap_;
    return ca;
  };
  int64_t prev = -1;  // the last chunk matched, whose result has not been moved yet
  for (uint32_t c = 0; c < nc; c++) {
    const uint32_t t0 = bounds_[c], t1 = bounds_[c + 1];
    if (t1 == t0) continue;
    const size_t p0 = size_t(t0) * kTile, p1 = std::min<size_t>(size_t(t1) * kTile, n);
    const size_t g0 = size_t(t0) * kGroupsPerTile, g1 = size_t(t1) * kGroupsPerTile;
    const uint64_t a0 = toff_[g0], a1 = toff_[g1];
    if (!ok(hipMemcpyAsync(db_.pk + p0, hb.pk.data() + p0, (p1 - p0) * sizeof(uint2), hipMemcpyHostToDevice, s_h2d_),
            "H2D packages", err) ||
        !ok(hipMemcpyAsync(db_.tile_off + g0, toff_.data() + g0, (g1 - g0 + 1) * 8, hipMemcpyHostToDevice, s_h2d_),
            "H2D group offsets", err) ||
        (a1 > a0 && !ok(hipMemcpyAsync(db_.arena + a0, hb.arena.data() + a0, a1 - a0, hipMemcpyHostToDevice, s_h2d_),
                        "H2D strings", err)) ||
        (!hb.attr.empty() &&
         !ok(hipMemcpyAsync(db_.attr + p0, hb.attr.data() + p0, (p1 - p0) * sizeof(uint2), hipMemcpyHostToDevice, s_h2d_),
             "H2D attributes", err)) ||
        !ok(hipEventRecord(ev_h_[c], s_h2d_), "hipEventRecord", err) ||
        !ok(hipStreamWaitEvent(s_k_, ev_h_[c], 0), "hipStreamWaitEvent", err))
      return false;
    h2d_ += (p1 - p0) * sizeof(uint2) + (g1 - g0 + 1) * 8 + (a1 - a0) + (hb.attr.empty() ? 0 : (p1 - p0) * sizeof(uint2));
    const CopyOutArgs prev_co = prev >= 0 ? copy_args(uint32_t(prev)) : CopyOutArgs{};
    if (!eng.launch_tiles(db_, m_, t0, t1, s_k_, s_k_, nullptr, err, prev >= 0 ? &prev_co : nullptr)) return false;
    OrderArgs oa;
    oa.dir = m_.dir;
    oa.pkg = m_.pkg;
    oa.adv = m_.adv;
    oa.csr_adv = csr_adv_d_;
    oa.row_end = row_end_d_;
    oa.cap = cap_;
    oa.status = status_d_;
    oa.ticket = tickets_d_ + c;
    oa.t0 = t0;
    oa.n = n;
    oa.pkg_base = db_.pkg_base;
    launch_order(t1 - t0, s_k_, oa);
    if (!ok(hipGetLastError(), "order kernel launch", err)) return false;
    prev = c;
  }
  if (prev >= 0) {
    launch_copy_out(s_k_, copy_args(uint32_t(prev)));
    if (!ok(hipGetLastError(), "copy-out kernel launch", err)) return false;
  }
  if (!ok(hipMemcpyAsync(ctl_h_, m_.ctl, 64, hipMemcpyDeviceToHost, s_k_), "D2H ctl", err) ||
      !ok(hipStreamSynchronize(s_k_), "pipeline", err))
    return false;
  d2h_ = uint64_t(n) * 4 + std::min<uint64_t>(ctl_h_[0], cap_) * 4;
  total = ctl_h_[0];
  err_pkg = ctl_h_[1] ? int64_t(n - ctl_h_[1]) : -1;
  err_bits = ctl_h_[3];
  return true;
}

}  // namespace tvm
