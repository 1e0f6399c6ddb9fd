// End-to-end pipelined match pass (pipeline.h): the batch's DMA upload, the match kernels
// and the order kernel's direct writes of the result into host memory overlap chunk by chunk.  Every buffer is sized once in prepare(); a pass
// allocates nothing.
#include "pipeline.h"
#include "host_par.h"
#include "pool.h"
#include "wire.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>

namespace tvm {

namespace {

bool ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

std::mutex& enc_mu() {
  static std::mutex m;
  return m;
}
std::vector<std::unique_ptr<WireEncoder>>& enc_pool() {
  static auto* v = new std::vector<std::unique_ptr<WireEncoder>>();  // never destroyed (static teardown)
  return *v;
}

__device__ __forceinline__ void copy_bytes(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, uint32_t n) {
  for (uint32_t k = 0; k < n; k += 8) {
    uint8_t t[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) t[u] = k + u < n ? s[k + u] : 0;
#pragma unroll
    for (uint32_t u = 0; u < 8; u++)
      if (k + u < n) d[k + u] = t[u];
  }
}

struct UnpackArgs {
  const uint8_t* wire;
  const uint32_t* nref;
  const uint32_t* vref;
  const uint16_t* lens;
  const uint8_t* plat;
  const uint64_t* toff;
  const uint2* attr_in;
  const uint32_t* ptab;
  uint2* pk;
  uint64_t* tile_off;
  uint8_t* arena;
  uint2* attr;
  uint32_t p0, m, g0, groups;
  uint64_t arena_cap;       // bytes of the batch arena (guard)
  uint64_t wire_cap;        // bytes of the device wire buffer (guard)
  unsigned long long* ctl;  // ctl[3] |= ERR_BOUNDS on a guard hit
};

// One chunk of the transport form -> the batch's own arrays in HBM (pk, tile_off, arena,
// attr: exactly what a raw upload would have put there).  One wavefront per 64-package
// group: the group's arena offset comes with the chunk, each package's offset within it is
// a wave scan of the lengths, and every lane copies its name and version bytes from their
// first occurrence in the wire buffer.
__global__ __launch_bounds__(256) void unpack_kernel(UnpackArgs a) {
  const uint32_t lane = threadIdx.x & 63, gl = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gl >= a.groups) return;  // whole wavefronts
  const uint32_t i = gl * 64 + lane;
  uint32_t nl = 0, vl = 0, nr = 0, vr = 0;
  if (i < a.m) {
    const uint32_t ln = a.lens[i];
    nl = ln & 255u;
    vl = ln >> 8;
    nr = a.nref[i];
    vr = a.vref[i];
    a.pk[a.p0 + i] = make_uint2(a.ptab[a.plat[i]], nl | (vl << 16));
    if (a.attr) a.attr[a.p0 + i] = a.attr_in[i];
  }
  const uint64_t g_off = a.toff[gl];
  if (lane == 0) {
    a.tile_off[a.g0 + gl] = g_off;
    if (gl + 1 == a.groups) a.tile_off[a.g0 + gl + 1] = a.toff[gl + 1];  // the next chunk's first group: read by this chunk's last tile
  }
  const uint32_t len = nl + vl;
  uint32_t x = len;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= uint32_t(o)) x += y;
  }
  // guard (never expected: build_wire and alloc_batch size both sides): an out-of-range
  // reference or destination fails the pass instead of touching memory
  const uint64_t dst = g_off + (x - len);
  if (dst + len > a.arena_cap || uint64_t(nr) + nl > a.wire_cap || uint64_t(vr) + vl > a.wire_cap) {
    atomicOr(a.ctl + 3, (unsigned long long)ERR_BOUNDS);
    return;
  }
  // 8 loads in flight per lane before any store (the wire and the arena never overlap)
  uint8_t* __restrict__ d = a.arena + dst;
  copy_bytes(d, a.wire + nr, nl);
  copy_bytes(d + nl, a.wire + vr, vl);
}

}  // namespace

// Encoders are kept between batches (their per-package arrays only grow): a fresh batch's
// preparation then touches no new pages.
static WireEncoder* take_encoder() {
  std::lock_guard<std::mutex> lk(enc_mu());
  auto& v = enc_pool();
  if (v.empty()) return new WireEncoder();
  WireEncoder* e = v.back().release();
  v.pop_back();
  return e;
}

void release_encoders() {
  std::lock_guard<std::mutex> lk(enc_mu());
  enc_pool().clear();
}

static void give_encoder(WireEncoder* e) {
  e->clear();
  std::lock_guard<std::mutex> lk(enc_mu());
  auto& v = enc_pool();
  if (v.size() < 4) v.emplace_back(e);
  else delete e;
}

bool Pipeline::build_wire(const HostBatch& hb, std::string& err) {
  const auto start = std::chrono::steady_clock::now();
  wc_.clear();
  std::unique_ptr<WireEncoder, void (*)(WireEncoder*)> enc(take_encoder(), give_encoder);
  if (!enc->plan(hb, toff_, bounds_, host_threads(), err)) return err.empty();  // no form: the batch goes raw
  const uint64_t bytes = std::max<uint64_t>(enc->bytes(), 16);
  if (!(wire_h_ = static_cast<uint8_t*>(pool_host_get(bytes, "hipHostMalloc(transport form)", err))) ||
      !(wire_d_ = static_cast<uint8_t*>(pool_device_get(dev_, bytes, "hipMalloc(transport form)", err))))
    return false;
  wire_bytes_ = bytes;
  const auto& ptab = enc->platforms();
  void* p = pool_device_get(dev_, ptab.size() * 4, "hipMalloc(platform table)", err);
  if (!p) return false;
  ptab_d_ = static_cast<uint32_t*>(p);
  if (!ok(hipMemcpy(p, ptab.data(), ptab.size() * 4, hipMemcpyHostToDevice), "H2D platform table", err)) return false;
  enc->emit(wire_h_);
  wc_ = enc->chunks();
  encode_us_ = uint64_t(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - start).count());
  return true;
}

// The raw form: the batch's arrays copied once into one pinned staging block (round 3
// pinned the caller's std::vector storage in place with hipHostRegister; heap vectors are
// not page-aligned, so a registration covered neighbouring heap objects' pages and two of a
// batch's registrations could share a page - the staging copy keeps the pinned range owned).
bool Pipeline::stage_raw(const HostBatch& hb, std::string& err) {
  const size_t b_pk = align16(hb.pk.size() * sizeof(uint2)), b_toff = align16(toff_.size() * 8),
               b_arena = align16(hb.arena.size()), b_attr = align16(hb.attr.size() * sizeof(uint2));
  void* p = pool_host_get(std::max<size_t>(b_pk + b_toff + b_arena + b_attr, 16), "hipHostMalloc(raw staging)", err);
  if (!p) return false;
  raw_h_ = static_cast<uint8_t*>(p);
  raw_pk_ = reinterpret_cast<uint2*>(raw_h_);
  raw_toff_ = reinterpret_cast<uint64_t*>(raw_h_ + b_pk);
  raw_arena_ = raw_h_ + b_pk + b_toff;
  raw_attr_ = reinterpret_cast<uint2*>(raw_h_ + b_pk + b_toff + b_arena);
  raw_staged_ = false;  // the first pass copies each chunk just before its upload (stage_chunk)
  return true;
}

// One chunk's slices of the batch arrays into the pinned staging block, on the host threads
// while the GPU works on the chunks before it (round 4: prepare copied the whole batch
// first, ~3 ms of the ~7 ms a fresh 4M-package batch took).
void Pipeline::stage_chunk(const HostBatch& hb, size_t p0, size_t p1, size_t g0, size_t g1, uint64_t a0, uint64_t a1) {
  struct Part {
    void* dst;
    const void* src;
    size_t bytes;
  };
  Part parts[4] = {{raw_pk_ + p0, hb.pk.data() + p0, (p1 - p0) * sizeof(uint2)},
                   {raw_toff_ + g0, toff_.data() + g0, (g1 - g0 + 1) * 8},
                   {raw_arena_ + a0, hb.arena.data() + a0, size_t(a1 - a0)},
                   {raw_attr_ + p0, hb.attr.empty() ? nullptr : hb.attr.data() + p0,
                    hb.attr.empty() ? 0 : (p1 - p0) * sizeof(uint2)}};
  constexpr size_t kPiece = size_t(256) << 10;  // many more pieces than threads: even shares
  std::vector<std::pair<int, size_t>> pieces;  // (part, offset)
  for (int k = 0; k < 4; k++)
    for (size_t o = 0; o < parts[k].bytes; o += kPiece) pieces.emplace_back(k, o);
  WorkerPool::get().parallel_for(pieces.size(), [&](size_t i) {
    const Part& pt = parts[pieces[i].first];
    const size_t o = pieces[i].second;
    std::memcpy(static_cast<char*>(pt.dst) + o, static_cast<const char*>(pt.src) + o, std::min(kPiece, pt.bytes - o));
  });
}

Pipeline::~Pipeline() { release(); }

void Pipeline::release() {
  if (dev_ < 0) return;
  (void)hipSetDevice(dev_);
  if (s_k_) (void)hipStreamSynchronize(s_k_);
  if (s_h2d_) (void)hipStreamSynchronize(s_h2d_);
  if (s_d2h_) (void)hipStreamSynchronize(s_d2h_);
  // every block goes back to the process-wide cache (pool.h): the streams are drained
  Engine::free_batch(dev_, db_, true);
  Engine::free_matches(dev_, m_, true);
  for (void* p : {static_cast<void*>(chunk_base_d_), static_cast<void*>(wire_d_), static_cast<void*>(ptab_d_),
                  static_cast<void*>(row_end_d_)})
    pool_device_put(dev_, p);
  for (void* p : {static_cast<void*>(wire_h_), static_cast<void*>(raw_h_), static_cast<void*>(adv_h_),
                  static_cast<void*>(row_end_h_), static_cast<void*>(ctl_h_)})
    pool_host_put(p);
  wire_h_ = nullptr;
  raw_h_ = nullptr;
  wire_bytes_ = 0;
  wire_d_ = nullptr;
  ptab_d_ = nullptr;
  wc_.clear();
  encode_us_ = 0;
  for (hipEvent_t e : ev_h_) (void)hipEventDestroy(e);
  for (hipEvent_t e : ev_k_) (void)hipEventDestroy(e);
  ev_h_.clear();
  ev_k_.clear();
  row_end_d_ = nullptr;
  for (hipStream_t s : {s_h2d_, s_k_, s_d2h_})
    if (s) (void)hipStreamDestroy(s);
  s_h2d_ = s_k_ = s_d2h_ = nullptr;
  adv_hd_ = row_end_hd_ = nullptr;
  chunk_base_d_ = nullptr;
  adv_h_ = row_end_h_ = nullptr;
  ctl_h_ = nullptr;
  prepared_ = false;
  dev_ = -1;
}

bool Pipeline::prepare(Engine& eng, const HostBatch& hb, uint64_t match_cap, uint32_t chunk_packages, bool transport,
                       bool packed, std::string& err) {
  release();
  const auto start = std::chrono::steady_clock::now();
  dev_ = eng.device();
  (void)hipSetDevice(dev_);
  const uint32_t n_tiles = hb.n_tiles();
  const uint32_t chunk_tiles = std::max<uint32_t>(1, (chunk_packages + kTile - 1) / kTile);
  bounds_.clear();
  // A batch of several chunks starts and ends with a quarter chunk: the first match launch
  // waits for one upload and the last result move runs alone, so short first and last
  // chunks shorten the pipeline's fill and drain (TVM_PIPE_NORAMP=1: equal chunks)
  static const bool no_ramp = std::getenv("TVM_PIPE_NORAMP") != nullptr;
  const uint32_t q = std::max<uint32_t>(1, chunk_tiles / 4);
  if (!no_ramp && n_tiles >= 3 * chunk_tiles) {
    uint32_t t = 0;
    bounds_.push_back(0);
    t += q;
    bounds_.push_back(t);
    while (n_tiles - t > chunk_tiles + q) {
      t += chunk_tiles;
      bounds_.push_back(t);
    }
    if (n_tiles - t > q) bounds_.push_back(n_tiles - q);
    bounds_.push_back(n_tiles);
  } else {
    for (uint32_t t = 0; t < n_tiles; t += chunk_tiles) bounds_.push_back(t);
    bounds_.push_back(n_tiles);
  }
  if (n_tiles == 0) bounds_ = {0, 0};
  const uint32_t nc = uint32_t(bounds_.size() - 1);
  toff_.assign(hb.tile_off.begin(), hb.tile_off.end());  // per 64-package group, + the arena end, padded to whole tiles
  toff_.resize(size_t(n_tiles) * kGroupsPerTile + 1, hb.arena.size());
  cap_ = std::max<uint64_t>(match_cap, 1);
  packed_ = packed;
  if (cap_ >= (1ull << 32)) {
    err = "pipeline: row ends are 32-bit; split the batch below 2^32 matches";
    return false;
  }
  ev_h_.resize(nc);
  ev_k_.resize(nc);
  for (hipEvent_t& e : ev_k_)
    if (!ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate", err)) return false;
  for (hipEvent_t& e : ev_h_)
    if (!ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate", err)) return false;
  if (!ok(hipStreamCreateWithFlags(&s_h2d_, hipStreamNonBlocking), "hipStreamCreate", err) ||
      !ok(hipStreamCreateWithFlags(&s_d2h_, hipStreamNonBlocking), "hipStreamCreate", err) ||
      !ok(hipStreamCreateWithFlags(&s_k_, hipStreamNonBlocking), "hipStreamCreate", err))
    return false;
  if (transport && !build_wire(hb, err)) return false;
  if (wc_.empty() && !stage_raw(hb, err)) return false;
  if (!eng.alloc_batch(hb, db_, err, true) || !eng.alloc_matches(cap_, db_.n, m_, err, true)) return false;
  if (!hb.cpe_bits.empty() && hb.cpe_words) {  // CPE sets: small, copied once here
    void* p = nullptr;
    if (!ok(hipMalloc(&p, hb.cpe_bits.size() * 4), "hipMalloc(cpe sets)", err) ||
        !ok(hipMemcpy(p, hb.cpe_bits.data(), hb.cpe_bits.size() * 4, hipMemcpyHostToDevice), "H2D cpe", err))
      return false;
    db_.cpe_bits = static_cast<uint32_t*>(p);
    db_.cpe_words = hb.cpe_words;
    db_.n_cpe_sets = uint32_t(hb.cpe_bits.size() / hb.cpe_words);
  }
  // CSR buffers padded to whole 16-byte units (the result move copies units)
  const size_t cap4 = (cap_ + 3) & ~size_t(3), n4 = (size_t(n_tiles) * kTile + 3) & ~size_t(3);
  adv_units_ = cap4 / 4;
  row_end_units_ = std::max<size_t>(n4, 4) / 4;
  void* p = nullptr;
  if (!(p = pool_device_get(dev_, (size_t(nc) + 1) * 8, "hipMalloc(chunk bases)", err))) return false;
  chunk_base_d_ = static_cast<unsigned long long*>(p);
  // the result lives in pinned host memory that the result move writes directly over PCIe
  // (measured, profiles/r03/pcie_probe.txt: kernel stores to host memory 55 GB/s, a DMA
  // device-to-host copy 28.6 GB/s; the DMA engine then only carries the batch upward)
  if (!(p = pool_host_get(cap4 * 4, "hipHostMalloc(adv)", err))) return false;
  adv_h_ = static_cast<uint32_t*>(p);
  if (!ok(hipHostGetDevicePointer(&p, adv_h_, 0), "hipHostGetDevicePointer(adv)", err)) return false;
  adv_hd_ = static_cast<uint32_t*>(p);
  if (!(p = pool_host_get(std::max<size_t>(n4, 4) * 4, "hipHostMalloc(row ends)", err))) return false;
  row_end_h_ = static_cast<uint32_t*>(p);
  if (!ok(hipHostGetDevicePointer(&p, row_end_h_, 0), "hipHostGetDevicePointer(row ends)", err)) return false;
  row_end_hd_ = static_cast<uint32_t*>(p);
  if (!(p = pool_device_get(dev_, std::max<size_t>(n4, 4) * 4, "hipMalloc(row ends)", err))) return false;
  row_end_d_ = static_cast<uint32_t*>(p);
  if (!(p = pool_host_get(64, "hipHostMalloc(ctl)", err))) return false;
  ctl_h_ = static_cast<unsigned long long*>(p);
  prepared_ = true;
  prepare_us_ = uint64_t(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - start).count());
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
      !ok(hipMemsetAsync(chunk_base_d_, 0, 8, s_k_), "memset(chunk base)", err))
    return false;
  // Per chunk: its upload on the copy stream; behind it, on the kernel stream, one match
  // launch whose first workgroups move the previous chunk's result out (engine.h
  // copy_out_tiles: tile directory -> host CSR).  All work is queued up front (measured: the
  // calls never block); the host waits once, at the end.
  // the result move leaves the row ends in HBM and the DMA engine carries them up on a third
  // stream while the kernels store the advisories (measured: 3.32 -> 3.20 ms per C2 pass; the
  // kernel stores alone reach 36-40 GB/s beside the match tiles; the row ends stored by the
  // move too: 2.93 ms against 2.77)
  auto copy_args = [&](uint32_t c) {
    CopyOutArgs ca;
    ca.dir = m_.dir;
    ca.pkg = m_.pkg;
    ca.adv = m_.adv;
    ca.row_end_h = row_end_d_;
    ca.adv_h = adv_hd_;
    ca.chunk_base = chunk_base_d_;
    ca.c = c;
    ca.t0 = bounds_[c];
    ca.t1 = bounds_[c + 1];
    ca.pkg_base = db_.pkg_base;
    ca.cap = cap_;
    ca.packed = packed_ ? 1u : 0u;
    ca.adv_units = adv_units_;
    ca.row_end_units = row_end_units_;
    ca.ctl = m_.ctl;
    return ca;
  };
  // measurement only: TVM_PIPE_TRACE=1 prints the host time spent in each call of a pass
  static const bool trace = std::getenv("TVM_PIPE_TRACE") != nullptr;
  // chunk c's result move is done (ev_k_[c]): the DMA engine carries its row ends up (third stream)
  auto rowend_up = [&](uint32_t c) {
    const size_t q0 = size_t(bounds_[c]) * kTile, q1 = size_t(bounds_[c + 1]) * kTile;
    return ok(hipEventRecord(ev_k_[c], s_k_), "hipEventRecord", err) &&
           ok(hipStreamWaitEvent(s_d2h_, ev_k_[c], 0), "hipStreamWaitEvent", err) &&
           ok(hipMemcpyAsync(row_end_h_ + q0, row_end_d_ + q0, (q1 - q0) * 4, hipMemcpyDeviceToHost, s_d2h_),
              "D2H row ends", err);
  };
  const auto T0 = std::chrono::steady_clock::now();
  auto us = [&]() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - T0).count(); };
  int64_t prev = -1;  // the last chunk matched, whose result has not been moved yet
  for (uint32_t c = 0; c < nc; c++) {
    const uint32_t t0 = bounds_[c], t1 = bounds_[c + 1];
    if (t1 == t0) continue;
    const size_t p0 = size_t(t0) * kTile, p1 = std::min<size_t>(size_t(t1) * kTile, n);
    const size_t g0 = size_t(t0) * kGroupsPerTile, g1 = size_t(t1) * kGroupsPerTile;
    const uint64_t a0 = toff_[g0], a1 = toff_[g1];
    if (!wc_.empty()) {  // transport form: one DMA, then the chunk is rebuilt in HBM
      const WireChunk& w = wc_[c];
      UnpackArgs ua;
      ua.wire = wire_d_;
      ua.nref = reinterpret_cast<const uint32_t*>(wire_d_ + w.o_nref);
      ua.vref = reinterpret_cast<const uint32_t*>(wire_d_ + w.o_vref);
      ua.lens = reinterpret_cast<const uint16_t*>(wire_d_ + w.o_lens);
      ua.plat = wire_d_ + w.o_plat;
      ua.toff = reinterpret_cast<const uint64_t*>(wire_d_ + w.o_toff);
      ua.attr_in = reinterpret_cast<const uint2*>(wire_d_ + w.o_attr);
      ua.ptab = ptab_d_;
      ua.pk = db_.pk;
      ua.tile_off = db_.tile_off;
      ua.arena = db_.arena;
      ua.attr = hb.attr.empty() ? nullptr : db_.attr;
      ua.p0 = uint32_t(p0);
      ua.m = w.m;
      ua.g0 = uint32_t(g0);
      ua.groups = w.groups;
      ua.arena_cap = db_.arena_bytes;
      ua.wire_cap = wire_bytes_;
      ua.ctl = m_.ctl;
      h2d_ += w.bytes;
      if (!ok(hipMemcpyAsync(wire_d_ + w.off, wire_h_ + w.off, w.bytes, hipMemcpyHostToDevice, s_h2d_), "H2D chunk", err) ||
          !ok(hipEventRecord(ev_h_[c], s_h2d_), "hipEventRecord", err) ||
          !ok(hipStreamWaitEvent(s_k_, ev_h_[c], 0), "hipStreamWaitEvent", err))
        return false;
      hipLaunchKernelGGL(unpack_kernel, dim3((w.groups + 3) / 4), dim3(256), 0, s_k_, ua);
      if (!ok(hipGetLastError(), "unpack kernel launch", err)) return false;
      if (trace) std::fprintf(stderr, "pipe c%u upload + unpack queued %.1f us\n", c, us());
    } else if ((!raw_staged_ && (stage_chunk(hb, p0, p1, g0, g1, a0, a1), false)) ||
        !ok(hipMemcpyAsync(db_.pk + p0, raw_pk_ + p0, (p1 - p0) * sizeof(uint2), hipMemcpyHostToDevice, s_h2d_),
            "H2D packages", err) ||
        !ok(hipMemcpyAsync(db_.tile_off + g0, raw_toff_ + g0, (g1 - g0 + 1) * 8, hipMemcpyHostToDevice, s_h2d_),
            "H2D group offsets", err) ||
        (a1 > a0 && !ok(hipMemcpyAsync(db_.arena + a0, raw_arena_ + a0, a1 - a0, hipMemcpyHostToDevice, s_h2d_),
                        "H2D strings", err)) ||
        (!hb.attr.empty() &&
         !ok(hipMemcpyAsync(db_.attr + p0, raw_attr_ + p0, (p1 - p0) * sizeof(uint2), hipMemcpyHostToDevice, s_h2d_),
             "H2D attributes", err)) ||
        !ok(hipEventRecord(ev_h_[c], s_h2d_), "hipEventRecord", err) ||
        !ok(hipStreamWaitEvent(s_k_, ev_h_[c], 0), "hipStreamWaitEvent", err)) {
      return false;
    } else {
      h2d_ += (p1 - p0) * sizeof(uint2) + (g1 - g0 + 1) * 8 + (a1 - a0) + (hb.attr.empty() ? 0 : (p1 - p0) * sizeof(uint2));
    }
    const CopyOutArgs prev_co = prev >= 0 ? copy_args(uint32_t(prev)) : CopyOutArgs{};
    if (!eng.launch_tiles(db_, m_, t0, t1, s_k_, s_k_, nullptr, err, prev >= 0 ? &prev_co : nullptr)) return false;
    if (prev >= 0 && !rowend_up(uint32_t(prev))) return false;
    if (trace) std::fprintf(stderr, "pipe c%u match %.1f us\n", c, us());
    prev = c;
  }
  raw_staged_ = true;  // (the raw form's chunks were staged on the way)
  if (prev >= 0) {
    launch_copy_out(s_k_, copy_args(uint32_t(prev)));
    if (!ok(hipGetLastError(), "copy-out kernel launch", err) || !rowend_up(uint32_t(prev))) return false;
  }
  if (!ok(hipMemcpyAsync(ctl_h_, m_.ctl, 64, hipMemcpyDeviceToHost, s_k_), "D2H ctl", err)) return false;
  if (trace) std::fprintf(stderr, "pipe ctl queued %.1f us\n", us());
  if (!ok(hipStreamSynchronize(s_k_), "pipeline", err) || !ok(hipStreamSynchronize(s_d2h_), "pipeline", err)) return false;
  if (trace) std::fprintf(stderr, "pipe done %.1f us\n", us());
  d2h_ = uint64_t(n) * 4 + std::min<uint64_t>(ctl_h_[0], cap_) * (packed_ ? 3 : 4);
  total = ctl_h_[0];
  err_pkg = ctl_h_[1] ? int64_t(n - ctl_h_[1]) : -1;
  err_bits = ctl_h_[3];
  return true;
}

}  // namespace tvm
