// Device engine (host side of the match path): HBM-resident advisory tables, batch
// upload, variant selection and launch of the two match kernels (match_kernel.h,
// instantiated in kern_*.hip), and read-back of the ordered match list.
#include "engine.h"
#include "host_par.h"
#include "pool.h"

#include <algorithm>
#include <mutex>
#include <memory>
#include <deque>
#include <condition_variable>
#include <cstdlib>
#include <cstring>

#include "db.h"
#include "match_kernel.h"
#include "match_variants.h"
#include "pipeline.h"

namespace tvm {

// kern_*.hip
ProbeFn probe_fn_DEB();
#ifdef TVM_DIAG
ProbeFn probe_fn_DEB_diag(int d);
#endif
ProbeFn probe_fn_OS();
ProbeFn probe_fn_ALL();
const SweepFn* sweep_table(bool filt);
const FusedFn* fused_table_DEB();
const FusedFn* fused_table_OS();
const FusedFn* fused_table_ALL();
const FusedFn* fused_table_LEAN();

namespace {

// Engine::launch splits an all-grammar batch in two launches when at most 1 tile in kSplitFull
// needs the all-grammar kernel (the rest run on GM_LEAN); Engine::upload orders tiles for it.
constexpr uint32_t kSplitFull = 10;
constexpr uint32_t kXcds = 8;  // MI355X: 8 XCDs, 32 CUs each

constexpr const char* kVariantNames[] = {
#define TVM_NAME_(F, K, MB, NAME) NAME,
    TVM_MATCH_VARIANTS(TVM_NAME_)
#undef TVM_NAME_
};
// Grammar-set index of a batch: 0 = dpkg only, 1 = OS grammars, 2 = any, 3 = library grammars
// without Maven / RubyGems (GM_LEAN; TVM_NO_LEAN=1: such batches take the all-grammar kernel,
// for measurement).
int grammar_index(uint32_t gm) {
  static const bool no_lean = std::getenv("TVM_NO_LEAN") != nullptr;
  return (gm & ~GM_DEB) == 0 ? 0 : (gm & ~GM_OS) == 0 ? 1 : ((gm & ~GM_LEAN) == 0 && !no_lean) ? 3 : 2;
}
constexpr int kNumVariants = 1 + kNumTuned;
constexpr bool kFusedVariant[] = {
#define TVM_F_(F, K, MB, NAME) F != 0,
    TVM_MATCH_VARIANTS(TVM_F_)
#undef TVM_F_
};

FusedFn fused_fn(uint32_t gm, int vi) {
  switch (grammar_index(gm)) {
    case 0: return fused_table_DEB()[vi - 1];
    case 1: return fused_table_OS()[vi - 1];
    case 3: return fused_table_LEAN()[vi - 1];
    default: return fused_table_ALL()[vi - 1];
  }
}


ProbeFn probe_fn(uint32_t gm) {
#ifdef TVM_DIAG  // measurement builds only (make DIAG=1): probe with parts switched off
  static const int diag = std::getenv("TVM_PROBE_DIAG") ? std::atoi(std::getenv("TVM_PROBE_DIAG")) : 0;
  if (diag && grammar_index(gm) == 0) return probe_fn_DEB_diag(diag);
#endif
  switch (grammar_index(gm)) {
    case 0: return probe_fn_DEB();
    case 1: return probe_fn_OS();
    default: return probe_fn_ALL();
  }
}

bool hip_ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

template <class T>
bool upload_vec(const std::vector<T>& v, T** dst, std::vector<void*>& allocs, uint64_t& bytes, std::string& err) {
  size_t n = std::max<size_t>(v.size(), 1) * sizeof(T);
  void* p = nullptr;
  if (!hip_ok(hipMalloc(&p, n), "hipMalloc(tables)", err)) return false;
  allocs.push_back(p);
  if (!v.empty() && !hip_ok(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy(tables)", err))
    return false;
  bytes += n;
  *dst = static_cast<T*>(p);
  return true;
}

// pool_dev >= 0: the block comes from the process-wide cache of that device (pool.h)
template <class T>
bool dmalloc(T** p, size_t count, const char* what, std::string& err, int pool_dev = -1) {
  void* q = nullptr;
  const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  if (pool_dev >= 0) {
    q = pool_device_get(pool_dev, bytes, what, err);
    if (!q) return false;
  } else if (!hip_ok(hipMalloc(&q, bytes), what, err)) {
    return false;
  }
  *p = static_cast<T*>(q);
  return true;
}

void dfree(void* p, bool pooled, int device) {
  if (!p) return;
  if (pooled) pool_device_put(device, p);
  else (void)hipFree(p);
}

}  // namespace

int num_variants() { return kNumVariants; }
const char* variant_name(int v) {
  if (v == 0) return "auto";
  return v > 0 && v < kNumVariants ? kVariantNames[v - 1] : nullptr;
}
// Grammar sets variant v is built for: bit 0 dpkg-only, bit 1 OS grammars, bit 2 all grammars,
// bit 3 GM_LEAN.
int variant_grammar_sets(int v) {
  if (v == 0) return 15;
  if (v < 0 || v >= kNumVariants) return 0;
  if (!kFusedVariant[v - 1]) return 15;
  return (fused_table_DEB()[v - 1] ? 1 : 0) | (fused_table_OS()[v - 1] ? 2 : 0) | (fused_table_ALL()[v - 1] ? 4 : 0) |
         (fused_table_LEAN()[v - 1] ? 8 : 0);
}

// "auto": per grammar set, the fastest variant of bench.py --sweep on MI355X:
// dpkg-only batches (C2) fused K=4; rpm/apk and mixed batches (C5, C4, C3) fused K=2, whose
// lower register count keeps 5 waves per SIMD where the filtered K=4 kernel drops to 4.
int resolve_variant(int v, uint32_t gm) {
  if (v != 0) return v;
  const int gi = grammar_index(gm);
  return 1 + (gi == 0 ? kAutoVariant : gi == 1 ? kAutoVariantOS : gi == 3 ? kAutoVariantLean : kAutoVariantFiltered);
}

// ---- Engine -----------------------------------------------------------------------------------

Engine::~Engine() {
  if (dev_ >= 0) (void)hipSetDevice(dev_);
  if (stream_) (void)hipStreamSynchronize(stream_);  // no queued launch may outlive the tables
  dropin_.reset();
  for (void* p : allocs_) (void)hipFree(p);
  if (stream_) (void)hipStreamDestroy(stream_);
}

Engine* Engine::open(const DB& db, int device, std::string& err) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    err = "no HIP device available (trivy_amd requires an MI355X / gfx950 GPU)";
    return nullptr;
  }
  if (device < 0 || device >= ndev) {
    err = "invalid HIP device index";
    return nullptr;
  }
  Engine* e = new Engine();
  e->dev_ = device;
  e->db_ = &db;
  if (const char* v = std::getenv("TVM_VARIANT")) e->set_variant(std::atoi(v));
  if (!hip_ok(hipSetDevice(device), "hipSetDevice", err) ||
      !hip_ok(hipStreamCreateWithFlags(&e->stream_, hipStreamNonBlocking), "hipStreamCreate", err)) {
    delete e;
    return nullptr;
  }
  Slot* sl; uint8_t* fp; uint8_t* na; Row* rows; RowOff* ro; uint64_t* kw; PlatInfo* pl; RowAux* ax; uint32_t* ai;
  bool ok = upload_vec(db.aux, &ax, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.aux_ids, &ai, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.slots, &sl, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.slot_fp, &fp, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.name_arena, &na, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.rows, &rows, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.row_off, &ro, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.key_words, &kw, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.plat_info, &pl, e->allocs_, e->table_bytes_, err);
  if (!ok) {
    delete e;
    return nullptr;
  }
  e->d_.slots = sl;
  e->d_.slot_fp = fp;
  e->d_.slot_mask = db.slot_mask;
  e->d_.name_arena = na;
  e->d_.rows = rows;
  e->d_.row_off = ro;
  e->d_.key_words = kw;
  e->d_.plats = pl;
  e->d_.aux = ax;
  e->d_.aux_ids = ai;
  e->d_.n_plats = uint32_t(db.plats.size());
  return e;
}

int Engine::set_variant(int v) {
  const int old = variant_;
  if (v >= 0 && v < kNumVariants) variant_ = v;
  return old;
}

// Grammar bits (1 << Cmp) of the platforms a batch touches.
uint32_t Engine::grammar_set(const HostBatch& hb) const {
  const auto& pi = db_->plat_info;
  std::atomic<uint32_t> gm{0};
  range_for(hb.pk.size(), 1 << 18, [&](size_t a, size_t b) {  // host threads: a fresh batch's prepare
    uint32_t g = 0, last = 0xFFFFFFFFu;
    for (size_t i = a; i < b; i++) {
      const uint32_t p = hb.pk[i].x;
      if (p != last && p < pi.size()) g |= 1u << pi[p].cmp;
      last = p;
    }
    gm.fetch_or(g, std::memory_order_relaxed);
  });
  return gm.load() & GM_ALL;
}

// Scratch words a batch may need: keys longer than 32 bytes (the widest grammar's bound)
// and, for Maven packages, the packed parse of the installed version (AUX_MVN rows).
uint64_t Engine::scratch_words(const HostBatch& hb) const {
  const auto& pi = db_->plat_info;
  std::atomic<uint64_t> total{0};
  range_for(hb.pk.size(), 1 << 18, [&](size_t a, size_t b) {
    uint64_t w = 0;
    for (size_t i = a; i < b; i++) {
      const uint2 d = hb.pk[i];
      const uint32_t vlen = d.y >> 16;
      const uint32_t need = (key_bound_any(vlen) + 7) / 8;
      const bool mvn = d.x < pi.size() && pi[d.x].cmp == CMP_MAVEN;
      if (need > (mvn ? 2u : kKeyWords)) w += need;  // Maven keys spill from 17 bytes (probe_one)
      if (mvn) w += (uint64_t(kMvnPackedWords) * std::min<uint32_t>(2 * vlen + 3, kMvnMaxTok) + 1) / 2;
    }
    total.fetch_add(w, std::memory_order_relaxed);
  });
  return total.load();
}

bool Engine::alloc_batch(const HostBatch& hb, DevBatch& b, std::string& err, bool pooled) {
  (void)hipSetDevice(dev_);
  const int pd = pooled ? dev_ : -1;
  b.n = uint32_t(hb.pk.size());
  b.n_tiles = hb.n_tiles();
  b.arena_bytes = hb.arena.size();
  b.gm = grammar_set(hb);
  b.spill_words = scratch_words(hb);
  if (!hb.attr.empty() && hb.attr.size() != hb.pk.size()) {
    err = "batch attributes do not cover every package";
    return false;
  }
  // every batch owns its scratch: launches of different batches (pipeline streams, the
  // engine stream, other threads) never write the same words
  b.spill_cap = std::max<uint64_t>(b.spill_words, 64);
  // test hook (tests/test_gpu_spill.py): TVM_TEST_SPILL_CAP words of usable scratch, so the
  // failure path of a long key (ERR_SPILL, no rows for the package) can be exercised; the
  // allocation itself keeps its size
  const uint64_t alloc_words = b.spill_cap;
  if (const char* cap = std::getenv("TVM_TEST_SPILL_CAP"))
    b.spill_cap = std::min<uint64_t>(b.spill_cap, std::strtoull(cap, nullptr, 10));
  // +32 B tail: the kernels stage whole 16-byte lines and read names as dword triples
  return dmalloc(&b.spill, alloc_words, "hipMalloc(batch scratch)", err, pd) &&
         dmalloc(&b.pk, hb.pk.size(), "hipMalloc(batch)", err, pd) &&
         dmalloc(&b.tile_off, size_t(b.n_tiles) * kGroupsPerTile + 1, "hipMalloc(group offsets)", err, pd) &&
         dmalloc(&b.arena, (hb.arena.size() + 32 + 15) & ~size_t(15), "hipMalloc(batch arena)", err, pd) &&
         (hb.attr.empty() || dmalloc(&b.attr, hb.attr.size(), "hipMalloc(batch attr)", err, pd)) &&
         dmalloc(&b.rec, hb.pk.size(), "hipMalloc(package records)", err, pd) &&
         dmalloc(&b.tail, hb.pk.size(), "hipMalloc(key tails)", err, pd);
}

// Tile order for a grid's XCDs: workgroups are dealt round-robin over the 8 XCDs (blocks b and
// b + 8 share one, MI355X_MICROARCH.md), and each XCD has its own L2.  The tiles, taken by
// platform (the first package's), are cut into kXcds runs of equal predicted weight; position
// b of the launch takes the next tile of run b % kXcds, heaviest first within the run, so one
// XCD's L2 holds the hot rows of one or two platforms instead of every platform's (and its CUs
// run one or two grammars' paths of the all-grammar kernel).  Runs that run out hand their
// positions to the others (the grid's tail).  `order`: in, heaviest first.  Used only where it
// measured faster (Engine::upload).
static void xcd_order(const HostBatch& hb, const std::vector<uint64_t>& w, std::vector<uint32_t>& order) {
  const uint32_t n = uint32_t(order.size());
  std::vector<uint32_t> by_plat(n);
  for (uint32_t t = 0; t < n; t++) by_plat[t] = t;
  std::stable_sort(by_plat.begin(), by_plat.end(),
                   [&](uint32_t x, uint32_t y) { return hb.pk[size_t(x) * kTile].x < hb.pk[size_t(y) * kTile].x; });
  uint64_t total = 0;
  for (uint64_t x : w) total += x;
  std::vector<uint32_t> run_of(n);
  uint64_t acc = 0;
  for (uint32_t t : by_plat) {
    run_of[t] = uint32_t(std::min<uint64_t>(kXcds - 1, total ? acc * kXcds / total : 0));
    acc += w[t];
  }
  std::vector<std::vector<uint32_t>> runs(kXcds);
  for (uint32_t t : order) runs[run_of[t]].push_back(t);  // heaviest first within each run
  std::vector<size_t> next(kXcds, 0);
  for (uint32_t b = 0; b < n; b++) {
    uint32_t r = b % kXcds;
    for (uint32_t k = 0; k < kXcds && next[r] == runs[r].size(); k++) r = (r + 1) % kXcds;
    order[b] = runs[r][next[r]++];
  }
}

bool Engine::upload(const HostBatch& hb, DevBatch& b, std::string& err) {
  if (!alloc_batch(hb, b, err)) return false;
  std::vector<uint64_t> toff(hb.tile_off.begin(), hb.tile_off.end());  // + the arena end, then padded to whole tiles
  toff.resize(size_t(hb.n_tiles()) * kGroupsPerTile + 1, hb.arena.size());
  if (!hb.pk.empty() && !hip_ok(hipMemcpy(b.pk, hb.pk.data(), hb.pk.size() * sizeof(uint2), hipMemcpyHostToDevice),
                                "H2D batch", err))
    return false;
  if (!hip_ok(hipMemcpy(b.tile_off, toff.data(), toff.size() * 8, hipMemcpyHostToDevice), "H2D tile offsets", err))
    return false;
  if (!hb.arena.empty() &&
      !hip_ok(hipMemcpy(b.arena, hb.arena.data(), hb.arena.size(), hipMemcpyHostToDevice), "H2D arena", err))
    return false;
  if (!hb.attr.empty() &&
      !hip_ok(hipMemcpy(b.attr, hb.attr.data(), hb.attr.size() * sizeof(uint2), hipMemcpyHostToDevice), "H2D attr", err))
    return false;
  static const bool no_order = std::getenv("TVM_NO_TILE_ORDER") != nullptr;  // measurement: tile order
  if (((b.gm & ~GM_OS) != 0 ? b.n_tiles > 1 : b.n_tiles >= 1024) && !no_order) {
    // the device-resident launch takes the tiles heaviest first (predicted rows from the host
    // index, Maven rows weighted 8x: a program row costs many interval rows), so the grid does
    // not end on a tail of heavy tiles - C2's row counts per tile are heavy-tailed (median
    // 2.1k pairs, p99 5.5k, max 11.9k): 0.425 -> 0.416 ms; C3 0.216 -> 0.211 ms
    const auto& pi = db_->plat_info;
    std::vector<uint64_t> off;
    hb.name_offsets(off);
    std::vector<uint64_t> w(b.n_tiles, 0);
    range_for(b.n_tiles, 64, [&](size_t t0, size_t t1) {
      for (size_t t = t0; t < t1; t++) {
        uint64_t s = 0;
        for (size_t p = t * kTile; p < std::min(hb.pk.size(), (t + 1) * kTile); p++) {
          const uint32_t plat = hb.pk[p].x;
          if (plat >= pi.size()) continue;
          const std::string_view name(reinterpret_cast<const char*>(hb.arena.data()) + off[p], hb.pk[p].y & 0xFFFFu);
          s += 1 + uint64_t(db_->key_rows(plat, name)) * (pi[plat].cmp == CMP_MAVEN ? 8 : 1);
        }
        w[t] = s;
      }
    });
    // all-grammar batches: the tiles without Maven / RubyGems packages first (their own launch
    // on the GM_LEAN kernel, Engine::launch), each part heaviest first
    std::vector<uint8_t> full(b.n_tiles, 1);
    static const bool no_lean = std::getenv("TVM_NO_LEAN") != nullptr;
    if (grammar_index(b.gm) == 2 && !no_lean)
      range_for(b.n_tiles, 64, [&](size_t t0, size_t t1) {
        for (size_t t = t0; t < t1; t++) {
          bool f = false;
          for (size_t p = t * kTile; p < std::min(hb.pk.size(), (t + 1) * kTile) && !f; p++) {
            const uint32_t plat = hb.pk[p].x;
            f = plat < pi.size() && ((GM_LEAN >> pi[plat].cmp) & 1u) == 0;
          }
          full[t] = f;
        }
      });
    std::vector<uint32_t> order(b.n_tiles);
    for (uint32_t t = 0; t < b.n_tiles; t++) order[t] = t;
    b.n_lean_tiles = 0;
    for (uint32_t t = 0; t < b.n_tiles; t++) b.n_lean_tiles += full[t] ? 0 : 1;
    // a batch Engine::launch splits keeps its parts apart (lean tiles first); one launch over
    // every tile takes them heaviest first whatever their kernel part (TVM_TILE_ORDER=lean:
    // the parts apart anyway, =full: the all-grammar tiles first - measurement only)
    static const char* ord = std::getenv("TVM_TILE_ORDER");
    const uint32_t n_full = b.n_tiles - b.n_lean_tiles;
    const bool split = n_full && n_full < b.n_tiles && n_full * kSplitFull <= b.n_tiles;
    const int mode = split || (ord && std::strcmp(ord, "lean") == 0) ? 0 : (ord && std::strcmp(ord, "full") == 0) ? 1 : 2;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
      if (mode == 0 && full[x] != full[y]) return full[x] < full[y];
      if (mode == 1 && full[x] != full[y]) return full[x] > full[y];
      return w[x] > w[y];
    });
    // XCD-affine runs for the all-grammar kernel in one launch (C3 0.1375 -> 0.1319 ms: one or
    // two grammars' code and rows per XCD); the dpkg and rpm / apk kernels keep the global
    // heaviest-first order (C2 0.383 -> 0.393, C5 1.81 -> 2.40 ms with the runs: per-platform
    // runs of equal predicted rows are not equal work there; profiles/r06/xcd/)
    if (mode == 2 && grammar_index(b.gm) == 2 && !(ord && std::strcmp(ord, "w") == 0) && b.n_tiles >= 8 * kXcds)
      xcd_order(hb, w, order);
    if (!dmalloc(&b.tile_map, order.size(), "hipMalloc(tile order)", err) ||
        !hip_ok(hipMemcpy(b.tile_map, order.data(), order.size() * 4, hipMemcpyHostToDevice), "H2D tile order", err))
      return false;
  }
  if (!hb.cpe_bits.empty() && hb.cpe_words) {
    if (!dmalloc(&b.cpe_bits, hb.cpe_bits.size(), "hipMalloc(cpe sets)", err) ||
        !hip_ok(hipMemcpy(b.cpe_bits, hb.cpe_bits.data(), hb.cpe_bits.size() * 4, hipMemcpyHostToDevice), "H2D cpe", err))
      return false;
    b.cpe_words = hb.cpe_words;
    b.n_cpe_sets = uint32_t(hb.cpe_bits.size() / hb.cpe_words);
  }
  return true;
}

void Engine::free_batch(int device, DevBatch& b, bool pooled) {
  (void)hipSetDevice(device);
  for (void* p : {static_cast<void*>(b.pk), static_cast<void*>(b.tile_off), static_cast<void*>(b.arena),
                  static_cast<void*>(b.attr), static_cast<void*>(b.rec), static_cast<void*>(b.tail),
                  static_cast<void*>(b.spill)})
    dfree(p, pooled, device);
  dfree(b.cpe_bits, false, device);  // never pooled (copied by the caller)
  dfree(b.tile_map, false, device);
  b = DevBatch{};
}

bool Engine::alloc_matches(uint64_t cap, uint32_t n_pkgs, DevMatches& m, std::string& err, bool pooled) {
  (void)hipSetDevice(dev_);
  const int pd = pooled ? dev_ : -1;
  m.cap = std::max<uint64_t>(cap, 1);
  m.dir_cap = std::max<uint32_t>((n_pkgs + kTile - 1) / kTile, 1);
  if (!dmalloc(&m.pkg, m.cap, "hipMalloc(matches)", err, pd) || !dmalloc(&m.adv, m.cap, "hipMalloc(matches)", err, pd) ||
      !dmalloc(&m.dir, m.dir_cap, "hipMalloc(tile dir)", err, pd) || !dmalloc(&m.ctl_mem, 16, "hipMalloc(ctl)", err, pd))
    return false;
  // both control blocks zero (Engine::launch alternates them)
  if (!hip_ok(hipMemset(m.ctl_mem, 0, 16 * sizeof(unsigned long long)), "memset(ctl)", err)) return false;
  m.ctl = m.ctl_mem;
  m.ctl_next = m.ctl_mem + 8;
  return true;
}

void Engine::free_matches(int device, DevMatches& m, bool pooled) {
  (void)hipSetDevice(device);
  for (void* p : {static_cast<void*>(m.pkg), static_cast<void*>(m.adv), static_cast<void*>(m.dir),
                  static_cast<void*>(m.ctl_mem ? m.ctl_mem : m.ctl)})
    dfree(p, pooled, device);
  m = DevMatches{};
}

bool Engine::fetch_ordered(const DevMatches& m, uint32_t n_pkgs, uint64_t total, std::vector<uint2>& out,
                           hipStream_t st, std::string& err) {
  out.clear();
  if (total > m.cap) {
    err = "match buffer too small";
    return false;
  }
  const uint32_t n_tiles = (n_pkgs + kTile - 1) / kTile;
  std::vector<TileDir> dir(n_tiles);
  std::vector<uint32_t> pk(total), ad(total);
  if ((n_tiles && !hip_ok(hipMemcpyAsync(dir.data(), m.dir, n_tiles * sizeof(TileDir), hipMemcpyDeviceToHost, st),
                          "D2H dir", err)) ||
      (total && (!hip_ok(hipMemcpyAsync(pk.data(), m.pkg, total * 4, hipMemcpyDeviceToHost, st), "D2H matches", err) ||
                 !hip_ok(hipMemcpyAsync(ad.data(), m.adv, total * 4, hipMemcpyDeviceToHost, st), "D2H matches", err))) ||
      !hip_ok(hipStreamSynchronize(st), "D2H matches", err))
    return false;
  out.reserve(total);
  for (const TileDir& d : dir)
    for (uint64_t i = d.base; i < d.base + d.count; i++) out.push_back(make_uint2(pk[i], ad[i]));
  return true;
}

bool Engine::launch_tiles(const DevBatch& b, const DevMatches& m, uint32_t t_begin, uint32_t t_end, hipStream_t pst,
                          hipStream_t sst, hipEvent_t ev, std::string& err, const CopyOutArgs* co,
                          unsigned long long* ctl_zero, const uint32_t* tmap, uint32_t tmap_n, uint32_t gm) {
  (void)hipSetDevice(dev_);
  if (t_end > b.n_tiles) t_end = b.n_tiles;
  if (t_begin >= t_end) return true;
  if (t_end > m.dir_cap) {
    err = "tile directory smaller than the batch";
    return false;
  }
  if (!gm) gm = b.gm;
  const int vi = resolve_variant(variant_, gm);
  if (tmap && (co || t_begin != 0 || t_end != b.n_tiles || !kFusedVariant[vi - 1] || tmap_n == 0)) {
    err = "a tile-list launch is a fused pass over the whole batch";
    return false;
  }
  last_launched_ = vi;
  const uint32_t nt = t_end - t_begin;
  const uint32_t p0 = t_begin * kTile;
  const uint32_t n = std::min<uint32_t>(b.n, t_end * kTile) - p0;
  ProbeArgs pa;
  pa.db = d_;
  pa.pk = b.pk + p0;
  pa.tile_off = b.tile_off + size_t(t_begin) * kGroupsPerTile;
  pa.arena = b.arena;
  pa.n = n;
  pa.p0 = p0;
  pa.n_total = b.n;
  pa.rec = b.rec + p0;
  pa.tail = b.tail + p0;
  pa.ctl = m.ctl;
  if (!b.spill || (b.spill_cap < b.spill_words && !std::getenv("TVM_TEST_SPILL_CAP"))) {
    err = "batch scratch missing or smaller than the batch needs";
    return false;
  }
  pa.spill = b.spill;
  pa.spill_cap = b.spill_cap;
  const bool fused = kFusedVariant[vi - 1];
  if (!fused && ctl_zero &&
      !hip_ok(hipMemsetAsync(ctl_zero, 0, 8 * sizeof(unsigned long long), pst), "memset(ctl)", err))
    return false;
  if (!fused) {
    if (co) launch_copy_out(pst, *co);
    probe_fn(b.gm)(nt, pst, pa);
    if (!hip_ok(hipGetLastError(), "probe kernel launch", err)) return false;
    if (sst != pst && (!hip_ok(hipEventRecord(ev, pst), "hipEventRecord", err) ||
                       !hip_ok(hipStreamWaitEvent(sst, ev, 0), "hipStreamWaitEvent", err)))
      return false;
  }
  SweepArgs sa;
  sa.db = d_;
  sa.rec = b.rec + p0;
  sa.tail = b.tail + p0;
  sa.spill = b.spill;
  sa.arena = b.arena;
  sa.attr = b.attr ? b.attr + p0 : nullptr;
  sa.cpe_bits = b.cpe_bits;
  sa.cpe_words = b.cpe_words;
  sa.n_cpe_sets = b.n_cpe_sets;
  sa.n = n;
  sa.p0 = p0;
  sa.out_base = b.pkg_base;
  sa.n_tiles = nt;
  sa.t0 = t_begin;
  sa.dir = m.dir;
  sa.out_pkg = m.pkg;
  sa.out_adv = m.adv;
  sa.out_cap = m.cap;
  sa.ctl = m.ctl;
  if (fused) {
    FusedArgs fa;
    fa.pa = pa;
    fa.sa = sa;
    if (co) {
      fa.co = *co;
      // 128 workgroups move a chunk's results beside its match tiles (measured, C2 end-to-end
      // with the wave-per-tile move: 32 3.60 ms, 64 2.81, 128 2.77; round 3's workgroup-per-tile
      // move: 64 3.10, 128 3.13, 256 3.25, profiles/r03/e2e_copy_width.txt); TVM_COPY_WG
      // overrides it for measurement
      static const uint32_t n_copy = [] {
        const char* v = std::getenv("TVM_COPY_WG");
        return v ? uint32_t(std::max(1, std::atoi(v))) : 128u;
      }();
      fa.n_copy = n_copy;
    }
    if (!co && t_begin == 0 && t_end == b.n_tiles) fa.tile_map = tmap ? tmap : b.tile_map;
    fa.ctl_zero = co ? nullptr : ctl_zero;
    const FusedFn fn = fused_fn(gm, vi);
    if (!fn) {
      err = std::string("match-path variant ") + kVariantNames[vi - 1] + " is not built for this batch's grammar set";
      return false;
    }
    fn(tmap ? tmap_n : nt, pst, fa);
    return hip_ok(hipGetLastError(), "match kernel launch", err);
  }
  const bool filt = (b.gm & ~GM_DEB) != 0;
  sweep_table(filt)[vi - 1](nt, sst, sa);
  return hip_ok(hipGetLastError(), "sweep kernel launch", err);
}

bool Engine::launch(const DevBatch& b, DevMatches& m, hipStream_t st, std::string& err) {
  (void)hipSetDevice(dev_);
  unsigned long long* zero = nullptr;  // the control block this pass leaves behind
  if (m.ctl_next) {
    std::swap(m.ctl, m.ctl_next);  // count into the block the last pass zeroed
    zero = m.ctl_next;
  } else if (!hip_ok(hipMemsetAsync(m.ctl, 0, 8 * sizeof(unsigned long long), st), "memset(ctl)", err)) {
    return false;
  }
  if (b.n_tiles == 0)
    return !zero || hip_ok(hipMemsetAsync(zero, 0, 8 * sizeof(unsigned long long), st), "memset(ctl)", err);
  // one launch over every tile (cutting the pass into chunks whose probe overlaps the
  // previous chunk's sweep on a second stream measured slower: DESIGN.md §4) - or, for an
  // all-grammar batch whose tiles are nearly all free of Maven / RubyGems packages (at most 1
  // in kSplitFull needs the all-grammar kernel), two back to back: those tiles on the GM_LEAN
  // kernel, then the rest (Engine::upload's tile_map order: lean tiles first, each part
  // heaviest first).  The second launch starts when the first has drained (kernels on two
  // streams did not overlap on this runtime either), so the split pays when the all-grammar
  // part is small: C4's 12.5M share (8 % Maven tiles) 1.554 -> 1.508 ms; C3 (20 %) 0.156 ->
  // 0.169 ms, which therefore stays one launch (profiles/r06/lean_ab/)
  const uint32_t nl = b.n_lean_tiles;
  if (nl && nl < b.n_tiles && (b.n_tiles - nl) * kSplitFull <= b.n_tiles && b.tile_map && grammar_index(b.gm) == 2 &&
      kFusedVariant[resolve_variant(variant_, b.gm) - 1] && kFusedVariant[resolve_variant(variant_, GM_LEAN) - 1]) {
    return launch_tiles(b, m, 0, b.n_tiles, st, st, nullptr, err, nullptr, zero, b.tile_map, nl, GM_LEAN) &&
           launch_tiles(b, m, 0, b.n_tiles, st, st, nullptr, err, nullptr, nullptr, b.tile_map + nl, b.n_tiles - nl,
                        b.gm);
  }
  return launch_tiles(b, m, 0, b.n_tiles, st, st, nullptr, err, nullptr, zero);
}

// ---- drop-in path: pooled buffers + coalescing of concurrent calls -------------------------
//
// The reference serves concurrent Detect calls (twirp server, server.go:45; the k8s
// scanner's worker pool, scanner.go:141) each with its own bbolt read transaction.  Here a
// call is a small batch (one target), so launches - not bandwidth - bound the rate: calls
// that arrive while a launch runs queue up, and the next launch serves all of them as one
// batch (their packages concatenated, pairs handed back by package range).  The first
// caller that finds no launch running leads; a leader hands over as soon as its own call
// is served.  Device buffers, pinned staging and the long-key scratch belong to the
// context and only grow, so a call allocates nothing.  A call whose batch carries package
// attributes (Red Hat CPE sets, arches) runs in a launch of its own, and a merged launch
// that meets a poisoned DB key re-runs its calls one by one, so every call sees exactly
// the error (first poisoned package of ITS batch) it would see alone.
struct Engine::DropinReq {
  const HostBatch* hb = nullptr;
  std::vector<uint2>* out = nullptr;
  int64_t err_pkg = -1;
  std::string err;
  bool ok = false, done = false;
};

struct Engine::Dropin {
  int dev = 0;
  hipStream_t st = nullptr;
  DevBatch b;  // device buffers at their capacities (the n / n_tiles / gm fields are per launch)
  uint64_t cap_pk = 0, cap_rec = 0, cap_tail = 0, cap_groups = 0, cap_arena = 0, cap_attr = 0, cap_cpe = 0;
  uint64_t cap_dir = 0, cap_adv = 0;
  DevMatches m;
  uint8_t* pin = nullptr;
  size_t pin_cap = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<DropinReq*> pending;
  bool leading = false;
  uint64_t launches = 0, calls = 0, merged = 0;
  ~Dropin() {
    (void)hipSetDevice(dev);
    for (void* p : {static_cast<void*>(b.pk), static_cast<void*>(b.tile_off), static_cast<void*>(b.arena),
                    static_cast<void*>(b.attr), static_cast<void*>(b.cpe_bits), static_cast<void*>(b.rec),
                    static_cast<void*>(b.tail), static_cast<void*>(b.spill), static_cast<void*>(m.pkg),
                    static_cast<void*>(m.adv), static_cast<void*>(m.dir), static_cast<void*>(m.ctl)})
      if (p) (void)hipFree(p);
    if (pin) (void)hipHostFree(pin);
    if (st) (void)hipStreamDestroy(st);
  }
};

Engine::Dropin* Engine::dropin(std::string& err) {
  std::lock_guard<std::mutex> lk(dropin_init_mu_);
  if (!dropin_) {
    (void)hipSetDevice(dev_);
    auto d = std::make_unique<Dropin>();
    d->dev = dev_;
    if (!hip_ok(hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking), "hipStreamCreate(drop-in)", err) ||
        !dmalloc(&d->m.ctl, 8, "hipMalloc(ctl)", err))
      return nullptr;
    dropin_ = std::move(d);
  }
  return dropin_.get();
}

void Engine::dropin_stats(uint64_t out[3]) {
  std::string e;
  Dropin* d = dropin(e);
  if (!d) {
    out[0] = out[1] = out[2] = 0;
    return;
  }
  std::lock_guard<std::mutex> lk(d->mu);
  out[0] = d->launches;
  out[1] = d->calls;
  out[2] = d->merged;
}

namespace {
// Grows a device buffer to at least n elements (contents not kept).
template <class T>
bool grow_dev(T*& p, uint64_t& cap, uint64_t n, const char* what, std::string& err) {
  if (n <= cap && p) return true;
  if (p) (void)hipFree(p);
  p = nullptr;
  const uint64_t c = std::max<uint64_t>(n + n / 4, 64);
  if (!hip_ok(hipMalloc(reinterpret_cast<void**>(&p), c * sizeof(T)), what, err)) {
    cap = 0;
    return false;
  }
  cap = c;
  return true;
}
}  // namespace

// One launch over the calls reqs[0..n) (n > 1: attribute-free batches, concatenated).
bool Engine::dropin_run(Dropin& d, DropinReq* const* reqs, size_t n, std::string& err) {
  (void)hipSetDevice(dev_);
  HostBatch merged;
  const HostBatch* hbp = reqs[0]->hb;
  std::vector<uint32_t> first(n + 1, 0);
  if (n > 1) {
    for (size_t k = 0; k < n; k++) {
      const HostBatch& h = *reqs[k]->hb;
      first[k] = uint32_t(merged.pk.size());
      merged.pk.insert(merged.pk.end(), h.pk.begin(), h.pk.end());
      merged.arena.insert(merged.arena.end(), h.arena.begin(), h.arena.end());
    }
    uint64_t o = 0;  // group offsets of the concatenation
    for (size_t j = 0; j < merged.pk.size(); j++) {
      if (j % kGroup == 0) merged.tile_off.push_back(o);
      o += (merged.pk[j].y & 0xFFFFu) + (merged.pk[j].y >> 16);
    }
    hbp = &merged;
  }
  const HostBatch& hb = *hbp;
  first[n] = uint32_t(hb.pk.size());
  DevBatch& b = d.b;
  b.n = uint32_t(hb.pk.size());
  b.n_tiles = hb.n_tiles();
  b.arena_bytes = hb.arena.size();
  b.gm = grammar_set(hb);
  b.spill_words = scratch_words(hb);
  if (!hb.attr.empty() && hb.attr.size() != hb.pk.size()) {
    err = "batch attributes do not cover every package";
    return false;
  }
  const uint64_t groups = uint64_t(b.n_tiles) * kGroupsPerTile + 1;
  const uint64_t arena_pad = (hb.arena.size() + 32 + 15) & ~uint64_t(15);
  if (!grow_dev(b.pk, d.cap_pk, b.n, "hipMalloc(drop-in batch)", err) ||
      !grow_dev(b.rec, d.cap_rec, b.n, "hipMalloc(drop-in records)", err) ||
      !grow_dev(b.tail, d.cap_tail, b.n, "hipMalloc(drop-in key tails)", err) ||
      !grow_dev(b.tile_off, d.cap_groups, groups, "hipMalloc(drop-in group offsets)", err) ||
      !grow_dev(b.arena, d.cap_arena, arena_pad, "hipMalloc(drop-in arena)", err) ||
      (!hb.attr.empty() && !grow_dev(b.attr, d.cap_attr, b.n, "hipMalloc(drop-in attr)", err)) ||
      (b.spill_words && !grow_dev(b.spill, b.spill_cap, b.spill_words, "hipMalloc(drop-in spill)", err)) ||
      (!hb.cpe_bits.empty() && !grow_dev(b.cpe_bits, d.cap_cpe, hb.cpe_bits.size(), "hipMalloc(drop-in cpe)", err)))
    return false;
  // matches: 4 per package to start, the exact count after an overflow
  uint64_t mcap = std::max<uint64_t>(uint64_t(b.n) * 4, 1024);
  const uint32_t n_tiles = b.n_tiles;
  if (!grow_dev(d.m.dir, d.cap_dir, std::max<uint32_t>(n_tiles, 1), "hipMalloc(drop-in tile dir)", err)) return false;
  d.m.dir_cap = uint32_t(std::min<uint64_t>(d.cap_dir, 0xFFFFFFFFu));
  // pinned staging: inputs, then the outputs of the same call
  const size_t in_bytes = b.n * 8 + groups * 8 + hb.arena.size() + hb.attr.size() * 8 + hb.cpe_bits.size() * 4;
  auto stage = [&](size_t need) {
    if (need <= d.pin_cap) return true;
    if (d.pin) (void)hipHostFree(d.pin);
    d.pin = nullptr;
    d.pin_cap = 0;
    const size_t c = need + need / 4 + 4096;
    if (!hip_ok(hipHostMalloc(reinterpret_cast<void**>(&d.pin), c, hipHostMallocDefault), "hipHostMalloc(drop-in)",
                err))
      return false;
    d.pin_cap = c;
    return true;
  };
  if (!stage(in_bytes + 128)) return false;  // + the control block read back after the launch
  uint8_t* h = d.pin;
  size_t at = 0;
  auto h2d = [&](void* dst, const void* src, size_t bytes, const char* what) {
    if (!bytes) return true;
    std::memcpy(h + at, src, bytes);
    const bool r = hip_ok(hipMemcpyAsync(dst, h + at, bytes, hipMemcpyHostToDevice, d.st), what, err);
    at += bytes;
    return r;
  };
  std::vector<uint64_t> toff(hb.tile_off.begin(), hb.tile_off.end());
  toff.resize(groups, hb.arena.size());
  b.cpe_words = hb.cpe_words;
  b.n_cpe_sets = hb.cpe_words ? uint32_t(hb.cpe_bits.size() / hb.cpe_words) : 0;
  if (!h2d(b.pk, hb.pk.data(), hb.pk.size() * 8, "H2D drop-in batch") ||
      !h2d(b.tile_off, toff.data(), groups * 8, "H2D drop-in offsets") ||
      !h2d(b.arena, hb.arena.data(), hb.arena.size(), "H2D drop-in arena") ||
      !h2d(b.attr, hb.attr.data(), hb.attr.size() * 8, "H2D drop-in attr") ||
      !h2d(b.cpe_bits, hb.cpe_bits.data(), hb.cpe_bits.size() * 4, "H2D drop-in cpe"))
    return false;
  DevBatch bl = b;
  if (hb.attr.empty()) bl.attr = nullptr;
  if (hb.cpe_bits.empty()) bl.cpe_bits = nullptr;
  unsigned long long* ctl = nullptr;
  for (int attempt = 0; attempt < 2; attempt++) {
    uint64_t pcap = d.m.cap;
    if (!grow_dev(d.m.pkg, pcap, mcap, "hipMalloc(drop-in matches)", err) ||
        !grow_dev(d.m.adv, d.cap_adv, mcap, "hipMalloc(drop-in matches)", err))
      return false;
    d.m.cap = std::min(pcap, d.cap_adv);
    if (!launch(bl, d.m, d.st, err)) return false;
    ctl = reinterpret_cast<unsigned long long*>(d.pin + ((at + 7) & ~size_t(7)));
    if (!hip_ok(hipMemcpyAsync(ctl, d.m.ctl, 64, hipMemcpyDeviceToHost, d.st), "D2H ctl", err) ||
        !hip_ok(hipStreamSynchronize(d.st), "drop-in match", err))
      return false;
    if (ctl[3]) {
      err = "match kernel internal error bits " + std::to_string(ctl[3]);
      return false;
    }
    if (ctl[0] <= d.m.cap) break;
    mcap = ctl[0];  // output buffer too small: once more with the exact size
  }
  const uint64_t total = ctl[0];
  const uint64_t poisoned = ctl[1];
  d.launches++;
  if (poisoned && n > 1) {  // each call alone, so each reports its own first poisoned package
    for (size_t k = 0; k < n; k++) {
      DropinReq* r = reqs[k];
      r->ok = dropin_run(d, &r, 1, r->err);
    }
    return true;
  }
  // ordered read-back through the pinned buffer: tile directory, then the two columns
  const size_t out_at = 0;
  const size_t need = n_tiles * sizeof(TileDir) + total * 8;
  if (!stage(need)) return false;
  TileDir* hdir = reinterpret_cast<TileDir*>(d.pin + out_at);
  uint32_t* hp = reinterpret_cast<uint32_t*>(d.pin + out_at + n_tiles * sizeof(TileDir));
  uint32_t* ha = hp + total;
  if ((n_tiles && !hip_ok(hipMemcpyAsync(hdir, d.m.dir, n_tiles * sizeof(TileDir), hipMemcpyDeviceToHost, d.st),
                          "D2H dir", err)) ||
      (total && (!hip_ok(hipMemcpyAsync(hp, d.m.pkg, total * 4, hipMemcpyDeviceToHost, d.st), "D2H matches", err) ||
                 !hip_ok(hipMemcpyAsync(ha, d.m.adv, total * 4, hipMemcpyDeviceToHost, d.st), "D2H matches", err))) ||
      !hip_ok(hipStreamSynchronize(d.st), "D2H matches", err))
    return false;
  for (size_t k = 0; k < n; k++) {
    reqs[k]->out->clear();
    reqs[k]->err_pkg = -1;
    reqs[k]->ok = true;
  }
  if (poisoned) reqs[0]->err_pkg = int64_t(b.n - poisoned);  // n == 1 here
  size_t k = 0;
  for (uint32_t t = 0; t < n_tiles; t++)
    for (uint64_t i = hdir[t].base; i < hdir[t].base + hdir[t].count; i++) {
      const uint32_t p = hp[i];
      while (p >= first[k + 1]) k++;  // packages ascend along the tile order
      reqs[k]->out->push_back(make_uint2(p - first[k], ha[i]));
    }
  return true;
}

bool Engine::match_host(const HostBatch& hb, std::vector<uint2>& out, int64_t& err_pkg, std::string& err) {
  out.clear();
  err_pkg = -1;
  if (hb.pk.empty()) return true;
  Dropin* dp = dropin(err);
  if (!dp) return false;
  Dropin& d = *dp;
  DropinReq r;
  r.hb = &hb;
  r.out = &out;
  std::unique_lock<std::mutex> lk(d.mu);
  d.pending.push_back(&r);
  d.calls++;
  while (!r.done) {
    if (d.leading) {
      d.cv.wait(lk);
      continue;
    }
    d.leading = true;  // lead: serve queued calls until this one is done
    while (!r.done && !d.pending.empty()) {
      std::vector<DropinReq*> grp;
      const bool attrs = !d.pending.front()->hb->attr.empty() || !d.pending.front()->hb->cpe_bits.empty();
      uint64_t pk = 0;
      for (auto it = d.pending.begin(); it != d.pending.end();) {
        const HostBatch* h = (*it)->hb;
        const bool a = !h->attr.empty() || !h->cpe_bits.empty();
        if ((attrs || a) && !grp.empty()) break;  // a call with attributes runs alone
        if (!grp.empty() && pk + h->pk.size() > (1u << 22)) break;
        grp.push_back(*it);
        pk += h->pk.size();
        it = d.pending.erase(it);
        if (attrs) break;
      }
      if (grp.size() > 1) d.merged += grp.size();
      lk.unlock();
      std::string e;
      if (!dropin_run(d, grp.data(), grp.size(), e))
        for (DropinReq* q : grp) {
          q->ok = false;
          q->err = e;
        }
      lk.lock();
      for (DropinReq* q : grp) q->done = true;
      d.cv.notify_all();
    }
    d.leading = false;
    d.cv.notify_all();  // a waiting caller takes over the queue
  }
  if (!r.ok) {
    err = r.err;
    return false;
  }
  err_pkg = r.err_pkg;
  return true;
}

bool Engine::verify(std::string& err) {
  (void)hipSetDevice(dev_);
  auto check = [&](const void* dev, const void* host, size_t bytes, const char* what) {
    if (!bytes) return true;
    std::vector<uint8_t> tmp(bytes);
    if (!hip_ok(hipMemcpy(tmp.data(), dev, bytes, hipMemcpyDeviceToHost), "D2H verify", err)) return false;
    if (std::memcmp(tmp.data(), host, bytes) != 0) {
      err = std::string("device table differs from the host image: ") + what;
      return false;
    }
    return true;
  };
  const DB& db = *db_;
  return check(d_.slots, db.slots.data(), db.slots.size() * sizeof(Slot), "slots") &&
         check(d_.slot_fp, db.slot_fp.data(), db.slot_fp.size(), "slot_fp") &&
         check(d_.name_arena, db.name_arena.data(), db.name_arena.size(), "name_arena") &&
         check(d_.rows, db.rows.data(), db.rows.size() * sizeof(Row), "rows") &&
         check(d_.row_off, db.row_off.data(), db.row_off.size() * sizeof(RowOff), "row_off") &&
         check(d_.key_words, db.key_words.data(), db.key_words.size() * 8, "key_words") &&
         check(d_.plats, db.plat_info.data(), db.plat_info.size() * sizeof(PlatInfo), "plats") &&
         check(d_.aux, db.aux.data(), db.aux.size() * sizeof(RowAux), "aux") &&
         check(d_.aux_ids, db.aux_ids.data(), db.aux_ids.size() * 4, "aux_ids");
}

}  // namespace tvm
