// Device engine (host side of the match path): HBM-resident advisory tables, batch
// upload, variant selection and launch of the match kernel (match_kernel.h, instantiated
// in kern_*.hip), and ordered read-back of the per-package advisory lists.
#include "engine.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "db.h"
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {

// kern_*.hip
const LaunchFn* launch_table_DEB_TUNED();
const LaunchFn* launch_table_OS_TUNED();
const LaunchFn* launch_table_ALL_TUNED();
const LaunchFn* launch_table_DEB_ABLATION();
const LaunchFn* launch_table_OS_ABLATION();
const LaunchFn* launch_table_ALL_ABLATION();

namespace {

// Variant table: index 0 = "auto" (kAutoVariant per grammar set), then the tuned list,
// then the ablations (match_variants.h).  The launch functions live in the kern_*.hip
// tables, indexed by (grammar set, list, position); the host launches the smallest
// grammar set that covers the batch's platforms, so a dpkg-only batch runs a kernel with
// only the dpkg encoder in it (no library-grammar register/scratch footprint).
struct VariantInfo {
  int tile;
  int kw;
  bool kg;       // installed keys in global memory (KW words per package)
  const char* name;
};
#define TVM_INFO_(T, KW, MB, KG, AB, NAME) {T, KW, KG, NAME},
constexpr VariantInfo kTunedInfo[] = {TVM_TUNED_VARIANTS(TVM_INFO_)};
constexpr VariantInfo kAblInfo[] = {TVM_ABLATION_VARIANTS(TVM_INFO_)};
#undef TVM_INFO_
static_assert(sizeof(kTunedInfo) / sizeof(VariantInfo) == kNumTuned, "tuned list");
static_assert(sizeof(kAblInfo) / sizeof(VariantInfo) == kNumAblations, "ablation list");
constexpr int kNumVariants = 1 + kNumTuned + kNumAblations;
constexpr int kMinTile = 64;
constexpr int kMinKeyWords = 4;

// Variant v (>= 1) of the table above.
const VariantInfo& variant_info(int v) { return v <= kNumTuned ? kTunedInfo[v - 1] : kAblInfo[v - 1 - kNumTuned]; }

// Grammar-set index of a batch: 0 = dpkg only, 1 = OS grammars, 2 = any.
int grammar_index(uint32_t gm) { return (gm & ~GM_DEB) == 0 ? 0 : (gm & ~GM_OS) == 0 ? 1 : 2; }

LaunchFn launch_fn(int gi, int v) {
  static const LaunchFn* const tuned[3] = {launch_table_DEB_TUNED(), launch_table_OS_TUNED(), launch_table_ALL_TUNED()};
  static const LaunchFn* const abl[3] = {launch_table_DEB_ABLATION(), launch_table_OS_ABLATION(),
                                         launch_table_ALL_ABLATION()};
  return v <= kNumTuned ? tuned[gi][v - 1] : abl[gi][v - 1 - kNumTuned];
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

}  // namespace

int num_variants() { return kNumVariants; }
const char* variant_name(int v) {
  if (v == 0) return "auto";
  return v > 0 && v < kNumVariants ? variant_info(v).name : nullptr;
}
int resolve_variant(int v, uint32_t gm) { return v == 0 ? 1 + kAutoVariant[grammar_index(gm)] : v; }

void HostBatch::add(uint32_t plat, std::string_view name, std::string_view ver) {
  uint4 d;
  d.x = plat;
  d.y = uint32_t(arena.size());
  arena.insert(arena.end(), name.begin(), name.end());
  d.z = uint32_t(arena.size());
  arena.insert(arena.end(), ver.begin(), ver.end());
  d.w = uint32_t(std::min<size_t>(name.size(), 0xFFFF)) | (uint32_t(std::min<size_t>(ver.size(), 0xFFFF)) << 16);
  desc.push_back(d);
  if (!attr.empty()) attr.push_back(make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu));
}

void HostBatch::add(uint32_t plat, std::string_view name, std::string_view ver, uint2 a) {
  if (attr.size() < desc.size()) attr.resize(desc.size(), make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu));
  add(plat, name, ver);
  if (attr.size() < desc.size()) attr.push_back(a);
  else attr.back() = a;
}

Engine::~Engine() {
  if (dev_ >= 0) (void)hipSetDevice(dev_);
  for (void* p : allocs_) (void)hipFree(p);
  if (spill_) (void)hipFree(spill_);
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
  Slot* sl; uint8_t* na; Row* rows; uint64_t* kw; PlatInfo* pl; RowAux* ax; uint32_t* ai;
  bool ok = upload_vec(db.aux, &ax, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.aux_ids, &ai, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.slots, &sl, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.name_arena, &na, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.rows, &rows, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.key_words, &kw, e->allocs_, e->table_bytes_, err) &&
            upload_vec(db.plat_info, &pl, e->allocs_, e->table_bytes_, err);
  if (!ok) {
    delete e;
    return nullptr;
  }
  e->d_.slots = sl;
  e->d_.slot_mask = db.slot_mask;
  e->d_.name_arena = na;
  e->d_.rows = rows;
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

bool Engine::ensure_scratch(uint64_t spill_words, std::string& err) {
  if (spill_words > spill_cap_) {
    if (spill_) (void)hipFree(spill_);
    spill_ = nullptr;
    const uint64_t cap = std::max<uint64_t>(spill_words, 4096);
    if (!hip_ok(hipMalloc(&spill_, cap * 8), "hipMalloc(spill)", err)) return false;
    spill_cap_ = cap;
  }
  return true;
}

// Grammar bits (1 << Cmp) of the platforms a batch touches.
uint32_t Engine::grammar_set(const HostBatch& hb) const {
  const auto& pi = db_->plat_info;
  std::vector<uint8_t> seen(pi.size(), 0);
  uint32_t gm = 0;
  for (const uint4& d : hb.desc)
    if (d.x < pi.size() && !seen[d.x]) {
      seen[d.x] = 1;
      gm |= 1u << pi[d.x].cmp;
    }
  return gm & GM_ALL;
}

bool Engine::upload(const HostBatch& hb, DevBatch& b, std::string& err) {
  (void)hipSetDevice(dev_);
  b.n = uint32_t(hb.desc.size());
  b.arena_bytes = hb.arena.size();
  b.spill_words = 0;
  b.gm = grammar_set(hb);
  for (const uint4& d : hb.desc) {
    const uint32_t need = (key_bound_any(d.w >> 16) + 7) / 8;  // the widest grammar bound
    if (need > uint32_t(kMinKeyWords)) b.spill_words += need;  // bound for every variant
  }
  if (!hip_ok(hipMalloc(&b.desc, std::max<size_t>(hb.desc.size(), 1) * sizeof(uint4)), "hipMalloc(batch)", err)) return false;
  // +32 B tail: the kernel stages whole 16-byte lines of the arena into LDS
  if (!hip_ok(hipMalloc(&b.arena, (hb.arena.size() + 32 + 15) & ~size_t(15)), "hipMalloc(batch arena)", err)) return false;
  if (!hb.desc.empty() &&
      !hip_ok(hipMemcpy(b.desc, hb.desc.data(), hb.desc.size() * sizeof(uint4), hipMemcpyHostToDevice), "H2D batch", err))
    return false;
  if (!hb.arena.empty() &&
      !hip_ok(hipMemcpy(b.arena, hb.arena.data(), hb.arena.size(), hipMemcpyHostToDevice), "H2D arena", err))
    return false;
  if (!hb.attr.empty()) {
    if (hb.attr.size() != hb.desc.size()) {
      err = "batch attributes do not cover every package";
      return false;
    }
    if (!hip_ok(hipMalloc(&b.attr, hb.attr.size() * sizeof(uint2)), "hipMalloc(batch attr)", err) ||
        !hip_ok(hipMemcpy(b.attr, hb.attr.data(), hb.attr.size() * sizeof(uint2), hipMemcpyHostToDevice), "H2D attr", err))
      return false;
  }
  if (!hb.cpe_bits.empty() && hb.cpe_words) {
    if (!hip_ok(hipMalloc(&b.cpe_bits, hb.cpe_bits.size() * 4), "hipMalloc(cpe sets)", err) ||
        !hip_ok(hipMemcpy(b.cpe_bits, hb.cpe_bits.data(), hb.cpe_bits.size() * 4, hipMemcpyHostToDevice), "H2D cpe", err))
      return false;
    b.cpe_words = hb.cpe_words;
    b.n_cpe_sets = uint32_t(hb.cpe_bits.size() / hb.cpe_words);
  }
  return true;
}

void Engine::free_batch(DevBatch& b) {
  (void)hipSetDevice(dev_);
  if (b.desc) (void)hipFree(b.desc);
  if (b.arena) (void)hipFree(b.arena);
  if (b.attr) (void)hipFree(b.attr);
  if (b.cpe_bits) (void)hipFree(b.cpe_bits);
  b = DevBatch{};
}

bool Engine::alloc_matches(uint64_t cap, uint32_t n_pkgs, DevMatches& m, std::string& err) {
  (void)hipSetDevice(dev_);
  m.cap = std::max<uint64_t>(cap, 1);
  m.dir_cap = std::max<uint32_t>((n_pkgs + kMinTile - 1) / kMinTile, 1);
  if (!hip_ok(hipMalloc(&m.pairs, m.cap * sizeof(uint2)), "hipMalloc(matches)", err)) return false;
  if (!hip_ok(hipMalloc(&m.dir, m.dir_cap * sizeof(TileDir)), "hipMalloc(tile dir)", err)) return false;
  if (!hip_ok(hipMalloc(&m.ctl, 8 * sizeof(unsigned long long)), "hipMalloc(ctl)", err)) return false;
  return true;
}

void Engine::free_matches(DevMatches& m) {
  (void)hipSetDevice(dev_);
  if (m.pairs) (void)hipFree(m.pairs);
  if (m.dir) (void)hipFree(m.dir);
  if (m.ctl) (void)hipFree(m.ctl);
  m = DevMatches{};
}

bool Engine::fetch_ordered(const DevMatches& m, uint32_t n_pkgs, uint64_t total, std::vector<uint2>& out,
                           std::string& err) {
  out.clear();
  if (total > m.cap) {
    err = "match buffer too small";
    return false;
  }
  unsigned long long ctl[8];
  if (!hip_ok(hipMemcpy(ctl, m.ctl, sizeof(ctl), hipMemcpyDeviceToHost), "D2H ctl", err)) return false;
  const uint32_t tile = ctl[5] ? uint32_t(ctl[5]) : 256;
  const uint32_t n_tiles = (n_pkgs + tile - 1) / tile;
  std::vector<TileDir> dir(n_tiles);
  std::vector<uint2> raw(total);
  if (n_tiles && !hip_ok(hipMemcpy(dir.data(), m.dir, n_tiles * sizeof(TileDir), hipMemcpyDeviceToHost), "D2H dir", err))
    return false;
  if (total && !hip_ok(hipMemcpy(raw.data(), m.pairs, total * sizeof(uint2), hipMemcpyDeviceToHost), "D2H matches", err))
    return false;
  out.reserve(total);
  for (const TileDir& d : dir) out.insert(out.end(), raw.begin() + d.base, raw.begin() + d.base + d.count);
  return true;
}

bool Engine::launch(const DevBatch& b, const DevMatches& m, hipStream_t st, std::string& err) {
  (void)hipSetDevice(dev_);
  const int vi = resolve_variant(variant_, b.gm);
  const VariantInfo& v = variant_info(vi);
  last_launched_ = vi;
  const uint32_t n_tiles = (b.n + v.tile - 1) / v.tile;
  if (n_tiles > m.dir_cap) {
    err = "tile directory smaller than the batch";
    return false;
  }
  const uint64_t kslots = v.kg ? uint64_t(n_tiles) * v.tile * v.kw : 0;  // KG: per-package key slots
  if (!ensure_scratch(b.spill_words + kslots, err)) return false;
  if (!hip_ok(hipMemsetAsync(m.ctl, 0, 8 * sizeof(unsigned long long), st), "memset(ctl)", err)) return false;
  if (n_tiles == 0) return true;
  MatchArgs a;
  a.db = d_;
  a.desc = b.desc;
  a.arena = b.arena;
  a.attr = b.attr;
  a.cpe_bits = b.cpe_bits;
  a.cpe_words = b.cpe_words;
  a.n_cpe_sets = b.n_cpe_sets;
  a.n = b.n;
  a.n_tiles = n_tiles;
  a.out = m.pairs;
  a.out_cap = m.cap;
  a.dir = m.dir;
  a.ctl = m.ctl;
  a.kbuf = spill_;
  a.spill = spill_ + kslots;
  a.spill_cap = spill_cap_ - kslots;
  launch_fn(grammar_index(b.gm), vi)(n_tiles, st, a);
  return hip_ok(hipGetLastError(), "match_kernel launch", err);
}

bool Engine::match_host(const HostBatch& hb, std::vector<uint2>& out, int64_t& err_pkg, std::string& err) {
  out.clear();
  err_pkg = -1;
  if (hb.desc.empty()) return true;
  std::lock_guard<std::mutex> lk(call_mu_);
  DevBatch b;
  if (!upload(hb, b, err)) {
    free_batch(b);
    return false;
  }
  uint64_t cap = std::max<uint64_t>(hb.desc.size() * 4, 1024);
  bool ok = true;
  for (int attempt = 0; attempt < 2 && ok; attempt++) {
    DevMatches m;
    ok = alloc_matches(cap, b.n, m, err) && launch(b, m, stream_, err) &&
         hip_ok(hipStreamSynchronize(stream_), "match_kernel", err);
    unsigned long long ctl[8] = {0};
    if (ok) ok = hip_ok(hipMemcpy(ctl, m.ctl, sizeof(ctl), hipMemcpyDeviceToHost), "D2H ctl", err);
    if (ok && ctl[3]) {
      err = "match kernel internal error bits " + std::to_string(ctl[3]);
      ok = false;
    }
    if (ok && ctl[0] > cap) {  // output buffer too small: rerun with the exact size
      cap = ctl[0];
      free_matches(m);
      continue;
    }
    if (ok) {
      err_pkg = ctl[1] ? int64_t(b.n - ctl[1]) : -1;
      ok = fetch_ordered(m, b.n, ctl[0], out, err);
    }
    free_matches(m);
    break;
  }
  free_batch(b);
  return ok;
}

}  // namespace tvm

namespace tvm {

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
         check(d_.name_arena, db.name_arena.data(), db.name_arena.size(), "name_arena") &&
         check(d_.rows, db.rows.data(), db.rows.size() * sizeof(Row), "rows") &&
         check(d_.key_words, db.key_words.data(), db.key_words.size() * 8, "key_words") &&
         check(d_.plats, db.plat_info.data(), db.plat_info.size() * sizeof(PlatInfo), "plats") &&
         check(d_.aux, db.aux.data(), db.aux.size() * sizeof(RowAux), "aux") &&
         check(d_.aux_ids, db.aux_ids.data(), db.aux_ids.size() * 4, "aux_ids");
}

}  // namespace tvm
