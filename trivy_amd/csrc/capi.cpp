// C-ABI implementation (include/trivy_amd.h).
#include "../../include/trivy_amd.h"

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "db.h"
#include "drivers.h"
#include "export.h"
#include "engine.h"
#include "libdb.h"
#include "libver.h"
#include "bbolt.h"
#include "host_par.h"
#include "pipeline.h"
#include "pool.h"
#include "sbom.h"
#include "wire.h"
#include "redhat.h"
#include "vulninfo.h"

using namespace tvm;

// The advisory side of every advisory's DetectedVulnerability (drivers.h advisory_templates)
// in C form, built once per DB on the first batch export.
struct VulnTemplates {
  std::vector<tvm::Vuln> v;
  std::vector<tvm_vuln> c;
  std::vector<std::vector<const char*>> vp;
};

struct tvm_db {
  DB db;
  VulnTable vt;  // bucket "vulnerability" (FillInfo tables)
  bool finalized = false;
  std::mutex tmpl_mu;
  std::unique_ptr<VulnTemplates> tmpl;
};

struct tvm_engine {
  std::shared_mutex mu;  // calls share; swap is exclusive (listen.go:154-190 quiesce)
  std::unique_ptr<Engine> eng;
  std::unique_ptr<FillEngine> fill;
  std::mutex rh_mu;                   // lazily built Red Hat fixed-version ranks (device)
  uint2* rh_rank = nullptr;  // per advisory {vulnerability-ID rank, rpm rank of FixedVersion} (Red Hat merge)
  ~tvm_engine() {
    if (rh_rank) {
      (void)hipSetDevice(device);
      (void)hipFree(rh_rank);
    }
  }
  tvm_db* db = nullptr;
  int device = 0;
  uint64_t gen = 0;  // table generation: tvm_engine_swap increments it (under the exclusive lock)
};

struct tvm_batch {
  HostBatch hb;
  DevBatch dev;
  DevMatches m;
  uint4* fill_out = nullptr;  // tvm_match_fill decisions, parallel to the match columns
  uint64_t fill_cap = 0;
  uint2* fill_side() const { return reinterpret_cast<uint2*>(fill_out + fill_cap); }
  std::vector<uint32_t> target_begin;  // first package of every result (one per add call)
  BatchFilter filter;                  // tvm_match_filter state
  // the list's length as last read back (match_status_locked), until the next launch / merge /
  // upload: tvm_match_filter reads it without a host round trip
  bool st_valid = false;
  uint64_t st_n = 0;
  int64_t st_errp = -1;
  // batch_has_redhat's answer for the first rh_seen_n packages against rh_seen_db
  mutable uint64_t rh_seen_n = ~0ull;
  mutable const void* rh_seen_db = nullptr;
  mutable bool rh_seen = false;
  // tvm_batch_set_report: per package PkgName / InstalledVersion / PkgPath overrides
  // (rep[f][i] counts where rep_has[f][i] is set; shorter vectors = defaults beyond)
  std::vector<std::string> rep[3];
  std::vector<uint8_t> rep_has[3];
  RedHatMerge rh;                      // tvm_match_redhat_merge / _result state
  bool merged = false;                 // the merged list (rh) is the current match list
  std::unique_ptr<Pipeline> pipe;      // tvm_pipeline_* state
  uint32_t pkg_base = 0;               // tvm_batch_set_package_base
  uint64_t pipe_total = 0;
  bool pipe_ok = false;                // the pipeline's last pass completed (its result is valid)
  int64_t pipe_errp = -1;              // that pass's first poisoned package (-1: none)
  RedHatMerge pipe_rh;                 // the per-CVE merge over a pipelined pass's list (tvm_pipeline_vulns)
  uint64_t pipe_runs = 0, pipe_wide_for = ~0ull;  // passes run; the pass pipe_wide was widened for
  std::vector<uint32_t> pipe_wide;                // 3-byte result indices widened (tvm_pipeline_result)
  unsigned long long* order_scratch = nullptr;  // tvm_match_order_into: ticket + look-back word per tile
  uint32_t order_cap = 0;
  bool external_out = false;  // m.pkg / m.adv belong to the caller (tvm_batch_upload_into)
  bool uploaded = false;      // dev / m hold real device buffers
  bool pinned = false;        // tvm_pipeline_prepare pinned the host arrays: no more adds
  int device = 0;
  // The engine and table generation the batch's platform / arch / CPE ids were resolved
  // against (bound at the first call that names an engine); after tvm_engine_swap the
  // batch must be rebuilt, since the new DB numbers its platforms differently.
  const tvm_engine* owner = nullptr;
  uint64_t gen = 0;
};

namespace {

void set_err(char* err, size_t errlen, const std::string& msg) {
  if (!err || errlen == 0) return;
  size_t n = std::min(errlen - 1, msg.size());
  memcpy(err, msg.data(), n);
  err[n] = 0;
}

std::string_view sv(const tvm_str& s) { return s.p ? std::string_view(s.p, s.n) : std::string_view(); }

// Binds a batch to (engine, generation) on first use; false when it belongs to another
// engine or to tables a swap has replaced.  Callers hold the engine's lock (shared).
bool bind(tvm_batch* b, const tvm_engine* e) {
  if (!b->owner) {
    b->owner = e;
    b->gen = e->gen;
    return true;
  }
  return b->owner == e && b->gen == e->gen;
}

// The batch's current match list: the merged one after tvm_match_redhat_merge.
const DevMatches& cur(const tvm_batch* b) { return b->merged ? b->rh.merged().m : b->m; }
const uint32_t* cur_base(const tvm_batch* b) { return b->merged ? b->rh.merged().base : nullptr; }

constexpr const char* kStale =
    "batch was built against other tables (another engine, or before tvm_engine_swap): rebuild it";

std::vector<Pkg> to_pkgs(const tvm_package* pkgs, size_t n) {
  std::vector<Pkg> out(n);
  for (size_t i = 0; i < n; i++) {
    const tvm_package& p = pkgs[i];
    Pkg& q = out[i];
    q.id = sv(p.id);
    q.name = sv(p.name);
    q.version = sv(p.version);
    q.release = sv(p.release);
    q.arch = sv(p.arch);
    q.epoch = p.epoch;
    q.src_name = sv(p.src_name);
    q.src_version = sv(p.src_version);
    q.src_release = sv(p.src_release);
    q.src_epoch = p.src_epoch;
    q.modularitylabel = sv(p.modularitylabel);
    q.has_build_info = p.has_build_info != 0;
    for (size_t k = 0; k < p.n_content_sets; k++) q.content_sets.push_back(sv(p.content_sets[k]));
    q.nvr = sv(p.nvr);
    q.build_arch = sv(p.build_arch);
    q.file_path = sv(p.file_path);
  }
  return out;
}

struct ResultStore {
  std::vector<Vuln> v;
  std::vector<tvm_vuln> c;
  std::vector<std::vector<const char*>> vendor_ptrs;
};

// One Vuln in C form; vp holds its VendorIDs pointers (both live as long as v).
void to_c(const DB& db, const Vuln& v, tvm_vuln& c, std::vector<const char*>& vp) {
  memset(&c, 0, sizeof(c));
  c.pkg_index = v.pkg;
  c.copy_flags = v.copy;
  c.vulnerability_id = v.vuln_id.c_str();
  if (!v.vendor_ids.empty()) {
    for (const std::string& s : v.vendor_ids) vp.push_back(s.c_str());
    c.vendor_ids = vp.data();
    c.n_vendor_ids = v.vendor_ids.size();
  }
  c.pkg_id = v.pkg_id.c_str();
  c.pkg_name = v.pkg_name.c_str();
  c.pkg_path = v.pkg_path.c_str();
  c.installed_version = v.installed.c_str();
  c.fixed_version = v.fixed.c_str();
  c.status = v.status;
  c.severity_source = v.severity_source.c_str();
  c.severity = v.severity.c_str();
  if (v.data_source >= 0) {
    const DataSource& ds = db.sources[size_t(v.data_source)];
    c.has_data_source = 1;
    c.data_source_id = ds.id.c_str();
    c.data_source_name = ds.name.c_str();
    c.data_source_url = ds.url.c_str();
  } else {
    c.data_source_id = c.data_source_name = c.data_source_url = "";
  }
  c.custom_json = v.has_custom ? v.custom.c_str() : nullptr;
}

void export_result(const DB& db, std::vector<Vuln>&& vulns, bool eosl, tvm_result* out) {
  auto* rs = new ResultStore();
  rs->v = std::move(vulns);
  rs->c.resize(rs->v.size());
  rs->vendor_ptrs.resize(rs->v.size());
  for (size_t i = 0; i < rs->v.size(); i++) to_c(db, rs->v[i], rs->c[i], rs->vendor_ptrs[i]);
  out->vulns = rs->c.data();
  out->n = rs->c.size();
  out->eosl = eosl ? 1 : 0;
  out->priv = rs;
}

}  // namespace

extern "C" {

const char* tvm_version(void) { return "trivy_amd 0.1.0 (gfx950)"; }
int tvm_abi_version(void) { return TVM_ABI_VERSION; }

tvm_db* tvm_db_new(void) { return new tvm_db(); }
void tvm_db_free(tvm_db* db) { delete db; }

int tvm_db_put(tvm_db* db, const tvm_str* path, size_t depth, const char* value, size_t vlen) {
  if (!db || db->finalized || !path || depth == 0) return TVM_EINVAL;
  std::vector<std::string> p(depth);
  for (size_t i = 0; i < depth; i++) p[i] = std::string(sv(path[i]));
  db->db.put(p, std::string_view(value ? value : "", value ? vlen : 0));
  return TVM_OK;
}

int tvm_bbolt_walk(const void* bytes, size_t len, tvm_bbolt_visit visit, void* ctx, char* err, size_t errlen) {
  if ((!bytes && len) || !visit) return TVM_EINVAL;
  std::vector<tvm_str> p;
  std::string msg;
  const bool ok = tvm::bbolt_walk(
      static_cast<const uint8_t*>(bytes), len,
      [&](const std::vector<std::string_view>& path, std::string_view v) {
        p.resize(path.size());
        for (size_t i = 0; i < path.size(); i++) p[i] = tvm_str{path[i].data(), path[i].size()};
        return visit(ctx, p.data(), p.size(), v.data(), v.size()) == 0;
      },
      msg);
  if (!ok) {
    set_err(err, errlen, msg);
    return TVM_EINVAL;
  }
  return TVM_OK;
}

int tvm_db_put_bbolt(tvm_db* db, const void* bytes, size_t len, char* err, size_t errlen) {
  if (!db || db->finalized || (!bytes && len)) return TVM_EINVAL;
  std::vector<std::string> p;
  std::string msg;
  const bool ok = tvm::bbolt_walk(
      static_cast<const uint8_t*>(bytes), len,
      [&](const std::vector<std::string_view>& path, std::string_view v) {
        p.resize(path.size());
        for (size_t i = 0; i < path.size(); i++) p[i].assign(path[i]);
        db->db.put(p, v);
        return true;
      },
      msg);
  if (!ok) {
    set_err(err, errlen, msg);
    return TVM_EINVAL;
  }
  return TVM_OK;
}

int tvm_db_put_many(tvm_db* db, size_t n, const tvm_str* paths, size_t depth, const tvm_str* values) {
  if (!db || db->finalized || (n && (!paths || !values)) || depth == 0) return TVM_EINVAL;
  std::vector<std::string> p(depth);
  for (size_t r = 0; r < n; r++) {
    for (size_t i = 0; i < depth; i++) p[i] = std::string(sv(paths[r * depth + i]));
    db->db.put(p, sv(values[r]));
  }
  return TVM_OK;
}

int tvm_db_put_arena(tvm_db* db, size_t n, size_t depth, const char* arena, const uint64_t* off,
                     const uint32_t* len) {
  if (!db || db->finalized || depth == 0 || (n && (!arena || !off || !len))) return TVM_EINVAL;
  std::vector<std::string> p(depth);
  for (size_t r = 0; r < n; r++) {
    const size_t b = r * (depth + 1);
    for (size_t i = 0; i < depth; i++) p[i].assign(arena + off[b + i], len[b + i]);
    db->db.put(p, std::string_view(arena + off[b + depth], len[b + depth]));
  }
  return TVM_OK;
}

int tvm_db_finalize(tvm_db* db, char* err, size_t errlen) {
  if (!db || db->finalized) return TVM_EINVAL;
  std::string e;
  if (!db->db.finalize(e)) {
    set_err(err, errlen, e);
    return TVM_EINVAL;
  }
  db->vt.build(db->db);
  db->finalized = true;
  return TVM_OK;
}

void tvm_db_stats(const tvm_db* db, uint64_t out[5]) {
  out[0] = db->db.plats.size();
  out[1] = db->db.keys.size();
  out[2] = db->db.advs.size();
  out[3] = db->db.rows.size();
  out[4] = db->db.key_words.size() * 8;
}

const char* tvm_db_advisory_vuln_id(const tvm_db* db, uint32_t adv) {
  return adv < db->db.advs.size() ? db->db.advs[adv].vuln_id.c_str() : nullptr;
}

// Devices an engine was opened on (bit d): tvm_shutdown drains those alone, and starts no
// HIP runtime in a process that never opened one (SBOM decode, host-only work)
static std::atomic<uint64_t> g_used_devices{0};

tvm_engine* tvm_engine_open(tvm_db* db, int device, char* err, size_t errlen) {
  if (device >= 0 && device < 64) g_used_devices.fetch_or(uint64_t(1) << device);
  if (!db || !db->finalized) {
    set_err(err, errlen, "tvm_engine_open: DB not finalized");
    return nullptr;
  }
  std::string e;
  Engine* eng = Engine::open(db->db, device, e);
  if (!eng) {
    set_err(err, errlen, e);
    return nullptr;
  }
  FillEngine* fill = FillEngine::open(db->vt, device, e);
  if (!fill) {
    delete eng;
    set_err(err, errlen, e);
    return nullptr;
  }
  auto* t = new tvm_engine();
  t->eng.reset(eng);
  t->fill.reset(fill);
  t->db = db;
  t->device = device;
  return t;
}

void tvm_engine_close(tvm_engine* e) { delete e; }

void tvm_shutdown(void) {
  // every device an engine of this library ran on: drain whatever the library queued
  const uint64_t used = g_used_devices.load();
  for (int d = 0; d < 64; d++)
    if ((used >> d) & 1u)
      if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
  WorkerPool::shutdown_all();
  release_encoders();
  pool_close();
}

int tvm_device_sync(int device, char* err, size_t errlen) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    set_err(err, errlen, "tvm_device_sync: no such HIP device");
    return TVM_EDEVICE;
  }
  (void)hipSetDevice(device);
  hipError_t st = hipDeviceSynchronize();
  if (st == hipSuccess) st = hipGetLastError();
  if (st != hipSuccess) {
    set_err(err, errlen, std::string("tvm_device_sync: ") + hipGetErrorString(st));
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

int tvm_engine_swap(tvm_engine* e, tvm_db* db, char* err, size_t errlen) {
  if (!e || !db || !db->finalized) return TVM_EINVAL;
  std::string msg;
  Engine* fresh = Engine::open(db->db, e->device, msg);  // build before quiescing
  FillEngine* fresh_fill = fresh ? FillEngine::open(db->vt, e->device, msg) : nullptr;
  if (!fresh || !fresh_fill) {
    delete fresh;
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  std::unique_lock<std::shared_mutex> lk(e->mu);
  (void)hipSetDevice(e->device);
  e->eng.reset(fresh);  // ~Engine drains its streams before it frees the tables
  e->fill.reset(fresh_fill);
  e->db = db;
  e->gen++;
  if (e->rh_rank) {
    (void)hipFree(e->rh_rank);
    e->rh_rank = nullptr;
  }
  return TVM_OK;
}

uint64_t tvm_engine_table_bytes(const tvm_engine* e) { return e ? e->eng->table_bytes() : 0; }

int tvm_engine_dropin_stats(tvm_engine* e, uint64_t* out3) {
  if (!e || !out3) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  e->eng->dropin_stats(out3);
  return TVM_OK;
}

int tvm_engine_verify(tvm_engine* e, char* err, size_t errlen) {
  if (!e) return TVM_EINVAL;
  std::unique_lock<std::shared_mutex> lk(e->mu);
  std::string msg;
  if (!e->eng->verify(msg)) {
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

int tvm_engine_set_variant(tvm_engine* e, int v) {
  if (!e) return -1;
  std::unique_lock<std::shared_mutex> lk(e->mu);
  return v < 0 ? e->eng->variant() : e->eng->set_variant(v);
}

const char* tvm_variant_name(int v) { return variant_name(v); }
int tvm_variant_grammar_sets(int v) { return variant_grammar_sets(v); }

int tvm_engine_last_variant(tvm_engine* e) {
  if (!e) return -1;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  return e->eng->last_launched();
}

static int detect_common(tvm_engine* e, bool full, const char* fam, const char* ver, const tvm_repository* repo,
                         const tvm_package* pkgs, size_t n, int64_t now, tvm_result* out, char* err,
                         size_t errlen) {
  if (!e || !fam || !ver || !out || (n && !pkgs)) return TVM_EINVAL;
  memset(out, 0, sizeof(*out));
  std::shared_lock<std::shared_mutex> lk(e->mu);
  std::vector<Pkg> p = to_pkgs(pkgs, n);
  Repo r;
  if (repo) {
    r.family = sv(repo->family);
    r.release = sv(repo->release);
  }
  std::vector<Vuln> vulns;
  std::string msg;
  bool eosl = false;
  if (full) {
    DetectStatus st = ospkg_detect(*e->eng, fam, ver, repo ? &r : nullptr, p, now, vulns, eosl, msg);
    if (st != DETECT_OK) {
      set_err(err, errlen, msg);
      return st == DETECT_UNSUPPORTED_OS ? TVM_EUNSUPPORTED_OS : TVM_EDETECT;
    }
  } else {
    const OsDriver* d = find_os_driver(fam);
    if (!d) {
      set_err(err, errlen, "unsupported os");
      return TVM_EUNSUPPORTED_OS;
    }
    if (!d->detect(*e->eng, ver, repo ? &r : nullptr, p, now, vulns, msg)) {
      set_err(err, errlen, msg);
      return TVM_EDETECT;
    }
  }
  export_result(e->eng->db(), std::move(vulns), eosl, out);
  return TVM_OK;
}

int tvm_ospkg_detect(tvm_engine* e, const char* f, const char* v, const tvm_repository* repo, const tvm_package* pkgs,
                     size_t n, int64_t now, tvm_result* out, char* err, size_t errlen) {
  return detect_common(e, true, f, v, repo, pkgs, n, now, out, err, errlen);
}

int tvm_ospkg_driver_detect(tvm_engine* e, const char* f, const char* v, const tvm_repository* repo,
                            const tvm_package* pkgs, size_t n, int64_t now, tvm_result* out, char* err,
                            size_t errlen) {
  return detect_common(e, false, f, v, repo, pkgs, n, now, out, err, errlen);
}

int tvm_ospkg_is_supported(const char* fam, const char* ver, int64_t now) {
  const OsDriver* d = fam ? find_os_driver(fam) : nullptr;
  if (!d || !ver) return -1;
  return d->is_supported(fam, ver, now) ? 1 : 0;
}

void tvm_result_free(tvm_result* r) {
  if (!r) return;
  delete static_cast<ResultStore*>(r->priv);
  memset(r, 0, sizeof(*r));
}

// ---- batches ------------------------------------------------------------------------------

tvm_batch* tvm_batch_new(void) { return new tvm_batch(); }

void tvm_batch_free(tvm_batch* b) {
  if (!b) return;
  b->pipe.reset();
  if (b->order_scratch) {
    (void)hipSetDevice(b->device);
    (void)hipFree(b->order_scratch);
  }
  if (b->uploaded) {
    (void)hipSetDevice(b->device);
    for (void* p : {static_cast<void*>(b->dev.pk), static_cast<void*>(b->dev.tile_off), static_cast<void*>(b->dev.arena),
                    static_cast<void*>(b->dev.attr), static_cast<void*>(b->dev.cpe_bits), static_cast<void*>(b->dev.rec),
                    static_cast<void*>(b->dev.tail), static_cast<void*>(b->dev.spill),
                    static_cast<void*>(b->external_out ? nullptr : b->m.pkg),
                    static_cast<void*>(b->external_out ? nullptr : b->m.adv), static_cast<void*>(b->m.dir),
                    static_cast<void*>(b->m.ctl),
                    static_cast<void*>(b->fill_out)})
      if (p) (void)hipFree(p);
  }
  delete b;
}

// Geometric growth: many small add_many calls (one per target) must not re-allocate the
// descriptor array to its exact size every time (quadratic copying).
static void reserve_more(HostBatch& hb, size_t n) {
  const size_t want = hb.pk.size() + n;
  if (want > hb.pk.capacity()) hb.pk.reserve(std::max(want, 2 * hb.pk.capacity()));
}

int64_t tvm_batch_add(tvm_batch* b, tvm_engine* e, const char* bucket, tvm_str name, tvm_str version) {
  if (!b || !e || !bucket || b->uploaded || b->pinned) return -1;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) return -1;
  b->target_begin.push_back(uint32_t(b->hb.pk.size()));
  int32_t plat = e->eng->db().find_plat(bucket);
  b->hb.add(plat < 0 ? 0xFFFFFFFFu : uint32_t(plat), sv(name), sv(version));
  return int64_t(b->hb.pk.size() - 1);
}

int64_t tvm_batch_add_many(tvm_batch* b, tvm_engine* e, const char* bucket, size_t n, const char* arena,
                           const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                           const uint32_t* ver_len) {
  if (!b || !e || !bucket || b->uploaded || b->pinned ||
      (n && (!arena || !name_off || !name_len || !ver_off || !ver_len)))
    return -1;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) return -1;
  int32_t plat = e->eng->db().find_plat(bucket);
  const uint32_t pid = plat < 0 ? 0xFFFFFFFFu : uint32_t(plat);
  const int64_t first = int64_t(b->hb.pk.size());
  b->target_begin.push_back(uint32_t(first));
  reserve_more(b->hb, n);
  for (size_t i = 0; i < n; i++)
    b->hb.add(pid, std::string_view(arena + name_off[i], name_len[i]), std::string_view(arena + ver_off[i], ver_len[i]));
  return first;
}

int64_t tvm_batch_add_many_ex(tvm_batch* b, tvm_engine* e, const char* bucket, size_t n, const char* arena,
                              const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                              const uint32_t* ver_len, const uint64_t* arch_off, const uint32_t* arch_len,
                              uint32_t flags) {
  if (flags & TVM_ATTR_CPESET) return -1;  // needs the set column: tvm_batch_add_many_attrs
  tvm_attr_cols cols{arch_off, arch_len, nullptr};
  return tvm_batch_add_many_attrs(b, e, bucket, n, arena, name_off, name_len, ver_off, ver_len, &cols, flags);
}

int64_t tvm_batch_cpe_set(tvm_batch* b, tvm_engine* e, const tvm_str* content_sets, size_t n, tvm_str nvr) {
  if (!b || !e || b->uploaded || b->pinned || (n && !content_sets)) return -1;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) return -1;
  const DB& db = e->eng->db();
  HostBatch& hb = b->hb;
  const uint32_t words = std::max<uint32_t>((db.n_cpe + 31) / 32, 1);
  if (hb.cpe_words == 0) hb.cpe_words = words;
  if (hb.cpe_words != words) return -1;
  std::vector<std::string_view> repos, nvrs;
  for (size_t i = 0; i < n; i++) repos.push_back(sv(content_sets[i]));
  nvrs.push_back(sv(nvr));
  const size_t id = hb.cpe_bits.size() / words;
  hb.cpe_bits.resize(hb.cpe_bits.size() + words, 0u);
  uint32_t* bits = hb.cpe_bits.data() + id * words;
  for (int64_t c : db.redhat_cpes(repos, nvrs))
    if (c >= 0 && uint64_t(c) < uint64_t(words) * 32) bits[c >> 5] |= 1u << (c & 31);
  return int64_t(id);
}

int64_t tvm_batch_add_many_attrs(tvm_batch* b, tvm_engine* e, const char* bucket, size_t n, const char* arena,
                                 const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                                 const uint32_t* ver_len, const tvm_attr_cols* cols, uint32_t flags) {
  const uint32_t known = TVM_ATTR_ARCH | TVM_ATTR_KSPLICE | TVM_ATTR_CPESET;
  if (!b || !e || !bucket || b->uploaded || b->pinned || (flags & ~known) ||
      ((flags & TVM_ATTR_KSPLICE) && (flags & TVM_ATTR_CPESET)) ||  // one attribute word: tag or CPE set
      (n && (!arena || !name_off || !name_len || !ver_off || !ver_len)) ||
      (n && (flags & (TVM_ATTR_ARCH | TVM_ATTR_CPESET)) && !cols) ||
      (n && (flags & TVM_ATTR_ARCH) && (!cols->arch_off || !cols->arch_len)) ||
      (n && (flags & TVM_ATTR_CPESET) && !cols->cpe_set))
    return -1;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) return -1;
  const DB& db = e->eng->db();
  const size_t n_sets = b->hb.cpe_words ? b->hb.cpe_bits.size() / b->hb.cpe_words : 0;
  if (flags & TVM_ATTR_CPESET)
    for (size_t i = 0; i < n; i++)
      if (cols->cpe_set[i] >= n_sets) return -1;
  int32_t plat = db.find_plat(bucket);
  const uint32_t pid = plat < 0 ? 0xFFFFFFFFu : uint32_t(plat);
  const int64_t first = int64_t(b->hb.pk.size());
  b->target_begin.push_back(uint32_t(first));
  reserve_more(b->hb, n);
  for (size_t i = 0; i < n; i++) {
    const std::string_view ver(arena + ver_off[i], ver_len[i]);
    uint2 a = make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu);
    if (flags & TVM_ATTR_ARCH) {
      const std::string_view arch(arena + cols->arch_off[i], cols->arch_len[i]);
      a.x = db.arch_id(arch) | (arch == "noarch" ? PA_NOARCH : 0u);  // redhat.go:129 "noarch" matches any
    }
    if (flags & TVM_ATTR_KSPLICE) {
      const size_t dash = ver.find('-');  // release = text after the first '-' (rpm split, rpm.c)
      a.y = db.ksplice_id(extract_ksplice(dash == std::string_view::npos ? std::string_view() : ver.substr(dash + 1)));
    }
    if (flags & TVM_ATTR_CPESET) a.y = cols->cpe_set[i];
    if (flags) b->hb.add(pid, std::string_view(arena + name_off[i], name_len[i]), ver, a);
    else b->hb.add(pid, std::string_view(arena + name_off[i], name_len[i]), ver);
  }
  return first;
}

// Many targets in one call, built on the host threads (pkg/scanner/local/scan.go:170-194 hands
// packages over per target; a fleet batch holds thousands of targets): a pass over the
// packages sums each piece's string bytes (and checks the CPE-set ids), one scan places the
// pieces, then every piece writes its package words, string bytes, group offsets and
// attributes straight into the batch arrays, sized once (BulkVec: no zero fill first).
static int64_t add_targets_bulk(tvm_batch* b, tvm_engine* e, size_t n_targets, const tvm_str* buckets,
                                const uint32_t* tflags, const uint64_t* target_end, const char* arena,
                                const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                                const uint32_t* ver_len, const tvm_attr_cols* cols) {
  const uint32_t known = TVM_ATTR_ARCH | TVM_ATTR_KSPLICE | TVM_ATTR_CPESET;
  if (!b || !e || b->uploaded || b->pinned || (n_targets && (!buckets || !target_end))) return -1;
  const uint64_t n = n_targets ? target_end[n_targets - 1] : 0;
  if (n && (!arena || !name_off || !name_len || !ver_off || !ver_len)) return -1;
  uint32_t any_flags = 0;
  for (size_t t = 0; t < n_targets; t++) {
    if (t && target_end[t] < target_end[t - 1]) return -1;
    const uint32_t f = tflags ? tflags[t] : 0u;
    if ((f & ~known) || ((f & TVM_ATTR_KSPLICE) && (f & TVM_ATTR_CPESET))) return -1;  // one attribute word
    any_flags |= f;
  }
  if (((any_flags & TVM_ATTR_ARCH) && (!cols || !cols->arch_off || !cols->arch_len)) ||
      ((any_flags & TVM_ATTR_CPESET) && (!cols || !cols->cpe_set)))
    return -1;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) return -1;
  const DB& db = e->eng->db();
  HostBatch& hb = b->hb;
  const uint64_t s0 = hb.pk.size(), a0 = hb.arena.size();
  if (s0 + n >= (uint64_t(1) << 32)) return -1;  // package indices are 32-bit
  // per target: its platform (a fleet's targets repeat a few buckets)
  std::vector<uint32_t> pid(n_targets);
  std::string_view last_bucket;
  uint32_t last_pid = 0xFFFFFFFFu;
  for (size_t t = 0; t < n_targets; t++) {
    const std::string_view bk = sv(buckets[t]);
    if (t == 0 || bk != last_bucket) {
      const int32_t plat = db.find_plat(bk);
      last_pid = plat < 0 ? 0xFFFFFFFFu : uint32_t(plat);
      last_bucket = bk;
    }
    pid[t] = last_pid;
  }
  const size_t n_sets = hb.cpe_words ? hb.cpe_bits.size() / hb.cpe_words : 0;
  WorkerPool& wp = WorkerPool::get();
  const size_t K = n ? std::min<size_t>(size_t(wp.size()) * 8, std::max<uint64_t>(1, n / 4096)) : 0;
  auto piece = [&](size_t k) { return std::make_pair(n * k / K, n * (k + 1) / K); };
  auto target_of = [&](uint64_t j) {  // the target holding new package j
    return size_t(std::upper_bound(target_end, target_end + n_targets, j) - target_end);
  };
  std::vector<uint64_t> bytes(K + 1, 0);
  std::atomic<bool> bad{false};
  wp.parallel_for(K, [&](size_t k) {
    const auto [j0, j1] = piece(k);
    uint64_t s = 0;
    size_t t = target_of(j0);
    for (uint64_t j = j0; j < j1; j++) {
      while (target_end[t] <= j) t++;
      s += std::min<uint32_t>(name_len[j], 0xFFFF) + std::min<uint32_t>(ver_len[j], 0xFFFF);
      if (tflags && (tflags[t] & TVM_ATTR_CPESET) && cols->cpe_set[j] >= n_sets) bad.store(true);
    }
    bytes[k + 1] = s;
  });
  if (bad.load()) return -1;
  for (size_t k = 0; k < K; k++) bytes[k + 1] += bytes[k];
  const bool with_attr = any_flags || !hb.attr.empty();
  const uint2 no_attr = make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu);
  try {
    hb.pk.resize(s0 + n);
    hb.arena.resize(a0 + (K ? bytes[K] : 0));
    hb.tile_off.resize((s0 + n + kGroup - 1) / kGroup);
    if (with_attr) {
      if (hb.attr.size() < s0) hb.attr.resize(s0, no_attr);
      hb.attr.resize(s0 + n);
    }
  } catch (const std::bad_alloc&) {
    hb.pk.resize(s0);
    hb.arena.resize(a0);
    hb.tile_off.resize((s0 + kGroup - 1) / kGroup);
    if (with_attr) hb.attr.resize(std::min<size_t>(hb.attr.size(), s0));
    return -1;
  }
  wp.parallel_for(K, [&](size_t k) {
    const auto [j0, j1] = piece(k);
    uint64_t o = a0 + bytes[k];
    size_t t = target_of(j0);
    std::string_view last_arch;
    uint32_t last_arch_id = PA_ARCH_NONE;
    bool have_arch = false;
    uint8_t* ar = hb.arena.data();
    for (uint64_t j = j0; j < j1; j++) {
      while (target_end[t] <= j) t++;
      const uint64_t i = s0 + j;
      const uint32_t nl = std::min<uint32_t>(name_len[j], 0xFFFF), vl = std::min<uint32_t>(ver_len[j], 0xFFFF);
      if (i % kGroup == 0) hb.tile_off[i / kGroup] = o;
      hb.pk[i] = make_uint2(pid[t], nl | (vl << 16));
      std::memcpy(ar + o, arena + name_off[j], nl);
      std::memcpy(ar + o + nl, arena + ver_off[j], vl);
      o += nl + vl;
      if (!with_attr) continue;
      const uint32_t f = tflags ? tflags[t] : 0u;
      uint2 a = no_attr;
      if (f & TVM_ATTR_ARCH) {
        const std::string_view arch(arena + cols->arch_off[j], cols->arch_len[j]);
        if (!have_arch || arch != last_arch) {  // packages of an image share a few arches
          last_arch_id = db.arch_id(arch) | (arch == "noarch" ? PA_NOARCH : 0u);  // redhat.go:129
          last_arch = arch;
          have_arch = true;
        }
        a.x = last_arch_id;
      }
      if (f & TVM_ATTR_KSPLICE) {
        const std::string_view ver(arena + ver_off[j], ver_len[j]);
        const size_t dash = ver.find('-');  // release = text after the first '-' (rpm split, rpm.c)
        a.y = db.ksplice_id(extract_ksplice(dash == std::string_view::npos ? std::string_view() : ver.substr(dash + 1)));
      }
      if (f & TVM_ATTR_CPESET) a.y = cols->cpe_set[j];
      hb.attr[i] = a;
    }
  });
  for (size_t t = 0; t < n_targets; t++) b->target_begin.push_back(uint32_t(s0 + (t ? target_end[t - 1] : 0)));
  return int64_t(s0);
}

int64_t tvm_batch_add_targets(tvm_batch* b, tvm_engine* e, size_t n_targets, const tvm_str* buckets,
                              const uint64_t* target_end, const char* arena, const uint64_t* name_off,
                              const uint32_t* name_len, const uint64_t* ver_off, const uint32_t* ver_len) {
  return add_targets_bulk(b, e, n_targets, buckets, nullptr, target_end, arena, name_off, name_len, ver_off, ver_len,
                          nullptr);
}

int64_t tvm_batch_add_targets_attrs(tvm_batch* b, tvm_engine* e, size_t n_targets, const tvm_str* buckets,
                                    const uint32_t* target_flags, const uint64_t* target_end, const char* arena,
                                    const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                                    const uint32_t* ver_len, const tvm_attr_cols* attrs) {
  return add_targets_bulk(b, e, n_targets, buckets, target_flags, target_end, arena, name_off, name_len, ver_off,
                          ver_len, attrs);
}

int64_t tvm_batch_size(const tvm_batch* b) { return b ? int64_t(b->hb.pk.size()) : 0; }

int tvm_batch_upload(tvm_engine* e, tvm_batch* b, uint64_t cap, char* err, size_t errlen) {
  if (!e || !b) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  std::string msg;
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  if (b->uploaded) {
    Engine::free_batch(b->device, b->dev);
    if (b->external_out) b->m.pkg = b->m.adv = nullptr;
    Engine::free_matches(b->device, b->m);
    b->external_out = false;
    b->uploaded = false;
  }
  b->st_valid = false;
  if (!e->eng->upload(b->hb, b->dev, msg) || !e->eng->alloc_matches(cap, b->dev.n, b->m, msg)) {
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  b->dev.pkg_base = b->pkg_base;
  b->uploaded = true;
  b->filter.reset_packages();
  b->rh.forget_tiles();
  b->device = e->device;
  return TVM_OK;
}

int tvm_batch_set_package_base(tvm_batch* b, uint32_t base) {
  if (!b) return TVM_EINVAL;
  b->pkg_base = base;
  b->dev.pkg_base = base;
  return TVM_OK;
}

int tvm_match_launch(tvm_engine* e, tvm_batch* b, char* err, size_t errlen) {
  if (!e || !b || !b->uploaded) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  std::string msg;
  b->merged = false;
  b->st_valid = false;
  if (!e->eng->launch(b->dev, b->m, e->eng->stream(), msg)) {
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

int tvm_engine_sync(tvm_engine* e, char* err, size_t errlen) {
  if (!e) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);  // a concurrent swap must not free the engine under us
  (void)hipSetDevice(e->device);
  hipError_t st = hipStreamSynchronize(e->eng->stream());
  if (st != hipSuccess) {
    set_err(err, errlen, std::string("hipStreamSynchronize: ") + hipGetErrorString(st));
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

// tvm_match_status with the engine's lock already held (shared) by the caller
static int match_status_locked(tvm_engine* e, tvm_batch* b, uint64_t* n_matches, int64_t* err_pkg, uint64_t* err_bits) {
  if (!e || !b || !b->uploaded) return TVM_EINVAL;
  unsigned long long ctl[8], mctl[8];
  (void)hipSetDevice(e->device);
  // the counters are read on the engine stream, behind the batch's launches (a plain
  // hipMemcpy runs on the null stream, which does not wait for the non-blocking engine stream)
  hipStream_t st = e->eng->stream();
  if (hipMemcpyAsync(ctl, b->m.ctl, sizeof(ctl), hipMemcpyDeviceToHost, st) != hipSuccess) return TVM_EDEVICE;
  if (b->merged && hipMemcpyAsync(mctl, cur(b).ctl, sizeof(mctl), hipMemcpyDeviceToHost, st) != hipSuccess)
    return TVM_EDEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return TVM_EDEVICE;
  b->st_n = b->merged ? mctl[0] : ctl[0];
  b->st_errp = ctl[1] ? int64_t(b->dev.n - ctl[1]) : -1;
  b->st_valid = true;
  if (n_matches) *n_matches = b->merged ? mctl[0] : ctl[0];
  if (err_pkg) *err_pkg = ctl[1] ? int64_t(b->dev.n - ctl[1]) : -1;
  if (err_bits) *err_bits = ctl[3] | (b->merged ? mctl[3] : 0ull);
  return TVM_OK;
}

int tvm_match_status(tvm_engine* e, tvm_batch* b, uint64_t* n_matches, int64_t* err_pkg, uint64_t* err_bits) {
  if (!e || !b || !b->uploaded) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  return match_status_locked(e, b, n_matches, err_pkg, err_bits);
}

int tvm_match_fetch(tvm_engine* e, tvm_batch* b, uint32_t* pairs, uint64_t cap, uint64_t* n_out) {
  uint64_t n = 0;
  int rc = tvm_match_status(e, b, &n, nullptr, nullptr);
  if (rc) return rc;
  if (n_out) *n_out = 0;
  if (n > cur(b).cap) return TVM_EINVAL;  // device buffer overflowed: re-upload with a larger cap
  std::vector<uint2> ordered;
  std::string msg;
  (void)hipSetDevice(e->device);
  if (!Engine::fetch_ordered(cur(b), b->dev.n, n, ordered, e->eng->stream(), msg)) return TVM_EDEVICE;
  n = std::min<uint64_t>(n, cap);
  if (n) memcpy(pairs, ordered.data(), n * sizeof(uint2));
  if (n_out) *n_out = n;
  return TVM_OK;
}

int tvm_match_copy_device(tvm_engine* e, tvm_batch* b, void* dst, uint64_t cap, uint64_t* n_out) {
  uint64_t n = 0;
  int rc = tvm_match_status(e, b, &n, nullptr, nullptr);
  if (rc) return rc;
  if (n_out) *n_out = 0;
  if (b->merged || n > b->m.cap) return TVM_EINVAL;  // raw lists only
  n = std::min<uint64_t>(n, cap);
  (void)hipSetDevice(e->device);
  hipStream_t st = e->eng->stream();
  // {pkg, adv} pairs interleaved from the two ordered arrays: two strided device copies
  if (n && (!dst ||
            hipMemcpy2DAsync(dst, 8, b->m.pkg, 4, 4, n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpy2DAsync(static_cast<char*>(dst) + 4, 8, b->m.adv, 4, 4, n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess))
    return TVM_EDEVICE;
  if (n_out) *n_out = n;
  return TVM_OK;
}

int tvm_match_order_into(tvm_engine* e, tvm_batch* b, void* csr_adv_dev, void* row_end_dev, uint64_t cap,
                         uint64_t* n_out, char* err, size_t errlen) {
  uint64_t n = 0;
  int rc = tvm_match_status(e, b, &n, nullptr, nullptr);
  if (rc) return rc;
  if (n_out) *n_out = n;
  if (b->merged || n > b->m.cap || n > cap || !row_end_dev || (n && !csr_adv_dev)) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  (void)hipSetDevice(e->device);
  hipStream_t st = e->eng->stream();
  const uint32_t nt = b->dev.n_tiles;
  if (nt == 0) return TVM_OK;
  if (b->order_cap < nt + 1) {
    if (b->order_scratch) (void)hipFree(b->order_scratch);
    b->order_scratch = nullptr;
    b->order_cap = 0;
    void* p = nullptr;
    if (hipMalloc(&p, size_t(nt + 1) * 8) != hipSuccess) {
      set_err(err, errlen, "hipMalloc(order scratch) failed");
      return TVM_EDEVICE;
    }
    b->order_scratch = static_cast<unsigned long long*>(p);
    b->order_cap = nt + 1;
  }
  OrderArgs oa;
  oa.dir = b->m.dir;
  oa.pkg = b->m.pkg;
  oa.adv = b->m.adv;
  oa.csr_adv = static_cast<uint32_t*>(csr_adv_dev);
  oa.row_end = static_cast<uint32_t*>(row_end_dev);
  oa.cap = std::min<uint64_t>(cap, b->m.cap);
  oa.ticket = b->order_scratch;
  oa.status = b->order_scratch + 1;
  oa.t0 = 0;
  oa.n = b->dev.n;
  oa.pkg_base = b->dev.pkg_base;
  if (hipMemsetAsync(b->order_scratch, 0, size_t(nt + 1) * 8, st) != hipSuccess) return TVM_EDEVICE;
  launch_order(nt, st, oa);
  const hipError_t le = hipGetLastError();
  const hipError_t se = le == hipSuccess ? hipStreamSynchronize(st) : le;
  if (se != hipSuccess) {
    set_err(err, errlen, std::string("order kernel: ") + hipGetErrorString(se));
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

int tvm_match_time(tvm_engine* e, tvm_batch* b, int steps, double* ms, char* err, size_t errlen) {
  if (!e || !b || !b->uploaded || steps <= 0 || !ms) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  (void)hipSetDevice(e->device);
  hipEvent_t t0 = nullptr, t1 = nullptr;
  hipStream_t st = e->eng->stream();
  std::string msg;
  int rc = TVM_OK;
  if (hipEventCreate(&t0) != hipSuccess || hipEventCreate(&t1) != hipSuccess || hipEventRecord(t0, st) != hipSuccess) {
    msg = "hipEvent setup failed";
    rc = TVM_EDEVICE;
  }
  b->merged = false;
  b->st_valid = false;
  for (int i = 0; rc == TVM_OK && i < steps; i++)
    if (!e->eng->launch(b->dev, b->m, st, msg)) rc = TVM_EDEVICE;
  float f = 0;
  if (rc == TVM_OK && (hipEventRecord(t1, st) != hipSuccess || hipEventSynchronize(t1) != hipSuccess ||
                       hipEventElapsedTime(&f, t0, t1) != hipSuccess)) {
    msg = "hipEvent timing failed";
    rc = TVM_EDEVICE;
  }
  if (t0) (void)hipEventDestroy(t0);
  if (t1) (void)hipEventDestroy(t1);
  if (rc != TVM_OK) {
    set_err(err, errlen, msg);
    return rc;
  }
  *ms = f;
  return TVM_OK;
}

uint64_t tvm_match_algorithmic_bytes(tvm_engine* e, tvm_batch* b) {
  // DESIGN.md "Roofline": per package 8 B package word + name + version bytes, per probed
  // package 8 B slot hash + 16 B slot value + name verify, per (package, row) 16 B row +
  // bound-key bytes, per match 8 B output.  Computed exactly from the batch + tables.
  if (!e || !b) return 0;
  const DB& db = e->eng->db();
  uint64_t bytes = 0, off = 0;
  for (const uint2& d : b->hb.pk) {
    const uint32_t nlen = d.y & 0xFFFF, vlen = d.y >> 16;
    const std::string_view name(reinterpret_cast<const char*>(b->hb.arena.data()) + off, nlen);
    off += nlen + vlen;
    bytes += 8 + nlen + vlen;  // package word, strings
    if (d.x >= db.plats.size()) continue;
    bytes += 24;
    int32_t k = db.find_key(d.x, name);
    if (k < 0) continue;
    bytes += nlen;
    const std::string ks = db.keys[size_t(k)].name;
    uint64_t h = pkg_key_hash(d.x, reinterpret_cast<const uint8_t*>(ks.data()), uint32_t(ks.size()));
    for (uint64_t i = h & db.slot_mask; db.slot_hash[i]; i = (i + 1) & db.slot_mask) {
      if (db.slot_key[i] != uint32_t(k)) continue;
      const SlotVal& v = db.slot_val[i];
      uint32_t cls = 0;  // a split key: the rows of the version's class (common.h SLOT_CLS_SPLIT)
      if (v.name_len & SLOT_CLS_SPLIT) {
        struct Sink {
          void put(uint8_t) {}
        } sk;
        const char* ver = name.data() + nlen;
        if (!encode_version_cls(db.plat_info[d.x].cmp, reinterpret_cast<const uint8_t*>(ver), vlen, sk, cls)) cls = 0;
      }
      const uint2 rr = slot_rows(v.name_len, v.row_begin, v.row_count, cls);
      for (uint32_t r = 0; r < rr.y; r++) {
        const Row& row = db.rows[rr.x + r];
        bytes += sizeof(Row);  // 16 B header + 16 B inline hi-key prefix
        if (!(row.hi_len & KEY_INF) && (row.hi_len & KEY_LEN_MASK) > 16) bytes += (row.hi_len & KEY_LEN_MASK) - 16;
        if (!(row.lo_len & KEY_INF)) bytes += row.lo_len & KEY_LEN_MASK;
      }
      break;
    }
  }
  uint64_t m = 0;
  if (b->uploaded) tvm_match_status(e, b, &m, nullptr, nullptr);
  return bytes + 8 * m;
}

int tvm_version_key(int grammar, const char* s, size_t n, uint8_t* out, size_t cap) {
  struct Sink {
    uint8_t* o;
    size_t cap, n = 0;
    void put(uint8_t b) {
      if (n < cap) o[n] = b;
      n++;
    }
  } sink{out, cap};
  if (grammar <= 0 || grammar > 255 || !s) return -1;
  uint32_t cls = 0;
  if (!encode_version_cls(uint8_t(grammar), reinterpret_cast<const uint8_t*>(s), uint32_t(n), sink, cls)) return -1;
  return int(sink.n);
}

int tvm_version_class(int grammar, const char* s, size_t n) {
  struct Sink {
    void put(uint8_t) {}
  } sink;
  uint32_t cls = 0;
  if (grammar <= 0 || grammar > 255 || !s) return -1;
  if (!encode_version_cls(uint8_t(grammar), reinterpret_cast<const uint8_t*>(s), uint32_t(n), sink, cls)) return -1;
  return int(cls);
}

int tvm_deb_fast_key_host(const char* s, size_t n, uint32_t shift, uint8_t* out, size_t cap) {
  if (!s || n > 4096 || shift > 3) return -3;
  uint8_t tab[128];
  for (uint32_t c = 0; c < 128; c++) tab[c] = deb_fast_code(c);
  std::vector<uint32_t> buf((shift + n) / 4 + 4, 0xA5A5A5A5u);  // padded like the LDS stage window
  uint8_t* b = reinterpret_cast<uint8_t*>(buf.data()) + shift;
  std::memcpy(b, s, n);
  uint8_t kb[kFastKeyStride];
  std::memset(kb, 0xEE, sizeof kb);
  uint32_t len = 0;
  const uint32_t st = deb_fast_key(b, uint32_t(n), kb, tab, len);
  if (st == FAST_INVALID) return -1;
  if (st == FAST_FALLBACK) return -2;
  for (uint32_t i = 0; i < len && i < cap; i++) out[i] = kb[i];
  return int(len);
}

int tvm_lib_is_vulnerable_host(int grammar, const char* ver, size_t ver_len, const char* advisory_json,
                               size_t json_len) {
  Advisory a;
  std::string e;
  if (!ver || !advisory_json || !decode_advisory(std::string_view(advisory_json, json_len), a, e)) return -1;
  // Maven: the rows DB::compile_rows builds - intervals over the numeric projection for an
  // advisory with numeric bounds, else the pairwise program; TVM_ISVULN_PAIRWISE: always the
  // pairwise program (ComparableVersion itself, the device's rows aside)
  const bool pairwise = (grammar & TVM_ISVULN_PAIRWISE) != 0;
  grammar &= ~TVM_ISVULN_PAIRWISE;
  if (grammar == CMP_MAVEN && (pairwise || !mvn_hybrid(a.vulnerable, a.patched, a.unaffected)))
    return mvn_is_vulnerable(a.vulnerable, a.patched, a.unaffected, std::string(ver, ver_len));
  const LibRows r = lib_compile_advisory(uint8_t(grammar), a.vulnerable, a.patched, a.unaffected);
  return lib_rows_contain(uint8_t(grammar), r, std::string(ver, ver_len)) ? 1 : 0;
}

int tvm_library_detect(tvm_engine* e, const char* lib_type, const tvm_package* pkgs, size_t n, tvm_result* out,
                       char* err, size_t errlen) {
  if (!e || !lib_type || !out || (n && !pkgs)) return TVM_EINVAL;
  memset(out, 0, sizeof(*out));
  std::shared_lock<std::shared_mutex> lk(e->mu);
  std::vector<Pkg> p = to_pkgs(pkgs, n);
  std::vector<Vuln> vulns;
  std::string msg;
  const DetectStatus st = library_detect(*e->eng, lib_type, p, vulns, msg);
  if (st == DETECT_UNSUPPORTED_OS) return TVM_EUNSUPPORTED_TYPE;
  if (st != DETECT_OK) {
    set_err(err, errlen, msg);
    return TVM_EDETECT;
  }
  export_result(e->eng->db(), std::move(vulns), false, out);
  return TVM_OK;
}

int tvm_library_detect_vulnerabilities(tvm_engine* e, const char* lib_type, tvm_str pkg_id, tvm_str pkg_name,
                                       tvm_str pkg_ver, tvm_result* out, char* err, size_t errlen) {
  if (!e || !lib_type || !out) return TVM_EINVAL;
  memset(out, 0, sizeof(*out));
  std::shared_lock<std::shared_mutex> lk(e->mu);
  std::vector<Pkg> p(1);
  p[0].id = sv(pkg_id);
  p[0].name = sv(pkg_name);
  p[0].version = sv(pkg_ver);
  std::vector<Vuln> vulns;
  std::string msg;
  const DetectStatus st = library_detect_vulnerabilities(*e->eng, lib_type, p, vulns, msg);
  if (st == DETECT_UNSUPPORTED_OS) return TVM_EUNSUPPORTED_TYPE;
  if (st != DETECT_OK) {
    set_err(err, errlen, msg);
    return TVM_EDETECT;
  }
  export_result(e->eng->db(), std::move(vulns), false, out);
  return TVM_OK;
}

const char* tvm_library_type(const char* lib_type) { return lib_type ? library_ecosystem(lib_type) : nullptr; }

}  // extern "C"

// ---- FillInfo (vulnerability.go:60-157) ----------------------------------------------

namespace {

struct FillPriv {
  std::vector<tvm_fill_out> items;
  std::deque<std::string> strs;  // owned strings; items point into them (deque: stable addresses)
};

}  // namespace

int tvm_fill_info(tvm_engine* e, const tvm_fill_in* in, size_t n, tvm_fill_result* out, char* err, size_t errlen) {
  if (!e || !out || (n && !in)) return TVM_EINVAL;
  *out = tvm_fill_result{nullptr, 0, nullptr};
  std::shared_lock<std::shared_mutex> lk(e->mu);
  const VulnTable& vt = e->fill->table();
  std::vector<uint4> items(n);
  std::vector<uint8_t> arena;
  for (size_t i = 0; i < n; i++) {
    const tvm_fill_in& x = in[i];
    const size_t len = std::min<size_t>(x.vulnerability_id.n, 0xFFFF);  // longer IDs: no record has one
    const uint32_t src = vt.source_id(std::string_view(x.data_source_id.p ? x.data_source_id.p : "", x.data_source_id.n));
    uint4 it;
    it.x = uint32_t(arena.size());
    it.y = uint32_t(len) | (src << 16);
    it.z = uint32_t(x.status & 0xFF) | (x.has_fixed_version ? FI_FIXED : 0u) | (x.severity_source.n ? FI_SEV_SRC : 0u);
    it.w = FILL_NOT_FOUND;
    if (len) arena.insert(arena.end(), x.vulnerability_id.p, x.vulnerability_id.p + len);
    items[i] = it;
  }
  std::vector<uint4> dec;
  std::string msg;
  if (!e->fill->run_host(items, arena, dec, msg)) {
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  auto* priv = new FillPriv();
  priv->items.resize(n);
  auto keep = [&](std::string s) -> const char* {
    priv->strs.push_back(std::move(s));
    return priv->strs.back().c_str();
  };
  for (size_t i = 0; i < n; i++) {
    const tvm_fill_in& x = in[i];
    const uint4 d = dec[i];
    tvm_fill_out& o = priv->items[i];
    o.status = int32_t(d.y);
    if (!x.has_fixed_version && x.status != 0 && (x.status & ~0xFF)) o.status = x.status;  // beyond the 8-bit item field
    o.severity = o.severity_source = o.primary_url = "";
    o.vulnerability_json = nullptr;
    o.found = d.x != FILL_NOT_FOUND && x.vulnerability_id.n <= 0xFFFF;
    if (!o.found) continue;
    const uint32_t code = d.z & 0xFFFFu, ssrc = d.z >> 16;
    std::string_view extra_src;
    int64_t extra_val = 0;
    if (code == SEV_KEEP) {  // the detector's package-specific severity (vulnerability.go:90-101)
      const std::string_view sev(x.severity.p ? x.severity.p : "", x.severity.n);
      extra_src = std::string_view(x.severity_source.p, x.severity_source.n);
      extra_val = fill_new_severity(sev);
      o.severity = keep(std::string(sev));
      o.severity_source = keep(std::string(extra_src));
    } else {
      o.severity = vt.severity_string(d.x, code).c_str();
      o.severity_source = ssrc == SRC_NONE ? "" : vt.source_name(ssrc).c_str();
    }
    o.primary_url = keep(vt.primary_url(d.x, d.w));
    o.vulnerability_json = keep(vt.vulnerability_json(d.x, o.severity, extra_src, extra_val));
  }
  out->items = priv->items.data();
  out->n = n;
  out->priv = priv;
  return TVM_OK;
}

void tvm_fill_result_free(tvm_fill_result* r) {
  if (!r) return;
  delete static_cast<FillPriv*>(r->priv);
  *r = tvm_fill_result{nullptr, 0, nullptr};
}

int tvm_match_fill(tvm_engine* e, tvm_batch* b, char* err, size_t errlen) {
  if (!e || !b || !b->uploaded) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  (void)hipSetDevice(e->device);
  const DevMatches& m = cur(b);
  if (b->fill_cap < m.cap) {
    if (b->fill_out) (void)hipFree(b->fill_out);
    b->fill_out = nullptr;
    b->fill_cap = 0;
    // decisions, then the filter's hand-off words (uint2) in the same allocation
    if (hipMalloc(&b->fill_out, std::max<uint64_t>(m.cap, 1) * (sizeof(uint4) + sizeof(uint2))) != hipSuccess) {
      set_err(err, errlen, "hipMalloc(fill decisions) failed");
      return TVM_EDEVICE;
    }
    b->fill_cap = m.cap;
  }
  std::string msg;
  if (!e->fill->launch_pairs(m.adv, cur_base(b), m.ctl, m.cap, b->fill_out, b->fill_side(), e->eng->stream(), msg)) {
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

int tvm_match_fill_fetch(tvm_engine* e, tvm_batch* b, uint32_t* out4, uint64_t cap, uint64_t* n_out) {
  if (!e || !b || !b->uploaded) return TVM_EINVAL;
  (void)hipSetDevice(e->device);
  if (hipStreamSynchronize(e->eng->stream()) != hipSuccess) return TVM_EDEVICE;
  uint64_t n = 0;
  int rc = tvm_match_status(e, b, &n, nullptr, nullptr);
  if (rc) return rc;
  if (n_out) *n_out = 0;
  if (n > cur(b).cap || n > b->fill_cap) return TVM_EINVAL;
  const uint32_t n_tiles = (b->dev.n + kTile - 1) / kTile;
  std::vector<TileDir> dir(n_tiles);
  std::vector<uint4> raw(n);
  if ((n_tiles && hipMemcpy(dir.data(), cur(b).dir, n_tiles * sizeof(TileDir), hipMemcpyDeviceToHost) != hipSuccess) ||
      (n && hipMemcpy(raw.data(), b->fill_out, n * sizeof(uint4), hipMemcpyDeviceToHost) != hipSuccess))
    return TVM_EDEVICE;
  uint64_t k = 0;
  for (const TileDir& d : dir)  // tile order = tvm_match_fetch's (package, advisory) order
    for (uint64_t i = d.base; i < d.base + d.count && k < cap; i++, k++)
      memcpy(out4 + 4 * k, &raw[i], sizeof(uint4));
  if (n_out) *n_out = k;
  return TVM_OK;
}

int tvm_match_fill_time(tvm_engine* e, tvm_batch* b, int steps, double* ms, char* err, size_t errlen) {
  if (!e || !b || !b->uploaded || steps <= 0 || !ms) return TVM_EINVAL;
  int rc = tvm_match_fill(e, b, err, errlen);  // sizes the decision buffer
  if (rc) return rc;
  (void)hipSetDevice(e->device);
  hipStream_t st = e->eng->stream();
  hipEvent_t t0 = nullptr, t1 = nullptr;
  std::string msg;
  float f = 0;
  bool ok = hipEventCreate(&t0) == hipSuccess && hipEventCreate(&t1) == hipSuccess && hipEventRecord(t0, st) == hipSuccess;
  const DevMatches& m = cur(b);
  for (int i = 0; ok && i < steps; i++)
    ok = e->fill->launch_pairs(m.adv, cur_base(b), m.ctl, m.cap, b->fill_out, b->fill_side(), st, msg);
  ok = ok && hipEventRecord(t1, st) == hipSuccess && hipEventSynchronize(t1) == hipSuccess &&
       hipEventElapsedTime(&f, t0, t1) == hipSuccess;
  if (t0) (void)hipEventDestroy(t0);
  if (t1) (void)hipEventDestroy(t1);
  if (!ok) {
    set_err(err, errlen, msg.empty() ? "hipEvent timing failed" : msg);
    return TVM_EDEVICE;
  }
  *ms = f;
  return TVM_OK;
}

uint64_t tvm_match_fill_algorithmic_bytes(tvm_engine* e, tvm_batch* b) {
  uint64_t n = 0;
  if (!e || !b || tvm_match_status(e, b, &n, nullptr, nullptr) || n > cur(b).cap) return 0;
  std::vector<uint32_t> adv(n), base;
  (void)hipSetDevice(e->device);
  if (n && hipMemcpy(adv.data(), cur(b).adv, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  if (cur_base(b)) {
    base.resize(n);
    if (n && hipMemcpy(base.data(), cur_base(b), n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  }
  return e->fill->pair_bytes(adv, base);
}

const char* tvm_fill_source_name(tvm_engine* e, uint32_t id) {
  if (!e || id == SRC_NONE) return "";
  const VulnTable& vt = e->fill->table();
  return id < 0x7FFF ? vt.source_name(id).c_str() : "";
}

// ---- result.Filter over a batch (filter.go:60-139, filter.hip) --------------------------

int tvm_batch_set_report(tvm_batch* b, uint64_t first, uint64_t n, const tvm_str* names, const tvm_str* versions,
                         const tvm_str* paths) {
  const uint64_t size = b ? b->hb.pk.size() : 0;
  if (!b || first > size || n > size - first) return TVM_EINVAL;
  const tvm_str* cols[3] = {names, versions, paths};
  for (int f = 0; f < 3; f++) {
    if (!cols[f]) continue;
    if (b->rep[f].size() < first + n) {
      b->rep[f].resize(first + n);
      b->rep_has[f].resize(first + n, 0);
    }
    for (uint64_t i = 0; i < n; i++) {
      b->rep[f][first + i] = std::string(sv(cols[f][i]));
      b->rep_has[f][first + i] = 1;
    }
  }
  b->filter.reset_packages();
  return TVM_OK;
}

namespace {

// The filter's package layout (FilterPackages): within every result (one add call) the
// packages sorted by (PkgName, InstalledVersion, PkgPath, index) - types.BySeverity's
// package keys and filterVulnerabilities' dedup key (filter.go:124); PkgName /
// InstalledVersion default to the batch (name, version), PkgPath to "".
//   The reference's dedup key is the string "vulnID/pkgName/installed/pkgPath"; comparing
// the fields instead differs only when a field itself holds a '/' that shifts the split
// (e.g. an InstalledVersion with a '/'), which no package grammar produces.
void package_layout(const tvm_batch* b, FilterPackages& fp) {
  const size_t n = b->hb.pk.size();
  std::vector<uint64_t> off;
  b->hb.name_offsets(off);
  const char* arena = reinterpret_cast<const char*>(b->hb.arena.data());
  auto field = [&](int f, uint32_t i) -> std::string_view {
    if (i < b->rep_has[f].size() && b->rep_has[f][i]) return b->rep[f][i];
    if (f == 0) return std::string_view(arena + off[i], b->hb.pk[i].y & 0xFFFFu);
    if (f == 1) return std::string_view(arena + off[i] + (b->hb.pk[i].y & 0xFFFFu), b->hb.pk[i].y >> 16);
    return std::string_view();
  };
  fp.perm.resize(n);
  fp.grp_b.assign(n, 0);
  fp.grp_e.assign(n, 0);
  fp.dkey.assign(n, 0);
  fp.prank.assign(n, 0);
  fp.dup.assign(n, 0);
  std::vector<uint32_t> bounds(b->target_begin);
  bounds.push_back(uint32_t(n));
  uint32_t next_d = 0;
  for (size_t t = 0; t + 1 < bounds.size(); t++) {
    uint32_t* idx = fp.perm.data() + bounds[t];
    const uint32_t len = bounds[t + 1] - bounds[t];
    for (uint32_t k = 0; k < len; k++) idx[k] = bounds[t] + k;
    std::sort(idx, idx + len, [&](uint32_t x, uint32_t y) {
      for (int f = 0; f < 3; f++) {
        const int c = field(f, x).compare(field(f, y));
        if (c) return c < 0;
      }
      return x < y;
    });
    for (uint32_t k = 0; k < len;) {  // groups of equal (PkgName, InstalledVersion)
      uint32_t e = k + 1;
      while (e < len && field(0, idx[e]) == field(0, idx[k]) && field(1, idx[e]) == field(1, idx[k])) e++;
      uint32_t pr = 0;
      for (uint32_t m = k; m < e; m++) {
        const uint32_t p = idx[m];
        const bool same_path = m > k && field(2, p) == field(2, idx[m - 1]);
        if (m > k && !same_path) pr++;
        if (m > k && !same_path) next_d++;
        fp.grp_b[p] = bounds[t] + k;
        fp.grp_e[p] = bounds[t] + e;
        fp.prank[p] = pr;
        fp.dkey[p] = next_d;
        if (same_path) fp.dup[p] = fp.dup[idx[m - 1]] = 1;
      }
      next_d++;
      k = e;
    }
  }
}

}  // namespace

int tvm_match_filter(tvm_engine* e, tvm_batch* b, const tvm_filter_opts* o, uint64_t* n_kept, uint64_t* n_ignored,
                     char* err, size_t errlen) {
  const auto t_call = std::chrono::steady_clock::now();
  if (!e || !b || !o || !b->uploaded || (o->n_vex && (!o->vex_pkgs || !o->vex_id_index)) ||
      (o->n_vex_ids && !o->vex_ids && !o->vex_id_ranks))
    return TVM_EINVAL;
  const tvm_ignore_rules* ig = o->ignore;
  if (ig && ((ig->n_ids && !ig->ids && !ig->id_ranks) || (ig->n_all && (!ig->all_id || !ig->all_prec)) ||
             (ig->n_pkg && (!ig->pkg_pkg || !ig->pkg_id || !ig->pkg_prec)) ||
             (ig->n_cls && (!ig->pkg_class || !ig->cls_class || !ig->cls_id || !ig->cls_prec))))
    return TVM_EINVAL;
  if (o->severity_mask >> 5) {  // SeverityNames has 5 entries (UNKNOWN..CRITICAL)
    set_err(err, errlen, "tvm_match_filter: severity_mask has bits above CRITICAL (4)");
    return TVM_EINVAL;
  }
  if (b->pkg_base) {
    set_err(err, errlen, "tvm_match_filter: the batch is a shard (package base set); filter whole results");
    return TVM_EINVAL;
  }
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  (void)hipSetDevice(e->device);
  hipStream_t st = e->eng->stream();
  uint64_t n = b->st_n;
  int64_t errp = b->st_errp;
  // the list's length: read back behind the batch's launches on st, once per launch / merge
  int rc = b->st_valid ? TVM_OK : match_status_locked(e, b, &n, &errp, nullptr);
  if (rc) return rc;
  if (n > cur(b).cap || n > b->fill_cap) {
    set_err(err, errlen, "tvm_match_filter: run tvm_match_launch + tvm_match_fill with a large enough match buffer first");
    return TVM_EINVAL;
  }
  std::string msg;
  if (!b->filter.has_packages()) {
    FilterPackages fp;
    package_layout(b, fp);
    if (!b->filter.set_packages(fp, msg)) {
      set_err(err, errlen, msg);
      return TVM_EDEVICE;
    }
  }
  const VulnTable& vt = e->fill->table();
  const uint64_t n_pkgs = uint64_t(tvm_batch_size(b));
  FilterRules rules;
  // each distinct ID ranked once (or by the caller, tvm_vuln_rank_many); IDs unknown to the
  // DB cannot name a detected vulnerability, so their rules drop out on the device
  auto ranks = [&](std::vector<uint32_t>& r, const tvm_str* ids, size_t k, const uint32_t* given) {
    r.resize(k);
    for (size_t i = 0; i < k; i++) r[i] = given ? given[i] : vt.vuln_rank(sv(ids[i]));
  };
  // bounds of the caller's arrays: subject < limit, ID index < ID count (vectorisable scans)
  auto below = [](const uint32_t* v, size_t k, uint64_t limit) {
    uint32_t mx = 0;
    for (size_t i = 0; i < k; i++) mx = std::max(mx, v[i]);
    return k == 0 || mx < limit;
  };
  bool good = true;
  auto list = [&](uint64_t tag, const uint32_t* subject, uint64_t subject_limit, const uint32_t* id, const uint32_t* prec,
                  size_t k, int table) {
    if (!k) return;
    if (tag != RULE_VEX)  // VEX statements (the long lists) are checked by the kernel that applies them
      good &= below(id, k, rules.rank[table].size()) && (!subject || below(subject, k, subject_limit));
    RuleList& l = rules.lists[rules.n_lists++];
    l.tag = tag;
    l.subject = subject;
    l.id = id;
    l.prec = prec;
    l.n = k;
    l.table = table;
    rules.kinds |= 1u << tag;
  };
  const uint64_t lim = std::min<uint64_t>(n_pkgs, 1ull << 30);
  if (ig) {
    ranks(rules.rank[0], ig->ids, ig->n_ids, ig->id_ranks);
    list(RULE_ALL, nullptr, 0, ig->all_id, ig->all_prec, ig->n_all, 0);
    list(RULE_PKG, ig->pkg_pkg, lim, ig->pkg_id, ig->pkg_prec, ig->n_pkg, 0);
    list(RULE_CLS, ig->cls_class, 1ull << 30, ig->cls_id, ig->cls_prec, ig->n_cls, 0);
    if (ig->n_cls) {
      rules.pkg_class = ig->pkg_class;
      good &= below(ig->pkg_class, n_pkgs, 1ull << 30);
    }
  }
  if (o->n_vex) {
    ranks(rules.rank[1], o->vex_ids, o->n_vex_ids, o->vex_id_ranks);
    list(RULE_VEX, o->vex_pkgs, lim, o->vex_id_index, nullptr, o->n_vex, 1);
  }
  if (!good) {
    set_err(err, errlen, "tvm_match_filter: rule / VEX package, class or ID index out of range");
    return TVM_EINVAL;
  }
  if (std::getenv("TVM_FILTER_TRACE"))
    std::fprintf(stderr, "filter C-ABI prologue %.1f us\n",
                 std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_call).count());
  if (!b->filter.run(e->fill->dev(), cur(b).pkg, cur(b).adv, b->fill_side(), n, rules, vt.n_vuln_ranks(), o->severity_mask,
                     o->ignore_status_mask, st, msg)) {
    set_err(err, errlen, msg);
    return msg.find("out of range") != std::string::npos ? TVM_EINVAL : TVM_EDEVICE;
  }
  if (n_kept) *n_kept = b->filter.survivors();
  if (n_ignored) *n_ignored = b->filter.ignored();
  return TVM_OK;
}

int tvm_vuln_rank_many(tvm_engine* e, const tvm_str* ids, size_t n, uint32_t* ranks) {
  if (!e || (n && (!ids || !ranks))) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  const VulnTable& vt = e->fill->table();
  for (size_t i = 0; i < n; i++) ranks[i] = vt.vuln_rank(sv(ids[i]));
  return TVM_OK;
}

int tvm_match_filter_fetch(tvm_engine* e, tvm_batch* b, uint32_t* pairs, uint64_t cap, uint64_t* n_out) {
  if (!e || !b || (cap && !pairs)) return TVM_EINVAL;
  (void)hipSetDevice(e->device);
  std::vector<uint2> out;
  std::string msg;
  if (!b->filter.fetch(out, e->eng->stream(), msg)) return TVM_EDEVICE;
  const uint64_t k = std::min<uint64_t>(cap, out.size());
  if (k) memcpy(pairs, out.data(), k * sizeof(uint2));
  if (n_out) *n_out = k;
  return TVM_OK;
}

int tvm_match_filter_ignored(tvm_engine* e, tvm_batch* b, uint32_t* triples, uint64_t cap, uint64_t* n_out) {
  if (!e || !b || (cap && !triples)) return TVM_EINVAL;
  (void)hipSetDevice(e->device);
  std::vector<uint32_t> out;
  std::string msg;
  if (!b->filter.fetch_ignored(out, e->eng->stream(), msg)) return TVM_EDEVICE;
  const uint64_t k = std::min<uint64_t>(cap, out.size() / 3);
  for (uint64_t i = 0; i < k; i++) {
    triples[3 * i] = out[3 * i];
    triples[3 * i + 1] = out[3 * i + 1];
    triples[3 * i + 2] = out[3 * i + 2] & 0x7FFFFFFFu;  // the finding index (precedence without the pass)
  }
  if (n_out) *n_out = k;
  return TVM_OK;
}

int tvm_match_filter_time(tvm_engine* e, tvm_batch* b, const tvm_filter_opts* o, int steps, double* ms, char* err,
                          size_t errlen) {
  if (!ms || steps <= 0) return TVM_EINVAL;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < steps; i++) {
    const int rc = tvm_match_filter(e, b, o, nullptr, nullptr, err, errlen);
    if (rc) return rc;
  }
  *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return TVM_OK;
}

// ---- end-to-end pipelined pass (pipeline.hip) -------------------------------------------

namespace {
bool batch_has_redhat(const tvm_batch* b, const DB& db);
}  // namespace

int tvm_pipeline_prepare(tvm_engine* e, tvm_batch* b, uint64_t match_cap, uint32_t chunk_packages, uint32_t flags,
                         char* err, size_t errlen) {
  if (!e || !b || chunk_packages == 0 ||
      (flags & ~uint32_t(TVM_PIPE_RAW | TVM_PIPE_ADV32)))
    return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  b->pipe.reset(new Pipeline());
  b->pipe_total = 0;  // no valid pass of the new pipeline yet
  b->pipe_ok = false;
  b->pipe_rh.forget_tiles();
  b->pipe_wide_for = ~0ull;
  std::string msg;
  const bool packed = !(flags & TVM_PIPE_ADV32) && e->db->db.advs.size() < (1ull << 24);
  if (!b->pipe->prepare(*e->eng, b->hb, match_cap, chunk_packages, !(flags & TVM_PIPE_RAW), packed, msg)) {
    b->pipe.reset();
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  b->pinned = true;  // the pipeline was sized for exactly these packages: no more adds
  (void)batch_has_redhat(b, e->eng->db());  // once per batch, here: tvm_pipeline_vulns reads the answer
  return TVM_OK;
}

int tvm_pipeline_run(tvm_engine* e, tvm_batch* b, uint64_t* n_matches, int64_t* err_pkg, double* ms, char* err,
                     size_t errlen) {
  if (!e || !b || !b->pipe) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  std::string msg;
  uint64_t total = 0, bits = 0;
  int64_t ep = -1;
  const auto t0 = std::chrono::steady_clock::now();
  b->pipe_total = 0;  // a failed pass leaves no result behind
  b->pipe_ok = false;
  b->pipe_wide_for = ~0ull;
  const bool ok = b->pipe->run(*e->eng, b->hb, total, ep, bits, msg);
  const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (!ok) {
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  if (bits) {
    set_err(err, errlen, "match kernel internal error bits " + std::to_string(bits));
    return TVM_EDEVICE;
  }
  b->pipe_total = total;
  b->pipe_runs++;
  if (n_matches) *n_matches = total;
  if (err_pkg) *err_pkg = ep;
  if (ms) *ms = dt;
  if (total > b->pipe->cap()) {
    set_err(err, errlen, "tvm_pipeline_run: match buffer too small (prepare with match_cap >= n_matches)");
    return TVM_EINVAL;
  }
  b->pipe_ok = true;
  b->pipe_errp = ep;
  return TVM_OK;
}

int tvm_pipeline_result(tvm_batch* b, const uint32_t** adv, const uint32_t** row_end, uint64_t* n_matches) {
  if (!b || !b->pipe || b->pipe_total > b->pipe->cap()) return TVM_EINVAL;
  if (adv && b->pipe->packed()) {  // widen the 3-byte indices once per pass (host side, after the pass)
    if (b->pipe_wide_for != b->pipe_runs) {
      const uint8_t* p = reinterpret_cast<const uint8_t*>(b->pipe->adv());
      b->pipe_wide.resize(b->pipe_total);
      uint32_t* w = b->pipe_wide.data();
      range_for(b->pipe_total, size_t(1) << 18, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; i++) w[i] = uint32_t(p[3 * i]) | uint32_t(p[3 * i + 1]) << 8 | uint32_t(p[3 * i + 2]) << 16;
      });
      b->pipe_wide_for = b->pipe_runs;
    }
    *adv = b->pipe_wide.data();
  } else if (adv) {
    *adv = b->pipe->adv();
  }
  if (row_end) *row_end = b->pipe->row_end();
  if (n_matches) *n_matches = b->pipe_total;
  return TVM_OK;
}

int tvm_pipeline_result_raw(tvm_batch* b, const void** adv, uint32_t* width, const uint32_t** row_end,
                            uint64_t* n_matches) {
  if (!b || !b->pipe || b->pipe_total > b->pipe->cap()) return TVM_EINVAL;
  if (adv) *adv = b->pipe->adv();
  if (width) *width = b->pipe->packed() ? 3 : 4;
  if (row_end) *row_end = b->pipe->row_end();
  if (n_matches) *n_matches = b->pipe_total;
  return TVM_OK;
}

int tvm_wire_encode(size_t n, const uint32_t* plat, const char* arena, const uint64_t* name_off, const uint32_t* name_len,
                    const uint64_t* ver_off, const uint32_t* ver_len, uint32_t chunk_packages, int threads, void* out,
                    uint64_t cap, uint64_t* bytes,
                    uint64_t* chunks, uint64_t chunks_cap, uint64_t* n_chunks, uint32_t* plats, uint32_t plats_cap,
                    uint32_t* n_plats) {
  if (!bytes || !n_chunks || !n_plats || chunk_packages == 0 || threads < 1 ||
      (n && (!plat || !arena || !name_off || !name_len || !ver_off || !ver_len)))
    return TVM_EINVAL;
  HostBatch hb;
  for (size_t i = 0; i < n; i++)
    hb.add(plat[i], std::string_view(arena + name_off[i], name_len[i]), std::string_view(arena + ver_off[i], ver_len[i]));
  const uint32_t n_tiles = hb.n_tiles(), chunk_tiles = (chunk_packages + kTile - 1) / kTile;
  std::vector<uint32_t> bounds;
  for (uint32_t t = 0; t < n_tiles; t += chunk_tiles) bounds.push_back(t);
  bounds.push_back(n_tiles);
  if (n_tiles == 0) bounds = {0, 0};
  std::vector<uint64_t> toff(hb.tile_off.begin(), hb.tile_off.end());
  toff.resize(size_t(n_tiles) * kGroupsPerTile + 1, hb.arena.size());
  WireEncoder enc;
  std::string msg;
  if (!enc.plan(hb, toff, bounds, threads, msg)) {
    *bytes = 0;
    *n_chunks = 0;
    *n_plats = 0;
    return msg.empty() ? TVM_OK : TVM_EINVAL;  // no transport form: zero bytes
  }
  *bytes = enc.bytes();
  *n_chunks = enc.chunks().size();
  *n_plats = uint32_t(enc.platforms().size());
  if (!out) return TVM_OK;
  if (cap < enc.bytes() || chunks_cap < enc.chunks().size() || plats_cap < enc.platforms().size() || !chunks || !plats)
    return TVM_EINVAL;
  enc.emit(static_cast<uint8_t*>(out));
  for (size_t c = 0; c < enc.chunks().size(); c++) {
    const WireChunk& w = enc.chunks()[c];
    const uint64_t v[10] = {w.off, w.bytes, w.o_nref, w.o_vref, w.o_lens, w.o_plat, w.o_toff, w.o_attr, w.m, w.groups};
    std::memcpy(chunks + 10 * c, v, sizeof(v));
  }
  std::memcpy(plats, enc.platforms().data(), enc.platforms().size() * 4);
  return TVM_OK;
}

int tvm_pipeline_times(tvm_batch* b, uint64_t* encode_us, uint64_t* prepare_us) {
  if (!b || !b->pipe) return TVM_EINVAL;
  if (encode_us) *encode_us = b->pipe->encode_us();
  if (prepare_us) *prepare_us = b->pipe->prepare_us();
  return TVM_OK;
}

void tvm_pool_stats(uint64_t out[4]) {
  unsigned long long o[4];
  pool_stats(o);
  for (int i = 0; i < 4; i++) out[i] = o[i];
}

void tvm_pool_trim(void) { pool_trim(); }

int tvm_runtime_info(int* hip_runtime, int* hip_driver, char* path, size_t pathlen) {
  int rt = 0, drv = 0;
  // the HIP runtime THIS library's calls bind to: with a host process that loaded another
  // libamdhip64.so.7 first (torch's bundled one), the dynamic linker hands that one to us too
  const bool ok = hipRuntimeGetVersion(&rt) == hipSuccess;
  (void)hipDriverGetVersion(&drv);
  if (hip_runtime) *hip_runtime = rt;
  if (hip_driver) *hip_driver = drv;
  if (path && pathlen) {
    Dl_info di{};
    const char* where = dladdr(reinterpret_cast<void*>(&hipRuntimeGetVersion), &di) && di.dli_fname ? di.dli_fname : "";
    std::snprintf(path, pathlen, "%s", where);
  }
  return ok ? TVM_OK : TVM_EDEVICE;
}

int tvm_pipeline_stats(tvm_batch* b, uint64_t out[5]) {
  if (!b || !b->pipe || !out) return TVM_EINVAL;
  out[0] = b->pipe->h2d_bytes();
  out[1] = b->pipe->d2h_bytes();
  out[2] = b->pipe->chunks();
  out[3] = b->pipe->transport_form() ? 1 : 0;
  out[4] = b->pipe->encode_us();
  return TVM_OK;
}

// ---- sharding support ------------------------------------------------------------------

int tvm_db_rows_many(const tvm_db* db, const char* bucket, size_t n, const char* arena, const uint64_t* name_off,
                     const uint32_t* name_len, uint32_t* out) {
  if (!db || !db->finalized || !bucket || (n && (!arena || !name_off || !name_len || !out))) return TVM_EINVAL;
  const DB& d = db->db;
  const int32_t plat = d.find_plat(bucket);
  for (size_t i = 0; i < n; i++)
    out[i] = plat < 0 ? 0u : d.key_rows(uint32_t(plat), std::string_view(arena + name_off[i], name_len[i]));
  return TVM_OK;
}

int tvm_batch_upload_into(tvm_engine* e, tvm_batch* b, void* pkg_dev, void* adv_dev, uint64_t cap, char* err,
                          size_t errlen) {
  if (!e || !b || !pkg_dev || !adv_dev || cap == 0) return TVM_EINVAL;
  const int rc = tvm_batch_upload(e, b, 1, err, errlen);
  if (rc) return rc;
  (void)hipSetDevice(e->device);
  (void)hipFree(b->m.pkg);
  (void)hipFree(b->m.adv);
  b->m.pkg = static_cast<uint32_t*>(pkg_dev);
  b->m.adv = static_cast<uint32_t*>(adv_dev);
  b->m.cap = cap;
  b->external_out = true;
  return TVM_OK;
}

// ---- Red Hat batch epilogue (redhat.hip) -------------------------------------------------

namespace {

// rpm-order ranks of the Red Hat advisories' fixed versions, built on first use (device).
bool ensure_rh_rank(tvm_engine* e, std::string& err) {
  std::lock_guard<std::mutex> g(e->rh_mu);
  if (e->rh_rank) return true;
  // the merge's two per-advisory gathers (its group key, its fixed-version rank) in one word pair
  const std::vector<uint32_t> r = redhat_fixed_ranks(e->eng->db());
  const std::vector<uint2>& ids = e->fill->table().adv_rank;
  std::vector<uint2> rk(r.size());
  for (size_t i = 0; i < r.size(); i++) rk[i] = make_uint2(i < ids.size() ? ids[i].x : 0xFFFFFFFFu, r[i]);
  void* p = nullptr;
  if (hipMalloc(&p, std::max<size_t>(rk.size(), 1) * sizeof(uint2)) != hipSuccess ||
      (!rk.empty() && hipMemcpy(p, rk.data(), rk.size() * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess)) {
    if (p) (void)hipFree(p);
    err = "redhat merge: advisory ranks upload failed";
    return false;
  }
  e->rh_rank = static_cast<uint2*>(p);
  return true;
}

// Per tile of the batch: 1 = it holds Red Hat packages (the merge gives those a wave each).
std::vector<uint8_t> rh_tile_flags(const HostBatch& hb, const DB& db, uint32_t n_tiles) {
  const auto& pi = db.plat_info;
  const size_t n = hb.pk.size();
  std::vector<uint8_t> flags(n_tiles, 0);
  range_for(flags.size(), 64, [&](size_t t0, size_t t1) {
    for (size_t t = t0; t < t1; t++)
      for (size_t p = t * kTile; p < std::min(n, (t + 1) * kTile) && !flags[t]; p++) {
        const uint32_t plat = hb.pk[p].x;
        flags[t] = plat < pi.size() && pi[plat].drv == DRV_REDHAT;
      }
  });
  return flags;
}

RhInputs rh_inputs(tvm_engine* e, tvm_batch* b) {
  RhInputs in;
  in.pk = b->dev.pk;
  in.plats = e->eng->device_plats();
  in.n_plats = uint32_t(e->eng->db().plat_info.size());
  in.raw = &b->m;
  in.n_tiles = b->dev.n_tiles;
  in.n = b->dev.n;
  in.pkg_base = b->dev.pkg_base;
  in.rk = e->rh_rank;
  return in;
}

// Enqueues the merge (caller holds the shared lock and has checked the batch).
bool rh_launch(tvm_engine* e, tvm_batch* b, std::string& err) {
  (void)hipSetDevice(e->device);
  if (!ensure_rh_rank(e, err)) return false;
  if (!b->rh.tiles_known() && !b->rh.set_tiles(rh_tile_flags(b->hb, e->eng->db(), b->dev.n_tiles), err))
    return false;  // once per upload: which tiles hold Red Hat packages
  const RhInputs in = rh_inputs(e, b);
  if (!b->rh.launch(in, e->eng->stream(), err)) return false;
  b->merged = true;
  b->st_valid = false;
  return true;
}

// Merged Red Hat vulnerabilities of the merged list's entries `want` (all when null).
bool rh_vulns(tvm_engine* e, tvm_batch* b, const std::vector<uint2>* want, std::vector<Vuln>& vulns, std::string& err) {
  const DB& db = e->eng->db();
  std::vector<uint32_t> pkg, adv, base, contrib;
  std::vector<uint2> grp;
  if (!b->rh.fetch(rh_inputs(e, b), pkg, adv, base, grp, contrib, e->eng->stream(), err)) return false;
  const auto& pi = db.plat_info;
  std::vector<RhRec> recs;
  std::unordered_map<uint64_t, size_t> at;  // (package, representative) -> merged entry
  for (size_t i = 0; i < pkg.size(); i++) {
    const uint32_t plat = b->hb.pk[pkg[i] - b->dev.pkg_base].x;
    if (plat >= pi.size() || pi[plat].drv != DRV_REDHAT) continue;
    RhRec r{};
    r.pkg = pkg[i];
    r.base = base[i];
    r.best = db.advs[adv[i]].fixed.empty() ? RH_NONE : adv[i];
    r.start = grp[i].x;
    r.len = grp[i].y;
    if (want) at.emplace((uint64_t(pkg[i]) << 32) | adv[i], recs.size());
    recs.push_back(r);
  }
  if (want) {
    std::vector<RhRec> sel;
    for (const uint2& q : *want) {
      auto it = at.find((uint64_t(q.x) << 32) | q.y);
      if (it != at.end()) sel.push_back(recs[it->second]);
    }
    recs.swap(sel);
  }
  redhat_batch_vulns(db, b->hb, recs, contrib, b->dev.pkg_base, vulns);
  return true;
}

}  // namespace

int tvm_match_redhat_merge(tvm_engine* e, tvm_batch* b, char* err, size_t errlen) {
  if (!e || !b || !b->uploaded) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  std::string msg;
  if (b->merged) return TVM_OK;  // already the merged list of the last launch
  if (!rh_launch(e, b, msg)) {
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

int tvm_match_redhat_result(tvm_engine* e, tvm_batch* b, tvm_result* out, char* err, size_t errlen) {
  if (!e || !b || !out || !b->uploaded) return TVM_EINVAL;
  memset(out, 0, sizeof(*out));
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  std::string msg;
  std::vector<Vuln> vulns;
  if ((!b->merged && !rh_launch(e, b, msg)) || !rh_vulns(e, b, nullptr, vulns, msg)) {
    set_err(err, errlen, "tvm_match_redhat_result: " + msg);
    return TVM_EDEVICE;
  }
  export_result(e->eng->db(), std::move(vulns), false, out);
  return TVM_OK;
}

int tvm_match_redhat_vulns(tvm_engine* e, tvm_batch* b, const uint32_t* pairs, uint64_t n, tvm_result* out, char* err,
                           size_t errlen) {
  if (!e || !b || !out || !b->uploaded || (n && !pairs)) return TVM_EINVAL;
  memset(out, 0, sizeof(*out));
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e) || !b->merged) {
    set_err(err, errlen, b->merged ? kStale : "tvm_match_redhat_vulns: run tvm_match_redhat_merge first");
    return TVM_EINVAL;
  }
  std::vector<uint2> want(n);
  for (uint64_t i = 0; i < n; i++) want[i] = make_uint2(pairs[2 * i], pairs[2 * i + 1]);
  std::string msg;
  std::vector<Vuln> vulns;
  if (!rh_vulns(e, b, &want, vulns, msg)) {
    set_err(err, errlen, "tvm_match_redhat_vulns: " + msg);
    return TVM_EDEVICE;
  }
  export_result(e->eng->db(), std::move(vulns), false, out);
  return TVM_OK;
}

int tvm_match_redhat_merge_time(tvm_engine* e, tvm_batch* b, int steps, double* ms, char* err, size_t errlen) {
  if (!e || !b || !b->uploaded || steps <= 0 || !ms) return TVM_EINVAL;
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  (void)hipSetDevice(e->device);
  std::string msg;
  if (!rh_launch(e, b, msg)) {  // sizes the buffers and builds the ranks outside the timed region
    set_err(err, errlen, msg);
    return TVM_EDEVICE;
  }
  hipStream_t st = e->eng->stream();
  hipEvent_t t0 = nullptr, t1 = nullptr;
  float f = 0;
  bool ok = hipEventCreate(&t0) == hipSuccess && hipEventCreate(&t1) == hipSuccess && hipEventRecord(t0, st) == hipSuccess;
  const RhInputs in = rh_inputs(e, b);
  for (int i = 0; ok && i < steps; i++) ok = b->rh.launch(in, st, msg);
  ok = ok && hipEventRecord(t1, st) == hipSuccess && hipEventSynchronize(t1) == hipSuccess &&
       hipEventElapsedTime(&f, t0, t1) == hipSuccess;
  if (t0) (void)hipEventDestroy(t0);
  if (t1) (void)hipEventDestroy(t1);
  if (!ok) {
    set_err(err, errlen, msg.empty() ? "hipEvent timing failed" : msg);
    return TVM_EDEVICE;
  }
  *ms = f;
  return TVM_OK;
}

// ---- DetectedVulnerability sets of a batch (the drivers' epilogues on the batch path) -------

namespace {

const VulnTemplates& templates(tvm_db* d) {
  std::lock_guard<std::mutex> g(d->tmpl_mu);
  if (!d->tmpl) {
    auto t = std::make_unique<VulnTemplates>();
    advisory_templates(d->db, t->v);
    t->c.resize(t->v.size());
    t->vp.resize(t->v.size());
    range_for(t->v.size(), 1 << 14, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; i++) to_c(d->db, t->v[i], t->c[i], t->vp[i]);
    });
    d->tmpl = std::move(t);
  }
  return *d->tmpl;
}

// What a tvm_vuln_set points into: the export's pinned lists (device-resident path) and the
// merged Red Hat groups' records; a pipelined pass's set points into its result (no copy).
struct VulnSetStore {
  VulnExport ex;
  std::vector<tvm_vuln> gc;
  std::vector<std::vector<const char*>> gvp;
};

bool batch_has_redhat(const tvm_batch* b, const DB& db) {
  // packages are only ever appended: the answer holds until the batch grows or the DB changes
  if (b->rh_seen_n == b->hb.pk.size() && b->rh_seen_db == &db) return b->rh_seen;
  const auto& pi = db.plat_info;
  std::atomic<bool> any{false};
  pool_range_for(b->hb.pk.size(), 1 << 16, [&](size_t a, size_t z) {
    uint32_t last = 0xFFFFFFFFu;
    for (size_t i = a; i < z && !any.load(std::memory_order_relaxed); i++) {
      const uint32_t pl = b->hb.pk[i].x;
      if (pl == last) continue;
      last = pl;
      if (pl < pi.size() && pi[pl].drv == DRV_REDHAT) any.store(true, std::memory_order_relaxed);
    }
  });
  b->rh_seen_n = b->hb.pk.size();
  b->rh_seen_db = &db;
  b->rh_seen = any.load();
  return b->rh_seen;
}

void set_out(tvm_db* d, VulnSetStore* st, const uint32_t* row_end, size_t n_pkgs, uint32_t first_pkg,
             const uint8_t* rec, uint32_t width, size_t n, tvm_vuln_set* out) {
  const VulnTemplates& t = templates(d);
  out->row_end = row_end;
  out->n_pkgs = n_pkgs;
  out->first_pkg = first_pkg;
  out->rec = rec;
  out->rec_width = width;
  out->n = n;
  out->adv_recs = t.c.data();
  out->n_adv_recs = t.c.size();
  out->grp_recs = st->gc.data();
  out->n_grp_recs = st->gc.size();
  out->priv = st;
}


// The DetectedVulnerability set of a device match list `in` (raw, or Red Hat-merged): the
// export's per-package record lists in pinned memory, and the records of the merged Red Hat
// groups built on the host threads from their members' own records - the first member's (ID,
// Status, Severity), the representative's FixedVersion, and VendorIDs: the first member's own
// when it is the one fixed member, else the sorted union of the fixed members'
// (ustrings.Unique; redhat.go:146-187) - as pointers into those records.
bool export_set(tvm_engine* e, const ExportList& in, size_t n_pkgs, uint32_t first_pkg, tvm_vuln_set* out,
                std::string& msg) {
  const DB& db = e->eng->db();
  const VulnTemplates& tp = templates(e->db);  // built by the first export of a DB
  auto st = std::make_unique<VulnSetStore>();
  if (!export_vulns(e->device, e->eng->stream(), in, uint32_t(db.advs.size()), st->ex, msg)) return false;
  const VulnExport& ex = st->ex;
  if (ex.n_groups) {
    st->gc.resize(ex.n_groups);
    st->gvp.resize(ex.n_groups);
    pool_range_for(ex.n_groups, 1 << 10, [&](size_t a, size_t z) {
      std::vector<const char*> ids;
      for (size_t k = a; k < z; k++) {
        const uint4 g = ex.groups[k];
        const tvm_vuln& base = tp.c[g.z];
        tvm_vuln& c = st->gc[k];
        c = base;
        const bool has_best = !db.advs[g.w].fixed.empty();
        c.fixed_version = has_best ? tp.c[g.w].fixed_version : "";
        uint32_t n_fixed = 0;
        ids.clear();
        for (uint32_t m = ex.moff[k]; m < ex.moff[k + 1]; m++) {
          const uint32_t adv = ex.members[m];
          if (adv >= db.advs.size() || db.advs[adv].fixed.empty()) continue;
          n_fixed++;
          const tvm_vuln& mv = tp.c[adv];
          ids.insert(ids.end(), mv.vendor_ids, mv.vendor_ids + mv.n_vendor_ids);
        }
        if (n_fixed == 1 && !db.advs[g.z].fixed.empty()) continue;  // the first member's list as it is
        c.vendor_ids = nullptr;
        c.n_vendor_ids = 0;
        if (!n_fixed) continue;
        std::sort(ids.begin(), ids.end(), [](const char* x, const char* y) { return std::strcmp(x, y) < 0; });
        ids.erase(std::unique(ids.begin(), ids.end(), [](const char* x, const char* y) { return !std::strcmp(x, y); }),
                  ids.end());
        st->gvp[k] = ids;
        c.vendor_ids = st->gvp[k].empty() ? nullptr : st->gvp[k].data();
        c.n_vendor_ids = st->gvp[k].size();
      }
    });
  }
  const VulnSetStore* sp = st.get();
  set_out(e->db, st.release(), sp->ex.row_end_h, n_pkgs, first_pkg, sp->ex.rec_h, sp->ex.width, sp->ex.n, out);
  return true;
}

}  // namespace

int tvm_match_vulns(tvm_engine* e, tvm_batch* b, tvm_vuln_set* out, char* err, size_t errlen) {
  if (!e || !b || !out || !b->uploaded) return TVM_EINVAL;
  memset(out, 0, sizeof(*out));
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  const DB& db = e->eng->db();
  std::string msg;
  (void)hipSetDevice(e->device);
  // Red Hat packages report merged groups (redhat.go:146-187): the merge runs first
  if (!b->merged && batch_has_redhat(b, db) && !rh_launch(e, b, msg)) {
    set_err(err, errlen, "tvm_match_vulns: " + msg);
    return TVM_EDEVICE;
  }
  uint64_t total = 0, bits = 0;
  int64_t ep = -1;
  if (match_status_locked(e, b, &total, &ep, &bits) != TVM_OK) {
    set_err(err, errlen, "tvm_match_vulns: reading the match status failed");
    return TVM_EDEVICE;
  }
  if (bits || ep >= 0 || total > cur(b).cap || b->m.ctl == nullptr) {
    set_err(err, errlen, bits ? "tvm_match_vulns: match kernel internal error bits " + std::to_string(bits)
                         : ep >= 0 ? "tvm_match_vulns: the batch met an undecodable advisory (package " +
                                         std::to_string(ep) + ")"
                                   : "tvm_match_vulns: the match buffer overflowed (upload with a larger cap)");
    return TVM_EINVAL;
  }
  ExportList in;
  in.list = cur(b);
  in.total = total;
  in.n_tiles = b->dev.n_tiles;
  in.pkg_base = b->dev.pkg_base;
  if (b->merged) {
    const RhMerged& mg = b->rh.merged();
    in.rh = true;
    in.base = mg.base;
    in.grp = mg.grp;
    in.raw_adv = b->m.adv;
    in.raw_cap = b->m.cap;
    in.pk = b->dev.pk;
    in.plats = e->eng->device_plats();
    in.n_plats = uint32_t(db.plat_info.size());
  }
  if (!export_set(e, in, b->hb.pk.size(), b->dev.pkg_base, out, msg)) {
    set_err(err, errlen, "tvm_match_vulns: " + msg);
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

int tvm_pipeline_vulns(tvm_engine* e, tvm_batch* b, tvm_vuln_set* out, char* err, size_t errlen) {
  if (!e || !b || !out) return TVM_EINVAL;
  memset(out, 0, sizeof(*out));
  if (!b->pipe || !b->pipe_ok || b->pipe_total > b->pipe->cap()) {
    set_err(err, errlen, "tvm_pipeline_vulns: no completed tvm_pipeline_run on this batch");
    return TVM_EINVAL;
  }
  std::shared_lock<std::shared_mutex> lk(e->mu);
  if (!bind(b, e)) {
    set_err(err, errlen, kStale);
    return TVM_EINVAL;
  }
  if (b->pipe_errp >= 0) {
    set_err(err, errlen, "tvm_pipeline_vulns: the batch met an undecodable advisory (package " +
                             std::to_string(b->pipe_errp) + ")");
    return TVM_EINVAL;
  }
  const DB& db = e->eng->db();
  if (!batch_has_redhat(b, db)) {  // the lists the pass left in pinned memory ARE the set (no copy)
    templates(e->db);
    auto st = std::make_unique<VulnSetStore>();
    set_out(e->db, st.release(), b->pipe->row_end(), b->hb.pk.size(), b->pkg_base,
            reinterpret_cast<const uint8_t*>(b->pipe->adv()), b->pipe->packed() ? 3u : 4u, b->pipe_total, out);
    return TVM_OK;
  }
  // Red Hat packages report merged groups (redhat.go:146-187): the pass's whole match list is
  // still in HBM (Pipeline::matches), so the device merge and the export run over it as over a
  // device-resident pass's list, and the set is the export's own copy
  std::string msg;
  (void)hipSetDevice(e->device);
  const Pipeline& P = *b->pipe;
  const DevBatch& dv = P.dev_batch();
  hipStream_t st = e->eng->stream();
  if (!ensure_rh_rank(e, msg) ||
      (!b->pipe_rh.tiles_known() && !b->pipe_rh.set_tiles(rh_tile_flags(b->hb, db, dv.n_tiles), msg))) {
    set_err(err, errlen, "tvm_pipeline_vulns: " + msg);
    return TVM_EDEVICE;
  }
  RhInputs ri;
  ri.pk = dv.pk;
  ri.plats = e->eng->device_plats();
  ri.n_plats = uint32_t(db.plat_info.size());
  ri.raw = &P.matches();
  ri.n_tiles = dv.n_tiles;
  ri.n = dv.n;
  ri.pkg_base = dv.pkg_base;
  ri.rk = e->rh_rank;
  unsigned long long mctl[8] = {};
  if (!b->pipe_rh.launch(ri, st, msg) ||
      hipMemcpyAsync(mctl, b->pipe_rh.merged().m.ctl, sizeof(mctl), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    set_err(err, errlen, "tvm_pipeline_vulns: " + (msg.empty() ? std::string("redhat merge failed") : msg));
    return TVM_EDEVICE;
  }
  if (mctl[3] || mctl[0] > b->pipe_rh.merged().cap) {
    set_err(err, errlen, (mctl[3] & ERR_RH_ORDER)
                             ? "tvm_pipeline_vulns: a Red Hat package's advisories are not grouped by VulnerabilityID"
                             : "tvm_pipeline_vulns: redhat merge error bits " + std::to_string(mctl[3]));
    return TVM_EDEVICE;
  }
  const RhMerged& mg = b->pipe_rh.merged();
  ExportList in;
  in.list = mg.m;
  in.total = mctl[0];
  in.n_tiles = dv.n_tiles;
  in.pkg_base = dv.pkg_base;
  in.rh = true;
  in.base = mg.base;
  in.grp = mg.grp;
  in.raw_adv = P.matches().adv;
  in.raw_cap = P.matches().cap;
  in.pk = dv.pk;
  in.plats = e->eng->device_plats();
  in.n_plats = uint32_t(db.plat_info.size());
  if (!export_set(e, in, b->hb.pk.size(), b->pkg_base, out, msg)) {
    set_err(err, errlen, "tvm_pipeline_vulns: " + msg);
    return TVM_EDEVICE;
  }
  return TVM_OK;
}

void tvm_vuln_set_free(tvm_vuln_set* s) {
  if (!s) return;
  delete static_cast<VulnSetStore*>(s->priv);
  memset(s, 0, sizeof(*s));
}

int tvm_vuln_set_walk(const tvm_vuln_set* s, const tvm_batch* b, uint64_t* n_out, uint64_t* digest) {
  if (!s || !b || (s->n_pkgs && !s->row_end) || (s->n && !s->rec) || s->n_pkgs > b->hb.pk.size() ||
      (s->rec_width != 3 && s->rec_width != 4))
    return TVM_EINVAL;
  const size_t np = s->n_pkgs;
  if (np && s->row_end[np - 1] != s->n) return TVM_EINVAL;
  const HostBatch& hb = b->hb;
  const uint32_t W = s->rec_width;
  auto rec_at = [&](uint64_t i) {
    const uint8_t* q = s->rec + i * W;
    uint64_t r = uint64_t(q[0]) | uint64_t(q[1]) << 8 | uint64_t(q[2]) << 16;
    return W == 4 ? r | uint64_t(q[3]) << 24 : r;
  };
  auto vuln_of = [&](uint64_t r) -> const tvm_vuln* {
    return r < s->n_adv_recs ? s->adv_recs + r
           : r - s->n_adv_recs < s->n_grp_recs ? s->grp_recs + (r - s->n_adv_recs) : nullptr;
  };
  std::atomic<uint64_t> dsum{0}, cnt{0}, bad{0};
  // pieces of whole 64-package groups: a group's first package offset is tile_off[g]
  const size_t groups = (np + kGroup - 1) / kGroup;
  pool_range_for(groups, 64, [&](size_t g0, size_t g1) {
    uint64_t d = 0, c = 0, nb = 0;
    const uint64_t i_end = std::min<size_t>(np, g1 * kGroup) ? s->row_end[std::min<size_t>(np, g1 * kGroup) - 1] : 0;
    // records are scattered over the DB's (~1.7M x 136 B): their loads overlap, every line a
    // record's fields span prefetched (a record straddles up to three 64-B lines)
    constexpr uint64_t kAhead = 32;
    for (size_t g = g0; g < g1; g++) {
      uint64_t off = hb.tile_off[g];
      for (size_t p = g * kGroup; p < std::min(np, (g + 1) * kGroup); p++) {
        const uint32_t nl = hb.pk[p].y & 0xFFFFu, vl = hb.pk[p].y >> 16;
        uint64_t ilen = vl;  // InstalledVersion: the report's override, else the batch version
        if (p < b->rep_has[1].size() && b->rep_has[1][p]) ilen = b->rep[1][p].size();
        else if (vl) (void)*static_cast<const volatile uint8_t*>(hb.arena.data() + off + nl);  // touched
        off += nl + vl;
        const uint64_t i0 = p ? s->row_end[p - 1] : 0, i1 = s->row_end[p];
        const uint64_t pg = uint64_t(s->first_pkg) + p;
        for (uint64_t i = i0; i < i1; i++) {
          if (i + kAhead < i_end)
            if (const tvm_vuln* ahead = vuln_of(rec_at(i + kAhead))) {
              const char* c = reinterpret_cast<const char*>(ahead);
              __builtin_prefetch(c);
              __builtin_prefetch(c + 64);
              __builtin_prefetch(c + sizeof(tvm_vuln) - 1);
            }
          const uint64_t r = rec_at(i);
          const tvm_vuln* v = vuln_of(r);
          if (!v) {
            nb++;
            continue;
          }
          // the record's value fields as a caller's copy reads them (its string pointers are
          // handed on, not dereferenced, as INTEGRATION.md §3's loop does)
          const uint64_t fl = uint64_t(uint32_t(v->status) & 0xFFu) << 32 | uint64_t(v->n_vendor_ids & 0xFFu) << 24 |
                              uint64_t(v->has_data_source & 1) << 8 | (v->copy_flags & 0xFFu);
          uint64_t h = pg * 0x9E3779B97F4A7C15ull + r * 0xC2B2AE3D27D4EB4Full + (ilen << 40) + fl;
          h ^= h >> 33;
          h *= 0xff51afd7ed558ccdull;
          h ^= h >> 33;
          h *= 0xc4ceb9fe1a85ec53ull;
          h ^= h >> 33;
          d += h;
          c++;
        }
      }
    }
    dsum.fetch_add(d, std::memory_order_relaxed);
    cnt.fetch_add(c, std::memory_order_relaxed);
    bad.fetch_add(nb, std::memory_order_relaxed);
  });
  if (bad.load()) return TVM_EINVAL;  // a record index beyond the set's records
  if (n_out) *n_out = cnt.load();
  if (digest) *digest = dsum.load();
  return TVM_OK;
}

int tvm_batch_report_get(const tvm_batch* b, uint64_t first, uint64_t n, tvm_str* names, tvm_str* versions,
                         tvm_str* paths) {
  const uint64_t size = b ? b->hb.pk.size() : 0;
  if (!b || first > size || n > size - first) return TVM_EINVAL;
  const char* arena = reinterpret_cast<const char*>(b->hb.arena.data());
  uint64_t off = n ? b->hb.name_off(first) : 0;
  for (uint64_t i = first; i < first + n; i++) {
    const uint32_t nl = b->hb.pk[i].y & 0xFFFFu, vl = b->hb.pk[i].y >> 16;
    auto rep = [&](int f, tvm_str dflt) {
      if (i < b->rep_has[f].size() && b->rep_has[f][i]) return tvm_str{b->rep[f][i].data(), b->rep[f][i].size()};
      return dflt;
    };
    if (names) names[i - first] = rep(0, tvm_str{nullptr, 0});
    if (versions) versions[i - first] = rep(1, tvm_str{arena + off + nl, vl});
    if (paths) paths[i - first] = rep(2, tvm_str{nullptr, 0});
    off += nl + vl;
  }
  return TVM_OK;
}

// ---- native CycloneDX decode (sbom.cpp) ---------------------------------------------------

struct tvm_sbom {
  Sbom s;
};

int tvm_sbom_decode_cyclonedx(const char* text, size_t len, uint32_t flags, tvm_sbom** out, char* err, size_t errlen) {
  if (!out || (len && !text) || (flags & ~uint32_t(TVM_SBOM_BORROW))) return TVM_EINVAL;
  *out = nullptr;
  auto* h = new (std::nothrow) tvm_sbom();
  if (!h) return TVM_EINVAL;
  std::string msg;
  bool good = false;
  try {  // a document of any size is untrusted input: running out of memory is an error, not an abort
    good = decode_cyclonedx(std::string_view(text, len), h->s, msg, (flags & TVM_SBOM_BORROW) != 0);
  } catch (const std::bad_alloc&) {
    msg = "failed to decode CycloneDX JSON: out of memory";
  }
  if (!good) {
    delete h;
    set_err(err, errlen, msg);
    return TVM_EINVAL;
  }
  *out = h;
  return TVM_OK;
}

void tvm_sbom_free(tvm_sbom* s) { delete s; }

int tvm_sbom_info(const tvm_sbom* h, int32_t* has_os, tvm_str* os_family, tvm_str* os_name, tvm_str* serial,
                  int64_t* version, size_t* n_apps) {
  if (!h) return TVM_EINVAL;
  const Sbom& s = h->s;
  if (has_os) *has_os = s.has_os ? 1 : 0;
  if (os_family) *os_family = tvm_str{s.os_family.data(), s.os_family.size()};
  if (os_name) *os_name = tvm_str{s.os_name.data(), s.os_name.size()};
  if (serial) *serial = tvm_str{s.serial.data(), s.serial.size()};
  if (version) *version = s.version;
  if (n_apps) *n_apps = s.targets.empty() ? 0 : s.targets.size() - 1;
  return TVM_OK;
}

int tvm_sbom_packages(const tvm_sbom* h, int64_t app, tvm_str* type, tvm_str* file_path, const tvm_package** pkgs,
                      size_t* n) {
  if (!h || app < -1 || size_t(app + 1) >= h->s.targets.size()) return TVM_EINVAL;
  const Sbom& s = h->s;
  const SbomTarget& t = s.targets[size_t(app + 1)];
  if (type) *type = tvm_str{t.type.data(), t.type.size()};
  if (file_path) *file_path = tvm_str{t.file_path.data(), t.file_path.size()};
  if (pkgs) *pkgs = s.view.data() + t.begin;
  if (n) *n = t.end - t.begin;
  return TVM_OK;
}

int tvm_sbom_package_extra(const tvm_sbom* h, int64_t app, size_t i, tvm_sbom_extra* out) {
  if (!h || !out || app < -1 || size_t(app + 1) >= h->s.targets.size()) return TVM_EINVAL;
  const SbomTarget& t = h->s.targets[size_t(app + 1)];
  if (i >= t.end - t.begin) return TVM_EINVAL;
  const SbomExtra& p = h->s.extra[t.begin + i];
  auto ts = [](std::string_view x) { return tvm_str{x.data(), x.size()}; };
  out->purl = ts(p.purl);
  out->bom_ref = ts(p.bom_ref);
  out->layer_digest = ts(p.layer_digest);
  out->layer_diff_id = ts(p.layer_diff_id);
  out->present = p.present;
  return TVM_OK;
}
