// Load-time flattener (see db.h).
#include "db.h"

#include <algorithm>

#include "json.h"
#include "verkey.h"

namespace tvm {
namespace {

struct VecSink {
  std::vector<uint8_t>* v;
  void put(uint8_t b) { v->push_back(b); }
};

bool dec_string(const JVal& v, std::string& out, const char* field, std::string& err) {
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Str) {
    err = std::string("json: cannot unmarshal ") + (v.kind == JVal::Arr ? "array" : v.kind == JVal::Obj ? "object" : v.kind == JVal::Num ? "number" : "bool") +
          " into Go struct field Advisory." + field + " of type string";
    return false;
  }
  out = v.s;
  return true;
}

bool dec_strings(const JVal& v, std::vector<std::string>& out, const char* field, std::string& err) {
  if (v.kind == JVal::Null) { out.clear(); return true; }
  if (v.kind != JVal::Arr) {
    err = std::string("json: cannot unmarshal into Go struct field Advisory.") + field + " of type []string";
    return false;
  }
  out.clear();
  for (const JVal& e : v.arr) {
    if (e.kind == JVal::Null) { out.emplace_back(); continue; }
    if (e.kind != JVal::Str) {
      err = std::string("json: cannot unmarshal into Go struct field Advisory.") + field + " of type string";
      return false;
    }
    out.push_back(e.s);
  }
  return true;
}

bool dec_int(const JVal& v, int64_t& out, const char* field, std::string& err) {
  if (v.kind == JVal::Null) return true;
  if (!json_int(v, out)) {
    err = std::string("json: cannot unmarshal ") + (v.kind == JVal::Num ? "number " + v.s : std::string("value")) +
          " into Go struct field Advisory." + field + " of type int";
    return false;
  }
  return true;
}

const char* const kStatuses[] = {"unknown", "not_affected", "affected", "fixed", "under_investigation",
                                 "will_not_fix", "fix_deferred", "end_of_life"};

bool dec_source(const JVal& v, DataSource& ds, std::string& err) {
  if (v.kind != JVal::Obj) {
    err = "json: cannot unmarshal into Go value of type types.DataSource";
    return false;
  }
  for (const auto& [k, x] : v.obj) {
    std::string* dst = json_key_eq(k, "ID") ? &ds.id : json_key_eq(k, "Name") ? &ds.name : json_key_eq(k, "URL") ? &ds.url : nullptr;
    if (!dst) continue;
    if (x.kind == JVal::Null) continue;
    if (x.kind != JVal::Str) {
      err = "json: cannot unmarshal into Go struct field DataSource." + k + " of type string";
      return false;
    }
    *dst = x.s;
  }
  return true;
}

}  // namespace

bool decode_advisory(std::string_view json, Advisory& a, std::string& err) {
  JVal v;
  if (!json_parse(json, v, err)) return false;
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Obj) {
    err = "json: cannot unmarshal into Go value of type types.Advisory";
    return false;
  }
  for (const auto& [k, x] : v.obj) {
    bool ok = true;
    if (json_key_eq(k, "VulnerabilityID")) { std::string tmp; ok = dec_string(x, tmp, "VulnerabilityID", err); }
    else if (json_key_eq(k, "VendorIDs")) ok = dec_strings(x, a.vendor_ids, "VendorIDs", err);
    else if (json_key_eq(k, "Arches")) ok = dec_strings(x, a.arches, "Arches", err);
    else if (json_key_eq(k, "Status")) {
      // trivy-db Status: integer in the DB (fixtures), string name accepted as well.
      if (x.kind == JVal::Str) {
        a.status = 0;
        for (int i = 0; i < 8; i++)
          if (x.s == kStatuses[i]) a.status = i;
      } else ok = dec_int(x, a.status, "Status", err);
    }
    else if (json_key_eq(k, "Severity")) ok = dec_int(x, a.severity, "Severity", err);
    else if (json_key_eq(k, "FixedVersion")) ok = dec_string(x, a.fixed, "FixedVersion", err);
    else if (json_key_eq(k, "AffectedVersion")) ok = dec_string(x, a.affected, "AffectedVersion", err);
    else if (json_key_eq(k, "VulnerableVersions")) ok = dec_strings(x, a.vulnerable, "VulnerableVersions", err);
    else if (json_key_eq(k, "PatchedVersions")) ok = dec_strings(x, a.patched, "PatchedVersions", err);
    else if (json_key_eq(k, "UnaffectedVersions")) ok = dec_strings(x, a.unaffected, "UnaffectedVersions", err);
    else if (json_key_eq(k, "DataSource")) {
      a.has_inline_source = false;
      a.inline_source = DataSource{};
      if (x.kind != JVal::Null) ok = a.has_inline_source = dec_source(x, a.inline_source, err);
    }
    else if (json_key_eq(k, "Custom")) a.custom = x.kind == JVal::Null ? std::string() : std::string(x.raw);
    if (!ok) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------------

void DB::put(const std::vector<std::string>& path, std::string_view value) {
  if (path.empty()) return;
  Bucket* b = &root_;
  for (size_t i = 0; i + 1 < path.size(); i++) b = &b->sub[path[i]];
  b->kv[path.back()] = std::string(value);
}

bool classify_os_bucket(std::string_view root, uint8_t& drv, uint8_t& cmp, uint32_t& flags) {
  auto starts = [&](const char* p) { return root.rfind(p, 0) == 0; };
  flags = 0;
  if (starts("debian ")) { drv = DRV_DEBIAN; cmp = CMP_DEB; return true; }
  if (starts("ubuntu ")) { drv = DRV_UBUNTU; cmp = CMP_DEB; flags = PLAT_LOOKUP_FIRST; return true; }
  if (starts("amazon linux ")) { drv = DRV_AMAZON; cmp = CMP_DEB; flags = PLAT_LOOKUP_FIRST; return true; }
  return false;
}

int32_t DB::find_plat(std::string_view root) const {
  auto it = plat_by_name_.find(std::string(root));
  return it == plat_by_name_.end() ? -1 : int32_t(it->second);
}

int32_t DB::find_key(uint32_t plat, std::string_view name) const {
  uint64_t h = key_hash(plat, reinterpret_cast<const uint8_t*>(name.data()), uint32_t(name.size()));
  if (slot_hash.empty()) return -1;
  for (uint64_t i = h & slot_mask; slot_hash[i]; i = (i + 1) & slot_mask) {
    if (slot_hash[i] != h) continue;
    const SlotVal& v = slot_val[i];
    if ((v.name_len & SLOT_LEN_MASK) == name.size() &&
        std::equal(name.begin(), name.end(), name_arena.begin() + v.name_off))
      return int32_t(slot_key[i]);
  }
  return -1;
}

uint32_t DB::intern_key(const std::vector<uint8_t>& k) {
  std::string s(k.begin(), k.end());
  auto it = key_dedup_.find(s);
  if (it != key_dedup_.end()) return it->second;
  uint32_t off = uint32_t(key_words.size());
  size_t nw = (k.size() + 7) / 8;
  key_words.resize(key_words.size() + (nw ? nw : 1), 0);
  for (size_t i = 0; i < k.size(); i++) key_words[off + i / 8] |= uint64_t(k[i]) << (8 * (i % 8));
  key_dedup_.emplace(std::move(s), off);
  return off;
}

void DB::flatten_os(uint32_t plat, const Bucket& root, int32_t ds) {
  for (const auto& [pkg, bkt] : root.sub) {
    Key key;
    key.plat = plat;
    key.name = pkg;
    for (const auto& [vid, val] : bkt.kv) {
      Advisory a;
      std::string err;
      if (!decode_advisory(val, a, err)) {
        if (!key.poisoned) key.err = "failed to unmarshal advisory JSON: " + err;
        key.poisoned = true;
        continue;
      }
      a.vuln_id = vid;
      // trivy-db GetAdvisories: the data-source bucket entry wins when non-empty,
      // otherwise the value's own DataSource (if any) stays.
      if (ds >= 0) {
        a.data_source = ds;
      } else if (a.has_inline_source) {
        sources.push_back(a.inline_source);
        a.data_source = int32_t(sources.size() - 1);
      }
      key.advs.push_back(uint32_t(advs.size()));
      advs.push_back(std::move(a));
    }
    if (key.poisoned) key.advs.clear();
    keys.push_back(std::move(key));
  }
}

void DB::build_index() {
  // rows + key arena
  rows.clear();
  std::vector<uint8_t> kb;
  std::vector<uint32_t> row_begin(keys.size()), row_count(keys.size());
  for (size_t k = 0; k < keys.size(); k++) {
    const Key& key = keys[k];
    const Platform& P = plats[key.plat];
    row_begin[k] = uint32_t(rows.size());
    for (uint32_t ai : key.advs) {
      const Advisory& a = advs[ai];
      Row r{};
      r.adv = ai;
      r.lo_len = KEY_INF;
      if (P.cmp == CMP_DEB) {
        if (a.fixed.empty()) {
          // debian.go:99-102 / ubuntu.go:110-113: unfixed is always reported;
          // amazon.go:73-77 parses "" and skips the advisory.
          if (P.drv == DRV_AMAZON) continue;
          r.hi_len = KEY_INF;
        } else {
          kb.clear();
          VecSink s{&kb};
          if (!deb_encode(reinterpret_cast<const uint8_t*>(a.fixed.data()), uint32_t(a.fixed.size()), s)) continue;
          r.hi_off = intern_key(kb);
          r.hi_len = uint16_t(kb.size());
          for (size_t i = 0; i < kb.size() && i < 16; i++)
            (i < 8 ? r.hi_pre0 : r.hi_pre1) |= uint64_t(kb[i]) << (8 * (i % 8));
        }
      } else {
        continue;
      }
      rows.push_back(r);
    }
    row_count[k] = uint32_t(rows.size()) - row_begin[k];
  }
  n_rows_total = rows.size();
  if (key_words.empty()) key_words.push_back(0);

  // hash index, load factor <= 0.5
  uint64_t cap = 16;
  while (cap < keys.size() * 2) cap <<= 1;
  slot_mask = cap - 1;
  slot_hash.assign(cap, 0);
  slot_val.assign(cap, SlotVal{});
  slot_key.assign(cap, 0);
  name_arena.clear();
  for (size_t k = 0; k < keys.size(); k++) {
    const Key& key = keys[k];
    uint64_t h = key_hash(key.plat, reinterpret_cast<const uint8_t*>(key.name.data()), uint32_t(key.name.size()));
    uint64_t i = h & slot_mask;
    while (slot_hash[i]) i = (i + 1) & slot_mask;
    slot_hash[i] = h;
    SlotVal v;
    v.name_off = uint32_t(name_arena.size());
    v.name_len = uint32_t(key.name.size()) | (key.poisoned ? SLOT_POISONED : 0);
    v.row_begin = row_begin[k];
    v.row_count = row_count[k];
    slot_val[i] = v;
    slot_key[i] = uint32_t(k);
    name_arena.insert(name_arena.end(), key.name.begin(), key.name.end());
  }
  if (name_arena.empty()) name_arena.push_back(0);

  plat_info.resize(plats.size());
  for (size_t p = 0; p < plats.size(); p++) {
    plat_info[p].cmp = plats[p].cmp;
    plat_info[p].drv = plats[p].drv;
    plat_info[p].flags = plats[p].flags;
  }
  if (plat_info.empty()) plat_info.push_back(PlatInfo{});
}

bool DB::finalize(std::string& err) {
  // data sources: bucket "data-source", key = root bucket name
  std::map<std::string, int32_t> ds_of_root;
  std::map<std::string, std::string> ds_err;
  auto it = root_.sub.find("data-source");
  sources.clear();
  if (it != root_.sub.end()) {
    for (const auto& [root, val] : it->second.kv) {
      JVal v;
      std::string e;
      DataSource ds;
      if (!json_parse(val, v, e) || (v.kind != JVal::Null && !dec_source(v, ds, e))) {
        ds_err[root] = "failed to get data source: " + e;
        continue;
      }
      sources.push_back(ds);
      ds_of_root[root] = int32_t(sources.size() - 1);
    }
  }
  for (const auto& [name, b] : root_.sub) {
    uint8_t drv, cmp;
    uint32_t flags;
    if (!classify_os_bucket(name, drv, cmp, flags)) continue;
    uint32_t pid = uint32_t(plats.size());
    plats.push_back(Platform{name, drv, cmp, flags});
    plat_by_name_[name] = pid;
    int32_t ds = -1;
    auto d = ds_of_root.find(name);
    if (d != ds_of_root.end() && !sources[size_t(d->second)].empty()) ds = d->second;
    size_t first = keys.size();
    flatten_os(pid, b, ds);
    auto de = ds_err.find(name);
    if (de != ds_err.end()) {
      for (size_t k = first; k < keys.size(); k++) {
        keys[k].poisoned = true;
        keys[k].err = de->second;
        keys[k].advs.clear();
      }
    }
  }
  if (advs.size() >= ROW_ADV_MASK) { err = "too many advisories"; return false; }
  build_index();
  return true;
}

}  // namespace tvm
