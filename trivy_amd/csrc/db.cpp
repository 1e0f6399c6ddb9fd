// Load-time flattener (see db.h).
#include "db.h"

#include <algorithm>
#include <cstdlib>

#include "json.h"
#include "libdb.h"
#include "libver.h"

namespace tvm {
namespace {

struct VecSink {
  std::vector<uint8_t>* v;
  void put(uint8_t b) { v->push_back(b); }
};

const char* kind_name(const JVal& v) {
  switch (v.kind) {
    case JVal::Arr: return "array";
    case JVal::Obj: return "object";
    case JVal::Num: return "number";
    case JVal::Bool: return "bool";
    case JVal::Str: return "string";
    default: return "null";
  }
}

bool dec_string(const JVal& v, std::string& out, const char* field, std::string& err) {
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Str) {
    err = std::string("json: cannot unmarshal ") + kind_name(v) + " into Go struct field Advisory." + field +
          " of type string";
    return false;
  }
  out = v.s;
  return true;
}

bool dec_strings(const JVal& v, std::vector<std::string>& out, const char* field, std::string& err) {
  if (v.kind == JVal::Null) { out.clear(); return true; }
  if (v.kind != JVal::Arr) {
    err = std::string("json: cannot unmarshal ") + kind_name(v) + " into Go struct field Advisory." + field +
          " of type []string";
    return false;
  }
  out.clear();
  for (const JVal& e : v.arr) {
    if (e.kind == JVal::Null) { out.emplace_back(); continue; }
    if (e.kind != JVal::Str) {
      err = std::string("json: cannot unmarshal ") + kind_name(e) + " into Go struct field Advisory." + field +
            " of type string";
      return false;
    }
    out.push_back(e.s);
  }
  return true;
}

bool dec_int(const JVal& v, int64_t& out, const char* field, std::string& err) {
  if (v.kind == JVal::Null) return true;
  if (!json_int(v, out)) {
    err = std::string("json: cannot unmarshal ") + (v.kind == JVal::Num ? "number " + v.s : std::string(kind_name(v))) +
          " into Go struct field Advisory." + field + " of type int";
    return false;
  }
  return true;
}

bool dec_ints(const JVal& v, std::vector<int64_t>& out, const char* field, std::string& err) {
  out.clear();
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Arr) {
    err = std::string("json: cannot unmarshal ") + kind_name(v) + " into Go struct field " + field + " of type []int";
    return false;
  }
  for (const JVal& e : v.arr) {
    int64_t x = 0;
    if (e.kind != JVal::Null && !dec_int(e, x, field, err)) return false;
    out.push_back(x);
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

bool decode_adv_value(const JVal& v, Advisory& a, std::string& err);

bool decode_adv_value(const JVal& v, Advisory& a, std::string& err) {
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Obj) {
    err = std::string("json: cannot unmarshal ") + kind_name(v) + " into Go value of type types.Advisory";
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
    else if (json_key_eq(k, "Entries")) {
      a.entries.clear();
      if (x.kind == JVal::Null) continue;
      if (x.kind != JVal::Arr) {
        err = std::string("json: cannot unmarshal ") + kind_name(x) + " into Go struct field Advisory.Entries";
        return false;
      }
      for (const JVal& e : x.arr) {
        Advisory sub;
        if (!decode_adv_value(e, sub, err)) return false;
        a.entries.push_back(std::move(sub));
      }
    }
    if (!ok) return false;
  }
  return true;
}

// trivy-db redhat-oval value: {Entries: [{FixedVersion, Affected: [int], Arches, Status,
// Cves: [{ID, Severity}]}]} (fixture pkg/detector/ospkg/redhat/testdata/fixtures/redhat.yaml).
struct RhCve {
  std::string id;
  int64_t severity = 0;
};
struct RhEntry {
  std::string fixed;
  std::vector<int64_t> affected;
  std::vector<std::string> arches;
  int64_t status = 0;
  std::vector<RhCve> cves;
};

bool decode_redhat(std::string_view text, std::vector<RhEntry>& out, std::string& err) {
  JVal v;
  if (!json_parse(text, v, err)) return false;
  out.clear();
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Obj) {
    err = std::string("json: cannot unmarshal ") + kind_name(v) + " into Go value of type redhatoval.Advisory";
    return false;
  }
  for (const auto& [k, ents] : v.obj) {
    if (!json_key_eq(k, "Entries")) continue;
    out.clear();
    if (ents.kind == JVal::Null) continue;
    if (ents.kind != JVal::Arr) {
      err = std::string("json: cannot unmarshal ") + kind_name(ents) +
            " into Go struct field Advisory.Entries of type []redhatoval.Entry";
      return false;
    }
    for (const JVal& e : ents.arr) {
      RhEntry re;
      if (e.kind != JVal::Null) {
        if (e.kind != JVal::Obj) {
          err = std::string("json: cannot unmarshal ") + kind_name(e) + " into Go value of type redhatoval.Entry";
          return false;
        }
        for (const auto& [ek, x] : e.obj) {
          bool ok = true;
          if (json_key_eq(ek, "FixedVersion")) ok = dec_string(x, re.fixed, "FixedVersion", err);
          else if (json_key_eq(ek, "Affected")) ok = dec_ints(x, re.affected, "Entry.Affected", err);
          else if (json_key_eq(ek, "Arches")) ok = dec_strings(x, re.arches, "Arches", err);
          else if (json_key_eq(ek, "Status")) ok = dec_int(x, re.status, "Status", err);
          else if (json_key_eq(ek, "Cves")) {
            re.cves.clear();
            if (x.kind == JVal::Null) continue;
            if (x.kind != JVal::Arr) {
              err = std::string("json: cannot unmarshal ") + kind_name(x) + " into Go struct field Entry.Cves";
              return false;
            }
            for (const JVal& c : x.arr) {
              RhCve rc;
              if (c.kind != JVal::Null) {
                if (c.kind != JVal::Obj) {
                  err = std::string("json: cannot unmarshal ") + kind_name(c) + " into Go value of type redhatoval.CveEntry";
                  return false;
                }
                for (const auto& [ck, cx] : c.obj) {
                  if (json_key_eq(ck, "ID")) ok = dec_string(cx, rc.id, "ID", err);
                  else if (json_key_eq(ck, "Severity")) ok = dec_int(cx, rc.severity, "Severity", err);
                  if (!ok) return false;
                }
              }
              re.cves.push_back(std::move(rc));
            }
          }
          if (!ok) return false;
        }
      }
      out.push_back(std::move(re));
    }
  }
  return true;
}

bool decode_int_list(std::string_view text, std::vector<int64_t>& out) {
  JVal v;
  std::string err;
  if (!json_parse(text, v, err)) return false;
  return dec_ints(v, out, "[]int", err);
}

}  // namespace

bool decode_advisory(std::string_view json, Advisory& a, std::string& err) {
  JVal v;
  if (!json_parse(json, v, err)) return false;
  return decode_adv_value(v, a, err);
}

std::string extract_ksplice(std::string_view v) {
  std::string low(v);
  for (char& c : low)
    if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
  size_t b = 0;
  for (;;) {
    size_t e = low.find('.', b);
    std::string_view seg = std::string_view(low).substr(b, e == std::string::npos ? std::string::npos : e - b);
    if (seg.rfind("ksplice", 0) == 0) return std::string(seg);
    if (e == std::string::npos) return "";
    b = e + 1;
  }
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
  // Lookup-first drivers run vs.Get before parsing the installed version, so a poisoned
  // key fails the call even for an unparsable package (ubuntu.go:86-96, amazon.go:57-71,
  // alpine.go:88-97, wolfi.go:37-49); rpm versions never fail to parse.
  flags = PLAT_LOOKUP_FIRST;
  if (starts("debian ")) { drv = DRV_DEBIAN; cmp = CMP_DEB; flags = 0; return true; }
  if (starts("ubuntu ")) { drv = DRV_UBUNTU; cmp = CMP_DEB; return true; }
  if (starts("amazon linux ")) { drv = DRV_AMAZON; cmp = CMP_DEB; return true; }
  if (starts("alpine ")) { drv = DRV_ALPINE; cmp = CMP_APK; return true; }
  if (root == "wolfi") { drv = DRV_WOLFI; cmp = CMP_APK; return true; }
  if (root == "chainguard") { drv = DRV_CHAINGUARD; cmp = CMP_APK; return true; }
  if (root == "Red Hat") { drv = DRV_REDHAT; cmp = CMP_RPM; return true; }
  if (starts("alma ")) { drv = DRV_ALMA; cmp = CMP_RPM; return true; }
  if (starts("rocky ")) { drv = DRV_ROCKY; cmp = CMP_RPM; return true; }
  if (starts("Oracle Linux ")) { drv = DRV_ORACLE; cmp = CMP_RPM; return true; }
  if (starts("SUSE Linux Enterprise ") || starts("openSUSE Leap ")) { drv = DRV_SUSE; cmp = CMP_RPM; return true; }
  if (starts("Photon OS ")) { drv = DRV_PHOTON; cmp = CMP_RPM; return true; }
  if (starts("CBL-Mariner ")) { drv = DRV_MARINER; cmp = CMP_RPM; return true; }
  return false;
}

int32_t DB::find_plat(std::string_view root) const {
  auto it = plat_by_name_.find(std::string(root));
  return it == plat_by_name_.end() ? -1 : int32_t(it->second);
}

int32_t DB::find_key(uint32_t plat, std::string_view name) const {
  uint64_t h = pkg_key_hash(plat, reinterpret_cast<const uint8_t*>(name.data()), uint32_t(name.size()));
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

uint32_t DB::key_rows(uint32_t plat, std::string_view name) const {
  if (slot_hash.empty()) return 0;
  const uint64_t h = pkg_key_hash(plat, reinterpret_cast<const uint8_t*>(name.data()), uint32_t(name.size()));
  for (uint64_t i = h & slot_mask; slot_hash[i]; i = (i + 1) & slot_mask) {
    const SlotVal& v = slot_val[i];
    if (slot_hash[i] == h && (v.name_len & SLOT_LEN_MASK) == name.size() &&
        std::equal(name.begin(), name.end(), name_arena.begin() + v.name_off))
      return slot_rows(v.name_len, v.row_begin, v.row_count, 1).y;  // the full list
  }
  return 0;
}

std::vector<int64_t> DB::redhat_cpes(const std::vector<std::string_view>& repos,
                                     const std::vector<std::string_view>& nvrs) const {
  std::vector<int64_t> out;
  auto add = [&](const std::unordered_map<std::string, std::vector<int64_t>>& m, std::string_view k) {
    auto it = m.find(std::string(k));
    if (it == m.end()) return;
    for (int64_t c : it->second)
      if (std::find(out.begin(), out.end(), c) == out.end()) out.push_back(c);
  };
  for (std::string_view r : repos) add(rh_repo_, r);
  for (std::string_view n : nvrs) add(rh_nvr_, n);
  return out;
}

uint32_t DB::arch_id(std::string_view arch) const {
  auto it = arch_ids_.find(std::string(arch));
  return it == arch_ids_.end() ? PA_ARCH_NONE : it->second;
}

uint32_t DB::ksplice_id(std::string_view tag) const {
  if (tag.empty()) return 0;
  auto it = ksplice_ids_.find(std::string(tag));
  return it == ksplice_ids_.end() ? 0xFFFFFFFFu : it->second;
}

uint32_t DB::intern_arch(const std::string& a) {
  auto it = arch_ids_.find(a);
  if (it != arch_ids_.end()) return it->second;
  const uint32_t id = uint32_t(arch_ids_.size());
  arch_ids_.emplace(a, id);
  return id;
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

uint8_t ecosystem_grammar(std::string_view eco) {
  if (eco == "rubygems" || eco == "cocoapods") return CMP_GEM;
  if (eco == "maven") return CMP_MAVEN;
  if (eco == "npm") return CMP_NPM;
  if (eco == "pip") return CMP_PEP440;
  if (eco == "bitnami") return CMP_BITNAMI;
  if (eco == "cargo" || eco == "composer" || eco == "go" || eco == "nuget" || eco == "pub" || eco == "erlang" ||
      eco == "conan" || eco == "swift" || eco == "k8s")
    return CMP_GENERIC;
  return CMP_NONE;
}

std::string create_fixed_versions(const Advisory& a) {
  std::vector<std::string> out;
  auto add = [&](std::string v) {
    if (std::find(out.begin(), out.end(), v) == out.end()) out.push_back(std::move(v));
  };
  auto trim = [](std::string_view v) {
    const char* ws = " \t\n\v\f\r";
    const size_t b = v.find_first_not_of(ws);
    if (b == std::string_view::npos) return std::string();
    return std::string(v.substr(b, v.find_last_not_of(ws) - b + 1));
  };
  if (!a.patched.empty()) {
    for (const std::string& v : a.patched) add(v);
  } else {
    for (const std::string& v : a.vulnerable) {
      size_t b = 0;
      for (;;) {
        const size_t e = v.find(',', b);
        std::string s = trim(std::string_view(v).substr(b, e == std::string::npos ? std::string::npos : e - b));
        if (s.rfind("<=", 0) != 0 && s.rfind("<", 0) == 0) add(trim(std::string_view(s).substr(1)));
        if (e == std::string::npos) break;
        b = e + 1;
      }
    }
  }
  std::string j;
  for (size_t i = 0; i < out.size(); i++) j += (i ? ", " : "") + out[i];
  return j;
}

// trivy-db GetAdvisories("<eco>::", name): every root bucket with the prefix, in bbolt
// key order; a later root overwrites an earlier one's value for the same vulnID; then
// each value is decoded (a failure poisons the key: the reference fails the call only
// when a package looks it up, driver_test.go "malformed JSON").
void DB::flatten_library(uint32_t plat, const std::vector<std::pair<const Bucket*, int32_t>>& roots) {
  std::map<std::string, std::map<std::string, std::pair<const std::string*, int32_t>>> merged;
  for (const auto& [root, ds] : roots)
    for (const auto& [pkg, bkt] : root->sub)
      for (const auto& [vid, val] : bkt.kv)
        if (!val.empty()) merged[pkg][vid] = {&val, ds};
  for (const auto& [pkg, vals] : merged) {
    Key key;
    key.plat = plat;
    key.name = pkg;
    for (const auto& [vid, v] : vals) {
      const auto& [val, ds] = v;
      if (ds == -2) {  // the root's data-source entry does not decode
        if (!key.poisoned) key.err = "failed to get data source";
        key.poisoned = true;
        continue;
      }
      Advisory a;
      std::string err;
      if (!decode_advisory(*val, a, err)) {
        if (!key.poisoned) key.err = "failed to unmarshal advisory JSON: " + err;
        key.poisoned = true;
        continue;
      }
      a.vuln_id = vid;
      if (ds >= 0) {
        a.data_source = ds;
      } else if (a.has_inline_source) {
        sources.push_back(a.inline_source);
        a.data_source = int32_t(sources.size() - 1);
      }
      a.entries.clear();
      a.lib_fixed = create_fixed_versions(a);
      key.advs.push_back(uint32_t(advs.size()));
      advs.push_back(std::move(a));
    }
    if (key.poisoned) key.advs.clear();
    keys.push_back(std::move(key));
  }
}

void DB::flatten_os(uint32_t plat, const Bucket& root, int32_t ds) {
  const Platform& P = plats[plat];
  for (const auto& [pkg, bkt] : root.sub) {
    Key key;
    key.plat = plat;
    key.name = pkg;
    auto poison = [&](const std::string& e) {
      if (!key.poisoned) key.err = "failed to unmarshal advisory JSON: " + e;
      key.poisoned = true;
    };
    std::vector<Advisory> rh;  // Red Hat: the key's advisories in Get order, numbered below
    for (const auto& [vid, val] : bkt.kv) {
      std::string err;
      if (val.empty()) continue;  // trivy-db forEach skips empty values
      if (P.drv == DRV_REDHAT) {
        // trivy-db redhat-oval Get: one advisory per (entry, CVE); CPE filtering per package
        std::vector<RhEntry> ents;
        if (!decode_redhat(val, ents, err)) { poison(err); continue; }
        for (const RhEntry& e : ents) {
          for (const RhCve& c : e.cves) {
            Advisory a;
            a.severity = c.severity;
            a.fixed = e.fixed;
            a.arches = e.arches;
            a.status = e.status;
            a.cpes = e.affected;
            if (vid.rfind("CVE-", 0) == 0) {
              a.vuln_id = vid;
            } else {
              a.vuln_id = c.id;
              a.vendor_ids = {vid};
            }
            rh.push_back(std::move(a));
          }
        }
        continue;
      }
      Advisory a;
      if (!decode_advisory(val, a, err)) { poison(err); continue; }
      a.vuln_id = vid;
      // trivy-db GetAdvisories: the data-source bucket entry wins when non-empty,
      // otherwise the value's own DataSource (if any) stays.
      if (ds >= 0) {
        a.data_source = ds;
      } else if (a.has_inline_source) {
        sources.push_back(a.inline_source);
        a.data_source = int32_t(sources.size() - 1);
      }
      if (P.drv == DRV_ROCKY && !a.entries.empty()) {
        // trivy-db rocky Get(release, name, arch): one advisory per arch entry
        for (const Advisory& e : a.entries) {
          Advisory b = a;
          b.entries.clear();
          b.fixed = e.fixed;
          b.vendor_ids = e.vendor_ids;
          b.arches = e.arches;
          b.arch_entry = true;
          key.advs.push_back(uint32_t(advs.size()));
          advs.push_back(std::move(b));
        }
        continue;
      }
      a.entries.clear();
      key.advs.push_back(uint32_t(advs.size()));
      advs.push_back(std::move(a));
    }
    // Red Hat: numbered in (VulnerabilityID, Get order) order - a stable sort, so the
    // advisories of one CVE stay in Get order.  redhat.go:146-187 keys its merge by the ID
    // (first matched member in Get order wins, fixed members merge) and sorts the result
    // by ID, so this order changes nothing in the output; it makes a package's matches
    // arrive grouped by ID, and the batch merge (redhat.hip) a single pass without a sort.
    std::stable_sort(rh.begin(), rh.end(), [](const Advisory& x, const Advisory& y) { return x.vuln_id < y.vuln_id; });
    for (Advisory& a : rh) {
      key.advs.push_back(uint32_t(advs.size()));
      advs.push_back(std::move(a));
    }
    if (key.poisoned) key.advs.clear();
    keys.push_back(std::move(key));
  }
}

// The hi key's first bytes as the row's big-endian head words (zero padded): 24 for the
// dpkg grammar (Row::hi_pre2), else 16.
static void set_head(Row& r, const std::vector<uint8_t>& kb, bool h24) {
  uint64_t* w[3] = {&r.hi_pre0, &r.hi_pre1, &r.hi_pre2};
  for (size_t i = 0; i < kb.size() && i < (h24 ? 24u : 16u); i++) *w[i / 8] |= uint64_t(kb[i]) << (8 * (7 - i % 8));
}

// Advisory -> interval row(s) of its driver (SURVEY.md §8a' "unfixed" and parse-error
// columns).  Returns false when the advisory can never be reported (no row).
bool DB::compile_rows(const Platform& P, const Advisory& a, uint32_t ai, std::vector<uint8_t>& kb) {
  // Maven: ComparableVersion is not an order, so in general no interval set
  // can stand for IsVulnerable: the row carries the advisory's program (AUX_MVN) and the
  // kernel evaluates it pairwise against the installed version.  Hybrid: when every bound
  // text is numeric (libver.h mvn_numeric), every installed version compares with the
  // bounds in the order of its numeric projection (libver.h mvn_numeric_projection), so the
  // advisory is its key-order intervals below and no program.
  if (P.drv == DRV_LIBRARY && P.cmp == CMP_MAVEN) {
    std::vector<uint32_t> w;
    const MvnProgState st = mvn_program(a.vulnerable, a.patched, a.unaffected, w);
    if (st == MVN_NEVER) return false;
    if (st != MVN_PROGRAM || !mvn_hybrid(a.vulnerable, a.patched, a.unaffected)) {
      Row r{};
      r.lo_len = r.hi_len = KEY_INF;
      RowAux x{};
      r.adv = ai | (st == MVN_ALWAYS ? ROW_ALWAYS : ROW_FILTER);
      if (st == MVN_PROGRAM) {
        x.kind = AUX_MVN;
        x.list_off = uint32_t(aux_ids.size());
        aux_ids.insert(aux_ids.end(), w.begin(), w.end());
        has_filters = true;
      }
      rows.push_back(r);
      row_off.push_back(RowOff{});
      aux.push_back(x);
      return true;
    }
  }
  if (P.drv == DRV_LIBRARY) {
    // compare.IsVulnerable as disjoint intervals per version class (libdb.h); classes
    // sharing an interval share its row; a row that holds for a subset of the classes
    // carries an AUX_CLASS filter.
    LibRows lr = lib_compile_advisory(P.cmp, a.vulnerable, a.patched, a.unaffected);
    if (lr.always) {
      Row r{};
      r.adv = ai | ROW_ALWAYS;
      r.lo_len = r.hi_len = KEY_INF;
      rows.push_back(r);
      row_off.push_back(RowOff{});
      aux.push_back(RowAux{});
      return true;
    }
    std::vector<std::pair<KInterval, uint32_t>> ivs;  // interval -> class mask
    auto same = [](const KBound& x, const KBound& y) {
      return x.inf == y.inf && (x.inf || (x.k == y.k && x.incl == y.incl));
    };
    for (int c = 0; c < lr.ncls; c++)
      for (const KInterval& v : lr.cls[size_t(c)]) {
        bool found = false;
        for (auto& [w, mask] : ivs)
          if (same(w.lo, v.lo) && same(w.hi, v.hi)) {
            mask |= 1u << c;
            found = true;
          }
        if (!found) ivs.push_back({v, 1u << c});
      }
    const uint32_t all = (1u << lr.ncls) - 1;
    for (const auto& [v, mask] : ivs) {
      Row r{};
      RowOff o{};
      r.adv = ai;
      r.lo_len = r.hi_len = KEY_INF;
      auto put = [&](const KBound& b, uint32_t& off, uint16_t& len, bool hi) {
        if (b.inf) return;
        kb.assign(b.k.begin(), b.k.end());
        off = intern_key(kb);
        len = uint16_t(std::min<size_t>(kb.size(), KEY_LEN_MASK) | (b.incl ? KEY_INCL : 0));
        if (hi) set_head(r, kb, false);
      };
      put(v.lo, o.lo_off, r.lo_len, false);
      put(v.hi, o.hi_off, r.hi_len, true);
      RowAux x{};
      if (mask != all) {
        r.adv |= ROW_FILTER;
        x.kind = AUX_CLASS;
        x.tag = mask;
        has_filters = true;
      }
      r.off = o;  // library rows: 16-byte heads, offsets inline
      rows.push_back(r);
      row_off.push_back(o);
      aux.push_back(x);
    }
    return !ivs.empty();
  }
  Row r{};
  RowOff o{};
  r.adv = ai;
  r.lo_len = KEY_INF;
  r.hi_len = KEY_INF;
  auto encode = [&](const std::string& v, uint32_t& off, uint16_t& len) {
    kb.clear();
    VecSink s{&kb};
    if (!encode_version(P.cmp, reinterpret_cast<const uint8_t*>(v.data()), uint32_t(v.size()), s)) return false;
    off = intern_key(kb);
    len = uint16_t(kb.size());
    return true;
  };
  auto set_hi = [&](const std::string& v) {
    if (!encode(v, o.hi_off, r.hi_len)) return false;
    set_head(r, kb, P.cmp == CMP_DEB);
    return true;
  };
  RowAux x{};
  switch (P.drv) {
    case DRV_DEBIAN:
    case DRV_UBUNTU:
    case DRV_MARINER:
      // debian.go:99-102, ubuntu.go:110-113, mariner.go:62-66: unfixed is reported;
      // an unparsable fixed version skips the advisory
      if (!a.fixed.empty() && !set_hi(a.fixed)) return false;
      break;
    case DRV_AMAZON:
    case DRV_WOLFI:
    case DRV_CHAINGUARD:
      // amazon.go:73-77, wolfi.go:66-71: the fixed version must parse ("" does not for dpkg)
      if (!set_hi(a.fixed)) return false;
      break;
    case DRV_ALPINE:
      // alpine.go:122-153: installed >= AffectedVersion when set; unfixed reported
      if (!a.affected.empty()) {
        uint16_t l = 0;
        if (!encode(a.affected, o.lo_off, l)) return false;
        r.lo_len = uint16_t(l | KEY_INCL);
      }
      if (!a.fixed.empty() && !set_hi(a.fixed)) return false;
      break;
    case DRV_REDHAT:
      // redhat.go:146-180: unfixed (first one wins, merged on the host) or installed < fixed
      if (!a.fixed.empty()) set_hi(a.fixed);
      if (!a.arches.empty()) x.kind |= AUX_ARCH_RH;
      x.kind |= AUX_CPE;
      break;
    case DRV_ROCKY:
      set_hi(a.fixed);
      if (a.arch_entry) x.kind |= AUX_ARCH_IN;
      break;
    case DRV_ORACLE: {
      // oracle.go:65-69: skip unless the ksplice tags agree
      set_hi(a.fixed);
      x.kind |= AUX_TAG;
      const std::string t = extract_ksplice(a.fixed);
      if (t.empty()) {
        x.tag = 0;
      } else {
        auto it = ksplice_ids_.find(t);
        if (it == ksplice_ids_.end()) it = ksplice_ids_.emplace(t, uint32_t(ksplice_ids_.size() + 1)).first;
        x.tag = it->second;
      }
      break;
    }
    case DRV_ALMA:
    case DRV_SUSE:
    case DRV_PHOTON:
      set_hi(a.fixed);  // rpm never fails; "" parses to the smallest version
      break;
    default:
      return false;
  }
  if (r.hi_len != KEY_INF) r.hi_len = uint16_t(r.hi_len & KEY_LEN_MASK);
  if (x.kind) {
    r.adv |= ROW_FILTER;
    x.list_off = uint32_t(aux_ids.size());
    if (x.kind & (AUX_ARCH_RH | AUX_ARCH_IN)) {
      for (const std::string& s : a.arches) aux_ids.push_back(intern_arch(s));
      x.n_arch = uint16_t(a.arches.size());
    }
    if (x.kind & AUX_CPE) {
      for (int64_t c : a.cpes) {
        aux_ids.push_back(c < 0 || c >= int64_t(0xFFFFFFFF) ? 0xFFFFFFFFu : uint32_t(c));
        if (c >= 0 && c < int64_t(1) << 24) n_cpe = std::max<uint32_t>(n_cpe, uint32_t(c) + 1);
      }
      x.n_cpe = uint16_t(a.cpes.size());
    }
    has_filters = true;
    // an rpm row whose predicates fit carries them inline (common.h ROW_INLINE); its key
    // offsets stay in row_off only (it has no lower bound, and its upper bound's offset is
    // read there on a 16-byte head tie)
    const uint32_t na = x.n_arch, nc = x.n_cpe;
    bool fits = P.cmp == CMP_RPM && r.lo_len == KEY_INF && !(x.kind & ~uint32_t(AUX_ARCH_RH | AUX_ARCH_IN | AUX_CPE | AUX_TAG));
    if (fits && (x.kind & AUX_TAG)) fits = x.kind == AUX_TAG;
    if (fits && !(x.kind & AUX_TAG)) {
      fits = na + nc <= kInlineIds && na <= 3 && nc <= 3;
      for (uint32_t i = 0; fits && i < na + nc; i++) fits = aux_ids[x.list_off + i] < 0xFFFFu;
    }
    if (fits) {
      r.adv |= ROW_INLINE;
      r.lo_len = uint16_t(KEY_INF | x.kind | (na << 4) | (nc << 6));
      if (x.kind & AUX_TAG) {
        r.off.lo_off = x.tag;
        r.off.hi_off = 0;
      } else {
        uint16_t ids[kInlineIds] = {0xFFFF, 0xFFFF, 0xFFFF, 0xFFFF};
        for (uint32_t i = 0; i < na + nc; i++) ids[i] = uint16_t(aux_ids[x.list_off + i]);
        r.off.lo_off = uint32_t(ids[0]) | uint32_t(ids[1]) << 16;
        r.off.hi_off = uint32_t(ids[2]) | uint32_t(ids[3]) << 16;
      }
      rows.push_back(r);
      row_off.push_back(o);
      aux.push_back(x);
      return true;
    }
  }
  if (P.cmp != CMP_DEB) r.off = o;  // else Row::hi_pre2 holds key bytes 16..23
  rows.push_back(r);
  row_off.push_back(o);
  aux.push_back(x);
  return true;
}

// A library key whose rows differ by version class gets the class-0 list A in front of its
// full list B (common.h SLOT_CLS_SPLIT): A holds, in advisory order, the rows a class-0
// version can match - unfiltered rows and AUX_CLASS rows that admit class 0, their filter
// dropped - so the plain release versions (most installed packages) sweep no row of another
// class and load no RowAux.  Measured on C3's PEP 440 keys: 10.6 rows on average, ~half of
// them for other classes.
void DB::split_by_class(const Platform& P, uint32_t rb, uint32_t& cnt) {
  if (P.drv != DRV_LIBRARY || P.cmp == CMP_MAVEN || cnt == 0 || cnt >= 0x10000u) return;
  std::vector<uint32_t> a;
  for (uint32_t r = rb; r < rb + cnt; r++) {
    const bool filt = rows[r].adv & ROW_FILTER;
    if (!filt || (aux[r].kind == AUX_CLASS && (aux[r].tag & 1u))) a.push_back(r);
    else if (aux[r].kind != AUX_CLASS) return;  // another filter kind: no split
  }
  if (a.size() == cnt) return;  // every row admits class 0: one list
  std::vector<Row> rb_rows(rows.begin() + rb, rows.end());
  std::vector<RowOff> rb_off(row_off.begin() + rb, row_off.end());
  std::vector<RowAux> rb_aux(aux.begin() + rb, aux.end());
  rows.resize(rb);
  row_off.resize(rb);
  aux.resize(rb);
  for (uint32_t r : a) {
    Row x = rb_rows[r - rb];
    RowAux y = rb_aux[r - rb];
    if ((x.adv & ROW_FILTER) && y.kind == AUX_CLASS) {  // admits class 0: the filter always passes here
      x.adv &= ~ROW_FILTER;
      y = RowAux{};
    }
    rows.push_back(x);
    row_off.push_back(rb_off[r - rb]);
    aux.push_back(y);
  }
  rows.insert(rows.end(), rb_rows.begin(), rb_rows.end());
  row_off.insert(row_off.end(), rb_off.begin(), rb_off.end());
  aux.insert(aux.end(), rb_aux.begin(), rb_aux.end());
  cnt = uint32_t(a.size()) | (cnt << 16) | kRowSplit;
}

void DB::build_index() {
  // rows + key arena
  rows.clear();
  row_off.clear();
  aux.clear();
  aux_ids.clear();
  std::vector<uint8_t> kb;
  std::vector<uint32_t> row_begin(keys.size()), row_count(keys.size());
  for (size_t k = 0; k < keys.size(); k++) {
    const Key& key = keys[k];
    const Platform& P = plats[key.plat];
    // every key's rows start on a 128-byte line (4 rows): an L2 miss fetches whole 128-B lines
    // (profiles/r06/calib.txt), so a run of n rows costs ceil(n / 4) lines instead of up to one
    // more; the pad rows between runs are never swept
    while (rows.size() % kRowsPerLine) {
      Row pad{};
      pad.lo_len = pad.hi_len = KEY_INF;
      rows.push_back(pad);
      row_off.push_back(RowOff{});
      aux.push_back(RowAux{});
    }
    row_begin[k] = uint32_t(rows.size());
    for (uint32_t ai : key.advs) compile_rows(P, advs[ai], ai, kb);
    row_count[k] = uint32_t(rows.size()) - row_begin[k];
    split_by_class(P, row_begin[k], row_count[k]);
  }
  n_rows_total = rows.size();
  if (key_words.empty()) key_words.push_back(0);
  if (aux_ids.empty()) aux_ids.push_back(0);
  // CPE indices present only in the repository / nvr maps widen the bitset too
  for (const auto* m : {&rh_repo_, &rh_nvr_})
    for (const auto& [k, v] : *m)
      for (int64_t c : v)
        if (c >= 0 && c < int64_t(1) << 24) n_cpe = std::max<uint32_t>(n_cpe, uint32_t(c) + 1);

  // hash index, load factor <= 1/8 (TVM_SLOT_LOAD overrides it, for measurement).  Every extra
  // slot a probe walks is a dependent round trip, and absent names (a quarter of the synthetic
  // batches) walk to an empty slot: at most 1/2 (0.29 for C2's 150k keys) -> 1/8 took C2 0.410
  // -> 0.394 ms, C3 0.154 -> 0.142, C5 2.08 -> 1.85 (profiles/r06/slotload/); 3/4 cost C2 26 %.
  // The table is 64 B a slot: 134 MB for C2's keys, nothing next to 288 GB of HBM
  static const double max_load = [] {
    const char* v = std::getenv("TVM_SLOT_LOAD");
    const double x = v ? std::atof(v) : 0.125;
    return x > 0.01 && x < 0.95 ? x : 0.125;
  }();
  uint64_t cap = 16;
  while (double(cap) * max_load < double(keys.size())) cap <<= 1;
  slot_mask = cap - 1;
  slot_hash.assign(cap, 0);
  slot_val.assign(cap, SlotVal{});
  slot_key.assign(cap, 0);
  slots.assign(cap, Slot{});
  slot_fp.assign(cap, 0);
  name_arena.clear();
  for (size_t k = 0; k < keys.size(); k++) {
    const Key& key = keys[k];
    uint64_t h = pkg_key_hash(key.plat, reinterpret_cast<const uint8_t*>(key.name.data()), uint32_t(key.name.size()));
    uint64_t i = h & slot_mask;
    while (slot_hash[i]) i = (i + 1) & slot_mask;
    slot_hash[i] = h;
    slot_fp[i] = slot_fp_of(h);
    // which installed-version classes meet a Maven program row of the key (the probe packs a
    // Maven package's parse only for those)
    const bool split = (row_count[k] & kRowSplit) != 0;
    const uint32_t cnt = row_count[k] & ~kRowSplit;
    uint32_t mvn = 0;
    const uint2 full = slot_rows(split ? SLOT_CLS_SPLIT : 0u, row_begin[k], cnt, 1);  // list B
    for (uint32_t r = full.x; r < full.x + full.y; r++) {
      if (!(rows[r].adv & ROW_FILTER) || !(aux[r].kind & AUX_MVN)) continue;
      const uint32_t admits = (aux[r].kind & AUX_CLASS) ? aux[r].tag : ~0u;
      mvn |= ((admits & 1u) ? SLOT_MVN_C0 : 0u) | ((admits & 2u) ? SLOT_MVN_C1 : 0u);
    }
    SlotVal v;
    v.name_off = uint32_t(name_arena.size());
    v.name_len = uint32_t(key.name.size()) | (key.poisoned ? SLOT_POISONED : 0) | mvn | (split ? SLOT_CLS_SPLIT : 0u);
    v.row_begin = row_begin[k];
    v.row_count = cnt;
    slot_val[i] = v;
    slot_key[i] = uint32_t(k);
    Slot& sl = slots[i];
    sl.hash = h;
    sl.row_begin = v.row_begin;
    sl.row_count = v.row_count;
    sl.name_len = v.name_len;
    sl.name_off = v.name_off;
    for (size_t b = 0; b < key.name.size() && b < 8 * kSlotNameWords; b++)
      sl.name[b / 8] |= uint64_t(uint8_t(key.name[b])) << (8 * (b % 8));
    name_arena.insert(name_arena.end(), key.name.begin(), key.name.end());
    name_arena.resize((name_arena.size() + 7) & ~size_t(7), 0);  // 8-B aligned names, zero padded
  }
  // tail: the probe kernel loads kNameWords whole words from any name's start
  name_arena.resize(name_arena.size() + 8 * kNameWords, 0);

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
  // Red Hat CPE maps: "Red Hat CPE" -> "repository" | "nvr" -> key -> JSON []int
  auto cpe = root_.sub.find("Red Hat CPE");
  if (cpe != root_.sub.end()) {
    for (const auto& [sub, dst] : {std::pair<const char*, decltype(&rh_repo_)>{"repository", &rh_repo_},
                                   std::pair<const char*, decltype(&rh_repo_)>{"nvr", &rh_nvr_}}) {
      auto b = cpe->second.sub.find(sub);
      if (b == cpe->second.sub.end()) continue;
      for (const auto& [k, v] : b->second.kv) {
        std::vector<int64_t> ids;
        if (decode_int_list(v, ids)) (*dst)[k] = std::move(ids);
      }
    }
  }
  // library ecosystems: root buckets "<eco>::<source>" grouped by prefix
  std::map<std::string, std::vector<std::pair<const Bucket*, int32_t>>> eco_roots;
  for (const auto& [name, b] : root_.sub) {
    const size_t sep = name.find("::");
    if (sep == std::string::npos) continue;
    const std::string eco = name.substr(0, sep);
    if (ecosystem_grammar(eco) == CMP_NONE) continue;
    int32_t ds = -1;
    auto d = ds_of_root.find(name);
    if (d != ds_of_root.end() && !sources[size_t(d->second)].empty()) ds = d->second;
    if (ds_err.count(name)) ds = -2;
    eco_roots[eco + "::"].push_back({&b, ds});
  }
  for (const auto& [prefix, roots] : eco_roots) {
    const uint32_t pid = uint32_t(plats.size());
    plats.push_back(Platform{prefix, DRV_LIBRARY, ecosystem_grammar(prefix.substr(0, prefix.size() - 2)),
                             PLAT_LOOKUP_FIRST});
    plat_by_name_[prefix] = pid;
    flatten_library(pid, roots);
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
