// Load-time decode of trivy-db bucket "vulnerability" into the FillInfo device tables
// (vulninfo.h).  Host side only; the per-match decisions run in fill.hip.
#include "vulninfo.h"

#include <algorithm>
#include <map>

#include "common.h"
#include "db.h"
#include "json.h"

namespace tvm {

namespace {

const char* const kSeverityNames[5] = {"UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"};

// vulnerability.go:15-39 primaryURLPrefixes (keys: trivy-db vulnsrc/vulnerability IDs).
struct UrlPrefixes {
  const char* source;
  const char* prefixes[2];
};
const UrlPrefixes kPrimaryUrlPrefixes[] = {
    {"debian", {"http://www.debian.org", "https://www.debian.org"}},
    {"ubuntu", {"http://www.ubuntu.com", "https://usn.ubuntu.com"}},
    {"redhat", {"https://access.redhat.com", nullptr}},
    {"suse-cvrf", {"http://lists.opensuse.org", "https://lists.opensuse.org"}},
    {"oracle-oval", {"http://linux.oracle.com/errata", "https://linux.oracle.com/errata"}},
    {"nodejs-security-wg", {"https://www.npmjs.com", "https://hackerone.com"}},
    {"ruby-advisory-db", {"https://groups.google.com", nullptr}},
};

bool starts_with(std::string_view s, std::string_view p) { return s.size() >= p.size() && s.substr(0, p.size()) == p; }

// Primary-URL kind that comes from the ID alone (vulnerability.go:138-146), else URL_NONE.
uint32_t id_url_kind(std::string_view id) {
  if (starts_with(id, "CVE-")) return URL_CVE;
  if (starts_with(id, "RUSTSEC-")) return URL_RUSTSEC;
  if (starts_with(id, "GHSA-")) return URL_GHSA;
  if (starts_with(id, "TEMP-")) return URL_TEMP;
  return URL_NONE;
}

void json_quote(std::string& o, std::string_view s) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back(char(c));
    } else if (c < 0x20) {
      o += "\\u00";
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    } else {
      o.push_back(char(c));
    }
  }
  o.push_back('"');
}

// time.Time.UnmarshalJSON: RFC 3339 "YYYY-MM-DDTHH:MM:SS[.frac](Z|+hh:mm|-hh:mm)".
bool rfc3339(std::string_view s) {
  auto dig = [&](size_t i, size_t n) {
    if (i + n > s.size()) return false;
    for (size_t k = i; k < i + n; k++)
      if (s[k] < '0' || s[k] > '9') return false;
    return true;
  };
  if (!dig(0, 4) || s.size() < 20 || s[4] != '-' || !dig(5, 2) || s[7] != '-' || !dig(8, 2) || s[10] != 'T' ||
      !dig(11, 2) || s[13] != ':' || !dig(14, 2) || s[16] != ':' || !dig(17, 2))
    return false;
  size_t i = 19;
  if (i < s.size() && s[i] == '.') {
    size_t j = i + 1;
    while (j < s.size() && s[j] >= '0' && s[j] <= '9') j++;
    if (j == i + 1) return false;
    i = j;
  }
  if (i < s.size() && s[i] == 'Z') return i + 1 == s.size();
  return i + 6 == s.size() && (s[i] == '+' || s[i] == '-') && dig(i + 1, 2) && s[i + 3] == ':' && dig(i + 4, 2);
}

bool dec_str(const JVal& x, std::string& out) {
  if (x.kind == JVal::Null) return true;  // null leaves the field unchanged
  if (x.kind != JVal::Str) return false;
  out = x.s;
  return true;
}

bool dec_strs(const JVal& x, std::vector<std::string>& out) {
  if (x.kind == JVal::Null) {
    out.clear();
    return true;
  }
  if (x.kind != JVal::Arr) return false;
  out.clear();
  for (const JVal& e : x.arr) {
    if (e.kind == JVal::Null) out.emplace_back();
    else if (e.kind == JVal::Str) out.push_back(e.s);
    else return false;
  }
  return true;
}

struct Cvss {
  std::string v2v, v3v, v2s, v3s;  // scores: JSON number literal text ("" = zero)
};

// One decoded trivy-db types.Vulnerability (json.Unmarshal semantics: ASCII
// case-insensitive field names, later duplicates win, maps merge, unknown fields ignored,
// any type mismatch makes the whole decode an error).
struct Decoded {
  std::string title, description, severity, published, last_modified, custom;
  std::vector<std::string> cwe, refs;
  bool has_cwe = false, has_refs = false, has_vendor = false, has_cvss = false;
  std::map<std::string, int64_t> vendor;
  std::map<std::string, Cvss> cvss;
};

bool decode_vuln(std::string_view text, Decoded& d) {
  JVal v;
  std::string e;
  if (!json_parse(text, v, e)) return false;
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Obj) return false;
  for (const auto& [k, x] : v.obj) {
    if (json_key_eq(k, "Title")) {
      if (!dec_str(x, d.title)) return false;
    } else if (json_key_eq(k, "Description")) {
      if (!dec_str(x, d.description)) return false;
    } else if (json_key_eq(k, "Severity")) {
      if (!dec_str(x, d.severity)) return false;
    } else if (json_key_eq(k, "CweIDs")) {
      if (!dec_strs(x, d.cwe)) return false;
      d.has_cwe = x.kind != JVal::Null;
    } else if (json_key_eq(k, "References")) {
      if (!dec_strs(x, d.refs)) return false;
      d.has_refs = x.kind != JVal::Null;
    } else if (json_key_eq(k, "VendorSeverity")) {
      if (x.kind == JVal::Null) {
        d.vendor.clear();
        d.has_vendor = false;
        continue;
      }
      if (x.kind != JVal::Obj) return false;
      d.has_vendor = true;
      for (const auto& [src, sv] : x.obj) {
        int64_t s = 0;
        if (sv.kind != JVal::Null && !json_int(sv, s)) return false;
        d.vendor[src] = s;
      }
    } else if (json_key_eq(k, "CVSS")) {
      if (x.kind == JVal::Null) {
        d.cvss.clear();
        d.has_cvss = false;
        continue;
      }
      if (x.kind != JVal::Obj) return false;
      d.has_cvss = true;
      for (const auto& [src, cv] : x.obj) {
        Cvss& c = d.cvss[src];
        if (cv.kind == JVal::Null) continue;
        if (cv.kind != JVal::Obj) return false;
        for (const auto& [f, fv] : cv.obj) {
          if (json_key_eq(f, "V2Vector")) {
            if (!dec_str(fv, c.v2v)) return false;
          } else if (json_key_eq(f, "V3Vector")) {
            if (!dec_str(fv, c.v3v)) return false;
          } else if (json_key_eq(f, "V2Score") || json_key_eq(f, "V3Score")) {
            if (fv.kind == JVal::Null) continue;
            if (fv.kind != JVal::Num) return false;
            (json_key_eq(f, "V2Score") ? c.v2s : c.v3s) = fv.s;
          }
        }
      }
    } else if (json_key_eq(k, "PublishedDate") || json_key_eq(k, "LastModifiedDate")) {
      std::string& dst = json_key_eq(k, "PublishedDate") ? d.published : d.last_modified;
      if (x.kind == JVal::Null) {
        dst.clear();
        continue;
      }
      if (x.kind != JVal::Str || !rfc3339(x.s)) return false;
      dst = x.s;
    } else if (json_key_eq(k, "Custom")) {
      d.custom = x.kind == JVal::Null ? std::string() : std::string(x.raw);
    }
  }
  return true;
}

bool zero_num(const std::string& lit) {
  if (lit.empty()) return true;
  for (char c : lit) {
    if (c == 'e' || c == 'E') break;
    if (c >= '1' && c <= '9') return false;
  }
  return true;
}

// The record's fields other than Severity/VendorSeverity as JSON members (omitempty),
// in types.Vulnerability field order.
std::string rest_members(const Decoded& d) {
  std::string o;
  auto sep = [&] {
    if (!o.empty()) o.push_back(',');
  };
  auto str_field = [&](const char* name, const std::string& v) {
    if (v.empty()) return;
    sep();
    json_quote(o, name);
    o.push_back(':');
    json_quote(o, v);
  };
  auto strs_field = [&](const char* name, const std::vector<std::string>& v) {
    if (v.empty()) return;
    sep();
    json_quote(o, name);
    o += ":[";
    for (size_t i = 0; i < v.size(); i++) {
      if (i) o.push_back(',');
      json_quote(o, v[i]);
    }
    o.push_back(']');
  };
  str_field("Title", d.title);
  str_field("Description", d.description);
  strs_field("CweIDs", d.cwe);
  if (!d.cvss.empty()) {
    sep();
    o += "\"CVSS\":{";
    bool first = true;
    for (const auto& [src, c] : d.cvss) {
      if (!first) o.push_back(',');
      first = false;
      json_quote(o, src);
      o += ":{";
      std::string m;
      auto add = [&](const char* n, const std::string& v, bool num) {
        if (num ? zero_num(v) : v.empty()) return;
        if (!m.empty()) m.push_back(',');
        json_quote(m, n);
        m.push_back(':');
        if (num) m += v;
        else json_quote(m, v);
      };
      add("V2Vector", c.v2v, false);
      add("V3Vector", c.v3v, false);
      add("V2Score", c.v2s, true);
      add("V3Score", c.v3s, true);
      o += m;
      o.push_back('}');
    }
    o.push_back('}');
  }
  strs_field("References", d.refs);
  str_field("PublishedDate", d.published);
  str_field("LastModifiedDate", d.last_modified);
  if (!d.custom.empty()) {
    sep();
    o += "\"Custom\":";
    o += d.custom;
  }
  return o;
}

}  // namespace

const char* fill_severity_name(int64_t s) { return (s >= 0 && s < 5) ? kSeverityNames[s] : kSeverityNames[0]; }

int64_t fill_new_severity(std::string_view s) {
  for (int i = 0; i < 5; i++)
    if (s == kSeverityNames[i]) return i;
  return 0;  // NewSeverity: SeverityUnknown (with an error FillInfo ignores, vulnerability.go:98)
}

uint32_t VulnTable::intern_source(const std::string& s) {
  auto it = src_ids_.find(s);
  if (it != src_ids_.end()) return it->second;
  const uint32_t id = uint32_t(src_names_.size());
  src_names_.push_back(s);
  src_ids_.emplace(s, id);
  return id;
}

uint32_t VulnTable::source_id(std::string_view s) const {
  auto it = src_ids_.find(std::string(s));
  return it == src_ids_.end() ? SRC_NONE : it->second;
}

uint32_t VulnTable::vuln_rank(std::string_view id) const {
  auto it = vuln_rank_.find(id);
  return it == vuln_rank_.end() ? 0xFFFFFFFFu : it->second;
}

int32_t VulnTable::find(std::string_view id) const {
  auto it = by_id_.find(id);
  return it == by_id_.end() ? -1 : it->second;
}

void VulnTable::build(const DB& db) {
  vulns.clear();
  by_id_.clear();
  src_ids_.clear();
  src_names_.clear();
  for (const auto& p : kPrimaryUrlPrefixes) intern_source(p.source);
  ghsa_ = intern_source("ghsa");
  nvd_ = intern_source("nvd");
  for (const auto& s : db.sources) intern_source(s.id);

  const auto& tree = db.tree();
  auto vb = tree.sub.find("vulnerability");
  std::vector<std::vector<uint32_t>> ents_of;
  if (vb != tree.sub.end()) {
    vulns.reserve(vb->second.kv.size());
    for (const auto& [id, text] : vb->second.kv) {
      VulnDetail v;
      v.id = id;
      Decoded d;
      if (!decode_vuln(text, d)) {
        v.bad = true;
      } else {
        v.severity = d.severity;
        v.vendor.assign(d.vendor.begin(), d.vendor.end());
        v.refs = d.refs;
        v.detail_json = rest_members(d);
      }
      vulns.push_back(std::move(v));
    }
  }
  // entries: VendorSeverity pairs, then primary-URL reference picks per source
  recs.assign(vulns.size(), make_uint4(0, 0, 0, 0));
  ents.clear();
  for (size_t i = 0; i < vulns.size(); i++) {
    VulnDetail& v = vulns[i];
    by_id_.emplace(std::string_view(v.id), int32_t(i));
    const uint32_t url_kind = id_url_kind(v.id);
    uint4 r = make_uint4(uint32_t(ents.size()), 0, 0, (v.bad ? REC_BAD : 0u) | (url_kind << REC_URL_SHIFT));
    if (!v.bad) {
      for (const auto& [src, s] : v.vendor) {
        const uint32_t sid = intern_source(src);
        const uint32_t val = (s >= 0 && s < 5) ? uint32_t(s) : SEV_OOR;
        ents.push_back((sid << 16) | val);
      }
      if (url_kind == URL_NONE) {
        for (const auto& p : kPrimaryUrlPrefixes) {
          int32_t pick = -1;
          for (const char* pre : p.prefixes) {
            if (!pre || pick >= 0) continue;
            for (size_t k = 0; k < v.refs.size() && pick < 0; k++)
              if (starts_with(v.refs[k], pre)) pick = int32_t(k);
          }
          if (pick >= 0) ents.push_back(ENT_URL | (source_id(p.source) << 16) | std::min<uint32_t>(pick, 0xFFFF));
        }
      }
      r.y = uint32_t(ents.size()) - r.x;
      int64_t code = SEV_RAW;
      if (v.severity.empty()) code = 0;  // getVendorSeverity: "" -> UNKNOWN (vulnerability.go:129-131)
      for (int s = 0; s < 5 && code == SEV_RAW; s++)
        if (v.severity == kSeverityNames[s]) code = s;
      r.z = uint32_t(code);
    }
    recs[i] = r;
  }
  // hash index on the vulnerability ID (load <= 0.5, linear probing)
  uint64_t cap = 16;
  while (cap < 2 * std::max<size_t>(vulns.size(), 1)) cap <<= 1;
  slot_mask = cap - 1;
  slot_hash.assign(cap, 0);
  slot_val.assign(cap, make_uint4(0, 0, 0, 0));
  id_arena.clear();
  for (size_t i = 0; i < vulns.size(); i++) {
    const std::string& id = vulns[i].id;
    const uint32_t off = uint32_t(id_arena.size());
    id_arena.insert(id_arena.end(), id.begin(), id.end());
    id_arena.resize((id_arena.size() + 7) & ~size_t(7), 0);
    const uint64_t h = key_hash(kVulnSeed, reinterpret_cast<const uint8_t*>(id.data()), uint32_t(id.size()));
    uint64_t s = h & slot_mask;
    while (slot_hash[s] != 0) s = (s + 1) & slot_mask;
    slot_hash[s] = h;
    slot_val[s] = make_uint4(off, uint32_t(id.size()), uint32_t(i), 0);
  }
  id_arena.resize(id_arena.size() + 8 * kNameWords, 0);

  // batch path: the FillInfo input of every advisory's detector output
  adv_items.assign(db.advs.size(), make_uint4(0, (SRC_NONE << 16) | 0xFFu, 0, FILL_NOT_FOUND));
  std::vector<std::string> fixed_out(db.advs.size());
  for (const Key& k : db.keys) {
    const uint8_t drv = db.plats[k.plat].drv;
    for (uint32_t ai : k.advs) {
      const Advisory& a = db.advs[ai];
      DetFill f;
      detector_fill_fields(drv, a, f);
      uint32_t src = SRC_NONE;
      if (f.data_source >= 0) src = source_id(db.sources[size_t(f.data_source)].id);
      else src = source_id("");
      const int32_t rec = find(a.vuln_id);
      uint4 it;
      it.x = 0;
      it.y = (src << 16) | (f.severity ? uint32_t(fill_new_severity(f.severity)) : 0xFFu);
      it.z = uint32_t(f.status & 0xFF) | (f.fixed ? FI_FIXED : 0u) | (f.severity_source ? FI_SEV_SRC : 0u);
      it.w = (rec >= 0 && !vulns[size_t(rec)].bad) ? uint32_t(rec) : FILL_NOT_FOUND;
      adv_items[ai] = it;
      fixed_out[ai] = std::move(f.fixed_version);
    }
  }
  // ranks for the batch filter: vulnerability IDs and output FixedVersions in byte order
  {
    std::vector<std::string_view> ids, fx;
    ids.reserve(db.advs.size());
    for (const Advisory& a : db.advs) ids.push_back(a.vuln_id);
    for (const std::string& f : fixed_out) fx.push_back(f);
    auto rank_of = [](std::vector<std::string_view> v) {
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
      return v;
    };
    const auto uid = rank_of(ids), ufx = rank_of(fx);
    vuln_rank_.clear();
    rank_names_.clear();
    rank_names_.reserve(uid.size());  // no reallocation below: the map's views stay valid
    for (size_t i = 0; i < uid.size(); i++) {
      rank_names_.emplace_back(uid[i]);
      vuln_rank_.emplace(std::string_view(rank_names_.back()), uint32_t(i));
    }
    adv_rank.assign(db.advs.size(), make_uint2(0, 0));
    for (size_t i = 0; i < db.advs.size(); i++) {
      adv_rank[i].x = uint32_t(std::lower_bound(uid.begin(), uid.end(), ids[i]) - uid.begin());
      adv_rank[i].y = uint32_t(std::lower_bound(ufx.begin(), ufx.end(), std::string_view(fixed_out[i])) - ufx.begin());
    }
  }
  built_ = true;
}

std::string VulnTable::vulnerability_json(uint32_t rec, std::string_view severity, std::string_view extra_src,
                                         int64_t extra_val) const {
  const VulnDetail& v = vulns[rec];
  std::map<std::string, int64_t> vendor(v.vendor.begin(), v.vendor.end());
  if (!extra_src.empty()) vendor[std::string(extra_src)] = extra_val;
  std::string o = "{";
  if (!severity.empty()) {
    o += "\"Severity\":";
    json_quote(o, severity);
  }
  if (!vendor.empty()) {
    if (o.size() > 1) o.push_back(',');
    o += "\"VendorSeverity\":{";
    bool first = true;
    for (const auto& [k, x] : vendor) {
      if (!first) o.push_back(',');
      first = false;
      json_quote(o, k);
      o.push_back(':');
      o += std::to_string(x);
    }
    o.push_back('}');
  }
  if (!v.detail_json.empty()) {
    if (o.size() > 1) o.push_back(',');
    o += v.detail_json;
  }
  o.push_back('}');
  return o;
}

std::string VulnTable::primary_url(uint32_t rec, uint32_t url_word) const {
  const VulnDetail& v = vulns[rec];
  switch (url_word >> URL_KIND_SHIFT) {
    case URL_CVE: {
      std::string lower = v.id;
      for (char& c : lower)
        if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');  // strings.ToLower (IDs are ASCII)
      return "https://avd.aquasec.com/nvd/" + lower;
    }
    case URL_RUSTSEC:
      return "https://osv.dev/vulnerability/" + v.id;
    case URL_GHSA:
      return "https://github.com/advisories/" + v.id;
    case URL_TEMP:
      return "https://security-tracker.debian.org/tracker/" + v.id;
    case URL_REF: {
      const uint32_t k = url_word & URL_REF_MASK;
      return k < v.refs.size() ? v.refs[k] : std::string();
    }
    default:
      return std::string();
  }
}

const std::string& VulnTable::severity_string(uint32_t rec, uint32_t code) const {
  static const std::string names[5] = {"UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"};
  if (code < 5) return names[code];
  if (code == SEV_RAW) return vulns[rec].severity;
  return names[0];  // SEV_OOR: Severity.String() of an out-of-range value (unpinned; Go panics)
}

}  // namespace tvm
