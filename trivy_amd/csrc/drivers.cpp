// OS drivers (see drivers.h).  Field population per driver follows SURVEY.md §8a'.
#include "drivers.h"

#include <algorithm>
#include <cstdio>
#include <map>

#include "db.h"

namespace tvm {

std::string format_version(int64_t epoch, std::string_view version, std::string_view release) {
  std::string v(version);
  if (!release.empty()) {
    v += '-';
    v += release;
  }
  if (epoch != 0) v = std::to_string(epoch) + ":" + v;
  return v;
}

std::string os_major(std::string_view v) { return std::string(v.substr(0, v.find('.'))); }

std::string os_minor(std::string_view v) {
  size_t d = v.find('.');
  if (d == std::string_view::npos) return std::string(v);
  std::string_view rest = v.substr(d + 1);
  return std::string(v.substr(0, d)) + "." + std::string(rest.substr(0, rest.find('.')));
}

int64_t eol_unix(int y, int m, int d) {
  // days_from_civil (proleptic Gregorian), then 23:59:59 UTC
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  const int64_t days = era * 146097 + doe - 719468;
  return days * 86400 + 23 * 3600 + 59 * 60 + 59;
}

namespace {

const char* const kSeverity[] = {"UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"};

struct Eol {
  const char* ver;
  int y, m, d;
};

using EolMap = std::map<std::string, int64_t, std::less<>>;

EolMap make_eol(std::initializer_list<Eol> l) {
  EolMap m;
  for (const Eol& e : l) m[e.ver] = eol_unix(e.y, e.m, e.d);
  return m;
}

// osver.Supported (version.go:31-38): unknown versions count as supported.
bool supported(const EolMap& eol, std::string_view ver, int64_t now) {
  auto it = eol.find(ver);
  if (it == eol.end()) return true;
  return now < it->second;
}

// Runs the GPU match for one target: per package (name, version) or skipped.
struct Plan {
  int32_t plat = -1;
  HostBatch batch;
  void add(bool skip, std::string_view name, std::string_view ver) {
    batch.add(skip || plat < 0 ? 0xFFFFFFFFu : uint32_t(plat), name, ver);
  }
};

bool run_plan(Engine& eng, const Plan& plan, std::vector<uint2>& pairs, std::string& key_err, std::string& err) {
  int64_t err_pkg = -1;
  if (!eng.match_host(plan.batch, pairs, err_pkg, err)) return false;
  key_err.clear();
  if (err_pkg >= 0) {
    const uint4& d = plan.batch.desc[size_t(err_pkg)];
    std::string_view name(reinterpret_cast<const char*>(plan.batch.arena.data()) + d.y, d.w & 0xFFFF);
    int32_t k = eng.db().find_key(d.x, name);
    key_err = k >= 0 ? eng.db().keys[size_t(k)].err : "advisory decode error";
    if (key_err.empty()) key_err = "advisory decode error";
  }
  return true;
}

void fill_common(Vuln& v, const Advisory& a) {
  v.vuln_id = a.vuln_id;
  v.fixed = a.fixed;
  v.data_source = a.data_source;
  v.has_custom = !a.custom.empty();
  v.custom = a.custom;
}

// ---------------------------------------------------------------- debian.go ----------
class Debian : public OsDriver {
  EolMap eol_ = make_eol({{"1.1", 1997, 6, 5}, {"1.2", 1998, 6, 5}, {"1.3", 1999, 3, 9}, {"2.0", 2000, 3, 9},
                          {"2.1", 2000, 10, 30}, {"2.2", 2003, 7, 30}, {"3.0", 2006, 6, 30}, {"3.1", 2008, 3, 30},
                          {"4.0", 2010, 2, 15}, {"5.0", 2012, 2, 6}, {"6.0", 2016, 2, 29}, {"7", 2018, 5, 31},
                          {"8", 2020, 6, 30}, {"9", 2022, 6, 30}, {"10", 2024, 6, 30}, {"11", 2026, 8, 14},
                          {"12", 2028, 6, 10}, {"13", 3000, 1, 1}});

 public:
  bool detect(Engine& eng, std::string_view os_ver, const Repo*, const std::vector<Pkg>& pkgs, int64_t,
              std::vector<Vuln>& out, std::string& err) const override {
    const DB& db = eng.db();
    Plan plan;
    plan.plat = db.find_plat("debian " + os_major(os_ver));  // debian.go:60,72
    std::vector<std::string> src(pkgs.size());
    for (size_t i = 0; i < pkgs.size(); i++) {
      src[i] = format_version(pkgs[i].src_epoch, pkgs[i].src_version, pkgs[i].src_release);
      plan.add(false, pkgs[i].src_name, src[i]);
    }
    std::vector<uint2> pairs;
    std::string key_err;
    if (!run_plan(eng, plan, pairs, key_err, err)) return false;
    if (!key_err.empty()) {
      err = "failed to get debian advisories: " + key_err;  // debian.go:73-75
      return false;
    }
    for (const uint2& m : pairs) {
      const Pkg& p = pkgs[m.x];
      const Advisory& a = db.advs[m.y];
      Vuln v;
      v.pkg = m.x;
      v.copy = COPY_PKG_ID | COPY_PKG_NAME | COPY_IDENTIFIER | COPY_LAYER;
      fill_common(v, a);
      v.vendor_ids = a.vendor_ids;
      v.pkg_id = std::string(p.id);
      v.pkg_name = std::string(p.name);
      v.installed = format_version(p.epoch, p.version, p.release);
      v.status = int32_t(a.status);
      if (a.severity != 0) {  // debian.go:92-98 package-specific severity
        v.severity_source = "debian";
        v.severity = (a.severity > 0 && a.severity < 5) ? kSeverity[a.severity] : kSeverity[0];
      }
      out.push_back(std::move(v));
    }
    return true;
  }
  bool is_supported(std::string_view, std::string_view os_ver, int64_t now) const override {
    return supported(eol_, os_major(os_ver), now);
  }
};

// ---------------------------------------------------------------- ubuntu.go ----------
class Ubuntu : public OsDriver {
  EolMap eol_ = make_eol({{"4.10", 2006, 4, 30}, {"5.04", 2006, 10, 31}, {"5.10", 2007, 4, 13},
                          {"6.06", 2011, 6, 1}, {"6.10", 2008, 4, 25}, {"7.04", 2008, 10, 19},
                          {"7.10", 2009, 4, 18}, {"8.04", 2013, 5, 9}, {"8.10", 2010, 4, 30},
                          {"9.04", 2010, 10, 23}, {"9.10", 2011, 4, 29}, {"10.04", 2015, 4, 29},
                          {"10.10", 2012, 4, 10}, {"11.04", 2012, 10, 28}, {"11.10", 2013, 5, 9},
                          {"12.04", 2019, 4, 26}, {"12.04-ESM", 2019, 4, 28}, {"12.10", 2014, 5, 16},
                          {"13.04", 2014, 1, 27}, {"13.10", 2014, 7, 17}, {"14.04", 2022, 4, 25},
                          {"14.04-ESM", 2024, 4, 25}, {"14.10", 2015, 7, 23}, {"15.04", 2016, 1, 23},
                          {"15.10", 2016, 7, 22}, {"16.04", 2021, 4, 21}, {"16.04-ESM", 2026, 4, 29},
                          {"16.10", 2017, 7, 20}, {"17.04", 2018, 1, 13}, {"17.10", 2018, 7, 19},
                          {"18.04", 2023, 5, 31}, {"18.04-ESM", 2028, 3, 31}, {"18.10", 2019, 7, 18},
                          {"19.04", 2020, 1, 18}, {"19.10", 2020, 7, 17}, {"20.04", 2025, 4, 23},
                          {"20.10", 2021, 7, 22}, {"21.04", 2022, 1, 20}, {"21.10", 2022, 7, 14},
                          {"22.04", 2027, 4, 23}, {"22.10", 2023, 7, 20}, {"23.04", 2024, 1, 20}});

  // versionFromEolDates (ubuntu.go:136-151); the reference reads time.Now() here, we use `now`.
  std::string version_from_eol(std::string_view os_ver, int64_t now) const {
    if (eol_.count(os_ver)) return std::string(os_ver);
    std::string ver(os_ver);
    while (!ver.empty() && std::string_view("-ESM").find(ver.back()) != std::string_view::npos) ver.pop_back();  // TrimRight cutset
    auto it = eol_.find(ver);
    if (it != eol_.end() && now < it->second) return ver;
    return std::string(os_ver);
  }

 public:
  bool detect(Engine& eng, std::string_view os_ver, const Repo*, const std::vector<Pkg>& pkgs, int64_t now,
              std::vector<Vuln>& out, std::string& err) const override {
    const DB& db = eng.db();
    Plan plan;
    plan.plat = pkgs.empty() ? -1 : db.find_plat("ubuntu " + version_from_eol(os_ver, now));
    std::vector<std::string> src(pkgs.size());
    for (size_t i = 0; i < pkgs.size(); i++) {
      src[i] = format_version(pkgs[i].src_epoch, pkgs[i].src_version, pkgs[i].src_release);
      plan.add(false, pkgs[i].src_name, src[i]);
    }
    std::vector<uint2> pairs;
    std::string key_err;
    if (!run_plan(eng, plan, pairs, key_err, err)) return false;
    if (!key_err.empty()) {
      err = "failed to get Ubuntu advisories: " + key_err;  // ubuntu.go:87-90
      return false;
    }
    for (const uint2& m : pairs) {
      const Pkg& p = pkgs[m.x];
      const Advisory& a = db.advs[m.y];
      Vuln v;
      v.pkg = m.x;
      v.copy = COPY_PKG_ID | COPY_PKG_NAME | COPY_IDENTIFIER | COPY_LAYER;
      fill_common(v, a);
      v.pkg_id = std::string(p.id);
      v.pkg_name = std::string(p.name);
      v.installed = format_version(p.epoch, p.version, p.release);
      out.push_back(std::move(v));
    }
    return true;
  }
  bool is_supported(std::string_view, std::string_view os_ver, int64_t now) const override {
    return supported(eol_, os_ver, now);
  }
};

// ---------------------------------------------------------------- amazon.go ----------
class Amazon : public OsDriver {
  EolMap eol_ = make_eol({{"1", 2023, 12, 31}, {"2", 2025, 6, 30}, {"2023", 2028, 3, 15}});

  static std::string norm(std::string_view os_ver) {  // amazon.go:46-52
    size_t b = os_ver.find_first_not_of(" \t\n\v\f\r");
    std::string_view f = b == std::string_view::npos ? std::string_view() : os_ver.substr(b);
    f = f.substr(0, f.find_first_of(" \t\n\v\f\r"));
    std::string v = os_major(f);
    if (v != "2" && v != "2022" && v != "2023") v = "1";
    return v;
  }

 public:
  bool detect(Engine& eng, std::string_view os_ver, const Repo*, const std::vector<Pkg>& pkgs, int64_t,
              std::vector<Vuln>& out, std::string& err) const override {
    const DB& db = eng.db();
    Plan plan;
    plan.plat = db.find_plat("amazon linux " + norm(os_ver));
    std::vector<std::string> inst(pkgs.size());
    for (size_t i = 0; i < pkgs.size(); i++) {
      inst[i] = format_version(pkgs[i].epoch, pkgs[i].version, pkgs[i].release);
      plan.add(false, pkgs[i].name, inst[i]);
    }
    std::vector<uint2> pairs;
    std::string key_err;
    if (!run_plan(eng, plan, pairs, key_err, err)) return false;
    if (!key_err.empty()) {
      err = "failed to get amazon advisories: " + key_err;  // amazon.go:59-61
      return false;
    }
    for (const uint2& m : pairs) {
      const Pkg& p = pkgs[m.x];
      const Advisory& a = db.advs[m.y];
      Vuln v;
      v.pkg = m.x;
      v.copy = COPY_PKG_ID | COPY_PKG_NAME | COPY_IDENTIFIER | COPY_LAYER;
      fill_common(v, a);
      v.pkg_id = std::string(p.id);
      v.pkg_name = std::string(p.name);
      v.installed = inst[m.x];
      out.push_back(std::move(v));
    }
    return true;
  }
  bool is_supported(std::string_view, std::string_view os_ver, int64_t now) const override {
    return supported(eol_, norm(os_ver), now);
  }
};

}  // namespace

const OsDriver* find_os_driver(std::string_view family) {
  static const Debian debian;
  static const Ubuntu ubuntu;
  static const Amazon amazon;
  if (family == "debian") return &debian;
  if (family == "ubuntu") return &ubuntu;
  if (family == "amazon") return &amazon;
  return nullptr;
}

DetectStatus ospkg_detect(Engine& eng, std::string_view family, std::string_view os_name, const Repo* repo,
                          const std::vector<Pkg>& pkgs, int64_t now, std::vector<Vuln>& out, bool& eosl,
                          std::string& err) {
  const OsDriver* d = find_os_driver(family);
  if (!d) {
    err = "unsupported os";
    return DETECT_UNSUPPORTED_OS;
  }
  eosl = !d->is_supported(family, os_name, now);
  // gpg-pubkey doesn't carry a real version (detect.go:71-75)
  std::vector<Pkg> kept;
  std::vector<uint32_t> idx;
  kept.reserve(pkgs.size());
  for (size_t i = 0; i < pkgs.size(); i++) {
    if (pkgs[i].name == "gpg-pubkey") continue;
    kept.push_back(pkgs[i]);
    idx.push_back(uint32_t(i));
  }
  if (!d->detect(eng, os_name, repo, kept, now, out, err)) {
    err = "failed detection: " + err;
    out.clear();
    eosl = false;
    return DETECT_ERROR;
  }
  for (Vuln& v : out) v.pkg = idx[v.pkg];
  return DETECT_OK;
}

}  // namespace tvm
