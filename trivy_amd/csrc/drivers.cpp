// OS drivers (see drivers.h).  Field population per driver follows SURVEY.md §8a'.
//
// Each driver keeps the reference's per-target prologue (which root bucket, which name,
// which formatted version, which packages are skipped before the lookup) and epilogue
// (which DetectedVulnerability fields are set, Red Hat's per-CVE merge).  The
// per-(package, advisory) loop runs in one GPU launch per call (Engine::match_host).
#include "drivers.h"
#include "redhat.h"
#include "vulninfo.h"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <map>

#include "db.h"
#include "verkey.h"

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
const char* severity_name(int64_t s) { return (s >= 0 && s < 5) ? kSeverity[s] : kSeverity[0]; }

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

// ---- eolDates of each driver (<os>/<os>.go; transcribed data) ----------------------------
const EolMap& debian_eol() {
  static const EolMap m = make_eol(
      {{"1.1", 1997, 6, 5}, {"1.2", 1998, 6, 5}, {"1.3", 1999, 3, 9}, {"2.0", 2000, 3, 9}, {"2.1", 2000, 10, 30},
       {"2.2", 2003, 7, 30}, {"3.0", 2006, 6, 30}, {"3.1", 2008, 3, 30}, {"4.0", 2010, 2, 15}, {"5.0", 2012, 2, 6},
       {"6.0", 2016, 2, 29}, {"7", 2018, 5, 31}, {"8", 2020, 6, 30}, {"9", 2022, 6, 30}, {"10", 2024, 6, 30},
       {"11", 2026, 8, 14}, {"12", 2028, 6, 10}, {"13", 3000, 1, 1}});
  return m;
}
const EolMap& ubuntu_eol() {
  static const EolMap m = make_eol(
      {{"4.10", 2006, 4, 30}, {"5.04", 2006, 10, 31}, {"5.10", 2007, 4, 13}, {"6.06", 2011, 6, 1},
       {"6.10", 2008, 4, 25}, {"7.04", 2008, 10, 19}, {"7.10", 2009, 4, 18}, {"8.04", 2013, 5, 9},
       {"8.10", 2010, 4, 30}, {"9.04", 2010, 10, 23}, {"9.10", 2011, 4, 29}, {"10.04", 2015, 4, 29},
       {"10.10", 2012, 4, 10}, {"11.04", 2012, 10, 28}, {"11.10", 2013, 5, 9}, {"12.04", 2019, 4, 26},
       {"12.04-ESM", 2019, 4, 28}, {"12.10", 2014, 5, 16}, {"13.04", 2014, 1, 27}, {"13.10", 2014, 7, 17},
       {"14.04", 2022, 4, 25}, {"14.04-ESM", 2024, 4, 25}, {"14.10", 2015, 7, 23}, {"15.04", 2016, 1, 23},
       {"15.10", 2016, 7, 22}, {"16.04", 2021, 4, 21}, {"16.04-ESM", 2026, 4, 29}, {"16.10", 2017, 7, 20},
       {"17.04", 2018, 1, 13}, {"17.10", 2018, 7, 19}, {"18.04", 2023, 5, 31}, {"18.04-ESM", 2028, 3, 31},
       {"18.10", 2019, 7, 18}, {"19.04", 2020, 1, 18}, {"19.10", 2020, 7, 17}, {"20.04", 2025, 4, 23},
       {"20.10", 2021, 7, 22}, {"21.04", 2022, 1, 20}, {"21.10", 2022, 7, 14}, {"22.04", 2027, 4, 23},
       {"22.10", 2023, 7, 20}, {"23.04", 2024, 1, 20}});
  return m;
}
const EolMap& alpine_eol() {
  static const EolMap m = [] {
    EolMap t = make_eol(
        {{"2.0", 2012, 4, 1}, {"2.1", 2012, 11, 1}, {"2.2", 2013, 5, 1}, {"2.3", 2013, 11, 1}, {"2.4", 2014, 5, 1},
         {"2.5", 2014, 11, 1}, {"2.6", 2015, 5, 1}, {"2.7", 2015, 11, 1}, {"3.0", 2016, 5, 1}, {"3.1", 2016, 11, 1},
         {"3.2", 2017, 5, 1}, {"3.3", 2017, 11, 1}, {"3.4", 2018, 5, 1}, {"3.5", 2018, 11, 1}, {"3.6", 2019, 5, 1},
         {"3.7", 2019, 11, 1}, {"3.8", 2020, 5, 1}, {"3.9", 2020, 11, 1}, {"3.10", 2021, 5, 1},
         {"3.11", 2021, 11, 1}, {"3.12", 2022, 5, 1}, {"3.13", 2022, 11, 1}, {"3.14", 2023, 5, 1},
         {"3.15", 2023, 11, 1}, {"3.16", 2024, 5, 23}, {"3.17", 2024, 11, 22}, {"3.18", 2025, 5, 9},
         {"3.19", 2025, 11, 1}});
    t["edge"] = eol_unix(9999, 1, 1) - (23 * 3600 + 59 * 60 + 59);  // time.Date(9999,1,1,0,0,0)
    return t;
  }();
  return m;
}
const EolMap& amazon_eol() {
  static const EolMap m = make_eol({{"1", 2023, 12, 31}, {"2", 2025, 6, 30}, {"2023", 2028, 3, 15}});
  return m;
}
const EolMap& redhat_eol() {
  static const EolMap m = make_eol({{"4", 2017, 5, 31}, {"5", 2020, 11, 30}, {"6", 2024, 6, 30},
                                    {"7", 3000, 1, 1}, {"8", 3000, 1, 1}, {"9", 3000, 1, 1}});
  return m;
}
const EolMap& centos_eol() {
  static const EolMap m = make_eol({{"3", 2010, 10, 31}, {"4", 2012, 2, 29}, {"5", 2017, 3, 31},
                                    {"6", 2020, 11, 30}, {"7", 2024, 6, 30}, {"8", 2021, 12, 31}});
  return m;
}
const EolMap& alma_eol() {
  static const EolMap m = make_eol({{"8", 2029, 3, 1}, {"9", 2032, 5, 31}});
  return m;
}
const EolMap& rocky_eol() {
  static const EolMap m = make_eol({{"8", 2029, 5, 31}, {"9", 2032, 5, 31}});
  return m;
}
const EolMap& oracle_eol() {
  static const EolMap m = make_eol({{"3", 2011, 12, 31}, {"4", 2013, 12, 31}, {"5", 2017, 12, 31},
                                    {"6", 2021, 3, 21}, {"7", 2024, 7, 23}, {"8", 2029, 7, 18}, {"9", 2032, 7, 18}});
  return m;
}
const EolMap& photon_eol() {
  static const EolMap m =
      make_eol({{"1.0", 2022, 2, 28}, {"2.0", 2022, 12, 31}, {"3.0", 2024, 6, 30}, {"4.0", 2025, 12, 31}});
  return m;
}
const EolMap& sles_eol() {
  static const EolMap m = make_eol(
      {{"10", 2007, 12, 31}, {"10.1", 2008, 11, 30}, {"10.2", 2010, 4, 11}, {"10.3", 2011, 10, 11},
       {"10.4", 2013, 7, 31}, {"11", 2010, 12, 31}, {"11.1", 2012, 8, 31}, {"11.2", 2014, 1, 31},
       {"11.3", 2016, 1, 31}, {"11.4", 2019, 3, 31}, {"12", 2016, 6, 30}, {"12.1", 2017, 5, 31},
       {"12.2", 2018, 3, 31}, {"12.3", 2019, 1, 30}, {"12.4", 2020, 6, 30}, {"12.5", 2024, 10, 31},
       {"15", 2019, 12, 31}, {"15.1", 2021, 1, 31}, {"15.2", 2021, 12, 31}, {"15.3", 2022, 12, 31},
       {"15.4", 2023, 12, 31}, {"15.5", 2028, 12, 31}});
  return m;
}
const EolMap& opensuse_eol() {
  static const EolMap m = make_eol(
      {{"42.1", 2017, 5, 17}, {"42.2", 2018, 1, 26}, {"42.3", 2019, 6, 30}, {"15.0", 2019, 12, 3},
       {"15.1", 2020, 11, 30}, {"15.2", 2021, 11, 30}, {"15.3", 2022, 11, 30}, {"15.4", 2023, 11, 30},
       {"15.5", 2024, 12, 31}});
  return m;
}

// amazon.go:46-52: first field, major, anything but 2/2022/2023 is "1"
std::string amazon_release(std::string_view os_ver) {
  size_t b = os_ver.find_first_not_of(" \t\n\v\f\r");
  std::string_view f = b == std::string_view::npos ? std::string_view() : os_ver.substr(b);
  f = f.substr(0, f.find_first_of(" \t\n\v\f\r"));
  std::string v = os_major(f);
  if (v != "2" && v != "2022" && v != "2023") v = "1";
  return v;
}

// ubuntu.go:136-151 versionFromEolDates (the reference reads time.Now(); we use `now`)
std::string ubuntu_release(std::string_view os_ver, int64_t now) {
  const EolMap& eol = ubuntu_eol();
  if (eol.count(os_ver)) return std::string(os_ver);
  std::string ver(os_ver);
  while (!ver.empty() && std::string_view("-ESM").find(ver.back()) != std::string_view::npos) ver.pop_back();
  auto it = eol.find(ver);
  if (it != eol.end() && now < it->second) return ver;
  return std::string(os_ver);
}

// alpine.go:155-169 repoRelease + the stream choice of Detect (alpine.go:67-83)
std::string alpine_stream(std::string_view os_ver, const Repo* repo) {
  std::string v = os_minor(os_ver);
  std::string rr;
  if (repo) {
    rr = std::string(repo->release);
    if (std::count(rr.begin(), rr.end(), '.') > 1) rr = rr.substr(0, rr.rfind('.'));
  }
  return (!rr.empty() && v != rr) ? rr : v;
}

// redhat.go:207-220 addModularNamespace
std::string modular_name(std::string_view name, std::string_view label) {
  int count = 0;
  for (size_t i = 0; i < label.size(); i++) {
    if (label[i] == ':') count++;
    if (count == 2) return std::string(label.substr(0, i)) + "::" + std::string(name);
  }
  return std::string(name);
}

// go-rpm-version Version.String(): epoch dropped unless positive
std::string rpm_string(std::string_view v) {
  int64_t epoch = 0;
  std::string_view rest = v;
  size_t c = v.find(':');
  if (c != std::string_view::npos) {
    std::string_view e = v.substr(0, c);
    size_t i = 0;
    bool neg = false, ok = !e.empty();
    if (!e.empty() && (e[0] == '+' || e[0] == '-')) {
      neg = e[0] == '-';
      i = 1;
      ok = e.size() > 1;
    }
    uint64_t x = 0;
    for (; ok && i < e.size(); i++) {
      if (e[i] < '0' || e[i] > '9') { ok = false; break; }
      const uint64_t d = uint64_t(e[i] - '0');
      if (x > (uint64_t(INT64_MAX) - d) / 10) { ok = false; break; }
      x = x * 10 + d;
    }
    epoch = ok ? (neg ? -int64_t(x) : int64_t(x)) : 0;
    rest = v.substr(c + 1);
  }
  std::string out = epoch > 0 ? std::to_string(epoch) + ":" : std::string();
  size_t d = rest.find('-');
  out += std::string(rest.substr(0, d));
  if (d != std::string_view::npos && d + 1 < rest.size()) {
    out += '-';
    out += std::string(rest.substr(d + 1));
  }
  return out;
}

struct VecSink {
  std::vector<uint8_t>* v;
  void put(uint8_t b) { v->push_back(b); }
};

// go-rpm-version a.LessThan(b), host side (sort keys, verkey.h)
bool rpm_less(std::string_view a, std::string_view b) {
  std::vector<uint8_t> ka, kb;
  VecSink sa{&ka}, sb{&kb};
  rpm_encode(reinterpret_cast<const uint8_t*>(a.data()), uint32_t(a.size()), sa);
  rpm_encode(reinterpret_cast<const uint8_t*>(b.data()), uint32_t(b.size()), sb);
  return std::lexicographical_compare(ka.begin(), ka.end(), kb.begin(), kb.end());
}

// ---- one GPU pass per Detect call ---------------------------------------------------------
struct Plan {
  int32_t plat = -1;
  HostBatch batch;
  void add(bool skip, std::string_view name, std::string_view ver) {
    batch.add(skip || plat < 0 ? 0xFFFFFFFFu : uint32_t(plat), name, ver);
  }
  void add(bool skip, std::string_view name, std::string_view ver, uint2 a) {
    batch.add(skip || plat < 0 ? 0xFFFFFFFFu : uint32_t(plat), name, ver, a);
  }
};

bool run_plan(Engine& eng, const Plan& plan, std::vector<uint2>& pairs, std::string& key_err, std::string& err) {
  int64_t err_pkg = -1;
  if (!eng.match_host(plan.batch, pairs, err_pkg, err)) return false;
  key_err.clear();
  if (err_pkg >= 0) {
    const std::string_view name = plan.batch.name(size_t(err_pkg));
    int32_t k = eng.db().find_key(plan.batch.pk[size_t(err_pkg)].x, name);
    key_err = k >= 0 ? eng.db().keys[size_t(k)].err : "advisory decode error";
    if (key_err.empty()) key_err = "advisory decode error";
  }
  return true;
}

// ---- table-driven drivers ------------------------------------------------------------------
enum NameSel { NAME_BIN, NAME_SRC, NAME_SRC_OR_BIN, NAME_MODULAR };
enum VerSel { VER_BIN, VER_SRC };
enum : uint32_t {
  F_PKGID = 1,        // PkgID copied
  F_CUSTOM = 2,       // Custom copied
  F_DEBIAN = 4,       // VendorIDs, Status, package-specific severity (debian.go:84-98)
  F_RPM_STRING = 8,   // FixedVersion = rpm Version.String()
  F_KSPLICE = 16,     // package ksplice tag attribute (oracle)
  F_ARCH = 32,        // package arch attribute (rocky)
};

// Per-driver flags of the table drivers (the drivers map below and the batch export).
uint32_t table_flags(uint8_t drv) {
  switch (drv) {
    case DRV_DEBIAN: return F_PKGID | F_CUSTOM | F_DEBIAN;
    case DRV_ALMA: return F_PKGID | F_CUSTOM | F_RPM_STRING;
    case DRV_ROCKY: return F_PKGID | F_CUSTOM | F_RPM_STRING | F_ARCH;
    case DRV_ORACLE: return F_PKGID | F_CUSTOM | F_KSPLICE;
    case DRV_MARINER: return F_RPM_STRING;  // mariner.go:50-57: no PkgID, no Custom
    default: return F_PKGID | F_CUSTOM;     // ubuntu, amazon, alpine, wolfi, chainguard, suse, photon
  }
}

// The advisory side of a table driver's DetectedVulnerability (e.g. debian.go:78-98,
// alma.go:64-71): everything but the package fields (PkgID / PkgName / InstalledVersion),
// which the caller sets from its package.
void table_epilogue(uint32_t flags, const Advisory& a, Vuln& v) {
  v.copy = COPY_PKG_NAME | COPY_IDENTIFIER | COPY_LAYER | ((flags & F_PKGID) ? COPY_PKG_ID : 0);
  v.vuln_id = a.vuln_id;
  v.data_source = a.data_source;
  if (flags & F_CUSTOM) {
    v.has_custom = !a.custom.empty();
    v.custom = a.custom;
  }
  v.fixed = (flags & F_RPM_STRING) && !a.fixed.empty() ? rpm_string(a.fixed) : a.fixed;
  if (flags & F_DEBIAN) {
    v.vendor_ids = a.vendor_ids;
    v.status = int32_t(a.status);
    if (a.severity != 0) {  // debian.go:92-98 package-specific severity
      v.severity_source = "debian";
      v.severity = severity_name(a.severity);
    }
  }
}

struct Spec {
  std::function<std::string(std::string_view os_ver, const Repo* repo, int64_t now)> bucket;
  NameSel name;
  VerSel ver;
  uint32_t flags;
  const char* err_prefix;
  std::function<bool(const Pkg&)> skip;  // skipped before the lookup (no error possible)
  std::function<bool(std::string_view family, std::string_view os_ver, int64_t now)> supported;
};

class TableDriver : public OsDriver {
  Spec s_;

 public:
  explicit TableDriver(Spec s) : s_(std::move(s)) {}

  bool detect(Engine& eng, std::string_view os_ver, const Repo* repo, const std::vector<Pkg>& pkgs, int64_t now,
              std::vector<Vuln>& out, std::string& err) const override {
    const DB& db = eng.db();
    Plan plan;
    plan.plat = db.find_plat(s_.bucket(os_ver, repo, now));
    std::vector<std::string> cmpv(pkgs.size()), names(pkgs.size());
    for (size_t i = 0; i < pkgs.size(); i++) {
      const Pkg& p = pkgs[i];
      cmpv[i] = s_.ver == VER_SRC ? format_version(p.src_epoch, p.src_version, p.src_release)
                                  : format_version(p.epoch, p.version, p.release);
      switch (s_.name) {
        case NAME_BIN: names[i] = std::string(p.name); break;
        case NAME_SRC: names[i] = std::string(p.src_name); break;
        case NAME_SRC_OR_BIN: names[i] = std::string(p.src_name.empty() ? p.name : p.src_name); break;
        case NAME_MODULAR: names[i] = modular_name(p.name, p.modularitylabel); break;
      }
      const bool skip = s_.skip && s_.skip(p);
      if (s_.flags & (F_KSPLICE | F_ARCH)) {
        uint2 a = make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu);
        if (s_.flags & F_ARCH) a.x = db.arch_id(p.arch);
        if (s_.flags & F_KSPLICE) a.y = db.ksplice_id(extract_ksplice(p.release));
        plan.add(skip, names[i], cmpv[i], a);
      } else {
        plan.add(skip, names[i], cmpv[i]);
      }
    }
    std::vector<uint2> pairs;
    std::string key_err;
    if (!run_plan(eng, plan, pairs, key_err, err)) return false;
    if (!key_err.empty()) {
      err = std::string(s_.err_prefix) + key_err;
      return false;
    }
    for (const uint2& m : pairs) {
      const Pkg& p = pkgs[m.x];
      Vuln v;
      v.pkg = m.x;
      table_epilogue(s_.flags, db.advs[m.y], v);
      if (s_.flags & F_PKGID) v.pkg_id = std::string(p.id);
      v.pkg_name = std::string(p.name);
      v.installed = format_version(p.epoch, p.version, p.release);
      out.push_back(std::move(v));
    }
    return true;
  }

  bool is_supported(std::string_view family, std::string_view os_ver, int64_t now) const override {
    return s_.supported(family, os_ver, now);
  }
};

// ---- redhat.go ---------------------------------------------------------------------------
const std::map<std::string, std::vector<std::string>, std::less<>>& redhat_default_content_sets() {
  static const std::map<std::string, std::vector<std::string>, std::less<>> m = {
      {"6", {"rhel-6-server-rpms", "rhel-6-server-extras-rpms"}},
      {"7", {"rhel-7-server-rpms", "rhel-7-server-extras-rpms"}},
      {"8", {"rhel-8-for-x86_64-baseos-rpms", "rhel-8-for-x86_64-appstream-rpms"}},
      {"9", {"rhel-9-for-x86_64-baseos-rpms", "rhel-9-for-x86_64-appstream-rpms"}},
  };
  return m;
}

class RedHat : public OsDriver {
 public:
  bool detect(Engine& eng, std::string_view os_ver_in, const Repo*, const std::vector<Pkg>& pkgs, int64_t,
              std::vector<Vuln>& out, std::string& err) const override {
    const DB& db = eng.db();
    const std::string os_ver = os_major(os_ver_in);
    Plan plan;
    plan.plat = db.find_plat("Red Hat");
    // CPE sets: one per distinct (content sets, NVR) among the packages (redhat.go:112-120)
    const uint32_t words = std::max<uint32_t>((db.n_cpe + 31) / 32, 1);
    std::map<std::vector<std::string>, uint32_t> set_ids;
    plan.batch.cpe_words = words;
    std::vector<std::string> inst(pkgs.size()), names(pkgs.size());
    for (size_t i = 0; i < pkgs.size(); i++) {
      const Pkg& p = pkgs[i];
      const bool remi = p.release.size() >= 5 && p.release.substr(p.release.size() - 5) == ".remi";
      names[i] = modular_name(p.name, p.modularitylabel);
      inst[i] = format_version(p.epoch, p.version, p.release);
      std::vector<std::string> key;  // content sets..., "\x01" + nvr
      std::vector<std::string_view> repos, nvrs;
      std::string nvr;
      if (!p.has_build_info) {
        auto it = redhat_default_content_sets().find(os_ver);
        if (it != redhat_default_content_sets().end())
          for (const std::string& c : it->second) repos.push_back(c);
      } else {
        repos = p.content_sets;
        nvr = std::string(p.nvr) + "-" + std::string(p.build_arch);
      }
      nvrs.push_back(nvr);
      for (std::string_view r : repos) key.emplace_back(r);
      key.push_back("\x01" + nvr);
      auto it = set_ids.find(key);
      if (it == set_ids.end()) {
        it = set_ids.emplace(key, uint32_t(set_ids.size())).first;
        plan.batch.cpe_bits.resize(plan.batch.cpe_bits.size() + words, 0u);
        uint32_t* bits = plan.batch.cpe_bits.data() + size_t(it->second) * words;
        for (int64_t c : db.redhat_cpes(repos, nvrs))
          if (c >= 0 && uint64_t(c) < uint64_t(words) * 32) bits[c >> 5] |= 1u << (c & 31);
      }
      uint2 a;
      a.x = db.arch_id(p.arch) | (p.arch == "noarch" ? PA_NOARCH : 0u);
      a.y = it->second;
      plan.add(remi, names[i], inst[i], a);  // isFromSupportedVendor (redhat.go:197-205)
    }
    std::vector<uint2> pairs;
    std::string key_err;
    if (!run_plan(eng, plan, pairs, key_err, err)) return false;
    if (!key_err.empty()) {
      err = "redhat vulnerability detection error: failed to get Red Hat advisories: " + key_err;
      return false;
    }
    // per package: uniqVulns merge (redhat.go:146-180), then sorted by VulnerabilityID
    size_t i = 0;
    while (i < pairs.size()) {
      const uint32_t pk = pairs[i].x;
      const Pkg& p = pkgs[pk];
      std::map<std::string, Vuln> uniq;
      for (; i < pairs.size() && pairs[i].x == pk; i++) {
        const Advisory& a = db.advs[pairs[i].y];
        Vuln v;
        v.pkg = pk;
        v.copy = COPY_PKG_ID | COPY_PKG_NAME | COPY_IDENTIFIER | COPY_LAYER;
        v.vuln_id = a.vuln_id;
        v.pkg_id = std::string(p.id);
        v.pkg_name = std::string(p.name);
        v.installed = inst[pk];
        v.status = int32_t(a.status);
        v.severity_source = "redhat";
        v.severity = severity_name(a.severity);
        auto it = uniq.find(a.vuln_id);
        if (a.fixed.empty()) {
          if (it == uniq.end()) uniq.emplace(a.vuln_id, std::move(v));
          continue;
        }
        v.vendor_ids = a.vendor_ids;
        v.fixed = rpm_string(a.fixed);
        if (it == uniq.end()) {
          uniq.emplace(a.vuln_id, std::move(v));
          continue;
        }
        Vuln& u = it->second;  // ustrings.Unique: sorted, de-duplicated union
        std::vector<std::string> ids = u.vendor_ids;
        ids.insert(ids.end(), v.vendor_ids.begin(), v.vendor_ids.end());
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        u.vendor_ids = std::move(ids);
        if (rpm_less(u.fixed, a.fixed)) u.fixed = v.fixed;
      }
      for (auto& [id, v] : uniq) out.push_back(std::move(v));
    }
    return true;
  }
  bool is_supported(std::string_view family, std::string_view os_ver, int64_t now) const override {
    return supported(family == "centos" ? centos_eol() : redhat_eol(), os_major(os_ver), now);
  }
};

bool always(std::string_view, std::string_view, int64_t) { return true; }

std::function<bool(std::string_view, std::string_view, int64_t)> eol_of(const EolMap& (*tab)(),
                                                                           std::string (*norm)(std::string_view)) {
  return [tab, norm](std::string_view, std::string_view v, int64_t now) {
    return supported(tab(), norm ? norm(v) : std::string(v), now);
  };
}

std::string os_minor_s(std::string_view v) { return os_minor(v); }
std::string os_major_s(std::string_view v) { return os_major(v); }
std::string amazon_release_s(std::string_view v) { return amazon_release(v); }

}  // namespace

const OsDriver* find_os_driver(std::string_view family) {
  static const std::map<std::string, std::unique_ptr<OsDriver>, std::less<>> drivers = [] {
    std::map<std::string, std::unique_ptr<OsDriver>, std::less<>> m;
    auto add = [&](const char* fam, Spec s) { m[fam] = std::make_unique<TableDriver>(std::move(s)); };
    add("debian", {[](std::string_view v, const Repo*, int64_t) { return "debian " + os_major(v); }, NAME_SRC, VER_SRC,
                   table_flags(DRV_DEBIAN), "failed to get debian advisories: ", nullptr,
                   eol_of(debian_eol, os_major_s)});
    add("ubuntu", {[](std::string_view v, const Repo*, int64_t now) { return "ubuntu " + ubuntu_release(v, now); },
                   NAME_SRC, VER_SRC, table_flags(DRV_UBUNTU), "failed to get Ubuntu advisories: ", nullptr,
                   eol_of(ubuntu_eol, nullptr)});
    add("amazon", {[](std::string_view v, const Repo*, int64_t) { return "amazon linux " + amazon_release(v); },
                   NAME_BIN, VER_BIN, table_flags(DRV_AMAZON), "failed to get amazon advisories: ", nullptr,
                   eol_of(amazon_eol, amazon_release_s)});
    add("alpine", {[](std::string_view v, const Repo* r, int64_t) { return "alpine " + alpine_stream(v, r); },
                   NAME_SRC_OR_BIN, VER_SRC, table_flags(DRV_ALPINE), "failed to get alpine advisories: ", nullptr,
                   eol_of(alpine_eol, os_minor_s)});
    add("wolfi", {[](std::string_view, const Repo*, int64_t) { return std::string("wolfi"); }, NAME_SRC_OR_BIN,
                  VER_BIN, table_flags(DRV_WOLFI), "failed to get Wolfi advisories: ", nullptr, always});
    add("chainguard", {[](std::string_view, const Repo*, int64_t) { return std::string("chainguard"); },
                       NAME_SRC_OR_BIN, VER_BIN, table_flags(DRV_CHAINGUARD), "failed to get Chainguard advisories: ", nullptr,
                       always});
    add("alma", {[](std::string_view v, const Repo*, int64_t) { return "alma " + os_major(v); }, NAME_MODULAR, VER_BIN,
                 table_flags(DRV_ALMA), "failed to get AlmaLinux advisories: ",
                 [](const Pkg& p) {  // alma.go:53-57
                   return p.release.find(".module_el") != std::string_view::npos && p.modularitylabel.empty();
                 },
                 eol_of(alma_eol, os_major_s)});
    add("rocky", {[](std::string_view v, const Repo*, int64_t) { return "rocky " + os_major(v); }, NAME_MODULAR,
                  VER_BIN, table_flags(DRV_ROCKY), "failed to get Rocky Linux advisories: ",
                  [](const Pkg& p) { return !p.modularitylabel.empty(); },  // rocky.go:52-56
                  eol_of(rocky_eol, os_major_s)});
    add("oracle", {[](std::string_view v, const Repo*, int64_t) { return "Oracle Linux " + os_major(v); }, NAME_BIN,
                   VER_BIN, table_flags(DRV_ORACLE), "failed to get Oracle Linux advisory: ", nullptr,
                   eol_of(oracle_eol, os_major_s)});
    add("opensuse.leap", {[](std::string_view v, const Repo*, int64_t) { return "openSUSE Leap " + std::string(v); },
                          NAME_BIN, VER_BIN, table_flags(DRV_SUSE),
                          "failed to get SUSE advisory: failed to get SUSE advisories: ", nullptr,
                          eol_of(opensuse_eol, nullptr)});
    add("suse linux enterprise server",
        {[](std::string_view v, const Repo*, int64_t) { return "SUSE Linux Enterprise " + std::string(v); }, NAME_BIN,
         VER_BIN, table_flags(DRV_SUSE), "failed to get SUSE advisory: failed to get SUSE advisories: ", nullptr,
         eol_of(sles_eol, nullptr)});
    add("photon", {[](std::string_view v, const Repo*, int64_t) { return "Photon OS " + std::string(v); }, NAME_SRC,
                   VER_BIN, table_flags(DRV_PHOTON),
                   "failed to get Photon Linux advisory: failed to get Photon advisories: ", nullptr,
                   eol_of(photon_eol, nullptr)});
    add("cbl-mariner", {[](std::string_view v, const Repo*, int64_t) { return "CBL-Mariner " + os_minor(v); },
                        NAME_SRC, VER_SRC, table_flags(DRV_MARINER), "failed to get CBL-Mariner advisories: ", nullptr, always});
    m["redhat"] = std::make_unique<RedHat>();
    m["centos"] = std::make_unique<RedHat>();
    return m;
  }();
  auto it = drivers.find(family);
  return it == drivers.end() ? nullptr : it->second.get();
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

// ---------------------------------------------------------------- library ------------------
const char* library_ecosystem(std::string_view t) {
  // NewDriver (driver.go:25-93): LangType -> ecosystem
  static const std::map<std::string, const char*, std::less<>> m = {
      {"bundler", "rubygems"}, {"gemspec", "rubygems"}, {"rustbinary", "cargo"}, {"cargo", "cargo"},
      {"composer", "composer"}, {"gobinary", "go"}, {"gomod", "go"}, {"jar", "maven"}, {"pom", "maven"},
      {"gradle", "maven"}, {"npm", "npm"}, {"yarn", "npm"}, {"pnpm", "npm"}, {"node-pkg", "npm"},
      {"javascript", "npm"}, {"nuget", "nuget"}, {"dotnet-core", "nuget"}, {"packages-props", "nuget"},
      {"pipenv", "pip"}, {"poetry", "pip"}, {"pip", "pip"}, {"python-pkg", "pip"}, {"pub", "pub"},
      {"hex", "erlang"}, {"conan", "conan"}, {"swift", "swift"}, {"cocoapods", "cocoapods"},
      {"bitnami", "bitnami"}, {"kubernetes", "k8s"},
  };
  auto it = m.find(t);
  return it == m.end() ? nullptr : it->second;
}

std::string normalize_pkg_name(std::string_view eco, std::string_view name) {
  std::string n(name);
  if (eco == "pip") {
    for (char& c : n) {
      if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
      else if (c == '_') c = '-';
    }
  }
  return n;
}

namespace {

// The advisory side of the library driver's DetectedVulnerability (driver.go:125-132;
// library.Detect adds Layer / PkgIdentifier / PkgPath, detect.go:33-37 when wrap).
void library_epilogue(bool wrap, const Advisory& a, Vuln& v) {
  v.copy = COPY_PKG_ID | COPY_PKG_NAME | (wrap ? COPY_IDENTIFIER | COPY_LAYER : 0);
  v.vuln_id = a.vuln_id;
  v.fixed = a.lib_fixed;
  v.data_source = a.data_source;
}

DetectStatus library_run(Engine& eng, std::string_view lib_type, const std::vector<Pkg>& pkgs, bool wrap,
                         std::vector<Vuln>& out, std::string& err) {
  const char* eco = library_ecosystem(lib_type);
  if (!eco) return DETECT_UNSUPPORTED_OS;
  const DB& db = eng.db();
  Plan plan;
  plan.plat = db.find_plat(std::string(eco) + "::");
  std::vector<std::string> names(pkgs.size());
  for (size_t i = 0; i < pkgs.size(); i++) {
    names[i] = normalize_pkg_name(eco, pkgs[i].name);
    plan.add(false, names[i], pkgs[i].version);
  }
  std::vector<uint2> pairs;
  std::string key_err;
  if (!run_plan(eng, plan, pairs, key_err, err)) return DETECT_ERROR;
  if (!key_err.empty()) {
    const std::string e(eco);
    err = "failed to get " + e + " advisories: " + key_err;  // driver.go:115-117
    if (wrap)  // detect.go:30-32, 18-20
      err = "failed to scan " + e + " vulnerabilities: failed to detect " + e + " vulnerabilities: " + err;
    return DETECT_ERROR;
  }
  for (const uint2& m : pairs) {
    const Pkg& p = pkgs[m.x];
    Vuln v;
    v.pkg = m.x;
    library_epilogue(wrap, db.advs[m.y], v);
    v.pkg_id = std::string(p.id);
    v.pkg_name = std::string(p.name);
    v.installed = std::string(p.version);
    if (wrap) v.pkg_path = std::string(p.file_path);  // detect.go:33-37
    out.push_back(std::move(v));
  }
  return DETECT_OK;
}

}  // namespace

DetectStatus library_detect(Engine& eng, std::string_view lib_type, const std::vector<Pkg>& pkgs,
                            std::vector<Vuln>& out, std::string& err) {
  return library_run(eng, lib_type, pkgs, true, out, err);
}

DetectStatus library_detect_vulnerabilities(Engine& eng, std::string_view lib_type, const std::vector<Pkg>& pkgs,
                                            std::vector<Vuln>& out, std::string& err) {
  return library_run(eng, lib_type, pkgs, false, out, err);
}

// FillInfo inputs of one detector output (vulninfo.h): the fields the epilogues above
// copy from advisory a for a driver of family drv (Status/SeveritySource for debian
// (debian.go:89-98) and Red Hat (redhat.go:160-161); no DataSource for Red Hat; rpm
// String() FixedVersion for Red Hat, Alma, Rocky and CBL-Mariner; createFixedVersions
// for library drivers).  The batch path uses it per (package, advisory) pair.
void detector_fill_fields(uint8_t drv, const Advisory& a, DetFill& f) {
  f = DetFill();
  f.data_source = drv == DRV_REDHAT ? -1 : a.data_source;
  const bool rpm_out = drv == DRV_REDHAT || drv == DRV_ALMA || drv == DRV_ROCKY || drv == DRV_MARINER;
  f.fixed_version = drv == DRV_LIBRARY ? a.lib_fixed : rpm_out && !a.fixed.empty() ? rpm_string(a.fixed) : a.fixed;
  switch (drv) {
    case DRV_DEBIAN:
      f.status = a.status;
      f.fixed = !a.fixed.empty();
      if (a.severity != 0) {
        f.severity_source = "debian";
        f.severity = severity_name(a.severity);
      }
      break;
    case DRV_REDHAT:
      f.status = a.status;
      f.fixed = !a.fixed.empty() && !rpm_string(a.fixed).empty();
      f.severity_source = "redhat";
      f.severity = severity_name(a.severity);
      break;
    case DRV_ALMA:
    case DRV_ROCKY:
    case DRV_MARINER:
      f.fixed = !a.fixed.empty() && !rpm_string(a.fixed).empty();
      break;
    case DRV_LIBRARY:
      f.fixed = !a.lib_fixed.empty();
      break;
    default:
      f.fixed = !a.fixed.empty();
  }
}


// ---- Red Hat batch epilogue (redhat.hip groups, host fields) ------------------------------

std::vector<uint32_t> redhat_fixed_ranks(const DB& db) {
  // rank of every Red Hat advisory's FixedVersion in go-rpm-version order (ties share a
  // rank); RH_NONE for unfixed advisories and other drivers' (the merge never reads them)
  std::vector<uint32_t> rank(db.advs.size(), RH_NONE);
  std::vector<std::pair<std::vector<uint8_t>, uint32_t>> keys;
  for (const Key& k : db.keys) {
    if (k.plat >= db.plats.size() || db.plats[k.plat].drv != DRV_REDHAT) continue;
    for (uint32_t a : k.advs) {
      if (db.advs[a].fixed.empty()) continue;
      std::vector<uint8_t> kb;
      VecSink s{&kb};
      rpm_encode(reinterpret_cast<const uint8_t*>(db.advs[a].fixed.data()), uint32_t(db.advs[a].fixed.size()), s);
      keys.emplace_back(std::move(kb), a);
    }
  }
  std::sort(keys.begin(), keys.end());
  uint32_t r = 0;
  for (size_t i = 0; i < keys.size(); i++) {
    if (i && keys[i].first != keys[i - 1].first) r++;
    rank[keys[i].second] = r;
  }
  return rank;
}

// The advisory side of the Red Hat driver's DetectedVulnerability for a group of one member
// (redhat.go:140-171: Status and Severity of the member; VendorIDs and the rpm String()
// FixedVersion only when it is fixed; no DataSource, no Custom).
void redhat_member_epilogue(const Advisory& a, Vuln& v) {
  v.copy = COPY_PKG_ID | COPY_PKG_NAME | COPY_IDENTIFIER | COPY_LAYER;
  v.vuln_id = a.vuln_id;
  v.status = int32_t(a.status);
  v.severity_source = "redhat";
  v.severity = severity_name(a.severity);
  if (!a.fixed.empty()) {
    v.vendor_ids = a.vendor_ids;
    v.fixed = rpm_string(a.fixed);
  }
}

void advisory_templates(const DB& db, std::vector<Vuln>& out) {
  std::vector<uint8_t> drv(db.advs.size(), DRV_NONE);
  for (const Key& k : db.keys)
    if (k.plat < db.plats.size())
      for (uint32_t a : k.advs) drv[a] = db.plats[k.plat].drv;
  out.assign(db.advs.size(), Vuln());
  for (size_t i = 0; i < db.advs.size(); i++) {
    const Advisory& a = db.advs[i];
    Vuln& v = out[i];
    v.pkg = 0;
    if (drv[i] == DRV_LIBRARY) library_epilogue(true, a, v);
    else if (drv[i] == DRV_REDHAT) redhat_member_epilogue(a, v);
    else table_epilogue(table_flags(drv[i]), a, v);
  }
}

void redhat_batch_vulns(const DB& db, const HostBatch& hb, const std::vector<RhRec>& recs,
                        const std::vector<uint32_t>& contrib, uint32_t pkg_base, std::vector<Vuln>& out) {
  for (const RhRec& r : recs) {
    const uint32_t pk = r.pkg - pkg_base;
    const Advisory& a = db.advs[r.base];
    Vuln v;
    v.pkg = pk;
    v.copy = COPY_PKG_ID | COPY_PKG_NAME | COPY_IDENTIFIER | COPY_LAYER;
    v.vuln_id = a.vuln_id;
    v.installed = std::string(hb.version(pk));
    v.status = int32_t(a.status);
    v.severity_source = "redhat";
    v.severity = severity_name(a.severity);
    if (r.best != RH_NONE) v.fixed = rpm_string(db.advs[r.best].fixed);
    // VendorIDs (redhat.go:163-170): a lone fixed first member keeps its list as is; every
    // merge of a fixed member makes it the sorted, de-duplicated union (ustrings.Unique)
    uint32_t n_fixed = 0;
    for (uint32_t j = r.start; j < r.start + r.len; j++) n_fixed += !db.advs[contrib[j]].fixed.empty();
    if (n_fixed == 1 && !a.fixed.empty()) {
      v.vendor_ids = a.vendor_ids;
    } else if (n_fixed) {
      for (uint32_t j = r.start; j < r.start + r.len; j++) {
        const Advisory& m = db.advs[contrib[j]];
        if (!m.fixed.empty()) v.vendor_ids.insert(v.vendor_ids.end(), m.vendor_ids.begin(), m.vendor_ids.end());
      }
      std::sort(v.vendor_ids.begin(), v.vendor_ids.end());
      v.vendor_ids.erase(std::unique(v.vendor_ids.begin(), v.vendor_ids.end()), v.vendor_ids.end());
    }
    out.push_back(std::move(v));
  }
}

}  // namespace tvm
