// Host-side mirror of the reference detector surfaces:
//   pkg/detector/ospkg/detect.go:57-91   Driver interface, drivers map, Detect
//   pkg/detector/ospkg/<os>/<os>.go       per-OS Scanner.Detect / IsSupportedVersion
// Each driver keeps the reference's prologue (bucket/release selection, which name
// and which formatted version are looked up) and epilogue (which DetectedVulnerability
// fields are populated); the per-(package, advisory) work runs on the GPU engine.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "engine.h"

namespace tvm {

// ftypes.Package fields the detectors read (pkg/fanal/types/artifact.go:68-105).
struct Pkg {
  std::string_view id, name, version, release, arch, src_name, src_version, src_release;
  std::string_view modularitylabel, nvr, build_arch, file_path;
  std::vector<std::string_view> content_sets;
  bool has_build_info = false;
  int64_t epoch = 0, src_epoch = 0;
};

struct Repo {
  std::string_view family, release;
};

// types.DetectedVulnerability (pkg/types/vulnerability.go:9-31).  Layer and
// PkgIdentifier are opaque to this layer: `copy` tells the caller which fields of
// input package `pkg` to copy (the reference copies them verbatim).
enum : uint32_t { COPY_PKG_ID = 1, COPY_PKG_NAME = 2, COPY_IDENTIFIER = 4, COPY_LAYER = 8 };
struct Vuln {
  uint32_t pkg = 0;
  uint32_t copy = 0;
  std::string vuln_id;
  std::vector<std::string> vendor_ids;
  std::string pkg_id, pkg_name, pkg_path, installed, fixed;
  int32_t status = 0;
  std::string severity_source, severity;
  int32_t data_source = -1;  // DB::sources index
  bool has_custom = false;
  std::string custom;
};

// utils.FormatVersion / FormatSrcVersion (pkg/scanner/utils/utils.go:10-29).
std::string format_version(int64_t epoch, std::string_view version, std::string_view release);
// osver.Major / Minor (pkg/detector/ospkg/version/version.go:15-29).
std::string os_major(std::string_view v);
std::string os_minor(std::string_view v);

enum DetectStatus { DETECT_OK = 0, DETECT_ERROR = 1, DETECT_UNSUPPORTED_OS = 2 };

class OsDriver {
 public:
  virtual ~OsDriver() = default;
  // Driver.Detect(osVer, repo, pkgs)
  virtual bool detect(Engine& eng, std::string_view os_ver, const Repo* repo, const std::vector<Pkg>& pkgs,
                      int64_t now, std::vector<Vuln>& out, std::string& err) const = 0;
  // Driver.IsSupportedVersion(ctx, osFamily, osVer) with clock.Now(ctx) == now
  virtual bool is_supported(std::string_view family, std::string_view os_ver, int64_t now) const = 0;
};

// drivers[osFamily] (detect.go:32-48); nullptr when unsupported.
const OsDriver* find_os_driver(std::string_view family);

// ospkg.Detect (detect.go:63-82): driver lookup, EOSL, gpg-pubkey filter, error wrap.
DetectStatus ospkg_detect(Engine& eng, std::string_view family, std::string_view os_name, const Repo* repo,
                          const std::vector<Pkg>& pkgs, int64_t now, std::vector<Vuln>& out, bool& eosl,
                          std::string& err);

// Unix time of time.Date(y, m, d, 23, 59, 59, 0, UTC).
int64_t eol_unix(int y, int m, int d);

// ---- library (pkg/detector/library) ------------------------------------------------
// NewDriver(libType) -> Driver.Type(): the ecosystem, or nullptr when unsupported.
const char* library_ecosystem(std::string_view lib_type);
// library.Detect (detect.go:11-42): DETECT_UNSUPPORTED_OS means NewDriver returned false
// (the reference returns nil, nil).  Vuln.pkg indexes pkgs (Name, Version, ID, FilePath).
DetectStatus library_detect(Engine& eng, std::string_view lib_type, const std::vector<Pkg>& pkgs,
                            std::vector<Vuln>& out, std::string& err);
// (*Driver).DetectVulnerabilities (driver.go:111-137) for each package, errors unwrapped.
DetectStatus library_detect_vulnerabilities(Engine& eng, std::string_view lib_type, const std::vector<Pkg>& pkgs,
                                            std::vector<Vuln>& out, std::string& err);
// Red Hat batch epilogue: rpm-order rank of every Red Hat advisory's FixedVersion
// (RH_NONE when unfixed), and the DetectedVulnerability of every merged group (redhat.hip)
// - Vuln.pkg is the batch index, InstalledVersion the batch version string.
struct RhRec;
std::vector<uint32_t> redhat_fixed_ranks(const DB& db);
void redhat_batch_vulns(const DB& db, const HostBatch& hb, const std::vector<RhRec>& recs,
                        const std::vector<uint32_t>& contrib, uint32_t pkg_base, std::vector<Vuln>& out);
// The advisory side of every advisory's DetectedVulnerability as its driver's epilogue
// populates it (out[adv]; table drivers: table_flags of the advisory's platform, library:
// library.Detect's fields, Red Hat: a merged group of that one member).  The package fields
// (PkgID / PkgName / InstalledVersion / PkgPath) are left empty: the batch export pairs these
// templates with the package of each match.
void advisory_templates(const DB& db, std::vector<Vuln>& out);
// vulnerability.NormalizePkgName (trivy-db): pip names lower-cased, "_" -> "-".
std::string normalize_pkg_name(std::string_view eco, std::string_view name);

}  // namespace tvm
