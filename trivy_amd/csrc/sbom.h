// Native CycloneDX decoder: a CycloneDX JSON document -> the detector input (the OS, its
// packages, the language applications and their libraries) without an intermediate DOM.
//
// Restates pkg/sbom/cyclonedx/unmarshal.go:63-230 (parseBOM / parseComponent: supported
// component types, PURL, "aquasecurity:trivy:" properties, the metadata component as root,
// dependencies as relationships between known bom-refs) and pkg/sbom/io/decode.go:47-380
// (Decoder.Decode: one OS component at most, applications by their Type property,
// decodeLibrary, fillSrcPkg, the OS's and each application's dependencies, the rest as OS
// packages of one PURL type and one application per language type, sorted), with the PURL
// rules of pkg/purl/purl.go:130-243 and packageurl-go's parser.  The Python restatement
// trivy_amd/sbom.py (pinned by the integration SBOM goldens) is the checker: the two agree
// field for field (tests/test_sbom_native.py).
//
// One pass over the text: the top-level members the decode needs are parsed straight into
// component records (strings are views into the text unless they hold escapes), everything
// else is validated and skipped.  Packages come out as the tvm_package records the
// detectors take.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/trivy_amd.h"

namespace tvm {

// Optional ftypes.Package fields a decoded package carries (the Python mirror's dict keys).
enum : uint32_t {
  SP_ARCH = 1, SP_EPOCH = 2, SP_RELEASE = 4, SP_MODULARITY = 8, SP_FILEPATH = 16, SP_SRCNAME = 32,
  SP_SRCVERSION = 64, SP_SRCRELEASE = 128, SP_SRCEPOCH = 256, SP_LAYER_DIGEST = 512, SP_LAYER_DIFFID = 1024,
};

struct SbomPkg {  // a decoded library (decodeLibrary) before it is placed in its target
  std::string_view id, name, version, release, arch, src_name, src_version, src_release, modularitylabel, file_path;
  std::string_view purl, bom_ref, layer_digest, layer_diff_id;
  int64_t epoch = 0, src_epoch = 0;
  uint32_t present = 0;  // SP_*
};

struct SbomExtra {  // the fields of a package beyond tvm_package
  std::string_view purl, bom_ref, layer_digest, layer_diff_id;
  uint32_t present = 0;  // SP_*
};

struct SbomTarget {  // target 0: the OS packages; then the applications, sorted
  std::string_view type, file_path;
  size_t begin = 0, end = 0;  // its packages: view / extra [begin, end)
};

// Large decode arrays come from anonymous mappings advised for transparent huge pages: a 1M-
// component document touches ~1 GB of fresh memory, and at 4 KB pages the page faults alone
// cost as much as the parse (measured: tools/sbom_rate.py, TVM_SBOM_TRACE=1).
void* huge_alloc(size_t bytes);
void huge_free(void* p, size_t bytes);

template <class T>
struct HugeAlloc {
  using value_type = T;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U>&) {}
  T* allocate(size_t n) { return static_cast<T*>(huge_alloc(n * sizeof(T))); }
  void deallocate(T* p, size_t n) { huge_free(p, n * sizeof(T)); }
  template <class U>
  bool operator==(const HugeAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const HugeAlloc<U>&) const { return false; }
};
template <class T>
using HugeVec = std::vector<T, HugeAlloc<T>>;

// Strings built by the decode (unescaped, joined): a bump arena of chunks that never move.
struct Arena {
  struct Chunk {
    char* p;
    size_t n;
  };
  std::vector<Chunk> chunks;
  size_t left = 0;
  char* at = nullptr;
  std::string_view keep(std::string_view a, std::string_view b = {}, std::string_view c = {});
  ~Arena();
};

struct Sbom {
  bool has_os = false;
  std::string_view os_family, os_name, serial;
  int64_t version = 0;
  HugeVec<tvm_package> view;  // detector input, target after target
  HugeVec<SbomExtra> extra;
  size_t n_view = 0;
  std::vector<SbomTarget> targets;
  std::string text;  // the document when it is copied (the views point into it or the caller's)
  std::vector<std::unique_ptr<Arena>> arenas;  // [0]: the parse; then one per parallel piece
  Arena& arena(size_t k) {
    while (arenas.size() <= k) arenas.emplace_back(new Arena());
    return *arenas[k];
  }
};

// false: err holds the reference's message ("failed to decode CycloneDX JSON: ...",
// "failed to parse root component: ...", "failed to decode components: ...",
// "failed to aggregate packages: ...").
// borrow: the views point into `text` itself, which must then outlive `out`; else it is copied.
bool decode_cyclonedx(std::string_view text, Sbom& out, std::string& err, bool borrow = false);

}  // namespace tvm
