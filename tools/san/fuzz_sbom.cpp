// libFuzzer harness (tools/san/run.sh, ASan + UBSan): the native CycloneDX decoder
// (trivy_amd/csrc/sbom.cpp) on arbitrary bytes, seeded with the reference's SBOM fixtures.
// Both ownership modes; a successful decode's views are read back whole, so a view past the
// text or into freed memory is caught.
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>

#include "sbom.h"

static uint64_t touch(std::string_view s) {
  uint64_t h = s.size();
  for (unsigned char c : s) h = h * 31 + c;
  return h;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  const std::string text(reinterpret_cast<const char*>(data), size);
  for (bool borrow : {false, true}) {
    tvm::Sbom s;
    std::string err;
    if (!tvm::decode_cyclonedx(text, s, err, borrow)) continue;
    volatile uint64_t h = touch(s.os_family) + touch(s.os_name) + touch(s.serial);
    for (const tvm::SbomTarget& t : s.targets) {
      h = h + touch(t.type) + touch(t.file_path);
      if (t.begin > t.end || t.end > s.view.size() || s.extra.size() < s.view.size()) __builtin_trap();
      for (size_t i = t.begin; i < t.end; i++) {
        const tvm_package& p = s.view[i];
        for (const tvm_str& x : {p.id, p.name, p.version, p.release, p.arch, p.src_name, p.src_version,
                                  p.src_release, p.modularitylabel, p.file_path})
          if (x.p) h = h + touch(std::string_view(x.p, x.n));
        const tvm::SbomExtra& e = s.extra[i];
        h = h + touch(e.purl) + touch(e.bom_ref) + touch(e.layer_digest) + touch(e.layer_diff_id);
      }
    }
    (void)h;
  }
  return 0;
}
