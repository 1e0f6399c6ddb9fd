// libFuzzer harness (tools/san/run.sh, ASan + UBSan): the read-only bbolt walker
// (trivy_amd/csrc/bbolt.cpp) on arbitrary file images, seeded with the reference's own bolt
// files (tests/golden/bbolt: the fanal cache fixtures, trivy's metadata DB).  Every path
// element and value handed to the visitor is read back whole.
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "bbolt.h"

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  std::vector<uint8_t> img(data, data + size);  // exact-size heap copy: reads past it are caught
  std::string err;
  volatile uint64_t h = 0;
  uint64_t visits = 0;
  (void)tvm::bbolt_walk(img.data(), img.size(),
                        [&](const std::vector<std::string_view>& path, std::string_view value) {
                          for (std::string_view p : path)
                            for (unsigned char c : p) h = h * 31 + c;
                          for (unsigned char c : value) h = h * 31 + c;
                          return ++visits < (1u << 20);
                        },
                        err);
  return 0;
}
