// Host decode of the byte result form (byte_form.h).
#include "byte_form.h"

#include <cstring>
#include <vector>

#include "engine.h"

namespace tvm {

uint32_t byte_decode_tile(const uint8_t* A, const uint16_t* hi, const uint32_t* wide, const uint32_t* row_end,
                          uint32_t t, uint32_t* adv) {
  // Two passes: each package's first index goes straight to its CSR position (256 stores)
  // and is flagged there; then one loop over the tile's matches whose only dependency from
  // one match to the next is the running value - a flagged position takes what was stored
  // there, any other adds its byte (a loop keyed on the next first position made that
  // position, loaded through the package counter, part of the chain: 3.8 ns a match).
  thread_local std::vector<uint8_t> flag;
  thread_local std::vector<uint32_t> fval;
  const uint32_t* re = row_end + size_t(t) * kTile;
  const uint16_t* h = hi + size_t(t) * kTile;
  const uint32_t b = t ? row_end[size_t(t) * kTile - 1] : 0u, end = re[kTile - 1];
  if (end <= b) return 0;
  const uint32_t count = end - b;
  if (flag.size() < count) {
    flag.resize(count);
    fval.resize(count);
  }
  uint8_t* fl = flag.data();
  uint32_t* fv = fval.data();
  std::memset(fl, 0, count);
  uint32_t prev = b;
  for (uint32_t p = 0; p < uint32_t(kTile); p++) {
    if (re[p] != prev) {
      fv[prev - b] = (uint32_t(h[p]) << 8) | A[prev];
      fl[prev - b] = 1;
    }
    prev = re[p];
  }
  uint32_t a = 0, esc = 0;
  uint32_t* o = adv + b;
  const uint8_t* x = A + b;
  for (uint32_t i = 0; i < count; i++) {
    const uint32_t xi = x[i], pre = fv[i];
    const bool f = fl[i] != 0;
    if (!f && xi == 0xFFu) {  // rare
      a = wide[b + i];
      esc++;
    } else {
      a = f ? pre : a + xi;
    }
    o[i] = a;
  }
  return esc;
}

}  // namespace tvm
