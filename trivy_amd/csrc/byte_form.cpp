// Host decode of the byte result form (byte_form.h).
#include "byte_form.h"

#include "engine.h"

namespace tvm {

uint32_t byte_decode_tile(const uint8_t* A, const uint16_t* hi, const uint32_t* wide, const uint32_t* row_end,
                          uint32_t t, uint32_t* adv) {
  const uint32_t* re = row_end + size_t(t) * kTile;
  const uint16_t* h = hi + size_t(t) * kTile;
  uint32_t first[kTile + 1], fpk[kTile + 1];
  uint32_t nf = 0, prev = t ? row_end[size_t(t) * kTile - 1] : 0u;
  const uint32_t b = prev;
  for (uint32_t p = 0; p < uint32_t(kTile); p++) {  // the packages' first positions, no branch
    first[nf] = prev;
    fpk[nf] = p;
    nf += re[p] != prev;
    prev = re[p];
  }
  first[nf] = 0xFFFFFFFFu;
  fpk[nf] = 0;
  const uint32_t end = re[kTile - 1];
  uint32_t a = 0, f = 0, next = first[0], esc = 0;
  for (uint32_t e = b; e < end; e++) {
    const uint32_t x = A[e];
    const bool is_first = e == next;
    const uint32_t fv = (uint32_t(h[fpk[f]]) << 8) | x;
    if (!is_first && x == 0xFFu) {  // rare
      a = wide[e];
      esc++;
    } else {
      a = is_first ? fv : a + x;
    }
    f += is_first;
    next = first[f];
    adv[e] = a;
  }
  return esc;
}

}  // namespace tvm
