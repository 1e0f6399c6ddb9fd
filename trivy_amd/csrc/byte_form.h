// The byte result form of the end-to-end pipeline (TVM_PIPE_BYTE): the per-package advisory
// lists as the GPU writes them into pinned host memory, and their host decode into the CSR.
//
// Match i of the pass (CSR position i; the row ends travel as in the CSR form) is one byte
// A[i]: for the first match of its package the low 8 bits of its advisory index, the package's
// high 16 bits being hi[package]; for a later match the difference from the match before when
// it is 1..254, else 0xFF with the index itself at wide[i] (a sparse array: only escapes are
// written).  A package's indices are mostly neighbouring advisories of one key, so C2 sends
// 20.5 MB of bytes + 8 MB of high halves instead of 61.7 MB of 3-byte indices, every position
// computable without a scan (the GPU writes whole words in place, the host decodes a tile in
// one loop with no data-dependent branch but the rare escape).  Needs < 2^24 advisories.
#pragma once
#include <cstdint>

namespace tvm {

// Tile t (packages [256 t, 256 t + 256)): its advisories into adv at their CSR positions.
// row_end: the pass's row ends (all tiles); returns the escapes it met.
uint32_t byte_decode_tile(const uint8_t* A, const uint16_t* hi, const uint32_t* wide, const uint32_t* row_end,
                          uint32_t t, uint32_t* adv);

}  // namespace tvm
