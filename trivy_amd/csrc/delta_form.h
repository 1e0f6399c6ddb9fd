// The delta result form of the end-to-end pipeline: the per-package advisory lists as the
// GPU writes them into pinned host memory when the pass runs with TVM_PIPE_DELTA, and their
// host decode into the CSR (row ends + advisory indices).
//
// Tile t (packages [256 t, 256 t + 256)) with count matches, the first at CSR position b
// (the counts of the tiles before it), is a byte stream at delta_region(t, b) (engine.h) of
// `bytes` bytes, tile_info[t] = {count, bytes}; a tile without matches has no stream:
//   256 count bytes, one per package (255: the count is >= 255 and follows as a 4-byte
//   little-endian integer in front of the package's list);
//   then, package by package, its advisory indices in the match order: the first as 3
//   bytes little endian, each next one as one byte d = index - previous index when that is
//   1..255, else 0 followed by the index as 3 bytes.
// A package's indices are mostly a run of neighbouring advisories of one key (the DB lays a
// key's advisories out together), so a match takes ~1.4 bytes instead of 3 (+ 4 for the row
// end): the C2 pass moves ~32 MB up the link instead of ~77 MB.  Needs < 2^24 advisories.
#pragma once
#include <cstdint>
#include <string>

#include <hip/hip_runtime.h>

namespace tvm {

// Decodes the streams of n_tiles tiles into adv (total entries) and row_end (n_tiles * 256
// entries: the CSR position after each package's list, padding packages included), on the
// host threads.  false (err set) when the streams are inconsistent with tile_info / total.
bool delta_decode(const uint8_t* stream, uint64_t stream_bytes, const uint2* tile_info, uint32_t n_tiles,
                  uint64_t total, uint32_t* adv, uint32_t* row_end, std::string& err);
// One tile (info = its {count, bytes}, pos0 = the CSR position of its first match): its 256
// row ends and its advisories; false when its stream is inconsistent with info.
bool delta_decode_tile(const uint8_t* stream, uint64_t stream_bytes, uint32_t t, uint64_t pos0, uint2 info,
                       uint32_t* adv, uint32_t* row_end);

}  // namespace tvm
