// The batch's transport form (pipeline.h): what crosses PCIe for a pipelined pass.  Per chunk
// ONE contiguous block {name ref u32, version ref u32, lengths u16 (name | version << 8),
// platform index u8 per package; the chunk's group offsets (u64, the arena's tile_off);
// attributes (uint2) when the batch has them; the bytes of the names and versions first seen
// in this chunk}, every section 16-byte aligned.  A reference is the wire offset of the
// string's first occurrence in the batch, so a repeated name or version crosses the link
// once; unpack_kernel (pipeline.hip) rebuilds pk / tile_off / arena / attr in HBM.
//
// Built on the host threads in two steps: plan() finds every string's first occurrence
// (hash-sharded dedup, shards in parallel, first occurrence = lowest package index) and the
// exact layout; the caller then provides a pinned block of bytes() and emit() fills it (string
// bytes and references in parallel blocks).  The output is byte-identical to a sequential
// encoder that walks the packages in order.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "engine.h"
#include "host_par.h"

namespace tvm {

struct WireChunk {
  uint64_t off = 0, bytes = 0;                                                       // block in the wire
  uint64_t o_nref = 0, o_vref = 0, o_lens = 0, o_plat = 0, o_toff = 0, o_attr = 0;  // section offsets (absolute)
  uint32_t m = 0, groups = 0;                                                        // packages, 64-package groups
};

class WireEncoder {
 public:
  // toff: tile_off padded to whole tiles + the arena end; bounds: chunk c = tiles
  // [bounds[c], bounds[c + 1]).  false with err empty: the batch has no transport form (a
  // string of 256 bytes or more, more than 255 platforms, or a form of 4 GiB or more).
  bool plan(const HostBatch& hb, const std::vector<uint64_t>& toff, const std::vector<uint32_t>& bounds, int threads,
            std::string& err);
  uint64_t bytes() const { return total_; }
  const std::vector<WireChunk>& chunks() const { return wc_; }
  const std::vector<uint32_t>& platforms() const { return ptab_; }  // platform index -> platform id
  void emit(uint8_t* wire);
  void clear();

 private:
  const HostBatch* hb_ = nullptr;
  const std::vector<uint64_t>* toff_ = nullptr;
  std::vector<uint32_t> bounds_;
  int threads_ = 1;
  std::vector<uint64_t> off_;    // per package: arena offset of its name
  std::vector<uint32_t> first_;  // per string (2i name, 2i+1 version): string id of its first occurrence
  std::vector<uint32_t> ref_;    // per first occurrence: its wire offset (emit)
  std::vector<uint8_t> pidx_of_;   // platform id -> index (ids below kDirectPlat)
  uint8_t pidx_absent_ = 0;        // index of the absent-bucket id 0xFFFFFFFF
  std::vector<uint32_t> ptab_;
  struct Block {
    uint32_t p0, p1;   // packages
    uint32_t chunk;
    uint64_t bytes;    // bytes of the strings first seen in this block
    uint64_t heap;     // wire offset of those bytes
  };
  std::vector<Block> blocks_;
  std::vector<WireChunk> wc_;
  uint64_t total_ = 0;
  uint8_t pidx(uint32_t plat) const { return plat < pidx_of_.size() ? pidx_of_[plat] : pidx_absent_; }
};

}  // namespace tvm
