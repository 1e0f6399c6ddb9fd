// End-to-end pipelined match pass: a host batch (pinned) in, the per-package advisory lists
// (CSR, pinned) out, with the link transfers overlapping the kernels.
#pragma once
#include <string>
#include <vector>

#include "engine.h"
#include "wire.h"

namespace tvm {

struct OrderArgs {
  const TileDir* dir;
  const uint32_t* pkg;
  const uint32_t* adv;
  uint32_t* csr_adv;
  uint32_t* row_end;
  uint64_t cap;                // match buffers' capacity (pkg / adv / csr_adv)
  unsigned long long* status;  // look-back word per tile (zeroed before the pass)
  unsigned long long* ticket;  // this launch's ticket counter (zeroed before the pass)
  uint32_t t0;                 // first tile of this launch
  uint32_t n;                  // packages in the batch
  uint32_t pkg_base = 0;       // added to every package index the match kernels wrote (a shard's first package)
};
void launch_order(uint32_t n_tiles, hipStream_t st, const OrderArgs& a);
void launch_copy_out(hipStream_t st, const CopyOutArgs& a);  // engine.h copy_out_tiles as its own kernel
void release_encoders();  // the transport-form encoders kept between batches (tvm_shutdown)


// One batch's pipeline state.  prepare() builds the batch's pinned transport form (or a
// pinned copy of its raw arrays), sizes the device batch, the match buffers and the pinned result buffers; run() then
// streams the batch through in chunks of whole tiles:
//   copy stream    DMA of chunk c to HBM (package words, tile offsets, string bytes, attributes);
//   kernel stream  (after chunk c's upload) one match launch whose first workgroups turn
//                  chunk c-1's match segments into the pinned host CSR (engine.h
//                  copy_out_tiles: 16-byte kernel stores, the link's other direction) while
//                  the rest match chunk c;
//   row-end stream DMA of chunk c-1's row ends (left in HBM by that result move) to the host;
// so chunk c+1's upload and chunk c-1's result move run under chunk c's matching, and the
// host waits once, at the end.  (Measured alternatives, DESIGN.md §7: a DMA device-to-host
// copy runs at half the rate of kernel stores, and a result kernel on its own stream did
// not overlap the match kernels on this runtime.)
class Pipeline {
 public:
  ~Pipeline();
  // transport: send the batch in its transport form when it has one (see build_wire)
  // packed: the result's advisory indices travel as 3 bytes each (the DB has < 2^24)
  bool prepare(Engine& eng, const HostBatch& hb, uint64_t match_cap, uint32_t chunk_packages, bool transport,
               bool packed, std::string& err);
  // One pass.  total = matches (> match_cap: nothing valid, re-prepare with a larger cap);
  // err_pkg = first poisoned package or -1.
  bool run(Engine& eng, const HostBatch& hb, uint64_t& total, int64_t& err_pkg, uint64_t& err_bits, std::string& err);
  // 4-byte indices, or 3-byte ones when packed()
  const uint32_t* adv() const { return adv_h_; }
  bool packed() const { return packed_; }
  const uint32_t* row_end() const { return row_end_h_; }
  uint32_t n_tiles() const { return bounds_.empty() ? 0 : bounds_.back(); }
  uint64_t cap() const { return cap_; }
  uint64_t h2d_bytes() const { return h2d_; }
  uint64_t d2h_bytes() const { return d2h_; }
  uint32_t chunks() const { return uint32_t(bounds_.size() - 1); }
  bool transport_form() const { return !wc_.empty(); }
  // The batch and the whole pass's match list as the pass left them in HBM (every chunk's
  // segments, tile directory over all tiles): the Red Hat merge of a pipelined pass reads them
  const DevBatch& dev_batch() const { return db_; }
  const DevMatches& matches() const { return m_; }
  uint64_t encode_us() const { return encode_us_; }    // building the transport form (host threads)
  uint64_t prepare_us() const { return prepare_us_; }  // the whole prepare(), encode included

 private:
  void release();
  // The batch's transport form (wire.h; pinned wire_h_, mirrored at the same offsets in
  // wire_d_), built on the host threads.  false: prepare fails; true with wc_ empty: no
  // transport form (a string of 256 bytes or more, more than 255 platforms, or 4 GiB).
  bool build_wire(const HostBatch& hb, std::string& err);
  std::vector<WireChunk> wc_;
  uint8_t* wire_h_ = nullptr;
  uint8_t* wire_d_ = nullptr;
  uint32_t* ptab_d_ = nullptr;  // platform index -> platform id
  uint64_t encode_us_ = 0, prepare_us_ = 0;
  int dev_ = -1;
  hipStream_t s_h2d_ = nullptr, s_k_ = nullptr, s_d2h_ = nullptr;
  std::vector<hipEvent_t> ev_h_, ev_k_;  // chunk uploaded / chunk's result move done
  uint32_t* row_end_d_ = nullptr;        // row ends in HBM when the DMA engine carries them up
  std::vector<uint32_t> bounds_;     // chunk c = tiles [bounds_[c], bounds_[c + 1])
  std::vector<uint64_t> toff_;       // tile offsets + the arena end
  // raw form: the batch's arrays in one pinned block (stage_raw)
  uint8_t* raw_h_ = nullptr;
  uint2* raw_pk_ = nullptr;
  uint64_t* raw_toff_ = nullptr;
  uint8_t* raw_arena_ = nullptr;
  uint2* raw_attr_ = nullptr;
  bool stage_raw(const HostBatch& hb, std::string& err);  // allocates; run() copies chunk by chunk
  void stage_chunk(const HostBatch& hb, size_t p0, size_t p1, size_t g0, size_t g1, uint64_t a0, uint64_t a1);
  bool raw_staged_ = false;
  DevBatch db_;
  DevMatches m_;
  unsigned long long* chunk_base_d_ = nullptr;  // chunk c's first CSR position (written by chunk c-1's move)
  uint32_t* adv_h_ = nullptr;
  uint32_t* row_end_h_ = nullptr;
  uint32_t* adv_hd_ = nullptr;      // device addresses of adv_h_ / row_end_h_ (result-move stores)
  uint32_t* row_end_hd_ = nullptr;
  unsigned long long* ctl_h_ = nullptr;
  uint64_t cap_ = 0, h2d_ = 0, d2h_ = 0;
  uint64_t wire_bytes_ = 0;                       // size of wire_h_ / wire_d_
  uint64_t adv_units_ = 0, row_end_units_ = 0;    // 16-byte units of adv_h_ / row_end_h_ (guards)
  bool prepared_ = false;
  bool packed_ = false;  // no Engine pointer: the batch may outlive a hot swap (the C-ABI checks the generation)
};

}  // namespace tvm
