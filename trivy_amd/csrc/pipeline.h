// End-to-end pipelined match pass: a host batch (pinned) in, the per-package advisory lists
// (CSR, pinned) out, with the link transfers overlapping the kernels.
#pragma once
#include <string>
#include <vector>

#include "engine.h"

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
void launch_copy_out(hipStream_t st, const CopyOutArgs& a);  // engine.h copy_out_range as its own kernel


// One batch's pipeline state.  prepare() pins the batch's host arrays (hipHostRegister),
// sizes the device batch, the match buffers and the pinned result buffers; run() then
// streams the batch through in chunks of whole tiles:
//   copy stream    DMA of chunk c to HBM (package words, tile offsets, string bytes, attributes);
//   kernel stream  (after chunk c's upload) one match launch whose first workgroups move chunk
//                  c-1's result into the pinned host result (engine.h CopyOutArgs: 16-byte
//                  kernel stores, the link's other direction, range read on the device) while
//                  the rest match chunk c; then order_kernel over chunk c (CSR in HBM);
// so chunk c+1's upload and chunk c-1's result move run under chunk c's matching, and the
// host waits once, at the end.  (Measured alternatives, DESIGN.md §7: a DMA device-to-host
// copy runs at half the rate of kernel stores, and a result kernel on its own stream did
// not overlap the match kernels on this runtime.)
class Pipeline {
 public:
  ~Pipeline();
  bool prepare(Engine& eng, const HostBatch& hb, uint64_t match_cap, uint32_t chunk_packages, std::string& err);
  // One pass.  total = matches (> match_cap: nothing valid, re-prepare with a larger cap);
  // err_pkg = first poisoned package or -1.
  bool run(Engine& eng, const HostBatch& hb, uint64_t& total, int64_t& err_pkg, uint64_t& err_bits, std::string& err);
  const uint32_t* adv() const { return adv_h_; }
  const uint32_t* row_end() const { return row_end_h_; }
  uint64_t cap() const { return cap_; }
  uint64_t h2d_bytes() const { return h2d_; }
  uint64_t d2h_bytes() const { return d2h_; }
  uint32_t chunks() const { return uint32_t(bounds_.size() - 1); }

 private:
  void release();
  int dev_ = -1;
  hipStream_t s_h2d_ = nullptr, s_k_ = nullptr;
  std::vector<hipEvent_t> ev_h_;
  std::vector<uint32_t> bounds_;     // chunk c = tiles [bounds_[c], bounds_[c + 1])
  std::vector<uint64_t> toff_;       // tile offsets + the arena end (registered)
  std::vector<void*> registered_;
  DevBatch db_;
  DevMatches m_;
  unsigned long long* status_d_ = nullptr;
  unsigned long long* tickets_d_ = nullptr;
  uint32_t* adv_h_ = nullptr;
  uint32_t* row_end_h_ = nullptr;
  uint32_t* csr_adv_d_ = nullptr;   // device CSR (order_kernel)
  uint32_t* row_end_d_ = nullptr;
  uint32_t* adv_hd_ = nullptr;      // device addresses of adv_h_ / row_end_h_ (result-move stores)
  uint32_t* row_end_hd_ = nullptr;
  unsigned long long* ctl_h_ = nullptr;
  uint64_t cap_ = 0, h2d_ = 0, d2h_ = 0;
  bool prepared_ = false;  // no Engine pointer: the batch may outlive a hot swap (the C-ABI checks the generation)
};

}  // namespace tvm
