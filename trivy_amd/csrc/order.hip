// order_kernel (gfx950): a match pass's per-tile segments -> the per-package advisory
// lists in global (package, advisory) order, as CSR: csr_adv[] plus row_end[p] (package p's
// advisories are csr_adv[row_end[p-1] .. row_end[p]), row_end[-1] = 0).  This is the form
// the pipelined end-to-end path (pipeline.hip) copies back to the host.
//
// The match kernels place each tile's segment by one atomic reservation (no inter-tile
// waiting); here every tile's size is known when its workgroup starts (the tile
// directory), so a decoupled look-back over those sizes - publish the aggregate at once,
// sum the predecessors' words back to the first inclusive one - resolves every tile's
// global offset with hardly any waiting, and the tile copies its segment there.  Tiles take
// tickets, so a tile only ever waits on tiles that started before it.  Chunks of a
// pipelined pass run in order on one stream, so a chunk's first tile looks back into the
// previous chunk's (finished) tiles: offsets are global across chunks.
#include "pipeline.h"

namespace tvm {

namespace {

enum : unsigned long long { LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1 };

// Publish-then-look-back for tile t; the status words carry their values (one 8-B
// agent-scope atomic each, never torn), so no payload fence is needed.
__device__ __forceinline__ unsigned long long lookback(unsigned long long* status, uint32_t t, uint32_t agg) {
  if (t == 0) {
    __hip_atomic_store(&status[0], LB_INC | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0ull;
  }
  __hip_atomic_store(&status[t], LB_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long excl = 0;
  for (int64_t i = int64_t(t) - 1; i >= 0;) {
    const unsigned long long v = __hip_atomic_load(&status[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long f = v & ~LB_VAL;
    if (f == 0) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    excl += v & LB_VAL;
    if (f == LB_INC) break;
    i--;
  }
  __hip_atomic_store(&status[t], LB_INC | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

__global__ __launch_bounds__(kTile) void order_kernel(OrderArgs a) {
  __shared__ uint32_t cnt[kTile];
  __shared__ uint32_t wsum[kTile / 64];
  __shared__ uint32_t tile;
  __shared__ unsigned long long base;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) tile = a.t0 + uint32_t(atomicAdd(a.ticket, 1ull));
  cnt[tid] = 0;
  __syncthreads();
  const uint32_t t = tile;
  const TileDir d = a.dir[t];
  if (tid == 0) base = lookback(a.status, t, d.count);
  __syncthreads();
  // per-package counts of the segment (its entries are in package order)
  const uint32_t p_first = t * kTile;
  // an overflowed pass (matches > cap) left segments past the buffers: count nothing, copy
  // nothing out of bounds; the host sees the total and re-runs with a larger buffer
  const unsigned long long b = base;
  const bool fits = d.base + d.count <= a.cap && b + d.count <= a.cap;
  if (fits)
    for (uint32_t i = tid; i < d.count; i += kTile) atomicAdd(&cnt[a.pkg[d.base + i] - a.pkg_base - p_first], 1u);
  __syncthreads();
  if (fits)
    for (uint32_t i = tid; i < d.count; i += kTile) a.csr_adv[b + i] = a.adv[d.base + i];
  // row_end = base + inclusive scan of the counts
  const uint32_t c = cnt[tid];
  uint32_t x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= uint32_t(o)) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  uint32_t off = 0;
#pragma unroll
  for (int w = 0; w < kTile / 64; w++) off += (uint32_t(w) < wave) ? wsum[w] : 0u;
  const uint32_t p = p_first + tid;
  if (p < a.n) a.row_end[p] = uint32_t(b + off + x);
}

__global__ __launch_bounds__(kTile) void copy_out_kernel(CopyOutArgs a) {
  __shared__ uint4 lds[kCopyLdsWords / 4];
  copy_out_tiles(a, blockIdx.x, gridDim.x, reinterpret_cast<uint32_t*>(lds));
}

}  // namespace

void launch_order(uint32_t n_tiles, hipStream_t st, const OrderArgs& a) {
  hipLaunchKernelGGL(order_kernel, dim3(n_tiles), dim3(kTile), 0, st, a);
}

void launch_copy_out(hipStream_t st, const CopyOutArgs& a) {
  hipLaunchKernelGGL(copy_out_kernel, dim3(kCopyWorkgroups), dim3(kTile), 0, st, a);
}


}  // namespace tvm
