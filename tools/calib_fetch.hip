// Calibration of the rocprofv3 HBM counters (FETCH_SIZE / WRITE_SIZE) on the load and store
// shapes the match kernel uses (MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE counts half the
// bytes of 16-B/lane streaming reads; other widths are uncalibrated).  Measurement only - not
// part of the product.  Every kernel touches a known number of distinct bytes of a 2 GiB
// buffer (far beyond the 32 MiB of L2 and the 256 MiB Infinity Cache, re-initialised between
// kernels), once per byte:
//   k_stream16   16 B / lane, consecutive lanes consecutive (staging windows, slot heads)
//   k_stream8    8 B / lane consecutive (package words pk[])
//   k_stream4    4 B / lane consecutive (match columns, tile offsets)
//   k_row32      32 B / lane as two 16-B loads, consecutive rows (the sweep's Row reads)
//   k_slot64     64 B / lane as four 16-B loads at a random 64-B line (hash-slot probes)
//   k_row32r     32 B / lane at a random 32-B row of a 2 GiB table (scattered row reads)
//   k_store4     4 B / lane consecutive stores (the match list's pkg / adv columns)
//   k_store16    16 B / lane consecutive stores
// Output: one line per kernel with its byte count, for tools/calib_summary.py to divide the
// per-kernel FETCH_SIZE / WRITE_SIZE by.  Build: hipcc --offload-arch=gfx950 -O3 -o
// tools/calib_fetch tools/calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int kB = 256;

// every kernel folds what it loads into one word per lane (kept, so no load is dead)
__global__ __launch_bounds__(kB) void k_stream16(const uint4* __restrict__ a, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB) {
    const uint4 v = a[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(kB) void k_stream8(const uint2* __restrict__ a, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB) {
    const uint2 v = a[i];
    acc ^= v.x + v.y;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(kB) void k_stream4(const uint32_t* __restrict__ a, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB) acc ^= a[i];
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// n rows of 32 B; lane j of a wave reads row base + j (two 16-B loads, like match_kernel.h's Row)
__global__ __launch_bounds__(kB) void k_row32(const uint4* __restrict__ a, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB) {
    const uint4 v0 = a[2 * i], v1 = a[2 * i + 1];
    acc ^= v0.x + v0.w + v1.y + v1.z;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// permutation index: an odd multiplier modulo a power of two visits every line once
__device__ __forceinline__ uint64_t scatter(uint64_t i, uint64_t mask) { return (i * 0x9E3779B1ull) & mask; }

// n random 64-B lines, each read once (four 16-B loads, like a hash-slot probe)
__global__ __launch_bounds__(kB) void k_slot64(const uint4* __restrict__ a, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB) {
    const uint64_t s = scatter(i, n - 1);
    const uint4 v0 = a[4 * s], v1 = a[4 * s + 1], v2 = a[4 * s + 2], v3 = a[4 * s + 3];
    acc ^= v0.x + v1.y + v2.z + v3.w;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// n random 32-B rows, each read once
__global__ __launch_bounds__(kB) void k_row32r(const uint4* __restrict__ a, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB) {
    const uint64_t s = scatter(i, n - 1);
    const uint4 v0 = a[2 * s], v1 = a[2 * s + 1];
    acc ^= v0.x + v1.w;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(kB) void k_store4(uint32_t* __restrict__ a, uint64_t n) {
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB) a[i] = uint32_t(i);
}

__global__ __launch_bounds__(kB) void k_store16(uint4* __restrict__ a, uint64_t n) {
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kB)
    a[i] = make_uint4(uint32_t(i), 1, 2, 3);
}

__global__ void k_fill(uint4* a, uint64_t n, uint32_t seed) {  // evicts the caches between kernels
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    a[i] = make_uint4(uint32_t(i) ^ seed, seed, uint32_t(i >> 32), 7);
}

int main() {
  const uint64_t bytes = uint64_t(2) << 30;  // 2 GiB: 64x L2, 8x the Infinity Cache
  void* buf = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4096));
  const uint32_t grid = 256 * 32;  // 32 workgroups per CU
  auto refill = [&](uint32_t s) {
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(kB), 0, 0, static_cast<uint4*>(buf), bytes / 16, s);
    CK(hipDeviceSynchronize());
  };
  std::printf("kernel,bytes,shape\n");
  const uint64_t B = uint64_t(1) << 30;  // bytes each kernel touches (1 GiB)
  for (int rep = 0; rep < 2; rep++) {
    refill(1 + rep);
    hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(kB), 0, 0, static_cast<const uint4*>(buf), B / 16, sink);
    CK(hipDeviceSynchronize());
    refill(11 + rep);
    hipLaunchKernelGGL(k_stream8, dim3(grid), dim3(kB), 0, 0, static_cast<const uint2*>(buf), B / 8, sink);
    CK(hipDeviceSynchronize());
    refill(21 + rep);
    hipLaunchKernelGGL(k_stream4, dim3(grid), dim3(kB), 0, 0, static_cast<const uint32_t*>(buf), B / 4, sink);
    CK(hipDeviceSynchronize());
    refill(31 + rep);
    hipLaunchKernelGGL(k_row32, dim3(grid), dim3(kB), 0, 0, static_cast<const uint4*>(buf), B / 32, sink);
    CK(hipDeviceSynchronize());
    refill(41 + rep);
    hipLaunchKernelGGL(k_slot64, dim3(grid), dim3(kB), 0, 0, static_cast<const uint4*>(buf), B / 64, sink);
    CK(hipDeviceSynchronize());
    refill(51 + rep);
    hipLaunchKernelGGL(k_row32r, dim3(grid), dim3(kB), 0, 0, static_cast<const uint4*>(buf), B / 32, sink);
    CK(hipDeviceSynchronize());
    refill(61 + rep);
    hipLaunchKernelGGL(k_store4, dim3(grid), dim3(kB), 0, 0, static_cast<uint32_t*>(buf), B / 4);
    CK(hipDeviceSynchronize());
    refill(71 + rep);
    hipLaunchKernelGGL(k_store16, dim3(grid), dim3(kB), 0, 0, static_cast<uint4*>(buf), B / 16);
    CK(hipDeviceSynchronize());
  }
  for (const char* k : {"k_stream16", "k_stream8", "k_stream4", "k_row32", "k_slot64", "k_row32r", "k_store4",
                        "k_store16"})
    std::printf("%s,%llu,%s\n", k, (unsigned long long)B, "2 launches, each touching these bytes once");
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
