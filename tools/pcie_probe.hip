// Host-link microbenchmark for the end-to-end path: how fast can a batch
// reach HBM and a match list leave it on this box?  Measures, for buffer sizes like C2's
// (136 MB up, 98 MB down):
//   h2d / d2h          one hipMemcpyAsync from / to pinned host memory (hipHostMalloc and
//                      hipHostRegister'ed pageable memory);
//   duplex             both at once on two streams (does the link run full-duplex?);
//   chunked            8 chunks each way on two streams;
//   zc_read / zc_write a kernel reading / writing pinned host memory directly (16 B per lane).
// Build: hipcc --offload-arch=gfx950 -O3 tools/pcie_probe.hip -o tools/pcie_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

__global__ void zc_read(const uint4* __restrict__ src, size_t n, uint4* __restrict__ sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const uint4 v = src[i];
    acc.x ^= v.x;
    acc.y ^= v.y;
    acc.z ^= v.z;
    acc.w ^= v.w;
  }
  if ((acc.x | acc.y | acc.z | acc.w) == 0x12345678u) sink[0] = acc;  // keeps the loads
}

__global__ void zc_write(uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    dst[i] = make_uint4(uint32_t(i), 1, 2, 3);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double best_of(int reps, F f) {
  double best = 1e30;
  for (int r = 0; r < reps; r++) {
    CK(hipDeviceSynchronize());
    const double t = now_ms();
    f();
    CK(hipDeviceSynchronize());
    best = std::min(best, now_ms() - t);
  }
  return best;
}

int main() {
  const size_t up = 136u << 20, down = 98u << 20;
  void *hu, *hd, *du, *dd, *sink;
  CK(hipHostMalloc(&hu, up, hipHostMallocDefault));
  CK(hipHostMalloc(&hd, down, hipHostMallocDefault));
  std::memset(hu, 1, up);
  std::memset(hd, 2, down);
  std::vector<char> pu(up, 3), pd(down, 4);
  CK(hipHostRegister(pu.data(), up, hipHostRegisterDefault));
  CK(hipHostRegister(pd.data(), down, hipHostRegisterDefault));
  CK(hipMalloc(&du, up));
  CK(hipMalloc(&dd, down));
  CK(hipMalloc(&sink, 64));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int R = 5;
  auto gbs = [](size_t b, double ms) { return b / (ms * 1e-3) / 1e9; };
  double t;
  t = best_of(R, [&] { CK(hipMemcpyAsync(du, hu, up, hipMemcpyHostToDevice, s1)); });
  std::printf("h2d hostmalloc   %7.3f ms  %6.1f GB/s\n", t, gbs(up, t));
  t = best_of(R, [&] { CK(hipMemcpyAsync(du, pu.data(), up, hipMemcpyHostToDevice, s1)); });
  std::printf("h2d registered   %7.3f ms  %6.1f GB/s\n", t, gbs(up, t));
  t = best_of(R, [&] { CK(hipMemcpyAsync(hd, dd, down, hipMemcpyDeviceToHost, s2)); });
  std::printf("d2h hostmalloc   %7.3f ms  %6.1f GB/s\n", t, gbs(down, t));
  t = best_of(R, [&] { CK(hipMemcpyAsync(pd.data(), dd, down, hipMemcpyDeviceToHost, s2)); });
  std::printf("d2h registered   %7.3f ms  %6.1f GB/s\n", t, gbs(down, t));
  t = best_of(R, [&] {
    CK(hipMemcpyAsync(du, hu, up, hipMemcpyHostToDevice, s1));
    CK(hipMemcpyAsync(hd, dd, down, hipMemcpyDeviceToHost, s2));
  });
  std::printf("duplex           %7.3f ms  %6.1f GB/s combined (h2d alone would take %.3f)\n", t, gbs(up + down, t),
              up / 55e9 * 1e3);
  t = best_of(R, [&] {
    for (int c = 0; c < 8; c++) {
      CK(hipMemcpyAsync(static_cast<char*>(du) + c * (up / 8), static_cast<char*>(hu) + c * (up / 8), up / 8,
                        hipMemcpyHostToDevice, s1));
      CK(hipMemcpyAsync(static_cast<char*>(hd) + c * (down / 8), static_cast<char*>(dd) + c * (down / 8), down / 8,
                        hipMemcpyDeviceToHost, s2));
    }
  });
  std::printf("duplex chunked8  %7.3f ms  %6.1f GB/s combined\n", t, gbs(up + down, t));
  void *zu = nullptr, *zd = nullptr;
  CK(hipHostGetDevicePointer(&zu, hu, 0));
  CK(hipHostGetDevicePointer(&zd, hd, 0));
  for (int blocks : {256, 1024, 4096}) {
    t = best_of(R, [&] { hipLaunchKernelGGL(zc_read, dim3(blocks), dim3(256), 0, s1, (const uint4*)zu, up / 16, (uint4*)sink); });
    std::printf("zc_read  %5d WG %7.3f ms  %6.1f GB/s\n", blocks, t, gbs(up, t));
    t = best_of(R, [&] { hipLaunchKernelGGL(zc_write, dim3(blocks), dim3(256), 0, s2, (uint4*)zd, down / 16); });
    std::printf("zc_write %5d WG %7.3f ms  %6.1f GB/s\n", blocks, t, gbs(down, t));
  }
  t = best_of(R, [&] {
    hipLaunchKernelGGL(zc_read, dim3(1024), dim3(256), 0, s1, (const uint4*)zu, up / 16, (uint4*)sink);
    hipLaunchKernelGGL(zc_write, dim3(1024), dim3(256), 0, s2, (uint4*)zd, down / 16);
  });
  std::printf("zc duplex        %7.3f ms  %6.1f GB/s combined\n", t, gbs(up + down, t));
  t = best_of(R, [&] {
    CK(hipMemcpyAsync(du, hu, up, hipMemcpyHostToDevice, s1));
    hipLaunchKernelGGL(zc_write, dim3(1024), dim3(256), 0, s2, (uint4*)zd, down / 16);
  });
  std::printf("dma h2d + zc d2h %7.3f ms  %6.1f GB/s combined\n", t, gbs(up + down, t));
  return 0;
}
