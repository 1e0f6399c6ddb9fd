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

int pipeline_shape();

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
  // does hipMemcpyAsync return before the copy ran?  (host time of the call itself, with a
  // long result kernel queued on another stream)
  for (int reg = 0; reg < 2; reg++) {
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(zc_write, dim3(128), dim3(256), 0, s2, (uint4*)zd, down / 16);
    const double c0 = now_ms();
    CK(hipMemcpyAsync(du, reg ? (void*)pu.data() : hu, up / 8, hipMemcpyHostToDevice, s1));
    const double c1 = now_ms();
    CK(hipDeviceSynchronize());
    std::printf("hipMemcpyAsync H2D %s: call returned after %.3f ms (copy %.3f ms)\n",
                reg ? "registered" : "hostmalloc", c1 - c0, up / 8 / 57e9 * 1e3);
  }
  return pipeline_shape();
}

// ---- stream-concurrency check of the pipeline's shape (upload kernel -> compute -> result
// kernel per chunk on three streams joined by events) -------------------------------------
__global__ __launch_bounds__(256) void spin_kernel(long long cycles, uint32_t* out) {
  __shared__ uint32_t lds[6400];  // ~25 KB per workgroup, like the match kernel
  lds[threadIdx.x] = threadIdx.x;
  const long long t0 = clock64();
  uint32_t acc = 0;
  while (clock64() - t0 < cycles) acc += lds[(threadIdx.x + acc) & 255];
  if (acc == 0xFFFFFFFFu) out[0] = acc;
}

int pipeline_shape() {
  const int chunks = 8;
  const size_t up = (136u << 20) / chunks, down = (98u << 20) / chunks;
  void *hu, *hd, *du, *dd, *sink, *zu, *zd;
  CK(hipHostMalloc(&hu, up * chunks, hipHostMallocDefault));
  CK(hipHostMalloc(&hd, down * chunks, hipHostMallocDefault));
  CK(hipMalloc(&du, up * chunks));
  CK(hipMalloc(&dd, down * chunks));
  CK(hipMalloc(&sink, 64));
  CK(hipHostGetDevicePointer(&zu, hu, 0));
  CK(hipHostGetDevicePointer(&zd, hd, 0));
  hipStream_t s[3];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  std::vector<hipEvent_t> e1(chunks), e2(chunks);
  for (int c = 0; c < chunks; c++) {
    CK(hipEventCreateWithFlags(&e1[c], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2[c], hipEventDisableTiming));
  }
  const long long spin = 120000;  // cycles per workgroup
  auto rd = [&](int c, hipStream_t st) {
    hipLaunchKernelGGL(zc_read, dim3(256), dim3(256), 0, st, (const uint4*)((char*)zu + c * up), up / 16, (uint4*)sink);
  };
  auto wr = [&](int c, hipStream_t st) {
    hipLaunchKernelGGL(zc_write, dim3(128), dim3(256), 0, st, (uint4*)((char*)zd + c * down), down / 16);
  };
  auto sp = [&](hipStream_t st) { hipLaunchKernelGGL(spin_kernel, dim3(2048), dim3(256), 0, st, spin, (uint32_t*)sink); };
  double t;
  t = best_of(3, [&] { sp(s[1]); });
  std::printf("shape: spin alone            %7.3f ms\n", t);
  t = best_of(3, [&] { rd(0, s[0]); });
  std::printf("shape: one upload chunk      %7.3f ms\n", t);
  t = best_of(3, [&] { wr(0, s[2]); });
  std::printf("shape: one result chunk      %7.3f ms\n", t);
  t = best_of(3, [&] {
    for (int c = 0; c < chunks; c++) { rd(c, s[0]); sp(s[1]); wr(c, s[2]); }
  });
  std::printf("shape: 3 streams, no events  %7.3f ms\n", t);
  t = best_of(3, [&] {
    for (int c = 0; c < chunks; c++) {
      rd(c, s[0]);
      CK(hipEventRecord(e1[c], s[0]));
      CK(hipStreamWaitEvent(s[1], e1[c], 0));
      sp(s[1]);
      CK(hipEventRecord(e2[c], s[1]));
      CK(hipStreamWaitEvent(s[2], e2[c], 0));
      wr(c, s[2]);
    }
  });
  std::printf("shape: 3 streams + events    %7.3f ms\n", t);
  t = best_of(3, [&] {
    for (int c = 0; c < chunks; c++) {
      CK(hipMemcpyAsync((char*)du + c * up, (char*)hu + c * up, up, hipMemcpyHostToDevice, s[0]));
      CK(hipEventRecord(e1[c], s[0]));
      CK(hipStreamWaitEvent(s[1], e1[c], 0));
      sp(s[1]);
      CK(hipEventRecord(e2[c], s[1]));
      CK(hipStreamWaitEvent(s[2], e2[c], 0));
      wr(c, s[2]);
    }
  });
  std::printf("shape: DMA up + events       %7.3f ms\n", t);
  auto chain = [&](hipStream_t* q) {
    for (int c = 0; c < chunks; c++) {
      rd(c, q[0]);
      CK(hipEventRecord(e1[c], q[0]));
      CK(hipStreamWaitEvent(q[1], e1[c], 0));
      sp(q[1]);
      CK(hipEventRecord(e2[c], q[1]));
      CK(hipStreamWaitEvent(q[2], e2[c], 0));
      wr(c, q[2]);
    }
  };
  // copy streams at high priority
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t p[3];
  CK(hipStreamCreateWithPriority(&p[0], hipStreamNonBlocking, hi));
  CK(hipStreamCreateWithPriority(&p[1], hipStreamNonBlocking, lo));
  CK(hipStreamCreateWithPriority(&p[2], hipStreamNonBlocking, hi));
  t = best_of(3, [&] { chain(p); });
  std::printf("shape: events, copy streams high priority %7.3f ms (priorities %d..%d)\n", t, lo, hi);
  // copy streams on a few CUs, compute on the rest
  hipDeviceProp_t prop{};
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  for (int reserve : {8, 16, 32}) {
    std::vector<uint32_t> mu((ncu + 31) / 32, 0), md((ncu + 31) / 32, 0), mk((ncu + 31) / 32, 0);
    for (int i = 0; i < ncu; i++) {
      // reserved CUs spread over the XCDs (logical CU ids interleave across them); the
      // upload and result streams get disjoint halves (distinct masks = distinct queues)
      const int k = i % (ncu / reserve);
      (k == 0 ? ((i / (ncu / reserve)) % 2 ? md : mu) : mk)[i / 32] |= 1u << (i % 32);
    }
    hipStream_t m[3];
    CK(hipExtStreamCreateWithCUMask(&m[0], uint32_t(mu.size()), mu.data()));
    CK(hipExtStreamCreateWithCUMask(&m[1], uint32_t(mk.size()), mk.data()));
    CK(hipExtStreamCreateWithCUMask(&m[2], uint32_t(md.size()), md.data()));
    t = best_of(3, [&] { chain(m); });
    std::printf("shape: events, copies on %2d CUs / compute on %d %7.3f ms\n", reserve, ncu - reserve, t);
    t = best_of(3, [&] { sp(m[1]); });
    std::printf("       spin alone on the compute CUs %7.3f ms; ", t);
    t = best_of(3, [&] { wr(0, m[2]); });
    std::printf("result chunk on the copy CUs %7.3f ms; ", t);
    t = best_of(3, [&] { rd(0, m[0]); });
    std::printf("upload chunk %7.3f ms\n", t);
  }
  return 0;
}
