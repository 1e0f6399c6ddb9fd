// Host-side parallel helpers for batch preparation (plain std::thread; no OpenMP runtime).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <utility>
#include <vector>

namespace tvm {

// Host threads for batch preparation: TVM_HOST_THREADS, else OMP_NUM_THREADS (the box's CPU
// share), else the machine's, at most 64.
inline int host_threads() {
  for (const char* k : {"TVM_HOST_THREADS", "OMP_NUM_THREADS"})
    if (const char* v = std::getenv(k)) {
      const int n = std::atoi(v);
      if (n > 0) return std::min(n, 64);
    }
  const unsigned hc = std::thread::hardware_concurrency();
  return std::clamp<int>(int(hc ? hc : 1), 1, 64);
}

// f(t) on threads t = 0..n-1 (t = 0 on the caller)
template <class F>
void run_threads(int n, F&& f) {
  std::vector<std::thread> th;
  th.reserve(size_t(n > 1 ? n - 1 : 0));
  for (int t = 1; t < n; t++) th.emplace_back([&f, t] { f(t); });
  f(0);
  for (auto& x : th) x.join();
}

// f(i) for i in [0, n), items handed out one at a time to at most `threads` threads
template <class F>
void dynamic_for(int threads, size_t n, F&& f) {
  std::atomic<size_t> next{0};
  run_threads(std::min<int>(threads, int(std::max<size_t>(n, 1))), [&](int) {
    for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) f(i);
  });
}

// f(begin, end) over [0, n) cut into pieces of at least `grain` items
template <class F>
void range_for(size_t n, size_t grain, F&& f) {
  const size_t pieces = std::max<size_t>(1, std::min<size_t>(size_t(host_threads()) * 4, n / std::max<size_t>(grain, 1)));
  dynamic_for(host_threads(), pieces, [&](size_t k) { f(n * k / pieces, n * (k + 1) / pieces); });
}

// memcpy on the host threads (pinned staging of large batches)
inline void par_memcpy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kGrain = size_t(4) << 20;
  if (bytes < 2 * kGrain) {
    if (bytes) std::memcpy(dst, src, bytes);
    return;
  }
  range_for(bytes, kGrain, [&](size_t a, size_t b) {
    std::memcpy(static_cast<char*>(dst) + a, static_cast<const char*>(src) + a, b - a);
  });
}

}  // namespace tvm
