// Host-side parallel helpers for batch preparation (plain std::thread; no OpenMP runtime).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
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

// A process-wide pool of host_threads() - 1 parked threads for work that recurs many times
// per call (the pipeline's per-chunk staging copies: spawning threads per chunk cost more than
// the copies).  One job at a time; the caller takes part.  shutdown() (tvm_shutdown) joins the
// threads before the HIP runtime and the C++ runtime tear down; later jobs run on the caller.
class WorkerPool {
 public:
  static WorkerPool& get() {
    std::lock_guard<std::mutex> g(inst_mu());
    WorkerPool*& p = inst();
    if (!p) p = new WorkerPool(host_threads());  // never destroyed: shutdown() stops its threads
    return *p;
  }
  // Joins the threads of the pool if one exists (idempotent).
  static void shutdown_all() {
    WorkerPool* p;
    {
      std::lock_guard<std::mutex> g(inst_mu());
      p = inst();
    }
    if (p) p->shutdown();
  }
  int size() const { return n_ + 1; }
  // f(i) for i in [0, n), handed out one at a time
  void parallel_for(size_t n, const std::function<void(size_t)>& f) {
    if (n == 0) return;
    std::lock_guard<std::mutex> one(job_mu_);
    if (stopped_) {
      for (size_t i = 0; i < n; i++) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      total_ = n;
      next_.store(0, std::memory_order_relaxed);
      busy_ = n_;
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return busy_ == 0; });
    job_ = nullptr;
  }
  void shutdown() {
    std::lock_guard<std::mutex> one(job_mu_);  // no job in flight
    if (stopped_) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
    th_.clear();
    stopped_ = true;
  }

 private:
  explicit WorkerPool(int threads) : n_(std::max(0, threads - 1)) {
    for (int i = 0; i < n_; i++) th_.emplace_back([this] { loop(); });
  }
  static std::mutex& inst_mu() {
    static std::mutex* m = new std::mutex();
    return *m;
  }
  static WorkerPool*& inst() {
    static WorkerPool* p = nullptr;
    return p;
  }
  void work() {
    for (size_t i; (i = next_.fetch_add(1, std::memory_order_relaxed)) < total_;) (*job_)(i);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_cv_.notify_one();
    }
  }
  const int n_;
  std::vector<std::thread> th_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t total_ = 0;
  std::atomic<size_t> next_{0};
  int busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false, stopped_ = false;
};

// range_for on the parked WorkerPool threads (no thread start per call: the batch export's
// loops run a few milliseconds each).  Not from inside another WorkerPool job.
template <class F>
void pool_range_for(size_t n, size_t grain, F&& f) {
  WorkerPool& wp = WorkerPool::get();
  const size_t pieces = std::max<size_t>(1, std::min<size_t>(size_t(wp.size()) * 4, n / std::max<size_t>(grain, 1)));
  wp.parallel_for(pieces, [&](size_t k) { f(n * k / pieces, n * (k + 1) / pieces); });
}

}  // namespace tvm
