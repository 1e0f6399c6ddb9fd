// Block cache for per-batch device / pinned host buffers (pool.h).
#include "pool.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <iterator>
#include <map>
#include <mutex>
#include <new>
#include <unordered_map>

namespace tvm {

void* huge_alloc(size_t bytes);  // sbom.cpp: anonymous mappings advised for transparent huge pages
void huge_free(void* p, size_t bytes);

namespace {

// Free bytes kept per kind before blocks are really freed (a C2 pipeline holds ~0.5 GB of
// device and ~0.3 GB of pinned host buffers; two in flight fit comfortably).
constexpr size_t kKeepDevice = size_t(8) << 30;
constexpr size_t kKeepHost = size_t(4) << 30;

struct Kind {
  std::multimap<size_t, void*> free_;           // capacity -> block
  std::unordered_map<void*, size_t> cap_;       // every live or cached block's capacity
  size_t cached = 0;
};

struct Pool {
  std::mutex mu;
  std::map<int, Kind> dev;  // per device
  Kind host;
  Kind heap;  // pageable (pool_heap_*)
  unsigned long long hits = 0, misses = 0;
  bool closed = false;  // pool_close: blocks put back are freed at once
};

Pool& pool() {
  static Pool* p = new Pool();  // never destroyed: blocks may be put back during static teardown
  return *p;
}

// A cached block of capacity in [bytes, 2 * bytes + 1 MiB) (never a far larger one).
void* take(Kind& k, size_t bytes) {
  auto it = k.free_.lower_bound(bytes);
  if (it == k.free_.end() || it->first > 2 * bytes + (size_t(1) << 20)) return nullptr;
  void* p = it->second;
  k.cached -= it->first;
  k.free_.erase(it);
  return p;
}

// Really frees the largest cached blocks until at most `keep` bytes stay cached.
template <class FreeFn>
void shrink(Kind& k, size_t keep, FreeFn&& fr) {
  while (k.cached > keep && !k.free_.empty()) {
    auto it = std::prev(k.free_.end());
    k.cached -= it->first;
    fr(it->second);  // before its capacity is forgotten (the heap kind's free needs it)
    k.cap_.erase(it->second);
    k.free_.erase(it);
  }
}

size_t round_up(size_t b) { return (std::max<size_t>(b, 1) + 4095) & ~size_t(4095); }

}  // namespace

void* pool_device_get(int device, size_t bytes, const char* what, std::string& err) {
  Pool& P = pool();
  bytes = round_up(bytes);
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (void* p = take(P.dev[device], bytes)) {
      P.hits++;
      return p;
    }
    P.misses++;
  }
  void* p = nullptr;
  (void)hipSetDevice(device);
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    // memory held by the cache may be what is missing: give it back and try once more
    pool_trim();
    (void)hipSetDevice(device);
    e = hipMalloc(&p, bytes);
  }
  if (e != hipSuccess) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(P.mu);
  P.dev[device].cap_[p] = bytes;
  return p;
}

void pool_device_put(int device, void* p) {
  if (!p) return;
  Pool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  Kind& k = P.dev[device];
  auto it = k.cap_.find(p);
  if (it == k.cap_.end()) {  // not ours: free it directly
    (void)hipSetDevice(device);
    (void)hipFree(p);
    return;
  }
  k.free_.emplace(it->second, p);
  k.cached += it->second;
  shrink(k, P.closed ? 0 : kKeepDevice, [&](void* q) {
    (void)hipSetDevice(device);
    (void)hipFree(q);
  });
}

void* pool_host_get(size_t bytes, const char* what, std::string& err) {
  Pool& P = pool();
  bytes = round_up(bytes);
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (void* p = take(P.host, bytes)) {
      P.hits++;
      return p;
    }
    P.misses++;
  }
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    pool_trim();
    e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
  }
  if (e != hipSuccess) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(P.mu);
  P.host.cap_[p] = bytes;
  return p;
}

void pool_host_put(void* p) {
  if (!p) return;
  Pool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  auto it = P.host.cap_.find(p);
  if (it == P.host.cap_.end()) {
    (void)hipHostFree(p);
    return;
  }
  P.host.free_.emplace(it->second, p);
  P.host.cached += it->second;
  shrink(P.host, P.closed ? 0 : kKeepHost, [](void* q) { (void)hipHostFree(q); });
}

void* pool_heap_get(size_t bytes) {
  Pool& P = pool();
  bytes = round_up(bytes);
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (void* p = take(P.heap, bytes)) return p;
  }
  void* p = nullptr;
  try {  // huge_alloc throws on failure; the C-ABI callers get a null block (an error), not an exception
    p = huge_alloc(bytes);
  } catch (const std::bad_alloc&) {
    return nullptr;
  }
  if (!p) return nullptr;
  std::lock_guard<std::mutex> lk(P.mu);
  P.heap.cap_[p] = bytes;
  return p;
}

void pool_heap_put(void* p) {
  if (!p) return;
  Pool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  auto it = P.heap.cap_.find(p);
  if (it == P.heap.cap_.end()) return;
  P.heap.free_.emplace(it->second, p);
  P.heap.cached += it->second;
  shrink(P.heap, P.closed ? 0 : kKeepHost, [&](void* q) {
    auto c = P.heap.cap_.find(q);
    huge_free(q, c == P.heap.cap_.end() ? 0 : c->second);
  });
}

void pool_close() {
  {
    std::lock_guard<std::mutex> lk(pool().mu);
    pool().closed = true;
  }
  pool_trim();
}

void pool_trim() {
  Pool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  for (auto& [d, k] : P.dev)
    shrink(k, 0, [&, d = d](void* q) {
      (void)hipSetDevice(d);
      (void)hipFree(q);
    });
  shrink(P.host, 0, [](void* q) { (void)hipHostFree(q); });
  shrink(P.heap, 0, [&](void* q) {
    auto c = P.heap.cap_.find(q);
    huge_free(q, c == P.heap.cap_.end() ? 0 : c->second);
  });
}

void pool_stats(unsigned long long out[4]) {
  Pool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  unsigned long long d = 0;
  for (auto& [dv, k] : P.dev) d += k.cached;
  out[0] = d;
  out[1] = P.host.cached;
  out[2] = P.hits;
  out[3] = P.misses;
}

}  // namespace tvm
