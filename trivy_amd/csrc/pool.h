// Process-wide cache of device and pinned host blocks for per-batch buffers.
//
// A fleet scan hands over a fresh batch every few milliseconds (pkg/scanner/local/scan.go:170
// per target, many concurrent callers).  hipMalloc / hipHostMalloc of a batch's buffers cost
// milliseconds (page pinning), and hipFree / hipHostFree synchronise the whole device, which
// would serialise a batch being prepared against the previous one still running.  Blocks are
// therefore returned to this cache when a batch or pipeline is released and handed to the next
// one of a similar size; the cache keeps at most a bounded number of free bytes per kind.
// The caller must have drained every stream that used a block before putting it back.
#pragma once
#include <cstddef>
#include <string>

namespace tvm {

// bytes >= 1; `what` names the buffer in the error message.
void* pool_device_get(int device, size_t bytes, const char* what, std::string& err);
void pool_device_put(int device, void* p);
void* pool_host_get(size_t bytes, const char* what, std::string& err);  // pinned, device-mapped
void pool_host_put(void* p);
// Pageable host blocks (huge-page mappings) for what only the host reads and writes: the CSR
// a pass decodes its result into (pinned memory is no place for a CPU loop's stores).
void* pool_heap_get(size_t bytes);
void pool_heap_put(void* p);
// Frees every cached block (tests; a process that wants its memory back).
void pool_trim();
// pool_trim, and from now on blocks put back are freed at once (tvm_shutdown: nothing of ours
// may be left for the HIP runtime's own teardown).
void pool_close();
// {cached device bytes, cached host bytes, hits, misses}
void pool_stats(unsigned long long out[4]);

}  // namespace tvm
