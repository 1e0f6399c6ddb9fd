// HostBatch (engine.h): the host-side package batch.  Plain host code, kept out of the HIP
// translation units so the host-only tools (the sanitizer harnesses under tools/san/) link it.
#include <algorithm>

#include "engine.h"

namespace tvm {

// ---- HostBatch ------------------------------------------------------------------------------

void HostBatch::add(uint32_t plat, std::string_view name, std::string_view ver) {
  if (pk.size() % kGroup == 0) tile_off.push_back(arena.size());
  const size_t nl = std::min<size_t>(name.size(), 0xFFFF), vl = std::min<size_t>(ver.size(), 0xFFFF);
  pk.push_back(make_uint2(plat, uint32_t(nl) | (uint32_t(vl) << 16)));
  arena.insert(arena.end(), name.begin(), name.begin() + nl);
  arena.insert(arena.end(), ver.begin(), ver.begin() + vl);
  if (!attr.empty()) attr.push_back(make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu));
}

void HostBatch::add(uint32_t plat, std::string_view name, std::string_view ver, uint2 a) {
  if (attr.size() < pk.size()) attr.resize(pk.size(), make_uint2(PA_ARCH_NONE, 0xFFFFFFFFu));
  add(plat, name, ver);
  if (attr.size() < pk.size()) attr.push_back(a);
  else attr.back() = a;
}

uint64_t HostBatch::name_off(size_t i) const {
  const size_t t = i / kGroup;
  uint64_t o = tile_off[t];
  for (size_t j = t * kGroup; j < i; j++) o += (pk[j].y & 0xFFFFu) + (pk[j].y >> 16);
  return o;
}

void HostBatch::name_offsets(std::vector<uint64_t>& off) const {
  off.resize(pk.size());
  uint64_t o = 0;
  for (size_t j = 0; j < pk.size(); j++) {
    off[j] = o;
    o += (pk[j].y & 0xFFFFu) + (pk[j].y >> 16);
  }
}

std::string_view HostBatch::name(size_t i) const {
  return std::string_view(reinterpret_cast<const char*>(arena.data()) + name_off(i), pk[i].y & 0xFFFFu);
}

std::string_view HostBatch::version(size_t i) const {
  return std::string_view(reinterpret_cast<const char*>(arena.data()) + name_off(i) + (pk[i].y & 0xFFFFu),
                          pk[i].y >> 16);
}

void HostBatch::clear() {
  pk.clear();
  arena.clear();
  tile_off.clear();
  attr.clear();
  cpe_bits.clear();
  cpe_words = 0;
}

}  // namespace tvm
