// Read-only bbolt file walker (bbolt.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <string_view>
#include <vector>

namespace tvm {

// path = bucket names from the root, then the record's key; return false to stop the walk.
using BboltVisit = std::function<bool(const std::vector<std::string_view>& path, std::string_view value)>;

// Every record of the file image, in bucket / key order.  false + err on a malformed file.
bool bbolt_walk(const uint8_t* bytes, size_t len, const BboltVisit& visit, std::string& err);

}  // namespace tvm
