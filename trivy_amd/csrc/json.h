// Minimal strict JSON reader for trivy-db advisory values (host side of the flattener).
//
// Mirrors the parts of Go's encoding/json that decide whether a trivy-db value
// decodes (reference call site: trivy-db db.Config.GetAdvisories, used from
// pkg/detector/library/driver.go:114 and every OS driver's vs.Get): strict
// RFC 8259 syntax, invalid UTF-8 in strings replaced by U+FFFD, surrogate
// escapes combined (lone surrogates -> U+FFFD), trailing data rejected.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace tvm {

struct JVal {
  enum Kind : uint8_t { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  std::string s;                                   // Str: decoded; Num: literal text
  std::vector<JVal> arr;                           // Arr
  std::vector<std::pair<std::string, JVal>> obj;   // Obj, document order
  std::string_view raw;                            // exact source text of this value
};

// Parses `text` completely. Returns false and fills `err` on a syntax error.
bool json_parse(std::string_view text, JVal& out, std::string& err);

// Go json.Unmarshal of a JSON number into a Go `int` (64-bit): integer literal in range.
bool json_int(const JVal& v, int64_t& out);

// ASCII case-insensitive key match, as encoding/json's field lookup (ASCII subset).
bool json_key_eq(std::string_view key, std::string_view field);

}  // namespace tvm
