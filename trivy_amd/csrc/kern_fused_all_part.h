// One piece of the all-grammar fused_kernel table (kern_fused_all.hip): the variants of part
// TVM_ALL_PART, nullptr elsewhere.  Parts: 0 fused K=4, 1 fused K=2, 2 fused K=1, 3 per-wave
// sweep segments, 4 per-wave staging + segments (match_variants.h F / K).
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {
namespace {
constexpr int fused_all_part(int F, int K) {
  return F == 1 ? (K == 4 ? 0 : K == 2 ? 1 : 2) : F == 4 ? 3 : F == 5 ? 4 : 5 + F;
}
template <int F, int K, int MB>
constexpr FusedFn fused_all_entry() {
  if constexpr (fused_all_part(F, K) == TVM_ALL_PART) return fused_entry<GM_ALL, 2, F, K, MB>();
  else return nullptr;
}
}  // namespace

#define TVM_CAT2_(a, b) a##b
#define TVM_CAT_(a, b) TVM_CAT2_(a, b)
const FusedFn* TVM_CAT_(fused_table_ALL_p, TVM_ALL_PART)() {
#define TVM_FUSED_(F, K, MB, NAME) fused_all_entry<F, K, MB>(),
  static const FusedFn t[] = {TVM_MATCH_VARIANTS(TVM_FUSED_)};
#undef TVM_FUSED_
  return t;
}
}  // namespace tvm
