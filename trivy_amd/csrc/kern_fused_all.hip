// Instantiates fused_kernel for grammar set GM_ALL (libver.h) and every fused variant
// (match_variants.h).
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {
const FusedFn* fused_table_ALL() {
#define TVM_FUSED_(F, K, MB, NAME) fused_entry<GM_ALL, 2, F, K, MB>(),
  static const FusedFn t[] = {TVM_MATCH_VARIANTS(TVM_FUSED_)};
#undef TVM_FUSED_
  return t;
}
}  // namespace tvm
