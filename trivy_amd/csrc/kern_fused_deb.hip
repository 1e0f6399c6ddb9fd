// Instantiates fused_kernel for grammar set GM_DEB (libver.h) and every fused variant
// (match_variants.h).
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {
const FusedFn* fused_table_DEB() {
#define TVM_FUSED_(F, K, MB, NAME) F ? &launch_fused<GM_DEB, K, MB, 0, (F >= 10 ? F - 10 : 0), TVM_FUSED_WPE(F)> : nullptr,
  static const FusedFn t[] = {TVM_MATCH_VARIANTS(TVM_FUSED_)};
#undef TVM_FUSED_
  return t;
}
}  // namespace tvm
