// Instantiates fused_kernel for grammar set GM_LEAN (libver.h: every grammar but Maven and
// RubyGems, row filters without the Maven program evaluator) and every fused variant
// (match_variants.h).
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {
const FusedFn* fused_table_LEAN() {
#define TVM_FUSED_(F, K, MB, NAME) fused_entry<GM_LEAN, 1, F, K, MB>(),
  static const FusedFn t[] = {TVM_MATCH_VARIANTS(TVM_FUSED_)};
#undef TVM_FUSED_
  return t;
}
}  // namespace tvm
