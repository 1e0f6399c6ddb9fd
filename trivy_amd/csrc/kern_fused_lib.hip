// Instantiates fused_kernel for the single-ecosystem library grammar sets (libver.h GM_NPM,
// GM_PEP, GM_GEN, GM_GEM, GM_MVN) in the filtered sets' auto variant (fused, K = 2, MB =
// 2048): a library batch's tiles are launched per grammar class (engine.hip), so a tile of
// npm or PyPI packages runs a kernel without the Maven / RubyGems parse arrays (no scratch).
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {
FusedFn fused_lib_fn(int cls) {
  static const FusedFn t[] = {
      fused_entry<GM_NPM, 1, 1, 2, 2048>(), fused_entry<GM_PEP, 1, 1, 2, 2048>(), fused_entry<GM_GEN, 1, 1, 2, 2048>(),
      fused_entry<GM_GEM, 1, 1, 2, 2048>(), fused_entry<GM_MVN, 2, 1, 2, 2048>()};
  return cls >= 0 && cls < int(sizeof(t) / sizeof(t[0])) ? t[cls] : nullptr;
}
}  // namespace tvm
