// Instantiates the ablation match-kernel variants for grammar set GM_OS (match_variants.h).
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {
const LaunchFn* launch_table_OS_ABLATION() {
#define TVM_LAUNCH_(T, KW, MB, KG, AB, NAME) &launch_one<T, KW, MB, KG, GM_OS, AB>,
  static const LaunchFn t[] = {TVM_ABLATION_VARIANTS(TVM_LAUNCH_)};
#undef TVM_LAUNCH_
  return t;
}
}  // namespace tvm
