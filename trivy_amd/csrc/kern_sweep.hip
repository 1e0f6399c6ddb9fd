// Instantiates sweep_kernel for the split variants (match_variants.h), without row filters
// (dpkg-only batches) and with them (rpm / apk / library rows: RowAux predicates per package).
#include "match_kernel.h"
#include "match_variants.h"

namespace tvm {
const SweepFn* sweep_table(bool filt) {
#define TVM_PLAIN_(F, K, MB, NAME) F ? nullptr : &launch_sweep<K, MB, 0>,
#define TVM_FILT_(F, K, MB, NAME) F ? nullptr : &launch_sweep<K, MB, 2>,
  static const SweepFn plain[] = {TVM_MATCH_VARIANTS(TVM_PLAIN_)};
  static const SweepFn filt_[] = {TVM_MATCH_VARIANTS(TVM_FILT_)};
#undef TVM_PLAIN_
#undef TVM_FILT_
  return filt ? filt_ : plain;
}
}  // namespace tvm
