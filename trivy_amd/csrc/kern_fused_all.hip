// The all-grammar fused_kernel table (grammar set GM_ALL, libver.h; every fused variant of
// match_variants.h).  The instantiations are spread over kern_fused_all_p*.hip, one variant
// family per translation unit: with the Maven program evaluator inlined, one unit holding
// them all took 12 minutes to compile; in pieces they build in parallel.
#include "match_kernel.h"
#include "match_variants.h"

#include <vector>

namespace tvm {
const FusedFn* fused_table_ALL_p0();
const FusedFn* fused_table_ALL_p1();
const FusedFn* fused_table_ALL_p2();
const FusedFn* fused_table_ALL_p3();
const FusedFn* fused_table_ALL_p4();

const FusedFn* fused_table_ALL() {
  static const std::vector<FusedFn> t = [] {
    std::vector<FusedFn> v(kNumTuned, nullptr);
    for (const FusedFn* part : {fused_table_ALL_p0(), fused_table_ALL_p1(), fused_table_ALL_p2(), fused_table_ALL_p3(),
                                fused_table_ALL_p4()}) {
      for (int i = 0; i < kNumTuned; i++)
        if (part[i]) v[i] = part[i];
    }
    return v;
  }();
  return t.data();
}
}  // namespace tvm
