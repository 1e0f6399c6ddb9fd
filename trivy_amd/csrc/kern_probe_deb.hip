// Instantiates probe_kernel for grammar set GM_DEB (libver.h): a batch whose platforms only
// use these grammars runs a probe kernel with only their encoders in it.
#include "match_kernel.h"

namespace tvm {
ProbeFn probe_fn_DEB() { return &launch_probe<GM_DEB>; }
#ifdef TVM_DIAG  // measurement builds only (make DIAG=1)
ProbeFn probe_fn_DEB_diag(int d) {
  return d == 1 ? &launch_probe<GM_DEB, 1> : d == 2 ? &launch_probe<GM_DEB, 2> : &launch_probe<GM_DEB, 3>;
}
#endif
}  // namespace tvm
