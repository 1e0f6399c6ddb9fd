// Instantiates probe_kernel for grammar set GM_ALL (libver.h): a batch whose platforms only
// use these grammars runs a probe kernel with only their encoders in it.
#include "match_kernel.h"

namespace tvm {
ProbeFn probe_fn_ALL() { return &launch_probe<GM_ALL>; }
}  // namespace tvm
