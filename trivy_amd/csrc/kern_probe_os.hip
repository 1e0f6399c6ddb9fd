// Instantiates probe_kernel for grammar set GM_OS (libver.h): a batch whose platforms only
// use these grammars runs a probe kernel with only their encoders in it.
#include "match_kernel.h"

namespace tvm {
ProbeFn probe_fn_OS() { return &launch_probe<GM_OS>; }
}  // namespace tvm
