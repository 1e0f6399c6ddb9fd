// Part 4 of the all-grammar fused_kernel table (kern_fused_all_part.h).
#define TVM_ALL_PART 4
#include "kern_fused_all_part.h"
