// Part 5 of the all-grammar fused_kernel table (kern_fused_all_part.h).
#define TVM_ALL_PART 5
#include "kern_fused_all_part.h"
