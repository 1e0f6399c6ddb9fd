// Match-path variants: X(FUSED, K pairs per lane per sweep round, MB LDS match-buffer
// entries, NAME).  FUSED = 1: probe and sweep of a tile in one kernel (kern_fused_*.hip, one
// translation unit per grammar set); 0: probe_kernel then sweep_kernel (kern_probe_*.hip,
// kern_sweep.hip).  engine.hip indexes the list in order; variant 0 ("auto") is
// kAutoVariant.
#pragma once

#define TVM_MATCH_VARIANTS(X)     \
  X(1, 2, 2048, "fused_k2_m2048") \
  X(1, 4, 2048, "fused_k4_m2048") \
  X(1, 1, 2048, "fused_k1_m2048") \
  X(0, 2, 2048, "split_k2_m2048") \
  X(0, 4, 2048, "split_k4_m2048")

#define TVM_VARIANT_COUNT_(F, K, MB, NAME) +1
constexpr int kNumTuned = 0 TVM_MATCH_VARIANTS(TVM_VARIANT_COUNT_);
#undef TVM_VARIANT_COUNT_

// Variant (index into the list) the engine launches by default.
constexpr int kAutoVariant = 1;  // fused_k4_m2048: fastest on C2 (bench.py --sweep, MI355X)
