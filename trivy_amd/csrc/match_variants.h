// Match-kernel variants: X(T tile packages, KW LDS key words per package, MB LDS match
// entries, KG installed keys in global memory, AB ablation, NAME).  Each list is
// instantiated for the three grammar sets (libver.h GM_DEB / GM_OS / GM_ALL) in its own
// translation unit (kern_*.hip); engine.hip indexes the tables in list order, tuned
// variants first, then ablations.
//
// Sweep on MI355X (bench.py --sweep, profiles/r01/sweep_*.txt): t256_k32_m1536 is the
// fastest for dpkg-only (C2) and library (C3) batches, t256_g64_m1536 for rpm/apk (C5);
// the others stay for the sweep and the every-variant parity tests.
#pragma once

#define TVM_TUNED_VARIANTS(X)                     \
  X(256, 4, 1536, false, 0, "t256_k32_m1536")     \
  X(256, 8, 1536, true, 0, "t256_g64_m1536")      \
  X(256, 8, 2048, false, 0, "t256_k64_m2048")     \
  X(256, 4, 2048, false, 0, "t256_k32_m2048")     \
  X(256, 6, 1536, false, 0, "t256_k48_m1536")     \
  X(256, 4, 1536, true, 0, "t256_g32_m1536")      \
  X(128, 4, 1024, false, 0, "t128_k32_m1024")

// AB (diagnostics only, wrong match lists by construction): 1 = stage+probe+encode+scan,
// 2 = no key compare, 3 = stage+encode+scan (no probe), 4 = stage+probe+scan (no encode).
#define TVM_ABLATION_VARIANTS(X)                  \
  X(256, 4, 1536, false, 1, "ablate_probe_only")  \
  X(256, 4, 1536, false, 2, "ablate_no_cmp")      \
  X(256, 4, 1536, false, 3, "ablate_encode_only") \
  X(256, 4, 1536, false, 4, "ablate_probe_no_encode")

#define TVM_VARIANT_COUNT_(T, KW, MB, KG, AB, NAME) +1
constexpr int kNumTuned = 0 TVM_TUNED_VARIANTS(TVM_VARIANT_COUNT_);
constexpr int kNumAblations = 0 TVM_ABLATION_VARIANTS(TVM_VARIANT_COUNT_);
#undef TVM_VARIANT_COUNT_

// Variant the engine launches by default for each grammar set (index into the tuned list).
constexpr int kAutoVariant[3] = {0 /* GM_DEB */, 1 /* GM_OS */, 0 /* GM_ALL */};
