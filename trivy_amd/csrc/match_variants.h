// Match-path variants: X(FUSED, K pairs per lane per sweep round, MB LDS match-buffer
// entries, NAME).  FUSED = 1 (10 + d: fused with measurement bits d, see fused_kernel): probe and sweep of a tile in one kernel (kern_fused_*.hip, one
// translation unit per grammar set); 0: probe_kernel then sweep_kernel (kern_probe_*.hip,
// kern_sweep.hip).  engine.hip indexes the list in order; variant 0 ("auto") is
// kAutoVariant.
#pragma once

#define TVM_MATCH_VARIANTS_PRODUCT(X)  \
  X(1, 4, 2048, "fused_k4_m2048")      \
  X(1, 2, 2048, "fused_k2_m2048")      \
  X(1, 1, 2048, "fused_k1_m2048")      \
  X(0, 2, 2048, "split_k2_m2048")      \
  X(0, 4, 2048, "split_k4_m2048")      \
  X(4, 4, 2400, "fused_k4_m2400_seg")  \
  X(5, 4, 2400, "fused_k4_m2400_wseg")  \
  X(6, 2, 2400, "fused_k2_m2400_wseg6") \
  X(6, 3, 2400, "fused_k3_m2400_wseg6")

// Measurement-only variants (wrong match lists by construction): built only with
// `make DIAG=1` (-DTVM_DIAG), never reachable in the product library.
#ifdef TVM_DIAG
#define TVM_MATCH_VARIANTS(X)      \
  TVM_MATCH_VARIANTS_PRODUCT(X)    \
  X(11, 4, 2048, "diag_no_encode") \
  X(12, 4, 2048, "diag_no_probe")  \
  X(14, 4, 2048, "diag_no_sweep")  \
  X(15, 4, 2048, "diag_stage_only")
#else
#define TVM_MATCH_VARIANTS(X) TVM_MATCH_VARIANTS_PRODUCT(X)
#endif

// Measured and dropped (round 5): F = 5 as a persistent kernel that loads the next tile's package
// words, offsets and string window during the sweep - C2 0.467 -> 0.634 ms, C5 2.39 -> 4.53 ms.
// Fused F = 2 / 3: the same kernel compiled for at least 6 / 8 waves per SIMD (register cap;
// measured within 1 % on C2, rounds 2-3, not in the list any more).
#define TVM_FUSED_WPE(F) ((F) == 2 ? 6 : (F) == 3 ? 8 : 1)

#define TVM_VARIANT_COUNT_(F, K, MB, NAME) +1
constexpr int kNumTuned = 0 TVM_MATCH_VARIANTS(TVM_VARIANT_COUNT_);
#undef TVM_VARIANT_COUNT_

// Variant (index into the list) the engine launches by default.
// bench.py --sweep on MI355X (profiles/r03/sweep_c2.txt, sweep_c3.txt): per-wave staging +
// sweep segments are fastest for dpkg-only batches (C2 0.485 -> 0.469 ms); for the filtered
// grammar sets (rpm/apk/library rows, uneven per-pair cost) the shared K=2 sweep stays fastest
// (C3 0.257 ms against 0.34-0.36 ms in segments).
constexpr int kAutoVariant = 6;          // fused_k4_m2400_wseg
constexpr int kAutoVariantFiltered = 1;  // fused_k2_m2048
// OS grammar sets with row filters (rpm / apk: no library rows): per-wave staging + segments
// at 6 waves, K = 2 (round 5 sweep, profiles/r05/sweep_c5.txt: C5 2.317 -> 2.283 ms)
constexpr int kAutoVariantOS = 7;        // fused_k2_m2400_wseg6
// library grammar sets without Maven / RubyGems (GM_LEAN): per-wave staging + segments at 6
// waves, K = 2, as the OS set (round 6 sweep, go / npm / PEP 440 at 1M packages: fused K = 2
// 0.1354 ms, wseg6 K = 2 0.1333, K = 3 0.1331; the all-grammar kernel 0.149;
// profiles/r06/lean_ab/)
constexpr int kAutoVariantLean = 7;  // fused_k2_m2400_wseg6
