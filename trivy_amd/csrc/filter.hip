// result.Filter for a batch of results on the GPU (gfx950): the vulnerability part of
// pkg/result/filter.go:60-139 over a batch's device match list, after FillInfo.
//
// Reference semantics per Result (= one tvm_batch_add* call):
//   filter.go:104-114   drop by severity ("" counts as UNKNOWN) and by ignored status;
//   filter.go:117-122   drop what the ignore file matches (MatchVulnerability: ID, paths
//                       against Target then PkgPath, PURLs) into ModifiedFindings;
//   filter.go:124-130   dedup on "vulnID/pkgName/installed/pkgPath": the greater
//                       FixedVersion string wins (shouldOverwrite, :345-348), ties keep
//                       the first seen;
//   filter.go:51-53     the VEX filter over the deduplicated list;
//   filter.go:77        sort.Sort(types.BySeverity) (pkg/types/vulnerability.go:41-58):
//                       PkgName, InstalledVersion, severity descending, VulnerabilityID,
//                       PkgPath.
// Strings are ranks fixed before the launch: every advisory's vulnerability ID and output
// FixedVersion (load time, vulninfo.cpp), every package's place in its result's
// (PkgName, InstalledVersion, PkgPath) order (host, once per batch: FilterPackages).
//
// The match list arrives grouped by package (each tile's segment is in package order, a
// package's advisories in trivy-db Get order), so no sort is needed:
//   filter_mark    per pair: severity / status; ignore rules (one hash-set probe per rule
//                  kind, smallest precedence wins); run bounds of every package and whether
//                  its IDs are strictly increasing;
//   filter_select  dedup: a pair of a package whose dedup key repeats looks the ID up in the
//                  runs of the other packages of that key (bisection of an ID-sorted run) and
//                  loses to a greater FixedVersion or an equal one seen first; then - only in
//                  runs whose IDs are not strictly increasing (one ID from two data sources,
//                  Red Hat's per-RHSA rows) - the first of the package's own pairs with the
//                  greatest FixedVersion; then the per-package class counters (survivors per
//                  severity, ignored) from wave ballots: a package whose run lies inside one
//                  64-pair wave segment stores them, one spread over several adds them
//                  atomically;
//   vex_mark       VEX statements drop survivors (and take them off the counters);
//   scans          survivor offsets of the package groups in perm order, ignored offsets
//                  in package order;
//   (round 4 counted in a kernel of its own, filter_count, and deduplicated through a hash
//   table sized after a host synchronisation; both are gone)
//   filter_place   a survivor of a package alone in its group whose run is ID-sorted (the
//                  bucket order of one trivy-db key: the common case) is placed in O(1):
//                  group offset + the package's survivors of higher severity + its
//                  same-severity survivors before it in the run (a block-wide prefix count
//                  over the 256-pair chunk plus, for the run that enters the chunk, the
//                  count over its earlier pairs); groups of several packages (same PkgName
//                  and InstalledVersion) and unsorted runs count keys over the group's runs;
//                  ignored findings go to their package's offset + their rank in the run
//                  (detection order).
// Integer work bound by HBM traffic (pairs, decisions, ranks); no MFMA.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "vulninfo.h"

namespace tvm {

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;       // key of a dropped pair / no precedence
constexpr unsigned long long kNoKey = ~0ull;   // empty rule-table slot
constexpr int kClasses = 6;                    // per-package counters: survivors of severity 0..4, ignored
constexpr int kIgnClass = 5;
constexpr int kCntStride = 8;                  // words per package counter record (32 B: whole-sector stores)
constexpr int kNoClass = 7;
constexpr int kChunkBits = 10;                 // packed in-chunk counters (chunk = kBlock pairs)
// Per-package flag bits: static (set_packages) FL_DUP / FL_SINGLE, per call FL_UNS (mark),
// FL_PKG / FL_VEX (rules_insert: the package has per-package rules, probe only those).
enum : uint32_t { FL_DUP = 1, FL_UNS = 2, FL_PKG = 4, FL_VEX = 8, FL_SINGLE = 16 };

// filter_select and filter_place give each wave a chunk of its own: kSpan pairs, kUS
// segments of 64 (pair s0 + k * 64 + lane), no workgroup barrier.  A package whose run crosses
// a chunk boundary leaves an edge record per chunk, which filter_edges turns into its counters
// and the chunks' entering-run carries.
constexpr int kUS = 4;
constexpr uint32_t kSpan = uint32_t(kUS) * 64;
// Edge record of a chunk: the package entering it (run started before the chunk) and the
// package leaving it (run goes on past its end), with their classes inside the chunk; a
// package spanning the whole chunk is both (in == out, counts in c_in).
struct Edge {
  uint32_t p_in, p_out;
  uint32_t c_in[kClasses], c_out[kClasses];
};

// Sets flag bits of package p in a byte array padded to whole words (word atomics).
__device__ __forceinline__ void set_flag(uint8_t* fl, uint32_t p, uint32_t bits) {
  atomicOr(reinterpret_cast<unsigned int*>(fl + (p & ~3u)), bits << (8 * (p & 3u)));
}

struct FilterArgs {
  FillDev t;
  const uint32_t* pkg;  // the match list (package, advisory columns), grouped by package
  const uint32_t* adv;
  const uint2* side;  // FillInfo's hand-off word per pair: {ID rank, severity index | status << 8}
  uint64_t n;
  uint32_t n_pkgs;
  // per package (FilterPackages)
  const uint32_t* perm;
  const uint32_t* grp_b;
  const uint32_t* grp_e;
  const uint32_t* dkey;
  const uint32_t* prank;
  const uint32_t* dk_b;  // perm range of the package's dedup key (FL_DUP packages)
  const uint32_t* dk_e;
  const uint8_t* dup;   // static flags: FL_DUP | FL_SINGLE
  const uint32_t* pkg_class;
  // per package, per call
  uint8_t* fl;         // per-call flags (FL_*), seeded from the static ones
  uint32_t* run_b;     // the package's pairs are [run_b, run_e) of the list
  uint32_t* run_e;
  uint32_t* cnt;       // kClasses counters per package (records of kCntStride words)
  uint32_t* surv;      // per package: its survivors (counters 0..4 summed), what the placement scan reads
  const uint32_t* off;      // survivor offset of perm position j (exclusive scan)
  const uint32_t* ign_off;  // ignored offset of package p
  // per pair
  uint32_t* mkey;  // after filter_mark: (4 - severity) << id_bits | ID rank, or kEmpty
  uint32_t* skey;  // after filter_select: the survivors' mkey, else kEmpty
  uint32_t* ign;   // precedence of the ignoring rule, kEmpty = not ignored
  uint8_t* pcls;   // after filter_select: the pair's counter class (pair_class)
  // tables
  const unsigned long long* rules;  // {key, precedence} x 2^k
  uint64_t rule_mask;
  uint32_t kinds;  // bit k: rules of tag k exist
  uint32_t sev_mask, status_mask, id_bits;
  uint2* out;      // survivors in report order
  uint32_t* iout;  // ignored {package, advisory, finding} in detection order
  Edge* edge;      // per select chunk
  uint32_t* carry_in;  // per chunk, kClasses: the entering run's classes before the chunk
  uint32_t diag;   // TVM_FILTER_DIAG (measurement): bit 0 no counters in select, bit 1 no dedup,
                   // bit 5 no slow placements, bit 6 no entering-run carry
};

__device__ __forceinline__ uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h;
}

// Precedence stored for a rule key (kEmpty when the set lacks it).
__device__ __forceinline__ uint32_t rule_find(const FilterArgs& a, unsigned long long key) {
  for (uint64_t s = mix64(key) & a.rule_mask;; s = (s + 1) & a.rule_mask) {
    const unsigned long long k = a.rules[2 * s];
    if (k == key) return uint32_t(a.rules[2 * s + 1]);
    if (k == kNoKey) return kEmpty;
  }
}

__device__ __forceinline__ unsigned long long rule_key(uint64_t tag, uint32_t subject, uint32_t rank) {
  return (tag << 62) | (uint64_t(subject) << 32) | rank;
}

// The counter class of a pair after filter_select.
__device__ __forceinline__ uint32_t pair_class(const FilterArgs& a, uint32_t skey, uint64_t i) {
  if (skey != kEmpty) return 4u - (skey >> a.id_bits);
  if ((a.kinds & 7u) && a.ign[i] != kEmpty) return kIgnClass;
  return kNoClass;
}

// Rule lists as uploaded: entry e of list k is (subject, ID index, precedence).
struct RuleDev {
  const uint32_t* subject[4];
  const uint32_t* id[4];
  const uint32_t* prec[4];
  const uint32_t* rank[4];
  uint64_t end[4];  // cumulative entry counts
  uint32_t tag[4];
  int n_lists;
};

__global__ __launch_bounds__(kBlock) void rules_insert(RuleDev r, unsigned long long* table, uint64_t mask,
                                                       uint8_t* fl) {
  const uint64_t g = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  int k = 0;
  while (k < r.n_lists && g >= r.end[k]) k++;
  if (k == r.n_lists) return;
  const uint64_t e = g - (k ? r.end[k - 1] : 0);
  const uint32_t rank = r.rank[k][r.id[k][e]];
  if (rank == kEmpty) return;  // an ID no advisory has: nothing to match
  const uint32_t subject = r.subject[k] ? r.subject[k][e] : 0u;
  const uint32_t prec = r.prec[k] ? r.prec[k][e] : 0u;
  const unsigned long long key = rule_key(r.tag[k], subject, rank);
  if (r.tag[k] == RULE_PKG || r.tag[k] == RULE_VEX)  // flag the subject package: probe only those
    set_flag(fl, subject, r.tag[k] == RULE_PKG ? FL_PKG : FL_VEX);
  for (uint64_t s = mix64(key) & mask;; s = (s + 1) & mask) {
    const unsigned long long prev = atomicCAS(&table[2 * s], kNoKey, key);
    if (prev == kNoKey || prev == key) {
      atomicMin(reinterpret_cast<unsigned int*>(&table[2 * s + 1]), prec);
      return;
    }
  }
}

// VEX (applied after the dedup, to survivors, as filter.go:51-53 does): each statement
// finds its package's run of the list (filter_mark's run_b / run_e; the list is grouped by
// package), bisects it for the ID (runs are ID-sorted unless FL_UNS) and drops that pair if
// filter_select kept it - no hash probe per survivor.  run_b of a package without pairs is
// stale: a start is taken only where it really is the first pair of that package.  The
// statements' indices are checked here rather than by a host scan before the call (*bad).
__global__ __launch_bounds__(kBlock) void vex_mark(RuleDev r, const uint32_t* pkg, const uint2* side,
                                                   const uint32_t* run_b, const uint32_t* run_e, const uint8_t* fl,
                                                   uint64_t n, uint32_t n_pkgs, uint32_t n_ids, uint32_t* skey,
                                                   uint8_t* pcls, uint32_t* cnt, uint32_t* surv, uint32_t* carry_in,
                                                   uint32_t* bad) {
  const uint64_t g = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  int k = 0;
  while (k < r.n_lists && g >= r.end[k]) k++;
  if (k == r.n_lists) return;
  const uint64_t e = g - (k ? r.end[k - 1] : 0);
  const uint32_t idx = r.id[k][e], p = r.subject[k][e];
  if (idx >= n_ids || p >= n_pkgs) {
    atomicOr(bad, 1u);
    return;
  }
  const uint32_t rank = r.rank[k][idx];
  if (rank == kEmpty) return;
  const uint32_t rb = run_b[p];
  if (rb >= n || pkg[rb] != p || (rb && pkg[rb - 1] == p)) return;  // no pairs (stale start)
  const uint32_t re = run_e[p];  // written by this call's filter_mark, as rb was
  auto drop = [&](uint32_t j) {
    if (skey[j] != kEmpty) {  // a survivor (so not ignored): it leaves every counter class
      const uint32_t c = pcls[j];
      atomicSub(&cnt[uint64_t(p) * kCntStride + c], 1u);
      atomicSub(&surv[p], 1u);
      // and the entering-run carries of the later chunks its run reaches (filter_place)
      for (uint64_t h = j / kSpan + 1; h * kSpan < re; h++) atomicSub(&carry_in[h * kClasses + c], 1u);
      skey[j] = kEmpty;
      pcls[j] = uint8_t(kNoClass);
    }
  };
  if (fl[p] & FL_UNS) {  // IDs not increasing along the run (two data sources of one ID): every pair
    for (uint32_t j = rb; j < re; j++)
      if (side[j].x == rank) drop(j);
    return;
  }
  uint32_t lo = rb, hi = re;  // strictly increasing IDs: the one pair, by bisection (runs can be thousands long)
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (side[mid].x < rank) lo = mid + 1;
    else hi = mid;
  }
  if (lo < re && side[lo].x == rank) drop(lo);
}

// Pairs per thread per step of the streaming kernels: every lane issues the loads of kU
// pairs (coalesced, kBlock apart) before it uses any, so kU gathers of per-package state
// are in flight together instead of one dependent chain per pair.
constexpr int kU = 8;

__global__ __launch_bounds__(kBlock) void filter_mark(FilterArgs a) {
  const uint64_t stride = uint64_t(gridDim.x) * kBlock * kU;
  const uint64_t n = a.n;
  for (uint64_t b0 = uint64_t(blockIdx.x) * kBlock * kU; b0 < n; b0 += stride) {
    uint32_t p[kU], pp[kU], pn[kU], f[kU];
    uint2 sd[kU];
    uint32_t vprev[kU];
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const uint64_t i = min(b0 + uint64_t(k) * kBlock + threadIdx.x, n - 1);
      p[k] = a.pkg[i];
      sd[k] = a.side[i];
      // the neighbours' words come from the neighbouring lanes; only the wave's edge lanes load
      pp[k] = (lane == 0 && i) ? a.pkg[i - 1] : 0xFFFFFFFFu;
      vprev[k] = (lane == 0 && i) ? a.side[i - 1].x : 0u;
      pn[k] = (lane == 63 && i + 1 < n) ? a.pkg[i + 1] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const uint64_t i = min(b0 + uint64_t(k) * kBlock + threadIdx.x, n - 1);
      const uint32_t up = __shfl_up(p[k], 1, 64), vup = __shfl_up(sd[k].x, 1, 64), dn = __shfl_down(p[k], 1, 64);
      if (lane != 0) {
        pp[k] = up;
        vprev[k] = vup;
      }
      if (lane != 63) pn[k] = i + 1 < n ? dn : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < kU; k++) f[k] = a.fl[p[k]];
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const uint64_t i = b0 + uint64_t(k) * kBlock + threadIdx.x;
      if (i >= n) break;
      const uint32_t pk = p[k];
      const uint32_t vr = sd[k].x, sev = sd[k].y & 0xFFu;
      // run bounds (the list is grouped by package) and whether the run is ID-sorted
      // run bounds only for the packages whose pairs are looked up by package: dedup (FL_DUP),
      // groups of several packages, and with VEX statements (vex_mark) every package
      const bool bounds = (a.kinds & (1u << RULE_VEX)) || (f[k] & FL_DUP) || !(f[k] & FL_SINGLE);
      if (pp[k] != pk) {
        if (bounds) a.run_b[pk] = uint32_t(i);
      } else if (vprev[k] >= vr && !(f[k] & FL_UNS)) {
        set_flag(a.fl, pk, FL_UNS);
      }
      if (pn[k] != pk && bounds) a.run_e[pk] = uint32_t(i + 1);
      bool keep = ((a.sev_mask >> sev) & 1u) && !((a.status_mask >> ((sd[k].y >> 8) & 31u)) & 1u);
      if (a.kinds & 7u) {  // ignore rules: the smallest precedence is the finding Match returns
        uint32_t prec = kEmpty;
        if (keep) {  // severity / status drop first (filter.go:108-114), silently
          if (a.kinds & (1u << RULE_ALL)) prec = min(prec, rule_find(a, rule_key(RULE_ALL, 0, vr)));
          if ((a.kinds & (1u << RULE_PKG)) && (f[k] & FL_PKG)) prec = min(prec, rule_find(a, rule_key(RULE_PKG, pk, vr)));
          if (a.kinds & (1u << RULE_CLS)) prec = min(prec, rule_find(a, rule_key(RULE_CLS, a.pkg_class[pk], vr)));
          keep = prec == kEmpty;
        }
        a.ign[i] = prec;
      }
      a.mkey[i] = keep ? ((4u - sev) << a.id_bits) | vr : kEmpty;
    }
  }
}

// Does package q hold a kept pair of vulnerability rank vr whose FixedVersion rank beats fr
// (greater, or equal with q seen first)?  q's run: bisection when its IDs are strictly
// increasing, else a walk.  A package without pairs has a stale run start (rejected).
__device__ __forceinline__ bool beaten_by(const FilterArgs& a, uint32_t q, uint32_t vr, uint32_t fr, bool q_first) {
  const uint32_t rb = a.run_b[q];
  if (rb >= a.n || a.pkg[rb] != q || (rb && a.pkg[rb - 1] == q)) return false;
  uint32_t lo = rb, hi = a.run_e[q];
  if (!(a.fl[q] & FL_UNS)) {
    uint32_t l = lo, h = hi;
    while (l < h) {
      const uint32_t mid = (l + h) >> 1;
      if (a.side[mid].x < vr) l = mid + 1;
      else h = mid;
    }
    lo = l;
    hi = min(hi, l + 1);
  }
  for (uint32_t j = lo; j < hi; j++) {
    if (a.side[j].x != vr || a.mkey[j] == kEmpty) continue;
    const uint32_t fj = a.t.adv_rank[a.adv[j]].y;
    if (fj > fr || (fj == fr && q_first)) return true;
  }
  return false;
}

// A package's counter record (every class, zeros included: whole 32-B sectors) and its
// survivor sum.
// Runs inside one chunk need only the sum: filter_place counts their classes from the chunk's
// prefixes (the records are kept when ignore rules need the ignored counts of every package).
__device__ __forceinline__ void store_sum(const FilterArgs& a, uint32_t p, const uint32_t* cc, uint32_t sum) {
  if (a.kinds & 7u) {
    uint4* o = reinterpret_cast<uint4*>(a.cnt + uint64_t(p) * kCntStride);
    o[0] = make_uint4(cc[0], cc[1], cc[2], cc[3]);
    o[1] = make_uint4(cc[4], cc[5], 0u, 0u);
  }
  a.surv[p] = sum;
}

__device__ __forceinline__ void store_counts(const FilterArgs& a, uint32_t p, const uint32_t* cc, uint32_t sum) {
  uint4* o = reinterpret_cast<uint4*>(a.cnt + uint64_t(p) * kCntStride);
  o[0] = make_uint4(cc[0], cc[1], cc[2], cc[3]);
  o[1] = make_uint4(cc[4], cc[5], 0u, 0u);
  a.surv[p] = sum;
}

// LDS slots of filter_select's split runs, per wave: one per 64-pair segment boundary of the
// chunk (+ the chunk's start): classes, survivor sum, package.
constexpr int kSlots = kUS + 1;

__device__ __forceinline__ void lds_order() {  // the wave's own LDS traffic, in program order
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kBlock) void filter_select(FilterArgs a) {
  __shared__ uint32_t lslot_all[kBlock / 64][kSlots][kClasses + 2];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t g = uint64_t(blockIdx.x) * (kBlock / 64) + wave;  // this wave's chunk
  const uint64_t n = a.n, s0 = g * kSpan;
  if (s0 >= n) return;  // whole wave
  uint32_t (*lslot)[kClasses + 2] = lslot_all[wave];
  if (lane < uint32_t(kSlots)) {
#pragma unroll
    for (int c = 0; c < kClasses + 1; c++) lslot[lane][c] = 0;
    lslot[lane][kClasses + 1] = kEmpty;
  }
  const uint32_t id_mask = (1u << a.id_bits) - 1u;
  uint32_t pv[kUS], kv[kUS], fv[kUS], pe[kUS], ne[kUS];
#pragma unroll
  for (int k = 0; k < kUS; k++) {
    const uint64_t sk = s0 + uint64_t(k) * 64, i = min(sk + lane, n - 1);
    pv[k] = a.pkg[i];
    kv[k] = a.mkey[i];
    // the packages just before and after the segment (edge lanes)
    pe[k] = (lane == 0 && sk > 0) ? a.pkg[sk - 1] : 0xFFFFFFFFu;
    ne[k] = (lane == 63 && sk + 64 < n) ? a.pkg[sk + 64] : 0xFFFFFFFFu;
  }
#pragma unroll
  for (int k = 0; k < kUS; k++) fv[k] = a.fl[pv[k]];
  lds_order();
  // the slot of the run that goes on from the segment before (0: the run entering the chunk),
  // and whether the chunk's last run leaves it (wave-uniform, segment by segment)
  uint32_t open_slot = 0;
  bool leaving = false;
#pragma unroll
  for (int k = 0; k < kUS; k++) {
    const uint64_t i = s0 + uint64_t(k) * 64 + lane;
    const bool valid = i < n;
    uint32_t p = valid ? pv[k] : 0xFFFFFFFFu, key = valid ? kv[k] : kEmpty;
    uint32_t cls = kNoClass;
    if (valid) {
      if (key != kEmpty) {
        const uint32_t vr = key & id_mask;
        const uint32_t f = fv[k];
        const bool dup = f & FL_DUP, uns = f & FL_UNS;
        // the FixedVersion rank is needed only to dedup (repeating packages, unsorted runs)
        const uint32_t fr = (dup || uns) ? a.t.adv_rank[a.adv[i]].y : 0u;
        if (dup && !(a.diag & 2)) {  // another package of the dedup key with a greater FixedVersion, or an equal one seen first
          for (uint32_t j = a.dk_b[p], je = a.dk_e[p]; j < je && key != kEmpty; j++) {
            const uint32_t q = a.perm[j];
            if (q != p && beaten_by(a, q, vr, fr, q < p)) key = kEmpty;
          }
        }
        if (key != kEmpty && uns && !(a.diag & 2)) {  // the package's own pairs of this ID: the first with the greatest FixedVersion
          uint32_t rb = uint32_t(i), re = uint32_t(i) + 1;  // its run, walked (filter_mark keeps no bounds for it)
          while (rb > 0 && a.pkg[rb - 1] == p) rb--;
          while (re < n && a.pkg[re] == p) re++;
          for (uint32_t j = rb; j < re; j++) {
            if (j == uint32_t(i)) continue;
            const uint32_t kj = a.mkey[j];
            if (kj == kEmpty || (kj & id_mask) != vr) continue;
            const uint32_t fj = a.t.adv_rank[a.adv[j]].y;
            if (fj > fr || (fj == fr && j < uint32_t(i))) {
              key = kEmpty;
              break;
            }
          }
        }
      }
      a.skey[i] = key;
      cls = pair_class(a, key, i);
      a.pcls[i] = uint8_t(cls);  // placed by filter_place
    }
    // per-package class counters over the segment's 64 pairs: the first lane of each package
    // counts its lanes' classes with six ballots; a package all inside the segment stores its
    // record, one that goes on before or after it adds its share to the wave's LDS slot of the
    // first segment boundary its run crosses (0: the chunk's start), flushed below
    if (a.diag & 1) continue;
    const uint32_t up = __shfl_up(p, 1, 64);
    const bool head = valid && (lane == 0 || up != p);
    const unsigned long long heads = __ballot(head);
    const unsigned long long above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
    const uint32_t end = above ? uint32_t(__builtin_ctzll(above)) : 64u;
    const unsigned long long span = (end == 64 ? ~0ull : ((1ull << end) - 1)) & (~0ull << lane);
    uint32_t cc[kClasses];
#pragma unroll
    for (uint32_t c = 0; c < uint32_t(kClasses); c++) cc[c] = uint32_t(__popcll(__ballot(cls == c) & span));
    const uint32_t next = __shfl(ne[k], 63, 64);
    const bool cont_in = __shfl(pe[k], 0, 64) == __shfl(p, 0, 64);  // lane 0's run started before the segment
    const uint32_t last = heads ? 63u - uint32_t(__builtin_clzll(heads)) : 0u;
    const bool cont_out = heads && next == __shfl(p, int(last), 64);   // the segment's last run goes on
    if (head) {
      const bool split = (lane == 0 && cont_in) || (end == 64 && next == p);
      const uint32_t sum = cc[0] + cc[1] + cc[2] + cc[3] + cc[4];
      if (split) {
        const uint32_t slot = (lane == 0 && cont_in) ? open_slot : uint32_t(k) + 1u;
        uint32_t* o = lslot[slot];
#pragma unroll
        for (int c = 0; c < kClasses; c++)
          if (cc[c]) atomicAdd(&o[c], cc[c]);
        if (sum) atomicAdd(&o[kClasses], sum);
        o[kClasses + 1] = p;
      } else {
        store_sum(a, p, cc, sum);
      }
    }
    if (cont_out) open_slot = (last == 0 && cont_in) ? open_slot : uint32_t(k) + 1u;
    leaving = cont_out && k == kUS - 1;
  }
  // the slots: a run inside this chunk stores its record; the chunk's edge record takes the run
  // that enters it (slot 0) and the one that goes on past its end (filter_edges adds them up)
  lds_order();
  Edge* e = a.edge + g;
  if (lane < uint32_t(kSlots)) {
    const uint32_t* o = lslot[lane];
    const uint32_t p = o[kClasses + 1];
    const bool leaves = leaving && lane == open_slot;
    if (p != kEmpty) {
      if (lane == 0 || leaves) {
        uint32_t* c = (lane == 0) ? e->c_in : e->c_out;
#pragma unroll
        for (int k = 0; k < kClasses; k++) c[k] = o[k];
        if (lane == 0) e->p_in = p;
        if (leaves) e->p_out = p;
      } else {
        uint32_t cc[kClasses];
#pragma unroll
        for (int k = 0; k < kClasses; k++) cc[k] = o[k];
        store_sum(a, p, cc, o[kClasses]);
      }
    } else if (lane == 0) {
      e->p_in = kEmpty;
    }
    if (lane == 0 && !leaving) e->p_out = kEmpty;  // the chunk's last run ends inside it
  }
}

// Runs that cross chunk boundaries: from the chunk where such a run starts, its classes are
// added up over the chunks it spans (their edge records), each of those chunks gets the
// classes before it (carry_in, filter_place's entering run), and the total is the package's
// counter record.  One thread per chunk; a run of L pairs walks L / kSpan records.
__global__ __launch_bounds__(kBlock) void filter_edges(FilterArgs a, uint32_t n_chunks) {
  const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
  if (g >= n_chunks) return;
  const uint32_t p = a.edge[g].p_out;
  if (p == kEmpty || a.edge[g].p_in == p) return;  // no run starts in this chunk and leaves it
  uint32_t acc[kClasses];
#pragma unroll
  for (int c = 0; c < kClasses; c++) acc[c] = a.edge[g].c_out[c];
  for (uint32_t h = g + 1; h < n_chunks; h++) {  // edge[h].p_in == p
#pragma unroll
    for (int c = 0; c < kClasses; c++) {
      a.carry_in[uint64_t(h) * kClasses + c] = acc[c];
      acc[c] += a.edge[h].c_in[c];
    }
    if (a.edge[h].p_out != p) break;  // the run ends in chunk h
  }
  store_counts(a, p, acc, acc[0] + acc[1] + acc[2] + acc[3] + acc[4]);
}


// One-hot of a class in the packed in-chunk counters (kChunkBits per class).
__device__ __forceinline__ unsigned long long one_hot(uint32_t cls) {
  return cls < uint32_t(kClasses) ? 1ull << (kChunkBits * cls) : 0ull;
}
__device__ __forceinline__ uint32_t chunk_field(unsigned long long v, uint32_t cls) {
  return uint32_t(v >> (kChunkBits * cls)) & ((1u << kChunkBits) - 1u);
}

// filter_place: a wave per chunk (filter_select's), its 256 pairs' packed class prefixes in
// the wave's LDS, the entering run's classes from filter_edges (carry_in).
static_assert(kSpan <= (1u << kChunkBits), "chunk prefixes fit the packed fields");

// A pair's placement inputs, loaded two steps ahead of its span (pair words, then its
// package's words, then the package's placement base for the pair's class).
struct PlacePair {
  uint32_t p, adv, cf;  // package (kEmpty past the list's end), advisory, class | flags << 8
  uint32_t loc;         // the run in the chunk: first pair | end << 9 | entering << 18 | leaving << 19
  uint32_t gb;          // group start
  uint32_t base;        // the pair's output base (SINGLE survivors / ignored), else unused; a run
                        // inside the chunk adds its survivors of higher severity from the prefixes
};
enum : uint32_t { LOC_ENTER = 1u << 18, LOC_LEAVE = 1u << 19 };

// (Every field is written unconditionally from locals: stores of struct fields under branches
// were merged into address selects, which put the chunk's pair arrays in scratch memory.)
__device__ __forceinline__ void place_load_pair(const FilterArgs& a, uint64_t i, PlacePair& q) {
  uint32_t p = kEmpty, adv = 0, cf = kNoClass;
  if (i < a.n) {
    p = a.pkg[i];
    adv = a.adv[i];
    cf = a.pcls[i];  // pair_class, from filter_select
  }
  q.p = p;
  q.adv = adv;
  q.cf = cf;
}
__device__ __forceinline__ void place_load_pkg(const FilterArgs& a, PlacePair& q) {
  uint32_t fl = 0, gb = 0;
  if ((q.cf & 0xFFu) < uint32_t(kClasses)) {
    fl = a.fl[q.p];
    gb = a.grp_b[q.p];
  }
  q.cf |= fl << 8;
  q.gb = gb;
}
__device__ __forceinline__ void place_load_base(const FilterArgs& a, PlacePair& q) {
  const uint32_t cls = q.cf & 0xFFu, f = q.cf >> 8;
  const bool inside = !(q.loc & (LOC_ENTER | LOC_LEAVE));
  uint32_t base = 0;
  if (cls == uint32_t(kIgnClass)) {
    base = a.ign_off[q.p];
  } else if (cls < uint32_t(kClasses) && (f & (FL_SINGLE | FL_UNS)) == FL_SINGLE && inside) {
    base = a.off[q.gb];  // + the run's survivors before it in report order (from the chunk's LDS)
  } else if (cls < uint32_t(kClasses) && (f & (FL_SINGLE | FL_UNS)) == FL_SINGLE) {
    // a run crossing the chunk (its record from filter_edges): severity desc, then run order
    // (class = severity index: the package's survivors of the classes above come first)
    const uint32_t* c = a.cnt + uint64_t(q.p) * kCntStride;
    const uint4 c03 = *reinterpret_cast<const uint4*>(c);
    const uint32_t c4 = c[4];
    base = a.off[q.gb] + (cls < 4 ? c4 : 0u) + (cls < 3 ? c03.w : 0u) + (cls < 2 ? c03.z : 0u) + (cls < 1 ? c03.y : 0u);
  }
  q.base = base;
}

// Keys in the run [rb, re) below key (or at most key).  16 keys per step (four 16-byte loads
// in flight): a lane's count over a long group run is a latency chain of re - rb loads otherwise.
__device__ __forceinline__ uint32_t count_below(const uint32_t* skey, uint32_t rb, uint32_t re, uint32_t key,
                                                bool inclusive) {
  auto below = [&](uint32_t k) { return (k < key || (inclusive && k == key)) ? 1u : 0u; };
  uint32_t c = 0, j = rb;
  for (; j < re && (j & 3u); j++) c += below(skey[j]);
  const uint4* v = reinterpret_cast<const uint4*>(skey);
  for (; j + 16 <= re; j += 16) {
    const uint4 x0 = v[j / 4], x1 = v[j / 4 + 1], x2 = v[j / 4 + 2], x3 = v[j / 4 + 3];
    c += below(x0.x) + below(x0.y) + below(x0.z) + below(x0.w) + below(x1.x) + below(x1.y) + below(x1.z) +
         below(x1.w) + below(x2.x) + below(x2.y) + below(x2.z) + below(x2.w) + below(x3.x) + below(x3.y) +
         below(x3.z) + below(x3.w);
  }
  for (; j < re; j++) c += below(skey[j]);
  return c;
}

// Output position of a survivor (key) of package p in a group of several packages (same
// PkgName and InstalledVersion: merged by severity, ID, PkgPath) or with an unsorted run:
// keys counted over the group's runs.  Rare: filter_place runs it once per lane, after the chunk.
__device__ __forceinline__ uint64_t place_slow(const FilterArgs& a, uint32_t p, uint64_t i, uint32_t key) {
  const uint32_t gb = a.grp_b[p], ge = a.grp_e[p];
  uint32_t r = 0;
  if (ge - gb == 1) {  // an unsorted run alone in its group: its bounds walked (filter_mark keeps none)
    uint32_t rb = uint32_t(i), re = uint32_t(i) + 1;
    while (rb > 0 && a.pkg[rb - 1] == p) rb--;
    while (re < a.n && a.pkg[re] == p) re++;
    r = count_below(a.skey, rb, re, key, false);
  } else {
    const uint32_t pr = a.prank[p];
    for (uint32_t g = gb; g < ge; g++) {
      const uint32_t q = a.perm[g];
      if (q != p && !a.surv[q]) continue;  // no survivors (its run bounds may be stale)
      r += count_below(a.skey, a.run_b[q], a.run_e[q], key, q != p && a.prank[q] < pr);
    }
  }
  return uint64_t(a.off[gb]) + r;
}

__global__ __launch_bounds__(kBlock) void filter_place(FilterArgs a) {
  __shared__ unsigned long long pre_all[kBlock / 64][kSpan];  // per wave: exclusive packed class counts
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t g = uint64_t(blockIdx.x) * (kBlock / 64) + wave;  // this wave's chunk
  const uint64_t s0 = g * kSpan;
  if (s0 >= a.n) return;  // whole wave
  unsigned long long* pre = pre_all[wave];
  PlacePair q[kUS];
#pragma unroll
  for (int k = 0; k < kUS; k++) place_load_pair(a, s0 + k * 64 + lane, q[k]);
  const uint32_t before_chunk = s0 ? a.pkg[s0 - 1] : kEmpty;
  const uint32_t after_chunk = s0 + kSpan < a.n ? a.pkg[s0 + kSpan] : kEmpty;
  // the runs inside the chunk from its package column alone: H[k] bit l = pair k * 64 + l
  // starts a run in the chunk (past the list's end the sentinel package starts one)
  unsigned long long H[kUS];
#pragma unroll
  for (int k = 0; k < kUS; k++) {
    const uint32_t up = __shfl_up(q[k].p, 1, 64);
    const uint32_t tail = __shfl(q[k ? k - 1 : 0].p, 63, 64);  // the segment before's last package
    const uint32_t prev = lane ? up : (k == 0 ? before_chunk : tail);
    H[k] = __ballot(q[k].p != prev);
  }
  {
    uint32_t first_after = kSpan;  // the first run start past segment k (kSpan: none in the chunk)
    uint32_t fa[kUS];
#pragma unroll
    for (int k = kUS - 1; k >= 0; k--) {
      fa[k] = first_after;
      if (H[k]) first_after = uint32_t(k) * 64 + uint32_t(__builtin_ctzll(H[k]));
    }
    int last_start = -1;  // the last run start before segment k (-1: the entering run)
#pragma unroll
    for (int k = 0; k < kUS; k++) {
      const unsigned long long upto = lane == 63 ? ~0ull : (2ull << lane) - 1ull;
      const unsigned long long mb = H[k] & upto, ma = H[k] & ~upto;
      const int rs = mb ? k * 64 + 63 - int(__builtin_clzll(mb)) : last_start;
      const uint32_t re = ma ? uint32_t(k) * 64 + uint32_t(__builtin_ctzll(ma)) : fa[k];
      const bool leave = re == kSpan && after_chunk == q[k].p;
      q[k].loc = uint32_t(rs < 0 ? 0 : rs) | (re << 9) | (rs < 0 ? LOC_ENTER : 0u) | (leave ? LOC_LEAVE : 0u);
      if (H[k]) last_start = k * 64 + 63 - int(__builtin_clzll(H[k]));
    }
  }
#pragma unroll
  for (int k = 0; k < kUS; k++) place_load_pkg(a, q[k]);
#pragma unroll
  for (int k = 0; k < kUS; k++) place_load_base(a, q[k]);
  // the run entering the chunk: its classes before s0 (filter_edges), per lane for its class
  uint32_t carry[kUS];
#pragma unroll
  for (int k = 0; k < kUS; k++) {
    const uint32_t cls = q[k].cf & 0xFFu;
    carry[k] = ((q[k].loc & LOC_ENTER) && cls < uint32_t(kClasses) && !(a.diag & 64)) ? a.carry_in[g * kClasses + cls] : 0u;
  }
  // packed one-hot class prefixes over the chunk, segment by segment
  unsigned long long run = 0;
#pragma unroll
  for (int k = 0; k < kUS; k++) {
    const unsigned long long oh = one_hot(q[k].cf & 0xFFu);
    unsigned long long x = oh;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long y = __shfl_up(x, o, 64);
      if (lane >= uint32_t(o)) x += y;
    }
    pre[k * 64 + lane] = run + x - oh;
    run += __shfl(x, 63, 64);
  }
  lds_order();
  uint32_t slow = 0;
#pragma unroll
  for (int k = 0; k < kUS; k++) {
    const uint64_t i = s0 + k * 64 + lane;
    const uint32_t cls = q[k].cf & 0xFFu, f = q[k].cf >> 8;
    if (i >= a.n || cls >= uint32_t(kClasses)) continue;
    const uint32_t rs = q[k].loc & 511u, re = (q[k].loc >> 9) & 511u;  // the run in the chunk
    // pairs of this package before pair i that share its class
    const uint32_t before = chunk_field(pre[k * 64 + lane] - pre[rs], cls) + carry[k];
    if (cls == uint32_t(kIgnClass)) {  // ModifiedFindings in detection order
      const uint64_t at = uint64_t(q[k].base) + before;
      if (at < a.n) {
        uint32_t* o = a.iout + 3 * at;
        o[0] = q[k].p;
        o[1] = q[k].adv;
        o[2] = a.ign[i];
      }
      continue;
    }
    if ((f & (FL_SINGLE | FL_UNS)) != FL_SINGLE) {
      slow |= 1u << k;  // below, once per lane
      continue;
    }
    uint64_t at = uint64_t(q[k].base) + before;
    if (!(q[k].loc & (LOC_ENTER | LOC_LEAVE))) {  // a run inside the chunk: its classes from the prefixes
      const unsigned long long cnt = (re < kSpan ? pre[re] : run) - pre[rs];
#pragma unroll
      for (uint32_t c = 1; c < 5; c++) at += c > cls ? chunk_field(cnt, c) : 0u;
    }
    if (at < a.n) a.out[at] = make_uint2(q[k].p, q[k].adv);  // always true for a list grouped by package
  }
  if (a.diag & 32) slow = 0;
  while (slow) {  // the slow placements, one code path (static selects of the lane's pair)
    const uint32_t k = uint32_t(__builtin_ctz(slow));
    slow &= slow - 1;
    uint32_t p = 0, adv = 0;
#pragma unroll
    for (int kk = 0; kk < kUS; kk++)
      if (uint32_t(kk) == k) {
        p = q[kk].p;
        adv = q[kk].adv;
      }
    const uint64_t i = s0 + k * 64 + lane;
    const uint64_t at = place_slow(a, p, i, a.skey[i]);
    if (at < a.n) a.out[at] = make_uint2(p, adv);
  }
}

// Scan inputs (one trailing zero, so the exclusive scan's last element is the total):
// survivors of the package at perm position j (its survivor sum: one 4-byte gather, not
// five counters of a 24-byte row - C5's scan read 409 MB for 20M packages) / ignored
// findings of package j.
struct GroupCount {
  const uint32_t* perm;  // nullptr: package j itself, ignored findings
  const uint32_t* cnt;   // perm: the survivor sums; else the counter records
  uint32_t n;
  __host__ __device__ uint32_t operator()(uint32_t j) const {
    if (j >= n) return 0u;
    if (!perm) return cnt[uint64_t(j) * kCntStride + kIgnClass];
    return cnt[perm[j]];
  }
};

bool ok(hipError_t e, const char* what, std::string& err) {
  if (e == hipSuccess) return true;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

template <class T>
T* as(void* p) {
  return static_cast<T*>(p);
}

}  // namespace

// buffers: 0 perm, 1 grp_b, 2 grp_e, 3 dkey, 4 prank, 5 static flags, 6 counters, 7 flags, 8 run_b,
// 9 run_e, 10 off, 11 ign_off, 12 mkey, 13 skey, 14 ign, 15 dk_b, 16 dk_e,
// 17 rule table, 18 rule keys, 19 rule precedences, 20 pkg_class, 21 out pairs,
// 22 ignored out, 23 scan temp, 24 pair classes, 26 index check, 27 chunk edges, 28 chunk carries
BatchFilter::~BatchFilter() {
  for (void* p : bufs_)
    if (p) (void)hipFree(p);
  if (pin_) (void)hipHostFree(pin_);
}

bool BatchFilter::grow(int i, uint64_t need, std::string& err) {
  if (caps_[i] >= need && bufs_[i]) return true;
  if (bufs_[i]) (void)hipFree(bufs_[i]);
  bufs_[i] = nullptr;
  caps_[i] = 0;
  if (!ok(hipMalloc(&bufs_[i], std::max<uint64_t>(need, 16)), "hipMalloc(filter)", err)) return false;
  caps_[i] = std::max<uint64_t>(need, 16);
  return true;
}

bool BatchFilter::set_packages(const FilterPackages& fp, std::string& err) {
  const uint64_t n = fp.perm.size();
  n_pkgs_ = 0;
  if (n >= (1ull << 30)) {
    err = "filter: at most 2^30 packages per batch";
    return false;
  }
  const std::vector<uint32_t>* cols[5] = {&fp.perm, &fp.grp_b, &fp.grp_e, &fp.dkey, &fp.prank};
  for (int k = 0; k < 5; k++)
    if (cols[k]->size() != n || !grow(k, n * 4, err) ||
        (n && !ok(hipMemcpy(bufs_[k], cols[k]->data(), n * 4, hipMemcpyHostToDevice), "hipMemcpy(filter packages)",
                  err)))
      return false;
  if (fp.dup.size() != n) {
    err = "filter: one dup flag per package";
    return false;
  }
  std::vector<uint8_t> fl(n);
  for (uint64_t p = 0; p < n; p++)
    fl[p] = uint8_t((fp.dup[p] ? FL_DUP : 0u) | (fp.grp_e[p] - fp.grp_b[p] == 1 ? FL_SINGLE : 0u));
  // the perm range of every package's dedup key (equal keys are adjacent in perm order)
  std::vector<uint32_t> dkb(n), dke(n);
  for (uint64_t j = 0; j < n;) {
    uint64_t e = j + 1;
    while (e < n && fp.dkey[fp.perm[e]] == fp.dkey[fp.perm[j]]) e++;
    for (uint64_t m = j; m < e; m++) {
      dkb[fp.perm[m]] = uint32_t(j);
      dke[fp.perm[m]] = uint32_t(e);
    }
    j = e;
  }
  for (int k : {15, 16})
    if (!grow(k, n * 4, err) ||
        (n && !ok(hipMemcpy(bufs_[k], (k == 15 ? dkb : dke).data(), n * 4, hipMemcpyHostToDevice), "hipMemcpy(dedup keys)",
                  err)))
      return false;
  if (!grow(5, (n + 3) & ~3ull, err) ||
      (n && !ok(hipMemcpy(bufs_[5], fl.data(), n, hipMemcpyHostToDevice), "hipMemcpy(filter flags)", err)))
    return false;
  for (int k : {8, 9, 20})
    if (!grow(k, n * 4, err)) return false;
  if (!grow(6, n * 4 * (kCntStride + 1), err) || !grow(7, (n + 3) & ~3ull, err) || !grow(10, (n + 1) * 4, err) ||
      !grow(11, (n + 1) * 4, err))
    return false;
  n_pkgs_ = n;
  return true;
}

bool BatchFilter::run(const FillDev& t, const uint32_t* pkg, const uint32_t* adv, const uint2* side, uint64_t n,
                      const FilterRules& rules, uint32_t n_ranks, uint32_t sev_mask, uint32_t status_mask,
                      hipStream_t st, std::string& err) {
  n_ = n;
  survivors_ = ignored_ = 0;
  // measurement only: TVM_FILTER_TRACE=1 prints the host time at each step of a call
  static const bool trace = std::getenv("TVM_FILTER_TRACE") != nullptr;
  const auto T0 = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (trace)
      std::fprintf(stderr, "filter %s %.1f us\n", what,
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - T0).count());
  };
  if (n == 0) return true;
  if (n >= 0xFFFFFFFFull) {
    err = "filter: too many pairs";
    return false;
  }
  uint32_t id_bits = 1;
  while (id_bits < 32 && (uint64_t(1) << id_bits) < n_ranks) id_bits++;
  if (id_bits > 29) {
    err = "filter: more than 2^29 vulnerability IDs";
    return false;
  }
  const uint32_t blocks_u = uint32_t(std::min<uint64_t>((n + kBlock * kU - 1) / (kBlock * kU), 256ull * 32));
  const uint64_t n_chunks = (n + kSpan - 1) / kSpan;
  const uint32_t blocks_s = uint32_t((n_chunks + kBlock / 64 - 1) / (kBlock / 64));  // a wave per chunk
  sev_mask &= 0x1Fu;  // SeverityNames only: a bit for "out of range" (5) would pass a severity 4 - 5 can't order
  const uint64_t np = n_pkgs_;
  // The rule lists go up in one pinned copy, staged while the GPU counts repeating pairs.
  // Ignore rules (ALL / PKG / CLS) become a hash set (rules_insert); VEX statements mark
  // their pairs directly once the package runs are known (vex_mark, after filter_mark).
  const uint64_t nr_all = rules.size();
  RuleDev rd{}, vd{};  // hash-set lists, VEX lists
  uint64_t nr = 0, nv = 0, nr_c = 0, nv_c = 0;  // entries per kind (totals; staged so far)
  for (int k = 0; k < rules.n_lists; k++) (rules.lists[k].tag == RULE_VEX ? nv : nr) += rules.lists[k].n;
  if (nr_all) {
    uint64_t words = rules.rank[0].size() + rules.rank[1].size();
    for (int k = 0; k < rules.n_lists; k++)
      words += rules.lists[k].n * (1 + (rules.lists[k].subject ? 1 : 0) + (rules.lists[k].prec ? 1 : 0));
    if (pin_cap_ < words * 4) {
      if (pin_) (void)hipHostFree(pin_);
      pin_ = nullptr;
      pin_cap_ = 0;
      if (!ok(hipHostMalloc(&pin_, words * 4, hipHostMallocDefault), "hipHostMalloc(filter rules)", err)) return false;
      pin_cap_ = words * 4;
    }
    if (!grow(18, words * 4, err)) return false;
  }
  // staging layout: per phase a rank table, then per list subject / id / prec columns (4 B
  // each); phase 0 = the ignore lists (filter_mark needs their hash set), phase 1 = VEX
  // (its host copy runs on a helper thread from here on, its upload is queued behind
  // filter_select: the kernel that needs it runs after)
  uint32_t* const h = static_cast<uint32_t*>(pin_);
  const uint32_t* const d = nr_all ? as<const uint32_t>(bufs_[18]) : nullptr;
  uint64_t at = 0, ph_b[3] = {0, 0, 0};
  struct Job {
    uint32_t* dst;
    const uint32_t* src;
    uint64_t cnt;
  };
  std::vector<Job> jobs[2];
  for (int phase = 0; phase < 2; phase++) {
    ph_b[phase] = at;
    const uint32_t* rank_dev = nullptr;
    auto put = [&](const uint32_t* src, uint64_t cnt) {
      jobs[phase].push_back({h + at, src, cnt});
      const uint32_t* where = d + at;
      at += cnt;
      return where;
    };
    for (int k = 0; k < rules.n_lists; k++) {
      const RuleList& l = rules.lists[k];
      if ((l.tag == RULE_VEX) != (phase == 1)) continue;
      if (!rank_dev) rank_dev = put(rules.rank[l.table].data(), rules.rank[l.table].size());
      RuleDev& r = phase ? vd : rd;
      uint64_t& cnt = phase ? nv_c : nr_c;
      const int i = r.n_lists++;
      r.subject[i] = l.subject ? put(l.subject, l.n) : nullptr;
      r.id[i] = put(l.id, l.n);
      r.prec[i] = l.prec ? put(l.prec, l.n) : nullptr;
      r.rank[i] = rank_dev;
      r.tag[i] = uint32_t(l.tag);
      cnt += l.n;
      r.end[i] = cnt;
    }
  }
  ph_b[2] = at;
  auto copy_jobs = [](const std::vector<Job>& js) {
    for (const Job& jb : js) memcpy(jb.dst, jb.src, jb.cnt * 4);
  };
  std::thread vex_copy;
  if (!jobs[1].empty()) vex_copy = std::thread(copy_jobs, std::cref(jobs[1]));
  struct Joiner {
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } joiner{vex_copy};
  auto upload = [&](int phase) {
    const uint64_t a0 = ph_b[phase], a1 = ph_b[phase + 1];
    return a1 == a0 || ok(hipMemcpyAsync(static_cast<uint8_t*>(bufs_[18]) + a0 * 4, static_cast<uint8_t*>(pin_) + a0 * 4,
                                         (a1 - a0) * 4, hipMemcpyHostToDevice, st),
                          "H2D rules", err);
  };
  copy_jobs(jobs[0]);
  if (!upload(0)) return false;
  mark("staged ignore lists");
  uint64_t rcap = 0;
  if (nr) {
    rcap = 16;
    while (rcap < 2 * nr) rcap <<= 1;
  }
  const bool has_ign = (rules.kinds & 7u) != 0;
  using Count = hipcub::CountingInputIterator<uint32_t>;
  using In = hipcub::TransformInputIterator<uint32_t, GroupCount, Count>;
  size_t scan_bytes = 0;
  if (!ok(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, In(Count(0), GroupCount{nullptr, nullptr, 0}),
                                           static_cast<uint32_t*>(nullptr), int(np + 1), st),
          "hipcub scan sizing", err))
    return false;
  if (!grow(12, n * 4, err) || !grow(13, n * 4, err) || (has_ign && !grow(14, n * 4, err)) ||
      (rcap && !grow(17, rcap * 16, err)) || !grow(21, n * 8, err) || !grow(24, n, err) ||
      (has_ign && !grow(22, n * 12, err)) || !grow(23, std::max<uint64_t>(scan_bytes, 16), err) ||
      !grow(26, 16, err) || !grow(27, n_chunks * sizeof(Edge), err) || !grow(28, n_chunks * 4 * kClasses, err))
    return false;
  // per-call flags start as the static ones (FL_DUP, FL_SINGLE)
  if (np && !ok(hipMemcpyAsync(bufs_[7], bufs_[5], np, hipMemcpyDeviceToDevice, st), "D2D flags", err)) return false;
  if (nr) {  // the rule hash set, built on the device
    if (!ok(hipMemsetAsync(bufs_[17], 0xFF, rcap * 16, st), "memset(rules)", err)) return false;
    hipLaunchKernelGGL(rules_insert, dim3(uint32_t((nr + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, rd,
                       as<unsigned long long>(bufs_[17]), rcap - 1, as<uint8_t>(bufs_[7]));
    if (!ok(hipGetLastError(), "rules_insert", err)) return false;
  }
  if (!ok(hipMemsetAsync(bufs_[26], 0, 4, st), "memset(bad index)", err)) return false;
  if (rules.pkg_class &&
      !ok(hipMemcpyAsync(bufs_[20], rules.pkg_class, np * 4, hipMemcpyHostToDevice, st), "H2D classes", err))
    return false;
  // survivor sums of every package (the placement scan reads them all); filter_select /
  // filter_edges store every counter record of a package with pairs, so the records are
  // zeroed only when the ignored findings' scan reads every package's
  if (!ok(has_ign ? hipMemsetAsync(bufs_[6], 0, np * 4 * (kCntStride + 1), st)
                  : hipMemsetAsync(static_cast<uint32_t*>(bufs_[6]) + np * kCntStride, 0, np * 4, st),
          "memset(counters)", err))
    return false;
  FilterArgs a{};
  a.t = t;
  a.pkg = pkg;
  a.adv = adv;
  a.side = side;
  a.n = n;
  a.n_pkgs = uint32_t(np);
  a.perm = as<const uint32_t>(bufs_[0]);
  a.grp_b = as<const uint32_t>(bufs_[1]);
  a.grp_e = as<const uint32_t>(bufs_[2]);
  a.dkey = as<const uint32_t>(bufs_[3]);
  a.prank = as<const uint32_t>(bufs_[4]);
  a.dk_b = as<const uint32_t>(bufs_[15]);
  a.dk_e = as<const uint32_t>(bufs_[16]);
  a.dup = as<const uint8_t>(bufs_[5]);
  a.pkg_class = as<const uint32_t>(bufs_[20]);
  a.cnt = as<uint32_t>(bufs_[6]);
  a.surv = as<uint32_t>(bufs_[6]) + np * kCntStride;
  a.fl = as<uint8_t>(bufs_[7]);
  a.run_b = as<uint32_t>(bufs_[8]);
  a.run_e = as<uint32_t>(bufs_[9]);
  a.off = as<const uint32_t>(bufs_[10]);
  a.ign_off = as<const uint32_t>(bufs_[11]);
  a.mkey = as<uint32_t>(bufs_[12]);
  a.skey = as<uint32_t>(bufs_[13]);
  a.ign = as<uint32_t>(bufs_[14]);
  a.pcls = as<uint8_t>(bufs_[24]);
  a.rules = as<const unsigned long long>(bufs_[17]);
  a.rule_mask = rcap ? rcap - 1 : 0;
  a.kinds = nv ? rules.kinds : rules.kinds & ~(1u << RULE_VEX);  // (empty VEX lists: nothing to test)
  a.sev_mask = sev_mask;
  a.status_mask = status_mask;
  a.id_bits = id_bits;
  a.out = as<uint2>(bufs_[21]);
  a.iout = as<uint32_t>(bufs_[22]);
  a.edge = as<Edge>(bufs_[27]);
  a.carry_in = as<uint32_t>(bufs_[28]);
  static const uint32_t diag = std::getenv("TVM_FILTER_DIAG") ? uint32_t(std::atoi(std::getenv("TVM_FILTER_DIAG"))) : 0u;
  a.diag = diag;
  hipLaunchKernelGGL(filter_mark, dim3(blocks_u), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(filter_select, dim3(blocks_s), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(filter_edges, dim3(uint32_t((n_chunks + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, a,
                     uint32_t(n_chunks));
  mark("select launched");
  if (vex_copy.joinable()) vex_copy.join();
  if (!upload(1)) return false;  // the VEX lists go up while mark / select run
  mark("vex staged");
  if (nv) hipLaunchKernelGGL(vex_mark, dim3(uint32_t((nv + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, vd, pkg, side,
                             as<const uint32_t>(bufs_[8]), as<const uint32_t>(bufs_[9]), as<const uint8_t>(bufs_[7]), n,
                             uint32_t(np), uint32_t(rules.rank[1].size()), a.skey, a.pcls, a.cnt, a.surv,
                             a.carry_in, as<uint32_t>(bufs_[26]));
  if (!ok(hipGetLastError(), "filter launch", err) ||
      !ok(hipcub::DeviceScan::ExclusiveSum(bufs_[23], scan_bytes, In(Count(0), GroupCount{a.perm, a.surv, uint32_t(np)}),
                                           as<uint32_t>(bufs_[10]), int(np + 1), st),
          "hipcub scan", err) ||
      (has_ign &&
       !ok(hipcub::DeviceScan::ExclusiveSum(bufs_[23], scan_bytes, In(Count(0), GroupCount{nullptr, a.cnt, uint32_t(np)}),
                                            as<uint32_t>(bufs_[11]), int(np + 1), st),
           "hipcub scan", err)))
    return false;
  hipLaunchKernelGGL(filter_place, dim3(blocks_s), dim3(kBlock), 0, st, a);
  uint32_t tot[2] = {0, 0}, bad = 0;
  if (!ok(hipGetLastError(), "filter_place", err) ||
      !ok(hipMemcpyAsync(&tot[0], as<uint32_t>(bufs_[10]) + np, 4, hipMemcpyDeviceToHost, st), "D2H kept", err) ||
      (nv && !ok(hipMemcpyAsync(&bad, bufs_[26], 4, hipMemcpyDeviceToHost, st), "D2H index check", err)) ||
      (has_ign && !ok(hipMemcpyAsync(&tot[1], as<uint32_t>(bufs_[11]) + np, 4, hipMemcpyDeviceToHost, st),
                      "D2H ignored", err)) ||
      !ok(hipStreamSynchronize(st), "filter sync", err))
    return false;
  if (bad) {
    err = "tvm_match_filter: rule / VEX package, class or ID index out of range";
    return false;
  }
  survivors_ = tot[0];
  mark("done");
  if (std::getenv("TVM_FILTER_STATS")) {  // measurement only: which placement path the pairs take
    std::vector<uint32_t> hp(n), hb(np), he(np);
    std::vector<uint8_t> hf(np), hc(n);
    (void)hipMemcpy(hp.data(), pkg, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hf.data(), bufs_[7], np, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hb.data(), bufs_[8], np * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(he.data(), bufs_[9], np * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hc.data(), bufs_[24], n, hipMemcpyDeviceToHost);
    uint64_t nsingle = 0, uns_in = 0, uns_x = 0, multi = 0, cross = 0, surv_pairs = 0, uns_x_len = 0;
    for (uint64_t i = 0; i < n; i++) {
      if (hc[i] >= kClasses) continue;
      surv_pairs++;
      const uint32_t p = hp[i], f = hf[p];
      const uint64_t c0 = i / kSpan * kSpan;
      const bool inside = hb[p] >= c0 && he[p] <= c0 + kSpan;
      if (!(f & FL_SINGLE)) multi++;
      else if (f & FL_UNS) { if (inside) uns_in++; else { uns_x++; uns_x_len += he[p] - hb[p]; } }
      else if (!inside) cross++;
      else nsingle++;
    }
    std::fprintf(stderr, "filter stats: classed %llu inside-sorted %llu crossing-sorted %llu uns-inside %llu uns-crossing %llu (mean run %.1f) multi %llu\n",
                 (unsigned long long)surv_pairs, (unsigned long long)nsingle, (unsigned long long)cross,
                 (unsigned long long)uns_in, (unsigned long long)uns_x, uns_x ? double(uns_x_len) / uns_x : 0.0,
                 (unsigned long long)multi);
  }
  ignored_ = tot[1];
  return true;
}

bool BatchFilter::fetch(std::vector<uint2>& out, hipStream_t st, std::string& err) {
  out.assign(survivors_, make_uint2(0, 0));
  if (!survivors_) return true;
  return ok(hipMemcpyAsync(out.data(), bufs_[21], survivors_ * 8, hipMemcpyDeviceToHost, st), "D2H filtered", err) &&
         ok(hipStreamSynchronize(st), "filter sync", err);
}

bool BatchFilter::fetch_ignored(std::vector<uint32_t>& out3, hipStream_t st, std::string& err) {
  out3.assign(ignored_ * 3, 0);
  if (!ignored_) return true;
  return ok(hipMemcpyAsync(out3.data(), bufs_[22], ignored_ * 12, hipMemcpyDeviceToHost, st), "D2H ignored", err) &&
         ok(hipStreamSynchronize(st), "filter sync", err);
}

}  // namespace tvm
