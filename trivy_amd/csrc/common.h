// Shared host/device definitions for the trivy_amd matching engine.
//
// Everything here is compiled twice by hipcc: once for the host flattener
// (advisory side, at DB load time) and once for gfx950 (installed-package side,
// inside the kernels), so both sides agree bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TVM_HD __host__ __device__ __forceinline__

namespace tvm {

// Version grammar of a platform (which third-party comparator the reference uses).
enum Cmp : uint8_t {
  CMP_NONE = 0,
  CMP_DEB = 1,   // knqyf263/go-deb-version (debian, ubuntu, amazon)
  CMP_APK = 2,   // knqyf263/go-apk-version (alpine, wolfi, chainguard)
  CMP_RPM = 3,   // knqyf263/go-rpm-version (redhat/centos, alma, rocky, oracle, suse, photon, mariner)
  // library grammars (libver.h; pkg/detector/library/driver.go:25-93)
  CMP_GENERIC = 4,  // aquasecurity/go-version (cargo, composer, go, nuget, pub, erlang, conan, swift, k8s)
  CMP_NPM = 5,      // aquasecurity/go-npm-version
  CMP_PEP440 = 6,   // aquasecurity/go-pep440-version
  CMP_MAVEN = 7,    // masahiro331/go-mvn-version
  CMP_GEM = 8,      // aquasecurity/go-gem-version (rubygems, cocoapods)
  CMP_BITNAMI = 9,  // bitnami/go-version
};

// Driver families (reference pkg/detector/ospkg/detect.go:32-48 and library/driver.go:25-93).
enum Drv : uint8_t {
  DRV_NONE = 0,
  DRV_DEBIAN = 1,
  DRV_UBUNTU = 2,
  DRV_AMAZON = 3,
  DRV_ALPINE = 4,
  DRV_WOLFI = 5,
  DRV_CHAINGUARD = 6,
  DRV_REDHAT = 7,
  DRV_ALMA = 8,
  DRV_ROCKY = 9,
  DRV_ORACLE = 10,
  DRV_SUSE = 11,
  DRV_PHOTON = 12,
  DRV_MARINER = 13,
  DRV_LIBRARY = 14,  // pkg/detector/library (one platform per ecosystem prefix "eco::")
};

// Per-platform flags (device-visible).
enum : uint32_t {
  PLAT_LOOKUP_FIRST = 1u << 0,  // DB lookup (and its decode error) precedes the installed parse
};

// One interval row: the advisory matches installed version v iff
//   ALWAYS, or v parsed and lo <=/< v and v </<= hi.
// Keys live in the key arena (8-byte aligned, little-endian words holding the
// sort-key bytes in memory order).  lo/hi lengths carry flags in their top bits.
// Key arena word offsets of a row's bounds.
struct RowOff {
  uint32_t lo_off;
  uint32_t hi_off;
};
struct alignas(16) Row {
  uint64_t hi_pre0;  // the hi key's first bytes inline as BIG-ENDIAN words, zero padded, so a
  uint64_t hi_pre1;  // compare is two / three u64 compares that rarely touch the key arena
  union {
    uint64_t hi_pre2;  // dpkg grammar: key bytes 16..23 (24-byte heads: its version keys are ~10-20
                       // bytes and tie often at 16); the offsets sit in DB::row_off
    RowOff off;        // the other grammars: 16-byte heads, offsets inline (their lower bounds,
                       // library / apk ranges, read the arena at once)
  };
  uint32_t adv;      // global advisory index (host-side record)
  uint16_t lo_len;   // bytes | flags
  uint16_t hi_len;
};
enum : uint16_t {
  KEY_LEN_MASK = 0x3FFF,
  KEY_INF = 0x8000,      // lo = -inf / hi = +inf
  KEY_INCL = 0x4000,     // bound is inclusive (lo default inclusive: set for lo; hi default exclusive)
};
enum : uint32_t {
  ROW_ALWAYS = 1u << 31, // in Row::adv: matches even when the installed version fails to parse
  ROW_FILTER = 1u << 30, // in Row::adv: also test the package against RowAux (arch / CPE / tag)
  ROW_INLINE = 1u << 29, // in Row::adv (with ROW_FILTER): the predicates sit in the row itself (below)
  ROW_ADV_MASK = 0x1FFFFFFFu,
};
// ROW_INLINE: an rpm-grammar row (only an upper bound: its lo_len is KEY_INF, its key offsets
// live in DB::row_off) whose filter fits the row carries it in place of the offsets, so the
// sweep tests it without the RowAux -> id-list chain of dependent loads:
//   lo_len = KEY_INF | AUX kind bits (ARCH_RH / ARCH_IN / CPE / TAG, low 4 bits) | n_arch << 4 |
//            n_cpe << 6 (2 bits each);
//   off    = AUX_TAG: lo_off = the ksplice tag; else four 16-bit ids, the arch ids then the CPE
//            indices (n_arch + n_cpe <= 4, every id < 0xFFFF).
constexpr uint32_t kInlineIds = 4;

// Per-(package, advisory) predicates beyond the version interval, read only for rows
// flagged ROW_FILTER (rows[] and aux[] are parallel arrays):
//   AUX_ARCH_RH   redhat.go:129-135: pass if no arches, or the package is noarch, or its
//                 arch is listed;
//   AUX_ARCH_IN   trivy-db rocky Get: pass only if the package arch is listed;
//   AUX_CPE       trivy-db redhat-oval Get: pass if one of the entry's affected CPE indices
//                 is in the package's CPE set (content sets + NVR, resolved on the host);
//   AUX_TAG       oracle.go:65-69: the advisory's ksplice tag equals the package's.
struct alignas(16) RowAux {
  uint32_t kind;
  uint32_t tag;
  uint32_t list_off;  // into aux_ids: n_arch arch ids, then n_cpe CPE indices
  uint16_t n_arch;
  uint16_t n_cpe;
};
//   AUX_CLASS     library rows: pass if bit <installed version class> of `tag` is set
//                 (libver.h classes: npm pre-release, PEP 440 local/pre/post; Maven has one).
//   AUX_MVN       Maven library rows: the advisory's IsVulnerable program at aux_ids[list_off]
//                 evaluated pairwise against the installed version (libver.h mvn_program_eval).
enum : uint32_t { AUX_ARCH_RH = 1, AUX_ARCH_IN = 2, AUX_CPE = 4, AUX_TAG = 8, AUX_CLASS = 16, AUX_MVN = 32 };

// Package attributes (uint2 per package, only for batches that carry filtered rows):
// x = arch id | PA_NOARCH, y = ksplice tag (oracle) or CPE-set id (redhat).
enum : uint32_t { PA_NOARCH = 1u << 31, PA_ARCH_MASK = 0x7FFFFFFFu, PA_ARCH_NONE = 0x7FFFFFFFu };

// Platform descriptor (device-visible).
struct alignas(8) PlatInfo {
  uint8_t cmp;
  uint8_t drv;
  uint16_t pad;
  uint32_t flags;
};

// Hash-index slot values.
struct alignas(16) SlotVal {
  uint32_t name_off;   // into the DB name arena
  uint32_t name_len;   // bytes | SLOT_POISONED
  uint32_t row_begin;
  uint32_t row_count;
};
// SLOT_MVN_C0 / C1: the key has a Maven program row (AUX_MVN) that admits installed versions
// of class 0 / 1: the probe packs a Maven package's parse only then.  Maven has one class
// since the numeric projection (libver.h mvn_numeric_projection), and program rows carry no
// class filter, so both bits are set together.
// SLOT_CLS_SPLIT: a library key whose rows differ by version class (PEP 440 local / pre / post,
// npm pre-release: AUX_CLASS rows) keeps two lists back to back - A, the rows that admit class
// 0 (the plain release versions most packages have), without their class filter, then B, every
// row in advisory order as before - and row_count = |A| | |B| << 16: a class-0 package sweeps
// [row_begin, row_begin + |A|), any other [row_begin + |A|, + |B|), each in advisory order.
enum : uint32_t {
  SLOT_POISONED = 1u << 31, SLOT_MVN_C0 = 1u << 30, SLOT_MVN_C1 = 1u << 29, SLOT_CLS_SPLIT = 1u << 28,
  SLOT_LEN_MASK = 0x0FFFFFFFu
};
// The rows a package of version class cls sweeps: {begin, count} of a slot's row range.
TVM_HD uint2 slot_rows(uint32_t name_len, uint32_t row_begin, uint32_t row_count, uint32_t cls) {
  if (!(name_len & SLOT_CLS_SPLIT)) return make_uint2(row_begin, row_count);
  const uint32_t na = row_count & 0xFFFFu;
  return cls == 0 ? make_uint2(row_begin, na) : make_uint2(row_begin + na, row_count >> 16);
}
// Device hash slot: one 64-B cache line holding the hash, the row range and the first
// kSlotNameWords*8 bytes of the name (memory order, zero padded), so a probe verifies the
// name from the same line it read the hash from; longer names finish against the name
// arena from byte 40 on.  (The host keeps slot_hash/slot_val for its own lookups.)
constexpr uint32_t kSlotNameWords = 5;
struct alignas(64) Slot {
  uint64_t hash;       // 0 = empty
  uint32_t row_begin;
  uint32_t row_count;
  uint32_t name_len;   // bytes | SLOT_POISONED
  uint32_t name_off;   // full name in the name arena
  uint64_t name[kSlotNameWords];
};
static_assert(sizeof(Slot) == 64, "one cache line per slot");
// Slot fingerprints (DB::slot_fp): one byte a slot, 0 = empty, else the hash's top byte (1 for
// 0).  The probe walks the chain in this array (1/64 of the slot bytes: 2 MB for 2^21 slots,
// L2-resident) and reads a 64-B slot only where the fingerprint is the name's: an absent name
// reads no slot at all.
TVM_HD uint8_t slot_fp_of(uint64_t h) {
  const uint8_t f = uint8_t(h >> 56);
  return f ? f : uint8_t(1);
}
// Names in the DB name arena start 8-byte aligned, zero padded to a word boundary, and
// the arena ends with kNameWords zero words: the probe verifies a name with kNameWords
// independent word loads (one memory round trip) instead of a byte loop.
constexpr uint32_t kNameWords = 4;

// 64-bit key hash of (platform, name): FNV-1a over the bytes seeded by the platform,
// finished with the murmur3 fmix64 avalanche.  Never 0 (0 marks an empty slot).
TVM_HD uint64_t key_hash_seed(uint32_t plat) { return 0xcbf29ce484222325ULL ^ (uint64_t(plat) * 0x9E3779B97F4A7C15ULL); }
TVM_HD uint64_t key_hash_step(uint64_t h, uint8_t c) { return (h ^ c) * 0x100000001b3ULL; }
TVM_HD uint64_t key_hash_fin(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h ? h : 1;
}
TVM_HD uint64_t key_hash(uint32_t plat, const uint8_t* s, uint32_t n) {
  uint64_t h = key_hash_seed(plat);
  for (uint32_t i = 0; i < n; i++) h = key_hash_step(h, s[i]);
  return key_hash_fin(h);
}

// Package-index hash of (platform, name): word at a time, so the probe kernel hashes a
// name with one multiply per 8 bytes (the words it also compares against the slot's
// inline name).  Seeded by the platform and the length; words are little-endian, the
// last one zero padded; finished with fmix64.  Never 0.
TVM_HD uint64_t key_hash_seed2(uint32_t plat, uint32_t n) {
  return 0xcbf29ce484222325ULL ^ (uint64_t(plat) * 0x9E3779B97F4A7C15ULL) ^ (uint64_t(n) * 0xC2B2AE3D27D4EB4FULL);
}
TVM_HD uint64_t key_hash_word(uint64_t h, uint64_t w) {
  h = (h ^ w) * 0x9FB21C651E98DF25ULL;
  return h ^ (h >> 29);
}
TVM_HD uint64_t pkg_key_hash(uint32_t plat, const uint8_t* s, uint32_t n) {
  uint64_t h = key_hash_seed2(plat, n);
  for (uint32_t i = 0; i < n; i += 8) {
    uint64_t w = 0;
    for (uint32_t b = 0; b < 8 && i + b < n; b++) w |= uint64_t(s[i + b]) << (8 * b);
    h = key_hash_word(h, w);
  }
  return key_hash_fin(h);
}

// Lexicographic compare of two sort keys held in 8-byte words (memory-order bytes,
// zero padded): memcmp over the common length, then shorter-first.
TVM_HD int key_cmp(const uint64_t* a, uint32_t na, const uint64_t* b, uint32_t nb) {
  uint32_t m = na < nb ? na : nb;
  uint32_t full = m >> 3, rem = m & 7;
  for (uint32_t w = 0; w < full; w++) {
    uint64_t x = a[w], y = b[w];
    if (x != y) {
      x = __builtin_bswap64(x);
      y = __builtin_bswap64(y);
      return x < y ? -1 : 1;
    }
  }
  if (rem) {
    uint64_t mask = (1ULL << (8 * rem)) - 1;  // low `rem` bytes in memory order
    uint64_t x = a[full] & mask, y = b[full] & mask;
    if (x != y) {
      x = __builtin_bswap64(x);
      y = __builtin_bswap64(y);
      return x < y ? -1 : 1;
    }
  }
  return (na > nb) - (na < nb);
}

// key_cmp(a, b) where the first two words of both keys are given inline (a0, a1, b0, b1)
// and the full keys live at a_full / b_full (read only when the first 16 bytes tie and
// both keys are longer).
TVM_HD int key_cmp_pre2(uint64_t a0, uint64_t a1, const uint64_t* a_full, uint32_t na, uint64_t b0, uint64_t b1,
                        const uint64_t* b_full, uint32_t nb) {
  const uint32_t m = na < nb ? na : nb;
  const uint64_t v[2] = {a0, a1};
  const uint64_t w[2] = {b0, b1};
#pragma unroll
  for (uint32_t i = 0; i < 2; i++) {
    if (8 * i >= m) return (na > nb) - (na < nb);
    uint64_t x = v[i], y = w[i];
    const uint32_t left = m - 8 * i;
    if (left < 8) {
      const uint64_t mask = (1ULL << (8 * left)) - 1;
      x &= mask;
      y &= mask;
    }
    if (x != y) {
      x = __builtin_bswap64(x);
      y = __builtin_bswap64(y);
      return x < y ? -1 : 1;
    }
  }
  if (m <= 16) return (na > nb) - (na < nb);
  return key_cmp(a_full + 2, na - 16, b_full + 2, nb - 16);
}
TVM_HD int key_cmp_pre(const uint64_t* a, uint32_t na, uint64_t b0, uint64_t b1, const uint64_t* b_full,
                       uint32_t nb) {
  return key_cmp_pre2(a[0], a[1], a, na, b0, b1, b_full, nb);
}

}  // namespace tvm
