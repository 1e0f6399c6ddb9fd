/*
 * ORACLE - TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference detector's matching arithmetic, used as the
 * checker for the HIP product path (tests/, __graft_entry__.smoke()) and as the
 * "port" CPU baseline in bench.py.  Nothing in trivy_amd/ links or calls this.
 *
 * The reference (fwereade/trivy @ 2025-01-14) is pure Go and its version
 * libraries are third-party modules that are not present in /root/reference
 * (SURVEY.md §8c).  Each comparator below restates the published algorithm of
 * the pinned module and is pinned by the reference's own test vectors
 * (tests/golden/cases/ and tests/golden/fixtures/).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- go-deb-version v0.0.0-20230223133812-3ed183d23422 (go.mod:62) ------------------------ */
typedef struct {
  int64_t epoch;
  const unsigned char* up;  /* upstream_version */
  size_t nup;
  const unsigned char* rev; /* debian_revision */
  size_t nrev;
} orc_deb;

/* NewVersion: 0 on success, -1 on error. */
int orc_deb_parse(const char* s, size_t n, orc_deb* out);
/* Version.Compare: <0, 0, >0. */
int orc_deb_cmp(const orc_deb* a, const orc_deb* b);
/* Convenience for tests: parse both, return 2 if a fails to parse, 3 if b fails,
 * else the sign of Compare (-1/0/1). */
int orc_deb_cmp_str(const char* a, size_t na, const char* b, size_t nb);

/* ---- go-apk-version v0.0.0-20200609155635-041fdbb8563f (go.mod:61) ----------------------- */
int orc_apk_valid(const char* s, size_t n);
int orc_apk_cmp(const char* a, size_t na, const char* b, size_t nb);
/* 2 if a fails to parse, 3 if b fails, else -1/0/1 */
int orc_apk_cmp_str(const char* a, size_t na, const char* b, size_t nb);

/* ---- go-rpm-version v0.0.0-20220614171824-631e686d1075 (go.mod:63) ------------------------ */
typedef struct {
  int64_t epoch;
  const char* ver;
  size_t nver;
  const char* rel;
  size_t nrel;
} orc_rpm;
void orc_rpm_parse(const char* s, size_t n, orc_rpm* out);  /* never fails */
int orc_rpmvercmp(const char* a, size_t na, const char* b, size_t nb);
int orc_rpm_cmp(const orc_rpm* a, const orc_rpm* b);
int orc_rpm_cmp_str(const char* a, size_t na, const char* b, size_t nb);

/* ---- driver-level batch matcher ----------------------------------------------------------
 * One OS bucket per package (platform id), advisories keyed by (platform, name).
 * Matches follow the per-driver semantics of SURVEY.md §8a' (the "unfixed" and
 * parse-error columns).  Used for large parity runs and the CPU baseline.        */
enum {
  ORC_DRV_DEBIAN = 1, /* debian.go:65-117: parse installed first, unfixed reported */
  ORC_DRV_UBUNTU = 2, /* ubuntu.go:86-126: lookup first, unfixed reported           */
};

typedef struct {
  /* DB: keys (platform, name) and their advisories (CSR: key_adv_begin[k]..key_adv_begin[k+1]) */
  int32_t n_keys;
  const int32_t* key_plat;
  const char* key_name_arena;
  const uint64_t* key_name_off;
  const uint32_t* key_name_len;
  const uint8_t* key_poisoned;      /* 1 = advisory JSON under this key fails to decode */
  const int64_t* key_adv_begin;     /* n_keys+1 */
  const char* adv_fixed_arena;      /* FixedVersion strings */
  const uint64_t* adv_fixed_off;
  const uint32_t* adv_fixed_len;
  /* per-platform driver kind (ORC_DRV_*) */
  int32_t n_plat;
  const int32_t* plat_driver;
} orc_db;

typedef struct {
  int64_t n;
  const int32_t* plat;              /* -1 = bucket absent */
  const char* name_arena;
  const uint64_t* name_off;
  const uint32_t* name_len;
  const char* ver_arena;            /* the formatted version the driver parses */
  const uint64_t* ver_off;
  const uint32_t* ver_len;
} orc_batch;

/* Computes matches as (pkg index, global advisory index) in (pkg, advisory) order.
 * Writes up to `cap` pairs; returns the total number of matches (call again with a
 * larger buffer if > cap), or -1 - i when package i hits a poisoned key first
 * (the Detect call would fail).  `n_threads` <= 0 means 1.                        */
int64_t orc_match(const orc_db* db, const orc_batch* b, int n_threads,
                  int64_t* out_pkg, int64_t* out_adv, int64_t cap);

/* ---- library comparers (libcmp.c): matchVersion per grammar, 1 / 0, -1 on a parse error -- */
enum { ORC_LIB_GENERIC = 1, ORC_LIB_NPM = 2, ORC_LIB_PEP440 = 3, ORC_LIB_MAVEN = 4 };
enum { ORC_LIB_HAS_VULN = 1, ORC_LIB_HAS_SECURE = 2, ORC_LIB_ALWAYS = 4 };
int orc_lib_match(int grammar, const char* ver, size_t nv, const char* c, size_t nc);
/* compare.IsVulnerable (compare.go:21-55): vuln / sec = the advisory's Vulnerable /
 * Patched+Unaffected lists joined with " || " (flags say which lists exist) */
int orc_lib_is_vulnerable(int grammar, const char* ver, size_t nv, uint32_t flags, const char* vuln, size_t nvu,
                          const char* sec, size_t nse);

/* ---- mixed-workload driver loops (mixmatch.c): the native CPU baseline of C3 / C4 / C5 ----
 * Advisories pre-decoded per (platform, lookup name) as "entries" (one per advisory; rocky:
 * one per arch entry; Red Hat: one per (advisory, entry, CVE)).  Per package the driver of
 * its platform runs the reference's loop over the key's entries. */
enum {
  ORC_MX_DEBIAN = 1, ORC_MX_UBUNTU = 2, ORC_MX_ALPINE = 3, ORC_MX_ALMA = 4, ORC_MX_ROCKY = 5, ORC_MX_ORACLE = 6,
  ORC_MX_REDHAT = 7, ORC_MX_LIB = 8,
};
typedef struct {
  int32_t n_plat;
  const int32_t* plat_driver;   /* ORC_MX_* */
  const int32_t* plat_grammar;  /* ORC_LIB_* for ORC_MX_LIB */
  int32_t n_keys;
  const int32_t* key_plat;
  const char* key_name_arena;
  const uint64_t* key_name_off;
  const uint32_t* key_name_len;
  const int64_t* key_begin;     /* n_keys + 1: the key's entries */
  /* entries */
  const char* arena;            /* every entry string */
  const uint64_t* fixed_off;    /* FixedVersion ("" = unfixed) */
  const uint32_t* fixed_len;
  const uint64_t* aff_off;      /* alpine AffectedVersion */
  const uint32_t* aff_len;
  const uint64_t* vul_off;      /* library lists (see orc_lib_is_vulnerable) */
  const uint32_t* vul_len;
  const uint64_t* sec_off;
  const uint32_t* sec_len;
  const uint32_t* lib_flags;
  const int32_t* vid;           /* vulnerability ID index (Red Hat merge key, parity checks) */
  const int64_t* ids_begin;     /* n_entries + 1 into ids: n_arch arch ids, then CPE indices */
  const int32_t* n_arch;
  const int32_t* ids;
} orc_mix_db;
typedef struct {
  int64_t n;
  const int32_t* plat;          /* -1: no bucket */
  const char* name_arena;       /* the driver's lookup name (modular namespace applied) */
  const uint64_t* name_off;
  const uint32_t* name_len;
  const char* ver_arena;        /* the version the driver compares (formatted) */
  const uint64_t* ver_off;
  const uint32_t* ver_len;
  const int32_t* arch;          /* arch id, -1 none; noarch_id = noarch */
  int32_t noarch_id;
  const uint8_t* skip;          /* 1: the driver skips the package */
  const int64_t* cpe_begin;     /* Red Hat: n + 1 into cpe_ids (the package's CPE set) */
  const int32_t* cpe_ids;
} orc_mix_batch;
/* (package, entry) pairs of every detected vulnerability, per package in the driver's output
 * order (Red Hat: one per VulnerabilityID after the merge - the entry that decided it).
 * Returns the count (call again with a larger buffer when > cap). */
int64_t orc_mix_match(const orc_mix_db* db, const orc_mix_batch* b, int n_threads, int64_t* out_pkg,
                      int64_t* out_entry, int64_t cap);
/* orc_mix_match with flags: ORC_MIX_MEMBERS also emits, after every Red Hat group's entry, the
 * group's members (the entries that entered redhat.go's uniqVulns map, Get order) as
 * -(entry + 1) - what the whole-batch DetectedVulnerability checks rebuild the merge from. */
enum { ORC_MIX_MEMBERS = 1 };
int64_t orc_mix_match_ex(const orc_mix_db* db, const orc_mix_batch* b, int n_threads, int64_t* out_pkg,
                         int64_t* out_entry, int64_t cap, int flags);

#ifdef __cplusplus
}
#endif
