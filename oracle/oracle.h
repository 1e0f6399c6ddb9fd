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

#ifdef __cplusplus
}
#endif
