/*
 * ORACLE - TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Driver-level batch matcher: the per-package loops of the reference OS drivers,
 * restated over an in-memory advisory table.  Per package it does what the Go
 * driver does per call (the bbolt View + JSON decode is replaced by an in-memory
 * lookup, which makes this a conservative, i.e. fast, CPU baseline):
 *   debian.go:65-117  - parse FormatSrcVersion(pkg) (skip pkg on error), Get(bucket,
 *                       SrcName), for each advisory: FixedVersion == "" -> report;
 *                       parse FixedVersion (skip advisory on error); report if
 *                       installed < fixed.
 *   ubuntu.go:86-126  - same comparisons, but the lookup (and so a decode error)
 *                       comes before the installed-version parse.
 * The advisory FixedVersion is re-parsed for every (package, advisory) pair, as the
 * reference does.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  uint64_t* h;   /* 0 = empty */
  int32_t* key;
  uint64_t mask;
} kmap;

static uint64_t fnv(int32_t plat, const char* s, size_t n) {
  uint64_t h = 1469598103934665603ULL ^ (uint64_t)(uint32_t)plat;
  for (size_t i = 0; i < n; i++) { h ^= (unsigned char)s[i]; h *= 1099511628211ULL; }
  return h | 1;
}

static void kmap_build(kmap* m, const orc_db* db) {
  uint64_t cap = 16;
  while (cap < (uint64_t)db->n_keys * 2) cap <<= 1;
  m->mask = cap - 1;
  m->h = calloc(cap, sizeof(uint64_t));
  m->key = calloc(cap, sizeof(int32_t));
  for (int32_t k = 0; k < db->n_keys; k++) {
    uint64_t h = fnv(db->key_plat[k], db->key_name_arena + db->key_name_off[k], db->key_name_len[k]);
    uint64_t i = h & m->mask;
    while (m->h[i]) i = (i + 1) & m->mask;
    m->h[i] = h;
    m->key[i] = k;
  }
}

static int32_t kmap_get(const kmap* m, const orc_db* db, int32_t plat, const char* s, size_t n) {
  uint64_t h = fnv(plat, s, n);
  for (uint64_t i = h & m->mask; m->h[i]; i = (i + 1) & m->mask) {
    if (m->h[i] != h) continue;
    int32_t k = m->key[i];
    if (db->key_plat[k] == plat && db->key_name_len[k] == n &&
        memcmp(db->key_name_arena + db->key_name_off[k], s, n) == 0)
      return k;
  }
  return -1;
}

typedef struct {
  const orc_db* db;
  const orc_batch* b;
  const kmap* m;
  int64_t lo, hi;
  int64_t* pk;
  int64_t* ad;
  int64_t n, cap;
  int64_t err_pkg; /* first poisoned package in [lo, hi) or -1 */
} job;

static void push(job* j, int64_t p, int64_t a) {
  if (j->n == j->cap) {
    j->cap = j->cap ? j->cap * 2 : 1024;
    j->pk = realloc(j->pk, sizeof(int64_t) * j->cap);
    j->ad = realloc(j->ad, sizeof(int64_t) * j->cap);
  }
  j->pk[j->n] = p;
  j->ad[j->n] = a;
  j->n++;
}

static void* run_job(void* arg) {
  job* j = arg;
  const orc_db* db = j->db;
  const orc_batch* b = j->b;
  for (int64_t i = j->lo; i < j->hi; i++) {
    int32_t plat = b->plat[i];
    if (plat < 0 || plat >= db->n_plat) continue;
    int drv = db->plat_driver[plat];
    const char* ver = b->ver_arena + b->ver_off[i];
    orc_deb inst;
    int inst_ok = orc_deb_parse(ver, b->ver_len[i], &inst) == 0;
    if (drv == ORC_DRV_DEBIAN && !inst_ok) continue; /* parse before lookup */
    int32_t k = kmap_get(j->m, db, plat, b->name_arena + b->name_off[i], b->name_len[i]);
    if (k < 0) continue;
    if (db->key_poisoned[k]) {
      if (j->err_pkg < 0) j->err_pkg = i;
      continue;
    }
    if (!inst_ok) continue;
    for (int64_t a = db->key_adv_begin[k]; a < db->key_adv_begin[k + 1]; a++) {
      uint32_t fl = db->adv_fixed_len[a];
      if (fl == 0) { push(j, i, a); continue; } /* unfixed: reported */
      orc_deb fx;
      if (orc_deb_parse(db->adv_fixed_arena + db->adv_fixed_off[a], fl, &fx)) continue;
      if (orc_deb_cmp(&inst, &fx) < 0) push(j, i, a);
    }
  }
  return NULL;
}

int64_t orc_match(const orc_db* db, const orc_batch* b, int n_threads, int64_t* out_pkg,
                  int64_t* out_adv, int64_t cap) {
  if (n_threads <= 0) n_threads = 1;
  kmap m;
  kmap_build(&m, db);
  job* jobs = calloc((size_t)n_threads, sizeof(job));
  pthread_t* th = calloc((size_t)n_threads, sizeof(pthread_t));
  int64_t per = (b->n + n_threads - 1) / n_threads;
  for (int t = 0; t < n_threads; t++) {
    jobs[t].db = db; jobs[t].b = b; jobs[t].m = &m;
    jobs[t].lo = (int64_t)t * per;
    jobs[t].hi = jobs[t].lo + per < b->n ? jobs[t].lo + per : b->n;
    if (jobs[t].lo > b->n) jobs[t].lo = b->n;
    jobs[t].err_pkg = -1;
    if (n_threads == 1) run_job(&jobs[t]);
    else pthread_create(&th[t], NULL, run_job, &jobs[t]);
  }
  int64_t total = 0, err = -1;
  for (int t = 0; t < n_threads; t++) {
    if (n_threads > 1) pthread_join(th[t], NULL);
    if (err < 0 && jobs[t].err_pkg >= 0) err = jobs[t].err_pkg;
  }
  if (err < 0) {
    for (int t = 0; t < n_threads; t++) {
      for (int64_t x = 0; x < jobs[t].n; x++, total++)
        if (total < cap) { out_pkg[total] = jobs[t].pk[x]; out_adv[total] = jobs[t].ad[x]; }
    }
  }
  for (int t = 0; t < n_threads; t++) { free(jobs[t].pk); free(jobs[t].ad); }
  free(jobs); free(th); free(m.h); free(m.key);
  return err >= 0 ? -1 - err : total;
}
