/*
 * ORACLE - TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Native CPU baseline of the mixed workloads (BASELINE configs C3 / C4 / C5): the per-package
 * loops of the reference drivers, restated over pre-decoded advisories (the entries of
 * orc_mix_db; decoding them once is what makes this a conservative - fast - baseline, as
 * SURVEY.md §8d prescribes for the C++ restatement), with threads over packages:
 *   debian.go:65-117       parse the source version first (skip the package on error), unfixed
 *                          entries reported, else installed < fixed (go-deb-version);
 *   ubuntu.go:86-126       the same comparisons, lookup first;
 *   alpine.go:75-129       AffectedVersion gate, then installed < fixed (go-apk-version);
 *   alma.go / rocky.go     installed < fixed (go-rpm-version); rocky: the advisory's entries
 *                          whose arches hold the package's arch (trivy-db rocky Get);
 *   oracle.go:55-84        the ksplice tags of fixed and installed release must agree;
 *   redhat.go:90-187       CPE set and arch filters, then the per-CVE merge: the first entry of
 *                          an ID gives it, a fixed one raises FixedVersion to the greatest;
 *                          output sorted by ID;
 *   library/driver.go:111-137  compare.IsVulnerable per advisory (libcmp.c).
 * Every comparison parses both versions per (package, entry) pair, as the reference does.
 * Checked against oracle/drivers.py + oracle/library.py by tests/test_cport.py.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  uint64_t* h;
  int32_t* key;
  uint64_t mask;
} kmap;

static uint64_t fnv(int32_t plat, const char* s, size_t n) {
  uint64_t h = 1469598103934665603ULL ^ (uint64_t)(uint32_t)plat;
  for (size_t i = 0; i < n; i++) {
    h ^= (unsigned char)s[i];
    h *= 1099511628211ULL;
  }
  return h | 1;
}

static void kmap_build(kmap* m, const orc_mix_db* db) {
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

static int32_t kmap_get(const kmap* m, const orc_mix_db* db, int32_t plat, const char* s, size_t n) {
  uint64_t h = fnv(plat, s, n);
  for (uint64_t i = h & m->mask; m->h[i]; i = (i + 1) & m->mask) {
    if (m->h[i] != h) continue;
    int32_t k = m->key[i];
    if (db->key_plat[k] == plat && db->key_name_len[k] == n && memcmp(db->key_name_arena + db->key_name_off[k], s, n) == 0)
      return k;
  }
  return -1;
}

typedef struct {
  const orc_mix_db* db;
  const orc_mix_batch* b;
  const kmap* m;
  int64_t lo, hi;
  int64_t *pk, *en;
  int64_t n, cap;
  int members; /* ORC_MIX_MEMBERS: after each Red Hat group's entry, its members as -(entry + 1) */
} job;

static void push(job* j, int64_t p, int64_t e) {
  if (j->n == j->cap) {
    j->cap = j->cap ? j->cap * 2 : 4096;
    j->pk = realloc(j->pk, sizeof(int64_t) * (size_t)j->cap);
    j->en = realloc(j->en, sizeof(int64_t) * (size_t)j->cap);
  }
  j->pk[j->n] = p;
  j->en[j->n] = e;
  j->n++;
}

/* oracle.go extractKsplice: the first "ksplice..." segment of the lower-cased release */
static void ksplice(const char* s, size_t n, const char** out, size_t* on) {
  size_t st = 0;
  *out = "";
  *on = 0;
  for (size_t i = 0; i <= n; i++) {
    if (i == n || s[i] == '.') {
      size_t l = i - st;
      if (l >= 7) {
        static const char kw[] = "ksplice";
        int ok = 1;
        for (size_t q = 0; q < 7 && ok; q++) ok = (s[st + q] | 0x20) == kw[q];
        if (ok) {
          *out = s + st;
          *on = l;
          return;
        }
      }
      st = i + 1;
    }
  }
}

static int ks_eq(const char* a, size_t na, const char* b, size_t nb) {
  if (na != nb) return 0;
  for (size_t i = 0; i < na; i++)
    if ((a[i] | 0x20) != (b[i] | 0x20)) return 0;
  return 1;
}

typedef struct {
  int32_t vid;
  int64_t first, best;  /* entries: the first of the ID, the one holding the greatest fixed version */
  int64_t head, tail;   /* its members (entries that entered the uniq map), a list in mem[] */
} rhslot;

typedef struct {
  int64_t e, next;
} rhmem;

static int rh_cmp(const void* x, const void* y) {
  const rhslot *a = x, *b = y;
  return (a->vid > b->vid) - (a->vid < b->vid);
}

static void* run_job(void* arg) {
  job* j = arg;
  const orc_mix_db* db = j->db;
  const orc_mix_batch* b = j->b;
  rhslot* rh = NULL;
  int64_t rh_cap = 0;
  rhmem* mem = NULL;
  int64_t mem_n = 0, mem_cap = 0;
#define MEM_ADD(slot, ent)                                                 \
  do {                                                                     \
    if (mem_n == mem_cap) {                                                \
      mem_cap = mem_cap ? mem_cap * 2 : 256;                               \
      mem = realloc(mem, sizeof(rhmem) * (size_t)mem_cap);                 \
    }                                                                      \
    mem[mem_n] = (rhmem){(ent), -1};                                       \
    if ((slot)->tail >= 0) mem[(slot)->tail].next = mem_n;                 \
    else (slot)->head = mem_n;                                             \
    (slot)->tail = mem_n++;                                                \
  } while (0)
  for (int64_t i = j->lo; i < j->hi; i++) {
    const int32_t plat = b->plat[i];
    if (plat < 0 || plat >= db->n_plat || (b->skip && b->skip[i])) continue;
    const int drv = db->plat_driver[plat];
    const char* ver = b->ver_arena + b->ver_off[i];
    const size_t nv = b->ver_len[i];
    const char* name = b->name_arena + b->name_off[i];
    const size_t nn = b->name_len[i];
    orc_deb inst;
    int inst_ok = 1;
    if (drv == ORC_MX_DEBIAN) {
      if (orc_deb_parse(ver, nv, &inst)) continue; /* parse before lookup */
    }
    const int32_t k = kmap_get(j->m, db, plat, name, nn);
    if (k < 0) continue;
    const int64_t e0 = db->key_begin[k], e1 = db->key_begin[k + 1];
    switch (drv) {
      case ORC_MX_DEBIAN:
      case ORC_MX_UBUNTU: {
        if (drv == ORC_MX_UBUNTU) inst_ok = orc_deb_parse(ver, nv, &inst) == 0;
        if (!inst_ok) break;
        for (int64_t e = e0; e < e1; e++) {
          const uint32_t fl = db->fixed_len[e];
          if (fl == 0) {
            push(j, i, e);
            continue;
          }
          orc_deb fx;
          if (orc_deb_parse(db->arena + db->fixed_off[e], fl, &fx)) continue;
          if (orc_deb_cmp(&inst, &fx) < 0) push(j, i, e);
        }
        break;
      }
      case ORC_MX_ALPINE: {
        if (!orc_apk_valid(ver, nv)) break;
        for (int64_t e = e0; e < e1; e++) {
          const char* aff = db->arena + db->aff_off[e];
          const size_t na = db->aff_len[e];
          if (na) {
            if (!orc_apk_valid(aff, na) || orc_apk_cmp(aff, na, ver, nv) > 0) continue;
          }
          const char* fx = db->arena + db->fixed_off[e];
          const size_t nf = db->fixed_len[e];
          if (nf == 0) {
            push(j, i, e);
            continue;
          }
          if (orc_apk_valid(fx, nf) && orc_apk_cmp(ver, nv, fx, nf) < 0) push(j, i, e);
        }
        break;
      }
      case ORC_MX_ALMA:
      case ORC_MX_ROCKY:
      case ORC_MX_ORACLE: {
        const char* rel = "";
        size_t nr = 0;
        if (drv == ORC_MX_ORACLE) {
          const char* dash = memchr(ver, '-', nv);
          if (dash) ksplice(dash + 1, nv - (size_t)(dash + 1 - ver), &rel, &nr);
        }
        for (int64_t e = e0; e < e1; e++) {
          if (drv == ORC_MX_ROCKY && db->n_arch[e] >= 0) { /* the entry's arches must hold the package's */
            int ok = 0;
            for (int64_t q = db->ids_begin[e]; q < db->ids_begin[e] + db->n_arch[e] && !ok; q++) ok = db->ids[q] == b->arch[i];
            if (!ok) continue;
          }
          const char* fx = db->arena + db->fixed_off[e];
          const size_t nf = db->fixed_len[e];
          if (drv == ORC_MX_ORACLE) {
            const char* fk;
            size_t fn;
            ksplice(fx, nf, &fk, &fn);
            if (!ks_eq(fk, fn, rel, nr)) continue;
          }
          if (orc_rpm_cmp_str(ver, nv, fx, nf) < 0) push(j, i, e);
        }
        break;
      }
      case ORC_MX_REDHAT: {
        int64_t nslot = 0;
        mem_n = 0;
        for (int64_t e = e0; e < e1; e++) {
          const int64_t q0 = db->ids_begin[e], na = db->n_arch[e] > 0 ? db->n_arch[e] : 0, q1 = db->ids_begin[e + 1];
          int cpe_ok = 0; /* one of the entry's affected CPEs in the package's CPE set */
          for (int64_t q = q0 + na; q < q1 && !cpe_ok; q++)
            for (int64_t c = b->cpe_begin[i]; c < b->cpe_begin[i + 1] && !cpe_ok; c++) cpe_ok = db->ids[q] == b->cpe_ids[c];
          if (!cpe_ok) continue;
          if (na && b->arch[i] != b->noarch_id) {
            int ok = 0;
            for (int64_t q = q0; q < q0 + na && !ok; q++) ok = db->ids[q] == b->arch[i];
            if (!ok) continue;
          }
          const int32_t vid = db->vid[e];
          int64_t s = -1;
          for (int64_t q = 0; q < nslot; q++)
            if (rh[q].vid == vid) {
              s = q;
              break;
            }
          const char* fx = db->arena + db->fixed_off[e];
          const size_t nf = db->fixed_len[e];
          if (nf == 0) {
            if (s < 0) {
              if (nslot == rh_cap) {
                rh_cap = rh_cap ? rh_cap * 2 : 64;
                rh = realloc(rh, sizeof(rhslot) * (size_t)rh_cap);
              }
              rh[nslot] = (rhslot){vid, e, e, -1, -1};
              MEM_ADD(&rh[nslot], e);
              nslot++;
            }
            continue;
          }
          if (orc_rpm_cmp_str(ver, nv, fx, nf) < 0) {
            if (s >= 0) {  /* VendorIDs union; FixedVersion raised to the greatest */
              const int64_t bst = rh[s].best;
              if (orc_rpm_cmp_str(db->arena + db->fixed_off[bst], db->fixed_len[bst], fx, nf) < 0) rh[s].best = e;
              MEM_ADD(&rh[s], e);
            } else {
              if (nslot == rh_cap) {
                rh_cap = rh_cap ? rh_cap * 2 : 64;
                rh = realloc(rh, sizeof(rhslot) * (size_t)rh_cap);
              }
              rh[nslot] = (rhslot){vid, e, e, -1, -1};
              MEM_ADD(&rh[nslot], e);
              nslot++;
            }
          }
        }
        qsort(rh, (size_t)nslot, sizeof(rhslot), rh_cmp);
        for (int64_t q = 0; q < nslot; q++) {
          push(j, i, rh[q].best);
          if (j->members)
            for (int64_t x = rh[q].head; x >= 0; x = mem[x].next) push(j, i, -(mem[x].e + 1));
        }
        break;
      }
      case ORC_MX_LIB: {
        const int g = db->plat_grammar[plat];
        for (int64_t e = e0; e < e1; e++)
          if (orc_lib_is_vulnerable(g, ver, nv, db->lib_flags[e], db->arena + db->vul_off[e], db->vul_len[e],
                                    db->arena + db->sec_off[e], db->sec_len[e]) > 0)
            push(j, i, e);
        break;
      }
      default:
        break;
    }
  }
  free(rh);
  free(mem);
#undef MEM_ADD
  return NULL;
}

int64_t orc_mix_match(const orc_mix_db* db, const orc_mix_batch* b, int n_threads, int64_t* out_pkg,
                      int64_t* out_entry, int64_t cap) {
  return orc_mix_match_ex(db, b, n_threads, out_pkg, out_entry, cap, 0);
}

int64_t orc_mix_match_ex(const orc_mix_db* db, const orc_mix_batch* b, int n_threads, int64_t* out_pkg,
                         int64_t* out_entry, int64_t cap, int flags) {
  if (n_threads <= 0) n_threads = 1;
  kmap m;
  kmap_build(&m, db);
  job* jobs = calloc((size_t)n_threads, sizeof(job));
  pthread_t* th = calloc((size_t)n_threads, sizeof(pthread_t));
  const int64_t per = (b->n + n_threads - 1) / n_threads;
  for (int t = 0; t < n_threads; t++) {
    jobs[t].db = db;
    jobs[t].b = b;
    jobs[t].m = &m;
    jobs[t].members = (flags & ORC_MIX_MEMBERS) != 0;
    jobs[t].lo = (int64_t)t * per < b->n ? (int64_t)t * per : b->n;
    jobs[t].hi = jobs[t].lo + per < b->n ? jobs[t].lo + per : b->n;
    if (n_threads == 1) run_job(&jobs[t]);
    else pthread_create(&th[t], NULL, run_job, &jobs[t]);
  }
  int64_t total = 0;
  for (int t = 0; t < n_threads; t++) {
    if (n_threads > 1) pthread_join(th[t], NULL);
  }
  for (int t = 0; t < n_threads; t++) {
    for (int64_t x = 0; x < jobs[t].n; x++, total++)
      if (total < cap) {
        out_pkg[total] = jobs[t].pk[x];
        out_entry[total] = jobs[t].en[x];
      }
    free(jobs[t].pk);
    free(jobs[t].en);
  }
  free(jobs);
  free(th);
  free(m.h);
  free(m.key);
  return total;
}
