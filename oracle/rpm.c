/*
 * ORACLE - TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * go-rpm-version v0.0.0-20220614171824-631e686d1075 (reference go.mod:63).  Call sites:
 * redhat/redhat.go:125,149,162, alma/alma.go:68,70, rocky/rocky.go:68,71,
 * oracle/oracle.go:63,71, suse/suse.go:104,106, photon/photon.go:54,56,
 * mariner/mariner.go:57,72.
 *
 * NewVersion never fails: "[epoch:]version[-release]" with epoch = strconv.Atoi of the
 * text before the first ':' (0 when absent or unparsable) and the release after the FIRST
 * '-' (pinned by redhat_test.go "advisories have different arches": installed
 * 3.10.0-326.36-3.el7 < fixed 0:3.10.0-327.36.3.el7 holds only with that split).
 * Compare: epoch, then rpmvercmp(version), then rpmvercmp(release), where rpmvercmp splits
 * a string into the segments matched by ([a-zA-Z]+)|([0-9]+)|(~) (everything else is a
 * separator) and compares segment by segment: '~' sorts below any other segment, a
 * numeric segment above an alphabetic one, numbers by value (leading zeros dropped, then
 * length, then digits), letters bytewise; when one side runs out of segments, a '~' next
 * on the other side makes that side smaller, otherwise the side with more segments wins.
 * String() drops a zero epoch (redhat_test.go: 0:3.36.0-9.el7_6 -> 3.36.0-9.el7_6).
 */
#include <string.h>

#include "oracle.h"

typedef struct {
  const char* p;
  size_t n;
  int kind; /* 0 tilde, 1 alpha, 2 digits */
} seg;

static int is_alpha(int c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
static int is_dig(int c) { return c >= '0' && c <= '9'; }

/* next segment at or after *i; 0 when none left */
static int next_seg(const char* s, size_t n, size_t* i, seg* out) {
  while (*i < n && !is_alpha(s[*i]) && !is_dig(s[*i]) && s[*i] != '~') (*i)++;
  if (*i >= n) return 0;
  size_t b = *i;
  if (s[b] == '~') {
    out->kind = 0;
    (*i)++;
  } else if (is_alpha(s[b])) {
    out->kind = 1;
    while (*i < n && is_alpha(s[*i])) (*i)++;
  } else {
    out->kind = 2;
    while (*i < n && is_dig(s[*i])) (*i)++;
  }
  out->p = s + b;
  out->n = *i - b;
  return 1;
}

static int bytes_cmp(const char* a, size_t na, const char* b, size_t nb) {
  size_t m = na < nb ? na : nb;
  int c = memcmp(a, b, m);
  if (c) return c < 0 ? -1 : 1;
  return (na > nb) - (na < nb);
}

int orc_rpmvercmp(const char* a, size_t na, const char* b, size_t nb) {
  if (na == nb && memcmp(a, b, na) == 0) return 0;
  size_t ia = 0, ib = 0;
  seg x, y;
  for (;;) {
    int ha = next_seg(a, na, &ia, &x);
    int hb = next_seg(b, nb, &ib, &y);
    if (!ha || !hb) {
      if (!ha && !hb) return 0;
      if (ha) return x.kind == 0 ? -1 : 1;
      return y.kind == 0 ? 1 : -1;
    }
    if (x.kind == 0 || y.kind == 0) {
      if (x.kind != 0) return 1;
      if (y.kind != 0) return -1;
    }
    if (x.kind == 2) {
      if (y.kind != 2) return 1;
      while (x.n && x.p[0] == '0') x.p++, x.n--;
      while (y.n && y.p[0] == '0') y.p++, y.n--;
      if (x.n != y.n) return x.n > y.n ? 1 : -1;
    } else if (y.kind == 2) {
      return -1;
    }
    int c = bytes_cmp(x.p, x.n, y.p, y.n);
    if (c) return c;
  }
}

void orc_rpm_parse(const char* s, size_t n, orc_rpm* v) {
  v->epoch = 0;
  const char* colon = memchr(s, ':', n);
  if (colon) {
    /* strconv.Atoi: optional sign, decimal digits, fits int64; anything else -> 0 */
    const char* p = s;
    size_t m = (size_t)(colon - s);
    int neg = 0;
    long long e = 0;
    int ok = m > 0;
    size_t i = 0;
    if (m > 0 && (p[0] == '+' || p[0] == '-')) {
      neg = p[0] == '-';
      i = 1;
      ok = m > 1;
    }
    for (; ok && i < m; i++) {
      if (!is_dig(p[i])) { ok = 0; break; }
      int d = p[i] - '0';
      if (e > (9223372036854775807LL - d) / 10) { ok = 0; break; }
      e = e * 10 + d;
    }
    v->epoch = ok ? (neg ? -e : e) : 0;
    n -= m + 1;
    s = colon + 1;
  }
  const char* dash = memchr(s, '-', n);
  v->ver = s;
  v->nver = dash ? (size_t)(dash - s) : n;
  v->rel = dash ? dash + 1 : s + n;
  v->nrel = dash ? n - v->nver - 1 : 0;
}

int orc_rpm_cmp(const orc_rpm* a, const orc_rpm* b) {
  if (a->epoch != b->epoch) return a->epoch > b->epoch ? 1 : -1;
  int c = orc_rpmvercmp(a->ver, a->nver, b->ver, b->nver);
  if (c) return c;
  return orc_rpmvercmp(a->rel, a->nrel, b->rel, b->nrel);
}

int orc_rpm_cmp_str(const char* a, size_t na, const char* b, size_t nb) {
  orc_rpm x, y;
  orc_rpm_parse(a, na, &x);
  orc_rpm_parse(b, nb, &y);
  return orc_rpm_cmp(&x, &y);
}
