/*
 * ORACLE - TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * C restatement of the library comparers of oracle/library.py (the pairwise checker pinned by
 * the reference's compare_test.go tables): compare.IsVulnerable over go-version (GENERIC),
 * go-npm-version, go-pep440-version and go-mvn-version constraint strings, parsing the
 * installed version and every constraint per call as the reference does
 * (pkg/detector/library/compare/compare.go:21-55, matchVersion per comparer).  Used only by
 * oracle/mixmatch.c, the native CPU baseline of the mixed workloads (bench.py cpu_baseline);
 * tests/test_cport.py checks it against oracle/library.py on the synthetic workloads and the
 * KAT tables.
 *
 * Every function returns 1 / 0 for a match, and -1 when a version or constraint does not
 * parse (matchVersion's error: IsVulnerable then reports "not vulnerable").
 */
#include <ctype.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "oracle.h"

#define MAXSEG 32
#define MAXPRE 16

static int icmp64(uint64_t a, uint64_t b) { return (a > b) - (a < b); }

static int parse_u64(const char* s, size_t n, uint64_t* out) {
  uint64_t v = 0;
  if (n == 0) return -1;
  for (size_t i = 0; i < n; i++) {
    if (s[i] < '0' || s[i] > '9') return -1;
    if (v > (UINT64_MAX - (uint64_t)(s[i] - '0')) / 10) return -1; /* > 64 bits: malformed (UNPINNED) */
    v = v * 10 + (uint64_t)(s[i] - '0');
  }
  *out = v;
  return 0;
}

typedef struct { const char* p; size_t n; } span;

static int is_ident_ch(char c, int tilde) {
  return isalnum((unsigned char)c) || c == '-' || (tilde && c == '~');
}

/* pre-release identifiers: numeric < alphanumeric, numeric by value, else bytewise */
static int cmp_ident(span x, span y) {
  int xn = 1, yn = 1;
  for (size_t i = 0; i < x.n; i++) xn &= isdigit((unsigned char)x.p[i]) != 0;
  for (size_t i = 0; i < y.n; i++) yn &= isdigit((unsigned char)y.p[i]) != 0;
  if (xn && yn) {
    uint64_t a = 0, b = 0;
    if (parse_u64(x.p, x.n, &a) || parse_u64(y.p, y.n, &b)) {  /* huge numeric identifiers: by length, then bytes */
      if (x.n != y.n) return x.n < y.n ? -1 : 1;
      int c = memcmp(x.p, y.p, x.n);
      return (c > 0) - (c < 0);
    }
    return icmp64(a, b);
  }
  if (xn != yn) return xn ? -1 : 1;
  size_t m = x.n < y.n ? x.n : y.n;
  int c = memcmp(x.p, y.p, m);
  if (c) return (c > 0) - (c < 0);
  return (x.n > y.n) - (x.n < y.n);
}

static int cmp_pre(const span* a, int na, const span* b, int nb) {
  if (!na && !nb) return 0;
  if (!na) return 1;
  if (!nb) return -1;
  for (int i = 0; i < na && i < nb; i++) {
    int c = cmp_ident(a[i], b[i]);
    if (c) return c;
  }
  return (na > nb) - (na < nb);
}

static int split_pre(const char* s, size_t n, span* out, int tilde) {
  int k = 0;
  size_t st = 0;
  for (size_t i = 0; i <= n; i++) {
    if (i == n || s[i] == '.') {
      if (i == st || k == MAXPRE) return -1;
      for (size_t j = st; j < i; j++)
        if (!is_ident_ch(s[j], tilde)) return -1;
      out[k].p = s + st;
      out[k].n = i - st;
      k++;
      st = i + 1;
    }
  }
  return k;
}

/* ================================================================== GENERIC (go-version) */
typedef struct {
  uint64_t seg[MAXSEG];
  int nseg;
  span pre[MAXPRE];
  int npre;
  int specified;
} genver;

static int gen_parse(const char* s, size_t n, genver* v) {
  size_t i = 0;
  memset(v, 0, sizeof *v);
  if (i < n && s[i] == 'v') i++;
  for (;;) {
    size_t st = i;
    while (i < n && isdigit((unsigned char)s[i])) i++;
    if (i == st || v->nseg == MAXSEG || parse_u64(s + st, i - st, &v->seg[v->nseg])) return -1;
    v->nseg++;
    if (i + 1 < n && s[i] == '.' && isdigit((unsigned char)s[i + 1])) {
      i++;
      continue;
    }
    break;
  }
  v->specified = v->nseg;
  size_t pend = n;
  for (size_t j = i; j < n; j++)
    if (s[j] == '+') {
      pend = j;
      break;
    }
  if (pend < n) {  /* build metadata: identifiers, ignored for ordering */
    span tmp[MAXPRE];
    if (split_pre(s + pend + 1, n - pend - 1, tmp, 1) < 0) return -1;
  }
  if (i < pend) {
    if (s[i] == '-') {
      i++;
    } else if (!(isalpha((unsigned char)s[i]) || s[i] == '~')) {
      return -1;
    }
    int k = split_pre(s + i, pend - i, v->pre, 1);
    if (k < 0) return -1;
    v->npre = k;
  }
  return 0;
}

static int gen_cmp(const genver* a, const genver* b) {
  int n = a->nseg > b->nseg ? a->nseg : b->nseg;
  for (int i = 0; i < n; i++) {
    uint64_t x = i < a->nseg ? a->seg[i] : 0, y = i < b->nseg ? b->seg[i] : 0;
    if (x != y) return icmp64(x, y);
  }
  return cmp_pre(a->pre, a->npre, b->pre, b->npre);
}

/* v < upper (zero padded release comparison, pre-releases of upper excluded) */
static int lt_segs(const genver* v, const uint64_t* up, int nup) {
  int n = v->nseg > nup ? v->nseg : nup;
  for (int i = 0; i < n; i++) {
    uint64_t x = i < v->nseg ? v->seg[i] : 0, y = i < nup ? up[i] : 0;
    if (x != y) return x < y;
  }
  return 0;
}

static int gen_op(const char* op, const genver* v, const genver* c) {
  int r = gen_cmp(v, c);
  if (!strcmp(op, "") || !strcmp(op, "=") || !strcmp(op, "==")) return r == 0;
  if (!strcmp(op, "!=")) return r != 0;
  if (!strcmp(op, ">")) return r > 0;
  if (!strcmp(op, "<")) return r < 0;
  if (!strcmp(op, ">=") || !strcmp(op, "=>")) return r >= 0;
  if (!strcmp(op, "<=") || !strcmp(op, "=<")) return r <= 0;
  uint64_t up[MAXSEG];
  int nup;
  if (r < 0) return 0;
  if (!strcmp(op, "~>")) {
    nup = c->specified - 1 > 1 ? c->specified - 1 : 1;
  } else if (!strcmp(op, "~")) {
    nup = c->specified >= 2 ? 2 : 1;
  } else { /* ^ */
    int i = 0;
    while (i < c->specified - 1 && c->seg[i] == 0) i++;
    nup = i + 1;
  }
  for (int i = 0; i < nup; i++) up[i] = c->seg[i];
  up[nup - 1]++;
  return lt_segs(v, up, nup);
}

static const char* GEN_OPS[] = {"~>", ">=", "=>", "<=", "=<", "!=", "==", ">", "<", "=", "~", "^"};

static int gen_ver_char(char c) { return isalnum((unsigned char)c) || c == '.' || c == '-' || c == '~' || c == '+'; }

/* one "||" alternative: comparators (op? version) separated by spaces / commas */
static int gen_alt(const genver* v, const char* s, size_t n) {
  size_t i = 0;
  int all = 1, any = 0;
  while (i < n) {
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == ',')) i++;
    if (i >= n) break;
    const char* op = "";
    for (size_t k = 0; k < sizeof GEN_OPS / sizeof GEN_OPS[0]; k++) {
      size_t l = strlen(GEN_OPS[k]);
      if (i + l <= n && !memcmp(s + i, GEN_OPS[k], l)) {
        op = GEN_OPS[k];
        i += l;
        break;
      }
    }
    while (i < n && (s[i] == ' ' || s[i] == '\t')) i++;
    size_t st = i;
    while (i < n && gen_ver_char(s[i])) i++;
    genver c;
    if (i == st || gen_parse(s + st, i - st, &c)) return -1;
    any = 1;
    if (all && !gen_op(op, v, &c)) all = 0;
  }
  (void)any;
  return all;  /* no comparator at all: the validation pattern accepts it and all([]) holds */
}

typedef int (*alt_fn)(const void* v, const char* s, size_t n);

/* constraint = alternatives joined by "||": every alternative is parsed (NewConstraints
 * fails on any malformed one), the match is their OR */
static int any_alt(const void* v, const char* s, size_t n, alt_fn f) {
  int hit = 0;
  size_t st = 0;
  for (size_t i = 0; i <= n; i++) {
    if (i == n || (i + 1 < n && s[i] == '|' && s[i + 1] == '|')) {
      int r = f(v, s + st, i - st);
      if (r < 0) return -1;
      hit |= r;
      if (i < n) i++;
      st = i + 1;
    }
  }
  return hit;
}

static int gen_alt_v(const void* v, const char* s, size_t n) { return gen_alt((const genver*)v, s, n); }

int orc_gen_match(const char* ver, size_t nv, const char* c, size_t nc) {
  genver v;
  if (gen_parse(ver, nv, &v)) return -1;
  return any_alt(&v, c, nc, gen_alt_v);
}

/* ========================================================================= NPM (semver) */
typedef struct {
  uint64_t t[3];
  span pre[MAXPRE];
  int npre;
} npmver;

static int npm_cmp(const npmver* a, const npmver* b) {
  for (int i = 0; i < 3; i++)
    if (a->t[i] != b->t[i]) return icmp64(a->t[i], b->t[i]);
  return cmp_pre(a->pre, a->npre, b->pre, b->npre);
}

/* [v=]* N.N.N (-?pre)? (+build)? with surrounding spaces */
static int npm_parse(const char* s, size_t n, npmver* v) {
  size_t i = 0;
  memset(v, 0, sizeof *v);
  while (i < n && s[i] == ' ') i++;
  while (n > i && s[n - 1] == ' ') n--;
  while (i < n && (s[i] == 'v' || s[i] == '=')) i++;
  while (i < n && s[i] == ' ') i++;
  for (int k = 0; k < 3; k++) {
    size_t st = i;
    while (i < n && isdigit((unsigned char)s[i])) i++;
    if (i == st || parse_u64(s + st, i - st, &v->t[k])) return -1;
    if (k < 2) {
      if (i >= n || s[i] != '.') return -1;
      i++;
    }
  }
  size_t pend = n;
  for (size_t j = i; j < n; j++)
    if (s[j] == '+') {
      pend = j;
      break;
    }
  if (pend < n) {
    span tmp[MAXPRE];
    if (split_pre(s + pend + 1, n - pend - 1, tmp, 0) < 0) return -1;
  }
  if (i < pend) {
    if (s[i] == '-') i++;
    int k = split_pre(s + i, pend - i, v->pre, 0);
    if (k < 0) return -1;
    v->npre = k;
  }
  return 0;
}

typedef struct {
  char op[3];
  npmver c;
} npmcmp;

static int is_xr(const char* s, size_t n) { return n == 1 && (s[0] == 'x' || s[0] == 'X' || s[0] == '*'); }

/* a partial version "[v=]* (x|N)(.(x|N)(.(x|N)(-pre)?(+b)?)?)?" -> numbers written before any x */
static int npm_partial(const char* s, size_t n, uint64_t* nums, int* nn, npmver* full) {
  size_t i = 0;
  *nn = 0;
  memset(full, 0, sizeof *full);
  while (i < n && (s[i] == 'v' || s[i] == '=')) i++;
  int stop = 0;
  for (int k = 0; k < 3; k++) {
    size_t st = i;
    while (i < n && (isdigit((unsigned char)s[i]) || s[i] == 'x' || s[i] == 'X' || s[i] == '*')) i++;
    if (i == st) return -1;
    if (is_xr(s + st, i - st)) {
      stop = 1;
    } else {
      for (size_t j = st; j < i; j++)
        if (!isdigit((unsigned char)s[j])) return -1;
      if (!stop) {
        if (parse_u64(s + st, i - st, &nums[*nn])) return -1;
        (*nn)++;
      }
    }
    if (i < n && s[i] == '.' && k < 2) {
      i++;
      continue;
    }
    break;
  }
  size_t pend = n;
  for (size_t j = i; j < n; j++)
    if (s[j] == '+') {
      pend = j;
      break;
    }
  if (i < pend) {
    if (*nn != 3 && !stop) return -1;
    if (s[i] == '-') i++;
    int k = split_pre(s + i, pend - i, full->pre, 0);
    if (k < 0) return -1;
    if (*nn == 3) full->npre = k;
  }
  for (int k = 0; k < 3; k++) full->t[k] = k < *nn ? nums[k] : 0;
  return 0;
}

static span kZero = {"0", 1};

static void mk(npmcmp* o, const char* op, const uint64_t* t, const span* pre, int npre) {
  strcpy(o->op, op);
  memset(&o->c, 0, sizeof o->c);
  for (int k = 0; k < 3; k++) o->c.t[k] = t[k];
  for (int k = 0; k < npre; k++) o->c.pre[k] = pre[k];
  o->c.npre = npre;
}

/* one comparator token -> primitive comparators (node-semver desugaring, oracle _cmp_lo /
 * _tilde / _caret) */
static int npm_desugar(const char* op, const char* s, size_t n, npmcmp* out, int* k) {
  uint64_t nums[3] = {0, 0, 0};
  int nn = 0;
  npmver full;
  if (npm_partial(s, n, nums, &nn, &full)) return -1;
  uint64_t z[3] = {0, 0, 0}, f[3] = {full.t[0], full.t[1], full.t[2]}, up[3] = {0, 0, 0};
  if (!strcmp(op, "~") || !strcmp(op, "~>")) {
    if (nn == 0) { mk(&out[(*k)++], ">=", z, NULL, 0); return 0; }
    if (nn == 1) up[0] = nums[0] + 1;
    else { up[0] = nums[0]; up[1] = nums[1] + 1; }
    mk(&out[(*k)++], ">=", f, full.pre, nn == 3 ? full.npre : 0);
    mk(&out[(*k)++], "<", up, &kZero, 1);
    return 0;
  }
  if (!strcmp(op, "^")) {
    if (nn == 0) { mk(&out[(*k)++], ">=", z, NULL, 0); return 0; }
    if (nums[0] != 0 || nn == 1) up[0] = nums[0] + 1;
    else if (nn == 2 || nums[1] != 0) up[1] = nums[1] + 1;
    else up[2] = nums[2] + 1;
    mk(&out[(*k)++], ">=", f, full.pre, nn == 3 ? full.npre : 0);
    mk(&out[(*k)++], "<", up, &kZero, 1);
    return 0;
  }
  if (nn == 0) {
    if (!*op || !strcmp(op, "=") || !strcmp(op, ">=") || !strcmp(op, "<=")) mk(&out[(*k)++], ">=", z, NULL, 0);
    else mk(&out[(*k)++], "<", z, &kZero, 1);
    return 0;
  }
  if (nn == 3) {
    mk(&out[(*k)++], *op ? op : "=", f, full.pre, full.npre);
    return 0;
  }
  for (int i = 0; i < nn; i++) up[i] = nums[i];
  up[nn - 1]++;
  if (!*op || !strcmp(op, "=")) {
    mk(&out[(*k)++], ">=", f, NULL, 0);
    mk(&out[(*k)++], "<", up, &kZero, 1);
  } else if (!strcmp(op, ">")) {
    mk(&out[(*k)++], ">=", up, NULL, 0);
  } else if (!strcmp(op, ">=")) {
    mk(&out[(*k)++], ">=", f, NULL, 0);
  } else if (!strcmp(op, "<")) {
    mk(&out[(*k)++], "<", f, &kZero, 1);
  } else if (!strcmp(op, "<=")) {
    mk(&out[(*k)++], "<", up, &kZero, 1);
  } else {
    return -1;
  }
  return 0;
}

static int npm_test(const char* op, const npmver* v, const npmver* c) {
  int r = npm_cmp(v, c);
  if (!*op || !strcmp(op, "=")) return r == 0;
  if (!strcmp(op, "<")) return r < 0;
  if (!strcmp(op, "<=")) return r <= 0;
  if (!strcmp(op, ">")) return r > 0;
  return r >= 0;
}

#define MAXCMP 64

static int npm_alt(const void* vp, const char* s0, size_t n0) {
  const npmver* v = (const npmver*)vp;
  char buf[512];
  if (n0 >= sizeof buf) return -1;
  for (size_t i = 0; i < n0; i++) buf[i] = s0[i] == ',' ? ' ' : s0[i];
  size_t b = 0, e = n0;
  while (b < e && isspace((unsigned char)buf[b])) b++;
  while (e > b && isspace((unsigned char)buf[e - 1])) e--;
  const char* s = buf + b;
  size_t n = e - b;
  npmcmp cs[MAXCMP];
  int k = 0;
  /* hyphen range "A - B" */
  size_t h = 0;
  int hy = 0;
  for (size_t i = 0; i + 2 < n; i++)
    if (s[i] == ' ' && s[i + 1] == '-' && s[i + 2] == ' ') {
      h = i;
      hy = 1;
      break;
    }
  if (hy) {
    size_t a0 = 0, a1 = h, b0 = h + 3, b1 = n;
    while (a1 > a0 && s[a1 - 1] == ' ') a1--;
    while (b0 < b1 && s[b0] == ' ') b0++;
    for (size_t i = a0; i < a1; i++)
      if (isspace((unsigned char)s[i])) return -1;
    for (size_t i = b0; i < b1; i++)
      if (isspace((unsigned char)s[i])) return -1;
    uint64_t lo[3], hi[3];
    int nl = 0, nh = 0;
    npmver fl, fh;
    if (npm_partial(s + a0, a1 - a0, lo, &nl, &fl) || npm_partial(s + b0, b1 - b0, hi, &nh, &fh)) return -1;
    uint64_t z[3] = {0, 0, 0};
    if (nl) mk(&cs[k++], ">=", fl.t, fl.pre, nl == 3 ? fl.npre : 0);
    if (nh == 3) {
      mk(&cs[k++], "<=", fh.t, fh.pre, fh.npre);
    } else if (nh) {
      uint64_t up[3] = {0, 0, 0};
      for (int i = 0; i < nh; i++) up[i] = hi[i];
      up[nh - 1]++;
      mk(&cs[k++], "<", up, &kZero, 1);
    }
    if (!k) mk(&cs[k++], ">=", z, NULL, 0);
  } else {
    size_t i = 0;
    while (i < n) {
      while (i < n && isspace((unsigned char)s[i])) i++;
      if (i >= n) break;
      char op[3] = "";
      static const char* OPS[] = {"<=", ">=", "~>", "<", ">", "=", "~", "^"};
      for (size_t q = 0; q < sizeof OPS / sizeof OPS[0]; q++) {
        size_t l = strlen(OPS[q]);
        if (i + l <= n && !memcmp(s + i, OPS[q], l)) {
          memcpy(op, OPS[q], l);
          op[l] = 0;
          i += l;
          break;
        }
      }
      while (i < n && isspace((unsigned char)s[i])) i++;
      size_t st = i;
      while (i < n && !isspace((unsigned char)s[i]) && !strchr("<>=~^,", s[i])) i++;
      if (i == st || k + 2 > MAXCMP) return -1;
      if (npm_desugar(op, s + st, i - st, cs, &k)) return -1;
    }
    if (!k) {
      uint64_t z[3] = {0, 0, 0};
      mk(&cs[k++], ">=", z, NULL, 0);
    }
  }
  for (int i = 0; i < k; i++)
    if (!npm_test(cs[i].op, v, &cs[i].c)) return 0;
  if (v->npre) { /* a pre-release only satisfies a set naming a pre-release of its [major, minor, patch] */
    for (int i = 0; i < k; i++)
      if (cs[i].c.npre && !memcmp(cs[i].c.t, v->t, sizeof v->t)) return 1;
    return 0;
  }
  return 1;
}

int orc_npm_match(const char* ver, size_t nv, const char* c, size_t nc) {
  npmver v;
  if (npm_parse(ver, nv, &v)) return -1;
  return any_alt(&v, c, nc, npm_alt);
}

/* =========================================================================== PEP 440 === */
typedef struct {
  uint64_t epoch;
  uint64_t rel[MAXSEG];
  int nrel;
  int pre_l;  /* -1 none, 0 a, 1 b, 2 rc */
  uint64_t pre_n;
  int has_post;
  uint64_t post;
  int has_dev;
  uint64_t dev;
  int has_local;
  span loc[MAXPRE];
  int nloc;
} pepver;

static int ieq(const char* s, size_t n, const char* w) { return strlen(w) == n && !strncasecmp(s, w, n); }

static int sep(char c) { return c == '-' || c == '_' || c == '.'; }

static size_t alpha_run(const char* s, size_t i, size_t n) {
  while (i < n && isalpha((unsigned char)s[i])) i++;
  return i;
}

static int num_opt(const char* s, size_t* i, size_t n, uint64_t* out) {
  size_t st = *i;
  while (*i < n && isdigit((unsigned char)s[*i])) (*i)++;
  if (*i == st) {
    *out = 0;
    return 0;
  }
  return parse_u64(s + st, *i - st, out);
}

static int pep_parse(const char* s, size_t n, pepver* v) {
  memset(v, 0, sizeof *v);
  v->pre_l = -1;
  size_t i = 0;
  while (i < n && isspace((unsigned char)s[i])) i++;
  while (n > i && isspace((unsigned char)s[n - 1])) n--;
  if (i < n && (s[i] == 'v' || s[i] == 'V')) i++;
  /* epoch */
  size_t j = i;
  while (j < n && isdigit((unsigned char)s[j])) j++;
  if (j < n && s[j] == '!' && j > i) {
    if (parse_u64(s + i, j - i, &v->epoch)) return -1;
    i = j + 1;
  }
  for (;;) {
    size_t st = i;
    while (i < n && isdigit((unsigned char)s[i])) i++;
    if (i == st || v->nrel == MAXSEG || parse_u64(s + st, i - st, &v->rel[v->nrel])) return -1;
    v->nrel++;
    if (i + 1 < n && s[i] == '.' && isdigit((unsigned char)s[i + 1])) {
      i++;
      continue;
    }
    break;
  }
  /* pre */
  {
    size_t k = i;
    if (k < n && sep(s[k])) k++;
    size_t e = alpha_run(s, k, n);
    const char* w = s + k;
    size_t wn = e - k;
    int l = -1;
    if (ieq(w, wn, "alpha") || ieq(w, wn, "a")) l = 0;
    else if (ieq(w, wn, "beta") || ieq(w, wn, "b")) l = 1;
    else if (ieq(w, wn, "c") || ieq(w, wn, "rc") || ieq(w, wn, "pre") || ieq(w, wn, "preview")) l = 2;
    if (l >= 0) {
      size_t q = e;
      if (q < n && sep(s[q]) && q + 1 < n && isdigit((unsigned char)s[q + 1])) q++;
      if (num_opt(s, &q, n, &v->pre_n)) return -1;
      v->pre_l = l;
      i = q;
    }
  }
  /* post */
  if (i < n && s[i] == '-' && i + 1 < n && isdigit((unsigned char)s[i + 1])) {
    size_t q = i + 1;
    if (num_opt(s, &q, n, &v->post)) return -1;
    v->has_post = 1;
    i = q;
  } else {
    size_t k = i;
    if (k < n && sep(s[k])) k++;
    size_t e = alpha_run(s, k, n);
    if (ieq(s + k, e - k, "post") || ieq(s + k, e - k, "rev") || ieq(s + k, e - k, "r")) {
      size_t q = e;
      if (q < n && sep(s[q]) && q + 1 < n && isdigit((unsigned char)s[q + 1])) q++;
      if (num_opt(s, &q, n, &v->post)) return -1;
      v->has_post = 1;
      i = q;
    }
  }
  /* dev */
  {
    size_t k = i;
    if (k < n && sep(s[k])) k++;
    size_t e = alpha_run(s, k, n);
    if (ieq(s + k, e - k, "dev")) {
      size_t q = e;
      if (q < n && sep(s[q]) && q + 1 < n && isdigit((unsigned char)s[q + 1])) q++;
      if (num_opt(s, &q, n, &v->dev)) return -1;
      v->has_dev = 1;
      i = q;
    }
  }
  /* local */
  if (i < n && s[i] == '+') {
    i++;
    size_t st = i;
    for (;;) {
      size_t a = i;
      while (i < n && isalnum((unsigned char)s[i])) i++;
      if (i == a || v->nloc == MAXPRE) return -1;
      v->loc[v->nloc].p = s + a;
      v->loc[v->nloc].n = i - a;
      v->nloc++;
      if (i < n && sep(s[i])) {
        i++;
        continue;
      }
      break;
    }
    v->has_local = i > st;
  }
  return i == n ? 0 : -1;
}

static int pep_is_pre(const pepver* v) { return v->pre_l >= 0 || v->has_dev; }

/* public part: epoch, release (trailing zeros ignored), pre, post, dev */
static int pep_cmp_public(const pepver* a, const pepver* b) {
  if (a->epoch != b->epoch) return icmp64(a->epoch, b->epoch);
  int n = a->nrel > b->nrel ? a->nrel : b->nrel;
  for (int i = 0; i < n; i++) {
    uint64_t x = i < a->nrel ? a->rel[i] : 0, y = i < b->nrel ? b->rel[i] : 0;
    if (x != y) return icmp64(x, y);
  }
  /* pre: dev-only release < pre-releases < release */
  int ka = (a->pre_l < 0 && !a->has_post && a->has_dev) ? -1 : a->pre_l < 0 ? 3 : 1;
  int kb = (b->pre_l < 0 && !b->has_post && b->has_dev) ? -1 : b->pre_l < 0 ? 3 : 1;
  if (ka != kb) return (ka > kb) - (ka < kb);
  if (ka == 1) {
    if (a->pre_l != b->pre_l) return (a->pre_l > b->pre_l) - (a->pre_l < b->pre_l);
    if (a->pre_n != b->pre_n) return icmp64(a->pre_n, b->pre_n);
  }
  if (a->has_post != b->has_post) return a->has_post ? 1 : -1;
  if (a->has_post && a->post != b->post) return icmp64(a->post, b->post);
  if (a->has_dev != b->has_dev) return a->has_dev ? -1 : 1;
  if (a->has_dev && a->dev != b->dev) return icmp64(a->dev, b->dev);
  return 0;
}

static int loc_cmp(span x, span y) {
  int xn = 1, yn = 1;
  for (size_t i = 0; i < x.n; i++) xn &= isdigit((unsigned char)x.p[i]) != 0;
  for (size_t i = 0; i < y.n; i++) yn &= isdigit((unsigned char)y.p[i]) != 0;
  if (xn && yn) return cmp_ident(x, y);
  if (xn != yn) return xn ? 1 : -1; /* numeric > alphanumeric */
  size_t m = x.n < y.n ? x.n : y.n;
  for (size_t i = 0; i < m; i++) {
    int a = tolower((unsigned char)x.p[i]), b = tolower((unsigned char)y.p[i]);
    if (a != b) return a < b ? -1 : 1;
  }
  return (x.n > y.n) - (x.n < y.n);
}

static int pep_cmp(const pepver* a, const pepver* b) {
  int r = pep_cmp_public(a, b);
  if (r) return r;
  if (a->has_local != b->has_local) return a->has_local ? 1 : -1;
  for (int i = 0; i < a->nloc && i < b->nloc; i++) {
    int c = loc_cmp(a->loc[i], b->loc[i]);
    if (c) return c;
  }
  return (a->nloc > b->nloc) - (a->nloc < b->nloc);
}

static int pep_base_eq(const pepver* a, const pepver* b) {
  if (a->epoch != b->epoch) return 0;
  int n = a->nrel > b->nrel ? a->nrel : b->nrel;
  for (int i = 0; i < n; i++) {
    uint64_t x = i < a->nrel ? a->rel[i] : 0, y = i < b->nrel ? b->rel[i] : 0;
    if (x != y) return 0;
  }
  return 1;
}

static int pep_prefix(const pepver* v, const pepver* s) {
  if (v->epoch != s->epoch) return 0;
  for (int i = 0; i < s->nrel; i++)
    if ((i < v->nrel ? v->rel[i] : 0) != s->rel[i]) return 0;
  return 1;
}

static int pep_check(const char* op, const pepver* v, const char* spec, size_t ns) {
  if (ns == 1 && spec[0] == '*') return 1;
  pepver s;
  int star = ns >= 2 && spec[ns - 1] == '*' && spec[ns - 2] == '.';
  if (pep_parse(spec, star ? ns - 2 : ns, &s)) return -1;
  if (!strcmp(op, "~=")) {
    if (s.nrel < 2) return -1;
    pepver pfx = s;
    pfx.nrel--;
    return pep_cmp_public(v, &s) >= 0 && pep_prefix(v, &pfx);
  }
  if ((!strcmp(op, "==") || !strcmp(op, "!=")) && star) {
    int r = pep_prefix(v, &s);
    return !strcmp(op, "==") ? r : !r;
  }
  if (!strcmp(op, "===")) return pep_cmp(v, &s) == 0;
  if (!strcmp(op, "==") || !strcmp(op, "!=")) {
    int r = s.has_local ? pep_cmp(v, &s) == 0 : pep_cmp_public(v, &s) == 0;
    return !strcmp(op, "==") ? r : !r;
  }
  if (!strcmp(op, "<=")) return pep_cmp_public(v, &s) <= 0;
  if (!strcmp(op, ">=")) return pep_cmp_public(v, &s) >= 0;
  if (!strcmp(op, "<")) {
    if (!(pep_cmp(v, &s) < 0)) return 0;
    if (!pep_is_pre(&s) && pep_is_pre(v) && pep_base_eq(v, &s)) return 0;
    return 1;
  }
  if (!strcmp(op, ">")) {
    if (!(pep_cmp(v, &s) > 0)) return 0;
    if (!s.has_post && v->has_post && pep_base_eq(v, &s)) return 0;
    if (v->has_local && pep_base_eq(v, &s)) return 0;
    return 1;
  }
  return -1;
}

static int pep_alt(const void* vp, const char* s, size_t n) {
  const pepver* v = (const pepver*)vp;
  size_t b = 0, e = n;
  while (b < e && isspace((unsigned char)s[b])) b++;
  while (e > b && isspace((unsigned char)s[e - 1])) e--;
  if (e - b == 1 && s[b] == '*') return 1;
  struct { char op[4]; size_t st, n; } cs[MAXCMP];
  int k = 0;
  size_t i = b;
  while (i < e) {
    if (s[i] == ',' || s[i] == ' ') {
      i++;
      continue;
    }
    char op[4] = "==";
    static const char* OPS[] = {"~=", "===", "==", "!=", "<=", ">=", "<", ">"};
    for (size_t q = 0; q < sizeof OPS / sizeof OPS[0]; q++) {
      size_t l = strlen(OPS[q]);
      if (i + l <= e && !memcmp(s + i, OPS[q], l)) {
        memcpy(op, OPS[q], l);
        op[l] = 0;
        i += l;
        break;
      }
    }
    while (i < e && isspace((unsigned char)s[i])) i++;
    size_t st = i;
    while (i < e && !isspace((unsigned char)s[i]) && !strchr(",<>=!~", s[i])) i++;
    if (i == st || k == MAXCMP) return -1;
    pepver chk;
    int star = i - st >= 2 && s[i - 1] == '*' && s[i - 2] == '.';
    if (pep_parse(s + st, star ? i - st - 2 : i - st, &chk)) return -1; /* NewSpecifiers validates all first */
    if (!strcmp(op, "~=") && chk.nrel < 2) return -1;
    strcpy(cs[k].op, op);
    cs[k].st = st;
    cs[k].n = i - st;
    k++;
  }
  if (!k) return -1;
  for (int q = 0; q < k; q++) {
    int r = pep_check(cs[q].op, v, s + cs[q].st, cs[q].n);
    if (r < 0) return -1;
    if (!r) return 0;
  }
  return 1;
}

int orc_pep_match(const char* ver, size_t nv, const char* c, size_t nc) {
  pepver v;
  if (pep_parse(ver, nv, &v)) return -1;
  return any_alt(&v, c, nc, pep_alt);
}

/* ============================================================= MAVEN (ComparableVersion) */
enum { MI_INT, MI_STR, MI_LIST };
typedef struct {
  int kind;
  uint64_t v;      /* int */
  int q;           /* str: qualifier rank (0..6) or 7 = unknown, ordered after by text */
  span s;          /* str text (lower-cased copy) */
  int first, n;    /* list: children items[first .. first + n) as child indices */
} mitem;

#define MAXMI 96
typedef struct {
  mitem it[MAXMI];
  int kids[MAXMI];  /* child index lists, per list contiguous */
  int nit;
  char low[256];
} mver;

static const char* QUALS[] = {"alpha", "beta", "milestone", "rc", "snapshot", "", "sp"};

static void mstr(mitem* m, const char* s, size_t n, int followed_by_digit) {
  m->kind = MI_STR;
  if (followed_by_digit && n == 1) {
    if (s[0] == 'a') { s = "alpha"; n = 5; }
    else if (s[0] == 'b') { s = "beta"; n = 4; }
    else if (s[0] == 'm') { s = "milestone"; n = 9; }
  }
  if ((n == 2 && !memcmp(s, "ga", 2)) || (n == 5 && !memcmp(s, "final", 5)) || (n == 7 && !memcmp(s, "release", 7)))
    n = 0;
  else if (n == 2 && !memcmp(s, "cr", 2)) { s = "rc"; n = 2; }
  m->s.p = s;
  m->s.n = n;
  m->q = 7;
  for (int i = 0; i < 7; i++)
    if (strlen(QUALS[i]) == n && !memcmp(QUALS[i], s, n)) m->q = i;
}

static int m_is_null(const mver* V, const mitem* m) {
  if (m->kind == MI_INT) return m->v == 0;
  if (m->kind == MI_STR) return m->s.n == 0;
  (void)V;
  return m->n == 0;
}

/* parse tree built with an explicit stack of open lists; children are recorded in order */
typedef struct {
  int list;                 /* item index of the list */
  int ch[MAXMI];
  int nch;
} mframe;

static int madd(mver* V, mframe* f, mitem m) {
  if (V->nit == MAXMI || f->nch == MAXMI) return -1;
  V->it[V->nit] = m;
  f->ch[f->nch++] = V->nit;
  return V->nit++;
}

static int mitem_of(mver* V, mframe* f, int is_digit, const char* s, size_t n) {
  mitem m;
  memset(&m, 0, sizeof m);
  if (is_digit) {
    m.kind = MI_INT;
    if (parse_u64(s, n, &m.v)) {  /* beyond 64 bits: saturate (UNPINNED; the oracle uses big ints) */
      m.v = UINT64_MAX;
    }
  } else {
    mstr(&m, s, n, 0);
  }
  return madd(V, f, m);
}

static int mvn_parse_c(const char* s0, size_t n, mver* V) {
  if (n >= sizeof V->low) return -1;
  for (size_t i = 0; i < n; i++) V->low[i] = (char)tolower((unsigned char)s0[i]);
  const char* s = V->low;
  V->nit = 0;
  mframe stack[32];
  int depth = 0, kidp = 0;
  mitem root;
  memset(&root, 0, sizeof root);
  root.kind = MI_LIST;
  V->it[V->nit++] = root;
  stack[0].list = 0;
  stack[0].nch = 0;
  int is_digit = 0;
  size_t start = 0;
  for (size_t i = 0; i < n; i++) {
    char c = s[i];
    mframe* f = &stack[depth];
    if (c == '.') {
      if (i == start) {
        mitem z;
        memset(&z, 0, sizeof z);
        z.kind = MI_INT;
        if (madd(V, f, z) < 0) return -1;
      } else if (mitem_of(V, f, is_digit, s + start, i - start) < 0) {
        return -1;
      }
      start = i + 1;
    } else if (c == '-') {
      if (i == start) {
        mitem z;
        memset(&z, 0, sizeof z);
        z.kind = MI_INT;
        if (madd(V, f, z) < 0) return -1;
      } else if (mitem_of(V, f, is_digit, s + start, i - start) < 0) {
        return -1;
      }
      start = i + 1;
      mitem l;
      memset(&l, 0, sizeof l);
      l.kind = MI_LIST;
      int li = madd(V, f, l);
      if (li < 0 || depth + 1 == 32) return -1;
      stack[++depth].list = li;
      stack[depth].nch = 0;
    } else if (c >= '0' && c <= '9') {
      if (!is_digit && i > start) {
        mitem m;
        memset(&m, 0, sizeof m);
        mstr(&m, s + start, i - start, 1);
        if (madd(V, f, m) < 0) return -1;
        start = i;
        mitem l;
        memset(&l, 0, sizeof l);
        l.kind = MI_LIST;
        int li = madd(V, f, l);
        if (li < 0 || depth + 1 == 32) return -1;
        stack[++depth].list = li;
        stack[depth].nch = 0;
      }
      is_digit = 1;
    } else {
      if (is_digit && i > start) {
        if (mitem_of(V, f, 1, s + start, i - start) < 0) return -1;
        start = i;
        mitem l;
        memset(&l, 0, sizeof l);
        l.kind = MI_LIST;
        int li = madd(V, f, l);
        if (li < 0 || depth + 1 == 32) return -1;
        stack[++depth].list = li;
        stack[depth].nch = 0;
      }
      is_digit = 0;
    }
  }
  if (n > start && mitem_of(V, &stack[depth], is_digit, s + start, n - start) < 0) return -1;
  /* close the lists innermost first: normalize (drop trailing nulls up to the last non-list)
   * and record their children */
  for (int d = depth; d >= 0; d--) {
    mframe* f = &stack[d];
    int k = f->nch;
    for (int i = k - 1; i >= 0; i--) {
      const mitem* m = &V->it[f->ch[i]];
      if (m_is_null(V, m)) {
        for (int j = i; j + 1 < k; j++) f->ch[j] = f->ch[j + 1];
        k--;
      } else if (m->kind != MI_LIST) {
        break;
      }
    }
    if (kidp + k > MAXMI) return -1;
    V->it[f->list].first = kidp;
    V->it[f->list].n = k;
    for (int i = 0; i < k; i++) V->kids[kidp++] = f->ch[i];
  }
  return 0;
}

static int qcmp(const mitem* a, const mitem* b) {
  if (a->q != b->q) return (a->q > b->q) - (a->q < b->q);
  if (a->q != 7) return 0;
  size_t m = a->s.n < b->s.n ? a->s.n : b->s.n;
  int c = memcmp(a->s.p, b->s.p, m);
  if (c) return (c > 0) - (c < 0);
  return (a->s.n > b->s.n) - (a->s.n < b->s.n);
}

static int m_cmp(const mver* A, const mitem* a, const mver* B, const mitem* b);

static int m_cmp_null(const mver* A, const mitem* a) {
  if (a->kind == MI_INT) return a->v == 0 ? 0 : 1;
  if (a->kind == MI_STR) {
    mitem r;
    memset(&r, 0, sizeof r);
    r.kind = MI_STR;
    r.q = 5;
    r.s.p = "";
    return qcmp(a, &r);
  }
  if (a->n == 0) return 0;
  return m_cmp_null(A, &A->it[A->kids[a->first]]);
}

static int m_cmp(const mver* A, const mitem* a, const mver* B, const mitem* b) {
  if (a->kind == MI_INT) {
    if (b->kind == MI_INT) return icmp64(a->v, b->v);
    return 1;
  }
  if (a->kind == MI_STR) {
    if (b->kind == MI_INT) return -1;
    if (b->kind == MI_STR) return qcmp(a, b);
    return -1;
  }
  if (b->kind == MI_INT) return -1;
  if (b->kind == MI_STR) return 1;
  int n = a->n > b->n ? a->n : b->n;
  for (int i = 0; i < n; i++) {
    const mitem* x = i < a->n ? &A->it[A->kids[a->first + i]] : NULL;
    const mitem* y = i < b->n ? &B->it[B->kids[b->first + i]] : NULL;
    int r = x == NULL ? (y == NULL ? 0 : -m_cmp_null(B, y)) : y == NULL ? m_cmp_null(A, x) : m_cmp(A, x, B, y);
    if (r) return r;
  }
  return 0;
}

static int mvn_valid(const char* s, size_t n) {
  if (n == 0 || !isalnum((unsigned char)s[0])) return 0;
  for (size_t i = 1; i < n; i++)
    if (!isalnum((unsigned char)s[i]) && !strchr(".-_+", s[i])) return 0;
  return 1;
}

static int mvn_new(const char* s, size_t n, mver* V) {
  while (n && isspace((unsigned char)*s)) { s++; n--; }
  while (n && isspace((unsigned char)s[n - 1])) n--;
  if (!mvn_valid(s, n)) return -1;
  return mvn_parse_c(s, n, V);
}

static int mvn_vcmp(const mver* a, const mver* b) { return m_cmp(a, &a->it[0], b, &b->it[0]); }

static int mvn_alt(const void* vp, const char* s, size_t n) {
  const mver* v = (const mver*)vp;
  size_t b = 0, e = n;
  while (b < e && isspace((unsigned char)s[b])) b++;
  while (e > b && isspace((unsigned char)s[e - 1])) e--;
  static __thread mver c, c2;
  if (b < e && (s[b] == '[' || s[b] == '(')) { /* range list "[a,b),(c,]" */
    size_t i = b;
    int hit = 0;
    while (i < e) {
      if (s[i] == ',' || s[i] == ' ') {
        i++;
        continue;
      }
      if (s[i] != '[' && s[i] != '(') return -1;
      size_t end = i + 1;
      while (end < e && s[end] != ']' && s[end] != ')') end++;
      if (end >= e) return -1;
      int lo_incl = s[i] == '[', hi_incl = s[end] == ']';
      size_t comma = i + 1;
      while (comma < end && s[comma] != ',') comma++;
      int ok;
      if (comma < end) {
        size_t l0 = i + 1, l1 = comma, h0 = comma + 1, h1 = end;
        while (l0 < l1 && isspace((unsigned char)s[l0])) l0++;
        while (l1 > l0 && isspace((unsigned char)s[l1 - 1])) l1--;
        while (h0 < h1 && isspace((unsigned char)s[h0])) h0++;
        while (h1 > h0 && isspace((unsigned char)s[h1 - 1])) h1--;
        ok = 1;
        if (l1 > l0) {
          if (mvn_new(s + l0, l1 - l0, &c)) return -1;
          int r = mvn_vcmp(v, &c);
          ok = lo_incl ? r >= 0 : r > 0;
        }
        if (h1 > h0) {
          if (mvn_new(s + h0, h1 - h0, &c2)) return -1;
          int r = mvn_vcmp(v, &c2);
          ok = ok && (hi_incl ? r <= 0 : r < 0);
        }
      } else {
        if (!(lo_incl && hi_incl) || end == i + 1) return -1;
        if (mvn_new(s + i + 1, end - i - 1, &c)) return -1;
        ok = mvn_vcmp(v, &c) == 0;
      }
      hit |= ok;
      i = end + 1;
    }
    return hit;
  }
  int all = 1, any = 0;
  size_t i = b;
  while (i < e) {
    if (s[i] == ',' || s[i] == ' ' || s[i] == '\t') {
      i++;
      continue;
    }
    char op[3] = "=";
    static const char* OPS[] = {">=", "<=", "!=", "==", "=", ">", "<"};
    for (size_t q = 0; q < sizeof OPS / sizeof OPS[0]; q++) {
      size_t l = strlen(OPS[q]);
      if (i + l <= e && !memcmp(s + i, OPS[q], l)) {
        memcpy(op, OPS[q], l);
        op[l] = 0;
        i += l;
        break;
      }
    }
    while (i < e && isspace((unsigned char)s[i])) i++;
    size_t st = i;
    while (i < e && !isspace((unsigned char)s[i]) && !strchr("<>=!,", s[i])) i++;
    if (i == st || mvn_new(s + st, i - st, &c)) return -1;
    any = 1;
    int r = mvn_vcmp(v, &c);
    int m = !strcmp(op, "=") || !strcmp(op, "==") ? r == 0 : !strcmp(op, "!=") ? r != 0 : !strcmp(op, ">") ? r > 0
          : !strcmp(op, "<") ? r < 0 : !strcmp(op, ">=") ? r >= 0 : r <= 0;
    if (!m) all = 0;
  }
  return any ? all : -1;
}

int orc_mvn_match(const char* ver, size_t nv, const char* c, size_t nc) {
  static __thread mver v;
  if (mvn_new(ver, nv, &v)) return -1;
  return any_alt(&v, c, nc, mvn_alt);
}

/* ========================================================== compare.IsVulnerable ====== */
int orc_lib_match(int grammar, const char* ver, size_t nv, const char* c, size_t nc) {
  switch (grammar) {
    case ORC_LIB_GENERIC: return orc_gen_match(ver, nv, c, nc);
    case ORC_LIB_NPM: return orc_npm_match(ver, nv, c, nc);
    case ORC_LIB_PEP440: return orc_pep_match(ver, nv, c, nc);
    case ORC_LIB_MAVEN: return orc_mvn_match(ver, nv, c, nc);
    default: return -1;
  }
}

/* flags: ORC_LIB_HAS_VULN / ORC_LIB_HAS_SECURE / ORC_LIB_ALWAYS (an empty vulnerable or
 * patched constraint); vuln / secure: the lists joined with " || " */
int orc_lib_is_vulnerable(int grammar, const char* ver, size_t nv, uint32_t flags, const char* vuln, size_t nvu,
                          const char* sec, size_t nse) {
  if (flags & ORC_LIB_ALWAYS) return 1;
  int matched = 0;
  if (flags & ORC_LIB_HAS_VULN) {
    int r = orc_lib_match(grammar, ver, nv, vuln, nvu);
    if (r <= 0) return 0;
    matched = 1;
  }
  if (!(flags & ORC_LIB_HAS_SECURE)) return matched;
  int r = orc_lib_match(grammar, ver, nv, sec, nse);
  return r == 0 ? 1 : 0;
}
