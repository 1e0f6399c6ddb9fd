/*
 * ORACLE - TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of github.com/knqyf263/go-deb-version @ v0.0.0-20230223133812-3ed183d23422
 * (reference go.mod:62; the module is not vendored in /root/reference).  Call sites
 * in the reference: pkg/detector/ospkg/debian/debian.go:66,107,113,
 * ubuntu/ubuntu.go:92,116,122, amazon/amazon.go:67,74,80.
 *
 * Published algorithm restated literally (NOT via the product's sort-key encoding):
 *   NewVersion: epoch = Atoi(text before the first ':') (error if not an integer or
 *     negative); the rest is split at the LAST '-' into upstream_version and
 *     debian_revision.  upstream must be non-empty and start with an ASCII digit; every
 *     rune of upstream must be a Unicode digit/letter or one of ".-+~:_"; every rune of
 *     the revision a digit/letter or one of "+.~_".
 *   Compare: epochs as integers, then compare(upstream), then compare(revision), where
 *     compare(v1, v2) extracts the [0-9]+ runs (strconv.Atoi, clamped at MaxInt64 on
 *     overflow) and the [^0-9]+ runs, prepends "" to the string runs when v starts with
 *     a digit, and walks i over the runs: compareString(strings[i]) then
 *     numbers[i] difference (missing entries are "" and 0).  compareString walks bytes
 *     with order(c): Unicode letter (byte taken as a rune) -> c, '~' -> -1,
 *     anything else -> c + 256; a missing byte has order 0.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "unicode_tab.h"

static int in_ranges(const unsigned int (*tab)[2], int n, uint32_t cp) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    if (cp < tab[mid][0]) hi = mid - 1;
    else if (cp > tab[mid][1]) lo = mid + 1;
    else return 1;
  }
  return 0;
}
static const unsigned int tvm_uni_letter[TVM_UNI_NLETTER][2] = {TVM_UNI_LETTER_RANGES};
static const unsigned int tvm_uni_digit[TVM_UNI_NDIGIT][2] = {TVM_UNI_DIGIT_RANGES};
static int is_letter(uint32_t cp) { return in_ranges(tvm_uni_letter, TVM_UNI_NLETTER, cp); }
static int is_digit(uint32_t cp) { return in_ranges(tvm_uni_digit, TVM_UNI_NDIGIT, cp); }

/* Go utf8.DecodeRuneInString: returns rune and width; invalid -> 0xFFFD, width 1. */
static uint32_t decode_rune(const unsigned char* s, size_t n, size_t* w) {
  unsigned c = s[0];
  *w = 1;
  if (c < 0x80) return c;
  unsigned lo = 0x80, hi = 0xBF;
  int need;
  uint32_t cp;
  if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) {
    need = 2; cp = c & 0x0F;
    if (c == 0xE0) lo = 0xA0;
    if (c == 0xED) hi = 0x9F;
  } else if (c >= 0xF0 && c <= 0xF4) {
    need = 3; cp = c & 0x07;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
  } else return 0xFFFD;
  if ((size_t)need >= n) return 0xFFFD;
  for (int i = 1; i <= need; i++) {
    unsigned d = s[i];
    if (i == 1 ? (d < lo || d > hi) : (d < 0x80 || d > 0xBF)) return 0xFFFD;
    cp = (cp << 6) | (d & 0x3F);
  }
  *w = (size_t)need + 1;
  return cp;
}

static int only_allowed(const unsigned char* s, size_t n, const char* sym) {
  size_t i = 0;
  while (i < n) {
    size_t w;
    uint32_t r = decode_rune(s + i, n - i, &w);
    if (!is_digit(r) && !is_letter(r) && !(r < 0x80 && r != 0 && strchr(sym, (int)r))) return 0;
    i += w;
  }
  return 1;
}

/* strconv.Atoi as used for the epoch: [+-]?[0-9]+ within int64, else error. */
static int atoi_strict(const unsigned char* s, size_t n, int64_t* out) {
  size_t i = 0;
  int neg = 0;
  if (n == 0) return -1;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i == n) return -1;
  uint64_t v = 0;
  for (; i < n; i++) {
    if (s[i] < '0' || s[i] > '9') return -1;
    unsigned d = s[i] - '0';
    if (v > (UINT64_MAX - d) / 10) return -1;
    v = v * 10 + d;
    if (v > (uint64_t)INT64_MAX + (uint64_t)neg) return -1;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return 0;
}

int orc_deb_parse(const char* str, size_t n, orc_deb* v) {
  const unsigned char* s = (const unsigned char*)str;
  const unsigned char* colon = memchr(s, ':', n);
  v->epoch = 0;
  if (colon) {
    if (atoi_strict(s, (size_t)(colon - s), &v->epoch)) return -1; /* epoch parse error */
    if (v->epoch < 0) return -1;                                  /* epoch is negative */
    n -= (size_t)(colon - s) + 1;
    s = colon + 1;
  }
  const unsigned char* dash = NULL;
  for (size_t i = n; i-- > 0;)
    if (s[i] == '-') { dash = s + i; break; }
  if (dash) {
    v->up = s; v->nup = (size_t)(dash - s);
    v->rev = dash + 1; v->nrev = n - v->nup - 1;
  } else {
    v->up = s; v->nup = n; v->rev = s + n; v->nrev = 0;
  }
  if (v->nup == 0) return -1;                                     /* upstream_version is empty */
  if (!(v->up[0] >= '0' && v->up[0] <= '9')) return -1;           /* must start with digit */
  if (!only_allowed(v->up, v->nup, ".-+~:_")) return -1;
  if (!only_allowed(v->rev, v->nrev, "+.~_")) return -1;
  return 0;
}

static int order(unsigned char c) {
  if (is_letter(c)) return c; /* rune(byte): Latin-1 code point */
  if (c == '~') return -1;
  return (int)c + 256;
}

typedef struct { const unsigned char* p; size_t n; } run;

/* extract(): digit runs -> numbers (Atoi clamped), non-digit runs -> strings */
static void extract(const unsigned char* s, size_t n, int64_t* nums, size_t* nn, run* strs, size_t* ns) {
  *nn = 0; *ns = 0;
  if (n > 0 && s[0] >= '0' && s[0] <= '9') { strs[0].p = s; strs[0].n = 0; *ns = 1; }
  size_t i = 0;
  while (i < n) {
    size_t j = i;
    if (s[i] >= '0' && s[i] <= '9') {
      uint64_t v = 0;
      int over = 0;
      while (j < n && s[j] >= '0' && s[j] <= '9') {
        unsigned d = s[j] - '0';
        if (!over) {
          if (v > ((uint64_t)INT64_MAX - d) / 10) over = 1;
          else v = v * 10 + d;
        }
        j++;
      }
      nums[(*nn)++] = over ? INT64_MAX : (int64_t)v;
    } else {
      while (j < n && !(s[j] >= '0' && s[j] <= '9')) j++;
      strs[*ns].p = s + i; strs[*ns].n = j - i; (*ns)++;
    }
    i = j;
  }
}

static int cmp_string(run a, run b) {
  if (a.n == b.n && memcmp(a.p, b.p, a.n) == 0) return 0;
  size_t m = a.n > b.n ? a.n : b.n;
  for (size_t i = 0; i < m; i++) {
    int x = i < a.n ? order(a.p[i]) : 0;
    int y = i < b.n ? order(b.p[i]) : 0;
    if (x != y) return x - y;
  }
  return 0;
}

static int compare_part(const unsigned char* a, size_t na, const unsigned char* b, size_t nb) {
  if (na == nb && memcmp(a, b, na) == 0) return 0;
  size_t cap_a = na + 2, cap_b = nb + 2;
  int64_t* n1 = malloc(sizeof(int64_t) * cap_a);
  int64_t* n2 = malloc(sizeof(int64_t) * cap_b);
  run* s1 = malloc(sizeof(run) * cap_a);
  run* s2 = malloc(sizeof(run) * cap_b);
  size_t nn1, ns1, nn2, ns2;
  extract(a, na, n1, &nn1, s1, &ns1);
  extract(b, nb, n2, &nn2, s2, &ns2);
  size_t m = ns1 > ns2 ? ns1 : ns2;
  int ret = 0;
  for (size_t i = 0; i < m && ret == 0; i++) {
    run e = {a, 0};
    int d = cmp_string(i < ns1 ? s1[i] : e, i < ns2 ? s2[i] : e);
    if (d) { ret = d; break; }
    int64_t x = i < nn1 ? n1[i] : 0, y = i < nn2 ? n2[i] : 0;
    if (x != y) ret = x > y ? 1 : -1;
  }
  free(n1); free(n2); free(s1); free(s2);
  return ret;
}

int orc_deb_cmp(const orc_deb* a, const orc_deb* b) {
  if (a->epoch != b->epoch) return a->epoch > b->epoch ? 1 : -1;
  int r = compare_part(a->up, a->nup, b->up, b->nup);
  if (r) return r;
  return compare_part(a->rev, a->nrev, b->rev, b->nrev);
}

int orc_deb_cmp_str(const char* a, size_t na, const char* b, size_t nb) {
  orc_deb x, y;
  if (orc_deb_parse(a, na, &x)) return 2;
  if (orc_deb_parse(b, nb, &y)) return 3;
  int r = orc_deb_cmp(&x, &y);
  return (r > 0) - (r < 0);
}
