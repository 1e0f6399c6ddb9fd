/*
 * ORACLE - TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * go-apk-version v0.0.0-20200609155635-041fdbb8563f (reference go.mod:61), the Go port of
 * apk-tools' version.c.  Call sites: pkg/detector/ospkg/alpine/alpine.go:93,126,141,
 * wolfi/wolfi.go:48,68, chainguard/chainguard.go:48,68.
 *
 * A version is read as a stream of tokens; each token's kind is decided before it is
 * read (the kind of the first token is DIGIT) and the reader moves to the next kind
 * from the characters that follow:
 *   digit run / leading zeros of a dot-component / one lower-case letter /
 *   "_" suffix name (alpha < beta < pre < rc < cvs < svn < git < hg < p) / suffix number /
 *   "-r" revision number / end.
 * Two versions compare token by token while both next kinds agree and the values are
 * equal; then the values decide, and when the kinds differ a pre-release suffix loses,
 * otherwise the greater kind (later in the list above) is the smaller version.
 * After a suffix name the next kind comes from the following character (a digit makes
 * it a suffix number, "_" another suffix): alpine_test.go "contain pre" pins
 * 0.1.0_alpha >= 0.1.0_alpha_pre2, which holds only with this reading.
 * Pinned by alpine_test.go / wolfi_test.go / chainguard_test.go (1.6_rc1-r0 < 1.6-r0 <
 * 1.6-r1, 0.1.0_alpha < 0.1.0_alpha2, 0.1.0_alpha >= 0.1.0_alpha_pre2, "invalid" fails).
 */
#include <string.h>

#include "oracle.h"

enum { T_INVALID = -1, T_DIGIT_OR_ZERO = 0, T_DIGIT, T_LETTER, T_SUFFIX, T_SUFFIX_NO, T_REVISION_NO, T_END };

typedef struct {
  const unsigned char* p;
  size_t n;
} blob;

static int is_lower(int c) { return c >= 'a' && c <= 'z'; }
static int is_dig(int c) { return c >= '0' && c <= '9'; }

static void next_kind(int* kind, blob* b) {
  int n = T_INVALID;
  if (b->n == 0 || b->p[0] == 0) {
    n = T_END;
  } else if ((*kind == T_DIGIT || *kind == T_DIGIT_OR_ZERO) && is_lower(b->p[0])) {
    n = T_LETTER;
  } else if (*kind == T_LETTER && is_dig(b->p[0])) {
    n = T_DIGIT;
  } else if (*kind == T_SUFFIX && is_dig(b->p[0])) {
    n = T_SUFFIX_NO;
  } else {
    switch (b->p[0]) {
      case '.': n = T_DIGIT_OR_ZERO; break;
      case '_': n = T_SUFFIX; break;
      case '-':
        if (b->n > 1 && b->p[1] == 'r') {
          n = T_REVISION_NO;
          b->p++;
          b->n--;
        } else {
          n = T_INVALID;
        }
        break;
    }
    b->p++;
    b->n--;
  }
  if (n < *kind) {
    if (!((n == T_DIGIT_OR_ZERO && *kind == T_DIGIT) || (n == T_SUFFIX && *kind == T_SUFFIX_NO) ||
          (n == T_DIGIT && *kind == T_LETTER)))
      n = T_INVALID;
  }
  *kind = n;
}

static const char* const k_pre[] = {"alpha", "beta", "pre", "rc"};
static const char* const k_post[] = {"cvs", "svn", "git", "hg", "p"};

static int starts(const blob* b, const char* s) {
  size_t l = strlen(s);
  return l <= b->n && memcmp(b->p, s, l) == 0;
}

/* Reads the token of kind *kind; leaves the next token's kind in *kind. */
static long long get_token(int* kind, blob* b) {
  long long v = 0;
  size_t i = 0;
  int nt = T_INVALID;
  if (b->n == 0) {
    *kind = T_END;
    return 0;
  }
  switch (*kind) {
    case T_DIGIT_OR_ZERO:
      if (b->p[0] == '0') { /* leading zeros of a dot-component */
        while (i < b->n && b->p[i] == '0') i++;
        nt = T_DIGIT;
        v = -(long long)i;
        break;
      }
      /* fallthrough */
    case T_DIGIT:
    case T_SUFFIX_NO:
    case T_REVISION_NO:
      while (i < b->n && is_dig(b->p[i])) v = v * 10 + (b->p[i++] - '0');
      break;
    case T_LETTER:
      v = b->p[i++];
      break;
    case T_SUFFIX: {
      int k;
      for (k = 0; k < 4; k++)
        if (starts(b, k_pre[k])) break;
      if (k < 4) {
        i = strlen(k_pre[k]);
        v = k - 4;
        break;
      }
      for (k = 0; k < 5; k++)
        if (starts(b, k_post[k])) break;
      if (k < 5) {
        i = strlen(k_post[k]);
        v = k;
        break;
      }
    }
      /* fallthrough */
    default:
      *kind = T_INVALID;
      return -1;
  }
  b->p += i;
  b->n -= i;
  if (b->n == 0)
    *kind = T_END;
  else if (nt != T_INVALID)
    *kind = nt;
  else
    next_kind(kind, b);
  return v;
}

int orc_apk_valid(const char* s, size_t n) {
  blob b = {(const unsigned char*)s, n};
  int k = T_DIGIT; /* "" reads as one END token: valid, as in apk-tools (unpinned) */
  while (k != T_END && k != T_INVALID) get_token(&k, &b);
  return k == T_END;
}

int orc_apk_cmp(const char* sa, size_t na, const char* sb, size_t nb) {
  blob a = {(const unsigned char*)sa, na}, b = {(const unsigned char*)sb, nb};
  int at = T_DIGIT, bt = T_DIGIT, tt;
  long long av = 0, bv = 0;
  while (at == bt && at != T_END && at != T_INVALID && av == bv) {
    av = get_token(&at, &a);
    bv = get_token(&bt, &b);
  }
  if (av < bv) return -1;
  if (av > bv) return 1;
  if (at == bt) return 0;
  tt = at;
  if (at == T_SUFFIX && get_token(&tt, &a) < 0) return -1;
  tt = bt;
  if (bt == T_SUFFIX && get_token(&tt, &b) < 0) return 1;
  if (at > bt) return -1;
  if (bt > at) return 1;
  return 0;
}

int orc_apk_cmp_str(const char* a, size_t na, const char* b, size_t nb) {
  if (!orc_apk_valid(a, na)) return 2;
  if (!orc_apk_valid(b, nb)) return 3;
  return orc_apk_cmp(a, na, b, nb);
}
