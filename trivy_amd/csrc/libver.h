// Sort-key encoders of the library (language-package) version grammars (host + device).
//
// Same contract as verkey.h: each grammar maps a version string to a byte string whose
// plain lexicographic order (common.h key_cmp) is the grammar's version order, plus a
// small "class" (npm: pre-release; PEP 440: local / pre-release / post-release) that the
// constraint compiler needs where a grammar's constraint semantics are not interval-shaped
// over the order alone (node-semver's pre-release rule, PEP 440's exclusive comparisons).
// Reference call sites: pkg/detector/library/compare/compare.go:58-78 and
// compare/{npm,pep440,maven,rubygems,bitnami}/compare.go:20-32.  The six third-party
// modules (reference go.mod:16-19,37,73) are absent; their published algorithms are
// restated (oracle/library.py is the independent pairwise restatement the keys are fuzzed
// against).  Parsing mirrors each module's regular expression.
#pragma once
#include "verkey.h"

namespace tvm {

// ---------------------------------------------------------------------------- helpers ---
TVM_HD bool lv_alpha(uint8_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
TVM_HD bool lv_alnum(uint8_t c) { return lv_alpha(c) || is_adigit(c); }
TVM_HD uint8_t lv_lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? uint8_t(c + 32) : c; }
TVM_HD bool lv_space(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

// Decimal digits [b, e) as a uint64; false on overflow.
TVM_HD bool lv_u64(const uint8_t* s, uint32_t b, uint32_t e, uint64_t& v) {
  v = 0;
  for (uint32_t i = b; i < e; i++) {
    const uint64_t d = uint64_t(s[i] - '0');
    if (v > (~0ULL - d) / 10) return false;
    v = v * 10 + d;
  }
  return true;
}

// Unsigned 64-bit values: 0x80+k then k big-endian bytes (put_sint's code for v >= 0).
template <class Sink>
TVM_HD void put_uvar(uint64_t u, Sink& o) {
  uint32_t k = 0;
  for (uint64_t t = u; t; t >>= 8) k++;
  o.put(uint8_t(0x80 + k));
  for (int b = int(k) - 1; b >= 0; b--) o.put(uint8_t(u >> (8 * b)));
}

// Arbitrary-precision decimal: leading zeros dropped, digit count, digits two per byte.
template <class Sink>
TVM_HD void put_digits(const uint8_t* s, uint32_t b, uint32_t e, Sink& o) {
  while (b < e && s[b] == '0') b++;
  const uint32_t len = e - b;
  if (len < 0xFA) {
    o.put(uint8_t(len));
  } else {
    o.put(0xFA);
    o.put(uint8_t(len >> 8));
    o.put(uint8_t(len));
  }
  for (uint32_t j = b; j < e; j += 2) {
    const uint8_t hi = uint8_t(s[j] - '0'), lo = j + 1 < e ? uint8_t(s[j + 1] - '0') : 0;
    o.put(uint8_t((hi << 4) | lo));
  }
}

// semver-style identifier list "a.b.c" over [b, e) with identifier bytes allowed by `ok`.
template <class F>
TVM_HD bool lv_idents(const uint8_t* s, uint32_t b, uint32_t e, F ok) {
  if (b >= e) return false;
  uint32_t run = 0;
  for (uint32_t i = b; i < e; i++) {
    if (s[i] == '.') {
      if (!run) return false;
      run = 0;
    } else if (ok(s[i])) {
      run++;
    } else {
      return false;
    }
  }
  return run > 0;
}

// Pre-release identifiers: numeric (all digits) = 0x01 + digits, else 0x02 + bytes + 0x00;
// list end 0x00 (a shorter list sorts first; numeric < alphanumeric).
template <class Sink>
TVM_HD void put_idents(const uint8_t* s, uint32_t b, uint32_t e, Sink& o) {
  uint32_t i = b;
  while (i < e) {
    uint32_t j = i;
    bool num = true;
    while (j < e && s[j] != '.') num &= is_adigit(s[j++]);
    if (num) {
      o.put(0x01);
      put_digits(s, i, j, o);
    } else {
      o.put(0x02);
      for (uint32_t k = i; k < j; k++) o.put(s[k]);
      o.put(0x00);
    }
    i = j + 1;
  }
  o.put(0x00);
}

TVM_HD bool gen_ident_char(uint8_t c) { return lv_alnum(c) || c == '-' || c == '~'; }
TVM_HD bool npm_ident_char(uint8_t c) { return lv_alnum(c) || c == '-'; }

// =========================================================================== GENERIC ====
// github.com/aquasecurity/go-version (go.mod:19), hashicorp-style:
//   v?N(.N)*  ( -IDENTS | [A-Za-z-~]IDENTS )?  (+IDENTS)?      IDENT = [0-9A-Za-z-~]+
// Order: zero-padded numeric segments, then pre-release (none > some; semver identifier
// precedence); build metadata ignored.  Bitnami (github.com/bitnami/go-version, go.mod:37)
// reads an all-digit "-N" as a package revision compared after everything else.
// Key: segments (trailing zeros dropped) as put_sint, 0x01, then 0x03 (release) or
// 0x02 + identifiers, then (bitnami) the revision digits.
struct GenParts {
  uint32_t rel_b, rel_e;   // release span (after the optional 'v')
  uint32_t pre_b, pre_e;   // pre-release identifiers (empty: none)
  uint32_t rev_b, rev_e;   // bitnami revision digits (empty: 0)
  uint32_t n_segs_key;     // segments up to the last non-zero one
};

TVM_HD bool gen_parse(const uint8_t* s, uint32_t n, bool bitnami, GenParts& g) {
  uint32_t i = 0;
  if (i < n && s[i] == 'v') i++;
  g.rel_b = i;
  uint32_t segs = 0, last_nz = 0;
  for (;;) {
    const uint32_t b = i;
    while (i < n && is_adigit(s[i])) i++;
    if (i == b) return false;
    uint64_t v;
    if (!lv_u64(s, b, i, v)) return false;  // part.NewUint64 overflow
    segs++;
    if (v) last_nz = segs;
    if (i + 1 < n && s[i] == '.' && is_adigit(s[i + 1])) {
      i++;
      continue;
    }
    break;
  }
  g.rel_e = i;
  g.n_segs_key = last_nz;
  uint32_t plus = n;
  for (uint32_t k = i; k < n; k++)
    if (s[k] == '+') { plus = k; break; }
  if (plus < n && !lv_idents(s, plus + 1, n, gen_ident_char)) return false;
  g.pre_b = g.pre_e = i;
  g.rev_b = g.rev_e = 0;
  if (i < plus) {
    if (s[i] == '-' && lv_idents(s, i + 1, plus, gen_ident_char)) {
      g.pre_b = i + 1;
      g.pre_e = plus;
      bool digits = true;
      for (uint32_t k = i + 1; k < plus; k++) digits &= is_adigit(s[k]);
      if (bitnami && digits) {
        g.rev_b = i + 1;
        g.rev_e = plus;
        g.pre_b = g.pre_e = i;
      }
    } else if ((lv_alpha(s[i]) || s[i] == '-' || s[i] == '~') && lv_idents(s, i, plus, gen_ident_char)) {
      g.pre_b = i;
      g.pre_e = plus;
    } else {
      return false;
    }
  }
  return true;
}

template <class Sink>
TVM_HD void gen_emit_release(const uint8_t* s, const GenParts& g, Sink& o) {
  uint32_t i = g.rel_b;
  for (uint32_t k = 0; k < g.n_segs_key; k++) {
    const uint32_t b = i;
    while (i < g.rel_e && is_adigit(s[i])) i++;  // bounded: the bytes after a version are arbitrary
    uint64_t v;
    lv_u64(s, b, i, v);
    put_uvar(v, o);
    i++;
  }
}

template <class Sink>
TVM_HD void gen_emit(const uint8_t* s, const GenParts& g, bool bitnami, Sink& o) {
  gen_emit_release(s, g, o);
  o.put(0x01);
  if (g.pre_e > g.pre_b) {
    o.put(0x02);
    put_idents(s, g.pre_b, g.pre_e, o);
  } else {
    o.put(0x03);
  }
  if (bitnami) put_digits(s, g.rev_b, g.rev_e, o);
}

template <class Sink>
TVM_HD bool gen_encode(const uint8_t* s, uint32_t n, bool bitnami, Sink& o) {
  GenParts g;
  if (!gen_parse(s, n, bitnami, g)) return false;
  gen_emit(s, g, bitnami, o);
  return true;
}

// =============================================================================== NPM ====
// github.com/aquasecurity/go-npm-version (go.mod:17), node-semver:
//   \s*[v=]*\s*N.N.N (-?IDENTS)? (+IDENTS)? \s*          IDENT = [0-9A-Za-z-]+
// Key: put_sint(major) put_sint(minor) put_sint(patch), then 0x03 (release) or 0x02 +
// identifiers.  Class 1 = has a pre-release (node-semver's pre-release gating).
struct NpmParts {
  uint32_t num_b[3], num_e[3];
  uint32_t pre_b, pre_e;
};

TVM_HD bool npm_parse(const uint8_t* s, uint32_t n, NpmParts& p) {
  uint32_t i = 0;
  while (i < n && lv_space(s[i])) i++;
  while (i < n && (s[i] == 'v' || s[i] == '=')) i++;
  while (i < n && lv_space(s[i])) i++;
  for (int k = 0; k < 3; k++) {
    if (k) {
      if (i >= n || s[i] != '.') return false;
      i++;
    }
    p.num_b[k] = i;
    while (i < n && is_adigit(s[i])) i++;
    p.num_e[k] = i;
    uint64_t v;
    if (p.num_e[k] == p.num_b[k] || !lv_u64(s, p.num_b[k], i, v)) return false;
  }
  uint32_t end = n;
  while (end > i && lv_space(s[end - 1])) end--;
  uint32_t plus = end;
  for (uint32_t k = i; k < end; k++)
    if (s[k] == '+') { plus = k; break; }
  if (plus < end && !lv_idents(s, plus + 1, end, npm_ident_char)) return false;
  p.pre_b = p.pre_e = i;
  if (i < plus) {
    if (s[i] == '-' && lv_idents(s, i + 1, plus, npm_ident_char)) {
      p.pre_b = i + 1;
    } else if (lv_idents(s, i, plus, npm_ident_char)) {
      p.pre_b = i;
    } else {
      return false;
    }
    p.pre_e = plus;
  }
  return true;
}

template <class Sink>
TVM_HD void npm_emit(const uint8_t* s, const NpmParts& p, Sink& o) {
  for (int k = 0; k < 3; k++) {
    uint64_t v;
    lv_u64(s, p.num_b[k], p.num_e[k], v);
    put_uvar(v, o);
  }
  if (p.pre_e > p.pre_b) {
    o.put(0x02);
    put_idents(s, p.pre_b, p.pre_e, o);
  } else {
    o.put(0x03);
  }
}

template <class Sink>
TVM_HD bool npm_encode(const uint8_t* s, uint32_t n, Sink& o, uint32_t& cls) {
  NpmParts p;
  if (!npm_parse(s, n, p)) return false;
  npm_emit(s, p, o);
  cls = p.pre_e > p.pre_b ? 1u : 0u;
  return true;
}

// ============================================================================ PEP 440 ====
// github.com/aquasecurity/go-pep440-version (go.mod:18), the PEP 440 / packaging
// VERSION_PATTERN (case-insensitive):
//   v? (N!)? N(.N)* ([-_.]?(alpha|a|beta|b|preview|pre|c|rc)[-_.]?N?)?
//   (-N | [-_.]?(post|rev|r)[-_.]?N?)? ([-_.]?dev[-_.]?N?)? (+L([-_.]L)*)?     L = [a-z0-9]+
// Key (packaging's _cmpkey): put_sint(epoch), release without trailing zeros, 0x01, then
// PRE (0x01 dev-only / 0x02 letter n / 0x03 none), POST (0x01 none / 0x02 n), DEV
// (0x01 n / 0x02 none), LOCAL (0x01 none / 0x02 segments 0x00; numeric segments above
// alphanumeric ones).  Class bits: 1 local, 2 pre-release (pre or dev), 4 post-release.
struct PepParts {
  uint64_t epoch;
  uint32_t rel_b, rel_e, rel_key_segs;
  int pre_l;                 // -1 none, 0 a, 1 b, 2 rc
  uint64_t pre_n, post_n, dev_n;
  bool post, dev;
  uint32_t loc_b, loc_e;     // local span (empty: none)
};

TVM_HD bool pep_sep(uint8_t c) { return c == '-' || c == '_' || c == '.'; }

// Case-insensitive keyword at i; returns its length or 0.
TVM_HD uint32_t pep_kw(const uint8_t* s, uint32_t n, uint32_t i, const char* w) {
  uint32_t k = 0;
  while (w[k]) {
    if (i + k >= n || lv_lower(s[i + k]) != uint8_t(w[k])) return 0;
    k++;
  }
  return k;
}

TVM_HD bool pep_num(const uint8_t* s, uint32_t n, uint32_t& i, uint64_t& v) {
  const uint32_t b = i;
  while (i < n && is_adigit(s[i])) i++;
  return lv_u64(s, b, i, v);
}

TVM_HD bool pep_parse(const uint8_t* s, uint32_t n, PepParts& p) {
  uint32_t i = 0;
  while (i < n && lv_space(s[i])) i++;
  while (n > i && lv_space(s[n - 1])) n--;
  if (i < n && (s[i] == 'v' || s[i] == 'V')) i++;
  p.epoch = 0;
  {  // (N!)?
    uint32_t j = i;
    while (j < n && is_adigit(s[j])) j++;
    if (j > i && j < n && s[j] == '!') {
      if (!lv_u64(s, i, j, p.epoch)) return false;
      i = j + 1;
    }
  }
  p.rel_b = i;
  uint32_t segs = 0, last_nz = 0;
  for (;;) {
    const uint32_t b = i;
    uint64_t v;
    if (!pep_num(s, n, i, v) || i == b) return false;
    segs++;
    if (v) last_nz = segs;
    if (i + 1 < n && s[i] == '.' && is_adigit(s[i + 1])) {
      i++;
      continue;
    }
    break;
  }
  p.rel_e = i;
  p.rel_key_segs = last_nz;
  // pre
  p.pre_l = -1;
  p.pre_n = 0;
  {
    uint32_t j = i;
    if (j < n && pep_sep(s[j])) j++;
    static constexpr const char* kPre[] = {"alpha", "a", "beta", "b", "preview", "pre", "c", "rc"};
    static constexpr int kPreL[] = {0, 0, 1, 1, 2, 2, 2, 2};
    for (int k = 0; k < 8; k++) {
      const uint32_t l = pep_kw(s, n, j, kPre[k]);
      if (!l) continue;
      p.pre_l = kPreL[k];
      j += l;
      if (j < n && pep_sep(s[j]) && !(j + 1 < n && is_adigit(s[j + 1])) && !(j + 1 < n && lv_alpha(s[j + 1]))) {
        j++;  // trailing optional separator, no number ([-_.]? with N? empty)
      } else if (j < n && pep_sep(s[j]) && j + 1 < n && is_adigit(s[j + 1])) {
        j++;
      }
      if (!pep_num(s, n, j, p.pre_n)) return false;
      i = j;
      break;
    }
  }
  // post: -N | [-_.]?(post|rev|r)[-_.]?N?
  p.post = false;
  p.post_n = 0;
  if (i + 1 < n && s[i] == '-' && is_adigit(s[i + 1])) {
    i++;
    if (!pep_num(s, n, i, p.post_n)) return false;
    p.post = true;
  } else {
    uint32_t j = i;
    if (j < n && pep_sep(s[j])) j++;
    uint32_t l = pep_kw(s, n, j, "post");
    if (!l) l = pep_kw(s, n, j, "rev");
    if (!l) l = pep_kw(s, n, j, "r");
    if (l) {
      j += l;
      if (j < n && pep_sep(s[j]) && !(j + 1 < n && lv_alpha(s[j + 1]))) j++;
      if (!pep_num(s, n, j, p.post_n)) return false;
      p.post = true;
      i = j;
    }
  }
  // dev
  p.dev = false;
  p.dev_n = 0;
  {
    uint32_t j = i;
    if (j < n && pep_sep(s[j])) j++;
    const uint32_t l = pep_kw(s, n, j, "dev");
    if (l) {
      j += l;
      if (j < n && pep_sep(s[j])) j++;
      if (!pep_num(s, n, j, p.dev_n)) return false;
      p.dev = true;
      i = j;
    }
  }
  // local
  p.loc_b = p.loc_e = i;
  if (i < n && s[i] == '+') {
    uint32_t j = i + 1, run = 0;
    for (; j < n; j++) {
      if (lv_alnum(s[j])) run++;
      else if (pep_sep(s[j]) && run) run = 0;
      else return false;
    }
    if (!run) return false;
    p.loc_b = i + 1;
    p.loc_e = n;
    i = n;
  }
  return i == n;
}

enum : uint32_t { PEP_CLS_LOCAL = 1, PEP_CLS_PRE = 2, PEP_CLS_POST = 4 };

TVM_HD uint32_t pep_class(const PepParts& p) {
  return (p.loc_e > p.loc_b ? PEP_CLS_LOCAL : 0) | ((p.pre_l >= 0 || p.dev) ? PEP_CLS_PRE : 0) |
         (p.post ? PEP_CLS_POST : 0);
}

// Emission stops after `upto`: 0 epoch+release+0x01 (the "base" prefix), 1 through DEV
// (the public version), 2 everything.
template <class Sink>
TVM_HD void pep_emit(const uint8_t* s, const PepParts& p, int upto, Sink& o) {
  put_uvar(p.epoch, o);
  uint32_t i = p.rel_b;
  for (uint32_t k = 0; k < p.rel_key_segs; k++) {
    uint64_t v;
    pep_num(s, p.rel_e, i, v);
    put_uvar(v, o);
    i++;
  }
  o.put(0x01);
  if (upto == 0) return;
  if (p.pre_l < 0 && !p.post && p.dev) {
    o.put(0x01);
  } else if (p.pre_l >= 0) {
    o.put(0x02);
    o.put(uint8_t(p.pre_l));
    put_uvar(p.pre_n, o);
  } else {
    o.put(0x03);
  }
  if (p.post) {
    o.put(0x02);
    put_uvar(p.post_n, o);
  } else {
    o.put(0x01);
  }
  if (p.dev) {
    o.put(0x01);
    put_uvar(p.dev_n, o);
  } else {
    o.put(0x02);
  }
  if (upto == 1) return;
  if (p.loc_e > p.loc_b) {
    o.put(0x02);
    uint32_t j = p.loc_b;
    while (j < p.loc_e) {
      uint32_t e = j;
      bool num = true;
      while (e < p.loc_e && !pep_sep(s[e])) num &= is_adigit(s[e++]);
      if (num) {
        o.put(0x02);
        put_digits(s, j, e, o);
      } else {
        o.put(0x01);
        for (uint32_t k = j; k < e; k++) o.put(lv_lower(s[k]));
        o.put(0x00);
      }
      j = e + 1;
    }
    o.put(0x00);
  } else {
    o.put(0x01);
  }
}

template <class Sink>
TVM_HD bool pep_encode(const uint8_t* s, uint32_t n, Sink& o, uint32_t& cls) {
  PepParts p;
  if (!pep_parse(s, n, p)) return false;
  pep_emit(s, p, 2, o);
  cls = pep_class(p);
  return true;
}

// ============================================================================== MAVEN ====
// github.com/masahiro331/go-mvn-version (go.mod:73), Maven's ComparableVersion: lower-cased;
// '.' separates items, '-' and digit<->letter transitions open a sub-list (always the last
// item of its parent); one-letter a/b/m before a digit read alpha/beta/milestone; ga,
// final, release -> "" and cr -> rc; each list drops trailing nulls (0, "", empty lists),
// looking through non-null sub-lists; lists compare item by item padded with null.
// Key per item (ComparableVersion is a total order for everything but exotic mixes of
// "0"/"" items with qualifiers at one position):
//   0x10+q  alpha/beta/milestone/rc/snapshot      0x20  sub-list below null (first item < null)
//   0x28    0 followed by something below null    0x30  end of list, and the "" qualifier
//   0x40    sp                                     0x50  other qualifier: bytes, 0x00
//   0x60    sub-list above null                    0x68  0 followed by something above null
//   0x70    integer > 0 (digits)
// Versions must match ^[0-9A-Za-z][0-9A-Za-z._+-]*$ (go-mvn-version rejects other bytes).
enum : uint8_t { MV_INT = 1, MV_STR = 2, MV_OPEN = 3 };
struct MvnTok {
  uint8_t kind;
  uint8_t q;          // MV_STR: 0..4 pre, 5 "", 6 sp, 7 other
  uint8_t removed;
  uint8_t zero;       // MV_INT: value is 0
  uint32_t b, e;      // source span (MV_INT digits, MV_STR raw letters)
};
constexpr int kMvnMaxTok = 48;

TVM_HD int mvn_qual(const uint8_t* s, uint32_t b, uint32_t e, bool followed_by_digit) {
  auto eq = [&](const char* w) {
    uint32_t k = 0;
    for (; w[k]; k++)
      if (b + k >= e || lv_lower(s[b + k]) != uint8_t(w[k])) return false;
    return b + k == e;
  };
  if (followed_by_digit && e - b == 1) {
    const uint8_t c = lv_lower(s[b]);
    if (c == 'a') return 0;
    if (c == 'b') return 1;
    if (c == 'm') return 2;
  }
  if (eq("alpha")) return 0;
  if (eq("beta")) return 1;
  if (eq("milestone")) return 2;
  if (eq("rc") || eq("cr")) return 3;
  if (eq("snapshot")) return 4;
  if (e == b || eq("ga") || eq("final") || eq("release")) return 5;
  if (eq("sp")) return 6;
  return 7;
}

struct MvnParse {
  MvnTok t[kMvnMaxTok];
  int n = 0;
};

TVM_HD bool mvn_push(MvnParse& P, uint8_t kind, uint32_t b, uint32_t e, const uint8_t* s, bool fbd) {
  if (P.n >= kMvnMaxTok) return false;
  MvnTok& k = P.t[P.n++];
  k.kind = kind;
  k.b = b;
  k.e = e;
  k.removed = 0;
  k.zero = 0;
  k.q = 0;
  if (kind == MV_INT) {
    uint32_t i = b;
    while (i < e && s[i] == '0') i++;
    k.zero = i == e;
  } else if (kind == MV_STR) {
    k.q = uint8_t(mvn_qual(s, b, e, fbd));
  }
  return true;
}

TVM_HD bool mvn_null(const MvnTok& k) {
  return (k.kind == MV_INT && k.zero) || (k.kind == MV_STR && k.q == 5);
}

TVM_HD bool mvn_parse(const uint8_t* s, uint32_t n, MvnParse& P) {
  uint32_t b0 = 0;
  while (b0 < n && lv_space(s[b0])) b0++;
  while (n > b0 && lv_space(s[n - 1])) n--;
  if (b0 >= n || !lv_alnum(s[b0])) return false;
  for (uint32_t i = b0; i < n; i++)
    if (!(lv_alnum(s[i]) || s[i] == '.' || s[i] == '-' || s[i] == '_' || s[i] == '+')) return false;
  P.n = 0;
  bool digit = false;
  uint32_t start = b0;
  for (uint32_t i = b0; i < n; i++) {
    const uint8_t c = s[i];
    if (c == '.' || c == '-') {
      if (i == start) {
        if (!mvn_push(P, MV_INT, i, i, s, false)) return false;
      } else if (!mvn_push(P, digit ? MV_INT : MV_STR, start, i, s, false)) {
        return false;
      }
      start = i + 1;
      if (c == '-' && !mvn_push(P, MV_OPEN, i, i, s, false)) return false;
    } else if (is_adigit(c)) {
      if (!digit && i > start) {
        if (!mvn_push(P, MV_STR, start, i, s, true) || !mvn_push(P, MV_OPEN, i, i, s, false)) return false;
        start = i;
      }
      digit = true;
    } else {
      if (digit && i > start) {
        if (!mvn_push(P, MV_INT, start, i, s, false) || !mvn_push(P, MV_OPEN, i, i, s, false)) return false;
        start = i;
      }
      digit = false;
    }
  }
  if (n > start && !mvn_push(P, digit ? MV_INT : MV_STR, start, n, s, false)) return false;
  // normalize, innermost list first: list l is the spine [starts[l], starts[l+1]) whose
  // last token (the OPEN of list l+1) is its sub-list item
  int list_end = P.n;
  // find list starts
  int starts[kMvnMaxTok + 1];
  int ns = 0;
  starts[ns++] = 0;
  for (int k = 0; k < P.n; k++)
    if (P.t[k].kind == MV_OPEN) starts[ns++] = k + 1;
  bool inner_null = true;  // the list after the current one is empty (null)
  for (int l = ns - 1; l >= 0; l--) {
    const int b = starts[l];
    const int e = list_end;  // items of list l: [b, e) minus the OPEN at e-1 if any
    bool stop = false;
    for (int k = e - 1; k >= b && !stop; k--) {
      MvnTok& t = P.t[k];
      if (t.removed) continue;
      if (t.kind == MV_OPEN) {
        if (inner_null) t.removed = 1;  // empty sub-list: null -> removed, keep looking
        continue;                       // non-null sub-list: look through it
      }
      if (mvn_null(t)) t.removed = 1;
      else stop = true;
    }
    inner_null = true;
    for (int k = b; k < e; k++)
      if (!P.t[k].removed) inner_null = false;
    list_end = b;  // the parent's range ends with this list's OPEN token
  }
  return true;
}

// Relation of the item starting at token k (skipping removed ones) to null:
// -1 below, 0 equal, +1 above.  For a sub-list: its first item's relation.
TVM_HD int mvn_rel(const MvnParse& P, int k) {
  for (; k < P.n; k++) {
    const MvnTok& t = P.t[k];
    if (t.removed) continue;
    if (t.kind == MV_OPEN) continue;  // first item of the sub-list decides
    if (t.kind == MV_INT) return t.zero ? 0 : 1;
    return t.q < 5 ? -1 : (t.q == 5 ? 0 : 1);
  }
  return 0;
}

template <class Sink>
TVM_HD void mvn_emit(const uint8_t* s, const MvnParse& P, Sink& o) {
  int depth = 0;
  for (int k = 0; k < P.n; k++) {
    const MvnTok& t = P.t[k];
    if (t.removed) continue;
    if (t.kind == MV_OPEN) {
      o.put(mvn_rel(P, k + 1) < 0 ? 0x20 : 0x60);
      depth++;
      continue;
    }
    if (t.kind == MV_INT) {
      if (!t.zero) {
        o.put(0x70);
        put_digits(s, t.b, t.e, o);
      } else {
        // lookahead: the next item of this list that is not a zero (a sub-list counts)
        int r = 0;
        for (int j = k + 1; j < P.n; j++) {
          const MvnTok& u = P.t[j];
          if (u.removed) continue;
          if (u.kind == MV_INT && u.zero) continue;
          r = u.kind == MV_OPEN ? mvn_rel(P, j + 1) : mvn_rel(P, j);
          break;
        }
        o.put(r < 0 ? 0x28 : 0x68);
      }
      continue;
    }
    if (t.q < 5) o.put(uint8_t(0x10 + t.q));
    else if (t.q == 5) o.put(0x30);
    else if (t.q == 6) o.put(0x40);
    else {
      o.put(0x50);
      for (uint32_t i = t.b; i < t.e; i++) o.put(lv_lower(s[i]));
      o.put(0x00);
    }
  }
  for (int d = 0; d <= depth; d++) o.put(0x30);
}

// Maven version class 1 ("numeric"): digit runs of 1..9 digits joined by single dots
// ("1.2.3").  ComparableVersion parses such a text into a flat list of int items, and two
// such lists compare as their zero-padded integer sequences - a total order, which the sort
// key reproduces exactly.  Every other text is class 0 and is compared through the
// pairwise program: the hybrid of db.cpp DB::compile_rows.
TVM_HD bool mvn_numeric(const uint8_t* s, uint32_t n) {
  if (n == 0) return false;
  uint32_t run = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    if (c >= '0' && c <= '9') {
      if (++run > 9) return false;
    } else if (c == '.') {
      if (run == 0) return false;
      run = 0;
    } else {
      return false;
    }
  }
  return run > 0;
}

template <class Sink>
TVM_HD bool mvn_encode(const uint8_t* s, uint32_t n, Sink& o) {
  MvnParse P;
  if (!mvn_parse(s, n, P)) return false;
  mvn_emit(s, P, o);
  return true;
}

// ---- Maven, pairwise: ComparableVersion.compareTo on two parses ----------------------------
// The sort key above is a total order; ComparableVersion is not, so the
// library rows of the Maven grammar are evaluated pairwise instead: each advisory becomes a
// small program (the OR of AND clauses IsVulnerable evaluates, compare.go:20-51) whose terms
// compare the installed version with the bound through mvn_cmp below - Item.compareTo of
// go-mvn-version exactly, int / string / list against each other and against null.
// A parse is a spine of lists: list l holds the tokens up to and including the MV_OPEN
// that starts list l + 1 (a sub-list is always its parent's last item).  Parses are read
// through views: a live MvnParse, or tokens packed two words each (w0 = kind | q << 8 |
// removed << 16 | zero << 24, w1 = b | e << 16) - the bounds' parses are packed into the
// program at load time and the installed version's into the batch scratch by the probe,
// so the sweep parses nothing.
// An int token of at most 9 significant digits: its value (the packed form carries it).
TVM_HD bool mvn_small_int(const uint8_t* s, uint32_t b, uint32_t e, uint32_t& v) {
  while (b < e && s[b] == '0') b++;
  if (e - b > 9) return false;
  v = 0;
  for (; b < e; b++) v = v * 10 + uint32_t(s[b] - '0');
  return true;
}

struct MvnParseView {
  const MvnParse* P;
  const uint8_t* s;
  TVM_HD bool has_val(int k) const {
    uint32_t v;
    return P->t[k].kind == MV_INT && mvn_small_int(s, P->t[k].b, P->t[k].e, v);
  }
  TVM_HD uint32_t val(int k) const {
    uint32_t v = 0;
    (void)mvn_small_int(s, P->t[k].b, P->t[k].e, v);
    return v;
  }
  TVM_HD int n() const { return P->n; }
  TVM_HD uint32_t kind(int k) const { return P->t[k].kind; }
  TVM_HD uint32_t q(int k) const { return P->t[k].q; }
  TVM_HD bool removed(int k) const { return P->t[k].removed; }
  TVM_HD bool zero(int k) const { return P->t[k].zero; }
  TVM_HD uint32_t b(int k) const { return P->t[k].b; }
  TVM_HD uint32_t e(int k) const { return P->t[k].e; }
};
// Packed tokens: w0 = kind | q << 8 | removed << 16 | zero << 24 | MVP_VAL, w1 = b | e << 16,
// or for an int of at most 9 significant digits (MVP_VAL) its value: the pairwise compare
// of two such ints reads no text (mvn_int_cmp), which took most of a program's dependent
// loads.
enum : uint32_t { MVP_VAL = 1u << 25 };
struct MvnPackedView {
  const uint32_t* t;
  int cnt;
  const uint8_t* s;
  TVM_HD int n() const { return cnt; }
  TVM_HD uint32_t kind(int k) const { return t[2 * k] & 0xFFu; }
  TVM_HD uint32_t q(int k) const { return (t[2 * k] >> 8) & 0xFFu; }
  TVM_HD bool removed(int k) const { return (t[2 * k] >> 16) & 0xFFu; }
  TVM_HD bool zero(int k) const { return (t[2 * k] >> 24) & 1u; }
  TVM_HD bool has_val(int k) const { return (t[2 * k] & MVP_VAL) != 0; }
  TVM_HD uint32_t val(int k) const { return t[2 * k + 1]; }
  TVM_HD uint32_t b(int k) const { return t[2 * k + 1] & 0xFFFFu; }
  TVM_HD uint32_t e(int k) const { return t[2 * k + 1] >> 16; }
};
constexpr int kMvnPackedWords = 2;  // words per packed token

TVM_HD void mvn_pack(const MvnParse& P, const uint8_t* s, uint32_t* out) {
  for (int k = 0; k < P.n; k++) {
    const MvnTok& t = P.t[k];
    uint32_t w0 = uint32_t(t.kind) | (uint32_t(t.q) << 8) | (uint32_t(t.removed) << 16) | (uint32_t(t.zero) << 24);
    uint32_t w1 = (t.b & 0xFFFFu) | (t.e << 16);
    uint32_t v;
    if (t.kind == MV_INT && mvn_small_int(s, t.b, t.e, v)) {
      w0 |= MVP_VAL;
      w1 = v;
    }
    out[2 * k] = w0;
    out[2 * k + 1] = w1;
  }
}

// Next item of the list at or after token k (removed tokens skipped); -1 at the list's end.
template <class V>
TVM_HD int mvn_next(const V& A, int k) {
  for (; k < A.n(); k++) {
    if (!A.removed(k)) return k;
    if (A.kind(k) == MV_OPEN) return -1;  // a removed sub-list ends its (then emptied) parent
  }
  return -1;
}

// Item at token k against null (-1 / 0 / +1).
template <class V>
TVM_HD int mvn_vs_null(const V& A, int k) {
  for (;;) {
    if (A.kind(k) == MV_INT) return A.zero(k) ? 0 : 1;
    if (A.kind(k) == MV_STR) return A.q(k) < 5 ? -1 : (A.q(k) == 5 ? 0 : 1);
    const int f = mvn_next(A, k + 1);  // a list: its first item decides (empty: equal)
    if (f < 0) return 0;
    k = f;
  }
}

template <class VA, class VB>
TVM_HD int mvn_int_cmp(const VA& A, int x, const VB& B, int y) {
  const bool va = A.has_val(x), vb = B.has_val(y);
  if (va && vb) {  // both below 10^9: the values (digit count, then digits, is the number order)
    const uint32_t p = A.val(x), q = B.val(y);
    return p == q ? 0 : (p < q ? -1 : 1);
  }
  if (va) return -1;  // has_val is exact on both views: the other has 10 or more significant digits
  if (vb) return 1;
  uint32_t i = A.b(x), j = B.b(y);
  const uint32_t ie = A.e(x), je = B.e(y);
  while (i < ie && A.s[i] == '0') i++;
  while (j < je && B.s[j] == '0') j++;
  if (ie - i != je - j) return ie - i < je - j ? -1 : 1;
  for (; i < ie; i++, j++)
    if (A.s[i] != B.s[j]) return A.s[i] < B.s[j] ? -1 : 1;
  return 0;
}

// Qualifier order (comparableQualifier): index among the known ones, unknown words after
// "sp" in byte order of their lower-case text.
template <class VA, class VB>
TVM_HD int mvn_str_cmp(const VA& A, int x, const VB& B, int y) {
  const uint32_t qx = A.q(x), qy = B.q(y);
  if (qx != 7 || qy != 7) return qx == qy ? 0 : (qx < qy ? -1 : 1);
  uint32_t i = A.b(x), j = B.b(y);
  const uint32_t ie = A.e(x), je = B.e(y);
  for (; i < ie && j < je; i++, j++) {
    const uint8_t c = lv_lower(A.s[i]), d = lv_lower(B.s[j]);
    if (c != d) return c < d ? -1 : 1;
  }
  return (i < ie) - (j < je);
}

// ComparableVersion(a).compareTo(b) over two parses.
template <class VA, class VB>
TVM_HD int mvn_cmp(const VA& A, const VB& B) {
  int ka = 0, kb = 0;  // current positions in the current lists of A and B
  for (;;) {
    const int x = mvn_next(A, ka), y = mvn_next(B, kb);
    if (x < 0 && y < 0) return 0;
    if (x < 0) {
      const int r = -mvn_vs_null(B, y);
      if (r) return r;
      kb = B.kind(y) == MV_OPEN ? B.n() : y + 1;  // nothing follows a sub-list item
      ka = A.n();
      continue;
    }
    if (y < 0) {
      const int r = mvn_vs_null(A, x);
      if (r) return r;
      ka = A.kind(x) == MV_OPEN ? A.n() : x + 1;
      kb = B.n();
      continue;
    }
    const uint32_t tx = A.kind(x), ty = B.kind(y);
    if (tx == MV_OPEN && ty == MV_OPEN) {  // list vs list: the sub-lists, item by item
      ka = x + 1;
      kb = y + 1;
      continue;
    }
    int r;
    if (tx == MV_INT) r = ty == MV_INT ? mvn_int_cmp(A, x, B, y) : 1;         // int > string, list
    else if (tx == MV_STR) r = ty == MV_STR ? mvn_str_cmp(A, x, B, y) : -1;   // string < int, list
    else r = ty == MV_INT ? -1 : 1;                                            // list < int, > string
    if (r) return r;
    ka = x + 1;
    kb = y + 1;
  }
}

// ---- Maven, the installed version's key against numeric bounds -----------------------------
// Against a numeric bound B (mvn_numeric: a flat list of ints) every installed version V
// compares like a numeric version give or take an infinitesimal: let P be V's leading int
// items at the top level (up to the first string or sub-list item) and T the rest.  Walking
// V and B item by item, the first difference inside P is an int against an int (or against
// null: B's zero padding), so it is P against B in zero-padded integer order; where B goes
// on past P with a non-zero int, T's first item (a string or a sub-list) meets an int and
// loses (int > string, int > list); where P and B are equal, B is exhausted and T against
// null decides (its first item of non-zero relation).  So
//   compare(V, B) = numeric(P) vs B, and on a tie sign(T against null),
// which is the key order of  key(P) + [0x20 if T < null | 0x40 if T > null] + 0x30 :
// 0x20 < end 0x30 < 0x40 < 0x68 / 0x70 (a zero / int item of any numeric extension of P).
// The rows of an advisory whose every bound is numeric are therefore intervals over this key
// for every installed version (db.cpp DB::compile_rows): no pairwise program runs for them.
// Exact by the argument above; tests/test_libver_host.py checks it against the oracle's
// ComparableVersion on the non-transitive shapes of DESIGN.md §2.2 as well.
template <class Sink>
TVM_HD bool mvn_numeric_projection(const uint8_t* s, uint32_t n, Sink& o) {
  MvnParse P;
  if (!mvn_parse(s, n, P)) return false;
  const MvnParseView V{&P, s};
  int pe = 0, last = -1;  // end of P; its last non-zero int
  for (; pe < P.n; pe++) {
    const MvnTok& t = P.t[pe];
    if (t.removed) {
      if (t.kind == MV_OPEN) break;  // an emptied sub-list ends the list
      continue;                      // a dropped zero
    }
    if (t.kind != MV_INT) break;
    if (!t.zero) last = pe;
  }
  for (int k = 0; k <= last; k++) {
    const MvnTok& t = P.t[k];
    if (t.removed) continue;
    if (t.zero) {
      o.put(0x68);  // a zero followed by a non-zero int
    } else {
      o.put(0x70);
      put_digits(s, t.b, t.e, o);
    }
  }
  int sg = 0;
  for (int k = pe;;) {  // T against null: its items in turn until one is not equal to null
    const int x = mvn_next(V, k);
    if (x < 0) break;
    sg = mvn_vs_null(V, x);
    if (sg || P.t[x].kind == MV_OPEN) break;  // a sub-list is its parent's last item
    k = x + 1;
  }
  if (sg) o.put(sg < 0 ? 0x20 : 0x40);
  o.put(0x30);
  return true;
}

// A Maven advisory program (u32 words, built by libdb.cpp mvn_program):
//   w[0] = n_vulnerable_groups | n_secure_groups << 16, then the groups in that order;
//   group = n_terms, then per term {op | n_tokens << 8 | text length << 16, word offset of
//   the bound's packed tokens, word offset of its text (4 bytes per word)}.
// IsVulnerable: (no vulnerable groups, or one of them holds) and none of the secure groups.
enum : uint32_t { MVO_EQ = 0, MVO_NE = 1, MVO_GT = 2, MVO_LT = 3, MVO_GE = 4, MVO_LE = 5 };

TVM_HD bool mvn_op(uint32_t op, int c) {
  switch (op) {
    case MVO_EQ: return c == 0;
    case MVO_NE: return c != 0;
    case MVO_GT: return c > 0;
    case MVO_LT: return c < 0;
    case MVO_GE: return c >= 0;
    default: return c <= 0;
  }
}

// The program at w against the installed version's parse V.
template <class V>
TVM_HD bool mvn_program_eval(const uint32_t* w, const V& inst) {
  const uint32_t nv = w[0] & 0xFFFFu, ns = w[0] >> 16;
  uint32_t at = 1;
  bool vul = nv == 0, sec = false;
  for (uint32_t g = 0; g < nv + ns; g++) {
    const uint32_t nt = w[at++];
    bool all = true;
    for (uint32_t t = 0; t < nt; t++) {
      const uint32_t d = w[at], tok = w[at + 1], txt = w[at + 2];
      at += 3;
      if (!all) continue;
      const MvnPackedView B{w + tok, int((d >> 8) & 0xFFu), reinterpret_cast<const uint8_t*>(w + txt)};
      all = mvn_op(d & 0xFFu, mvn_cmp(inst, B));
    }
    if (g < nv) vul = vul || all;
    else sec = sec || all;
  }
  return vul && !sec;
}

// =========================================================================== RUBYGEMS ====
// github.com/aquasecurity/go-gem-version (go.mod:16), Gem::Version:
//   \s*( N(.[0-9a-zA-Z]+)* (-[0-9A-Za-z-]+(.[0-9A-Za-z-]+)*)? )?\s*     ("" reads "0")
// '-' reads ".pre."; segments = digit runs (integers) and letter runs (strings); canonical
// segments drop trailing zeros of the numeric prefix and of the string part; comparison
// pads with 0, strings sort below integers.
// Key: string 0x01 bytes 0x00 | zero followed by a string 0x02 | end 0x03 | zero followed
// by an integer 0x04 | integer > 0: 0x05 digits.
struct GemSeg {
  uint8_t str;    // 1 letters, 0 digits
  uint8_t zero;
  uint32_t b, e;  // span; b == e for the synthetic "pre" of a '-'
};
constexpr int kGemMaxSeg = 48;

TVM_HD bool gem_parse(const uint8_t* s, uint32_t n, GemSeg* seg, int& ns) {
  uint32_t i = 0;
  while (i < n && lv_space(s[i])) i++;
  while (n > i && lv_space(s[n - 1])) n--;
  ns = 0;
  if (i == n) {  // "" is "0"
    seg[0] = GemSeg{0, 1, 0, 0};
    ns = 1;
    return true;
  }
  // validate: digits, then (.[0-9a-zA-Z]+)*, then optional -[0-9A-Za-z-]+(.[0-9A-Za-z-]+)*
  uint32_t j = i;
  while (j < n && is_adigit(s[j])) j++;
  if (j == i) return false;
  while (j < n && s[j] == '.') {
    const uint32_t b = ++j;
    while (j < n && lv_alnum(s[j])) j++;
    if (j == b) return false;
  }
  if (j < n) {
    if (s[j] != '-') return false;
    j++;
    uint32_t run = 0;
    for (; j < n; j++) {
      if (lv_alnum(s[j]) || s[j] == '-') run++;
      else if (s[j] == '.' && run) run = 0;
      else return false;
    }
    if (!run) return false;
  }
  for (uint32_t k = i; k < n;) {
    if (s[k] == '-') {  // ".pre."
      if (ns >= kGemMaxSeg) return false;
      seg[ns++] = GemSeg{1, 0, k, k};
      k++;
    } else if (is_adigit(s[k]) || lv_alpha(s[k])) {
      const bool d = is_adigit(s[k]);
      const uint32_t b = k;
      while (k < n && (d ? is_adigit(s[k]) : lv_alpha(s[k]))) k++;
      if (ns >= kGemMaxSeg) return false;
      bool zero = false;
      if (d) {
        uint32_t z = b;
        while (z < k && s[z] == '0') z++;
        zero = z == k;
      }
      seg[ns++] = GemSeg{uint8_t(d ? 0 : 1), uint8_t(zero), b, k};
    } else {
      k++;
    }
  }
  return true;
}

// Canonical segments: marks dropped ones with e = b = ~0u.
TVM_HD void gem_canonical(GemSeg* seg, int ns) {
  int first_str = ns;
  for (int k = 0; k < ns; k++)
    if (seg[k].str) { first_str = k; break; }
  for (int k = first_str - 1; k >= 0 && !seg[k].str && seg[k].zero; k--) seg[k].b = seg[k].e = ~0u;
  for (int k = ns - 1; k >= first_str && !seg[k].str && seg[k].zero; k--) seg[k].b = seg[k].e = ~0u;
}

template <class Sink>
TVM_HD void gem_emit(const uint8_t* s, const GemSeg* seg, int ns, Sink& o) {
  for (int k = 0; k < ns; k++) {
    const GemSeg& g = seg[k];
    if (g.b == ~0u) continue;
    if (g.str) {
      o.put(0x01);
      if (g.b == g.e) {
        o.put('p'); o.put('r'); o.put('e');
      } else {
        for (uint32_t i = g.b; i < g.e; i++) o.put(s[i]);
      }
      o.put(0x00);
    } else if (!g.zero) {
      o.put(0x05);
      put_digits(s, g.b, g.e, o);
    } else {
      int nxt = 0;  // 1 integer, -1 string
      for (int j = k + 1; j < ns; j++) {
        if (seg[j].b == ~0u || (!seg[j].str && seg[j].zero)) continue;
        nxt = seg[j].str ? -1 : 1;
        break;
      }
      o.put(nxt < 0 ? 0x02 : 0x04);
    }
  }
  o.put(0x03);
}

template <class Sink>
TVM_HD bool gem_encode(const uint8_t* s, uint32_t n, Sink& o) {
  GemSeg seg[kGemMaxSeg];
  int ns;
  if (!gem_parse(s, n, seg, ns)) return false;
  gem_canonical(seg, ns);
  gem_emit(s, seg, ns, o);
  return true;
}

// ------------------------------------------------------------------ grammar dispatch ----
// Only the grammars of set GM are compiled in (a kernel specialised for go-version tiles
// carries neither the Maven parse nor the RubyGems segment arrays, and so no scratch).
template <uint32_t GM, class Sink>
TVM_HD bool encode_version_cls_gm(uint8_t cmp, const uint8_t* s, uint32_t n, Sink& o, uint32_t& cls) {
  cls = 0;
  if constexpr ((GM >> 4) & 1u) {  // CMP_GENERIC
    if (cmp == CMP_GENERIC) return gen_encode(s, n, false, o);
  }
  if constexpr ((GM >> 9) & 1u) {  // CMP_BITNAMI
    if (cmp == CMP_BITNAMI) return gen_encode(s, n, true, o);
  }
  if constexpr ((GM >> 5) & 1u) {  // CMP_NPM
    if (cmp == CMP_NPM) return npm_encode(s, n, o, cls);
  }
  if constexpr ((GM >> 6) & 1u) {  // CMP_PEP440
    if (cmp == CMP_PEP440) return pep_encode(s, n, o, cls);
  }
  if constexpr ((GM >> 7) & 1u) {  // CMP_MAVEN
    if (cmp == CMP_MAVEN) return mvn_numeric_projection(s, n, o);  // one class (see above)
  }
  if constexpr ((GM >> 8) & 1u) {  // CMP_GEM
    if (cmp == CMP_GEM) return gem_encode(s, n, o);
  }
  if constexpr ((GM & 0xEu) != 0) {  // the OS grammars
    if (cmp == CMP_DEB || cmp == CMP_APK || cmp == CMP_RPM) return encode_version(cmp, s, n, o);
  }
  return false;
}

template <class Sink>
TVM_HD bool encode_version_cls(uint8_t cmp, const uint8_t* s, uint32_t n, Sink& o, uint32_t& cls) {
  return encode_version_cls_gm<0x3FEu>(cmp, s, n, o, cls);
}

// Grammar sets a match kernel is specialised for (bit c = Cmp c): a batch whose platforms
// only use the dpkg grammar runs a kernel with no other encoder in it, so the register and
// scratch footprint is the dpkg one.  The host picks the smallest set covering the batch.
enum : uint32_t {
  GM_DEB = 1u << CMP_DEB,
  GM_OS = GM_DEB | (1u << CMP_APK) | (1u << CMP_RPM),
  GM_ALL = 0x3FEu,
  // every grammar but Maven and RubyGems: their parses (MvnParse, GemSeg arrays) and the Maven
  // program evaluator are what put the all-grammar kernel at 96 VGPRs + ~800 B of scratch per
  // lane; a kernel without them runs the lockfile ecosystems most tiles hold (go, npm, PEP 440,
  // Bitnami) and the OS grammars
  GM_LEAN = GM_ALL & ~((1u << CMP_MAVEN) | (1u << CMP_GEM)),
};

template <uint32_t GM, class Sink>
TVM_HD bool encode_version_gm(uint8_t cmp, const uint8_t* s, uint32_t n, Sink& o, uint32_t& cls) {
  cls = 0;
  if (!((GM >> cmp) & 1u)) return false;
  if constexpr (GM == GM_DEB) {
    return deb_encode(s, n, o);
  } else if constexpr ((GM & ~GM_OS) == 0) {
    return encode_version(cmp, s, n, o);
  } else {
    return encode_version_cls_gm<GM>(cmp, s, n, o, cls);
  }
}

}  // namespace tvm
