// Version sort-key encoders (host + device).
//
// Every supported version grammar is mapped to a byte string whose plain
// lexicographic order (common.h key_cmp) IS the reference comparator's order.
// The flattener encodes advisory bounds (FixedVersion, AffectedVersion, ...) once
// at load time with these functions; the probe kernel encodes each installed
// version on the GPU with the very same code, so a (package, advisory) test is
// one short word-wise compare instead of a parse + compare per pair.
//
// ---- dpkg: github.com/knqyf263/go-deb-version (reference go.mod:62) ---------------------
// Call sites: pkg/detector/ospkg/debian/debian.go:66,107,113, ubuntu/ubuntu.go:92,116,122,
// amazon/amazon.go:67,74,80.  go-deb-version compares epoch (int), then upstream, then
// revision; each part is cut into pairs (non-digit run, digit run) - the first run is
// "" when the part starts with a digit, missing entries are ("", 0) - and a pair
// compares its runs byte by byte with weights '~' < end-of-run < letters < others
// (letter = unicode.IsLetter of the byte read as a Latin-1 rune), then its digit runs
// as integers (strconv.Atoi, which clamps at MaxInt64 on overflow).
//
// Key layout:  EPOCH  PART(upstream)  PART(revision)
//   EPOCH        = nbytes(1) + big-endian minimal bytes
//   PART("")     = TERM0 END            (the empty part equals one ("", 0) pair)
//   PART(s)      = { code(c) for c in run ; TERM_k ; k big-endian bytes of the number }* END
//   codes: '~'=0x01 < END=0x02 < TERM_k=0x03+k (k=0..8) < letters 0x0C..0x80 < others 0x81..0xFF
// TERM_k both ends the run (end-of-run weight 0 sits between '~' and letters) and
// orders numbers by byte length before value.  A missing pair at index >= 1 is
// represented by END, which sorts exactly like the ("", 0) padding against any real
// pair (whose run is non-empty there).  Bound: len(key) <= 2*len(version) + 12.
#pragma once
#include "common.h"
#include "unicode_tab.h"

namespace tvm {

// ------------------------------------------------------------------ Unicode categories ----
static __constant__ uint32_t d_uni_letter[TVM_UNI_NLETTER][2] = {TVM_UNI_LETTER_RANGES};
static __constant__ uint32_t d_uni_digit[TVM_UNI_NDIGIT][2] = {TVM_UNI_DIGIT_RANGES};
static const uint32_t h_uni_letter[TVM_UNI_NLETTER][2] = {TVM_UNI_LETTER_RANGES};
static const uint32_t h_uni_digit[TVM_UNI_NDIGIT][2] = {TVM_UNI_DIGIT_RANGES};

TVM_HD bool uni_in(const uint32_t (*t)[2], int n, uint32_t cp) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    if (cp < t[mid][0]) hi = mid - 1;
    else if (cp > t[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}
// unicode.IsLetter
TVM_HD bool rune_letter(uint32_t cp) {
  if (cp < 0x80) return ((cp | 0x20) >= 'a' && (cp | 0x20) <= 'z');
#ifdef __HIP_DEVICE_COMPILE__
  return uni_in(d_uni_letter, TVM_UNI_NLETTER, cp);
#else
  return uni_in(h_uni_letter, TVM_UNI_NLETTER, cp);
#endif
}
// unicode.IsDigit
TVM_HD bool rune_digit(uint32_t cp) {
  if (cp < 0x80) return cp >= '0' && cp <= '9';
#ifdef __HIP_DEVICE_COMPILE__
  return uni_in(d_uni_digit, TVM_UNI_NDIGIT, cp);
#else
  return uni_in(h_uni_digit, TVM_UNI_NDIGIT, cp);
#endif
}
// utf8.DecodeRuneInString: invalid -> U+FFFD with width 1.
TVM_HD uint32_t decode_rune(const uint8_t* s, uint32_t n, uint32_t* w) {
  uint32_t c = s[0];
  *w = 1;
  if (c < 0x80) return c;
  uint32_t lo = 0x80, hi = 0xBF, need, cp;
  if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) { need = 2; cp = c & 0x0F; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
  else if (c >= 0xF0 && c <= 0xF4) { need = 3; cp = c & 0x07; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
  else return 0xFFFD;
  if (need >= n) return 0xFFFD;
  for (uint32_t k = 1; k <= need; k++) {
    uint32_t d = s[k];
    if (k == 1 ? (d < lo || d > hi) : (d < 0x80 || d > 0xBF)) return 0xFFFD;
    cp = (cp << 6) | (d & 0x3F);
  }
  *w = need + 1;
  return cp;
}

TVM_HD bool is_adigit(uint8_t c) { return c >= '0' && c <= '9'; }

// ------------------------------------------------------------------------------ dpkg -----
enum : uint8_t { DEB_TILDE = 0x01, DEB_END = 0x02, DEB_TERM0 = 0x03 };

struct DebCodes { uint8_t v[256]; };
constexpr bool latin1_letter(int b) {
  return (b >= 'A' && b <= 'Z') || (b >= 'a' && b <= 'z') || b == 0xAA || b == 0xB5 || b == 0xBA ||
         (b >= 0xC0 && b <= 0xFF && b != 0xD7 && b != 0xF7);
}
constexpr DebCodes make_deb_codes() {
  DebCodes t{};
  int code = 0x0C;
  for (int b = 0; b < 256; b++)
    if (latin1_letter(b)) t.v[b] = uint8_t(code++);
  for (int b = 1; b < 256; b++)
    if (!latin1_letter(b) && !(b >= '0' && b <= '9') && b != '~') t.v[b] = uint8_t(code++);
  t.v['~'] = DEB_TILDE;
  return t;
}
static_assert(make_deb_codes().v[0xFF] == 0x80 && make_deb_codes().v[0xF7] == 0xFF &&
                  make_deb_codes().v['A'] == 0x0C && make_deb_codes().v['.'] > 0x80,
              "dpkg code table must fill 0x0C..0xFF exactly");
static __constant__ DebCodes d_deb_codes = make_deb_codes();
static constexpr DebCodes h_deb_codes = make_deb_codes();

// ASCII bytes by arithmetic (no table load in the per-lane parse loop): letters take
// 0x0C.. in byte order, the other non-digit bytes 0x81.. in byte order ('~' aside).
TVM_HD constexpr uint8_t deb_code_ascii(uint8_t b) {
  return b >= 'a' && b <= 'z'   ? uint8_t(b - 'a' + 0x26)
         : b >= 'A' && b <= 'Z' ? uint8_t(b - 'A' + 0x0C)
         : b == '~'             ? uint8_t(DEB_TILDE)
         : b < 0x30             ? uint8_t(b + 0x80)
         : b < 0x41             ? uint8_t(b + 0x76)
         : b < 0x61             ? uint8_t(b + 0x5C)
         : b < 0x7F             ? uint8_t(b + 0x42)
                                : uint8_t(0xC0);
}
constexpr bool deb_code_ascii_ok() {
  for (int b = 1; b < 0x80; b++)
    if (!(b >= '0' && b <= '9') && deb_code_ascii(uint8_t(b)) != make_deb_codes().v[b]) return false;
  return true;
}
static_assert(deb_code_ascii_ok(), "dpkg ASCII codes must equal the table");

TVM_HD uint8_t deb_code(uint8_t b) {
  if (b < 0x80) return deb_code_ascii(b);
#ifdef __HIP_DEVICE_COMPILE__
  return d_deb_codes.v[b];
#else
  return h_deb_codes.v[b];
#endif
}

// verifyUpstreamVersion / verifyDebianRevision rune checks.
TVM_HD bool deb_valid_runes(const uint8_t* s, uint32_t n, bool upstream) {
  uint32_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) {
      bool ok = is_adigit(c) || ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') || c == '.' || c == '+' ||
                c == '~' || c == '_' || (upstream && (c == '-' || c == ':'));
      if (!ok) return false;
      i++;
    } else {
      uint32_t w;
      uint32_t r = decode_rune(s + i, n - i, &w);
      if (!rune_letter(r) && !rune_digit(r)) return false;
      i += w;
    }
  }
  return true;
}

// One digit run [i, e) as TERM_k + k big-endian bytes; strconv.Atoi clamps at MaxInt64.
// Runs of <= 9 significant digits (nearly all) accumulate in 32 bits.
template <class Sink>
TVM_HD void deb_number(const uint8_t* s, uint32_t i, uint32_t e, Sink& o) {
  while (i < e && s[i] == '0') i++;
  uint64_t v;
  if (e - i <= 9) {
    uint32_t v32 = 0;
    for (; i < e; i++) v32 = v32 * 10u + uint32_t(s[i] - '0');
    v = v32;
  } else if (e - i > 19) {
    v = uint64_t(INT64_MAX);
  } else {
    v = 0;
    bool over = false;
    for (; i < e && !over; i++) {
      const uint64_t d = uint64_t(s[i] - '0');
      if (v > (uint64_t(INT64_MAX) - d) / 10) over = true;
      else v = v * 10 + d;
    }
    if (over) v = uint64_t(INT64_MAX);
  }
  const uint32_t k = v ? uint32_t(8 - (__builtin_clzll(v) >> 3)) : 0u;
  o.put(uint8_t(DEB_TERM0 + k));
  for (int b = int(k) - 1; b >= 0; b--) o.put(uint8_t(v >> (8 * b)));
}

// PART(s) of the key layout above (s already validated).
template <class Sink>
TVM_HD void deb_part(const uint8_t* s, uint32_t n, Sink& o) {
  if (n == 0) {
    o.put(DEB_TERM0);
    o.put(DEB_END);
    return;
  }
  uint32_t i = 0;
  while (i < n) {
    while (i < n && !is_adigit(s[i])) o.put(deb_code(s[i++]));
    uint32_t e = i;
    while (e < n && is_adigit(s[e])) e++;
    deb_number(s, i, e, o);
    i = e;
  }
  o.put(DEB_END);
}

// ASCII bytes go-deb-version accepts in an upstream version (digits, letters, . + ~ _ - :);
// the revision accepts the same set minus '-' and ':'.
constexpr uint64_t kDebOk0 = (1ull << '.') | (1ull << '+') | (1ull << '-') | (1ull << ':') | (0x3FFull << '0');
constexpr uint64_t kDebOk1 = (1ull << ('_' - 64)) | (1ull << ('~' - 64)) | (0x3FFFFFFull << ('A' - 64)) |
                             (0x3FFFFFFull << ('a' - 64));

// go-deb-version NewVersion + key emission.  Returns false on a parse error (the sink
// may have received a partial key, which the caller discards).  One pre-pass finds the
// first ':' (epoch), the last '-' (revision) and checks the ASCII character sets; only a
// string with non-ASCII bytes takes the rune-decoding validity check.
template <class Sink>
TVM_HD bool deb_encode(const uint8_t* s, uint32_t n, Sink& o) {
  uint32_t colon = n, dash = n, last_colon = n;
  bool bad = false, high = false;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    if (c == ':') {
      if (colon == n) colon = i;
      last_colon = i;
    } else if (c == '-') {
      dash = i;
    }
    if (c >= 0x80) high = true;
    else bad |= !(((c < 64 ? kDebOk0 >> c : kDebOk1 >> (c - 64)) & 1u));
  }
  // epoch: strconv.Atoi of the text before the first ':'; negative -> error
  uint64_t epoch = 0;
  uint32_t r0 = 0;
  if (colon < n) {
    uint32_t i = 0;
    bool neg = false;
    if (colon > 0 && (s[0] == '+' || s[0] == '-')) { neg = s[0] == '-'; i = 1; }
    if (i == colon) return false;
    for (; i < colon; i++) {
      if (!is_adigit(s[i])) return false;
      uint64_t d = uint64_t(s[i] - '0');
      if (epoch > (~0ULL - d) / 10) return false;
      epoch = epoch * 10 + d;
      if (epoch > uint64_t(INT64_MAX) + (neg ? 1 : 0)) return false;
    }
    if (neg && epoch != 0) return false;  // epoch is negative
    r0 = colon + 1;
  }
  // split the rest at its last '-'
  const bool has_rev = dash < n && dash >= r0;
  const uint8_t* up = s + r0;
  const uint32_t nup = (has_rev ? dash : n) - r0;
  const uint8_t* rev = has_rev ? s + dash + 1 : s + n;
  const uint32_t nrev = has_rev ? n - dash - 1 : 0;
  if (nup == 0 || !is_adigit(up[0])) return false;
  if (high) {
    if (!deb_valid_runes(up, nup, true) || !deb_valid_runes(rev, nrev, false)) return false;
  } else {
    // the epoch text was checked above; the rest must be in the ASCII sets, and the
    // revision (after the last '-') may not hold a ':'
    if (bad) {
      if (!deb_valid_runes(up, nup, true) || !deb_valid_runes(rev, nrev, false)) return false;
    }
    if (has_rev && last_colon < n && last_colon > dash) return false;
  }
  const uint32_t k = epoch ? uint32_t(8 - (__builtin_clzll(epoch) >> 3)) : 0u;
  o.put(uint8_t(k));
  for (int b = int(k) - 1; b >= 0; b--) o.put(uint8_t(epoch >> (8 * b)));
  deb_part(up, nup, o);
  deb_part(rev, nrev, o);
  return true;
}

// ---- dpkg sort key, lane-serial over dwords (the match kernel's common case) -------------
//
// The same key as verkey.h deb_encode (go-deb-version order, layout documented there) for
// versions that are all ASCII with an epoch of at most 9 digits, digit runs of at most 9
// significant digits and a key of at most kFastKeyCap bytes - everything else returns
// FAST_FALLBACK and takes the generic encoder.  It differs in how it runs, not in what it
// produces (host test: tests/test_fastdeb_host.py runs this very function against
// deb_encode):
//   * the version is read from LDS a dword at a time (aligned reads + v_alignbyte) and its
//     bytes taken with constant shifts, instead of one ds_read_u8 per byte per pass;
//   * one SWAR pre-pass per dword finds the first / last ':' and the last '-' and flags
//     non-ASCII bytes (exact per-byte equality masks, no per-byte branch);
//   * the emission pass is branch-free per byte: the number token TERM_k + k big-endian
//     bytes and the next code byte are always written at the lane's key position in LDS,
//     and only the position advance depends on the byte, so lanes at different points of
//     their strings never diverge; character codes and validity come from a 128-byte LDS
//     table (code 0 = not in go-deb-version's ASCII sets).
constexpr uint32_t kFastKeyStride = 44;  // LDS bytes per lane: 11 dwords, co-prime with the 64 banks
constexpr uint32_t kFastKeyCap = 32;     // longest key kept (writes land at most 5 bytes past the clamped position)
enum : uint32_t { FAST_INVALID = 0, FAST_OK = 1, FAST_FALLBACK = 2 };

// Code byte of each ASCII non-digit for deb_part, 0 where go-deb-version rejects the byte
// (verifyUpstreamVersion / verifyDebianRevision): filled per workgroup into LDS.
TVM_HD uint8_t deb_fast_code(uint32_t c) {
  const bool ok = c < 64 ? ((kDebOk0 >> c) & 1u) : c < 128 ? ((kDebOk1 >> (c - 64)) & 1u) : false;
  return ok ? deb_code_ascii(uint8_t(c)) : uint8_t(0);
}

// Bit 7 of byte i set iff byte i of x equals the byte of pat (exact, no borrow artefacts).
TVM_HD uint32_t byte_eq_mask(uint32_t x, uint32_t pat) {
  const uint32_t t = x ^ pat;
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}

// Dword i of a byte string at any alignment (bytes 4i .. 4i+3, little-endian); the words
// past the end may hold anything (callers mask), but must be readable.
TVM_HD uint32_t str_dword(const uint32_t* base, uint32_t sh, uint32_t i) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_alignbyte(base[i + 1], base[i], sh);
#else
  return uint32_t(((uint64_t(base[i + 1]) << 32) | base[i]) >> (8 * sh));
#endif
}

TVM_HD uint32_t clz32(uint32_t v) {
#ifdef __HIP_DEVICE_COMPILE__
  return uint32_t(__clz(int(v)));  // 32 for 0
#else
  return v ? uint32_t(__builtin_clz(v)) : 32u;
#endif
}

// Emission state of deb_fast_key: key position, value of the digit run so far, previous
// byte a digit, a rejected byte seen, a run over 9 significant digits seen.
struct DebFastState {
  uint32_t pos, v;
  bool pd, bad, ovf;
};

// One byte of a part (c < 0x80; split: the '-' between upstream and revision).  The token
// of a run that ends here (TERM_k + k big-endian bytes; v = 0 gives TERM0, the empty run
// a split closes) and the byte's code (END at the split) are written unconditionally at
// pos; only the advance depends on the byte, so the loop has no branch.
TVM_HD void deb_fast_byte(uint32_t c, bool split, uint8_t* kb, const uint8_t* tab, DebFastState& st) {
  const uint32_t d = c - '0';
  const bool isd = d < 10u;
  const uint32_t code = tab[c & 0x7Fu];
  const uint32_t v = st.v;
  const uint32_t k = (39u - clz32(v)) >> 3;     // bytes of v (0 for v = 0)
  const uint32_t vb = v << ((32u - 8u * k) & 31u);  // v = 0 when k = 0, so the shift wrap is harmless
  const uint32_t at = st.pos < kFastKeyCap ? st.pos : kFastKeyCap;
  uint8_t* o = kb + at;
  o[0] = uint8_t(DEB_TERM0 + k);
  o[1] = uint8_t(vb >> 24);
  o[2] = uint8_t(vb >> 16);
  o[3] = uint8_t(vb >> 8);
  o[4] = uint8_t(vb);
  const bool flush = !isd && (st.pd || split);
  const uint32_t tk = flush ? k + 1 : 0u;
  o[tk] = split ? uint8_t(DEB_END) : uint8_t(code);
  st.pos += tk + (isd ? 0u : 1u);
  st.bad = st.bad || (!isd && !split && code == 0u);
  st.ovf = st.ovf || (isd && v >= 100000000u);  // a 10th significant digit
  st.v = isd ? (v << 3) + (v << 1) + d : 0u;
  st.pd = isd;
}

// Key of dpkg version s[0, n) into kb[0, len) (kb: kFastKeyStride writable bytes).
// Returns FAST_OK, FAST_INVALID (go-deb-version NewVersion error) or FAST_FALLBACK.
TVM_HD uint32_t deb_fast_key(const uint8_t* s, uint32_t n, uint8_t* kb, const uint8_t* tab, uint32_t& len) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(s);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t sh = uint32_t(a & 3);
  // pre-pass: first and last ':', last '-', any byte >= 0x80
  uint32_t colon = n, lcolon = n, dash = n, high = 0;
  for (uint32_t j = 0; j < n; j += 4) {
    uint32_t x = str_dword(base, sh, j >> 2);
    if (n - j < 4) x &= (1u << (8 * (n - j))) - 1u;
    high |= x;
    const uint32_t md = byte_eq_mask(x, 0x2D2D2D2Du), mc = byte_eq_mask(x, 0x3A3A3A3Au);
    if (md) dash = j + ((31u - uint32_t(__builtin_clz(md))) >> 3);
    if (mc) {
      if (colon == n) colon = j + (uint32_t(__builtin_ctz(mc)) >> 3);
      lcolon = j + ((31u - uint32_t(__builtin_clz(mc))) >> 3);
    }
  }
  if (high & 0x80808080u) return FAST_FALLBACK;
  // epoch: 1..9 digits before the first ':' (signs, overflow, empty: the generic parser)
  uint32_t epoch = 0, r0 = 0;
  if (colon < n) {
    if (colon == 0 || colon > 9) return FAST_FALLBACK;
    for (uint32_t i = 0; i < colon; i++) {
      const uint32_t d = uint32_t(s[i]) - '0';
      if (d >= 10) return FAST_FALLBACK;
      epoch = epoch * 10u + d;
    }
    r0 = colon + 1;
  }
  const bool has_rev = dash < n && dash >= r0;
  if (r0 >= (has_rev ? dash : n) || uint32_t(s[r0]) - '0' >= 10u) return FAST_INVALID;
  if (has_rev && lcolon < n && lcolon > dash) return FAST_INVALID;
  // EPOCH
  const uint32_t ke = epoch ? (39u - uint32_t(__builtin_clz(epoch))) >> 3 : 0u;
  const uint32_t eb = ke ? epoch << (32 - 8 * ke) : 0u;
  kb[0] = uint8_t(ke);
  kb[1] = uint8_t(eb >> 24);
  kb[2] = uint8_t(eb >> 16);
  kb[3] = uint8_t(eb >> 8);
  kb[4] = uint8_t(eb);
  uint32_t pos = 1 + ke;
  // PART(upstream) PART(revision): per byte, always write the pending number token and the
  // byte's code at the current position (clamped to the buffer); advance only over what the
  // byte emits.  Bytes from r0 on: whole dwords, then the last 0..3 bytes one by one.
  DebFastState st{pos, 0u, false, false, false};
  const uint8_t* s2 = s + r0;
  const uint32_t m = n - r0, sp2 = has_rev ? dash - r0 : 0xFFFFFFFFu;
  const uintptr_t a2 = reinterpret_cast<uintptr_t>(s2);
  const uint32_t* base2 = reinterpret_cast<const uint32_t*>(a2 & ~uintptr_t(3));
  const uint32_t sh2 = uint32_t(a2 & 3);
  for (uint32_t j = 0; j + 4 <= m; j += 4) {
    const uint32_t x = str_dword(base2, sh2, j >> 2);
#pragma unroll
    for (uint32_t b = 0; b < 4; b++) deb_fast_byte((x >> (8 * b)) & 0xFFu, j + b == sp2, kb, tab, st);
  }
  for (uint32_t j = m & ~3u; j < m; j++) deb_fast_byte(s2[j], j == sp2, kb, tab, st);
  if (st.bad) return FAST_INVALID;
  if (st.ovf) return FAST_FALLBACK;  // a run may exceed 32 bits (or clamp at MaxInt64)
  pos = st.pos;
  const uint32_t v = st.v;
  // end of the last part, then PART("") when there is no revision
  {
    const uint32_t k = (39u - clz32(v)) >> 3;
    const uint32_t vb = v << ((32u - 8u * k) & 31u);
    uint8_t* o = kb + (pos < kFastKeyCap ? pos : kFastKeyCap);
    o[0] = uint8_t(DEB_TERM0 + k);
    o[1] = uint8_t(vb >> 24);
    o[2] = uint8_t(vb >> 16);
    o[3] = uint8_t(vb >> 8);
    o[4] = uint8_t(vb);
    pos += k + 1;
    kb[pos < kFastKeyCap ? pos : kFastKeyCap] = DEB_END;
    pos++;
    if (!has_rev) {
      kb[pos < kFastKeyCap ? pos : kFastKeyCap] = DEB_TERM0;
      kb[pos + 1 < kFastKeyCap ? pos + 1 : kFastKeyCap] = DEB_END;
      pos += 2;
    }
  }
  if (pos > kFastKeyCap) return FAST_FALLBACK;
  len = pos;
  return FAST_OK;
}

// ------------------------------------------------------------------- signed integers -----
// Order-preserving variable-length code of a signed 64-bit value: v >= 0 as 0x80+k then
// k big-endian bytes (k minimal, 0 for v = 0); v < 0 as 0x7F-k then the k bytes of
// ~(-(v+1)) (more negative -> smaller).  Self-delimiting, so a following token starts at
// the same offset in two keys whose values are equal.
template <class Sink>
TVM_HD void put_sint(int64_t v, Sink& o) {
  if (v >= 0) {
    const uint64_t u = uint64_t(v);
    uint32_t k = 0;
    for (uint64_t t = u; t; t >>= 8) k++;
    o.put(uint8_t(0x80 + k));
    for (int b = int(k) - 1; b >= 0; b--) o.put(uint8_t(u >> (8 * b)));
  } else {
    const uint64_t m = ~uint64_t(v);  // -(v+1) >= 0
    uint32_t k = 0;
    for (uint64_t t = m; t; t >>= 8) k++;
    o.put(uint8_t(0x7F - k));
    for (int b = int(k) - 1; b >= 0; b--) o.put(uint8_t(~(m >> (8 * b))));
  }
}

// ------------------------------------------------------------------------------- apk -----
// github.com/knqyf263/go-apk-version (reference go.mod:61), the Go port of apk-tools'
// version.c.  Call sites: alpine/alpine.go:93,126,141, wolfi/wolfi.go:48,68,
// chainguard/chainguard.go:48,68.  A version is a stream of tokens whose kind is decided
// before each read (first kind: DIGIT); two versions compare value by value while the
// kinds agree; when the kinds differ, a pre-release suffix (_alpha/_beta/_pre/_rc) is
// smaller than anything, otherwise the LATER kind in the list DOZ, DIGIT, LETTER, SUFFIX,
// SUFFIX_NO, REVISION_NO, END is the smaller version.  Key = one class byte per token
// (that order inverted, pre-suffixes first) followed by put_sint(value); END ends it.
enum : int { APK_INVALID = -1, APK_DOZ = 0, APK_DIGIT, APK_LETTER, APK_SUFFIX, APK_SUFFIX_NO, APK_REV, APK_END };
enum : uint8_t {
  APKC_SUFPRE = 0x01, APKC_END = 0x02, APKC_REV = 0x03, APKC_SUFNO = 0x04, APKC_SUFPOST = 0x05,
  APKC_LETTER = 0x06, APKC_DIGIT = 0x07, APKC_DOZ = 0x08,
};

TVM_HD bool apk_lower(uint8_t c) { return c >= 'a' && c <= 'z'; }

// next_token of version.c: the kind of the token that starts at s[i] (consumes separators).
TVM_HD int apk_next_kind(int kind, const uint8_t* s, uint32_t n, uint32_t& i) {
  int k = APK_INVALID;
  if (i >= n || s[i] == 0) {
    k = APK_END;
  } else if ((kind == APK_DIGIT || kind == APK_DOZ) && apk_lower(s[i])) {
    k = APK_LETTER;
  } else if (kind == APK_LETTER && is_adigit(s[i])) {
    k = APK_DIGIT;
  } else if (kind == APK_SUFFIX && is_adigit(s[i])) {
    k = APK_SUFFIX_NO;
  } else {
    if (s[i] == '.') k = APK_DOZ;
    else if (s[i] == '_') k = APK_SUFFIX;
    else if (s[i] == '-') {
      if (i + 1 < n && s[i + 1] == 'r') {
        k = APK_REV;
        i++;
      }
    }
    i++;
  }
  if (k < kind && !((k == APK_DOZ && kind == APK_DIGIT) || (k == APK_SUFFIX && kind == APK_SUFFIX_NO) ||
                    (k == APK_DIGIT && kind == APK_LETTER)))
    k = APK_INVALID;
  return k;
}

TVM_HD bool apk_prefix(const uint8_t* s, uint32_t n, uint32_t i, const char* w, uint32_t wl) {
  if (i + wl > n) return false;
  for (uint32_t j = 0; j < wl; j++)
    if (s[i + j] != uint8_t(w[j])) return false;
  return true;
}

template <class Sink>
TVM_HD bool apk_encode(const uint8_t* s, uint32_t n, Sink& o) {
  int kind = APK_DIGIT;
  uint32_t i = 0;
  for (;;) {
    if (i >= n) {
      // get_token on an empty rest ("" or a trailing separator) still yields a token of
      // the pending kind with value 0, then END ("1_" == "1_cvs", "" == "0")
      static constexpr uint8_t kCls[] = {APKC_DOZ, APKC_DIGIT, APKC_LETTER, APKC_SUFPOST, APKC_SUFNO, APKC_REV};
      if (kind >= APK_DOZ && kind <= APK_REV) {
        o.put(kCls[kind]);
        put_sint(0, o);
      }
      o.put(APKC_END);
      return true;
    }
    int64_t v = 0;
    int nt = APK_INVALID;
    uint8_t cls;
    switch (kind) {
      case APK_DOZ:
        if (s[i] == '0') {
          uint32_t z = 0;
          while (i < n && s[i] == '0') i++, z++;
          v = -int64_t(z);
          nt = APK_DIGIT;
          cls = APKC_DOZ;
          break;
        }
        [[fallthrough]];
      case APK_DIGIT:
      case APK_SUFFIX_NO:
      case APK_REV: {
        uint64_t u = 0;  // Go int arithmetic: wraps like the reference on overflow
        while (i < n && is_adigit(s[i])) u = u * 10 + uint64_t(s[i++] - '0');
        v = int64_t(u);
        cls = kind == APK_DOZ ? APKC_DOZ : kind == APK_DIGIT ? APKC_DIGIT : kind == APK_REV ? APKC_REV : APKC_SUFNO;
        break;
      }
      case APK_LETTER:
        v = s[i++];
        cls = APKC_LETTER;
        break;
      case APK_SUFFIX: {
        // pre: alpha beta pre rc -> -4..-1 ; post: cvs svn git hg p -> 0..4
        if (apk_prefix(s, n, i, "alpha", 5)) { v = -4; i += 5; }
        else if (apk_prefix(s, n, i, "beta", 4)) { v = -3; i += 4; }
        else if (apk_prefix(s, n, i, "pre", 3)) { v = -2; i += 3; }
        else if (apk_prefix(s, n, i, "rc", 2)) { v = -1; i += 2; }
        else if (apk_prefix(s, n, i, "cvs", 3)) { v = 0; i += 3; }
        else if (apk_prefix(s, n, i, "svn", 3)) { v = 1; i += 3; }
        else if (apk_prefix(s, n, i, "git", 3)) { v = 2; i += 3; }
        else if (apk_prefix(s, n, i, "hg", 2)) { v = 3; i += 2; }
        else if (apk_prefix(s, n, i, "p", 1)) { v = 4; i += 1; }
        else return false;
        cls = v < 0 ? APKC_SUFPRE : APKC_SUFPOST;
        break;
      }
      default:
        return false;
    }
    o.put(cls);
    put_sint(v, o);
    if (i >= n) kind = APK_END;
    else if (nt != APK_INVALID) kind = nt;
    else kind = apk_next_kind(kind, s, n, i);
    if (kind == APK_INVALID) return false;
    if (kind == APK_END) {
      o.put(APKC_END);
      return true;
    }
  }
}

// ------------------------------------------------------------------------------- rpm -----
// github.com/knqyf263/go-rpm-version (reference go.mod:63).  Never fails.  Epoch =
// strconv.Atoi before the first ':' (0 when absent or unparsable); release after the
// FIRST '-' (pinned by redhat_test.go "advisories have different arches").  rpmvercmp
// segments ([a-zA-Z]+ | [0-9]+ | ~; other bytes separate): '~' < end-of-string < letters <
// numbers; letters bytewise, numbers by value.  Key = put_sint(epoch) PART(version)
// PART(release), PART = segments then END:
//   '~' = 0x01, END = 0x02, letters = 0x03 + the letters (0x41..0x7A, above every class
//   byte, so a shorter run sorts first), number = 0x04 + digit count (leading zeros
//   dropped; 1 byte < 0xFA, else 0xFA + 2 bytes) + digits packed two per byte.
enum : uint8_t { RPM_TILDE = 0x01, RPM_END = 0x02, RPM_ALPHA = 0x03, RPM_NUM = 0x04 };

TVM_HD bool rpm_alpha(uint8_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

template <class Sink>
TVM_HD void rpm_part(const uint8_t* s, uint32_t n, Sink& o) {
  uint32_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c == '~') {
      o.put(RPM_TILDE);
      i++;
    } else if (rpm_alpha(c)) {
      o.put(RPM_ALPHA);
      while (i < n && rpm_alpha(s[i])) o.put(s[i++]);
    } else if (is_adigit(c)) {
      while (i < n && s[i] == '0') i++;
      uint32_t b = i;
      while (i < n && is_adigit(s[i])) i++;
      const uint32_t len = i - b;
      o.put(RPM_NUM);
      if (len < 0xFA) {
        o.put(uint8_t(len));
      } else {
        o.put(0xFA);
        o.put(uint8_t(len >> 8));
        o.put(uint8_t(len));
      }
      for (uint32_t j = b; j < i; j += 2) {
        const uint8_t hi = uint8_t(s[j] - '0'), lo = j + 1 < i ? uint8_t(s[j + 1] - '0') : 0;
        o.put(uint8_t((hi << 4) | lo));
      }
    } else {
      i++;
    }
  }
  o.put(RPM_END);
}

template <class Sink>
TVM_HD bool rpm_encode(const uint8_t* s, uint32_t n, Sink& o) {
  int64_t epoch = 0;
  uint32_t colon = n;
  for (uint32_t i = 0; i < n; i++)
    if (s[i] == ':') { colon = i; break; }
  const uint8_t* r = s;
  uint32_t rn = n;
  if (colon < n) {
    uint32_t i = 0;
    bool neg = false, ok = colon > 0;
    if (colon > 0 && (s[0] == '+' || s[0] == '-')) {
      neg = s[0] == '-';
      i = 1;
      ok = colon > 1;
    }
    uint64_t e = 0;
    for (; ok && i < colon; i++) {
      if (!is_adigit(s[i])) { ok = false; break; }
      const uint64_t d = uint64_t(s[i] - '0');
      if (e > (uint64_t(INT64_MAX) - d) / 10) { ok = false; break; }
      e = e * 10 + d;
    }
    epoch = ok ? (neg ? -int64_t(e) : int64_t(e)) : 0;
    r = s + colon + 1;
    rn = n - colon - 1;
  }
  uint32_t dash = rn;
  for (uint32_t i = 0; i < rn; i++)
    if (r[i] == '-') { dash = i; break; }
  put_sint(epoch, o);
  rpm_part(r, dash, o);
  if (dash < rn) rpm_part(r + dash + 1, rn - dash - 1, o);
  else rpm_part(r, 0, o);
  return true;
}

// Upper bound on the key length of a version string of n bytes (every grammar fits in
// key_bound_any).
TVM_HD uint32_t key_bound(uint8_t cmp, uint32_t n) {
  switch (cmp) {
    case CMP_APK: return 4 * n + 16;
    case CMP_RPM: return 3 * n + 16;
    case CMP_DEB: return 2 * n + 16;
    case CMP_GEM: return 5 * n + 16;
    default: return 3 * n + 24;  // library grammars (libver.h)
  }
}

TVM_HD uint32_t key_bound_any(uint32_t n) { return 5 * n + 24; }

// ---------------------------------------------------------------------------- sinks -----
// Device sink: packs bytes into little-endian 64-bit words and stores whole words.
struct WordSink {
  uint64_t* dst;
  uint64_t acc = 0;
  uint32_t n = 0;
  TVM_HD explicit WordSink(uint64_t* d) : dst(d) {}
  TVM_HD void put(uint8_t b) {
    acc |= uint64_t(b) << (8 * (n & 7));
    if ((++n & 7) == 0) {
      dst[(n >> 3) - 1] = acc;
      acc = 0;
    }
  }
  TVM_HD void flush() {
    if (n & 7) dst[n >> 3] = acc;
  }
};

// Device sink with a capacity: stores the key while it fits in cap_bytes (whole words)
// and counts every byte, so one pass both encodes a typical key and sizes a long one.
struct CapWordSink {
  uint64_t* dst;
  uint32_t cap;
  uint64_t acc = 0;
  uint32_t n = 0;
  TVM_HD CapWordSink(uint64_t* d, uint32_t cap_bytes) : dst(d), cap(cap_bytes) {}
  TVM_HD void put(uint8_t b) {
    if (n < cap) {
      acc |= uint64_t(b) << (8 * (n & 7));
      if ((n & 7) == 7) {
        dst[n >> 3] = acc;
        acc = 0;
      }
    }
    n++;
  }
  TVM_HD void flush() {
    if (n < cap && (n & 7)) dst[n >> 3] = acc;
  }
};

// Counting sink (length only).
struct CountSink {
  uint32_t n = 0;
  TVM_HD void put(uint8_t) { n++; }
};

// Dispatch by grammar.
template <class Sink>
TVM_HD bool encode_version(uint8_t cmp, const uint8_t* s, uint32_t n, Sink& o) {
  switch (cmp) {
    case CMP_DEB: return deb_encode(s, n, o);
    case CMP_APK: return apk_encode(s, n, o);
    case CMP_RPM: return rpm_encode(s, n, o);
    default: return false;
  }
}

}  // namespace tvm
