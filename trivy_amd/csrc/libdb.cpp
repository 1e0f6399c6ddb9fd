// Load-time compilation of library advisories into interval rows (see libdb.h).
//
// Each grammar's constraint parser mirrors the module the reference calls (and the
// oracle's restatement in oracle/library.py); each primitive becomes an interval of the
// grammar's key order (libver.h), combined with set algebra per version class.
#include "libdb.h"

#include <algorithm>
#include <cstring>

#include "libver.h"

namespace tvm {
namespace {

// ------------------------------------------------------------------ key helpers --------
struct StrSink {
  std::string* s;
  void put(uint8_t b) { s->push_back(char(b)); }
};

const uint8_t* U(const std::string& s) { return reinterpret_cast<const uint8_t*>(s.data()); }

int kcmp(const std::string& a, const std::string& b) {
  const int c = std::memcmp(a.data(), b.data(), std::min(a.size(), b.size()));
  if (c) return c < 0 ? -1 : 1;
  return (a.size() > b.size()) - (a.size() < b.size());
}

// The smallest key greater than every key that starts with p ("" when none exists).
bool key_succ(std::string p, std::string& out) {
  while (!p.empty() && uint8_t(p.back()) == 0xFF) p.pop_back();
  if (p.empty()) return false;
  p.back() = char(uint8_t(p.back()) + 1);
  out = p;
  return true;
}

// ------------------------------------------------------------------ interval sets -------
// lower bounds: -inf < [k < (k ; upper bounds: k) < k] < +inf
int cmp_lo(const KBound& a, const KBound& b) {
  if (a.inf || b.inf) return (b.inf - a.inf);
  const int c = kcmp(a.k, b.k);
  if (c) return c;
  return (a.incl == b.incl) ? 0 : (a.incl ? -1 : 1);
}
int cmp_hi(const KBound& a, const KBound& b) {
  if (a.inf || b.inf) return (a.inf - b.inf);
  const int c = kcmp(a.k, b.k);
  if (c) return c;
  return (a.incl == b.incl) ? 0 : (a.incl ? 1 : -1);
}
bool nonempty(const KInterval& v) {
  if (v.lo.inf || v.hi.inf) return true;
  const int c = kcmp(v.lo.k, v.hi.k);
  return c < 0 || (c == 0 && v.lo.incl && v.hi.incl);
}
// does interval a's upper end reach (overlap or touch) b's lower end?
bool reaches(const KBound& hi, const KBound& lo) {
  if (hi.inf || lo.inf) return true;
  const int c = kcmp(lo.k, hi.k);
  return c < 0 || (c == 0 && (hi.incl || lo.incl));
}

KSet normalize(KSet s) {
  s.erase(std::remove_if(s.begin(), s.end(), [](const KInterval& v) { return !nonempty(v); }), s.end());
  std::sort(s.begin(), s.end(), [](const KInterval& a, const KInterval& b) { return cmp_lo(a.lo, b.lo) < 0; });
  KSet out;
  for (const KInterval& v : s) {
    if (!out.empty() && reaches(out.back().hi, v.lo)) {
      if (cmp_hi(v.hi, out.back().hi) > 0) out.back().hi = v.hi;
    } else {
      out.push_back(v);
    }
  }
  return out;
}

KSet all_set() { return {KInterval{}}; }
KSet unite(const KSet& a, const KSet& b) {
  KSet s = a;
  s.insert(s.end(), b.begin(), b.end());
  return normalize(std::move(s));
}
KSet isect(const KSet& a, const KSet& b) {
  KSet s;
  for (const KInterval& x : a)
    for (const KInterval& y : b) {
      KInterval v;
      v.lo = cmp_lo(x.lo, y.lo) >= 0 ? x.lo : y.lo;
      v.hi = cmp_hi(x.hi, y.hi) <= 0 ? x.hi : y.hi;
      if (nonempty(v)) s.push_back(v);
    }
  return normalize(std::move(s));
}
KSet complement(const KSet& a) {
  KSet out;
  KBound lo;  // -inf
  for (const KInterval& v : a) {
    if (!v.lo.inf) {
      KInterval g;
      g.lo = lo;
      g.hi = KBound{false, v.lo.k, !v.lo.incl};
      if (nonempty(g)) out.push_back(g);
    }
    if (v.hi.inf) return out;
    lo = KBound{false, v.hi.k, !v.hi.incl};
  }
  KInterval g;
  g.lo = lo;
  out.push_back(g);
  return out;
}

KSet half(bool upper, const std::string& k, bool incl) {
  KInterval v;
  (upper ? v.hi : v.lo) = KBound{false, k, incl};
  return {v};
}
KSet lt(const std::string& k) { return half(true, k, false); }
KSet le(const std::string& k) { return half(true, k, true); }
KSet gt(const std::string& k) { return half(false, k, false); }
KSet ge(const std::string& k) { return half(false, k, true); }
KSet eq(const std::string& k) { return {KInterval{KBound{false, k, true}, KBound{false, k, true}}}; }
KSet range(const std::string& lo, bool lo_incl, const std::string& hi, bool hi_incl) {
  return normalize({KInterval{KBound{false, lo, lo_incl}, KBound{false, hi, hi_incl}}});
}
// every key starting with prefix p
KSet prefix_set(const std::string& p) {
  std::string s;
  if (!key_succ(p, s)) return ge(p);
  return range(p, true, s, false);
}

bool contains(const KSet& s, const std::string& k) {
  for (const KInterval& v : s) {
    const bool lo_ok = v.lo.inf || (v.lo.incl ? kcmp(k, v.lo.k) >= 0 : kcmp(k, v.lo.k) > 0);
    const bool hi_ok = v.hi.inf || (v.hi.incl ? kcmp(k, v.hi.k) <= 0 : kcmp(k, v.hi.k) < 0);
    if (lo_ok && hi_ok) return true;
  }
  return false;
}

using VS = std::vector<KSet>;  // one set per class
VS vs_all(int n) { return VS(size_t(n), all_set()); }
VS vs_none(int n) { return VS(size_t(n)); }
VS vs_same(int n, const KSet& s) { return VS(size_t(n), s); }
VS vs_and(const VS& a, const VS& b) {
  VS o(a.size());
  for (size_t c = 0; c < a.size(); c++) o[c] = isect(a[c], b[c]);
  return o;
}
VS vs_or(const VS& a, const VS& b) {
  VS o(a.size());
  for (size_t c = 0; c < a.size(); c++) o[c] = unite(a[c], b[c]);
  return o;
}
VS vs_not(const VS& a) {
  VS o(a.size());
  for (size_t c = 0; c < a.size(); c++) o[c] = complement(a[c]);
  return o;
}

// ------------------------------------------------------------------ text helpers --------
bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }
std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && is_ws(s[b])) b++;
  while (e > b && is_ws(s[e - 1])) e--;
  return s.substr(b, e - b);
}
std::vector<std::string> split(const std::string& s, const std::string& sep) {
  std::vector<std::string> out;
  size_t b = 0;
  for (;;) {
    const size_t e = s.find(sep, b);
    out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
    if (e == std::string::npos) return out;
    b = e + sep.size();
  }
}
bool dig(char c) { return c >= '0' && c <= '9'; }
bool alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
bool alnum(char c) { return dig(c) || alpha(c); }

// ================================================================= GENERIC / BITNAMI ====
// Version token of go-version's constraint regex (oracle _GEN_VER), matched greedily at i.
size_t gen_ver_len(const std::string& s, size_t i) {
  const size_t b = i;
  auto idents = [&](size_t& j) {  // [0-9A-Za-z-~]+(\.[0-9A-Za-z-~]+)*, greedy
    auto ic = [&](char c) { return alnum(c) || c == '-' || c == '~'; };
    size_t k = j;
    if (k >= s.size() || !ic(s[k])) return false;
    while (k < s.size() && ic(s[k])) k++;
    while (k + 1 < s.size() && s[k] == '.' && ic(s[k + 1])) {
      k++;
      while (k < s.size() && ic(s[k])) k++;
    }
    j = k;
    return true;
  };
  if (i < s.size() && s[i] == 'v') i++;
  if (i >= s.size() || !dig(s[i])) return 0;
  while (i < s.size() && dig(s[i])) i++;
  while (i + 1 < s.size() && s[i] == '.' && dig(s[i + 1])) {
    i++;
    while (i < s.size() && dig(s[i])) i++;
  }
  if (i < s.size() && s[i] == '-') {
    size_t j = i + 1;
    if (idents(j)) i = j;
    else if (idents(i)) {
    }
  } else if (i < s.size() && (alpha(s[i]) || s[i] == '~')) {
    size_t j = i;
    // [A-Za-z-~][0-9A-Za-z-~]*(\.[0-9A-Za-z-~]+)*
    if (idents(j)) i = j;
  }
  if (i < s.size() && s[i] == '+') {
    size_t j = i + 1;
    if (idents(j)) i = j;
  }
  return i - b;
}

const char* const kGenOps[] = {"~>", ">=", "=>", "<=", "=<", "!=", "==", ">", "<", "=", "~", "^", ""};

struct GenC {
  std::string op, ver;
};

bool gen_parse_alt(const std::string& alt, std::vector<GenC>& out) {
  size_t i = 0;
  const size_t n = alt.size();
  for (;;) {
    while (i < n && is_ws(alt[i])) i++;
    if (i >= n) return true;
    std::string op;
    size_t vl = 0, vb = 0;
    for (const char* o : kGenOps) {
      const size_t ol = std::strlen(o);
      if (alt.compare(i, ol, o) != 0) continue;
      size_t j = i + ol;
      while (j < n && is_ws(alt[j])) j++;
      vl = gen_ver_len(alt, j);
      if (vl) {
        op = o;
        vb = j;
        break;
      }
    }
    if (!vl) return false;
    out.push_back(GenC{op, alt.substr(vb, vl)});
    i = vb + vl;
    while (i < n && is_ws(alt[i])) i++;
    if (i < n && alt[i] == ',') i++;
  }
}

std::string gen_key(const std::string& v, bool bitnami, bool& ok) {
  std::string k;
  StrSink o{&k};
  ok = gen_encode(U(v), uint32_t(v.size()), bitnami, o);
  return k;
}

// Written release segments of a go-version token (values).
std::vector<uint64_t> gen_segs(const std::string& v) {
  std::vector<uint64_t> segs;
  size_t i = (!v.empty() && v[0] == 'v') ? 1 : 0;
  while (i < v.size() && dig(v[i])) {
    uint64_t x = 0;
    while (i < v.size() && dig(v[i])) x = x * 10 + uint64_t(v[i++] - '0');
    segs.push_back(x);
    if (i + 1 < v.size() && v[i] == '.' && dig(v[i + 1])) i++;
    else break;
  }
  return segs;
}

// keys < the smallest key whose (zero-padded) release is >= upper
KSet gen_below_release(std::vector<uint64_t> upper) {
  while (!upper.empty() && upper.back() == 0) upper.pop_back();
  std::string p;
  StrSink o{&p};
  for (uint64_t x : upper) put_uvar(x, o);
  p.push_back(0x01);
  return lt(p);
}

bool gen_compile(const std::string& constraint, bool bitnami, KSet& out) {
  out.clear();
  for (const std::string& alt : split(constraint, "||")) {
    std::vector<GenC> cs;
    if (!gen_parse_alt(alt, cs)) return false;
    KSet acc = all_set();
    for (const GenC& c : cs) {
      bool ok;
      const std::string k = gen_key(c.ver, bitnami, ok);
      if (!ok) return false;
      KSet p;
      const std::string& op = c.op;
      if (op.empty() || op == "=" || op == "==") p = eq(k);
      else if (op == "!=") p = complement(eq(k));
      else if (op == ">") p = gt(k);
      else if (op == "<") p = lt(k);
      else if (op == ">=" || op == "=>") p = ge(k);
      else if (op == "<=" || op == "=<") p = le(k);
      else {
        std::vector<uint64_t> segs = gen_segs(c.ver);
        const size_t n = segs.size();
        size_t keep;
        if (op == "~>") keep = std::max<size_t>(1, n - 1);
        else if (op == "~") keep = n >= 2 ? 2 : 1;
        else {  // ^
          size_t i = 0;
          while (i + 1 < n && segs[i] == 0) i++;
          keep = i + 1;
        }
        segs.resize(keep);
        segs.back()++;
        p = isect(ge(k), gen_below_release(segs));
      }
      acc = isect(acc, p);
    }
    out = unite(out, acc);
  }
  return true;
}

// ======================================================================== NPM ==========
struct NpmV {
  uint64_t t[3];
  std::vector<std::string> pre;
};

std::string npm_key(const NpmV& v) {
  std::string k;
  StrSink o{&k};
  for (uint64_t x : v.t) put_uvar(x, o);
  if (v.pre.empty()) {
    o.put(0x03);
  } else {
    o.put(0x02);
    std::string joined;
    for (size_t i = 0; i < v.pre.size(); i++) joined += (i ? "." : "") + v.pre[i];
    put_idents(U(joined), 0, uint32_t(joined.size()), o);
  }
  return k;
}
std::string npm_tuple_prefix(const uint64_t t[3]) {
  std::string k;
  StrSink o{&k};
  for (int i = 0; i < 3; i++) put_uvar(t[i], o);
  return k;
}

bool npm_u64(const std::string& s, uint64_t& v) {
  uint8_t tmp[1];
  (void)tmp;
  return lv_u64(U(s), 0, uint32_t(s.size()), v);
}

// _PARTIAL of oracle/library.py: [v=]*(XR)(.(XR)(.(XR)(-?IDENTS)?(+IDENTS)?)?)?
bool npm_partial(const std::string& s, std::vector<uint64_t>& nums, std::vector<std::string>& pre) {
  nums.clear();
  pre.clear();
  size_t i = 0;
  while (i < s.size() && (s[i] == 'v' || s[i] == '=')) i++;
  bool stop = false;
  for (int k = 0; k < 3; k++) {
    if (k) {
      if (i >= s.size()) break;
      if (s[i] != '.') return false;
      i++;
    }
    if (i < s.size() && (s[i] == 'x' || s[i] == 'X' || s[i] == '*')) {
      i++;
      stop = true;
      continue;
    }
    const size_t b = i;
    while (i < s.size() && dig(s[i])) i++;
    if (i == b) return false;
    uint64_t v;
    if (!lv_u64(U(s), uint32_t(b), uint32_t(i), v)) return false;
    if (!stop) nums.push_back(v);
  }
  if (i < s.size()) {
    // only after a third component: (-?IDENTS)?(+IDENTS)?
    size_t dots = 0;
    for (size_t k = 0; k < i; k++) dots += s[k] == '.';
    if (dots < 2) return false;
    const size_t plus = s.find('+', i);
    const size_t pe = plus == std::string::npos ? s.size() : plus;
    if (plus != std::string::npos && !lv_idents(U(s), uint32_t(plus + 1), uint32_t(s.size()), npm_ident_char))
      return false;
    if (i < pe) {
      size_t pb;
      if (s[i] == '-' && lv_idents(U(s), uint32_t(i + 1), uint32_t(pe), npm_ident_char)) pb = i + 1;
      else if (lv_idents(U(s), uint32_t(i), uint32_t(pe), npm_ident_char)) pb = i;
      else return false;
      if (nums.size() == 3) pre = split(s.substr(pb, pe - pb), ".");
    }
  }
  return true;
}

NpmV npm_make(std::vector<uint64_t> t, std::vector<std::string> pre) {
  NpmV v;
  for (int i = 0; i < 3; i++) v.t[i] = i < int(t.size()) ? t[size_t(i)] : 0;
  v.pre = std::move(pre);
  return v;
}

struct NpmC {
  std::string op;  // = < <= > >=
  NpmV v;
};

bool npm_desugar(const std::string& op, const std::vector<uint64_t>& nums, const std::vector<std::string>& pre,
                 std::vector<NpmC>& out) {
  const size_t n = nums.size();
  const NpmV zero = npm_make({0, 0, 0}, {});
  if (op == "~" || op == "~>" || op == "^") {
    if (n == 0) {
      out.push_back({">=", zero});
      return true;
    }
    std::vector<uint64_t> up;
    if (op == "^") {
      if (nums[0] != 0 || n == 1) up = {nums[0] + 1, 0, 0};
      else if (n == 2 || nums[1] != 0) up = {0, nums[1] + 1, 0};
      else up = {0, 0, nums[2] + 1};
    } else {
      up = n == 1 ? std::vector<uint64_t>{nums[0] + 1, 0, 0} : std::vector<uint64_t>{nums[0], nums[1] + 1, 0};
    }
    out.push_back({">=", npm_make(nums, n == 3 ? pre : std::vector<std::string>{})});
    out.push_back({"<", npm_make(up, {"0"})});
    return true;
  }
  if (n == 0) {
    if (op.empty() || op == "=" || op == ">=" || op == "<=") out.push_back({">=", zero});
    else out.push_back({"<", npm_make({0, 0, 0}, {"0"})});
    return true;
  }
  if (n == 3) {
    out.push_back({op.empty() ? "=" : op, npm_make(nums, pre)});
    return true;
  }
  std::vector<uint64_t> up = nums;
  up.back()++;
  if (op.empty() || op == "=") {
    out.push_back({">=", npm_make(nums, {})});
    out.push_back({"<", npm_make(up, {"0"})});
  } else if (op == ">") out.push_back({">=", npm_make(up, {})});
  else if (op == ">=") out.push_back({">=", npm_make(nums, {})});
  else if (op == "<") out.push_back({"<", npm_make(nums, {"0"})});
  else if (op == "<=") out.push_back({"<", npm_make(up, {"0"})});
  else return false;
  return true;
}

bool npm_set(std::string s, std::vector<NpmC>& out) {
  for (char& c : s)
    if (c == ',') c = ' ';
  s = trim(s);
  // hyphen range: ^(\S+)\s+-\s+(\S+)$
  {
    size_t a = 0;
    while (a < s.size() && !is_ws(s[a])) a++;
    size_t b = a;
    while (b < s.size() && is_ws(s[b])) b++;
    if (a > 0 && b > a && b < s.size() && s[b] == '-' && b + 1 < s.size() && is_ws(s[b + 1])) {
      size_t c = b + 1;
      while (c < s.size() && is_ws(s[c])) c++;
      size_t d = c;
      while (d < s.size() && !is_ws(s[d])) d++;
      if (c < s.size() && d == s.size()) {
        std::vector<uint64_t> lo, hi;
        std::vector<std::string> lp, hp;
        if (!npm_partial(s.substr(0, a), lo, lp) || !npm_partial(s.substr(c), hi, hp)) return false;
        if (!lo.empty()) out.push_back({">=", npm_make(lo, lo.size() == 3 ? lp : std::vector<std::string>{})});
        if (hi.size() == 3) out.push_back({"<=", npm_make(hi, hp)});
        else if (!hi.empty()) {
          std::vector<uint64_t> up = hi;
          up.back()++;
          out.push_back({"<", npm_make(up, {"0"})});
        }
        if (out.empty()) out.push_back({">=", npm_make({0, 0, 0}, {})});
        return true;
      }
    }
  }
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && is_ws(s[i])) i++;
    if (i >= s.size()) break;
    std::string op;
    for (const char* o : {"<=", ">=", "<", ">", "=", "~>", "~", "^"}) {
      const size_t l = std::strlen(o);
      if (s.compare(i, l, o) == 0) {
        op = o;
        break;
      }
    }
    size_t j = i + op.size();
    while (j < s.size() && is_ws(s[j])) j++;
    const size_t vb = j;
    while (j < s.size() && !is_ws(s[j]) && !std::strchr("<>=~^,", s[j])) j++;
    if (j == vb) return false;
    std::vector<uint64_t> nums;
    std::vector<std::string> pre;
    if (!npm_partial(s.substr(vb, j - vb), nums, pre)) return false;
    if (!npm_desugar(op, nums, pre, out)) return false;
    i = j;
  }
  if (out.empty()) out.push_back({">=", npm_make({0, 0, 0}, {})});
  return true;
}

KSet npm_prim(const NpmC& c) {
  const std::string k = npm_key(c.v);
  if (c.op == "=") return eq(k);
  if (c.op == "<") return lt(k);
  if (c.op == "<=") return le(k);
  if (c.op == ">") return gt(k);
  return ge(k);
}

bool npm_compile(const std::string& constraint, VS& out) {
  out = vs_none(2);
  for (const std::string& alt : split(constraint, "||")) {
    std::vector<NpmC> cs;
    if (!npm_set(alt, cs)) return false;
    KSet rel = all_set();
    for (const NpmC& c : cs) rel = isect(rel, npm_prim(c));
    KSet pre;  // pre-releases: only tuples a pre-release comparator of the set names
    for (const NpmC& c : cs) {
      if (c.v.pre.empty()) continue;
      const std::string t = npm_tuple_prefix(c.v.t);
      pre = unite(pre, isect(rel, range(t + char(0x02), true, t + char(0x03), false)));
    }
    out[0] = unite(out[0], rel);
    out[1] = unite(out[1], pre);
  }
  return true;
}

// ===================================================================== PEP 440 =========
bool pep_parts(const std::string& v, PepParts& p) { return pep_parse(U(v), uint32_t(v.size()), p); }
std::string pep_key(const std::string& v, const PepParts& p, int upto) {
  std::string k;
  StrSink o{&k};
  pep_emit(U(v), p, upto, o);
  return k;
}

// "==V.*": same epoch, zero-padded release starting with V's release.
bool pep_prefix(const std::string& spec, KSet& out) {
  PepParts p;
  if (!pep_parts(spec, p)) return false;
  std::vector<uint64_t> rel;
  uint32_t i = p.rel_b;
  const uint8_t* s = U(spec);
  while (i < p.rel_e) {
    uint64_t x;
    pep_num(s, p.rel_e, i, x);
    rel.push_back(x);
    i++;
  }
  size_t j = rel.size();
  while (j > 0 && rel[j - 1] == 0) j--;
  std::string pj, pk;
  StrSink oj{&pj}, ok{&pk};
  put_uvar(p.epoch, oj);
  put_uvar(p.epoch, ok);
  for (size_t k = 0; k < j; k++) put_uvar(rel[k], oj);
  for (size_t k = 0; k < rel.size(); k++) put_uvar(rel[k], ok);
  out = unite(range(pj + char(0x01), true, pj + char(0x02), false), prefix_set(pk));
  return true;
}

bool pep_spec(const std::string& op, const std::string& spec, VS& out) {
  const int N = 8;
  if (spec == "*") {
    out = vs_all(N);
    return true;
  }
  if (op == "~=") {
    PepParts p;
    if (!pep_parts(spec, p)) return false;
    std::vector<std::string> segs = split(spec.substr(p.rel_b, p.rel_e - p.rel_b), ".");
    if (segs.size() < 2) return false;
    std::string prefix;
    for (size_t k = 0; k + 1 < segs.size(); k++) prefix += (k ? "." : "") + segs[k];
    if (p.epoch) prefix = std::to_string(p.epoch) + "!" + prefix;
    VS ge_v;
    KSet pre;
    if (!pep_spec(">=", spec, ge_v) || !pep_prefix(prefix, pre)) return false;
    out = vs_and(ge_v, vs_same(N, pre));
    return true;
  }
  if ((op == "==" || op == "!=") && spec.size() >= 2 && spec.compare(spec.size() - 2, 2, ".*") == 0) {
    KSet s;
    if (!pep_prefix(spec.substr(0, spec.size() - 2), s)) return false;
    out = vs_same(N, op == "==" ? s : complement(s));
    return true;
  }
  PepParts p;
  if (!pep_parts(spec, p)) return false;
  const std::string full = pep_key(spec, p, 2), pub = pep_key(spec, p, 1), base = pep_key(spec, p, 0);
  const bool local = p.loc_e > p.loc_b, spec_pre = p.pre_l >= 0 || p.dev, spec_post = p.post;
  if (op == "==" || op == "!=" || op == "===") {
    // UNPINNED: "===" (arbitrary string equality) approximated by version equality
    const KSet s = (local || op == "===") ? eq(full) : range(pub + char(0x01), true, pub + char(0x03), false);
    out = vs_same(N, op == "!=" ? complement(s) : s);
    return true;
  }
  if (op == "<=") {
    out = vs_same(N, lt(pub + char(0x03)));
    return true;
  }
  if (op == ">=") {
    out = vs_same(N, ge(pub + char(0x01)));
    return true;
  }
  out = VS(N);
  for (int c = 0; c < N; c++) {
    if (op == "<") {
      // packaging _compare_less_than: no pre-release of the spec's own base version
      out[size_t(c)] = ((c & PEP_CLS_PRE) && !spec_pre) ? lt(base) : lt(full);
    } else if (op == ">") {
      // _compare_greater_than: no post-release (unless the spec is one) and no local
      // version of the spec's own base version
      out[size_t(c)] = ((c & PEP_CLS_LOCAL) || ((c & PEP_CLS_POST) && !spec_post)) ? ge(base + char(0x04)) : gt(full);
    } else {
      return false;
    }
  }
  return true;
}

bool pep_compile(const std::string& constraint, VS& out) {
  out = vs_none(8);
  for (const std::string& alt0 : split(constraint, "||")) {
    const std::string a = trim(alt0);
    VS acc = vs_all(8);
    size_t n_specs = 0;
    if (a == "*") {
      n_specs = 1;
    } else {
      size_t i = 0;
      while (i < a.size()) {
        if (a[i] == ',' || a[i] == ' ') {
          i++;
          continue;
        }
        // \s*(~=|===|==|!=|<=|>=|<|>)?\s*([^\s,<>=!~]+)\s*
        size_t j = i;
        while (j < a.size() && is_ws(a[j])) j++;
        std::string op;
        for (const char* o : {"~=", "===", "==", "!=", "<=", ">=", "<", ">"}) {
          const size_t l = std::strlen(o);
          if (a.compare(j, l, o) == 0) {
            op = o;
            break;
          }
        }
        j += op.size();
        while (j < a.size() && is_ws(a[j])) j++;
        const size_t vb = j;
        while (j < a.size() && !is_ws(a[j]) && !std::strchr(",<>=!~", a[j])) j++;
        if (j == vb) return false;
        const std::string spec = a.substr(vb, j - vb);
        if (spec.size() < 2 || spec.compare(spec.size() - 2, 2, ".*") != 0) {
          PepParts p;
          if (!pep_parts(spec, p)) return false;
        }
        VS s;
        if (!pep_spec(op.empty() ? "==" : op, spec, s)) return false;
        acc = vs_and(acc, s);
        n_specs++;
        while (j < a.size() && is_ws(a[j])) j++;
        i = j;
      }
    }
    if (!n_specs) return false;
    out = vs_or(out, acc);
  }
  return true;
}

// ======================================================================= MAVEN =========
std::string mvn_key(const std::string& v, bool& ok) {
  std::string k;
  StrSink o{&k};
  ok = mvn_encode(U(v), uint32_t(v.size()), o);
  return k;
}

bool mvn_ranges(const std::string& spec, KSet& out) {
  out.clear();
  const std::string s = trim(spec);
  size_t pos = 0;
  while (pos < s.size()) {
    if (s[pos] == ',' || s[pos] == ' ') {
      pos++;
      continue;
    }
    if (s[pos] != '[' && s[pos] != '(') return false;
    size_t e1 = s.find(']', pos), e2 = s.find(')', pos);
    const size_t end = std::min(e1, e2);
    if (end == std::string::npos) return false;
    const std::string body = s.substr(pos + 1, end - pos - 1);
    const bool lo_incl = s[pos] == '[', hi_incl = s[end] == ']';
    const size_t comma = body.find(',');
    KInterval iv;
    if (comma != std::string::npos) {
      const std::string lo = trim(body.substr(0, comma)), hi = trim(body.substr(comma + 1));
      bool ok = true;
      if (!lo.empty()) iv.lo = KBound{false, mvn_key(lo, ok), lo_incl};
      if (!ok) return false;
      if (!hi.empty()) iv.hi = KBound{false, mvn_key(hi, ok), hi_incl};
      if (!ok) return false;
    } else {
      if (!(lo_incl && hi_incl) || trim(body).empty()) return false;
      bool ok;
      const std::string k = mvn_key(body, ok);
      if (!ok) return false;
      iv.lo = iv.hi = KBound{false, k, true};
    }
    out = unite(out, normalize({iv}));
    pos = end + 1;
  }
  return true;
}

bool mvn_compile(const std::string& constraint, KSet& out) {
  out.clear();
  for (const std::string& alt0 : split(constraint, "||")) {
    const std::string a = trim(alt0);
    if (!a.empty() && (a[0] == '[' || a[0] == '(')) {
      KSet r;
      if (!mvn_ranges(a, r)) return false;
      out = unite(out, r);
      continue;
    }
    KSet acc = all_set();
    size_t i = 0, n_cs = 0;
    while (i < a.size()) {
      if (a[i] == ',' || a[i] == ' ' || a[i] == '\t') {
        i++;
        continue;
      }
      std::string op;
      for (const char* o : {">=", "<=", "!=", "==", "=", ">", "<"}) {
        const size_t l = std::strlen(o);
        if (a.compare(i, l, o) == 0) {
          op = o;
          break;
        }
      }
      size_t j = i + op.size();
      while (j < a.size() && is_ws(a[j])) j++;
      const size_t vb = j;
      while (j < a.size() && !is_ws(a[j]) && !std::strchr("<>=!,", a[j])) j++;
      if (j == vb) return false;
      bool ok;
      const std::string k = mvn_key(a.substr(vb, j - vb), ok);
      if (!ok) return false;
      KSet p;
      if (op.empty() || op == "=" || op == "==") p = eq(k);
      else if (op == "!=") p = complement(eq(k));
      else if (op == ">") p = gt(k);
      else if (op == "<") p = lt(k);
      else if (op == ">=") p = ge(k);
      else p = le(k);
      acc = isect(acc, p);
      n_cs++;
      i = j;
    }
    if (!n_cs) return false;
    out = unite(out, acc);
  }
  return true;
}

// The same constraint grammar as an IsVulnerable program for pairwise evaluation (libver.h
// mvn_program_eval): alternatives = groups, a group = AND of (op, bound text) terms; a
// Maven range list "[a,b),(c,]" gives one group per range.
using MvnGroups = std::vector<std::vector<std::pair<uint32_t, std::string>>>;

static bool mvn_text_ok(const std::string& v) {
  bool ok = false;
  (void)mvn_key(v, ok);
  return ok;
}

bool mvn_groups(const std::string& constraint, MvnGroups& out) {
  for (const std::string& alt0 : split(constraint, "||")) {
    const std::string a = trim(alt0);
    if (!a.empty() && (a[0] == '[' || a[0] == '(')) {
      size_t pos = 0;
      while (pos < a.size()) {
        if (a[pos] == ',' || a[pos] == ' ') {
          pos++;
          continue;
        }
        if (a[pos] != '[' && a[pos] != '(') return false;
        const size_t e1 = a.find(']', pos), e2 = a.find(')', pos), end = std::min(e1, e2);
        if (end == std::string::npos) return false;
        const std::string body = a.substr(pos + 1, end - pos - 1);
        const bool lo_incl = a[pos] == '[', hi_incl = a[end] == ']';
        const size_t comma = body.find(',');
        std::vector<std::pair<uint32_t, std::string>> g;
        if (comma != std::string::npos) {
          const std::string lo = trim(body.substr(0, comma)), hi = trim(body.substr(comma + 1));
          if (!lo.empty()) {
            if (!mvn_text_ok(lo)) return false;
            g.push_back({lo_incl ? MVO_GE : MVO_GT, lo});
          }
          if (!hi.empty()) {
            if (!mvn_text_ok(hi)) return false;
            g.push_back({hi_incl ? MVO_LE : MVO_LT, hi});
          }
        } else {
          const std::string v = trim(body);
          if (!(lo_incl && hi_incl) || v.empty() || !mvn_text_ok(v)) return false;
          g.push_back({MVO_EQ, v});
        }
        out.push_back(std::move(g));
        pos = end + 1;
      }
      continue;
    }
    std::vector<std::pair<uint32_t, std::string>> g;
    size_t i = 0;
    while (i < a.size()) {
      if (a[i] == ',' || a[i] == ' ' || a[i] == '\t') {
        i++;
        continue;
      }
      std::string op;
      for (const char* o : {">=", "<=", "!=", "==", "=", ">", "<"}) {
        const size_t l = std::strlen(o);
        if (a.compare(i, l, o) == 0) {
          op = o;
          break;
        }
      }
      size_t j = i + op.size();
      while (j < a.size() && is_ws(a[j])) j++;
      const size_t vb = j;
      while (j < a.size() && !is_ws(a[j]) && !std::strchr("<>=!,", a[j])) j++;
      if (j == vb) return false;
      const std::string v = a.substr(vb, j - vb);
      if (!mvn_text_ok(v)) return false;
      const uint32_t code = op.empty() || op == "=" || op == "==" ? MVO_EQ
                            : op == "!="                          ? MVO_NE
                            : op == ">"                           ? MVO_GT
                            : op == "<"                           ? MVO_LT
                            : op == ">="                          ? MVO_GE
                                                                  : MVO_LE;
      g.push_back({code, v});
      i = j;
    }
    if (g.empty()) return false;
    out.push_back(std::move(g));
  }
  return true;
}

// ==================================================================== RUBYGEMS =========
bool gem_compile(const std::string& constraint, KSet& out) {
  out.clear();
  for (const std::string& alt : split(constraint, "||")) {
    KSet acc = all_set();
    for (const std::string& part : split(alt, ",")) {
      // ^\s*(=|!=|>=|<=|>|<|~>)?\s*(\S.*?)\s*$
      const std::string p = trim(part);
      std::string op;
      for (const char* o : {"=", "!=", ">=", "<=", ">", "<", "~>"}) {
        const size_t l = std::strlen(o);
        if (p.compare(0, l, o) == 0 && l > op.size()) op = o;
      }
      // Python alternation order: "=" then "!=" ... - "=" never prefixes the others except
      // itself, so the longest listed operator that matches is the regex's choice
      const std::string ver = trim(p.substr(op.size()));
      if (ver.empty()) return false;
      std::string k;
      StrSink o{&k};
      GemSeg seg[kGemMaxSeg];
      int ns;
      if (!gem_parse(U(ver), uint32_t(ver.size()), seg, ns)) return false;
      gem_canonical(seg, ns);
      gem_emit(U(ver), seg, ns, o);
      KSet s;
      if (op.empty() || op == "=") s = eq(k);
      else if (op == "!=") s = complement(eq(k));
      else if (op == ">") s = gt(k);
      else if (op == "<") s = lt(k);
      else if (op == ">=") s = ge(k);
      else if (op == "<=") s = le(k);
      else {  // "~>": v >= r and v.release < r.bump
        // bump: the raw (non-canonical) segments up to the first string, last one dropped
        // when there are several, then the new last one incremented
        std::vector<std::string> num;
        {
          GemSeg raw[kGemMaxSeg];
          int nr;
          gem_parse(U(ver), uint32_t(ver.size()), raw, nr);
          for (int i = 0; i < nr && !raw[i].str; i++) num.push_back(ver.substr(raw[i].b, raw[i].e - raw[i].b));
        }
        if (num.size() > 1) num.pop_back();
        // increment the last numeric segment (decimal string)
        std::string& last = num.back();
        int i = int(last.size()) - 1;
        while (i >= 0 && last[size_t(i)] == '9') last[size_t(i--)] = '0';
        if (i < 0) last.insert(last.begin(), '1');
        else last[size_t(i)]++;
        std::string b;
        for (size_t j = 0; j < num.size(); j++) b += (j ? "." : "") + num[j];
        std::string bk;
        StrSink ob{&bk};
        GemSeg bs[kGemMaxSeg];
        int nb;
        gem_parse(U(b), uint32_t(b.size()), bs, nb);
        gem_canonical(bs, nb);
        gem_emit(U(b), bs, nb, ob);
        bk.pop_back();          // drop the end marker: every version whose release starts here
        bk.push_back(0x01);     // ... and continues with anything is >= bump
        s = isect(ge(k), lt(bk));
      }
      acc = isect(acc, s);
    }
    out = unite(out, acc);
  }
  return true;
}

}  // namespace

int lib_classes(uint8_t cmp) {
  switch (cmp) {
    case CMP_NPM: return 2;
    case CMP_PEP440: return 8;
    case CMP_MAVEN: return 1;  // one class: the numeric projection (libver.h mvn_numeric_projection)
    default: return 1;
  }
}

bool lib_compile_constraint(uint8_t cmp, const std::string& constraint, std::vector<KSet>& out) {
  const int n = lib_classes(cmp);
  if (cmp == CMP_NPM) return npm_compile(constraint, out);
  if (cmp == CMP_PEP440) return pep_compile(constraint, out);
  KSet s;
  bool ok = false;
  switch (cmp) {
    case CMP_GENERIC: ok = gen_compile(constraint, false, s); break;
    case CMP_BITNAMI: ok = gen_compile(constraint, true, s); break;
    case CMP_MAVEN: ok = mvn_compile(constraint, s); break;
    case CMP_GEM: ok = gem_compile(constraint, s); break;
    default: return false;
  }
  out = vs_same(n, s);
  return ok;
}

LibRows lib_compile_advisory(uint8_t cmp, const std::vector<std::string>& vulnerable,
                             const std::vector<std::string>& patched, const std::vector<std::string>& unaffected) {
  LibRows r;
  r.ncls = lib_classes(cmp);
  r.cls = vs_none(r.ncls);
  for (const auto* l : {&vulnerable, &patched})
    for (const std::string& v : *l)
      if (v.empty()) {
        r.ok = r.always = true;
        return r;
      }
  auto join = [](const std::vector<std::string>& a, const std::vector<std::string>& b) {
    std::string s;
    bool first = true;
    for (const auto* l : {&a, &b})
      for (const std::string& x : *l) {
        if (!first) s += " || ";
        s += x;
        first = false;
      }
    return s;
  };
  VS m = vs_all(r.ncls);
  if (!vulnerable.empty() && !lib_compile_constraint(cmp, join(vulnerable, {}), m)) return r;
  if (patched.empty() && unaffected.empty()) {
    if (!vulnerable.empty()) r.cls = m;
    r.ok = true;
    return r;
  }
  VS sec;
  if (!lib_compile_constraint(cmp, join(patched, unaffected), sec)) return r;
  r.cls = vs_and(m, vs_not(sec));
  r.ok = true;
  return r;
}

bool lib_rows_contain(uint8_t cmp, const LibRows& r, const std::string& installed) {
  if (r.always) return true;
  std::string k;
  StrSink o{&k};
  uint32_t cls = 0;
  if (!encode_version_cls(cmp, U(installed), uint32_t(installed.size()), o, cls)) return false;
  if (cls >= r.cls.size()) return false;
  return contains(r.cls[cls], k);
}

MvnProgState mvn_program(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                         const std::vector<std::string>& unaffected, std::vector<uint32_t>& words) {
  words.clear();
  for (const auto* l : {&vulnerable, &patched})
    for (const std::string& v : *l)
      if (v.empty()) return MVN_ALWAYS;
  auto join = [](std::initializer_list<const std::vector<std::string>*> ls) {
    std::string s;
    for (const auto* l : ls)
      for (const std::string& x : *l) s += (s.empty() ? "" : " || ") + x;
    return s;
  };
  MvnGroups vg, sg;
  if (!vulnerable.empty() && !mvn_groups(join({&vulnerable}), vg)) return MVN_NEVER;
  if (patched.empty() && unaffected.empty()) {
    if (vulnerable.empty()) return MVN_NEVER;
  } else if (!mvn_groups(join({&patched, &unaffected}), sg)) {
    return MVN_NEVER;
  }
  words.push_back(uint32_t(vg.size()) | (uint32_t(sg.size()) << 16));
  struct Fix {
    size_t at;
    const std::string* txt;
  };
  std::vector<Fix> fix;  // (word holding the term's token offset, text)
  for (const MvnGroups* gs : {&vg, &sg})
    for (const auto& g : *gs) {
      words.push_back(uint32_t(g.size()));
      for (const auto& [op, txt] : g) {
        MvnParse P;
        (void)mvn_parse(U(txt), uint32_t(txt.size()), P);  // checked by mvn_groups
        words.push_back(op | (uint32_t(P.n) << 8) | (uint32_t(txt.size()) << 16));
        fix.push_back({words.size(), &txt});
        words.push_back(0);
        words.push_back(0);
      }
    }
  for (const Fix& f : fix) {  // packed parses, then the texts, behind the groups
    MvnParse P;
    (void)mvn_parse(U(*f.txt), uint32_t(f.txt->size()), P);
    words[f.at] = uint32_t(words.size());
    const size_t base = words.size();
    words.resize(base + size_t(kMvnPackedWords) * P.n);
    mvn_pack(P, U(*f.txt), words.data() + base);
    words[f.at + 1] = uint32_t(words.size());
    std::vector<uint32_t> packed((f.txt->size() + 3) / 4 + 1, 0);
    std::memcpy(packed.data(), f.txt->data(), f.txt->size());
    words.insert(words.end(), packed.begin(), packed.end());
  }
  return MVN_PROGRAM;
}

bool mvn_bounds_numeric(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                        const std::vector<std::string>& unaffected) {
  for (const auto* l : {&vulnerable, &patched, &unaffected})
    for (const std::string& c : *l) {
      MvnGroups g;
      if (!mvn_groups(c, g)) return false;
      for (const auto& alt : g)
        for (const auto& [op, txt] : alt)
          if (!mvn_numeric(U(txt), uint32_t(txt.size()))) return false;
    }
  return true;
}

bool mvn_hybrid(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                const std::vector<std::string>& unaffected) {
  std::vector<uint32_t> w;
  return mvn_program(vulnerable, patched, unaffected, w) == MVN_PROGRAM &&
         mvn_bounds_numeric(vulnerable, patched, unaffected) &&
         lib_compile_advisory(CMP_MAVEN, vulnerable, patched, unaffected).ok;
}

int mvn_is_vulnerable(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                      const std::vector<std::string>& unaffected, const std::string& installed) {
  std::vector<uint32_t> w;
  const MvnProgState st = mvn_program(vulnerable, patched, unaffected, w);
  if (st != MVN_PROGRAM) return st == MVN_ALWAYS ? 1 : 0;
  MvnParse V;
  if (!mvn_parse(U(installed), uint32_t(installed.size()), V)) return 0;  // NewVersion error: not vulnerable
  return mvn_program_eval(w.data(), MvnParseView{&V, U(installed)}) ? 1 : 0;
}

}  // namespace tvm
