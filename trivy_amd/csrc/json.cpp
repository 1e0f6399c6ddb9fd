// Strict JSON reader (see json.h).
#include "json.h"

#include <cstring>

namespace tvm {
namespace {

struct Parser {
  std::string_view t;
  size_t i = 0;
  std::string err;
  int depth = 0;

  bool fail(const char* m) {
    if (err.empty()) err = std::string(m) + " at offset " + std::to_string(i);
    return false;
  }
  void ws() {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\t' || t[i] == '\n' || t[i] == '\r')) i++;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += char(cp);
    else if (cp < 0x800) { o += char(0xC0 | (cp >> 6)); o += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      o += char(0xE0 | (cp >> 12)); o += char(0x80 | ((cp >> 6) & 0x3F)); o += char(0x80 | (cp & 0x3F));
    } else {
      o += char(0xF0 | (cp >> 18)); o += char(0x80 | ((cp >> 12) & 0x3F));
      o += char(0x80 | ((cp >> 6) & 0x3F)); o += char(0x80 | (cp & 0x3F));
    }
  }
  // Validates one UTF-8 sequence at i; returns its width or 0 if invalid.
  size_t utf8_width() const {
    const unsigned char* s = reinterpret_cast<const unsigned char*>(t.data()) + i;
    size_t n = t.size() - i;
    unsigned c = s[0];
    if (c < 0x80) return 1;
    unsigned lo = 0x80, hi = 0xBF;
    size_t need;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c >= 0xE0 && c <= 0xEF) { need = 2; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
    else if (c >= 0xF0 && c <= 0xF4) { need = 3; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
    else return 0;
    if (need >= n) return 0;
    for (size_t k = 1; k <= need; k++) {
      unsigned d = s[k];
      if (k == 1 ? (d < lo || d > hi) : (d < 0x80 || d > 0xBF)) return 0;
    }
    return need + 1;
  }
  bool hex4(uint32_t& v) {
    if (i + 4 > t.size()) return fail("short \\u escape");
    v = 0;
    for (int k = 0; k < 4; k++) {
      char c = t[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= uint32_t(c - '0');
      else if (c >= 'a' && c <= 'f') v |= uint32_t(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= uint32_t(c - 'A' + 10);
      else return fail("bad \\u escape");
    }
    return true;
  }
  bool str(std::string& o) {
    i++;  // opening quote
    for (;;) {
      if (i >= t.size()) return fail("unterminated string");
      unsigned char c = static_cast<unsigned char>(t[i]);
      if (c == '"') { i++; return true; }
      if (c < 0x20) return fail("control character in string");
      if (c == '\\') {
        if (++i >= t.size()) return fail("bad escape");
        char e = t[i++];
        switch (e) {
          case '"': o += '"'; break;
          case '\\': o += '\\'; break;
          case '/': o += '/'; break;
          case 'b': o += '\b'; break;
          case 'f': o += '\f'; break;
          case 'n': o += '\n'; break;
          case 'r': o += '\r'; break;
          case 't': o += '\t'; break;
          case 'u': {
            uint32_t cp;
            if (!hex4(cp)) return false;
            if (cp >= 0xD800 && cp < 0xDC00) {
              // high surrogate: needs a following \uDC00-\uDFFF, else U+FFFD (Go behaviour)
              if (i + 6 <= t.size() && t[i] == '\\' && t[i + 1] == 'u') {
                size_t save = i;
                i += 2;
                uint32_t lo;
                if (!hex4(lo)) return false;
                if (lo >= 0xDC00 && lo < 0xE000) { put_utf8(o, 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00)); break; }
                i = save;
              }
              put_utf8(o, 0xFFFD);
            } else if (cp >= 0xDC00 && cp < 0xE000) {
              put_utf8(o, 0xFFFD);
            } else {
              put_utf8(o, cp);
            }
            break;
          }
          default: return fail("bad escape");
        }
        continue;
      }
      size_t w = utf8_width();
      if (w == 0) { put_utf8(o, 0xFFFD); i++; continue; }
      o.append(t.data() + i, w);
      i += w;
    }
  }
  bool num(JVal& v) {
    size_t s = i;
    if (t[i] == '-') i++;
    if (i >= t.size()) return fail("bad number");
    if (t[i] == '0') i++;
    else if (t[i] >= '1' && t[i] <= '9') while (i < t.size() && t[i] >= '0' && t[i] <= '9') i++;
    else return fail("bad number");
    if (i < t.size() && t[i] == '.') {
      i++;
      if (i >= t.size() || !(t[i] >= '0' && t[i] <= '9')) return fail("bad number");
      while (i < t.size() && t[i] >= '0' && t[i] <= '9') i++;
    }
    if (i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
      i++;
      if (i < t.size() && (t[i] == '+' || t[i] == '-')) i++;
      if (i >= t.size() || !(t[i] >= '0' && t[i] <= '9')) return fail("bad number");
      while (i < t.size() && t[i] >= '0' && t[i] <= '9') i++;
    }
    v.kind = JVal::Num;
    v.s.assign(t.data() + s, i - s);
    return true;
  }
  bool lit(const char* w, size_t n) {
    if (t.compare(i, n, w) != 0) return fail("bad literal");
    i += n;
    return true;
  }
  bool val(JVal& v) {
    ws();
    if (i >= t.size()) return fail("unexpected end");
    if (++depth > 10000) return fail("nesting too deep");
    size_t start = i;
    bool ok;
    char c = t[i];
    if (c == '{') {
      v.kind = JVal::Obj;
      i++;
      ws();
      if (i < t.size() && t[i] == '}') { i++; ok = true; }
      else {
        ok = false;
        for (;;) {
          ws();
          if (i >= t.size() || t[i] != '"') { fail("expected key"); break; }
          std::string k;
          if (!str(k)) break;
          ws();
          if (i >= t.size() || t[i] != ':') { fail("expected ':'"); break; }
          i++;
          JVal x;
          if (!val(x)) break;
          v.obj.emplace_back(std::move(k), std::move(x));
          ws();
          if (i < t.size() && t[i] == ',') { i++; continue; }
          if (i < t.size() && t[i] == '}') { i++; ok = true; }
          else fail("expected ',' or '}'");
          break;
        }
      }
    } else if (c == '[') {
      v.kind = JVal::Arr;
      i++;
      ws();
      if (i < t.size() && t[i] == ']') { i++; ok = true; }
      else {
        ok = false;
        for (;;) {
          JVal x;
          if (!val(x)) break;
          v.arr.push_back(std::move(x));
          ws();
          if (i < t.size() && t[i] == ',') { i++; continue; }
          if (i < t.size() && t[i] == ']') { i++; ok = true; }
          else fail("expected ',' or ']'");
          break;
        }
      }
    } else if (c == '"') {
      v.kind = JVal::Str;
      ok = str(v.s);
    } else if (c == 't') {
      v.kind = JVal::Bool; v.b = true; ok = lit("true", 4);
    } else if (c == 'f') {
      v.kind = JVal::Bool; v.b = false; ok = lit("false", 5);
    } else if (c == 'n') {
      v.kind = JVal::Null; ok = lit("null", 4);
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      ok = num(v);
    } else {
      ok = fail("invalid character");
    }
    depth--;
    if (ok) v.raw = t.substr(start, i - start);
    return ok;
  }
};

}  // namespace

bool json_parse(std::string_view text, JVal& out, std::string& err) {
  Parser p{text, 0, {}, 0};
  if (!p.val(out)) { err = p.err; return false; }
  p.ws();
  if (p.i != text.size()) { err = "invalid character after top-level value"; return false; }
  return true;
}

bool json_int(const JVal& v, int64_t& out) {
  if (v.kind != JVal::Num) return false;
  const std::string& s = v.s;
  if (s.find_first_of(".eE") != std::string::npos) return false;
  size_t k = 0;
  bool neg = false;
  if (s[0] == '-') { neg = true; k = 1; }
  uint64_t acc = 0;
  for (; k < s.size(); k++) {
    unsigned d = unsigned(s[k] - '0');
    if (acc > (UINT64_MAX - d) / 10) return false;
    acc = acc * 10 + d;
  }
  if (!neg && acc > uint64_t(INT64_MAX)) return false;
  if (neg && acc > uint64_t(INT64_MAX) + 1) return false;
  out = neg ? int64_t(0 - acc) : int64_t(acc);
  return true;
}

bool json_key_eq(std::string_view key, std::string_view field) {
  if (key.size() != field.size()) return false;
  for (size_t k = 0; k < key.size(); k++) {
    char a = key[k], b = field[k];
    if (a >= 'A' && a <= 'Z') a = char(a - 'A' + 'a');
    if (b >= 'A' && b <= 'Z') b = char(b - 'A' + 'a');
    if (a != b) return false;
  }
  return true;
}

}  // namespace tvm
