// Native CycloneDX decoder (sbom.h).
#include "sbom.h"

#include "host_par.h"

#include <algorithm>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>

#include <sys/mman.h>

namespace tvm {

namespace {

constexpr std::string_view kNamespace = "aquasecurity:trivy:";

// ---- a strict JSON reader that parses the members the decode needs and skips the rest ----

struct Reader {
  const char* s;
  size_t n, i = 0;
  Arena& owned;
  std::string err;
  int depth = 0;

  bool fail(const char* m) {
    if (err.empty()) err = std::string(m) + " at offset " + std::to_string(i);
    return false;
  }
  void ws() {
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
  }
  bool peek(char c) {
    ws();
    return i < n && s[i] == c;
  }
  bool eat(char c) {
    ws();
    if (i < n && s[i] == c) {
      i++;
      return true;
    }
    return false;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
      o += char(cp);
    } else if (cp < 0x800) {
      o += char(0xC0 | (cp >> 6));
      o += char(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += char(0xE0 | (cp >> 12));
      o += char(0x80 | ((cp >> 6) & 0x3F));
      o += char(0x80 | (cp & 0x3F));
    } else {
      o += char(0xF0 | (cp >> 18));
      o += char(0x80 | ((cp >> 12) & 0x3F));
      o += char(0x80 | ((cp >> 6) & 0x3F));
      o += char(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(uint32_t& v) {
    if (i + 4 > n) return fail("short \\u escape");
    v = 0;
    for (int k = 0; k < 4; k++) {
      const int h = hexv(s[i + k]);
      if (h < 0) return fail("bad \\u escape");
      v = v << 4 | uint32_t(h);
    }
    i += 4;
    return true;
  }
  // a string token: a view into the text, or its unescaped copy
  bool str(std::string_view& out) {
    ws();
    if (i >= n || s[i] != '"') return fail("expected a string");
    const size_t a = ++i;
    // eight bytes at a time to the first quote, backslash or control byte (SWAR)
    constexpr uint64_t kOnes = 0x0101010101010101ull, kHigh = 0x8080808080808080ull;
    while (i + 8 <= n) {
      uint64_t w;
      std::memcpy(&w, s + i, 8);
      const uint64_t q = w ^ (kOnes * '"'), b = w ^ (kOnes * '\\');
      const uint64_t hit = ((q - kOnes) & ~q) | ((b - kOnes) & ~b) | ((w - kOnes * 0x20) & ~w);
      if (hit & kHigh) {
        i += size_t(__builtin_ctzll(hit & kHigh)) >> 3;
        break;
      }
      i += 8;
    }
    while (i < n && s[i] != '"' && s[i] != '\\') {
      if (uint8_t(s[i]) < 0x20) return fail("control character in string");
      i++;
    }
    if (i < n && uint8_t(s[i]) < 0x20) return fail("control character in string");
    if (i >= n) return fail("unterminated string");
    if (s[i] == '"') {
      out = std::string_view(s + a, i - a);
      i++;
      return true;
    }
    std::string o(s + a, i - a);
    while (i < n && s[i] != '"') {
      const char c = s[i];
      if (uint8_t(c) < 0x20) return fail("control character in string");
      if (c != '\\') {
        o += c;
        i++;
        continue;
      }
      if (++i >= n) return fail("unterminated escape");
      const char e = s[i++];
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
          uint32_t v;
          if (!hex4(v)) return false;
          if (v >= 0xD800 && v < 0xDC00 && i + 6 <= n && s[i] == '\\' && s[i + 1] == 'u') {
            const size_t save = i;
            i += 2;
            uint32_t w;
            if (!hex4(w)) return false;
            if (w >= 0xDC00 && w < 0xE000) v = 0x10000 + ((v - 0xD800) << 10) + (w - 0xDC00);
            else i = save, v = 0xFFFD;
          } else if (v >= 0xD800 && v < 0xE000) {
            v = 0xFFFD;  // a lone surrogate
          }
          put_utf8(o, v);
          break;
        }
        default: return fail("bad escape");
      }
    }
    if (i >= n) return fail("unterminated string");
    i++;
    out = owned.keep(o);
    return true;
  }
  bool number(std::string_view& lit) {
    ws();
    const size_t a = i;
    if (i < n && s[i] == '-') i++;
    if (i >= n) return fail("bad number");
    if (s[i] == '0') {
      i++;
    } else if (s[i] >= '1' && s[i] <= '9') {
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    } else {
      return fail("bad number");
    }
    if (i < n && s[i] == '.') {
      i++;
      if (i >= n || s[i] < '0' || s[i] > '9') return fail("bad number");
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
      i++;
      if (i < n && (s[i] == '+' || s[i] == '-')) i++;
      if (i >= n || s[i] < '0' || s[i] > '9') return fail("bad number");
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    }
    lit = std::string_view(s + a, i - a);
    return true;
  }
  bool literal(const char* w) {
    const size_t l = std::strlen(w);
    if (i + l > n || std::memcmp(s + i, w, l) != 0) return fail("bad literal");
    i += l;
    return true;
  }
  bool skip() {
    ws();
    if (i >= n) return fail("unexpected end of input");
    const char c = s[i];
    if (c == '"') {
      std::string_view v;
      return str(v);
    }
    if (c == '{' || c == '[') {
      if (++depth > 10000) return fail("nesting too deep");
      i++;
      const char close = c == '{' ? '}' : ']';
      if (eat(close)) {
        depth--;
        return true;
      }
      for (;;) {
        if (c == '{') {
          std::string_view k;
          if (!str(k) || !eat(':') ) return fail("expected ':'");
        }
        if (!skip()) return false;
        if (eat(',')) continue;
        if (eat(close)) break;
        return fail("expected ',' or a closing bracket");
      }
      depth--;
      return true;
    }
    if (c == 't') return literal("true");
    if (c == 'f') return literal("false");
    if (c == 'n') return literal("null");
    std::string_view lit;
    return number(lit);
  }
  // members of an object: f(key) parses the value (returns false on error)
  template <class F>
  bool object(F&& f) {
    if (!eat('{')) return fail("expected an object");
    if (eat('}')) return true;
    for (;;) {
      std::string_view k;
      if (!str(k)) return false;
      if (!eat(':')) return fail("expected ':'");
      if (!f(k)) return false;
      if (eat(',')) continue;
      if (eat('}')) return true;
      return fail("expected ',' or '}'");
    }
  }
  template <class F>
  bool array(F&& f) {
    if (!eat('[')) return fail("expected an array");
    if (eat(']')) return true;
    for (;;) {
      if (!f()) return false;
      if (eat(',')) continue;
      if (eat(']')) return true;
      return fail("expected ',' or ']'");
    }
  }
  // a string member value; other JSON kinds read as "" (validated and skipped)
  bool str_or_empty(std::string_view& out) {
    if (peek('"')) return str(out);
    out = {};
    return skip();
  }
};

// ---- PURL (packageurl-go FromString as trivy_amd/sbom.py parse_purl restates it) ----------

using KV = std::pair<std::string_view, std::string_view>;

struct Purl {
  std::string_view type, ns, name, version, subpath;
  uint32_t q0 = 0, nq = 0;  // qualifiers (lower-cased key, value), in order: Pools::quals[qt][q0, q0 + nq)
  uint32_t qt = 0;
};

// Shared storage of every component's properties (the parse) and qualifiers (one vector per
// parallel piece of the PURL pass): no vector per component.
struct Pools {
  HugeVec<KV> props;
  std::vector<std::vector<KV>> quals;
};

struct Strs {
  Arena& owned;
  std::vector<KV>& quals;
  uint32_t qt;
  std::string_view keep(const std::string& x) { return owned.keep(x); }
  // urllib.parse.unquote: %XX decoded, malformed escapes kept
  std::string_view unq(std::string_view x) {
    if (x.find('%') == std::string_view::npos) return x;
    std::string o;
    o.reserve(x.size());
    for (size_t k = 0; k < x.size(); k++) {
      if (x[k] == '%' && k + 2 < x.size()) {
        const int h = Reader::hexv(x[k + 1]), l = Reader::hexv(x[k + 2]);
        if (h >= 0 && l >= 0) {
          o += char(h * 16 + l);
          k += 2;
          continue;
        }
      }
      o += x[k];
    }
    return keep(o);
  }
  std::string_view lower(std::string_view x) {
    bool any = false;
    for (char c : x) any |= c >= 'A' && c <= 'Z';
    if (!any) return x;
    std::string o(x);
    for (char& c : o)
      if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
    return keep(o);
  }
  std::string_view join(std::string_view a, std::string_view sep, std::string_view b) { return owned.keep(a, sep, b); }
};

std::string_view strip(std::string_view x, char c) {
  while (!x.empty() && x.front() == c) x.remove_prefix(1);
  while (!x.empty() && x.back() == c) x.remove_suffix(1);
  return x;
}

// nullptr, or the error trivy_amd/sbom.py parse_purl raises
const char* parse_purl(std::string_view s, Strs& S, Purl& p) {
  if (s.substr(0, 4) != "pkg:") return "failed to parse PURL: scheme is not \"pkg\"";
  std::string_view rest = s.substr(4);
  while (!rest.empty() && rest.front() == '/') rest.remove_prefix(1);
  p = Purl{};
  p.qt = S.qt;
  p.q0 = uint32_t(S.quals.size());
  if (const size_t h = rest.find('#'); h != std::string_view::npos) {
    const std::string_view sp = strip(rest.substr(h + 1), '/');
    rest = rest.substr(0, h);
    std::string o;
    bool first = true;
    for (size_t a = 0; a <= sp.size();) {
      size_t b = sp.find('/', a);
      if (b == std::string_view::npos) b = sp.size();
      const std::string_view seg = sp.substr(a, b - a);
      if (!seg.empty() && seg != "." && seg != "..") {
        if (!first) o += '/';
        o.append(S.unq(seg));
        first = false;
      }
      a = b + 1;
    }
    p.subpath = S.keep(o);
  }
  if (const size_t q = rest.find('?'); q != std::string_view::npos) {
    const std::string_view qs = rest.substr(q + 1);
    rest = rest.substr(0, q);
    for (size_t a = 0; a <= qs.size();) {
      size_t b = qs.find('&', a);
      if (b == std::string_view::npos) b = qs.size();
      const std::string_view kv = qs.substr(a, b - a);
      const size_t e = kv.find('=');
      const std::string_view k = kv.substr(0, e), v = e == std::string_view::npos ? std::string_view() : kv.substr(e + 1);
      if (!kv.empty() && !v.empty()) {
        S.quals.emplace_back(S.lower(k), S.unq(v));
        p.nq++;
      }
      a = b + 1;
    }
  }
  const size_t sl = rest.find('/');
  const std::string_view typ = rest.substr(0, sl);
  rest = sl == std::string_view::npos ? std::string_view() : rest.substr(sl + 1);
  if (typ.empty() || rest.empty()) return "failed to parse PURL: missing type or name";
  if (const size_t at = rest.rfind('@'); at != std::string_view::npos) {
    p.version = S.unq(rest.substr(at + 1));
    rest = rest.substr(0, at);
  }
  rest = strip(rest, '/');
  // segments: all but the last form the namespace (empty ones dropped), the last the name
  const size_t last = rest.rfind('/');
  p.name = S.unq(last == std::string_view::npos ? rest : rest.substr(last + 1));
  if (last != std::string_view::npos) {
    const std::string_view nsraw = rest.substr(0, last);
    std::string o;
    for (size_t a = 0; a <= nsraw.size();) {
      size_t b = nsraw.find('/', a);
      if (b == std::string_view::npos) b = nsraw.size();
      const std::string_view seg = S.unq(nsraw.substr(a, b - a));
      if (!seg.empty()) {
        if (!o.empty()) o += '/';
        o.append(seg);
      }
      a = b + 1;
    }
    p.ns = S.keep(o);
  }
  p.type = S.lower(typ);
  return nullptr;
}

// purl.go:130-179 LangType
std::string_view lang_type(const Purl& p) {
  static const std::unordered_map<std::string_view, std::string_view> lang = {
      {"composer", "composer"}, {"maven", "jar"},  {"gem", "gemspec"},     {"conda", "conda-pkg"}, {"pypi", "python-pkg"},
      {"golang", "gobinary"},   {"npm", "node-pkg"}, {"cargo", "cargo"},   {"nuget", "nuget"},     {"swift", "swift"},
      {"cocoapods", "cocoapods"}, {"hex", "hex"},  {"conan", "conan"},     {"pub", "pub"},         {"bitnami", "bitnami"}};
  static const std::unordered_map<std::string_view, std::string_view> k8s = {
      {"eks", "eks"}, {"gke", "gke"}, {"aks", "aks"}, {"ocp", "ocp"}, {"", "kubernetes"}};
  if (p.type == "k8s") {
    auto it = k8s.find(p.ns);
    return it == k8s.end() ? std::string_view() : it->second;
  }
  auto it = lang.find(p.type);
  return it == lang.end() ? std::string_view() : it->second;
}

bool is_os_type(std::string_view t) { return t == "apk" || t == "deb" || t == "rpm"; }

// purl.go:181-193 Class: 1 os-pkgs, 2 lang-pkgs, 0 neither
int purl_class(const Purl& p) { return is_os_type(p.type) ? 1 : (lang_type(p).empty() ? 0 : 2); }

bool ascii_digits(std::string_view v) {
  if (v.empty()) return false;
  for (char c : v)
    if (c < '0' || c > '9') return false;
  return true;
}

// strconv.Atoi (decode.go:209, purl.go:230): an optional sign, then ASCII digits only (no
// spaces), within int64; false on a syntax or range error
bool go_atoi(std::string_view v, int64_t& out) {
  bool neg = false;
  if (!v.empty() && (v.front() == '+' || v.front() == '-')) {
    neg = v.front() == '-';
    v.remove_prefix(1);
  }
  if (!ascii_digits(v)) return false;
  uint64_t x = 0;
  const uint64_t lim = neg ? (uint64_t(1) << 63) : (uint64_t(1) << 63) - 1;
  for (char c : v) {
    const uint64_t d = uint64_t(c - '0');
    if (x > (lim - d) / 10) return false;
    x = x * 10 + d;
  }
  out = neg ? int64_t(0 - x) : int64_t(x);
  return true;
}

struct Comp {
  std::string_view type, name, group, version, bom_ref, purl_str;
  uint32_t p0 = 0, np = 0;  // properties (namespace prefix removed): Pools::props[p0, p0 + np)
  bool has_purl = false;
  Purl purl;
};

enum CompType : uint8_t { CT_OTHER, CT_CONTAINER, CT_APPLICATION, CT_LIBRARY, CT_OS, CT_PLATFORM };

CompType comp_type(std::string_view t) {
  if (t == "library") return CT_LIBRARY;
  if (t == "application") return CT_APPLICATION;
  if (t == "operating-system") return CT_OS;
  if (t == "container") return CT_CONTAINER;
  if (t == "platform") return CT_PLATFORM;
  return CT_OTHER;
}

bool read_component(Reader& R, Pools& P, Comp& c, size_t* members = nullptr) {
  c = Comp{};
  return R.object([&](std::string_view k) {
    if (members) ++*members;
    if (k == "type") return R.str_or_empty(c.type);
    if (k == "name") return R.str_or_empty(c.name);
    if (k == "group") return R.str_or_empty(c.group);
    if (k == "version") return R.str_or_empty(c.version);
    if (k == "bom-ref") return R.str_or_empty(c.bom_ref);
    if (k == "purl") return R.str_or_empty(c.purl_str);
    if (k == "properties") {
      c.p0 = uint32_t(P.props.size());  // a repeated member: the last one wins
      c.np = 0;
      if (!R.peek('[')) return R.skip();
      return R.array([&] {
        std::string_view pn, pv;
        if (!R.peek('{')) return R.skip();
        if (!R.object([&](std::string_view f) {
              if (f == "name") return R.str_or_empty(pn);
              if (f == "value") return R.str_or_empty(pv);
              return R.skip();
            }))
          return false;
        if (pn.substr(0, kNamespace.size()) == kNamespace) pn.remove_prefix(kNamespace.size());
        P.props.emplace_back(pn, pv);
        c.np++;
        return true;
      });
    }
    return R.skip();
  });
}

// bom-ref -> component: open addressing over (hash, component); a later put of the same
// ref replaces the earlier component (a JSON decode into a map keeps the last)
class RefMap {
 public:
  explicit RefMap(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 2) cap <<= 1;
    e_.assign(cap, E{0, nullptr});  // (HugeVec)
    mask_ = cap - 1;
  }
  void put(std::string_view k, Comp* c) { put(k, c, hash(k)); }
  void put(std::string_view k, Comp* c, uint64_t h) {
    for (size_t i = h & mask_;; i = (i + 1) & mask_) {
      if (!e_[i].c) {
        e_[i] = E{h, c};
        return;
      }
      if (e_[i].h == h && e_[i].c->bom_ref == k) {
        e_[i].c = c;
        return;
      }
    }
  }
  Comp* get(std::string_view k) const {
    const uint64_t h = hash(k);
    for (size_t i = h & mask_;; i = (i + 1) & mask_) {
      if (!e_[i].c) return nullptr;
      if (e_[i].h == h && e_[i].c->bom_ref == k) return e_[i].c;
    }
  }

 private:
  struct E {
    uint64_t h;
    Comp* c;
  };
  HugeVec<E> e_;
  size_t mask_ = 0;

 public:
  static uint64_t hash(std::string_view k) {
    uint64_t h = 1469598103934665603ull ^ k.size();
    size_t i = 0;
    for (; i + 8 <= k.size(); i += 8) {
      uint64_t w;
      std::memcpy(&w, k.data() + i, 8);
      h = (h ^ w) * 0x9E3779B97F4A7C15ull;
      h ^= h >> 29;
    }
    for (; i < k.size(); i++) h = (h ^ uint8_t(k[i])) * 1099511628211ull;
    h ^= h >> 32;
    return h * 0xD6E8FEB86659FD93ull;
  }
};

struct Dep {
  std::string_view ref;
  std::vector<std::string_view> on;
  bool has_ref = false;
};

}  // namespace

void* huge_alloc(size_t bytes) {
  constexpr size_t kHuge = size_t(2) << 20;
  if (bytes < kHuge) {
    void* p = std::malloc(std::max<size_t>(bytes, 1));
    if (!p) throw std::bad_alloc();
    return p;
  }
  const size_t len = (bytes + kHuge - 1) & ~(kHuge - 1);
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
  (void)madvise(p, len, MADV_HUGEPAGE);
  return p;
}

void huge_free(void* p, size_t bytes) {
  constexpr size_t kHuge = size_t(2) << 20;
  if (!p) return;
  if (bytes < kHuge) {
    std::free(p);
    return;
  }
  munmap(p, (bytes + kHuge - 1) & ~(kHuge - 1));
}

Arena::~Arena() {
  for (const Chunk& c : chunks) huge_free(c.p, c.n);
}

std::string_view Arena::keep(std::string_view a, std::string_view b, std::string_view c) {
  const size_t n = a.size() + b.size() + c.size();
  if (n == 0) return {};
  if (n > left) {
    const size_t sz = std::max<size_t>(n, size_t(2) << 20);
    chunks.push_back(Chunk{static_cast<char*>(huge_alloc(sz)), sz});
    at = chunks.back().p;
    left = sz;
  }
  char* d = at;
  if (!a.empty()) std::memcpy(d, a.data(), a.size());  // (an empty view may have a null data(): UBSan, tools/san)
  if (!b.empty()) std::memcpy(d + a.size(), b.data(), b.size());
  if (!c.empty()) std::memcpy(d + a.size() + b.size(), c.data(), c.size());
  at += n;
  left -= n;
  return std::string_view(d, n);
}

namespace {
// TVM_SBOM_TRACE=1 (measurement only): per-phase host times on stderr
struct Lap {
  bool on = std::getenv("TVM_SBOM_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void operator()(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "sbom %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};
}  // namespace

bool decode_cyclonedx(std::string_view text_in, Sbom& out, std::string& err, bool borrow) {
  Lap lap;
  std::string_view text = text_in;
  if (!borrow) {
    out.text.assign(text_in.data(), text_in.size());
    text = out.text;
  }
  lap("copy");
  Reader R{text.data(), text.size(), 0, out.arena(0), {}, 0};
  Pools pools;
  pools.props.reserve(text.size() / 128 + 16);
  HugeVec<Comp> comps;
  comps.reserve(text.size() / 256 + 16);  // a component is a few hundred bytes of JSON
  Comp root;
  bool has_root = false;
  std::vector<Dep> deps;
  std::string_view serial;
  int64_t version = 0;
  // the document: the members the decode reads, the rest validated and skipped (a repeated
  // member: the last one wins, as a JSON decode into a map does)
  const bool ok = R.object([&](std::string_view k) {
    if (k == "components") {
      comps.clear();
      if (!R.peek('[')) return R.skip();
      return R.array([&] {
        comps.emplace_back();
        if (!R.peek('{')) {
          comps.pop_back();
          return R.skip();
        }
        return read_component(R, pools, comps.back());
      });
    }
    if (k == "metadata") {
      has_root = false;
      if (!R.peek('{')) return R.skip();
      return R.object([&](std::string_view f) {
        if (f != "component") return R.skip();
        if (!R.peek('{')) {
          has_root = false;
          return R.skip();
        }
        size_t members = 0;
        const bool good = read_component(R, pools, root, &members);
        has_root = members > 0;  // an empty metadata component is no root
        return good;
      });
    }
    if (k == "dependencies") {
      deps.clear();
      if (!R.peek('[')) return R.skip();
      return R.array([&] {
        if (!R.peek('{')) return R.skip();
        deps.emplace_back();
        Dep& d = deps.back();
        return R.object([&](std::string_view f) {
          if (f == "ref") {
            d.has_ref = R.peek('"');
            return R.str_or_empty(d.ref);
          }
          if (f == "dependsOn") {
            d.on.clear();
            if (!R.peek('[')) return R.skip();
            return R.array([&] {
              std::string_view x;
              if (!R.peek('"')) return R.skip();
              if (!R.str(x)) return false;
              d.on.push_back(x);
              return true;
            });
          }
          return R.skip();
        });
      });
    }
    if (k == "serialNumber") return R.str_or_empty(serial);
    if (k == "version") {
      std::string_view lit;
      if (R.peek('"') || R.peek('{') || R.peek('[') || R.peek('t') || R.peek('f') || R.peek('n')) {
        version = 0;
        return R.skip();
      }
      if (!R.number(lit)) return false;
      int64_t v = 0;
      version = go_atoi(lit, v) ? v : 0;
      return true;
    }
    return R.skip();
  });
  R.ws();
  if (!ok || R.i != R.n) {
    err = "failed to decode CycloneDX JSON: " + (R.err.empty() ? std::string("trailing data") : R.err);
    return false;
  }
  out.serial = serial;
  out.version = version;
  lap("parse");

  // parseComponents: unsupported types dropped, a component whose PURL does not parse skipped
  // (the PURLs in parallel pieces, each with its own arena and qualifier vector)
  const int T = host_threads();
  const size_t pieces = std::max<size_t>(1, std::min<size_t>(size_t(T) * 4, comps.size() / 4096));
  pools.quals.resize(pieces + 1);
  std::vector<uint8_t> keep_comp(comps.size(), 0);
  for (size_t k = 0; k <= pieces; k++) out.arena(k + 1);
  dynamic_for(T, pieces, [&](size_t k) {
    Strs S{*out.arenas[k + 1], pools.quals[k], uint32_t(k)};
    const size_t a = comps.size() * k / pieces, b = comps.size() * (k + 1) / pieces;
    for (size_t i = a; i < b; i++) {
      Comp& c = comps[i];
      if (comp_type(c.type) == CT_OTHER) continue;
      if (!c.purl_str.empty()) {
        if (parse_purl(c.purl_str, S, c.purl)) continue;  // parseComponents logs and skips it
        c.has_purl = true;
      }
      keep_comp[i] = 1;
    }
  });
  std::vector<Comp*> order;
  order.reserve(comps.size() + 1);
  for (size_t i = 0; i < comps.size(); i++)
    if (keep_comp[i]) order.push_back(&comps[i]);
  if (has_root) {
    if (comp_type(root.type) == CT_OTHER) {
      err = "failed to parse root component: unsupported component type";
      return false;
    }
    if (!root.purl_str.empty()) {
      Strs S{*out.arenas[pieces + 1], pools.quals[pieces], uint32_t(pieces)};
      if (const char* e = parse_purl(root.purl_str, S, root.purl)) {
        err = e;
        return false;
      }
      root.has_purl = true;
    }
    order.push_back(&root);
  }
  lap("purls");
  // bom-ref -> component (a later one with the same ref replaces an earlier one)
  RefMap by_ref(order.size());
  {
    std::vector<uint64_t> h(order.size());
    range_for(order.size(), 8192, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; i++) h[i] = RefMap::hash(order[i]->bom_ref);
    });
    for (size_t i = 0; i < order.size(); i++) by_ref.put(order[i]->bom_ref, order[i], h[i]);
  }
  std::unordered_map<const Comp*, std::vector<Comp*>> rels;
  for (const Dep& d : deps) {
    if (!d.has_ref) continue;
    Comp* parent = by_ref.get(d.ref);
    if (!parent) continue;
    std::vector<Comp*>& v = rels[parent];
    std::vector<Comp*> found(d.on.size());
    range_for(d.on.size(), 8192, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; i++) found[i] = by_ref.get(d.on[i]);
    });
    v.clear();
    for (Comp* child : found)
      if (child) v.push_back(child);
  }

  lap("refs");
  // Decoder.Decode
  const Comp* os_c = nullptr;
  struct App {
    const Comp* c;
    std::string_view type, file_path;
  };
  std::vector<App> apps;
  // component (index in comps, root last) -> its package in pkgs, -1 for none
  std::vector<int64_t> pkg_of(comps.size() + 1, -1);
  auto comp_index = [&](const Comp* c) { return c == &root ? comps.size() : size_t(c - comps.data()); };
  // pass A (in order): the OS, the applications, the library candidates; the first error in
  // component order is the one the reference reports
  static const std::string_view kAggregating[] = {"python-pkg", "conda-pkg", "gemspec", "node-pkg", "jar"};
  std::vector<uint32_t> cand;  // positions in `order` of the components decodeLibrary reads
  cand.reserve(order.size());
  size_t os_err_at = order.size();
  for (size_t oi = 0; oi < order.size(); oi++) {
    const Comp* c = order[oi];
    const CompType ct = comp_type(c->type);
    if (ct == CT_OS) {
      if (os_c) {
        os_err_at = oi;
        break;
      }
      os_c = c;
      out.has_os = true;
      out.os_family = c->name;
      out.os_name = c->version;
      continue;
    }
    if (ct == CT_APPLICATION) {
      std::string_view t;
      bool has_t = false;
      for (uint32_t q = c->p0; q < c->p0 + c->np; q++)
        if (const auto& [k, v] = pools.props[q]; k == "Type") {
          t = v;
          has_t = true;
          break;
        }
      if (has_t && !t.empty()) {
        const bool agg = std::find(std::begin(kAggregating), std::end(kAggregating), t) != std::end(kAggregating);
        apps.push_back(App{c, t, agg ? std::string_view() : c->name});
        continue;
      }
    }
    if (c->has_purl && purl_class(c->purl)) cand.push_back(uint32_t(oi));
  }
  // decodeLibrary of one component; false: its SrcEpoch property is not an integer
  auto decode_lib = [&](const Comp* c, Strs& S, SbomPkg& k) -> bool {
    const Purl& p = c->purl;
    const int cls = purl_class(p);
    const bool maven = p.type == "maven" || p.type == "gradle";
    k.name = p.name;
    if (!p.ns.empty() && cls != 1) k.name = S.join(p.ns, maven ? ":" : "/", p.name);
    if (!p.subpath.empty() && p.type == "cocoapods") k.name = S.join(p.name, "/", p.subpath);
    k.version = p.version;
    for (uint32_t q = p.q0; q < p.q0 + p.nq; q++) {
      const auto& [qk, qv] = pools.quals[p.qt][q];
      if (qk == "arch") {
        k.arch = qv;
        k.present |= SP_ARCH;
      } else if (qk == "modularitylabel") {
        k.modularitylabel = qv;
        k.present |= SP_MODULARITY;
      } else if (qk == "epoch") {
        int64_t e;
        if (go_atoi(qv, e)) {  // purl.go:229-233: an error leaves Epoch as it is
          k.epoch = e;
          k.present |= SP_EPOCH;
        }
      }
    }
    if (p.type == "rpm") {  // go-rpm-version: [epoch:]version[-release], the release after the FIRST '-' (rpm.c)
      std::string_view v = p.version;
      if (const size_t col = v.find(':'); col != std::string_view::npos) v = v.substr(col + 1);
      const size_t dash = v.find('-');
      k.version = dash == std::string_view::npos ? v : v.substr(0, dash);
      k.release = dash == std::string_view::npos ? std::string_view() : v.substr(dash + 1);
      k.present |= SP_RELEASE;
    }
    if (p.type != "cocoapods") k.name = c->group.empty() ? c->name : S.join(c->group, maven ? ":" : "/", c->name);
    // dependency.ID (pkg/dependency/id.go:9-27)
    {
      const std::string_view lt = lang_type(p);
      if (p.version.empty()) {
        k.id = k.name;
      } else if (lt == "conan") {
        k.id = S.join(k.name, "/", p.version);
      } else if ((lt == "gomod" || lt == "gobinary") && p.version.front() != 'v') {
        k.id = S.owned.keep(k.name, "@v", p.version);
      } else if (lt == "jar" || lt == "pom" || lt == "gradle") {
        k.id = S.join(k.name, ":", p.version);
      } else {
        k.id = S.join(k.name, "@", p.version);
      }
    }
    for (uint32_t q = c->p0; q < c->p0 + c->np; q++) {
      const auto& [pk, pv] = pools.props[q];
      if (pk == "PkgID") {
        k.id = pv;
      } else if (pk == "FilePath") {
        k.file_path = pv;
        k.present |= SP_FILEPATH;
      } else if (pk == "SrcName") {
        k.src_name = pv;
        k.present |= SP_SRCNAME;
      } else if (pk == "SrcVersion") {
        k.src_version = pv;
        k.present |= SP_SRCVERSION;
      } else if (pk == "SrcRelease") {
        k.src_release = pv;
        k.present |= SP_SRCRELEASE;
      } else if (pk == "Modularitylabel") {
        k.modularitylabel = pv;
        k.present |= SP_MODULARITY;
      } else if (pk == "SrcEpoch") {
        int64_t e;
        if (!go_atoi(pv, e)) return false;  // "invalid src epoch" (decode.go:208-211 strconv.Atoi)
        k.src_epoch = e;
        k.present |= SP_SRCEPOCH;
      } else if (pk == "LayerDigest") {
        k.layer_digest = pv;
        k.present |= SP_LAYER_DIGEST;
      } else if (pk == "LayerDiffID") {
        k.layer_diff_id = pv;
        k.present |= SP_LAYER_DIFFID;
      }
    }
    k.purl = c->purl_str;
    k.bom_ref = c->bom_ref;
    if (cls == 1) {  // fillSrcPkg (decode.go:260-279): empty source fields default to the binary's
      if (k.src_name.empty()) k.src_name = k.name;
      if (k.src_version.empty()) k.src_version = k.version;
      if (k.src_release.empty()) k.src_release = k.release;
      if (k.src_epoch == 0) k.src_epoch = k.epoch;
      k.present |= SP_SRCNAME | SP_SRCVERSION | SP_SRCRELEASE | SP_SRCEPOCH;
    }
    return true;
  };
  // pass B (parallel pieces, each with its own arena): the libraries
  HugeVec<SbomPkg> pkgs(cand.size());
  std::vector<uint8_t> bad(cand.size(), 0);
  {
    const size_t lp = std::max<size_t>(1, std::min<size_t>(size_t(T) * 4, cand.size() / 4096));
    const size_t a0 = out.arenas.size();
    for (size_t k = 0; k < lp; k++) out.arena(a0 + k);
    dynamic_for(T, lp, [&](size_t k) {
      std::vector<KV> unused;
      Strs S{*out.arenas[a0 + k], unused, 0};
      const size_t a = cand.size() * k / lp, b = cand.size() * (k + 1) / lp;
      for (size_t j = a; j < b; j++) bad[j] = decode_lib(order[cand[j]], S, pkgs[j]) ? 0 : 1;
    });
  }
  for (size_t j = 0; j < cand.size() && cand[j] < os_err_at; j++)
    if (bad[j]) {
      err = "failed to decode components: failed to decode library: invalid src epoch";
      return false;
    }
  if (os_err_at < order.size()) {
    err = "failed to decode components: multiple OS components are not supported";
    return false;
  }
  std::vector<const Comp*> pkg_comp(cand.size());
  for (size_t j = 0; j < cand.size(); j++) {
    pkg_comp[j] = order[cand[j]];
    pkg_of[comp_index(pkg_comp[j])] = int64_t(j);
  }
  std::vector<uint8_t> taken;
  taken.assign(pkgs.size(), 0);
  // targets as index lists into pkgs: the OS packages, then every application
  std::vector<std::vector<uint32_t>> tidx(1);
  std::vector<std::pair<std::string_view, std::string_view>> tmeta(1);
  auto take = [&](const Comp* d, std::vector<uint32_t>& dst) {
    const int64_t k = pkg_of[comp_index(d)];
    if (k < 0 || taken[size_t(k)]) return;
    taken[size_t(k)] = 1;
    dst.push_back(uint32_t(k));
  };
  if (os_c) {
    auto it = rels.find(os_c);
    if (it != rels.end())
      for (const Comp* d : it->second) take(d, tidx[0]);
  }
  for (const App& a : apps) {
    tidx.emplace_back();
    tmeta.emplace_back(a.type, a.file_path);
    auto it = rels.find(a.c);
    if (it != rels.end())
      for (const Comp* d : it->second) take(d, tidx.back());
  }
  // the rest: OS packages of one PURL type, one application per language type
  std::vector<std::string_view> os_types, lang_types;
  std::vector<std::vector<uint32_t>> os_rest, lang_rest;
  for (size_t k = 0; k < pkgs.size(); k++) {
    if (taken[k]) continue;
    const Purl& p = pkg_comp[k]->purl;
    const bool os = purl_class(p) == 1;
    auto& types = os ? os_types : lang_types;
    auto& groups = os ? os_rest : lang_rest;
    const std::string_view key = os ? p.type : lang_type(p);
    size_t g = std::find(types.begin(), types.end(), key) - types.begin();
    if (g == types.size()) {
      types.push_back(key);
      groups.emplace_back();
    }
    groups[g].push_back(uint32_t(k));
  }
  if (os_rest.size() > 1) {
    err = "failed to aggregate packages: multiple types of OS packages in SBOM are not supported";
    return false;
  }
  auto by_name = [&](uint32_t x, uint32_t y) {  // Packages.Less (artifact.go:203-211), byte order
    const SbomPkg &a = pkgs[x], &b = pkgs[y];
    if (a.name != b.name) return a.name < b.name;
    if (a.version != b.version) return a.version < b.version;
    return a.file_path < b.file_path;
  };
  if (!os_rest.empty() && out.has_os && !out.os_family.empty()) {
    std::stable_sort(os_rest[0].begin(), os_rest[0].end(), by_name);
    tidx[0].insert(tidx[0].end(), os_rest[0].begin(), os_rest[0].end());
  }
  for (size_t g = 0; g < lang_rest.size(); g++) {
    std::stable_sort(lang_rest[g].begin(), lang_rest[g].end(), by_name);
    tidx.push_back(std::move(lang_rest[g]));
    tmeta.emplace_back(lang_types[g], std::string_view());
  }
  // applications ordered by (Type, FilePath), stable
  std::vector<size_t> order_apps(tidx.size() - 1);
  for (size_t a = 0; a < order_apps.size(); a++) order_apps[a] = a + 1;
  std::stable_sort(order_apps.begin(), order_apps.end(), [&](size_t x, size_t y) {
    if (tmeta[x].first != tmeta[y].first) return tmeta[x].first < tmeta[y].first;
    return tmeta[x].second < tmeta[y].second;
  });
  lap("assemble");
  // detector input: every target's packages contiguous (tvm_package + the extra fields),
  // filled in parallel pieces
  std::vector<uint32_t> flat;
  {
    size_t total = tidx[0].size();
    for (size_t a : order_apps) total += tidx[a].size();
    flat.reserve(total);
  }
  auto place = [&](const std::vector<uint32_t>& idx, std::string_view type, std::string_view fp) {
    out.targets.push_back(SbomTarget{type, fp, flat.size(), flat.size() + idx.size()});
    flat.insert(flat.end(), idx.begin(), idx.end());
  };
  place(tidx[0], {}, {});
  for (size_t a : order_apps) place(tidx[a], tmeta[a].first, tmeta[a].second);
  out.n_view = flat.size();
  out.view.resize(flat.size());
  out.extra.resize(flat.size());
  auto ts = [](std::string_view v) { return tvm_str{v.data(), v.size()}; };
  range_for(flat.size(), 16384, [&](size_t a, size_t b) {
    for (size_t at = a; at < b; at++) {
      const SbomPkg& p = pkgs[flat[at]];
      tvm_package& q = out.view[at];
      std::memset(&q, 0, sizeof q);
      q.id = ts(p.id);
      q.name = ts(p.name);
      q.version = ts(p.version);
      q.release = ts(p.release);
      q.arch = ts(p.arch);
      q.epoch = p.epoch;
      q.src_name = ts(p.src_name);
      q.src_version = ts(p.src_version);
      q.src_release = ts(p.src_release);
      q.src_epoch = p.src_epoch;
      q.modularitylabel = ts(p.modularitylabel);
      q.file_path = ts(p.file_path);
      out.extra[at] = SbomExtra{p.purl, p.bom_ref, p.layer_digest, p.layer_diff_id, p.present};
    }
  });
  lap("views");
  return true;
}

}  // namespace tvm
