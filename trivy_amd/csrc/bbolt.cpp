// Read-only walker of a bbolt file image (the format trivy.db ships in; the reference opens it
// with go.etcd.io/bbolt, pkg/db/db.go, and reads buckets in Get / ForEach,
// trivy-db pkg/db/db.go).  This restates the published on-disk format, not bbolt's code:
//   page      16-byte header {id u64, flags u16, count u16, overflow u32}, then `count`
//             elements; a page spans 1 + overflow page-size units;
//   meta      pages 0 and 1: {magic 0xED0CDAED, version 2, page size, flags, root bucket
//             {root pgid, sequence}, freelist, high-water pgid, txid, checksum = FNV-1a 64 of
//             the preceding meta bytes}; the valid one with the larger txid is current;
//   branch    16-byte elements {pos u32, ksize u32, child pgid u64}, key at element + pos;
//   leaf      16-byte elements {flags u32, pos u32, ksize u32, vsize u32}, key at element +
//             pos, value right after it; flags bit 0 = the value is a nested bucket
//             {root pgid u64, sequence u64}, root 0 = an inline bucket whose leaf page
//             follows the 16-byte header inside the value.
// Every record is reported as (bucket path..., key) -> value in key order; nothing in the
// file is executed or trusted: every offset is bounds-checked.
#include "bbolt.h"

#include <cstring>

namespace tvm {

namespace {

constexpr uint32_t kMagic = 0xED0CDAEDu;
constexpr uint16_t kBranch = 0x01, kLeaf = 0x02, kMeta = 0x04;
constexpr uint32_t kBucketLeaf = 0x01;
constexpr int kMaxDepth = 64;

template <class T>
T rd(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

uint64_t fnv1a64(const uint8_t* p, size_t n) {
  uint64_t h = 14695981039346656037ull;  // FNV-1a 64 offset basis
  for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

struct Walker {
  const uint8_t* b;
  size_t len;
  uint32_t psz = 0;
  const BboltVisit& visit;
  std::string& err;
  std::vector<std::string_view> path;
  std::vector<uint8_t> seen;  // file pages already walked: in a valid tree each page is reached once

  bool fail(const std::string& m) {
    err = "bbolt: " + m;
    return false;
  }
  // page `id` as a byte range [p, p + span)
  bool page(uint64_t id, const uint8_t*& p, size_t& span) {
    if (psz == 0 || id >= (len / psz)) return fail("page id out of range");
    // a crafted file whose branch elements all name one child would otherwise be walked
    // exponentially often (count^depth): reject any page reached twice
    if (seen.size() != len / psz) seen.assign(len / psz, 0);
    if (seen[size_t(id)]) return fail("page referenced twice");
    seen[size_t(id)] = 1;
    const size_t off = size_t(id) * psz;
    if (off + 16 > len) return fail("page past the end of the file");
    p = b + off;
    span = (size_t(rd<uint32_t>(p + 12)) + 1) * psz;
    if (off + span > len) return fail("page overflow past the end of the file");
    return true;
  }
  // the elements of a page image [p, p + span) (a file page or an inline bucket's page)
  bool node(const uint8_t* p, size_t span, int depth) {
    if (depth > kMaxDepth) return fail("buckets nested too deep");
    if (span < 16) return fail("short page");
    const uint16_t flags = rd<uint16_t>(p + 8), count = rd<uint16_t>(p + 10);
    if (size_t(16) + size_t(count) * 16 > span) return fail("element table past the page");
    const uint8_t* el = p + 16;
    for (uint32_t i = 0; i < count; i++, el += 16) {
      const size_t at = size_t(el - p);
      if (flags & kBranch) {
        const uint32_t pos = rd<uint32_t>(el), ks = rd<uint32_t>(el + 4);
        if (at + size_t(pos) + ks > span) return fail("branch key past the page");
        const uint8_t* cp;
        size_t cs;
        if (!page(rd<uint64_t>(el + 8), cp, cs) || !node(cp, cs, depth + 1)) return false;
      } else if (flags & kLeaf) {
        const uint32_t ef = rd<uint32_t>(el), pos = rd<uint32_t>(el + 4), ks = rd<uint32_t>(el + 8),
                       vs = rd<uint32_t>(el + 12);
        if (at + size_t(pos) + ks + vs > span) return fail("leaf key / value past the page");
        const char* k = reinterpret_cast<const char*>(el + pos);
        const uint8_t* v = el + pos + ks;
        if (ef & kBucketLeaf) {
          if (vs < 16) return fail("short bucket header");
          const uint64_t root = rd<uint64_t>(v);
          path.emplace_back(k, ks);
          bool ok;
          if (root == 0) {  // inline bucket: its leaf page follows the header
            ok = node(v + 16, vs - 16, depth + 1);
          } else {
            const uint8_t* cp;
            size_t cs;
            ok = page(root, cp, cs) && node(cp, cs, depth + 1);
          }
          path.pop_back();
          if (!ok) return false;
        } else {
          path.emplace_back(k, ks);
          const bool go = visit(path, std::string_view(reinterpret_cast<const char*>(v), vs));
          path.pop_back();
          if (!go) return fail("walk stopped by the caller");
        }
      } else {
        return fail("page is neither a branch nor a leaf");
      }
    }
    return true;
  }
};

}  // namespace

bool bbolt_walk(const uint8_t* bytes, size_t len, const BboltVisit& visit, std::string& err) {
  Walker w{bytes, len, 0, visit, err, {}, {}};
  // the current meta page: magic, version, checksum; larger txid wins
  int best = -1;
  uint64_t best_tx = 0, root = 0;
  for (int m = 0; m < 2; m++) {
    // page 0 sits at offset 0; page 1 at one page size, which page 0's meta states (or,
    // when page 0 is damaged, the common 4096)
    size_t off = 0;
    if (m == 1) {
      off = (len >= 16 + 12 && rd<uint32_t>(bytes + 16) == kMagic) ? rd<uint32_t>(bytes + 24) : 4096;
      if (off == 0) continue;
    }
    if (off + 16 + 64 > len) continue;
    const uint8_t* p = bytes + off;
    const uint8_t* mt = p + 16;
    if (!(rd<uint16_t>(p + 8) & kMeta) || rd<uint32_t>(mt) != kMagic || rd<uint32_t>(mt + 4) != 2) continue;
    if (fnv1a64(mt, 56) != rd<uint64_t>(mt + 56)) continue;
    const uint64_t tx = rd<uint64_t>(mt + 48);
    if (best < 0 || tx > best_tx) {
      best = m;
      best_tx = tx;
      w.psz = rd<uint32_t>(mt + 8);
      root = rd<uint64_t>(mt + 16);
    }
  }
  if (best < 0) {
    err = "bbolt: no valid meta page (not a bbolt file?)";
    return false;
  }
  if (w.psz < 512 || (w.psz & (w.psz - 1))) {
    err = "bbolt: bad page size";
    return false;
  }
  const uint8_t* p;
  size_t span;
  return w.page(root, p, span) && w.node(p, span, 0);
}

}  // namespace tvm
