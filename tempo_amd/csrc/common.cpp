// common.cpp — hashes, snappy framing, strings.ToLower, file helpers.
#include "common.hpp"

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <exception>
#include <mutex>
#include <thread>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <fcntl.h>
#include <sys/types.h>
#include <strings.h>

namespace tsg {

uint32_t json_u32(std::string_view v, const char *field) {
  while (!v.empty() && (v.front() == ' ' || v.front() == '\t' || v.front() == '\n' || v.front() == '\r')) v.remove_prefix(1);
  while (!v.empty() && (v.back() == ' ' || v.back() == '\t' || v.back() == '\n' || v.back() == '\r')) v.remove_suffix(1);
  if (v.empty() || v.size() > 10) fail(TSG_E_CORRUPT, std::string("meta.json: bad ") + field);
  uint64_t x = 0;
  for (char c : v) {
    if (c < '0' || c > '9') fail(TSG_E_CORRUPT, std::string("meta.json: bad ") + field);
    x = x * 10 + uint64_t(c - '0');
  }
  if (x > 0xffffffffull) fail(TSG_E_CORRUPT, std::string("meta.json: ") + field + " out of range");
  return uint32_t(x);
}

// ---- xxhash64 (github.com/cespare/xxhash v1.1.0) -------------------------------
static constexpr uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL,
                          P3 = 1609587929392839161ULL, P4 = 9650029242287828579ULL,
                          P5 = 2870177450012600261ULL;
static inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t xr(uint64_t a, uint64_t in) { return rotl(a + in * P2, 31) * P1; }
static inline uint64_t xm(uint64_t a, uint64_t v) { return (a ^ xr(0, v)) * P1 + P4; }

uint64_t xxhash64(const uint8_t *p, size_t n) {
  const uint8_t *e = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    do {
      v1 = xr(v1, le64(p));
      v2 = xr(v2, le64(p + 8));
      v3 = xr(v3, le64(p + 16));
      v4 = xr(v4, le64(p + 24));
      p += 32;
    } while (e - p >= 32);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xm(xm(xm(xm(h, v1), v2), v3), v4);
  } else {
    h = P5;
  }
  h += n;
  for (; e - p >= 8; p += 8) h = rotl(h ^ xr(0, le64(p)), 27) * P1 + P4;
  if (e - p >= 4) {
    h = rotl(h ^ (uint64_t(le32(p)) * P1), 23) * P2 + P3;
    p += 4;
  }
  for (; p < e; p++) h = rotl(h ^ (uint64_t(*p) * P5), 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

uint32_t fnv1_32(const uint8_t *p, size_t n) {
  uint32_t h = 2166136261u;
  for (size_t i = 0; i < n; i++) h = (h * 16777619u) ^ p[i];
  return h;
}

static inline uint64_t fmix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
void murmur3_128(const uint8_t *p, size_t n, uint64_t &o1, uint64_t &o2) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 0, h2 = 0;
  size_t nb = n / 16;
  for (size_t i = 0; i < nb; i++) {
    uint64_t k1 = le64(p + 16 * i), k2 = le64(p + 16 * i + 8);
    h1 ^= rotl(k1 * c1, 31) * c2;
    h1 = (rotl(h1, 27) + h2) * 5 + 0x52dce729;
    h2 ^= rotl(k2 * c2, 33) * c1;
    h2 = (rotl(h2, 31) + h1) * 5 + 0x38495ab5;
  }
  const uint8_t *t = p + 16 * nb;
  size_t r = n & 15;
  uint64_t k1 = 0, k2 = 0;
  for (size_t i = r; i > 8; i--) k2 ^= uint64_t(t[i - 1]) << (8 * (i - 9));
  if (r > 8) h2 ^= rotl(k2 * c2, 33) * c1;
  for (size_t i = (r > 8 ? 8 : r); i > 0; i--) k1 ^= uint64_t(t[i - 1]) << (8 * (i - 1));
  if (r > 0) h1 ^= rotl(k1 * c1, 31) * c2;
  h1 ^= n;
  h2 ^= n;
  h1 += h2;
  h2 += h1;
  h1 = fmix(h1);
  h2 = fmix(h2);
  h1 += h2;
  h2 += h1;
  o1 = h1;
  o2 = h2;
}

static uint32_t g_crc[8][256];
static std::once_flag g_crc_once;
static void crc_init() {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_crc[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; i++)
    for (int t = 1; t < 8; t++) g_crc[t][i] = (g_crc[t - 1][i] >> 8) ^ g_crc[0][g_crc[t - 1][i] & 0xff];
}
// the host CPU's CRC32C instruction (SSE4.2), three independent streams over thirds of
// the buffer combined by table-free shifts would be faster still; one stream is ~8 B/cycle/3
__attribute__((target("sse4.2"))) static uint32_t crc32c_hw(const uint8_t *p, size_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = uint32_t(c);
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return ~c32;
}
uint32_t crc32c(const uint8_t *p, size_t n) {
  static const bool hw = __builtin_cpu_supports("sse4.2");
  if (hw) return crc32c_hw(p, n);
  std::call_once(g_crc_once, crc_init);
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {  // slicing-by-8
    uint64_t v = le64(p) ^ c;
    c = g_crc[7][v & 0xff] ^ g_crc[6][(v >> 8) & 0xff] ^ g_crc[5][(v >> 16) & 0xff] ^
        g_crc[4][(v >> 24) & 0xff] ^ g_crc[3][(v >> 32) & 0xff] ^ g_crc[2][(v >> 40) & 0xff] ^
        g_crc[1][(v >> 48) & 0xff] ^ g_crc[0][(v >> 56) & 0xff];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_crc[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return ~c;
}
static inline uint32_t snappy_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// ---- snappy -----------------------------------------------------------------
static constexpr size_t kMaxBlock = 65536, kMaxEnc = 76490;

static void snappy_block_decode(const uint8_t *src, size_t sl, uint8_t *dst, size_t dl) {
  size_t d = 0, s = 0;
  while (s < sl) {
    uint8_t tag = src[s] & 3;
    size_t len, off;
    if (tag == 0) {
      uint32_t x = src[s] >> 2;
      if (x < 60) {
        s += 1;
        // a short literal with 16 bytes of slack on both sides: one fixed-size copy
        if (x < 16 && sl - s >= 16 && dl - d >= 16) {
          std::memcpy(dst + d, src + s, 16);
          d += x + 1;
          s += x + 1;
          continue;
        }
      } else {
        size_t nb = x - 59;
        s += 1 + nb;
        if (s > sl) fail(TSG_E_CORRUPT, "snappy: literal header out of range");
        x = 0;
        for (size_t i = 0; i < nb; i++) x |= uint32_t(src[s - nb + i]) << (8 * i);
      }
      len = size_t(x) + 1;
      if (len > dl - d || len > sl - s) fail(TSG_E_CORRUPT, "snappy: literal out of range");
      if (len <= 16 && sl - s >= 16 && dl - d >= 16) {
        // a short literal (most are): one fixed 16-byte copy, no call; the bytes past `len`
        // land inside the block and later ops overwrite them
        std::memcpy(dst + d, src + s, 16);
      } else {
        std::memcpy(dst + d, src + s, len);
      }
      d += len;
      s += len;
      continue;
    }
    if (tag == 1) {
      s += 2;
      if (s > sl) fail(TSG_E_CORRUPT, "snappy: copy1 out of range");
      len = 4 + ((src[s - 2] >> 2) & 7);
      off = (size_t(src[s - 2] & 0xe0) << 3) | src[s - 1];
    } else if (tag == 2) {
      s += 3;
      if (s > sl) fail(TSG_E_CORRUPT, "snappy: copy2 out of range");
      len = 1 + (src[s - 3] >> 2);
      off = size_t(src[s - 2]) | (size_t(src[s - 1]) << 8);
    } else {
      s += 5;
      if (s > sl) fail(TSG_E_CORRUPT, "snappy: copy4 out of range");
      len = 1 + (src[s - 5] >> 2);
      off = le32(src + s - 4);
    }
    if (off == 0 || d < off || len > dl - d) fail(TSG_E_CORRUPT, "snappy: bad copy");
    if (off >= 8 && dl - d >= ((len + 7) & ~size_t(7))) {
      // 8 bytes at a time: every chunk reads bytes written before it (off >= 8); the last
      // may write up to 7 bytes past the copy, inside the block, which later ops overwrite
      uint8_t *o = dst + d;
      const uint8_t *in = o - off;
      for (size_t k = 0; k < len; k += 8) std::memcpy(o + k, in + k, 8);
    } else if (off >= len) {
      std::memcpy(dst + d, dst + d - off, len);
    } else {
      for (size_t i = 0; i < len; i++) dst[d + i] = dst[d - off + i];
    }
    d += len;
  }
  if (d != dl) fail(TSG_E_CORRUPT, "snappy: short block");
}

// Decoded size of a framed stream, from its chunk headers (no checks beyond what reading them
// needs: stops at the first chunk it cannot read; the decode below does the checking)
static size_t snappy_framed_size(const uint8_t *src, size_t n) {
  size_t s = 0, total = 0;
  while (n - s >= 4) {
    const uint8_t ct = src[s];
    const size_t cl = size_t(src[s + 1]) | (size_t(src[s + 2]) << 8) | (size_t(src[s + 3]) << 16);
    s += 4;
    if (cl > n - s) break;
    const uint8_t *b = src + s;
    s += cl;
    if (ct == 0x00) {
      uint64_t v = 0;
      int shift = 0;
      for (size_t i = 0; 4 + i < cl && i < 10; i++) {
        v |= uint64_t(b[4 + i] & 0x7f) << shift;
        if (b[4 + i] < 0x80) {
          total += std::min<uint64_t>(v, kMaxBlock);
          break;
        }
        shift += 7;
      }
    } else if (ct == 0x01 && cl >= 4) {
      total += std::min<size_t>(cl - 4, kMaxBlock);
    }
  }
  return total;
}

void snappy_framed_decode(const uint8_t *src, size_t n, std::vector<uint8_t> &out) {
  out.clear();
  // one allocation (and one zero fill) for the whole stream instead of a growing vector; the
  // chunk headers are not checked yet, so the reserve is capped (a corrupt header can claim
  // 64 KiB for an 11-byte chunk) and the vector grows past it if it must
  out.reserve(std::min<size_t>(snappy_framed_size(src, n), 16 * n + (size_t(1) << 20)));
  size_t s = 0;
  bool hdr = false;
  while (s < n) {
    if (n - s < 4) fail(TSG_E_CORRUPT, "snappy: truncated chunk header");
    uint8_t ct = src[s];
    size_t cl = size_t(src[s + 1]) | (size_t(src[s + 2]) << 8) | (size_t(src[s + 3]) << 16);
    s += 4;
    if (!hdr) {
      if (ct != 0xff) fail(TSG_E_CORRUPT, "snappy: missing stream identifier");
      hdr = true;
    }
    if (cl > kMaxEnc + 4) fail(TSG_E_CORRUPT, "snappy: chunk too large");
    if (cl > n - s) fail(TSG_E_CORRUPT, "snappy: truncated chunk");
    const uint8_t *b = src + s;
    s += cl;
    if (ct == 0x00 || ct == 0x01) {
      if (cl < 4) fail(TSG_E_CORRUPT, "snappy: chunk without checksum");
      uint32_t csum = le32(b);
      size_t base = out.size();
      if (ct == 0x00) {
        // varint decoded length (decode.go:30-43)
        uint64_t v = 0;
        size_t i = 0;
        int shift = 0;
        for (;; i++) {
          if (4 + i >= cl || i >= 10) fail(TSG_E_CORRUPT, "snappy: bad varint");
          uint8_t c = b[4 + i];
          v |= uint64_t(c & 0x7f) << shift;
          if (c < 0x80) break;
          shift += 7;
        }
        if (v > kMaxBlock) fail(TSG_E_CORRUPT, "snappy: block too large");
        out.resize(base + v);
        snappy_block_decode(b + 5 + i, cl - 5 - i, out.data() + base, v);
      } else {
        if (cl - 4 > kMaxBlock) fail(TSG_E_CORRUPT, "snappy: block too large");
        out.insert(out.end(), b + 4, b + cl);
      }
      if (snappy_mask(crc32c(out.data() + base, out.size() - base)) != csum)
        fail(TSG_E_CORRUPT, "snappy: checksum mismatch");
    } else if (ct == 0xff) {
      if (cl != 6 || std::memcmp(b, "sNaPpY", 6) != 0) fail(TSG_E_CORRUPT, "snappy: bad stream identifier");
    } else if (ct <= 0x7f) {
      fail(TSG_E_CORRUPT, "snappy: reserved unskippable chunk");
    }
  }
}

// Block encoder: greedy LZ77 with a 2^14 hash table over 4-byte windows. Any
// valid snappy block decodes identically; byte-identity with the Go encoder is
// not required (writer byte layout is not a parity surface).
static void emit_literal(std::vector<uint8_t> &o, const uint8_t *p, size_t n) {
  size_t m = n - 1;
  if (m < 60) {
    o.push_back(uint8_t(m << 2));
  } else if (m < 256) {
    o.push_back(60 << 2);
    o.push_back(uint8_t(m));
  } else {
    o.push_back(61 << 2);
    o.push_back(uint8_t(m));
    o.push_back(uint8_t(m >> 8));
  }
  o.insert(o.end(), p, p + n);
}
static void emit_copy(std::vector<uint8_t> &o, size_t off, size_t len) {
  while (len >= 68) {
    o.push_back(uint8_t(63 << 2 | 2));
    o.push_back(uint8_t(off));
    o.push_back(uint8_t(off >> 8));
    len -= 64;
  }
  if (len > 64) {
    o.push_back(uint8_t(59 << 2 | 2));
    o.push_back(uint8_t(off));
    o.push_back(uint8_t(off >> 8));
    len -= 60;
  }
  if (len >= 12 || off >= 2048) {
    o.push_back(uint8_t((len - 1) << 2 | 2));
    o.push_back(uint8_t(off));
    o.push_back(uint8_t(off >> 8));
  } else {
    o.push_back(uint8_t(((off >> 8) << 5) | ((len - 4) << 2) | 1));
    o.push_back(uint8_t(off));
  }
}
static void snappy_block_encode(const uint8_t *src, size_t n, std::vector<uint8_t> &o) {
  o.clear();
  uint64_t v = n;
  while (v >= 0x80) {
    o.push_back(uint8_t(v | 0x80));
    v >>= 7;
  }
  o.push_back(uint8_t(v));
  if (n < 16) {
    if (n) emit_literal(o, src, n);
    return;
  }
  static thread_local std::vector<int32_t> table;
  table.assign(1 << 14, -1);
  size_t lit = 0, i = 0;
  const size_t limit = n - 4;
  size_t skip = 32;
  while (i <= limit) {
    uint32_t w = le32(src + i);
    uint32_t h = (w * 0x1e35a7bdu) >> 18;
    int32_t c = table[h];
    table[h] = int32_t(i);
    if (c >= 0 && le32(src + c) == w && i - size_t(c) < 65536) {
      size_t len = 4;
      while (i + len < n && src[c + len] == src[i + len]) len++;
      if (i > lit) emit_literal(o, src + lit, i - lit);
      emit_copy(o, i - size_t(c), len);
      i += len;
      lit = i;
      skip = 32;
    } else {
      i += skip++ >> 5;
    }
  }
  if (lit < n) emit_literal(o, src + lit, n - lit);
}

void snappy_framed_encode(const uint8_t *src, size_t n, std::vector<uint8_t> &out) {
  static const uint8_t magic[10] = {0xff, 0x06, 0x00, 0x00, 's', 'N', 'a', 'P', 'p', 'Y'};
  out.insert(out.end(), magic, magic + 10);
  std::vector<uint8_t> comp;
  for (size_t off = 0; off < n; off += kMaxBlock) {
    size_t len = n - off < kMaxBlock ? n - off : kMaxBlock;
    const uint8_t *u = src + off;
    uint32_t csum = snappy_mask(crc32c(u, len));
    snappy_block_encode(u, len, comp);
    bool use_comp = comp.size() < len - len / 8;
    size_t cl = 4 + (use_comp ? comp.size() : len);
    out.push_back(use_comp ? 0x00 : 0x01);
    out.push_back(uint8_t(cl));
    out.push_back(uint8_t(cl >> 8));
    out.push_back(uint8_t(cl >> 16));
    put_le32(out, csum);
    if (use_comp) out.insert(out.end(), comp.begin(), comp.end());
    else out.insert(out.end(), u, u + len);
  }
}

// ---- strings.ToLower ------------------------------------------------------------
static uint32_t uni_lower(uint32_t r) {
  if (r >= 'A' && r <= 'Z') return r + 32;
  if (r < 0x80) return r;
  if (r >= 0xC0 && r <= 0xDE && r != 0xD7) return r + 32;
  if (r == 0x130) return 0x69;
  if (r == 0x178) return 0xFF;
  if ((r >= 0x100 && r <= 0x12F) || (r >= 0x132 && r <= 0x137) || (r >= 0x14A && r <= 0x177))
    return (r & 1) ? r : r + 1;
  if ((r >= 0x139 && r <= 0x148) || (r >= 0x179 && r <= 0x17E)) return (r & 1) ? r + 1 : r;
  if (r == 0x386) return 0x3AC;
  if (r >= 0x388 && r <= 0x38A) return r + 37;
  if (r == 0x38C) return 0x3CC;
  if (r == 0x38E || r == 0x38F) return r + 63;
  if ((r >= 0x391 && r <= 0x3A1) || (r >= 0x3A3 && r <= 0x3AB)) return r + 32;
  if (r >= 0x400 && r <= 0x40F) return r + 80;
  if (r >= 0x410 && r <= 0x42F) return r + 32;
  if (r >= 0x531 && r <= 0x556) return r + 48;
  return r;
}
std::string go_to_lower(std::string_view s) {
  bool ascii = true;
  for (unsigned char c : s)
    if (c >= 0x80) {
      ascii = false;
      break;
    }
  std::string o;
  o.reserve(s.size());
  if (ascii) {
    for (unsigned char c : s) o.push_back(char(c >= 'A' && c <= 'Z' ? c + 32 : c));
    return o;
  }
  const auto *p = reinterpret_cast<const uint8_t *>(s.data());
  size_t n = s.size();
  for (size_t i = 0; i < n;) {
    uint8_t c = p[i];
    uint32_t r = 0xFFFD;
    size_t w = 1, need = 0;
    uint32_t minv = 0;
    if (c < 0x80) { r = c; need = 1; }
    else if (c >= 0xC2 && c <= 0xDF) { need = 2; r = c & 0x1F; minv = 0x80; }
    else if (c >= 0xE0 && c <= 0xEF) { need = 3; r = c & 0x0F; minv = 0x800; }
    else if (c >= 0xF0 && c <= 0xF4) { need = 4; r = c & 0x07; minv = 0x10000; }
    if (need > 1) {
      bool ok = n - i >= need;
      for (size_t k = 1; ok && k < need; k++) {
        if ((p[i + k] & 0xC0) != 0x80) ok = false;
        else r = (r << 6) | (p[i + k] & 0x3F);
      }
      if (ok && !(r < minv || r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF))) w = need;
      else r = 0xFFFD;
    } else if (need == 0) {
      r = 0xFFFD;
    }
    r = uni_lower(r);
    if (r < 0x80) o.push_back(char(r));
    else if (r < 0x800) { o.push_back(char(0xC0 | (r >> 6))); o.push_back(char(0x80 | (r & 0x3F))); }
    else if (r < 0x10000) {
      o.push_back(char(0xE0 | (r >> 12))); o.push_back(char(0x80 | ((r >> 6) & 0x3F))); o.push_back(char(0x80 | (r & 0x3F)));
    } else {
      o.push_back(char(0xF0 | (r >> 18))); o.push_back(char(0x80 | ((r >> 12) & 0x3F)));
      o.push_back(char(0x80 | ((r >> 6) & 0x3F))); o.push_back(char(0x80 | (r & 0x3F)));
    }
    i += w;
  }
  return o;
}

// ---- files ----------------------------------------------------------------------
bool read_file(const std::string &path, std::vector<uint8_t> &out) {
  FILE *f = std::fopen(path.c_str(), "rb");
  if (!f) {
    if (errno == ENOENT) return false;
    fail(TSG_E_IO, "open " + path + ": " + std::strerror(errno));
  }
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? size_t(n) : 0);
  if (n > 0 && std::fread(out.data(), 1, size_t(n), f) != size_t(n)) {
    std::fclose(f);
    fail(TSG_E_IO, "short read " + path);
  }
  std::fclose(f);
  return true;
}
bool read_file(const std::string &path, Bytes &out) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (errno == ENOENT) return false;
    fail(TSG_E_IO, "open " + path + ": " + std::strerror(errno));
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    fail(TSG_E_IO, "stat " + path + ": " + std::strerror(errno));
  }
  const size_t n = st.st_size > 0 ? size_t(st.st_size) : 0;
  out.resize(n);
  advise_huge(out.data(), n);
  // chunks of 32 MiB on up to 8 threads (one pread loop each)
  std::atomic<bool> bad{false};
  parallel_ranges(n, size_t(32) << 20, 8, [&](size_t lo, size_t hi) {
    while (lo < hi) {
      const ssize_t r = ::pread(fd, out.data() + lo, hi - lo, off_t(lo));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) {
        bad.store(true);
        return;
      }
      lo += size_t(r);
    }
  });
  ::close(fd);
  if (bad.load()) fail(TSG_E_IO, "short read " + path);
  return true;
}
void write_file(const std::string &path, const uint8_t *p, size_t n) {
  FILE *f = std::fopen(path.c_str(), "wb");
  if (!f) fail(TSG_E_IO, "create " + path + ": " + std::strerror(errno));
  if (n && std::fwrite(p, 1, n, f) != n) {
    std::fclose(f);
    fail(TSG_E_IO, "short write " + path);
  }
  std::fclose(f);
}
void make_dirs(const std::string &path) {
  std::string cur;
  for (size_t i = 0; i <= path.size(); i++) {
    if (i == path.size() || path[i] == '/') {
      if (!cur.empty()) ::mkdir(cur.c_str(), 0755);
    }
    if (i < path.size()) cur.push_back(path[i]);
  }
}

static const char *kEncNames[] = {"none", "gzip", "lz4-64k", "lz4-256k", "lz4-1M", "lz4", "snappy", "zstd", "s2"};
int parse_encoding(std::string_view s) {
  for (int i = 0; i < 9; i++) {
    std::string_view n = kEncNames[i];
    if (n.size() == s.size() && ::strncasecmp(n.data(), s.data(), s.size()) == 0) return i;
  }
  return -1;
}
const char *encoding_name(int e) { return (e >= 0 && e < 9) ? kEncNames[e] : "unsupported"; }

namespace {
struct ProfTable {
  std::mutex mu;
  std::vector<std::pair<std::string, std::vector<double>>> rows;
  ~ProfTable() { dump(nullptr); }
  void dump(const char *label) {
    if (rows.empty()) return;
    if (label) std::fprintf(stderr, "[tsg] prof [%s]\n", label);
    std::fprintf(stderr, "[tsg] prof p50 us:");
    for (auto &r : rows) {
      std::sort(r.second.begin(), r.second.end());
      std::fprintf(stderr, " %s=%.2f", r.first.c_str(), r.second[r.second.size() / 2]);
    }
    std::fprintf(stderr, " (n=%zu)\n", rows[0].second.size());
    std::fprintf(stderr, "[tsg] prof p90/p99/max us:");
    for (auto &r : rows) {
      const auto &v = r.second;
      std::fprintf(stderr, " %s=%.1f/%.1f/%.1f(n=%zu)", r.first.c_str(), v[v.size() * 9 / 10], v[v.size() * 99 / 100],
                   v.back(), v.size());
    }
    std::fprintf(stderr, "\n");
  }
};
ProfTable &prof_table() {
  static ProfTable t;
  return t;
}
}  // namespace

// Diagnostics (TSG_PROF): print the phase table so far under `label` and start a new one
// (tools/c45_prof.py: one table per query). Not part of include/tsg.h.
extern "C" __attribute__((visibility("default"))) void tsgx_prof_flush(const char *label) {
  ProfTable &t = prof_table();
  std::lock_guard<std::mutex> lk(t.mu);
  t.dump(label ? label : "");
  t.rows.clear();
}
int host_threads() {
  static const int n = [] {
    int c = int(std::max(1u, std::thread::hardware_concurrency()));
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) c = std::max(1, std::min(c, CPU_COUNT(&set)));
    // a cgroup CPU quota (cpu.max "quota period"): the CPUs' worth of time this job may use
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {};
      long long period = 0;
      if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
        c = std::max(1, std::min(c, int((std::atoll(q) + period - 1) / period)));
      std::fclose(f);
    }
    return c;
  }();
  return n;
}

void advise_huge(void *p, size_t bytes) {
  constexpr uintptr_t kHuge = uintptr_t(2) << 20;
  if (!p || bytes < 2 * kHuge) return;
  const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kHuge - 1);
  if (b > a) madvise(reinterpret_cast<void *>(a), b - a, MADV_HUGEPAGE);
}

int host_threads_now() {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) return std::max(1, std::min(host_threads(), CPU_COUNT(&set)));
  return host_threads();
}

void parallel_ranges(size_t n, size_t grain, int max_threads, const std::function<void(size_t, size_t)> &f) {
  if (n == 0) return;
  const size_t hw = size_t(host_threads_now());
  size_t nt = std::min<size_t>({size_t(std::max(1, max_threads)), hw, (n + std::max<size_t>(grain, 1) - 1) /
                                                                        std::max<size_t>(grain, 1)});
  if (nt <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::exception_ptr> errs(nt);
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (size_t t = 1; t < nt; t++)
    th.emplace_back([&, t] {
      try {
        f(n * t / nt, n * (t + 1) / nt);
      } catch (...) {
        errs[t] = std::current_exception();
      }
    });
  try {
    f(0, n / nt);
  } catch (...) {
    errs[0] = std::current_exception();
  }
  for (auto &x : th) x.join();
  for (auto &e : errs)
    if (e) std::rethrow_exception(e);
}

bool prof_on() {
  static const bool on = std::getenv("TSG_PROF") != nullptr;
  return on;
}
void prof_add(const char *name, double us) {
  ProfTable &t = prof_table();
  std::lock_guard<std::mutex> lk(t.mu);
  for (auto &r : t.rows)
    if (r.first == name) {
      r.second.push_back(us);
      return;
    }
  t.rows.push_back({name, {us}});
}

}  // namespace tsg
