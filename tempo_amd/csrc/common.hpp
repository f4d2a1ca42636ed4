// common.hpp — shared host utilities of libtsg: byte order, status/errors,
// hashes used by the on-disk formats, snappy framing (decode + encode).
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <new>
#include <stdexcept>
#include <type_traits>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "../../include/tsg.h"

namespace tsg {

// ---- errors ---------------------------------------------------------------
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
[[noreturn]] inline void fail(int code, const std::string &msg) { throw Error(code, msg); }
void set_last_error(const std::string &m);

// ---- byte order (encoding/binary) -------------------------------------------
inline uint16_t le16(const uint8_t *p) { return uint16_t(p[0] | (p[1] << 8)); }
inline uint32_t le32(const uint8_t *p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t le64(const uint8_t *p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
inline uint64_t be64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
  return v;
}
inline void put_le16(std::vector<uint8_t> &o, uint16_t v) {
  o.push_back(uint8_t(v));
  o.push_back(uint8_t(v >> 8));
}
inline void put_le32(std::vector<uint8_t> &o, uint32_t v) {
  for (int i = 0; i < 4; i++) o.push_back(uint8_t(v >> (8 * i)));
}
inline void put_le64(std::vector<uint8_t> &o, uint64_t v) {
  for (int i = 0; i < 8; i++) o.push_back(uint8_t(v >> (8 * i)));
}
inline void put_be64(std::vector<uint8_t> &o, uint64_t v) {
  for (int i = 7; i >= 0; i--) o.push_back(uint8_t(v >> (8 * i)));
}

// bytes.Compare
inline int bytes_compare(const uint8_t *a, size_t al, const uint8_t *b, size_t bl) {
  size_t n = al < bl ? al : bl;
  int c = n ? std::memcmp(a, b, n) : 0;
  if (c) return c < 0 ? -1 : 1;
  return al == bl ? 0 : (al < bl ? -1 : 1);
}

// ---- hashes -----------------------------------------------------------------
uint64_t xxhash64(const uint8_t *p, size_t n);  // cespare/xxhash Sum64 (seed 0)
// A meta.json number field as uint32 (decimal digits only, <= 2^32-1); anything else -> TSG_E_CORRUPT
uint32_t json_u32(std::string_view v, const char *field);
uint32_t fnv1_32(const uint8_t *p, size_t n);   // hash/fnv New32 (pkg/util/hash.go:15-20)
void murmur3_128(const uint8_t *p, size_t n, uint64_t &h1, uint64_t &h2);  // spaolacci/murmur3 Sum128
uint32_t crc32c(const uint8_t *p, size_t n);

// Streaming xxhash64 for writeKeyValues' cache key (searchdatamap.go:115-128).
struct XXH64Stream {
  std::vector<uint8_t> buf;
  void reset() { buf.clear(); }
  void write(const void *p, size_t n) {
    auto *b = static_cast<const uint8_t *>(p);
    buf.insert(buf.end(), b, b + n);
  }
  uint64_t sum() const { return xxhash64(buf.data(), buf.size()); }
};

// ---- snappy framing (github.com/golang/snappy v0.0.4 wire format) ------------
// Decode a complete framed stream (one v2 data page payload).
void snappy_framed_decode(const uint8_t *src, size_t n, std::vector<uint8_t> &out);
// Encode like snappy.NewBufferedWriter + Close: stream identifier, 64 KiB chunks,
// compressed unless the saving is < 12.5 % (encode.go:218-235).
void snappy_framed_encode(const uint8_t *src, size_t n, std::vector<uint8_t> &out);

// ---- strings.ToLower (ASCII exact, documented subset beyond) ---
std::string go_to_lower(std::string_view s);

// ---- files --------------------------------------------------------------------
bool read_file(const std::string &path, std::vector<uint8_t> &out);  // false if missing

// A byte vector whose resize leaves new bytes uninitialised (a file's bytes are written
// once by the read: no zero fill of a 1 GB header first).
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    if constexpr (sizeof...(A) == 0) ::new (static_cast<void *>(p)) U;
    else ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
  }
};
using Bytes = std::vector<uint8_t, NoInitAlloc<uint8_t>>;
// Large files are read with parallel preads (several threads copying from the page cache)
// into huge-page advised memory; false if missing.
bool read_file(const std::string &path, Bytes &out);
void write_file(const std::string &path, const uint8_t *p, size_t n);
void make_dirs(const std::string &path);

// ---- host parallelism -----------------------------------------------------------
// CPUs this process may use: its affinity mask, capped by a cgroup CPU quota (a GPU box's
// job share); std::thread::hardware_concurrency counts the whole machine
int host_threads();
// the same, for the calling thread's current affinity (a caller pinned to a few CPUs)
int host_threads_now();
// f(lo, hi) over [0, n) split into contiguous ranges of at least `grain` items, on up to
// max_threads threads (the caller runs the first range). Exceptions: the first is rethrown.
void parallel_ranges(size_t n, size_t grain, int max_threads, const std::function<void(size_t, size_t)> &f);

// A growable array of trivially copyable T without value-initialisation on resize (a result
// of millions of records is written once; zero-filling it first would be a second pass).
// Large host arrays written once per query (result columns, record vectors): ask for
// transparent huge pages on the 2 MiB-aligned interior before its first touch (THP is
// "madvise" on the GPU hosts; 4 KiB pages cost the dense result fill a TLB miss per few records).
void advise_huge(void *p, size_t bytes);

template <class T>
struct RawVec {
  static_assert(std::is_trivially_copyable<T>::value, "RawVec holds plain data");
  T *p = nullptr;
  size_t n = 0, cap = 0;
  RawVec() = default;
  RawVec(const RawVec &) = delete;
  RawVec &operator=(const RawVec &) = delete;
  ~RawVec() { std::free(p); }
  void reserve(size_t c) {
    if (c <= cap) return;
    T *q = static_cast<T *>(std::realloc(p, c * sizeof(T)));
    if (!q) throw std::bad_alloc();
    p = q;
    cap = c;
    advise_huge(p, c * sizeof(T));
  }
  void resize(size_t m) {
    if (m > cap) reserve(std::max(m, cap * 2));
    n = m;
  }
  void assign(size_t m, const T &v) {
    resize(m);
    for (size_t i = 0; i < m; i++) p[i] = v;
  }
  void push_back(const T &v) {
    if (n == cap) reserve(std::max<size_t>(16, cap * 2));
    p[n++] = v;
  }
  void clear() { n = 0; }
  size_t size() const { return n; }
  size_t capacity() const { return cap; }
  bool empty() const { return n == 0; }
  T *data() { return p; }
  const T *data() const { return p; }
  T &operator[](size_t i) { return p[i]; }
  const T &operator[](size_t i) const { return p[i]; }
  T &back() { return p[n - 1]; }
};

// backend.Encoding names (tempodb/backend/encoding.go:40-62)
int parse_encoding(std::string_view s);
// TSG_PROF=1: host phase times accumulated per name, averages printed at exit
bool prof_on();
void prof_add(const char *name, double us);
const char *encoding_name(int e);

}  // namespace tsg
