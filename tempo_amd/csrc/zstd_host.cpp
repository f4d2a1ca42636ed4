// zstd_host.cpp — the zstd frame decoder of zstd_dev.hpp built for the host: the proto
// loader (proto.cpp) decodes zstd data pages once at open (the v2 data default,
// modules/storage/config.go:39-53; reference: klauspost/compress/zstd DecodeAll,
// tempodb/encoding/v2/data_reader.go:111-117). findOne runs the same code on the GPU.
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>
#define __device__
#define __constant__
#define __forceinline__ inline
static inline int __clz(uint32_t x) { return x ? __builtin_clz(x) : 32; }
#include "tsg.h"
#define TSG_ZSTD_HOST
#include "zstd_dev.hpp"

namespace tsg {

int zstd_host_decode(const uint8_t *src, size_t n, std::vector<uint8_t> &out) {
  if (n > 0xffffffffu) return TSG_E_CORRUPT;
  // 8-byte aligned copy with slack on both sides (the backward bit reader loads whole words)
  std::vector<uint64_t> al((n + 64) / 8 + 2, 0);
  uint8_t *base = reinterpret_cast<uint8_t *>(al.data()) + 8;
  std::memcpy(base, src, n);
  thread_local std::unique_ptr<zdev::Work> W;
  if (!W) W.reset(new zdev::Work);
  uint64_t bound = 0;
  int st = zdev::zstd_size(base, uint32_t(n), bound);
  if (st != TSG_OK) return st;
  out.assign(bound + 16, 0);
  uint64_t len = 0;
  st = zdev::zstd_decode(base, uint32_t(n), out.data(), bound, len, *W);
  if (st != TSG_OK) return st;
  out.resize(len);
  return TSG_OK;
}

}  // namespace tsg
