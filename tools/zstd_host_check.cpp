// zstd_host_check.cpp — builds the device zstd decoder (tempo_amd/csrc/zstd_dev.hpp) for the
// host and decodes every page of a v2 data file, writing the decoded pages to stdout as
// [u32 len][bytes] (or [u32 0xffffffff][i32 status]) so a test can compare them with an
// independent zstd (pyarrow / libzstd). Test tooling: the product runs the same code on the GPU.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define __device__
#define __constant__
#define __forceinline__ inline
static inline int __clz(uint32_t x) { return x ? __builtin_clz(x) : 32; }
#include "../include/tsg.h"
#define TSG_ZSTD_HOST
#include "../tempo_amd/csrc/zstd_dev.hpp"

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> d;
  uint8_t buf[65536];
  size_t r;
  while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + r);
  std::fclose(f);
  // 8-byte aligned copy with slack on both sides (the backward reader loads whole words)
  std::vector<uint64_t> al((d.size() + 64) / 8 + 2, 0);
  uint8_t *base = reinterpret_cast<uint8_t *>(al.data()) + 8;
  std::memcpy(base, d.data(), d.size());
  auto *W = new tsg::zdev::Work;
  size_t off = 0;
  while (off + 6 <= d.size()) {
    uint32_t tl;
    std::memcpy(&tl, base + off, 4);
    const uint8_t *p = base + off + 6;
    const uint32_t n = tl - 6;
    uint64_t bound = 0;
    int st = tsg::zdev::zstd_size(p, n, bound);
    std::vector<uint8_t> out(bound + 16);
    uint64_t len = 0;
    if (st == TSG_OK) st = tsg::zdev::zstd_decode(p, n, out.data(), bound, len, *W);
    if (st != TSG_OK) {
      uint32_t m = 0xffffffffu;
      std::fwrite(&m, 4, 1, stdout);
      std::fwrite(&st, 4, 1, stdout);
    } else {
      uint32_t l = uint32_t(len);
      std::fwrite(&l, 4, 1, stdout);
      std::fwrite(out.data(), 1, len, stdout);
    }
    off += tl;
  }
  return 0;
}
