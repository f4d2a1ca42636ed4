// san_host.cpp — TEST INFRASTRUCTURE ONLY: libtsg's host parsers under AddressSanitizer + UBSan
// (tests/sanitize/Makefile, tests/test_sanitizers.py). No GPU.
//
// 1. The search-block loader (block.cpp decode_search_block, the parallel three-phase decode of
//    untrusted on-disk bytes) over synthetic blocks (snappy and none), then a corruption fuzz:
//    random bytes of one of the four files flipped, runs of bytes zeroed, files truncated; every
//    decode either succeeds or throws a tsg error — never an out-of-bounds access.
// 2. The v2 trace blocks the reference ships (tests/golden/v2test: snappy, tests/golden/tempo_cli:
//    zstd): index pages (xxhash64 checksums) and data pages decoded, then fuzzed the same way.
// 3. snappy framing round trips, and the host zstd decoder on corrupted frames.
// Usage: san_host <tmpdir> <golden dir> <fuzz iterations>
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../tempo_amd/csrc/block.hpp"
#include "../../tempo_amd/csrc/common.hpp"
#include "../../tempo_amd/csrc/writer.hpp"

using namespace tsg;

static std::vector<uint8_t> slurp(const std::string &p) {
  std::vector<uint8_t> v;
  FILE *f = std::fopen(p.c_str(), "rb");
  if (!f) return v;
  std::fseek(f, 0, SEEK_END);
  v.resize(size_t(std::ftell(f)));
  std::fseek(f, 0, SEEK_SET);
  if (!v.empty() && std::fread(v.data(), 1, v.size(), f) != v.size()) v.clear();
  std::fclose(f);
  return v;
}

static void mutate(std::vector<uint8_t> &v, std::mt19937_64 &rng) {
  if (v.empty()) return;
  switch (rng() % 4) {
    case 0:  // flip a few bytes
      for (int i = 0, k = 1 + int(rng() % 8); i < k; i++) v[rng() % v.size()] ^= uint8_t(1 + rng() % 255);
      break;
    case 1: {  // zero a run
      const size_t a = rng() % v.size(), l = std::min<size_t>(v.size() - a, 1 + rng() % 64);
      std::memset(v.data() + a, 0, l);
      break;
    }
    case 2:  // truncate
      v.resize(rng() % v.size());
      break;
    default: {  // a large length field: 0xff bytes at a word
      const size_t a = rng() % v.size();
      for (size_t i = a; i < std::min(v.size(), a + 4); i++) v[i] = 0xff;
    }
  }
}

struct SearchFiles {
  std::vector<uint8_t> meta, header, index, data;
};

static bool decode(const SearchFiles &f, uint64_t *entries) {
  try {
    Bytes hdr;
    hdr.resize(f.header.size());
    if (!f.header.empty()) std::memcpy(hdr.data(), f.header.data(), f.header.size());
    HostBlock hb;
    decode_search_block(f.meta.data(), f.meta.size(), true, std::move(hdr), f.index.data(), f.index.size(),
                        f.data.data(), f.data.size(), 2, hb);
    if (entries) *entries = hb.n;
    return true;
  } catch (const Error &) {
    return false;
  }
}

static int fail_count = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      fail_count++;                                                \
    }                                                              \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s tmpdir golden iters\n", argv[0]);
    return 2;
  }
  const std::string tmp = argv[1], golden = argv[2];
  const int iters = std::atoi(argv[3]);
  std::mt19937_64 rng(12345);
  // ---- 1. search blocks
  for (int enc : {6 /* snappy */, 0 /* none */}) {
    const std::string dir = tmp + "/blk" + std::to_string(enc);
    synth_search_block(dir, 20000, 77 + uint64_t(enc), 0, enc, 32 << 10);
    SearchFiles f{slurp(dir + "/search.meta.json"), slurp(dir + "/search-header"), slurp(dir + "/search-index"),
                  slurp(dir + "/search")};
    uint64_t n = 0;
    CHECK(decode(f, &n));
    CHECK(n == 20000);
    int ok = 0, bad = 0;
    for (int it = 0; it < iters; it++) {
      SearchFiles g = f;
      std::vector<uint8_t> *which[] = {&g.meta, &g.header, &g.index, &g.data};
      mutate(*which[rng() % 4], rng);
      (decode(g, nullptr) ? ok : bad)++;
    }
    std::printf("search enc %d: %d decodes ok, %d rejected under corruption\n", enc, ok, bad);
  }
  // ---- 2. the reference's v2 blocks: index + data pages
  struct V2 {
    const char *name;
    uint32_t page_size, total;
    int enc;
  } v2s[] = {{"v2test", 1000, 2, 6}, {"tempo_cli", 256000, 611, 7}};
  for (const V2 &b : v2s) {
    const std::vector<uint8_t> index = slurp(golden + "/" + b.name + "/index"), data = slurp(golden + "/" + b.name + "/data");
    CHECK(!index.empty() && !data.empty());
    std::vector<IndexRecord> recs;
    try {
      recs = read_index(index.data(), index.size(), b.page_size, b.total);
    } catch (const Error &e) {
      std::fprintf(stderr, "%s index: %s\n", b.name, e.what());
    }
    CHECK(recs.size() == b.total);
    size_t pages = 0;
    std::vector<uint8_t> out;
    for (const auto &r : recs) {
      try {
        read_data_page(data.data(), data.size(), r, b.enc, out);
        pages++;
      } catch (const Error &e) {
        std::fprintf(stderr, "%s page: %s\n", b.name, e.what());
      }
    }
    CHECK(pages == recs.size());
    int rej = 0;
    for (int it = 0; it < iters; it++) {
      std::vector<uint8_t> ix = index, dt = data;
      mutate(rng() % 2 ? ix : dt, rng);
      try {
        bool prefix = false;
        const auto rr = read_index(ix.data(), ix.size(), b.page_size, b.total, &prefix);
        for (size_t k = 0; k < rr.size() && k < 16; k++) read_data_page(dt.data(), dt.size(), rr[(k * 37) % rr.size()], b.enc, out);
      } catch (const Error &) {
        rej++;
      }
    }
    std::printf("%s: %zu records, %zu pages decoded; fuzz: %d of %d rejected\n", b.name, recs.size(), pages, rej, iters);
  }
  // ---- 3. snappy framing round trips + the host zstd decoder on corrupted frames
  for (int it = 0; it < 64; it++) {
    std::vector<uint8_t> src(size_t(rng() % 300000));
    for (auto &x : src) x = uint8_t(rng() % 7 ? rng() % 16 : rng());  // (compressible)
    std::vector<uint8_t> enc, dec;
    snappy_framed_encode(src.data(), src.size(), enc);
    snappy_framed_decode(enc.data(), enc.size(), dec);
    CHECK(dec == src);
    mutate(enc, rng);
    try {
      snappy_framed_decode(enc.data(), enc.size(), dec);
    } catch (const Error &) {
    }
  }
  {
    const std::vector<uint8_t> index = slurp(golden + "/tempo_cli/index"), data = slurp(golden + "/tempo_cli/data");
    const auto recs = read_index(index.data(), index.size(), 256000, 611);
    int rej = 0;
    std::vector<uint8_t> out;
    for (int it = 0; it < iters; it++) {
      const IndexRecord &r = recs[size_t(rng() % recs.size())];
      // the page's zstd frame: after the v2 page header ([u32 total][u16 hdr len][hdr])
      std::vector<uint8_t> page(data.begin() + long(r.start), data.begin() + long(r.start + r.length));
      if (page.size() < 6) continue;
      const uint16_t hl = uint16_t(page[4] | page[5] << 8);
      std::vector<uint8_t> frame(page.begin() + std::min<long>(long(page.size()), 6 + hl), page.end());
      if (it == 0) CHECK(zstd_host_decode(frame.data(), frame.size(), out) == TSG_OK);  // (the frame as shipped)
      mutate(frame, rng);
      if (zstd_host_decode(frame.data(), frame.size(), out) != TSG_OK) rej++;
    }
    std::printf("zstd fuzz: %d of %d frames rejected\n", rej, iters);
  }
  std::printf("san_host: %s\n", fail_count ? "FAILED" : "ok");
  return fail_count ? 1 : 0;
}
