// Host-only probe of the search-block loader (block.cpp decode_search_block), no GPU: writes
// synthetic config-2 blocks (synth.cpp) once, then decodes K of them at once, each on its share
// of T threads, R times, and prints the wall time per round and the TSG_PROF phase table.
// Build (tools/probe/Makefile.decode): g++ -O3 -std=c++17 -pthread -I include ... -o /tmp/decode_probe
// Run: TSG_PROF=1 /tmp/decode_probe <dir> <entries> <blocks K> <threads T> <rounds R>
#include <sys/stat.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../tempo_amd/csrc/block.hpp"
#include "../../tempo_amd/csrc/common.hpp"

namespace tsg {
void synth_search_block(const std::string &dir, uint64_t n, uint64_t seed, int profile, int enc, uint32_t page_size);
}

int main(int argc, char **argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s dir entries blocks threads rounds [profile]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const uint64_t n = std::strtoull(argv[2], nullptr, 10);
  const int K = std::atoi(argv[3]), T = std::atoi(argv[4]), R = std::atoi(argv[5]);
  const int profile = argc > 6 ? std::atoi(argv[6]) : 0;
  std::vector<std::string> paths;
  for (int k = 0; k < K; k++) {
    const std::string p = dir + "/b" + std::to_string(k);
    struct stat st;
    if (stat((p + "/search.meta.json").c_str(), &st) != 0) tsg::synth_search_block(p, n, 100 + k, profile, 6 /* snappy */, 1 << 20);
    paths.push_back(p);
  }
  struct Files {
    std::vector<uint8_t> meta, index, data;
  };
  std::vector<Files> files(K);
  uint64_t bytes = 0;
  for (int k = 0; k < K; k++) {
    tsg::read_file(paths[k] + "/search.meta.json", files[k].meta);
    tsg::read_file(paths[k] + "/search-index", files[k].index);
    tsg::read_file(paths[k] + "/search", files[k].data);
    bytes += files[k].data.size();
  }
  for (int r = 0; r < R; r++) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int k = 0; k < K; k++)
      th.emplace_back([&, k] {
        tsg::Bytes header;
        tsg::read_file(paths[k] + "/search-header", header);
        tsg::HostBlock hb;
        tsg::decode_search_block(files[k].meta.data(), files[k].meta.size(), true, std::move(header),
                                 files[k].index.data(), files[k].index.size(), files[k].data.data(),
                                 files[k].data.size(), 0, hb);
        if (k == 0 && r == 0 && std::getenv("DECODE_KEYS"))
          for (const auto &kc : hb.keys)
            std::printf("key %-24s nvals %8u dict %10zu B nsets %8u\n", kc.name.c_str(), kc.nvals(), kc.dict_bytes.size(),
                        kc.nsets());
      });
    for (auto &t : th) t.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("round %d: %d blocks x %llu entries, %.3f s, %.2f GB/s of flatbuffer (T=%d)\n", r, K,
                (unsigned long long)n, s, double(bytes) / s / 1e9, T);
  }
  return 0;
}
