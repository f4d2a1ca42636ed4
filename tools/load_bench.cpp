// Host-only timing of the columnar loader (decode_search_block, no device): one block,
// or the same block decoded by N threads at once (bench.py opens its 10 blocks that way).
// Build: g++ -O2 -std=c++17 tools/load_bench.cpp -Itempo_amd/csrc -Iinclude -Ltempo_amd -ltsg
//        -Wl,-rpath,$PWD/tempo_amd -lpthread -o /tmp/load_bench
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include "block.hpp"
int main(int argc, char **argv) {
  using namespace tsg;
  if (argc < 2) return 2;
  const std::string d = argv[1];
  const int par = argc > 2 ? std::atoi(argv[2]) : 1, nth = argc > 3 ? std::atoi(argv[3]) : 0;
  std::vector<uint8_t> m, h, i, s;
  read_file(d + "/search.meta.json", m);
  read_file(d + "/search-header", h);
  read_file(d + "/search-index", i);
  read_file(d + "/search", s);
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  std::vector<uint64_t> fb(par);
  for (int k = 0; k < par; k++)
    th.emplace_back([&, k] {
      HostBlock hb;
      decode_search_block(m.data(), m.size(), true, h, i.data(), i.size(), s.data(), s.size(), nth, hb);
      fb[k] = hb.fb_bytes;
    });
  for (auto &x : th) x.join();
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t tot = 0;
  for (auto x : fb) tot += x;
  std::printf("{\"blocks\": %d, \"s\": %.3f, \"fb_gb\": %.3f, \"gb_per_s\": %.3f}\n", par, sec, tot / 1e9, tot / 1e9 / sec);
  return 0;
}
