// Host-side probe of the dense result fill (capi.cpp fill_records_direct): gather a
// match's fields from per-entry columns at sorted positions (density ~18 %, config 4's
// statement+url query) into the 12 result arrays, on T threads. Prints ms per fill for
// the column gather, a plain sequential copy of the same output bytes, and a single-stream
// read, so the fill can be compared with what the host's memory gives.
// g++ -O2 -std=c++17 -pthread tools/probe/fill_probe.cpp -o /tmp/fill_probe
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;

template <class F>
static double run(int nt, size_t n, F &&f) {
  std::vector<std::thread> th;
  const auto t0 = clk::now();
  for (int t = 1; t < nt; t++) th.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt); });
  f(0, n / nt);
  for (auto &x : th) x.join();
  return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

int main(int argc, char **argv) {
  const int nt = argc > 1 ? std::atoi(argv[1]) : 16;
  const size_t nent = 1000000, nblk = 10;
  const double dens = argc > 2 ? std::atof(argv[2]) : 0.185;
  std::vector<uint8_t> ids(16 * nent), il(nent);
  std::vector<uint64_t> st(nent), en(nent);
  std::vector<uint32_t> sv(nent), nm(nent);
  std::mt19937_64 r(1);
  for (size_t e = 0; e < nent; e++) {
    for (int k = 0; k < 16; k++) ids[16 * e + k] = uint8_t(r());
    il[e] = 16;
    st[e] = r();
    en[e] = st[e] + (r() % 1000000000);
    sv[e] = uint32_t(r() % 20);
    nm[e] = uint32_t(r() % 200);
  }
  std::vector<uint64_t> pos;
  for (size_t b = 0; b < nblk; b++)
    for (size_t e = 0; e < nent; e++)
      if ((r() % 1000) < dens * 1000) pos.push_back(e | (uint64_t(b) << 32));
  const size_t n = pos.size();
  // output arrays: malloc'd (4 KiB pages), or with argv[3] = 1 mmap'd + MADV_HUGEPAGE before first touch
  const bool huge = argc > 3 && std::atoi(argv[3]) == 1;
  auto A = [&](size_t bytes) -> void * {
    if (!huge) return std::malloc(bytes);
    const size_t b = (bytes + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
    void *p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(p, b, MADV_HUGEPAGE);
    return p;
  };
  uint8_t *o_ids = (uint8_t *)A(16 * n), *o_il = (uint8_t *)A(n);
  uint64_t *o_st = (uint64_t *)A(8 * n), *o_en = (uint64_t *)A(8 * n), *o_entry = (uint64_t *)A(8 * n),
           *o_so = (uint64_t *)A(8 * n), *o_no = (uint64_t *)A(8 * n);
  uint32_t *o_dur = (uint32_t *)A(4 * n), *o_blk = (uint32_t *)A(4 * n), *o_sl = (uint32_t *)A(4 * n),
           *o_nl = (uint32_t *)A(4 * n);
  const char **o_sp = (const char **)A(8 * n), **o_np = (const char **)A(8 * n);
  std::printf("outputs on %s pages\n", huge ? "2 MiB (THP)" : "malloc");
  std::vector<uint64_t> soff(20), noff(200);
  std::vector<uint32_t> slen(20, 7), nlen(200, 11);
  static char arena[4096];
  for (int rep = 0; rep < 5; rep++) {
    const double ms = run(nt, n, [&](size_t lo, size_t hi) {
      for (size_t o = lo; o < hi; o++) {
        const uint32_t e = uint32_t(pos[o]);
        std::memcpy(&o_ids[16 * o], &ids[16 * size_t(e)], 16);
        o_il[o] = il[e];
        const uint64_t s = st[e], x = en[e];
        o_st[o] = s;
        o_en[o] = x;
        o_dur[o] = uint32_t((x - s) / 1000000ull);
        o_blk[o] = uint32_t(pos[o] >> 32);
        o_entry[o] = e;
        const uint32_t a = sv[e], c = nm[e];
        o_so[o] = soff[a];
        o_sl[o] = slen[a];
        o_sp[o] = arena + soff[a];
        o_no[o] = noff[c];
        o_nl[o] = nlen[c];
        o_np[o] = arena + noff[c];
      }
    });
    // the same fill as column passes: each pass one or two input columns and its outputs
    const double ms2 = run(nt, n, [&](size_t lo, size_t hi) {
      for (size_t o = lo; o < hi; o++) std::memcpy(&o_ids[16 * o], &ids[16 * size_t(uint32_t(pos[o]))], 16);
      for (size_t o = lo; o < hi; o++) o_il[o] = il[uint32_t(pos[o])];
      for (size_t o = lo; o < hi; o++) {
        const uint32_t e = uint32_t(pos[o]);
        const uint64_t s = st[e], x = en[e];
        o_st[o] = s;
        o_en[o] = x;
        o_dur[o] = uint32_t((x - s) / 1000000ull);
      }
      for (size_t o = lo; o < hi; o++) {
        o_blk[o] = uint32_t(pos[o] >> 32);
        o_entry[o] = uint32_t(pos[o]);
      }
      for (size_t o = lo; o < hi; o++) {
        const uint32_t a = sv[uint32_t(pos[o])];
        o_so[o] = soff[a];
        o_sl[o] = slen[a];
        o_sp[o] = arena + soff[a];
      }
      for (size_t o = lo; o < hi; o++) {
        const uint32_t c = nm[uint32_t(pos[o])];
        o_no[o] = noff[c];
        o_nl[o] = nlen[c];
        o_np[o] = arena + noff[c];
      }
    });
    // record-at-a-time again, in chunks of 4096 records per column pass
    const double ms3 = run(nt, n, [&](size_t lo, size_t hi) {
      for (size_t c0 = lo; c0 < hi; c0 += 4096) {
        const size_t c1 = std::min(hi, c0 + 4096);
        for (size_t o = c0; o < c1; o++) std::memcpy(&o_ids[16 * o], &ids[16 * size_t(uint32_t(pos[o]))], 16);
        for (size_t o = c0; o < c1; o++) {
          const uint32_t e = uint32_t(pos[o]);
          o_il[o] = il[e];
          const uint64_t s = st[e], x = en[e];
          o_st[o] = s;
          o_en[o] = x;
          o_dur[o] = uint32_t((x - s) / 1000000ull);
          o_blk[o] = uint32_t(pos[o] >> 32);
          o_entry[o] = e;
        }
        for (size_t o = c0; o < c1; o++) {
          const uint32_t e = uint32_t(pos[o]);
          const uint32_t a = sv[e], c = nm[e];
          o_so[o] = soff[a];
          o_sl[o] = slen[a];
          o_sp[o] = arena + soff[a];
          o_no[o] = noff[c];
          o_nl[o] = nlen[c];
          o_np[o] = arena + noff[c];
        }
      }
    });
    std::printf("  column passes %.2f ms, chunked passes %.2f ms\n", ms2, ms3);
    std::vector<uint8_t> src(89 * n), dst(89 * n);
    std::memset(src.data(), 1, src.size());
    std::memset(dst.data(), 2, dst.size());
    const double cp = run(nt, src.size(), [&](size_t lo, size_t hi) { std::memcpy(&dst[lo], &src[lo], hi - lo); });
    std::printf("threads %d records %zu: gather-fill %.2f ms (%.2f ns/record), copy of %zu MB %.2f ms (%.1f GB/s)\n", nt,
                n, ms, ms * 1e6 / double(n), src.size() >> 20, cp, 2.0 * double(src.size()) / cp / 1e6);
  }
  cpu_set_t set;
  sched_getaffinity(0, sizeof set, &set);
  std::printf("cpus allowed %d, hw %u\n", CPU_COUNT(&set), std::thread::hardware_concurrency());
  return 0;
}
