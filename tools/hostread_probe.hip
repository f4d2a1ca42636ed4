// hostread_probe.hip — how fast the host reads result records the GPU wrote into
// pinned memory, by allocation flavour (diagnostics for the search result path).
// A kernel writes 400 scattered 48-byte records (stride 768 B) with system-scope
// stores; the host then copies them out. Prints one JSON line per flavour.
//   hipcc -O3 --offload-arch=gfx950 tools/hostread_probe.hip -o build/hostread_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

__global__ void write_recs(unsigned long long *buf, int nseg, int stride_words, unsigned long long tag) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  for (int i = 0; i < 6; i++)
    __hip_atomic_store(buf + size_t(s) * stride_words + i, tag + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
  const int nseg = 400, stride = 96;  // 768 B
  const size_t bytes = size_t(nseg) * stride * 8 + 4096;
  struct F { const char *name; unsigned flags; } fl[] = {
      {"mapped|coherent", hipHostMallocMapped | hipHostMallocCoherent},
      {"mapped|noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
      {"default", hipHostMallocDefault}};
  std::vector<unsigned long long> dst(size_t(nseg) * 6);
  for (auto &f : fl) {
    void *p;
    CK(hipHostMalloc(&p, bytes, f.flags));
    auto *b = static_cast<unsigned long long *>(p);
    double best = 1e9, sum = 0, best_seq = 1e9;
    const int reps = 50;
    for (int r = 0; r < reps + 3; r++) {
      write_recs<<<(nseg + 63) / 64, 64>>>(b, nseg, stride, 1000ull * r);
      CK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      for (int s = 0; s < nseg; s++) std::memcpy(&dst[size_t(s) * 6], b + size_t(s) * stride, 48);
      auto t1 = std::chrono::steady_clock::now();
      const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
      if (dst[6 * (nseg - 1) + 5] != 1000ull * r + 5) { std::fprintf(stderr, "stale read\n"); return 1; }
      // contiguous 24 KB read of the same buffer (after another GPU write)
      write_recs<<<(nseg + 63) / 64, 64>>>(b, nseg, 6, 7ull * r);
      CK(hipDeviceSynchronize());
      auto t2 = std::chrono::steady_clock::now();
      std::memcpy(dst.data(), b, size_t(nseg) * 48);
      auto t3 = std::chrono::steady_clock::now();
      const double us2 = std::chrono::duration<double, std::micro>(t3 - t2).count();
      if (r >= 3) { sum += us; best = us < best ? us : best; best_seq = us2 < best_seq ? us2 : best_seq; }
    }
    std::printf("{\"alloc\": \"%s\", \"scattered_avg_us\": %.2f, \"scattered_best_us\": %.2f, \"contig24k_best_us\": %.2f}\n",
                f.name, sum / reps, best, best_seq);
    CK(hipHostFree(p));
  }
  return 0;
}
