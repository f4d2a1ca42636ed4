// shape_probe.hip — measurement tool (not part of libtsg): how fast can one launch stream the
// main line's filter columns (10 M entries: ds u32, start_s u32, three 1-byte tag columns =
// 11 B/entry, 110 MB) with the resident kernel's access shape, and which part of that shape
// costs what. Four disjoint copies are swept in turn (440 MB > the 256 MiB Infinity Cache), as
// the bench's main line does. Each mode is timed with hipEvents over `reps` launches.
//
//   mode 0  the search kernels' shape: 512-entry units, per lane 2 x (ds, start) 16-B loads and
//           2 x 3 tag 4-B loads (lane l: entries k*256 + 4l .. +3)
//   mode 1  the same with the tag columns read by 16-B loads (lanes 0..31, 512 B per column)
//   mode 2  the ds and start columns alone (16-B loads; 8 B/entry)
//   mode 3  the same 5,632 B per unit as one contiguous array, 16-B loads (the shape's ceiling)
//
// Workgroups: 256 x (waves x 64); each owns a contiguous unit run (equal shares), its waves
// take the run's units from an LDS counter, two units in flight per wave (the search kernels'
// pipelining). Build: hipcc -O3 --offload-arch=gfx950 tools/shape_probe.hip -o tools/_bin/shape_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kUnit = 512;

struct Set {
  const uint32_t *ds, *st;
  const uint8_t *t[3];
  const uint8_t *flat;  // mode 3: 5632 B per unit
};

template <bool NT>
__device__ __forceinline__ u32x4 ld4(const void *p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  else return *reinterpret_cast<const u32x4 *>(p);
}
template <bool NT>
__device__ __forceinline__ uint32_t ld1(const void *p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(p));
  else return *reinterpret_cast<const uint32_t *>(p);
}

struct Regs {
  u32x4 a[2], b[2];
  u32x4 t4[3];
  uint32_t t[3][2];
  u32x4 f[6];
};

template <int MODE, bool NT>
__device__ __forceinline__ void load(Regs &R, const Set &S, uint32_t u, int lane) {
  const uint64_t e0 = uint64_t(u) * kUnit;
  if (MODE == 3) {
    const uint8_t *p = S.flat + uint64_t(u) * (kUnit * 11);
#pragma unroll
    for (int k = 0; k < 6; k++) {  // 5632 B = 5.5 x 1024: the last load by lanes 0..31
      const uint32_t off = k * 1024 + lane * 16;
      R.f[k] = off < kUnit * 11 ? ld4<NT>(p + off) : u32x4{0, 0, 0, 0};
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint64_t e = e0 + k * 256 + lane * 4;
    R.a[k] = ld4<NT>(S.ds + e);
    R.b[k] = ld4<NT>(S.st + e);
  }
  if (MODE == 0) {
#pragma unroll
    for (int q = 0; q < 3; q++)
#pragma unroll
      for (int k = 0; k < 2; k++) R.t[q][k] = ld1<NT>(S.t[q] + e0 + k * 256 + lane * 4);
  } else if (MODE == 1) {
#pragma unroll
    for (int q = 0; q < 3; q++) R.t4[q] = lane < 32 ? ld4<NT>(S.t[q] + e0 + lane * 16) : u32x4{0, 0, 0, 0};
  }
}

template <int MODE>
__device__ __forceinline__ uint32_t use(const Regs &R) {
  uint32_t x = 0;
  if (MODE == 3) {
#pragma unroll
    for (int k = 0; k < 6; k++) x ^= R.f[k].x ^ R.f[k].y ^ R.f[k].z ^ R.f[k].w;
    return x;
  }
#pragma unroll
  for (int k = 0; k < 2; k++) x ^= R.a[k].x ^ R.a[k].y ^ R.a[k].z ^ R.a[k].w ^ R.b[k].x ^ R.b[k].y ^ R.b[k].z ^ R.b[k].w;
  if (MODE == 0)
#pragma unroll
    for (int q = 0; q < 3; q++) x ^= R.t[q][0] ^ R.t[q][1];
  if (MODE == 1)
#pragma unroll
    for (int q = 0; q < 3; q++) x ^= R.t4[q].x ^ R.t4[q].y ^ R.t4[q].z ^ R.t4[q].w;
  return x;
}

template <int MODE, bool NT, bool EXACT = false>
__global__ void __launch_bounds__(1024, 1) probe(Set S, uint32_t nunits, uint32_t *out) {
  __shared__ uint32_t s_next;
  const int lane = threadIdx.x & 63;
  const uint32_t nwv = blockDim.x >> 6, wave = threadIdx.x >> 6, w = blockIdx.x, G = gridDim.x;
  const uint32_t q = nunits / G, r = nunits % G;
  const uint32_t ua = w * q + min(w, r), nk = q + (w < r ? 1u : 0u);
  if (threadIdx.x == 0) s_next = 0;
  __syncthreads();
  auto claim = [&]() -> uint32_t {
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&s_next, 1u);
    return 2 * nwv + uint32_t(__builtin_amdgcn_readfirstlane(c));
  };
  Regs ra, rb;
  uint32_t ka = wave, kb = wave + nwv, acc = 0;
  if constexpr (EXACT) {
    // every iteration issues both streams' loads (a unit past the run re-reads the run's first
    // unit, L2-hot): the compiler's vmcnt bookkeeping stays exact, so the wait for one unit's
    // data does not also wait for the other unit's loads (two units in flight, not one)
    load<MODE, NT>(ra, S, ua + min(ka, nk - 1), lane);
    load<MODE, NT>(rb, S, ua + min(kb, nk - 1), lane);
    while (ka < nk || kb < nk) {
      const uint32_t xa = use<MODE>(ra);
      acc ^= ka < nk ? xa : 0u;
      ka = ka < nk ? claim() : ka;
      load<MODE, NT>(ra, S, ua + min(ka, nk - 1), lane);
      const uint32_t xb = use<MODE>(rb);
      acc ^= kb < nk ? xb : 0u;
      kb = kb < nk ? claim() : kb;
      load<MODE, NT>(rb, S, ua + min(kb, nk - 1), lane);
    }
    if (acc == 0x9E3779B9u) out[w] = acc;
    return;
  }
  if (ka < nk) load<MODE, NT>(ra, S, ua + ka, lane);
  if (kb < nk) load<MODE, NT>(rb, S, ua + kb, lane);
  while (ka < nk || kb < nk) {
    if (ka < nk) {
      acc ^= use<MODE>(ra);
      ka = claim();
      if (ka < nk) load<MODE, NT>(ra, S, ua + ka, lane);
    }
    if (kb < nk) {
      acc ^= use<MODE>(rb);
      kb = claim();
      if (kb < nk) load<MODE, NT>(rb, S, ua + kb, lane);
    }
  }
  if (acc == 0x9E3779B9u) out[w] = acc;  // (keeps the loads; never true in practice)
}

template <int MODE, bool NT, bool EXACT = false>
static void run(const std::vector<Set> &sets, uint32_t nunits, int waves, int reps, uint32_t *out, double bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 8; i++) probe<MODE, NT, EXACT><<<256, waves * 64>>>(sets[i % sets.size()], nunits, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int i = 0; i < reps; i++) {
    CK(hipEventRecord(a));
    probe<MODE, NT, EXACT><<<256, waves * 64>>>(sets[i % sets.size()], nunits, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float t = 0;
    CK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double med = ms[ms.size() / 2] * 1e3, best = ms[0] * 1e3;
  std::printf("mode %d%s nt %d waves %2d: median %7.2f us  best %7.2f us  -> %6.0f GB/s (11 B/entry basis %6.0f)\n", MODE,
              EXACT ? "x" : " ", int(NT), waves, med, best, bytes / med / 1e3, 110.0e6 / med / 1e3);
}

int main(int argc, char **argv) {
  const uint64_t N = 10000000 / kUnit * kUnit;  // 10 M entries (whole units)
  const uint32_t nunits = uint32_t(N / kUnit);
  const int nsets = 4, reps = argc > 1 ? std::atoi(argv[1]) : 50;
  std::vector<Set> sets(nsets);
  for (int s = 0; s < nsets; s++) {
    uint8_t *p = nullptr;
    const size_t bytes = N * 11;
    CK(hipMalloc(&p, bytes * 2));  // columns, then the flat copy
    CK(hipMemset(p, s + 1, bytes * 2));
    sets[s].ds = reinterpret_cast<const uint32_t *>(p);
    sets[s].st = reinterpret_cast<const uint32_t *>(p + N * 4);
    for (int q = 0; q < 3; q++) sets[s].t[q] = p + N * 8 + N * q;
    sets[s].flat = p + bytes;
  }
  uint32_t *out = nullptr;
  CK(hipMalloc(&out, 256 * 4));
  const double b11 = double(N) * 11, b8 = double(N) * 8;
  for (int waves : {8, 12, 16}) {
    run<0, true, true>(sets, nunits, waves, reps, out, b11);
    run<3, true, true>(sets, nunits, waves, reps, out, b11);
    run<0, true>(sets, nunits, waves, reps, out, b11);
    run<0, false>(sets, nunits, waves, reps, out, b11);
    run<1, true>(sets, nunits, waves, reps, out, b11);
    run<2, true>(sets, nunits, waves, reps, out, b8);
    run<3, true>(sets, nunits, waves, reps, out, b11);
  }
  return 0;
}
