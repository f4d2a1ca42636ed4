// scan_probe.hip — where the search scan loses time against a plain stream: the config-2
// column layout (10 blocks x ~1 M entries; per block dur32|start_s|end_s u32 columns in one
// allocation, 20 one-byte key columns in another, the query reading 3 of them = 15 B/entry,
// 150 MB per set, 4 sets in rotation = HBM regime) scanned by
//   static1024: one 1024-thread workgroup per CU, static contiguous unit runs per wave,
//               2 units (512 entries) in flight per wave, the pool kernel's load pattern
//   grid256:    one 256-thread workgroup per 2048-entry tile, the hardware dispatcher
//               balancing (8 entries per lane)
//   grid256x2:  the same with 2 tiles per workgroup (both loaded up front)
// timed with HIP events and with events stamped from the dispatch (hipExtLaunchKernel).
//   hipcc -O3 --offload-arch=gfx950 tools/scan_probe.hip -o build/scan_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kBlocks = 10;
constexpr uint32_t kUnit = 512;
constexpr uint32_t kUnitsPerBlock = 1954;
constexpr uint32_t kN = kUnit * kUnitsPerBlock;  // entries per block (1,000,448)
constexpr uint32_t kNpad = 1003520;              // multiple of 4096
constexpr int kSlots = 20;

struct Set {
  const uint32_t *scan[kBlocks];
  const uint8_t *col[kBlocks][3];
};
struct Args {
  Set s;
  uint32_t min32, max32, start_s, end_s;
  uint32_t bm[3][8];
  unsigned *sink;
};

template <bool NT>
__device__ __forceinline__ u32x4 ld4(const uint32_t *p) {
  return NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p)) : *reinterpret_cast<const u32x4 *>(p);
}
template <bool NT>
__device__ __forceinline__ uint32_t ld1(const uint8_t *p) {
  return NT ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(p)) : *reinterpret_cast<const uint32_t *>(p);
}
template <bool NT>
__device__ __forceinline__ u32x2 ld2(const uint8_t *p) {
  return NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(p)) : *reinterpret_cast<const u32x2 *>(p);
}

struct Regs {
  u32x4 d[2], s[2], e[2];
  uint32_t t[3][2];
};

template <bool NT>
__device__ __forceinline__ void load_unit(Regs &R, const Args &A, uint32_t u, int lane) {
  const uint32_t b = u / kUnitsPerBlock, e0 = (u % kUnitsPerBlock) * kUnit;
  const uint32_t *scan = A.s.scan[b];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint32_t e = e0 + k * 256 + lane * 4;
    R.d[k] = ld4<NT>(scan + e);
    R.s[k] = ld4<NT>(scan + kNpad + e);
    R.e[k] = ld4<NT>(scan + 2 * kNpad + e);
#pragma unroll
    for (int q = 0; q < 3; q++) R.t[q][k] = ld1<NT>(A.s.col[b][q] + e);
  }
}
__device__ __forceinline__ uint32_t eval_unit(const Regs &R, const Args &A, const uint32_t *bm) {
  uint32_t mask = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint32_t dv[4] = {R.d[k].x, R.d[k].y, R.d[k].z, R.d[k].w};
    const uint32_t sv[4] = {R.s[k].x, R.s[k].y, R.s[k].z, R.s[k].w};
    const uint32_t ev[4] = {R.e[k].x, R.e[k].y, R.e[k].z, R.e[k].w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t ok = uint32_t(dv[j] >= A.min32) & uint32_t(dv[j] <= A.max32) & uint32_t(A.start_s <= ev[j]) &
                    uint32_t(A.end_s >= sv[j]);  // (branch-free, as the engine's unit_mask)
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const uint32_t x = (R.t[q][k] >> (8 * j)) & 0xffu;
        ok &= bm[q * 8 + (x >> 5)] >> (x & 31);
      }
      mask |= (ok & 1u) << (4 * k + j);
    }
  }
  return mask;
}

struct BigArgs {  // the pool kernel's argument size (~3.7 KB)
  Args a;
  uint32_t ubase[kBlocks + 1];
  uint32_t pad[800];
  unsigned *hcount;  // pinned host memory
};

template <bool NT, bool HOSTCOUNT, bool WALK>
__global__ void __launch_bounds__(1024, 1) static_big(BigArgs BA) {
  const Args &A = BA.a;
  __shared__ uint32_t bm[24];
  if (threadIdx.x < 24) bm[threadIdx.x] = A.bm[threadIdx.x / 8][threadIdx.x % 8];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t units = kBlocks * kUnitsPerBlock;
  const uint32_t waves = gridDim.x * 16, gw = blockIdx.x * 16 + wave;
  const uint32_t u0 = uint32_t(uint64_t(units) * gw / waves), u1 = uint32_t(uint64_t(units) * (gw + 1) / waves);
  uint32_t cnt = 0;
  if (WALK) {  // the static kernel's walk over the unit bases (scalar loads of the arguments)
    uint32_t b = 0;
    while (b + 1 < kBlocks && u0 >= BA.ubase[b + 1]) b++;
    cnt += b == 0xffffu;
  }
  Regs ra, rb;
  uint32_t u = u0;
  if (u < u1) load_unit<NT>(ra, A, u, lane);
  for (; u < u1; u += 2) {
    if (u + 1 < u1) load_unit<NT>(rb, A, u + 1, lane);
    cnt += __popc(eval_unit(ra, A, bm));
    if (u + 2 < u1) load_unit<NT>(ra, A, u + 2, lane);
    if (u + 1 < u1) cnt += __popc(eval_unit(rb, A, bm));
  }
  if (cnt) atomicAdd(A.sink, cnt);
  if (HOSTCOUNT) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(BA.hcount + blockIdx.x, cnt + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <bool NT, bool SPREAD = false>
__global__ void __launch_bounds__(1024, 1) static1024(Args A) {
  __shared__ uint32_t bm[24];
  if (threadIdx.x < 24) bm[threadIdx.x] = A.bm[threadIdx.x / 8][threadIdx.x % 8];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t units = kBlocks * kUnitsPerBlock;
  const uint32_t waves = gridDim.x * 16, gw = blockIdx.x * 16 + wave;
  const uint32_t per = (units + waves - 1) / waves, u0 = gw * per, u1 = min(units, u0 + per);
  uint32_t cnt = 0;
  Regs ra, rb;
  uint32_t u = u0;
  if (u < u1) load_unit<NT>(ra, A, u, lane);
  for (; u < u1; u += 2) {
    if (u + 1 < u1) load_unit<NT>(rb, A, u + 1, lane);
    cnt += __popc(eval_unit(ra, A, bm));
    if (u + 2 < u1) load_unit<NT>(ra, A, u + 2, lane);
    if (u + 1 < u1) cnt += __popc(eval_unit(rb, A, bm));
  }
  if (SPREAD) {  // one word per wave: no same-address atomics at the end
    if (cnt == 0x7fffffffu) A.sink[gw & 15] = cnt;
  } else if (cnt) atomicAdd(A.sink, cnt);
}

// one workgroup per TILES x 2048 entries (tiles never straddle blocks: a block is 977 tiles
// + a 1024-entry remainder, handled as a half tile)
template <bool NT, int TILES>
__global__ void __launch_bounds__(256) grid256(Args A) {
  __shared__ uint32_t bm[24];
  if (threadIdx.x < 24) bm[threadIdx.x] = A.bm[threadIdx.x / 8][threadIdx.x % 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // wave-unit space: every wave takes whole 512-entry units (4 per 2048-entry tile)
  const uint32_t units = kBlocks * kUnitsPerBlock;
  Regs r[TILES];
  uint32_t uu[TILES];
#pragma unroll
  for (int t = 0; t < TILES; t++) {
    uu[t] = (blockIdx.x * TILES + t) * 4 + wave;
    if (uu[t] < units) load_unit<NT>(r[t], A, uu[t], lane);
  }
  __syncthreads();
  uint32_t cnt = 0;
#pragma unroll
  for (int t = 0; t < TILES; t++)
    if (uu[t] < units) cnt += __popc(eval_unit(r[t], A, bm));
  if (cnt) atomicAdd(A.sink, cnt);
}

struct Stat {
  std::vector<float> v;
  void print(const char *name, const char *timing, double bytes) {
    std::sort(v.begin(), v.end());
    double s = 0;
    for (float x : v) s += x;
    const double avg = s / v.size();
    std::printf("{\"kernel\": \"%s\", \"timing\": \"%s\", \"avg_us\": %.2f, \"p10_us\": %.2f, \"p50_us\": %.2f, "
                "\"p90_us\": %.2f, \"gbps\": %.1f, \"frac\": %.3f}\n",
                name, timing, avg, v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], bytes / (avg * 1e3),
                bytes / (avg * 1e3) / 8000.0);
    std::fflush(stdout);
  }
};

int main() {
  const bool rand_data = std::getenv("PROBE_RAND") != nullptr;
  int cu = 0;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<Args> sets(4);
  unsigned *sink;
  CK(hipMalloc(&sink, 64));
  for (auto &A : sets) {
    for (int b = 0; b < kBlocks; b++) {
      uint32_t *scan;
      uint8_t *ncol;
      CK(hipMalloc(&scan, size_t(3) * kNpad * 4));
      CK(hipMalloc(&ncol, size_t(kSlots) * kNpad));
      CK(hipMemset(scan, 0x11, size_t(3) * kNpad * 4));
      CK(hipMemset(ncol, 0x03, size_t(kSlots) * kNpad));
      if (rand_data) {  // PROBE_RAND=1: config-2-like values (varied durations, times, value-set ids)
        static std::vector<uint32_t> hs(size_t(3) * kNpad);
        static std::vector<uint8_t> hc(size_t(kSlots) * kNpad);
        uint64_t x = 0x9e3779b97f4a7c15ull * uint64_t(b + 1);
        auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return uint32_t(x); };
        for (uint32_t e = 0; e < kNpad; e++) {
          const uint32_t st = 1700000000u + rnd() % 3600u;
          hs[e] = rnd() % 2000000000u;                 // dur32 (ns)
          hs[kNpad + e] = st;                          // start_s
          hs[2 * kNpad + e] = st + rnd() % 3u;         // end_s
        }
        for (size_t i = 0; i < hc.size(); i++) hc[i] = uint8_t(rnd() % 16u);
        CK(hipMemcpy(scan, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(ncol, hc.data(), hc.size(), hipMemcpyHostToDevice));
      }
      A.s.scan[b] = scan;
      A.s.col[b][0] = ncol;
      A.s.col[b][1] = ncol + size_t(7) * kNpad;
      A.s.col[b][2] = ncol + size_t(13) * kNpad;
    }
    A.min32 = 10000000;
    A.max32 = 1000000000;
    A.start_s = 100;
    A.end_s = 200;
    for (int q = 0; q < 3; q++)
      for (int w = 0; w < 8; w++) A.bm[q][w] = rand_data && w == 0 ? (q == 0 ? 0x80u : q == 1 ? 0x3u : 0x4u) : 0u;
    A.sink = sink;
  }
  const double bytes = double(kBlocks) * kN * 15;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint32_t units = kBlocks * kUnitsPerBlock;
  unsigned *hcount;
  CK(hipHostMalloc(&hcount, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  std::vector<BigArgs> big(4);
  for (int i = 0; i < 4; i++) {
    big[i].a = sets[i];
    for (int b = 0; b <= kBlocks; b++) big[i].ubase[b] = b * kUnitsPerBlock;
    big[i].hcount = hcount;
  }
  auto run = [&](const char *name, const void *f, unsigned grid, unsigned threads, bool bigargs = false,
                 size_t lds = 0, int nsets = 4) {
    Stat ev, ext;
    if (lds) CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    for (int mode = 0; mode < 2; mode++)
      for (int r = 0; r < 64; r++) {
        Args &A = sets[r % nsets];
        BigArgs &BA = big[r % nsets];
        void *args1[] = {&A};
        void *args2[] = {&BA};
        void **args = bigargs ? args2 : args1;
        if (mode == 0) {
          CK(hipEventRecord(a, s));
          CK(hipExtLaunchKernel(f, dim3(grid), dim3(threads), args, lds, s, nullptr, nullptr, 0));
          CK(hipEventRecord(b, s));
        } else {
          CK(hipExtLaunchKernel(f, dim3(grid), dim3(threads), args, lds, s, a, b, 0));
        }
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 4) (mode ? ext : ev).v.push_back(ms * 1e3f);
      }
    ev.print(name, "events", bytes);
    ext.print(name, "ext_events", bytes);
  };
  if (rand_data) {
    for (auto &A : sets) { A.min32 = 10000000; A.max32 = 1000000000; A.start_s = 1700000900; A.end_s = 1700002700; }
    run("rand_static1024_nt", reinterpret_cast<const void *>(static1024<true>), cu, 1024);
    run("rand_static1024_nt_mall", reinterpret_cast<const void *>(static1024<true>), cu, 1024, false, 0, 1);
    run("rand_static1024_nt_noatomic", reinterpret_cast<const void *>(static1024<true, true>), cu, 1024);
    return 0;
  }
  run("static1024_nt", reinterpret_cast<const void *>(static1024<true>), cu, 1024);
  run("static1024_nt_mall", reinterpret_cast<const void *>(static1024<true>), cu, 1024, false, 0, 1);
  run("big_nt", reinterpret_cast<const void *>(static_big<true, false, false>), cu, 1024, true);
  run("big_nt_lds96k", reinterpret_cast<const void *>(static_big<true, false, false>), cu, 1024, true, 96 << 10);
  run("big_nt_hostcount", reinterpret_cast<const void *>(static_big<true, true, false>), cu, 1024, true);
  run("big_nt_walk", reinterpret_cast<const void *>(static_big<true, false, true>), cu, 1024, true);
  run("big_nt_all", reinterpret_cast<const void *>(static_big<true, true, true>), cu, 1024, true, 96 << 10);
  run("big_nt_all_mall", reinterpret_cast<const void *>(static_big<true, true, true>), cu, 1024, true, 96 << 10, 1);
  run("grid256_nt", reinterpret_cast<const void *>(grid256<true, 1>), (units + 3) / 4, 256);
  return 0;
}
