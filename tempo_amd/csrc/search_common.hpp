// search_common.hpp — definitions shared by the search kernels (search.hip) and the
// pool search path (pool.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "devctx.hpp"

namespace tsg {

struct ScanSeg {
  uint64_t n;
  const uint32_t *dur32;
  const uint64_t *dur64;
  const uint32_t *start_s, *end_s;
  const uint8_t *ids;
  const uint64_t *start_ns, *end_ns;
  const uint32_t *names;
  const uint8_t *id_len;
  uint32_t tail, nunits;        // scan units (kUnit entries) in the block; the last `tail` tiles of
                                // them are claimed dynamically (segment mode: work stealing)
  uint32_t first_wg, nwg, tpw;  // workgroups owning this block (units split evenly), max tiles per workgroup
  uint32_t term0, nterms, lds_words;
  uint32_t block_idx, steal_base;  // claim counter value at launch start (tail tiles)
  uint64_t cap;  // limit mode: records kept from this block
  uint64_t e0;   // first scan position searched (a multiple of the pool unit; 0 = the whole block up to n)
  uint64_t bm_word0;  // bitmap mode: the block's first word in ScanParams::bitmap (nunits x 16 words)
};

struct MatchRec {  // == SearchOut::Rec
  uint8_t id[16];
  uint64_t start, end;
  uint32_t entry;
  uint32_t block_il;  // block index | id length << 24
  uint32_t svc, name;
};
static_assert(sizeof(MatchRec) == 48, "record layout");
static_assert(sizeof(MatchRec) == sizeof(SearchOut::Rec), "record layout");

constexpr int kThreads = 256;
// A query's shape for the pool kernels' overflow memory (DeviceCtx::pool_skip): its terms,
// duration bounds and time range. A record-buffer overflow skips the pool for the next few
// searches of the SAME query only: other queries interleaved with a dense one (concurrent
// callers) keep the resident kernel.
inline uint64_t pool_query_key(const tsg_query &q) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t(q.nterms) << 40) ^ (uint64_t(q.has_min) << 33) ^
               (uint64_t(q.has_max) << 34) ^ (uint64_t(q.has_range) << 35);
  h ^= q.min_ns * 0xBF58476D1CE4E5B9ull ^ q.max_ns * 0x94D049BB133111EBull ^
       (uint64_t(q.start_s) << 32 | q.end_s) * 0xD6E8FEB86659FD93ull;
  for (uint32_t t = 0; t < q.nterms; t++)
    h = (h ^ xxhash64(q.keys[t], q.key_lens[t]) ^ (xxhash64(q.values[t], q.value_lens[t]) * 31)) *
        0x9E3779B97F4A7C15ull;
  return h;
}
constexpr int kSteps = 2;                     // 8 entries per thread per tile
constexpr int kTile = kThreads * 4 * kSteps;  // 2048 entries
constexpr uint32_t kMaskAll = (1u << (4 * kSteps)) - 1;
constexpr int kUnit = kThreads * 4;           // 1024 entries: workgroup ranges are whole units
constexpr uint32_t kNoLds = 0xffffffffu;

// Pointers inside descriptors are generic to the compiler; casting them to the
// global address space turns flat loads (which wait on vmcnt AND lgkmcnt) into
// global_load_dword{,x2,x4}.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *G(const T *p) {
  return (const __attribute__((address_space(1))) T *)(p);
}
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *G(const void *p) {
  return (const __attribute__((address_space(1))) T *)(p);
}

// The pool kernels' compact duration column (devctx.hip, ds = D16 | span16 << 16): D16 =
// 2 x whole ms + (a sub-ms remainder), saturated at 0xffff, is exact for duration bounds up
// to this many ms (larger bounds take the other search paths)
constexpr uint64_t kDs16MaxMs = 32767;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// (tile registers are kept as 128-bit vectors, not 4 scalars: a quad returned by one
// dwordx4 load then stays one register tuple across the loop, instead of being
// copied into scalar registers right after the load, which waits for it)
__device__ __forceinline__ u32x4 load4_u32(const uint32_t *p, uint64_t e) { return *G<u32x4>(p + e); }

// Stores to pinned host memory (records, counts, header): relaxed system-scope
// stores, i.e. write-through, no cache maintenance. A workgroup makes them complete
// with one s_waitcnt before it arrives at the completion counter; no L2 writeback /
// invalidate fence (a per-workgroup __threadfence_system() stalls the whole L2 of
// its XCD while the other workgroups stream).
template <typename T>
__device__ __forceinline__ void host_store(T *p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kStampSlots = 9;     // TSG_STAMPS: start setup scan lookback end | desc staged inlds | hw id

constexpr uint32_t kCountPending = 0xffffffffu;  // segment mode: a workgroup count not stored yet (host sentinel)

constexpr int kArgSegs = 32, kArgTerms = 4, kArgNeedle = 256, kArgBms = 16;

// Resident descriptors are immutable while a search runs: read them through the
// constant address space so uniform reads become scalar loads (s_load, one round
// trip for all fields) instead of vector loads serialised by vmcnt.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T *K4(const T *p) {
  return (const __attribute__((address_space(4))) T *)(p);
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Tracer {
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  char buf[512];
  int len = 0;
  bool prof = prof_on();
  Tracer() : on(std::getenv("TSG_TRACE") != nullptr) {
    if (on || prof) t0 = last = std::chrono::steady_clock::now();
  }
  void mark(const char *name) {
    if (!on && !prof) return;
    auto now = std::chrono::steady_clock::now();
    if (prof) {
      prof_add(name, std::chrono::duration<double, std::micro>(now - last).count());
      last = now;
      if (!on) return;
    }
    len += std::snprintf(buf + len, sizeof buf - size_t(len), " %s=%.1f", name,
                         std::chrono::duration<double, std::micro>(now - last).count());
    last = now;
  }
  ~Tracer() {
    if (on && len) std::fprintf(stderr, "[tsg] device_search us:%s total=%.1f\n", buf,
                                std::chrono::duration<double, std::micro>(last - t0).count());
  }
};

// narrow mode: per block its scan / one-byte column bases and per term the column slot
// and interned dictionary
struct NarrowSeg {
  const uint32_t *scan;
  const uint8_t *ncol;
  uint32_t npad;
  std::array<uint8_t, kArgTerms> slot, nsets;
  std::array<const NarrowDict *, kArgTerms> dict;
};

void print_stamps(DeviceCtx &dc, uint32_t nwg, bool fast);

// pool.hip: one search_pool_kernel (or search_static_kernel) launch for a narrow search;
// limit L > 0 keeps each block part's first L records. false (and nothing written to
// `out`) when the caller should run the segment / look-back path
bool pool_search(DeviceCtx &dc, const std::vector<std::pair<uint32_t, Block *>> &blocks, const tsg_query &q,
                 uint32_t limit, uint32_t flags, const std::vector<ScanSeg> &segs, const std::vector<NarrowSeg> &nsegv,
                 const std::vector<std::array<uint32_t, 8>> &nbms,
                 const std::vector<std::array<uint8_t, kArgTerms>> &nbmi,
                 const std::vector<const DevBlockDesc *> &seg_desc, bool has_dur, Tracer &tr, SearchOut &out,
                 std::unique_lock<std::mutex> &lk);

}  // namespace tsg
