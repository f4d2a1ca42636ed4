// pool.hip — MI355X (gfx950) pool search: narrow full scans (limit 0) of Tempo search
// blocks with one workgroup per CU and a CU-wide work pool. The same predicates,
// records and result order as search_fast_kernel (search.hip); see DESIGN.md §4.
#include <dirent.h>
#include <fcntl.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <map>
#include <mutex>
#include <thread>
#include <vector>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <string>
#include <cstring>

#include "aql.hpp"
#include "search_common.hpp"

namespace tsg {

// ------------------------------------------------------------------------------------
// pool search: narrow full scans (limit 0) with a CU-wide work pool
//
// One 1024-thread workgroup per CU (16 waves; its LDS request keeps a second one off the
// CU). The query's blocks form one space of 512-entry units (a wave tile: 8 entries per
// lane). A workgroup owns a static run of units, handed out one unit per claim from an
// LDS counter to whichever of its waves is free, so the waves of a CU finish together
// whatever order the CU's issue arbitration serves them in (the static split's four
// workgroups per CU finished as a ladder 22/25/28/33 us, profiles/r02_prio). The last
// units of the launch are claimed in chunks from one device counter (dequeue: one
// returning atomic per chunk, issued `lookahead` claims before the chunk is needed), so
// CUs that the fabric serves faster take more of them. Matches go to the workgroup's LDS
// record buffer as they are found (gathered from the cold columns right away; record
// order inside a workgroup is claim order — the host sorts each block's records by scan
// position, which is the reference order), then to the workgroup's segment of pinned
// host memory with write-through stores, then its count. Records beyond the LDS capacity
// are counted, not kept: the host then reruns the query on the segment/look-back path.
constexpr int kPoolWaves = 16;
constexpr int kPoolThreads = kPoolWaves * 64;
constexpr uint32_t kPoolTile = 512;       // entries per unit (wave tile)
constexpr uint32_t kPoolChunks = 1024;    // dynamic chunks one workgroup can take
constexpr uint32_t kPoolPending = 0xffffffffu, kPoolNone = 0xfffffffeu;
constexpr uint32_t kPoolSpinMax = 1u << 24;  // LDS poll bound (~1 s of s_sleep 2)
static_assert(kColPad % kPoolTile == 0, "column padding covers whole units");

struct PoolBlk {           // 64 B, staged in LDS
  const uint32_t *scan;    // dur32 | start_s | end_s | ds, npad entries each (the pool reads ds, start_s)
  const uint8_t *col[4];   // one-byte term columns
  uint32_t npad, nent;
  uint32_t ubase;          // first unit of the block in the launch's unit space
  uint32_t bmi4, nsets4;   // per term: bitmap index into `bms`, value-set count (bytes)
  uint32_t block_idx;
};
static_assert(sizeof(PoolBlk) == 64, "pool block layout");
struct PoolArgs {
  PoolBlk blk[kArgSegs];
  const DevBlockDesc *desc[kArgSegs];  // cold columns (ids, times, names) of matches
  uint32_t bms[kArgBms][8];
  uint32_t ubase[kArgSegs + 1];  // first unit of each block, units at nsegs (static kernel's block walk)
  uint32_t ebase[kArgSegs];      // scan position of each block's first unit (a limit wave's part of a block)
  uint32_t nsegs, units, static_per_wg, dyn0;  // static run of workgroup w: [w*S, w*S+S); dynamic [dyn0, units)
  uint32_t chunk_shift, lookahead, rec_cap, seg_cap, has_min, has_max, min32, max32, start_s, end_s;
  unsigned *head;       // this launch's dynamic-chunk counter (zero at launch)
  unsigned *head_next;  // the next launch's counter: zeroed by this one
  uint8_t *recs;        // pinned host: workgroup w's first seg_cap records at w * seg_cap (rec_cap: LDS records)
  uint32_t *counts;     // pinned host: workgroup w's match count, stored after its records
  unsigned long long *stamps;
  uint32_t *err;        // pinned host: set when an LDS poll ran past its bound (the host fails the query)
  // limit L > 0: a unit keeps its first L matches in scan order (a block's first L records lie
  // in the first L of each of its units; the host cuts each block to L): a dense limit query
  // hands over at most L records per unit instead of every match
  uint32_t unit_cap;
  // the launch shape, passed explicitly: the kernels read no implicit kernel argument (blockDim /
  // gridDim come from them), so an AQL packet of our own needs none (aql.cpp)
  uint32_t nthreads, ngroups;
  // static kernel: the launch's NW waves split the units as wave g -> [g*sq + min(g, sr), ...),
  // the first sr waves one unit more (sq, sr = units / NW, units % NW: no division on the device)
  uint32_t sq, sr;
  uint32_t nbms;                     // bitmaps in `bms` (the resident kernel's slot checksum)
  uint32_t cstride;                  // resident kernel: workgroup w's count at counts[w * cstride] (0 = 1)
  uint32_t wq, wr;                   // resident kernel: workgroup w scans units [w*wq + min(w, wr), +wq + (w < wr))
  // resident kernel, XCD-weighted split (xsplit != 0; W a multiple of 8): workgroup w = 8i + x (XCD x)
  // scans xn[x] + (i < xr[x]) units, the runs in workgroup order (pool.hip res_split)
  uint32_t xsplit;
  unsigned long long *qstamps;       // resident kernel, timed queries: per workgroup {seen, end} (100 MHz)
  uint32_t xn[8], xr[8];
};
static_assert(sizeof(PoolArgs) <= 4096, "kernel arguments");

// The unit's matches (mask bit 4k + j of lane l = entry e0 + 256k + 4l + j) cut to the first
// `cap` in scan order (k, then lane, then j): each match's rank from per-step ballots.
__device__ __forceinline__ uint32_t cap_unit_mask(uint32_t mask, uint32_t cap, int lane) {
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t out = 0, before = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t nib = (mask >> (4 * k)) & 0xfu;
    uint32_t lower = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t b = __ballot((nib >> j) & 1u);
      lower += uint32_t(__popcll(b & below));
      tot += uint32_t(__popcll(b));
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t rank = before + lower + uint32_t(__popc(nib & ((1u << j) - 1u)));
      if (((nib >> j) & 1u) && rank < cap) out |= 1u << (4 * k + j);
    }
    before += tot;
  }
  return out;
}

// A pointer read from LDS by every lane (same value), moved to SGPRs. (readfirstlane
// returns int: each half goes through uint32_t, or the low half sign-extends.)
template <typename T>
__device__ __forceinline__ T *uniform_ptr(T *p) {
  const uint64_t v = uint64_t(uintptr_t(p));
  const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(v)));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(v >> 32)));
  return reinterpret_cast<T *>((uint64_t(hi) << 32) | lo);
}

template <int NT>
struct PoolRegs {
  u32x4 d[kSteps], s[kSteps];  // ds (duration | span), start seconds
  uint32_t tv[NT > 0 ? NT : 1][kSteps];
  uint32_t blk, e0;  // wave-uniform: block slot, first entry of the unit in its block
};

// Stream loads: default cache policy, or non-temporal (NTL: `nt`, the once-read filter
// columns do not displace the L2 / MALL lines other work reuses).
template <bool NTL>
__device__ __forceinline__ u32x4 stream4(const uint32_t *p, uint64_t e) {
  if constexpr (NTL) return __builtin_nontemporal_load(G<u32x4>(p + e));
  else return *G<u32x4>(p + e);
}
template <bool NTL>
__device__ __forceinline__ uint32_t stream1(const uint8_t *p, uint64_t e) {
  if constexpr (NTL) return __builtin_nontemporal_load(G<uint32_t>(p + e));
  else return *G<uint32_t>(p + e);
}

// The predicates of one unit (8 entries per lane) as a 32-bit lane mask, branch-free: every
// test is evaluated for every entry and combined with bitwise ands (short-circuit tests
// compiled to ~130 exec-mask branches per unit; with real, mixed values the lanes diverge
// and the 150 MB scan ran 8 us longer than with uniform data, profiles/r03_launch).
// ds: the compact duration | span column (devctx.hip), sv / ev: start / end seconds;
// lo/hi: the duration bounds in ds's units (0 / 2^32-1 when a side is absent); bm: the LDS
// bitmaps.
template <int NT, bool DUR, bool RANGE>
__device__ __forceinline__ uint32_t unit_mask(const u32x4 (&d)[kSteps], const u32x4 (&sv4)[kSteps],
                                              const u32x4 (&ev4)[kSteps], const uint32_t (&tv)[NT > 0 ? NT : 1][kSteps],
                                              uint32_t e0, uint32_t n, uint32_t lo, uint32_t hi, uint32_t start_s,
                                              uint32_t end_s, uint32_t bmi4, uint32_t ns4, const uint32_t *s_bm,
                                              int lane) {
  uint32_t mask = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t dv[4] = {d[k].x & 0xffffu, d[k].y & 0xffffu, d[k].z & 0xffffu, d[k].w & 0xffffu};
    const uint32_t sv[4] = {sv4[k].x, sv4[k].y, sv4[k].z, sv4[k].w};
    const uint32_t ev[4] = {ev4[k].x, ev4[k].y, ev4[k].z, ev4[k].w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t ok = uint32_t(e0 + uint32_t(k) * 256 + uint32_t(lane) * 4 + uint32_t(j) < n);
      if (DUR) ok &= uint32_t(dv[j] >= lo) & uint32_t(dv[j] <= hi);
      // req.Start <= endSeconds && req.End >= startSeconds (pipeline.go:62-63)
      if (RANGE) ok &= uint32_t(start_s <= ev[j]) & uint32_t(end_s >= sv[j]);
#pragma unroll
      for (int q = 0; q < (NT > 0 ? NT : 1); q++) {
        if (NT <= 0) break;
        const uint32_t x = (tv[q][k] >> (8 * j)) & 0xffu;
        const uint32_t wd = s_bm[((bmi4 >> (8 * q)) & 0xffu) * 8 + (x >> 5)];  // (x < 256: in the 256-bit map)
        ok &= uint32_t(x < ((ns4 >> (8 * q)) & 0xffu)) & (wd >> (x & 31));
      }
      mask |= (ok & 1u) << (4 * k + j);
    }
  }
  return mask;
}

// A workgroup barrier that waits for this wave's LDS and scalar-memory operations only
// (lgkmcnt), not for its vector loads in flight: __syncthreads()' fence also waits
// vmcnt(0), which at the staging barrier drained the units each wave had already asked for
// (the whole launch-wide burst: ~8-10 us before any wave evaluated its first unit). The
// staging below reads the kernel arguments with scalar loads, so nothing it needs is
// counted by vmcnt. (asm memory clobber: no LDS access moves across it)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// End seconds of a unit's entries: start + span from the ds column, or, for a lane's four
// entries of a step where some span did not fit 16 bits (ends 18 h or more after the start,
// or before it: the escape 0xffff, e.g. the end = 0 entries of pitfall P1), those four from
// the exact end column (rare; only the lanes that need them load: a unit-wide reload moved
// 16 MB more per config-2 query, the PMC count in profiles/r04_final).
template <bool NTL>
__device__ __forceinline__ void unit_ends(const u32x4 (&ds)[kSteps], const u32x4 (&sv)[kSteps], u32x4 (&ev)[kSteps],
                                          const uint32_t *scan, uint32_t npad, uint32_t e0, int lane) {
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t sp[4] = {ds[k].x >> 16, ds[k].y >> 16, ds[k].z >> 16, ds[k].w >> 16};
    const bool esc = sp[0] == 0xffffu || sp[1] == 0xffffu || sp[2] == 0xffffu || sp[3] == 0xffffu;
    ev[k].x = sv[k].x + sp[0];
    ev[k].y = sv[k].y + sp[1];
    ev[k].z = sv[k].z + sp[2];
    ev[k].w = sv[k].w + sp[3];
    if (esc) ev[k] = stream4<NTL>(scan + 2ull * npad, uint64_t(e0) + uint64_t(k) * 256 + uint64_t(lane) * 4);
  }
}

template <int NT, bool DUR, bool RANGE, bool NTL>
__global__ void __launch_bounds__(kPoolThreads, 1) search_pool_kernel(PoolArgs A) {
  const unsigned long long t_start = A.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  __shared__ __attribute__((aligned(16))) PoolBlk s_blk[kArgSegs];
  __shared__ uint32_t s_ub[kArgSegs + 1];
  __shared__ uint32_t s_bm[kArgBms * 8];
  __shared__ uint32_t s_chunk[kPoolChunks];
  __shared__ uint32_t s_next, s_nrec;
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_rec[];  // rec_cap x 6 words
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = blockIdx.x, nsegs = A.nsegs, units = A.units;
  const uint32_t S = A.static_per_wg, L = A.lookahead, cs = A.chunk_shift;
  const uint32_t wv = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(tid) >> 6)), nwv = A.nthreads >> 6;
  // ---- the first two units of a wave, before anything is staged: a wave's first two claims
  // are wv and wv + nwv (claims below S map to the workgroup's static run in order), so their
  // loads go out with the block found by a scalar walk over the kernel arguments (the claims'
  // bookkeeping, a chunk request they may trigger, runs after the staging)
  PoolRegs<NT> ra, rb;
  auto load_arg = [&](PoolRegs<NT> &R, uint32_t u) {
    uint32_t b = 0;
    while (b + 1 < nsegs && u >= A.ubase[b + 1]) b++;
    R.blk = b;
    const PoolBlk &B = A.blk[b];
    const uint32_t npad = B.npad;
    const uint32_t *scan = B.scan;
    R.e0 = A.ebase[b] + (u - A.ubase[b]) * kPoolTile;
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      const uint64_t e = uint64_t(R.e0) + uint64_t(k) * 256 + uint64_t(lane) * 4;
      if (DUR || RANGE) R.d[k] = stream4<NTL>(scan + 3ull * npad, e);
      if (RANGE) R.s[k] = stream4<NTL>(scan + npad, e);
    }
#pragma unroll
    for (int q = 0; q < (NT > 0 ? NT : 1); q++) {
      if (NT <= 0) break;
#pragma unroll
      for (int k = 0; k < kSteps; k++)
        R.tv[q][k] = stream1<NTL>(B.col[q], uint64_t(R.e0) + uint64_t(k) * 256 + uint64_t(lane) * 4);
    }
  };
  // the staging's kernel-argument words first, by vector loads issued ahead of the units'
  // loads: vector loads complete in issue order, so the wait for these (before the LDS
  // writes below) does not wait for the burst of unit loads behind them. The units' loads
  // are unconditional (a wave without a unit reloads unit 0), so the compiler's count of the
  // loads issued after these is the same on every path.
  const uint32_t *blk_words = reinterpret_cast<const uint32_t *>(A.blk);
  const uint32_t xblk = uint32_t(tid) < nsegs * 16 ? blk_words[tid] : 0u;
  const uint32_t xub = uint32_t(tid) < nsegs ? A.blk[tid].ubase : units;
  const uint32_t xbm = tid < kArgBms * 8 ? reinterpret_cast<const uint32_t *>(A.bms)[tid] : 0u;
  const bool pre0 = wv < S, pre1 = wv + nwv < S;
  uint32_t ua = kPoolNone, ub = kPoolNone;
  if (pre0 && uint64_t(w) * S + wv < units) ua = w * S + wv;
  if (pre1 && uint64_t(w) * S + wv + nwv < units) ub = w * S + wv + nwv;
  load_arg(ra, ua != kPoolNone ? ua : 0u);
  load_arg(rb, ub != kPoolNone ? ub : 0u);
  // ---- stage the launch's tables (scalar loads of the kernel arguments; the barrier does not
  // wait for the units' loads above)
  {
    static_assert(kArgSegs * 16 <= kPoolThreads && kArgBms * 8 <= kPoolThreads, "one staging word per thread");
    if (uint32_t(tid) < nsegs * 16) reinterpret_cast<uint32_t *>(s_blk)[tid] = xblk;
    if (uint32_t(tid) <= nsegs) s_ub[tid] = xub;
    if (tid < kArgBms * 8) s_bm[tid] = xbm;
    for (uint32_t i = tid; i < kPoolChunks; i += A.nthreads) s_chunk[i] = kPoolPending;
    if (tid == 0) {
      s_next = min(2 * nwv, S);  // (the claims below it are the waves' first two)
      s_nrec = 0;
      if (w == 0) __hip_atomic_store(A.head_next, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  lds_barrier();
  unsigned long long *const stamps = A.stamps;
  if (stamps && tid == 0) {
    stamps[uint64_t(w) * kStampSlots] = t_start;
    stamps[uint64_t(w) * kStampSlots + 1] = __builtin_amdgcn_s_memrealtime();
    const unsigned long long hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    const unsigned long long xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    stamps[uint64_t(w) * kStampSlots + 8] = (xcc << 32) | hw;
  }
  const uint32_t rec_cap = A.rec_cap;
  const uint32_t dlo = A.has_min ? A.min32 : 0u, dhi = A.has_max ? A.max32 : 0xffffffffu;
  // An LDS chunk slot once its answer is in. Bounded: never reached unless the protocol
  // is broken, and then the query fails on the host instead of the GPU hanging.
  auto poll_chunk = [&](uint32_t k) -> uint32_t {
    uint32_t v, spins = 0;
    while ((v = __hip_atomic_load(&s_chunk[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == kPoolPending) {
      if (++spins > kPoolSpinMax) {
        host_store(A.err, 1u);
        return kPoolNone;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    return v;
  };
  // claim -> unit (or kPoolNone): claims below S are this workgroup's static run; claim
  // S + k*C + off is unit `off` of its k-th dynamic chunk, which the claim L before the
  // chunk's first one requested from the device counter (so a wave rarely waits for it)
  auto trigger = [&](uint32_t c) {
    if (c + L >= S) {
      const uint32_t t = c + L - S;
      const uint32_t k = t >> cs;
      if ((t & ((1u << cs) - 1)) == 0 && k < kPoolChunks) {
        // chunks are requested in order (chunk k after chunk k-1 has its answer), so once
        // one comes back empty every later one is empty too and a wave may stop at the
        // first empty claim without stranding units this workgroup took
        if (lane == 0) {
          uint32_t prev = 0;
          if (k > 0) prev = poll_chunk(k - 1);
          uint32_t val = kPoolNone;
          if (prev != kPoolNone) {
            const uint32_t g = __hip_atomic_fetch_add(A.head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t u0 = uint64_t(A.dyn0) + (uint64_t(g) << cs);
            if (u0 < units) val = uint32_t(u0);
          }
          __hip_atomic_store(&s_chunk[k], val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  };
  auto claim = [&]() -> uint32_t {
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&s_next, 1u);
    c = __builtin_amdgcn_readfirstlane(c);
    trigger(c);
    if (c < S) {  // (a small search's last static runs end at `units`: past it, no work)
      const uint32_t u = w * S + c;
      return u < units ? u : kPoolNone;
    }
    const uint32_t d = c - S, k = d >> cs;
    if (k >= kPoolChunks) return kPoolNone;
    uint32_t v = poll_chunk(k);
    v = __builtin_amdgcn_readfirstlane(v);
    if (v == kPoolNone) return kPoolNone;
    const uint32_t u = v + (d & ((1u << cs) - 1));
    return u < units ? u : kPoolNone;
  };
  // unit -> block slot: lanes test the block boundaries, the ballot counts those passed
  auto load = [&](PoolRegs<NT> &R, uint32_t u) {
    const bool past = uint32_t(lane) < nsegs && u >= s_ub[lane + 1];
    const uint32_t b = __popcll(__ballot(past));
    R.blk = b;
    const PoolBlk &B = s_blk[b];
    const uint32_t npad = __builtin_amdgcn_readfirstlane(B.npad);
    const uint32_t *scan = uniform_ptr(B.scan);
    R.e0 = uint32_t(__builtin_amdgcn_readfirstlane(A.ebase[b])) + (u - __builtin_amdgcn_readfirstlane(B.ubase)) * kPoolTile;
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      const uint64_t e = uint64_t(R.e0) + uint64_t(k) * 256 + uint64_t(lane) * 4;
      if (DUR || RANGE) R.d[k] = stream4<NTL>(scan + 3ull * npad, e);
      if (RANGE) R.s[k] = stream4<NTL>(scan + npad, e);
    }
#pragma unroll
    for (int q = 0; q < (NT > 0 ? NT : 1); q++) {
      if (NT <= 0) break;
      const uint8_t *col = uniform_ptr(B.col[q]);
#pragma unroll
      for (int k = 0; k < kSteps; k++)
        R.tv[q][k] = stream1<NTL>(col, uint64_t(R.e0) + uint64_t(k) * 256 + uint64_t(lane) * 4);
    }
  };
  auto eval = [&](const PoolRegs<NT> &R) {
    const PoolBlk &B = s_blk[R.blk];
    const uint32_t n = __builtin_amdgcn_readfirstlane(B.nent);
    const uint32_t bmi4 = __builtin_amdgcn_readfirstlane(B.bmi4), ns4 = __builtin_amdgcn_readfirstlane(B.nsets4);
    u32x4 ev[kSteps];
    if (RANGE) unit_ends<NTL>(R.d, R.s, ev, uniform_ptr(B.scan), __builtin_amdgcn_readfirstlane(B.npad), R.e0, lane);
    uint32_t mask = unit_mask<NT, DUR, RANGE>(R.d, R.s, ev, R.tv, R.e0, n, dlo, dhi, A.start_s, A.end_s, bmi4,
                                               ns4, s_bm, lane);
    if (__ballot(mask != 0) == 0) return;
    if (A.unit_cap) mask = cap_unit_mask(mask, A.unit_cap, lane);
    // matches: slots in the workgroup's LDS record buffer, record fields gathered now
    const DevBlockDesc *D = A.desc[R.blk];
    const auto *Dc = K4(D);
    const uint8_t *ids = Dc->ids;
    const uint64_t *st_ns = Dc->start_ns, *en_ns = Dc->end_ns;
    const uint32_t *names = Dc->names;
    const uint8_t *id_len = Dc->id_len;
    const uint32_t bidx = __builtin_amdgcn_readfirstlane(B.block_idx);
    const uint32_t cnt = __popc(mask);
    uint32_t slot = 0;
    if (cnt) slot = atomicAdd(&s_nrec, cnt);
    for (int b = 0; b < 4 * kSteps; b++) {
      if (!(mask & (1u << b))) continue;
      const uint32_t r = slot++;
      if (r >= rec_cap) continue;
      const uint32_t ei = R.e0 + uint32_t(b >> 2) * 256 + uint32_t(lane) * 4 + uint32_t(b & 3);
      const u32x4 id = *G<u32x4>(ids + uint64_t(ei) * 16);
      const uint64_t st = G(st_ns)[ei], en = G(en_ns)[ei];
      const uint64_t nm = G(reinterpret_cast<const uint64_t *>(names))[ei];
      const uint32_t il = G(id_len)[ei];
      unsigned long long *d = s_rec + uint64_t(r) * 6;
      d[0] = (unsigned long long)id.x | (unsigned long long)id.y << 32;
      d[1] = (unsigned long long)id.z | (unsigned long long)id.w << 32;
      d[2] = st;
      d[3] = en;
      d[4] = (unsigned long long)ei | (unsigned long long)(bidx | (il << 24)) << 32;
      d[5] = nm;
    }
  };
  // ---- scan: two units in flight per wave (the first two loaded above when static). Every
  // claim index is triggered exactly once, by the wave that holds it, whether or not it
  // maps to a unit: a chunk request it owes is polled by later claims
  if (pre0) trigger(wv);
  if (pre1) trigger(wv + nwv);
  if (!pre0) {
    ua = claim();
    if (ua != kPoolNone) load(ra, ua);
  }
  if (ua != kPoolNone) {
    if (!pre1) {
      ub = claim();
      if (ub != kPoolNone) load(rb, ub);
    }
    for (;;) {
      eval(ra);
      if (ub == kPoolNone) break;
      ua = claim();
      if (ua != kPoolNone) load(ra, ua);
      eval(rb);
      if (ua == kPoolNone) break;
      ub = claim();
      if (ub != kPoolNone) load(rb, ub);
    }
  }
  __syncthreads();
  if (stamps && tid == 0) {
    stamps[uint64_t(w) * kStampSlots + 2] = __builtin_amdgcn_s_memrealtime();
    stamps[uint64_t(w) * kStampSlots + 3] = __builtin_amdgcn_s_memrealtime();
  }
  // ---- records to the workgroup's host segment (write-through), then the count
  const uint32_t total = s_nrec;
  const uint32_t nw = min(total, min(rec_cap, A.seg_cap)) * 6;
  if (nw) {
    auto *dst = reinterpret_cast<unsigned long long *>(A.recs) + uint64_t(w) * A.seg_cap * 6;
    for (uint32_t i = tid; i < nw; i += A.nthreads) host_store(dst + i, s_rec[i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (tid == 0) {
    host_store(A.counts + w, total);
    if (stamps) stamps[uint64_t(w) * kStampSlots + 4] = __builtin_amdgcn_s_memrealtime();
  }
}

// ------------------------------------------------------------------------------------
// static search: the pool kernel's loads, predicates and record hand-off without its
// machinery. One 1024-thread workgroup per CU; wave g of the launch owns the contiguous
// unit run [g * sq + min(g, sr), ...) of the launch's unit space (NW waves, runs differ
// by at most one unit), two units in flight. The block of a unit comes from the wave's own
// walk over the kernel arguments' unit bases (scalar loads, once per block boundary), not
// from LDS: the first loads are issued before anything is staged, and nothing is claimed.
// (scan_probe.hip measured this shape at 27.0 us for 150 MB against 32.4 us for the pool
// kernel with its LDS claims, staging and dynamic chunks.)
template <int NT, bool DUR, bool RANGE, bool NTL>
__global__ void __launch_bounds__(kPoolThreads, 1) search_static_kernel(PoolArgs A) {
  const unsigned long long t_start = A.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  __shared__ uint32_t s_bm[kArgBms * 8];
  __shared__ uint32_t s_nrec;
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_rec[];  // rec_cap x 6 words
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = blockIdx.x, nsegs = A.nsegs, units = A.units;
  const uint32_t nwv = A.nthreads >> 6;
  const uint32_t wave = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(tid) >> 6));
  const uint32_t gw = w * nwv + wave;
  const uint32_t u_begin = gw * A.sq + min(gw, A.sr), u_end = u_begin + A.sq + (gw < A.sr ? 1u : 0u);
  // the wave's current block (all scalar)
  uint32_t b = 0;
  while (b + 1 < nsegs && u_begin >= A.ubase[b + 1]) b++;
  struct Blk {
    const uint32_t *scan;
    const uint8_t *col[NT > 0 ? NT : 1];
    uint32_t npad, nent, ub, ue, eb, bmi4, nsets4, block_idx;
  } B;
  auto set_block = [&](uint32_t bb) {
    const PoolBlk &P = A.blk[bb];
    B.scan = P.scan;
#pragma unroll
    for (int q = 0; q < (NT > 0 ? NT : 1); q++)
      if (NT > 0) B.col[q] = P.col[q];
    B.npad = P.npad;
    B.nent = P.nent;
    B.ub = A.ubase[bb];
    B.ue = A.ubase[bb + 1];
    B.eb = A.ebase[bb];
    B.bmi4 = P.bmi4;
    B.nsets4 = P.nsets4;
    B.block_idx = P.block_idx;
  };
  set_block(b);
  struct Regs {
    u32x4 d[kSteps], s[kSteps];  // ds (duration | span), start seconds
    uint32_t tv[NT > 0 ? NT : 1][kSteps];
    uint32_t e0;
  };
  auto load = [&](Regs &R, uint32_t u) {
    if (u >= B.ue) {  // (runs are short and blocks long: at most a step or two)
      while (b + 1 < nsegs && u >= A.ubase[b + 1]) b++;
      set_block(b);
    }
    R.e0 = B.eb + (u - B.ub) * kPoolTile;
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      const uint64_t e = uint64_t(R.e0) + uint64_t(k) * 256 + uint64_t(lane) * 4;
      if (DUR || RANGE) R.d[k] = stream4<NTL>(B.scan + 3ull * B.npad, e);
      if (RANGE) R.s[k] = stream4<NTL>(B.scan + B.npad, e);
    }
#pragma unroll
    for (int q = 0; q < (NT > 0 ? NT : 1); q++) {
      if (NT <= 0) break;
#pragma unroll
      for (int k = 0; k < kSteps; k++)
        R.tv[q][k] = stream1<NTL>(B.col[q], uint64_t(R.e0) + uint64_t(k) * 256 + uint64_t(lane) * 4);
    }
  };
  const uint32_t rec_cap = A.rec_cap;
  const uint32_t dlo = A.has_min ? A.min32 : 0u, dhi = A.has_max ? A.max32 : 0xffffffffu;
  // (evaluated right after the unit's load, while the block state still describes it)
  auto eval = [&](const Regs &R, uint32_t bslot) {
    const PoolBlk &P = A.blk[bslot];
    const uint32_t n = P.nent, bmi4 = P.bmi4, ns4 = P.nsets4;
    u32x4 ev[kSteps];
    if (RANGE) unit_ends<NTL>(R.d, R.s, ev, P.scan, P.npad, R.e0, lane);
    uint32_t mask = unit_mask<NT, DUR, RANGE>(R.d, R.s, ev, R.tv, R.e0, n, dlo, dhi, A.start_s, A.end_s, bmi4,
                                               ns4, s_bm, lane);
    if (__ballot(mask != 0) == 0) return;
    if (A.unit_cap) mask = cap_unit_mask(mask, A.unit_cap, lane);
    const DevBlockDesc *D = A.desc[bslot];
    const auto *Dc = K4(D);
    const uint8_t *ids = Dc->ids;
    const uint64_t *st_ns = Dc->start_ns, *en_ns = Dc->end_ns;
    const uint32_t *names = Dc->names;
    const uint8_t *id_len = Dc->id_len;
    const uint32_t bidx = P.block_idx;
    const uint32_t cnt = __popc(mask);
    uint32_t slot = 0;
    if (cnt) slot = atomicAdd(&s_nrec, cnt);
    for (int bit = 0; bit < 4 * kSteps; bit++) {
      if (!(mask & (1u << bit))) continue;
      const uint32_t r = slot++;
      if (r >= rec_cap) continue;
      const uint32_t ei = R.e0 + uint32_t(bit >> 2) * 256 + uint32_t(lane) * 4 + uint32_t(bit & 3);
      const u32x4 id = *G<u32x4>(ids + uint64_t(ei) * 16);
      const uint64_t st = G(st_ns)[ei], en = G(en_ns)[ei];
      const uint64_t nm = G(reinterpret_cast<const uint64_t *>(names))[ei];
      const uint32_t il = G(id_len)[ei];
      unsigned long long *d = s_rec + uint64_t(r) * 6;
      d[0] = (unsigned long long)id.x | (unsigned long long)id.y << 32;
      d[1] = (unsigned long long)id.z | (unsigned long long)id.w << 32;
      d[2] = st;
      d[3] = en;
      d[4] = (unsigned long long)ei | (unsigned long long)(bidx | (il << 24)) << 32;
      d[5] = nm;
    }
  };
  // the bitmap words by vector loads issued ahead of the first unit's loads (in-order
  // completion: their wait does not wait for those); the first unit's loads are
  // unconditional (a wave without units reloads the launch's last unit), so every path issues
  // the same loads after these
  const uint32_t xbm = tid < kArgBms * 8 ? reinterpret_cast<const uint32_t *>(A.bms)[tid] : 0u;
  Regs ra, rb;
  uint32_t u = u_begin, ba = b, bb = b;
  load(ra, u < u_end ? u : (units ? units - 1 : 0u));
  ba = b;
  if (tid < kArgBms * 8) s_bm[tid] = xbm;
  if (tid == 0) s_nrec = 0;
  lds_barrier();  // (not waiting for the first unit's loads)
  unsigned long long *const stamps = A.stamps;
  if (stamps && tid == 0) {
    stamps[uint64_t(w) * kStampSlots] = t_start;
    stamps[uint64_t(w) * kStampSlots + 1] = __builtin_amdgcn_s_memrealtime();
    const unsigned long long hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    const unsigned long long xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    stamps[uint64_t(w) * kStampSlots + 8] = (xcc << 32) | hw;
  }
  // two units in flight: ra (u), rb (u + 1)
  while (u < u_end) {
    const bool has_b = u + 1 < u_end;
    if (has_b) {
      load(rb, u + 1);
      bb = b;
    }
    eval(ra, ba);
    if (!has_b) break;
    const bool has_a = u + 2 < u_end;
    if (has_a) {
      load(ra, u + 2);
      ba = b;
    }
    eval(rb, bb);
    u += 2;
  }
  __syncthreads();
  if (stamps && tid == 0) {
    stamps[uint64_t(w) * kStampSlots + 2] = __builtin_amdgcn_s_memrealtime();
    stamps[uint64_t(w) * kStampSlots + 3] = __builtin_amdgcn_s_memrealtime();
  }
  // ---- records to the workgroup's host segment (write-through), then the count
  const uint32_t total = s_nrec;
  const uint32_t nw = min(total, min(rec_cap, A.seg_cap)) * 6;
  if (nw) {
    auto *dst = reinterpret_cast<unsigned long long *>(A.recs) + uint64_t(w) * A.seg_cap * 6;
    for (uint32_t i = tid; i < nw; i += A.nthreads) host_store(dst + i, s_rec[i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (tid == 0) {
    host_store(A.counts + w, total);
    if (stamps) stamps[uint64_t(w) * kStampSlots + 4] = __builtin_amdgcn_s_memrealtime();
  }
}

// ------------------------------------------------------------------------------------
// resident search (TSG_RESIDENT): the static kernel's scan as a kernel that stays on the
// device and takes its queries from a mailbox.
//
// A narrow search's kernel launch costs more than its own duration suggests: the command
// processor fetches the AQL packet over PCIe after the doorbell, runs the acquire fence, then
// launches 4096 waves, whose first loads go out together and whose kernel-argument loads
// queue behind them (the round-4 staging barrier passed 7 us into a 24 us kernel). A
// resident launch has its waves in place: the host writes a query's arguments into a
// mailbox slot of uncached device memory through the BAR, then the slot's header, then the
// doorbell word; each workgroup's first lane polls the doorbell, the workgroup loads the
// slot into LDS (one word per thread), checks the header's sequence number and the checksum
// of the words the query uses (a slot read before the host's writes landed is read again),
// and scans.
//
// Records come out in scan order: wave g of the launch owns a contiguous unit run (the
// static split), keeps its matches in its own LDS region in scan order (ranks from per-step
// ballots), and the workgroup writes its waves' regions one after another to its host
// segment; workgroup w's runs precede workgroup w+1's, so the segments in workgroup order
// are the reference order and the host only concatenates them (no sort). A wave whose
// region overflows reports the workgroup as overflowing (the host reruns the query on the
// other paths).
//
// Lifetime: a workgroup leaves when the host posts a quit, or when no query has been posted
// for idle_ticks of the 100 MHz clock (every wave reaches one of the two); the host relaunches
// at its next query. A post that races the idle exit is seen by the host as the launch
// completing with counts missing: it relaunches and posts again (pool.hip resident_*).
constexpr uint32_t kResSlots = 64, kResSlotBytes = 8192, kResHdrBytes = 64;
constexpr uint32_t kResSearch = 1, kResQuit = 2;
constexpr uint32_t kResMaxUnits = 2048;  // units per workgroup (the LDS tables); larger queries launch plainly
constexpr uint32_t kResRejectWord = 8;   // ResidentArgs::err word counting rejected slot reads
// a timed query's {seen, end} stamps, one 64-byte line per workgroup: four workgroups' 16-byte
// stamps in one line had been partial-line writes to a shared line from four CUs, which land one
// after another (the count lines' lesson, round 5): ~5 us more per timed query
constexpr uint32_t kResStampStride = 8;
struct ResHeader {  // the first 16 B of a mailbox slot; PoolArgs at +kResHdrBytes
  uint32_t seq, cmd, h0, h1;  // h0, h1: res_hash of (seq, cmd, the used argument words)
};
// The slot check: two independently keyed 32-bit sums of a nonlinear per-word mix of (word, its
// index, seq). A slot read while the host's writes were still landing holds some words of query
// seq - kResSlots: an additive checksum accepted any such mix whose plain sum happened to equal
// the new one; here a stale/new mix passes with probability ~2^-64, and a stale
// header (another seq, another cmd) never does.
__host__ __device__ inline uint32_t res_mix(uint32_t x, uint32_t wi, uint32_t seq, uint32_t key) {
  uint32_t h = x ^ (wi * 0x9E3779B1u) ^ (seq * 0x85EBCA77u) ^ key;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
constexpr uint32_t kResKey0 = 0x2545F491u, kResKey1 = 0x6C8E9CF5u;
constexpr uint32_t kResCmdWord = 0xffffffffu;  // (the word index the command is mixed under)
struct ResidentArgs {
  const uint32_t *door;  // uncached device memory: [0] = the last posted sequence number
  const uint8_t *slots;  // uncached device memory: kResSlots x kResSlotBytes (slot = seq % kResSlots)
  uint32_t *err;         // pinned host: [0] set when a slot never verified (the host fails the query),
                         // [kResRejectWord] the slot reads a workgroup rejected (hash mismatch) for a query
  uint32_t first_seq;    // the first query of this launch
  uint32_t idle_ticks;   // s_memrealtime ticks without a post before a workgroup leaves
  uint32_t nthreads, ngroups;
  uint32_t mode, pad;  // TSG_RES_MODE (experiments): bit 0 = units interleaved over the waves (no LDS claims),
                       // bit 3 = no gathers (zero records), bit 4 = no records stored (counts only),
                       // bit 2 = poll the slot header alone, load the arguments once it shows the query,
                       // bit 1 = longer sleeps between doorbell polls
};
static_assert(sizeof(PoolArgs) <= kResSlotBytes - kResHdrBytes && sizeof(PoolArgs) % 4 == 0, "mailbox slot");

// The argument words a query with nsegs blocks and nbms bitmaps uses (the host writes only
// those; the checksum covers exactly them): the block table, descriptors, bitmaps, unit and
// entry bases, and the scalars from `nsegs` on.
__host__ __device__ inline bool res_word_used(uint32_t off, uint32_t nsegs, uint32_t nbms) {
  auto in = [&](uint32_t a, uint32_t n) { return off >= a && off < a + n; };
  return in(uint32_t(offsetof(PoolArgs, blk)), nsegs * uint32_t(sizeof(PoolBlk))) ||
         in(uint32_t(offsetof(PoolArgs, desc)), nsegs * 8u) || in(uint32_t(offsetof(PoolArgs, bms)), nbms * 32u) ||
         in(uint32_t(offsetof(PoolArgs, ubase)), (nsegs + 1) * 4u) || in(uint32_t(offsetof(PoolArgs, ebase)), nsegs * 4u) ||
         (off >= uint32_t(offsetof(PoolArgs, nsegs)) && off < uint32_t(sizeof(PoolArgs)));
}

// 12 waves per workgroup (one workgroup per CU): 168 registers per lane, where the pool kernels'
// 16 waves allow 128 and this kernel's state (two units in flight, the mailbox checks, the
// ordered record output) spilled to scratch; 24 units in flight per CU still cover the HBM
// latency (config 2: 34 MB in flight)
constexpr uint32_t kResWaves = 12, kResThreads = kResWaves * 64;
constexpr uint32_t kResMaxRecs = (96u << 10) / 48;  // the LDS record buffer (kPoolLds / sizeof(MatchRec))
template <int NT, bool DUR, bool RANGE, bool NTL>
__global__ void __launch_bounds__(kResThreads, 1) search_resident_kernel(ResidentArgs R) {
  __shared__ __attribute__((aligned(16))) uint32_t s_args[sizeof(PoolArgs) / 4];
  __shared__ uint32_t s_ctl[4];   // [0] command for this round, [1] checksum, [2] header seq, [3] header csum
  __shared__ uint32_t s_wn[kPoolWaves + 1];
  __shared__ uint32_t s_ub[kResMaxUnits], s_uc[kResMaxUnits];  // per unit of the run: LDS record base, count
  __shared__ uint32_t s_map[kResMaxRecs];  // output record p (scan order) -> its LDS record
  __shared__ uint32_t s_next, s_nrec;
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_rec[];  // rec_cap x 6 words
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = blockIdx.x, nthreads = R.nthreads, nwv = nthreads >> 6;
  const uint32_t wave = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(tid) >> 6));
  const PoolArgs &A = *reinterpret_cast<const PoolArgs *>(s_args);
  constexpr uint32_t kWords = uint32_t(sizeof(PoolArgs) / 4);
  for (uint32_t seq = R.first_seq;; seq++) {
    // ---- wait for query `seq`: wave 0 polls its mailbox slot itself (header + the argument
    // struct, 16-byte system-coherent loads: 52 lines per poll), so the poll that sees the
    // header's sequence number already holds the arguments; they count when the checksum of
    // the words the query uses matches the header's (a slot read while the host's writes were
    // still landing is read again). No post for idle_ticks: the workgroup leaves.
    const uint8_t *slot = R.slots + uint64_t(seq % kResSlots) * kResSlotBytes;
    const uint32_t *words = reinterpret_cast<const uint32_t *>(slot + kResHdrBytes);
    if (wave == 0) {
      constexpr uint32_t kQuads = (kWords + 3) / 4;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t got = 0, bad = 0;  // got: 1 verified, 2 idle, 3 never verified
      const bool hdr_first = (R.mode & 4u) != 0;  // (experiment: poll the header line alone, then load the slot)
      for (uint32_t n = 0; !got; n++) {
        u32x4 hq, v[(kQuads + 63) / 64];
        {
          const u32x4 *hp = reinterpret_cast<const u32x4 *>(slot);
          asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(hq) : "v"(hp) : "memory");
        }
        if (hdr_first) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (uint32_t(__builtin_amdgcn_readfirstlane(hq.x)) != seq) {
            if ((n & 15u) == 15u && __builtin_amdgcn_s_memrealtime() - t0 > R.idle_ticks) got = 2;
            else __builtin_amdgcn_s_sleep(2);
            continue;
          }
        }
#pragma unroll
        for (uint32_t k = 0; k < (kQuads + 63) / 64; k++) {
          const uint32_t qi = min(k * 64 + uint32_t(lane), kQuads - 1);
          const u32x4 *qp = reinterpret_cast<const u32x4 *>(words) + qi;
          asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v[k]) : "v"(qp) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t hseq = uint32_t(__builtin_amdgcn_readfirstlane(hq.x));
        if (hseq != seq) {  // not posted yet
          if ((n & 15u) == 15u && __builtin_amdgcn_s_memrealtime() - t0 > R.idle_ticks) got = 2;
          else if (R.mode & 2u) __builtin_amdgcn_s_sleep(32);
          else __builtin_amdgcn_s_sleep(2);
          continue;
        }
        // nsegs / nbms, from the lanes holding them
        constexpr uint32_t kNs = uint32_t(offsetof(PoolArgs, nsegs) / 4), kNb = uint32_t(offsetof(PoolArgs, nbms) / 4);
        uint32_t ns = 0, nb = 0;
#pragma unroll
        for (uint32_t k = 0; k < (kQuads + 63) / 64; k++) {
          const uint32_t w0 = (k * 64 + uint32_t(lane)) * 4;
          const uint32_t x[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
          for (uint32_t j = 0; j < 4; j++) {
            if (w0 + j == kNs) ns = x[j];
            if (w0 + j == kNb) nb = x[j];
          }
        }
        for (int o = 32; o > 0; o >>= 1) {
          ns |= __shfl_xor(ns, o);
          nb |= __shfl_xor(nb, o);
        }
        const uint32_t cmd = uint32_t(__builtin_amdgcn_readfirstlane(hq.y));
        uint32_t p0 = 0, p1 = 0;
        const bool sane = ns <= uint32_t(kArgSegs) && nb <= uint32_t(kArgBms) && cmd == kResSearch;
#pragma unroll
        for (uint32_t k = 0; k < (kQuads + 63) / 64; k++) {
          const uint32_t qi = k * 64 + uint32_t(lane);
          if (qi >= kQuads) continue;
          const uint32_t x[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
          for (uint32_t j = 0; j < 4; j++) {
            const uint32_t wi = qi * 4 + j;
            if (wi < kWords) {
              s_args[wi] = x[j];
              if (sane && res_word_used(4 * wi, ns, nb)) {
                p0 += res_mix(x[j], wi, seq, kResKey0);
                p1 += res_mix(x[j], wi, seq, kResKey1);
              }
            }
          }
        }
        for (int o = 32; o > 0; o >>= 1) {
          p0 += __shfl_xor(p0, o);
          p1 += __shfl_xor(p1, o);
        }
        p0 += res_mix(cmd, kResCmdWord, seq, kResKey0);
        p1 += res_mix(cmd, kResCmdWord, seq, kResKey1);
        const bool vok = (cmd == kResQuit || sane) && p0 == hq.z && p1 == hq.w;
        if (__builtin_amdgcn_readfirstlane(uint32_t(vok))) {
          got = 1;
          if (lane == 0) {
            s_ctl[0] = cmd;
            if (bad) host_store(R.err + kResRejectWord, bad);
          }
        } else if (++bad > 4096) {
          got = 3;
        } else {
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (lane == 0) s_ctl[1] = got;
    }
    __syncthreads();
    const unsigned long long t_seen = __builtin_amdgcn_s_memrealtime();
    if (s_ctl[1] == 2) return;  // idle
    const bool ok = s_ctl[1] == 1;
    if (!ok) {  // the slot never verified: the host fails the query (err)
      if (tid == 0) host_store(R.err, 1u);
      return;
    }
    if (s_ctl[0] == kResQuit) return;
    // ---- the query. Workgroup w owns the contiguous unit run [ua, ua + nk) (runs differ by at
    // most one unit: every CU the same share); its waves take the run's units one at a time
    // from an LDS counter (the first two of each wave implied), so they finish together; a
    // unit's matches go to the LDS record buffer at once, in scan order, and the unit
    // remembers where (s_ub / s_uc). At the end the units' counts are prefix-summed and each
    // unit's records written to the workgroup's host segment at its offset: the segment is in
    // scan order whichever wave took which unit.
    const uint32_t nsegs = uint32_t(__builtin_amdgcn_readfirstlane(A.nsegs));
    const uint32_t wq = uint32_t(__builtin_amdgcn_readfirstlane(A.wq)), wr = uint32_t(__builtin_amdgcn_readfirstlane(A.wr));
    uint32_t ua = w * wq + min(w, wr), nk = wq + (w < wr ? 1u : 0u);
    if (__builtin_amdgcn_readfirstlane(A.xsplit)) {
      // XCD-weighted runs (the host's measured per-XCD rates, res_split): workgroup w = 8i + x;
      // the runs of every workgroup before it, in workgroup order
      const uint32_t x = w & 7u, i = w >> 3;
      uint32_t s = 0;
#pragma unroll
      for (uint32_t y = 0; y < 8; y++) {
        const uint32_t n = uint32_t(__builtin_amdgcn_readfirstlane(A.xn[y]));
        const uint32_t r = uint32_t(__builtin_amdgcn_readfirstlane(A.xr[y]));
        s += i * n + min(i, r) + (y < x ? n + (i < r ? 1u : 0u) : 0u);
      }
      ua = s;
      nk = uint32_t(__builtin_amdgcn_readfirstlane(A.xn[x])) + (i < uint32_t(__builtin_amdgcn_readfirstlane(A.xr[x])) ? 1u : 0u);
    }
    const uint32_t rec_cap = uint32_t(__builtin_amdgcn_readfirstlane(A.rec_cap));
    auto rfl = [](uint32_t v) { return uint32_t(__builtin_amdgcn_readfirstlane(v)); };
    const uint32_t dlo = rfl(A.has_min ? A.min32 : 0u), dhi = rfl(A.has_max ? A.max32 : 0xffffffffu);
    const uint32_t start_s = rfl(A.start_s), end_s = rfl(A.end_s), ucap = rfl(A.unit_cap);
    const uint32_t *s_bm = reinterpret_cast<const uint32_t *>(A.bms);
    for (uint32_t i = uint32_t(tid); i < nk; i += nthreads) s_uc[i] = 0;
    if (tid == 0) {
      s_next = 0;
      s_nrec = 0;
    }
    __syncthreads();
    // the block of the wave's last load (its fields are read from LDS per load); from the
    // block holding the run's first unit (a walk from block 0 had put up to nsegs dependent LDS
    // reads before a late workgroup's first loads)
    uint32_t b = uint32_t(__popcll(__ballot(uint32_t(lane) + 1 < nsegs && ua >= A.ubase[lane + 1])));
    struct Regs {
      u32x4 d[kSteps], s[kSteps];
      uint32_t tv[NT > 0 ? NT : 1][kSteps];
      uint32_t e0, k;
    };
    // (a wave's claims only grow: the block walk only moves forward)
    auto load = [&](Regs &Rg, uint32_t k) {
      const uint32_t u = ua + k;
      while (b + 1 < nsegs && u >= uint32_t(__builtin_amdgcn_readfirstlane(A.ubase[b + 1]))) b++;
      const PoolBlk &P = A.blk[b];
      const uint32_t *scan = uniform_ptr(P.scan);
      const uint32_t npad = uint32_t(__builtin_amdgcn_readfirstlane(P.npad));
      Rg.k = k;
      Rg.e0 = uint32_t(__builtin_amdgcn_readfirstlane(A.ebase[b])) +
              (u - uint32_t(__builtin_amdgcn_readfirstlane(A.ubase[b]))) * kPoolTile;
#pragma unroll
      for (int kk = 0; kk < kSteps; kk++) {
        const uint64_t e = uint64_t(Rg.e0) + uint64_t(kk) * 256 + uint64_t(lane) * 4;
        if (DUR || RANGE) Rg.d[kk] = stream4<NTL>(scan + 3ull * npad, e);
        if (RANGE) Rg.s[kk] = stream4<NTL>(scan + npad, e);
      }
#pragma unroll
      for (int q = 0; q < (NT > 0 ? NT : 1); q++) {
        if (NT <= 0) break;
        const uint8_t *col = uniform_ptr(P.col[q]);
#pragma unroll
        for (int kk = 0; kk < kSteps; kk++)
          Rg.tv[q][kk] = stream1<NTL>(col, uint64_t(Rg.e0) + uint64_t(kk) * 256 + uint64_t(lane) * 4);
      }
    };
    // the unit's matches into the LDS buffer in scan order (k-step, lane, j), in two halves:
    // eval_a finds them, ranks them and issues the gathers of each lane's first match into a
    // Pend (registers); eval_b stores them to LDS one unit of the same stream later (the loop
    // below). A lane's further matches (rare) are gathered and stored at once. A gather is a
    // full memory latency under the scan's load: waited for before the next unit's loads it had
    // left the wave one unit in flight meanwhile (workgroups holding matches ended ≈ 0.8 us
    // after those without); waited for right after them, ≈ 0.17 us per record (r06 stamps,
    // profiles/r06_xsplit/analysis.txt); one unit later, nothing: the wave waits there for the
    // loads issued after the gathers anyway.
    struct Pend {
      u32x4 id;
      uint64_t st, en, nm;
      uint32_t ei, r, ilw, bidx;  // ilw: the aligned word holding the id length byte
      bool has;
    };
    auto put = [&](uint32_t r, const u32x4 &id, uint64_t st, uint64_t en, uint32_t ei, uint32_t bidx, uint32_t il,
                   uint64_t nm) {
      unsigned long long *d = s_rec + uint64_t(r) * 6;
      d[0] = (unsigned long long)id.x | (unsigned long long)id.y << 32;
      d[1] = (unsigned long long)id.z | (unsigned long long)id.w << 32;
      d[2] = st;
      d[3] = en;
      d[4] = (unsigned long long)ei | (unsigned long long)(bidx | (il << 24)) << 32;
      d[5] = nm;
    };
    auto eval_a = [&](const Regs &Rg, Pend &Pd) {
      Pd.has = false;
      // the unit's block: lanes test the block boundaries, the ballot counts those passed
      const uint32_t u = ua + Rg.k;
      const uint32_t blk = uint32_t(__popcll(__ballot(uint32_t(lane) + 1 < nsegs + 0u && uint32_t(lane) < nsegs &&
                                                      u >= A.ubase[lane + 1])));
      const PoolBlk &P = A.blk[blk];
      const uint32_t n = uint32_t(__builtin_amdgcn_readfirstlane(P.nent));
      const uint32_t bmi4 = uint32_t(__builtin_amdgcn_readfirstlane(P.bmi4)), ns4 = uint32_t(__builtin_amdgcn_readfirstlane(P.nsets4));
      u32x4 ev[kSteps];
      if (RANGE) unit_ends<NTL>(Rg.d, Rg.s, ev, uniform_ptr(P.scan), uint32_t(__builtin_amdgcn_readfirstlane(P.npad)), Rg.e0, lane);
      uint32_t mask = unit_mask<NT, DUR, RANGE>(Rg.d, Rg.s, ev, Rg.tv, Rg.e0, n, dlo, dhi, start_s, end_s, bmi4, ns4,
                                                 s_bm, lane);
      if (__ballot(mask != 0) == 0) return;
      if (ucap) mask = cap_unit_mask(mask, ucap, lane);
      uint32_t cnt = uint32_t(__popc(mask));
      for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
      cnt = uint32_t(__builtin_amdgcn_readfirstlane(cnt));
      if (!cnt) return;
      uint32_t base = 0;
      if (lane == 0) {
        base = atomicAdd(&s_nrec, cnt);
        s_ub[Rg.k] = base;
        s_uc[Rg.k] = cnt;
      }
      base = uint32_t(__builtin_amdgcn_readfirstlane(base));
      const DevBlockDesc *D = uniform_ptr(A.desc[blk]);
      const auto *Dc = K4(D);
      const uint8_t *ids = Dc->ids, *id_len = Dc->id_len;
      const uint64_t *st_ns = Dc->start_ns, *en_ns = Dc->end_ns;
      const uint64_t *names = reinterpret_cast<const uint64_t *>(Dc->names);
      const uint32_t bidx = uint32_t(__builtin_amdgcn_readfirstlane(P.block_idx));
      Pd.bidx = bidx;
      const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
      // each step's first rank for this lane (ballots: every lane takes part)
      uint32_t rank0[kSteps], before = 0;
#pragma unroll
      for (int kk = 0; kk < kSteps; kk++) {
        const uint32_t nib = (mask >> (4 * kk)) & 0xfu;
        uint32_t lower = 0, tot = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint64_t bb = __ballot((nib >> j) & 1u);
          lower += uint32_t(__popcll(bb & below));
          tot += uint32_t(__popcll(bb));
        }
        rank0[kk] = base + before + lower;
        before += tot;
      }
      if (!mask) return;
      {
        const uint32_t bit = uint32_t(__builtin_ctz(mask)), kk = bit >> 2, j = bit & 3u;
        const uint32_t r = (kk ? rank0[1] : rank0[0]) + uint32_t(__popc((mask >> (4 * kk)) & ((1u << j) - 1u)));
        const uint32_t ei = Rg.e0 + kk * 256 + uint32_t(lane) * 4 + j;
        if (r < rec_cap && (R.mode & 8u)) {  // (experiment: no gathers, zero records)
          Pd.has = true;
          Pd.ei = ei;
          Pd.r = r;
          Pd.id = u32x4{0, 0, 0, 0};
          Pd.st = Pd.en = Pd.nm = 0;
          Pd.ilw = 0;
        } else if (r < rec_cap) {
          Pd.has = true;
          Pd.ei = ei;
          Pd.id = *G<u32x4>(ids + uint64_t(ei) * 16);
          Pd.st = G(st_ns)[ei];
          Pd.en = G(en_ns)[ei];
          Pd.nm = G(names)[ei];
          // (the id length's aligned word, untouched until the store: no arithmetic on a
          // gathered value here, or the wave waits for the gathers at once)
          Pd.r = r;
          Pd.ilw = *G<uint32_t>(id_len + (ei & ~3u));
        }
      }
      // a lane's further matches, one at a time (a loop kept rolled: the gathers of 8 records
      // at once had pushed the kernel past its registers)
#pragma unroll 1
      for (uint32_t m = mask & (mask - 1u); m; m &= m - 1) {
        const uint32_t bit = uint32_t(__builtin_ctz(m)), kk = bit >> 2, j = bit & 3u;
        const uint32_t r = (kk ? rank0[1] : rank0[0]) + uint32_t(__popc((mask >> (4 * kk)) & ((1u << j) - 1u)));
        if (r >= rec_cap) continue;
        const uint32_t ei = Rg.e0 + kk * 256 + uint32_t(lane) * 4 + j;
        const u32x4 id = *G<u32x4>(ids + uint64_t(ei) * 16);
        put(r, id, G(st_ns)[ei], G(en_ns)[ei], ei, bidx, G(id_len)[ei], G(names)[ei]);
      }
    };
    auto eval_b = [&](const Pend &Pd) {
      if (Pd.has) put(Pd.r, Pd.id, Pd.st, Pd.en, Pd.ei, Pd.bidx, (Pd.ilw >> (8 * (Pd.ei & 3u))) & 0xffu, Pd.nm);
    };
    const bool interleave = (R.mode & 1u) != 0;
    auto claim = [&](uint32_t prev) -> uint32_t {
      if (interleave) return prev + 2 * nwv;
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(&s_next, 1u);
      return 2 * nwv + uint32_t(__builtin_amdgcn_readfirstlane(c));
    };
    Regs ra, rb;
    uint32_t ka = wave, kb = wave + nwv;
    if (ka < nk) load(ra, ka);
    if (kb < nk) load(rb, kb);
    // a unit's gathers are stored one unit later (eval_b of unit n of a stream runs before
    // eval_a of unit n+1 of the same stream): by then the loads issued after them are being
    // waited for anyway (vector loads complete in order), so a match costs the wave no stall
    Pend pa, pb;
    pa.has = pb.has = false;
    while (ka < nk || kb < nk) {
      if (ka < nk) {
        eval_b(pa);
        eval_a(ra, pa);
        ka = claim(ka);
        if (ka < nk) load(ra, ka);
      }
      if (kb < nk) {
        eval_b(pb);
        eval_a(rb, pb);
        kb = claim(kb);
        if (kb < nk) load(rb, kb);
      }
    }
    eval_b(pa);
    eval_b(pb);
    __syncthreads();
    // ---- units' counts -> exclusive offsets (s_uc in place), then each unit's records to the
    // host segment at its offset, then the count
    const uint32_t total = s_nrec;
    // (two units per thread per pass: a run longer than 2 x nthreads units takes more passes,
    // each carrying the previous passes' total)
    for (uint32_t base = 0, carry = 0; base < nk; base += 2 * nthreads) {
      const uint32_t i0 = base + 2 * uint32_t(tid), i1 = i0 + 1;
      const uint32_t c0 = i0 < nk ? s_uc[i0] : 0u, c1 = i1 < nk ? s_uc[i1] : 0u;
      const uint32_t mine = c0 + c1;
      uint32_t incl = mine;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      if (lane == 63) s_wn[wave] = incl;
      __syncthreads();
      uint32_t woff = 0, pass = 0;
      for (uint32_t v = 0; v < nwv; v++) {
        const uint32_t t = s_wn[v];
        if (v < wave) woff += t;
        pass += t;
      }
      const uint32_t ex = carry + woff + incl - mine;
      __syncthreads();  // (every c0 / c1 / s_wn read before they are overwritten)
      if (i0 < nk) s_uc[i0] = ex;
      if (i1 < nk) s_uc[i1] = ex + c0;
      carry += pass;
      __syncthreads();
    }
    const uint32_t seg_cap = uint32_t(__builtin_amdgcn_readfirstlane(A.seg_cap));
    const bool over = total > rec_cap;
    if (!over && total <= seg_cap && total && !(R.mode & 16u)) {  // (mode 16: experiment, no records out)
      // output record p -> its LDS record: each unit with matches writes its range of the map
      // (a binary search of the offsets per output word had been ~7 dependent LDS reads)
      for (uint32_t k = uint32_t(tid); k < nk; k += nthreads) {
        const uint32_t o = s_uc[k], o1 = k + 1 < nk ? s_uc[k + 1] : total;
        for (uint32_t p = o; p < o1; p++) s_map[p] = s_ub[k] + (p - o);
      }
      __syncthreads();
      // consecutive lanes store consecutive words of the segment (the fabric merges them into
      // whole-line PCIe writes; a record per thread, 8-byte stores each, had been 8x the
      // transactions and made the host wait ~50 us per query for the last count)
      auto *dst0 = reinterpret_cast<unsigned long long *>(uniform_ptr(A.recs)) + uint64_t(w) * seg_cap * 6;
      for (uint32_t i = uint32_t(tid); i < total * 6; i += nthreads) {
        const uint32_t p = i / 6, j = i - p * 6;
        host_store(dst0 + i, s_rec[uint64_t(s_map[p]) * 6 + j]);
      }
    }
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the count last (more matches than the LDS buffer holds: the host reruns the query on the
    // segment / look-back path)
    // with the low 32 bits of the seen / end stamps in the same 16-byte store: a timed query's
    // span costs no store of its own (separate stamp stores had cost ~4-6 us per timed query:
    // before the count, the count waited for their round trip; after it, the next query's first
    // waits did)
    if (tid == 0) {
      uint32_t *cl = uniform_ptr(A.counts) + uint64_t(w) * max(1u, uint32_t(__builtin_amdgcn_readfirstlane(A.cstride)));
      const u32x4 v = {over ? max(total, rec_cap + 1) : total, uint32_t(t_seen), uint32_t(t_end), 0u};
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(cl), "v"(v) : "memory");
    }
    // the full stamps (diagnostics: TSG_RES_DUMP, the XCD calibration) after the count
    if (tid == 0 && A.qstamps) {  // (a 64-byte line per workgroup: kResStampStride)
      unsigned long long *qs = uniform_ptr(A.qstamps) + uint64_t(w) * kResStampStride;
      host_store(qs, t_seen);
      host_store(qs + 1, t_end);
    }
    __syncthreads();  // (the LDS tables are reused by the next query)
  }
}

// ------------------------------------------------------------------------------------
// host
using PoolFn = void (*)(PoolArgs);
template <int NT, bool NTL>
static PoolFn pick_pool3(bool dur, bool range) {
  if (dur && range) return search_pool_kernel<NT, true, true, NTL>;
  if (dur) return search_pool_kernel<NT, true, false, NTL>;
  if (range) return search_pool_kernel<NT, false, true, NTL>;
  return search_pool_kernel<NT, false, false, NTL>;
}
template <bool NTL>
static PoolFn pick_pool_t(uint32_t nterms, bool dur, bool range) {
  switch (nterms) {
    case 0: return pick_pool3<0, NTL>(dur, range);
    case 1: return pick_pool3<1, NTL>(dur, range);
    case 2: return pick_pool3<2, NTL>(dur, range);
    case 3: return pick_pool3<3, NTL>(dur, range);
    default: return pick_pool3<4, NTL>(dur, range);
  }
}
static PoolFn pick_pool(uint32_t nterms, bool dur, bool range, bool ntl) {
  return ntl ? pick_pool_t<true>(nterms, dur, range) : pick_pool_t<false>(nterms, dur, range);
}
template <int NT, bool NTL>
static PoolFn pick_static3(bool dur, bool range) {
  if (dur && range) return search_static_kernel<NT, true, true, NTL>;
  if (dur) return search_static_kernel<NT, true, false, NTL>;
  if (range) return search_static_kernel<NT, false, true, NTL>;
  return search_static_kernel<NT, false, false, NTL>;
}
template <bool NTL>
static PoolFn pick_static_t(uint32_t nterms, bool dur, bool range) {
  switch (nterms) {
    case 0: return pick_static3<0, NTL>(dur, range);
    case 1: return pick_static3<1, NTL>(dur, range);
    case 2: return pick_static3<2, NTL>(dur, range);
    case 3: return pick_static3<3, NTL>(dur, range);
    default: return pick_static3<4, NTL>(dur, range);
  }
}
static PoolFn pick_static(uint32_t nterms, bool dur, bool range, bool ntl) {
  return ntl ? pick_static_t<true>(nterms, dur, range) : pick_static_t<false>(nterms, dur, range);
}
// the device symbol of pick_pool / pick_static's kernel (Itanium mangling of the template)
static std::string kernel_symbol(bool is_static, uint32_t nterms, bool dur, bool range, bool ntl) {
  char b[128];
  std::snprintf(b, sizeof b, "_ZN3tsg%s_kernelILi%uELb%dELb%dELb%dEEEvNS_8PoolArgsE",
                is_static ? "20search_static" : "18search_pool", std::min(nterms, 4u), int(dur), int(range), int(ntl));
  return b;
}

// ---- resident search: host side -------------------------------------------------------
template <int NT, bool NTL>
static void *resident_fn_t(bool dur, bool range) {
  if (dur && range) return reinterpret_cast<void *>(search_resident_kernel<NT, true, true, NTL>);
  if (dur) return reinterpret_cast<void *>(search_resident_kernel<NT, true, false, NTL>);
  if (range) return reinterpret_cast<void *>(search_resident_kernel<NT, false, true, NTL>);
  return reinterpret_cast<void *>(search_resident_kernel<NT, false, false, NTL>);
}
// (every instantiation referenced, so that the code object beside libtsg.so holds them all:
// the resident kernel is launched by symbol through the AQL queue only)
[[maybe_unused]] static void *resident_fn(uint32_t nterms, bool dur, bool range, bool ntl) {
  switch (std::min(nterms, 4u)) {
    case 0: return ntl ? resident_fn_t<0, true>(dur, range) : resident_fn_t<0, false>(dur, range);
    case 1: return ntl ? resident_fn_t<1, true>(dur, range) : resident_fn_t<1, false>(dur, range);
    case 2: return ntl ? resident_fn_t<2, true>(dur, range) : resident_fn_t<2, false>(dur, range);
    case 3: return ntl ? resident_fn_t<3, true>(dur, range) : resident_fn_t<3, false>(dur, range);
    default: return ntl ? resident_fn_t<4, true>(dur, range) : resident_fn_t<4, false>(dur, range);
  }
}
static std::string resident_symbol(uint32_t nterms, bool dur, bool range, bool ntl) {
  char b[128];
  std::snprintf(b, sizeof b, "_ZN3tsg22search_resident_kernelILi%uELb%dELb%dELb%dEEEvNS_12ResidentArgsE",
                std::min(nterms, 4u), int(dur), int(range), int(ntl));
  return b;
}
constexpr size_t kResDoorBytes = 256;  // the doorbell word's page ahead of the slots

// Device contexts open in this process, by device ordinal. A resident launch fills every CU
// of its device; a second context on the same device (the bench's concurrent streams, a
// second engine) would wait behind it, so resident launches run only while a context is
// alone on its device, and opening a second one ends the first one's launch.
static std::mutex g_ctx_mu;
// held by context_opened while it ends other contexts' launches and by context_closed before a
// context leaves the table: a context being shut down is never touched after it left (ADVICE r5;
// order: g_life_mu, then a context's mu — nothing holding a context's mu takes g_life_mu)
static std::mutex g_life_mu;
static std::multimap<int, DeviceCtx *> g_ctxs;
int contexts_on(int ordinal) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  return int(g_ctxs.count(ordinal));
}

// ---- other processes on the device. A resident launch holds every CU: a second
// process's kernels on the same GPU would wait behind it until its idle exit, or starve while it
// stays busy. Each process with a context on a GPU holds an flock on a file of its own named after
// the GPU's PCI bus id (TSG_COTENANT_DIR, default /dev/shm, else /tmp) and bumps a generation word
// in a shared page of that GPU; the resident path runs only while no other live process is
// registered on the GPU, re-counted (a directory scan; a file whose lock can be taken is a dead
// process's, removed) whenever the generation word has moved. TSG_COTENANT=0: no check.
struct CoTenant {
  int refs = 0, gen_fd = -1, live_fd = -1;
  uint32_t *gen = nullptr;
  std::string dir, prefix, live_path;
};
static std::mutex g_cot_mu;
static std::map<std::string, CoTenant> g_cot;
static std::string bus_id(int ordinal) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, ordinal) != hipSuccess) return std::string();
  for (char *c = bus; *c; c++) *c = char(std::tolower(uint8_t(*c)));
  return bus;
}
static void cotenant_register(DeviceCtx &dc) {
  if (DeviceCtx::env_u32("TSG_COTENANT", 1, 0, 1) == 0) return;
  const std::string bus = bus_id(dc.ordinal);
  if (bus.empty()) return;
  std::lock_guard<std::mutex> lk(g_cot_mu);
  CoTenant &ct = g_cot[bus];
  struct Publish {  // (every context of the GPU in this process reads the same registration)
    DeviceCtx &dc;
    CoTenant &ct;
    ~Publish() {
      dc.cot_gen = ct.gen;
      dc.cot_dir = ct.dir;
      dc.cot_prefix = ct.prefix;
    }
  } publish{dc, ct};
  if (ct.refs++ > 0) return;
  const char *e = std::getenv("TSG_COTENANT_DIR");
  ct.dir = e && *e ? e : access("/dev/shm", W_OK) == 0 ? "/dev/shm" : "/tmp";
  ct.prefix = "tsg-gpu-" + bus + ".";
  const std::string gpath = ct.dir + "/" + ct.prefix + "gen";
  ct.gen_fd = open(gpath.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (ct.gen_fd < 0) return;
  (void)fchmod(ct.gen_fd, 0666);  // (another user's process shares the GPU too)
  struct stat st;
  if (fstat(ct.gen_fd, &st) == 0 && st.st_size < 4096 && ftruncate(ct.gen_fd, 4096) != 0) {
    close(ct.gen_fd);
    ct.gen_fd = -1;
    return;
  }
  void *m = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, ct.gen_fd, 0);
  if (m == MAP_FAILED) {
    close(ct.gen_fd);
    ct.gen_fd = -1;
    return;
  }
  ct.gen = static_cast<uint32_t *>(m);
  ct.live_path = ct.dir + "/" + ct.prefix + std::to_string(getpid());
  ct.live_fd = open(ct.live_path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
  if (ct.live_fd >= 0 && flock(ct.live_fd, LOCK_EX | LOCK_NB) != 0) {
    close(ct.live_fd);
    ct.live_fd = -1;
  }
  __atomic_fetch_add(ct.gen, 1u, __ATOMIC_SEQ_CST);
}
static void cotenant_unregister(DeviceCtx &dc) {
  if (!dc.cot_gen) return;
  dc.cot_gen = nullptr;
  const std::string bus = bus_id(dc.ordinal);
  std::lock_guard<std::mutex> lk(g_cot_mu);
  auto it = g_cot.find(bus);
  if (it == g_cot.end() || --it->second.refs > 0) return;
  CoTenant &ct = it->second;
  if (ct.live_fd >= 0) {
    (void)unlink(ct.live_path.c_str());
    close(ct.live_fd);  // (the lock goes with it)
  }
  if (ct.gen) {
    __atomic_fetch_add(ct.gen, 1u, __ATOMIC_SEQ_CST);
    munmap(ct.gen, 4096);
  }
  if (ct.gen_fd >= 0) close(ct.gen_fd);
  g_cot.erase(it);
}
// other live processes registered on dc's GPU (0 when the check is off or unavailable)
static int cotenant_others(DeviceCtx &dc) {
  uint32_t *gen = dc.cot_gen;  // (mapped while this context is registered)
  if (!gen) return 0;
  const uint32_t g = __atomic_load_n(gen, __ATOMIC_ACQUIRE);
  if (dc.res_cotenant >= 0 && g == dc.res_cotenant_gen) return dc.res_cotenant;
  const std::string &dir = dc.cot_dir, &prefix = dc.cot_prefix, mine = prefix + std::to_string(getpid());
  int others = 0;
  if (DIR *d = opendir(dir.c_str())) {
    while (dirent *de = readdir(d)) {
      const std::string name = de->d_name;
      if (name.compare(0, prefix.size(), prefix) != 0 || name == prefix + "gen" || name == mine) continue;
      const std::string path = dir + "/" + name;
      const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) continue;
      if (flock(fd, LOCK_EX | LOCK_NB) == 0) {  // nobody holds it: a process that died registered
        (void)unlink(path.c_str());
      } else {
        others++;
      }
      close(fd);
    }
    closedir(d);
  }
  dc.res_cotenant = others;
  dc.res_cotenant_gen = g;
  return others;
}

void context_opened(DeviceCtx &dc) {
  cotenant_register(dc);
  std::lock_guard<std::mutex> life(g_life_mu);
  std::vector<DeviceCtx *> others;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto r = g_ctxs.equal_range(dc.ordinal);
    for (auto it = r.first; it != r.second; ++it) others.push_back(it->second);
    g_ctxs.emplace(dc.ordinal, &dc);
  }
  for (DeviceCtx *o : others) {
    std::lock_guard<std::mutex> lk(o->mu);
    resident_quit(*o);
  }
}
void context_closed(DeviceCtx &dc) {
  {
    std::lock_guard<std::mutex> life(g_life_mu);
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto r = g_ctxs.equal_range(dc.ordinal);
    for (auto it = r.first; it != r.second; ++it)
      if (it->second == &dc) {
        g_ctxs.erase(it);
        break;
      }
  }
  cotenant_unregister(dc);
}

// A query (or a quit) into mailbox slot seq % kResSlots: the argument words the query uses
// (`parts`: the same words res_word_used names, summed for the checksum), then the header
// whose sequence number the kernel polls — write-combined stores drained by sfence, pushed past
// the host data path by a posted HDP flush (the kernel re-reads a slot whose checksum does not
// match yet).
std::atomic<uint32_t> g_res_torn{0};  // test hook (tsg_debug_set "res_torn"): posts left to tear
static void res_post(DeviceCtx &dc, uint32_t seq, uint32_t cmd, const PoolArgs *PA,
                     const std::vector<std::pair<uint32_t, uint32_t>> *parts) {
  uint8_t *slot = dc.res_mem + kResDoorBytes + size_t(seq % kResSlots) * kResSlotBytes;
  uint32_t h0 = res_mix(cmd, kResCmdWord, seq, kResKey0), h1 = res_mix(cmd, kResCmdWord, seq, kResKey1);
  const auto *src = reinterpret_cast<const uint8_t *>(PA);
  if (PA) {
    for (const auto &pt : *parts) {
      std::memcpy(slot + kResHdrBytes + pt.first, src + pt.first, pt.second);
      for (uint32_t o = 0; o < pt.second; o += 4) {
        uint32_t v;
        std::memcpy(&v, src + pt.first + o, 4);
        h0 += res_mix(v, (pt.first + o) / 4, seq, kResKey0);
        h1 += res_mix(v, (pt.first + o) / 4, seq, kResKey1);
      }
    }
  }
  // test hook: the slot as a read that caught the host's writes half landed would see it — two
  // used words moved by +-d (the plain sum of the words unchanged: the additive check of round 5
  // accepted it) — repaired after 200 us; the kernel must re-read, not run it
  uint32_t torn = g_res_torn.load(std::memory_order_relaxed);
  const bool tear = PA && cmd == kResSearch && torn && g_res_torn.compare_exchange_strong(torn, torn - 1);
  const uint32_t o_s = uint32_t(offsetof(PoolArgs, start_s)), o_e = uint32_t(offsetof(PoolArgs, end_s));
  if (tear) {
    uint32_t a, b;
    std::memcpy(&a, src + o_s, 4);
    std::memcpy(&b, src + o_e, 4);
    a += 0x01000000u;
    b -= 0x01000000u;
    std::memcpy(slot + kResHdrBytes + o_s, &a, 4);
    std::memcpy(slot + kResHdrBytes + o_e, &b, 4);
  }
  __builtin_ia32_sfence();
  // the header's check words, then (after an sfence: posted writes arrive in order) its sequence
  // number, so a read that sees the new seq sees the new check words with it
  const ResHeader h{seq - 1, cmd, h0, h1};
  std::memcpy(slot + 4, reinterpret_cast<const uint8_t *>(&h) + 4, sizeof h - 4);
  __builtin_ia32_sfence();
  std::memcpy(slot, &seq, 4);
  __builtin_ia32_sfence();
  aql_hdp_flush(dc.aql);
  if (tear) {
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) __builtin_ia32_pause();
    std::memcpy(slot + kResHdrBytes + o_s, src + o_s, 4);
    std::memcpy(slot + kResHdrBytes + o_e, src + o_e, 4);
    __builtin_ia32_sfence();
    aql_hdp_flush(dc.aql);
  }
}

// A resident launch of kernel `sym` serving queries from `first_seq` on. false: unavailable.
// `profiled`: the dispatch gets a completion signal with dispatch timestamps of its own
// (tsg_search_batch: the launch's device time, the clock rocprofv3's kernel trace reads).
static bool resident_launch(DeviceCtx &dc, const std::string &sym, uint32_t threads, uint32_t W, uint32_t first_seq) {
  if (!dc.res_mem) {
    void *p = nullptr;
    const size_t bytes = kResDoorBytes + size_t(kResSlots) * kResSlotBytes;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) return false;
    HIP_OK(hipMemsetAsync(p, 0, bytes, dc.stream));
    HIP_OK(hipStreamSynchronize(dc.stream));
    dc.res_mem = static_cast<uint8_t *>(p);
    *reinterpret_cast<volatile uint32_t *>(dc.res_mem) = dc.res_seq;
  }
  const AqlKernel ak = aql_kernel(dc.aql, sym.c_str(), uint32_t(sizeof(ResidentArgs)));
  if (!ak.kobj) return false;
  dc.res_host.ensure(64);
  auto *err = static_cast<uint32_t *>(dc.res_host.p);
  __atomic_store_n(err, 0u, __ATOMIC_RELEASE);
  ResidentArgs RA{};
  RA.door = reinterpret_cast<const uint32_t *>(dc.res_mem);
  RA.slots = dc.res_mem + kResDoorBytes;
  RA.err = err;
  RA.first_seq = first_seq;
  RA.idle_ticks = DeviceCtx::env_u32("TSG_RESIDENT_IDLE_US", 10000, 100, 10000000) * 100u;  // (s_memrealtime: 100 MHz)
  RA.nthreads = threads;
  RA.ngroups = W;
  RA.mode = DeviceCtx::env_u32("TSG_RES_MODE", 0, 0, 255);
  const std::vector<std::pair<uint32_t, uint32_t>> parts{{0u, uint32_t(sizeof RA)}};
  constexpr size_t kPoolLds = 96 << 10;
  const bool prof = dc.res_profile_next;
  dc.res_profile_next = false;
  const int ps = aql_dispatch(dc.aql, ak, W, threads, uint32_t(kPoolLds), &RA, parts, prof);
  if (prof) dc.res_profile_slot = ps;
  dc.res_alive = true;
  dc.res_kernel = sym;
  dc.res_threads = threads;
  dc.res_groups = W;
  dc.res_epoch = dc.mem_epoch;
  dc.res_launches++;
  return true;
}

void resident_quit(DeviceCtx &dc) {
  if (!dc.res_alive) return;
  dc.res_alive = false;
  if (!dc.aql || aql_done(dc.aql)) return;  // (left on its own: idle)
  const uint32_t seq = ++dc.res_seq;
  res_post(dc, seq, kResQuit, nullptr, nullptr);
  dc.res_quits++;
  // (the launch serves every query posted before the quit first: their callers may be waiting)
  const auto t0 = std::chrono::steady_clock::now();
  while (!aql_done(dc.aql)) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
      fail(TSG_E_DEVICE, "resident search kernel did not leave after a quit (5 s)");
    __builtin_ia32_pause();
  }
}

void resident_release(DeviceCtx &dc) {
  resident_quit(dc);
  if (dc.res_mem) (void)hipFree(dc.res_mem);
  dc.res_mem = nullptr;
  dc.res_host.release();
  for (auto &a : dc.res_areas) a.buf.release();
  dc.res_areas.clear();
  for (auto &b : dc.res_quarantine) b.release();
  dc.res_quarantine.clear();
}

uint64_t resident_batch_begin(DeviceCtx &dc) {
  std::lock_guard<std::mutex> lk(dc.mu);
  resident_quit(dc);
  dc.res_profile_next = true;
  dc.res_profile_slot = -1;
  return dc.res_launches;
}
uint64_t resident_batch_end(DeviceCtx &dc, uint64_t launches_before) {
  std::lock_guard<std::mutex> lk(dc.mu);
  const bool one = dc.res_launches == launches_before + 1 && dc.res_profile_slot >= 0;
  resident_quit(dc);  // (the dispatch completes: its end timestamp is written)
  dc.res_profile_next = false;
  const uint64_t ns = one && dc.aql ? aql_time_ns(dc.aql, dc.res_profile_slot) : 0;
  dc.res_profile_slot = -1;
  return ns;
}
static std::atomic<uint32_t> g_groups{0};
// (off by default: equalising the XCDs' mean ends raised every XCD's time per unit, span 24.9 vs
// 24.2 us in paired runs, profiles/r06_xsplit; TSG_RES_XSPLIT=1 turns it on)
static std::atomic<bool> g_xsplit{DeviceCtx::env_u32("TSG_RES_XSPLIT", 0, 0, 1) != 0};
static std::atomic<uint32_t> g_lb_bitmap{DeviceCtx::env_u32("TSG_LB_BITMAP", 2, 0, 2)};
uint32_t debug_groups() { return g_groups.load(std::memory_order_relaxed); }
uint32_t debug_lb_bitmap() { return g_lb_bitmap.load(std::memory_order_relaxed); }
bool debug_xsplit() { return g_xsplit.load(std::memory_order_relaxed); }
int debug_set(const char *name, int64_t value) {
  if (!name) return TSG_E_INVALID;
  if (!std::strcmp(name, "res_torn")) {
    g_res_torn.store(uint32_t(std::max<int64_t>(0, value)));
    return TSG_OK;
  }
  if (!std::strcmp(name, "groups")) {
    g_groups.store(uint32_t(std::min<int64_t>(4096, std::max<int64_t>(0, value))));
    return TSG_OK;
  }
  if (!std::strcmp(name, "xsplit")) {
    g_xsplit.store(value != 0);
    return TSG_OK;
  }
  if (!std::strcmp(name, "lb_bitmap")) {
    g_lb_bitmap.store(uint32_t(std::min<int64_t>(2, std::max<int64_t>(0, value))));
    return TSG_OK;
  }
  return TSG_E_INVALID;
}

// A query's result area (pinned, device-written): [256 B header | counts, cstride words per
// workgroup | stamps, 2 x u64 per workgroup | records, seg_cap per workgroup]. Queries in flight
// at once (concurrent callers, tsg_search_batch) hold one each; an area is reused only after its
// query's records were read.
static constexpr uint32_t kResCountStride = 16;  // one 64-byte line per workgroup's count
static size_t res_area_bytes(uint32_t W, uint32_t seg) {
  return 256 + align_up(size_t(W) * 4 * kResCountStride, 256) + align_up(size_t(W) * 8 * kResStampStride, 256) +
         size_t(W) * seg * sizeof(MatchRec);
}

// The oldest posted query whose counts are not all in, when the launch is gone (it left on its
// idle timeout just as queries were posted): launched again from that query with its kernel; it
// serves the posted queries from their slots (identical results). Queries that completed are never
// served again: their areas may have been reused. Caller holds dc.mu.
static void res_relaunch_inflight(DeviceCtx &dc) {
  if (!dc.aql || !aql_done(dc.aql)) return;
  for (const auto &kv : dc.res_inflight) {
    const DeviceCtx::ResArea &a = dc.res_areas[kv.second];
    const auto *counts = reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(a.buf.p) + 256);
    bool complete = true;
    for (uint32_t w = 0; w < a.W && complete; w++)
      complete = __atomic_load_n(counts + size_t(w) * kResCountStride, __ATOMIC_ACQUIRE) != kCountPending;
    if (complete) continue;
    if (!resident_launch(dc, a.sym, dc.res_threads ? dc.res_threads : kResThreads, a.W, kv.first))
      fail(TSG_E_DEVICE, "resident search relaunch failed");
    dc.res_relaunches++;
    return;
  }
}

// Wait, with dc.mu released, until pred() holds (pred is evaluated with dc.mu held).
template <class P>
static void res_wait_unlocked(DeviceCtx &dc, std::unique_lock<std::mutex> &lk, P &&pred, const char *what) {
  const auto t0 = std::chrono::steady_clock::now();
  while (!pred()) {
    res_relaunch_inflight(dc);
    lk.unlock();
    for (int i = 0; i < 64; i++) __builtin_ia32_pause();
    std::this_thread::yield();
    lk.lock();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) fail(TSG_E_DEVICE, what);
  }
}

// The XCD-weighted split of U units over W workgroups (W = 8 x G): XCD x's share of the units from
// the measured rates (res_xf), each XCD's share even over its G workgroups. Off (even runs) for
// small queries, W not a multiple of 8, or TSG_RES_XSPLIT=0.
static void res_split(const DeviceCtx &dc, PoolArgs &PA, uint32_t U, uint32_t W) {
  PA.xsplit = 0;
  if (!debug_xsplit() || W % 8 || U < 16u * W) return;
  const uint32_t G = W / 8;
  uint32_t T[8], sum = 0;
  for (int x = 0; x < 8; x++) {
    T[x] = uint32_t(double(U) * dc.res_xf[x]);
    sum += T[x];
  }
  for (int x = 0; sum < U; x = (x + 1) & 7, sum++) T[x]++;  // (rounding: a unit each, in XCD order)
  for (int x = 0; x < 8 && sum > U; x = (x + 1) & 7)
    if (T[x]) T[x]--, sum--;
  for (int x = 0; x < 8; x++) {
    PA.xn[x] = T[x] / G;
    PA.xr[x] = T[x] % G;
  }
  PA.xsplit = 1;
}
static uint32_t res_max_run(const PoolArgs &PA, uint32_t U, uint32_t W) {
  if (!PA.xsplit) return (U + W - 1) / W;
  uint32_t m = 0;
  for (int x = 0; x < 8; x++) m = std::max(m, PA.xn[x] + (PA.xr[x] ? 1u : 0u));
  return m;
}

// One query's workgroup stamps {seen, end} -> the XCDs' shares for the next queries. XCD x's
// workgroups took E_x (mean end after the first seen) for n_x units; its rate n_x / (E_x - c) with
// c ~ 2 us of fixed cost (first loads, output) moves the shares toward equal ends — the fixed point
// of the update is E_x equal whatever c is. Shares are smoothed (half old, half new) and kept
// within +-15 % of even. Queries below 32 units per workgroup are not used (their ends are fixed cost).
static void res_calibrate(DeviceCtx &dc, const unsigned long long *qst, const PoolArgs &PA, uint32_t U, uint32_t W) {
  if (W % 8 || U < 32u * W) return;
  unsigned long long lo = ~0ull;
  for (uint32_t w = 0; w < W; w++) lo = std::min(lo, qst[size_t(w) * kResStampStride]);
  double E[8] = {}, n[8] = {};
  uint32_t cnt[8] = {};
  for (uint32_t w = 0; w < W; w++) {
    const uint32_t x = w & 7u, i = w >> 3;
    const unsigned long long e = qst[size_t(w) * kResStampStride + 1];
    if (e < lo || e - lo > 100000000ull) return;  // (a stamp not written: skip the sample)
    E[x] += double(e - lo);
    n[x] += PA.xsplit ? double(PA.xn[x] + (i < PA.xr[x] ? 1u : 0u)) : double(PA.wq + (w < PA.wr ? 1u : 0u));
    cnt[x]++;
  }
  double r[8], rs = 0;
  for (int x = 0; x < 8; x++) {
    if (!cnt[x]) return;
    const double ex = E[x] / cnt[x], nx = n[x] / cnt[x];
    r[x] = nx / std::max(ex - 200.0, 0.25 * ex);  // (100 MHz ticks: 200 = 2 us)
    rs += r[x];
  }
  double fs = 0;
  for (int x = 0; x < 8; x++) {
    const double f = 0.5 * dc.res_xf[x] + 0.5 * r[x] / rs;
    dc.res_xf[x] = std::min(0.125 * 1.15, std::max(0.125 * 0.85, f));
    fs += dc.res_xf[x];
  }
  for (int x = 0; x < 8; x++) dc.res_xf[x] /= fs;
  dc.res_xsamples++;
}

// The resident path of pool_search: 1 = served (out filled), 0 = the records overflowed (the
// caller runs the segment / look-back path), -1 = not available (normal launches). dc.mu (lk) is
// released while the query runs: other callers plan and post their queries meanwhile, and the
// launch serves them back to back.
static int resident_search(DeviceCtx &dc, std::unique_lock<std::mutex> &lk, PoolArgs &PA,
                           const std::vector<ScanSeg> &segs, const std::vector<std::pair<uint32_t, Block *>> &blocks,
                           const tsg_query &q, uint32_t limit, uint32_t flags, bool has_dur, uint32_t threads,
                           uint32_t W, uint32_t rec_cap, Tracer &tr, SearchOut &out) {
  const std::string sym = resident_symbol(q.nterms, has_dur, q.has_range, dc.pool_nt);
  const uint32_t U = PA.units;
  res_split(dc, PA, U, W);
  if (res_max_run(PA, U, W) > kResMaxUnits) return -1;
  // a free result area (D = TSG_RES_DEPTH queries in flight; a caller beyond that waits for one)
  static const uint32_t depth = DeviceCtx::env_u32("TSG_RES_DEPTH", 16, 1, kResSlots - 1);
  if (dc.res_areas.size() < depth) dc.res_areas.resize(depth);
  auto free_area = [&]() -> int {
    for (size_t i = 0; i < dc.res_areas.size(); i++)
      if (!dc.res_areas[i].busy) return int(i);
    return -1;
  };
  if (free_area() < 0)
    res_wait_unlocked(dc, lk, [&] { return free_area() >= 0; }, "resident search: no result area freed (5 s)");
  const int ai = free_area();
  DeviceCtx::ResArea &area = dc.res_areas[size_t(ai)];
  area.busy = true;
  area.sym = sym;
  area.W = W;
  struct AreaRelease {  // (the area and the in-flight entry go back on every exit; under dc.mu)
    DeviceCtx &dc;
    DeviceCtx::ResArea &area;
    std::unique_lock<std::mutex> &lk;
    uint32_t seq = 0;
    bool posted = false;
    ~AreaRelease() {
      if (!lk.owns_lock()) lk.lock();
      if (posted) dc.res_inflight.erase(seq);
      area.busy = false;
    }
  } rel{dc, area, lk};
  // the live launch must serve this shape from the next sequence number: another shape, new
  // block memory, or a launch that left, and no query of another caller still in flight ->
  // quit / launch; queries in flight are served first (a quit is posted behind them)
  for (;;) {
    const bool dead = dc.res_alive && aql_done(dc.aql);
    if (dc.res_alive && !dead && dc.res_kernel == sym && dc.res_groups == W && dc.res_epoch == dc.mem_epoch) break;
    if (dc.res_inflight.empty()) {
      resident_quit(dc);
      if (!resident_launch(dc, sym, threads, W, dc.res_seq + 1)) return -1;
      break;
    }
    res_wait_unlocked(dc, lk, [&] { return dc.res_inflight.empty(); }, "resident search: queries in flight never completed (5 s)");
  }
  const uint32_t nsegs = PA.nsegs, nbms = PA.nbms;
  // the argument words this query uses (res_word_used)
  thread_local std::vector<std::pair<uint32_t, uint32_t>> parts;
  parts.clear();
  parts.push_back({uint32_t(offsetof(PoolArgs, blk)), uint32_t(nsegs * sizeof(PoolBlk))});
  parts.push_back({uint32_t(offsetof(PoolArgs, desc)), uint32_t(nsegs * sizeof(PA.desc[0]))});
  if (nbms) parts.push_back({uint32_t(offsetof(PoolArgs, bms)), uint32_t(nbms * sizeof(PA.bms[0]))});
  parts.push_back({uint32_t(offsetof(PoolArgs, ubase)), uint32_t((nsegs + 1) * sizeof(PA.ubase[0]))});
  parts.push_back({uint32_t(offsetof(PoolArgs, ebase)), uint32_t(nsegs * sizeof(PA.ebase[0]))});
  parts.push_back({uint32_t(offsetof(PoolArgs, nsegs)), uint32_t(sizeof(PoolArgs) - offsetof(PoolArgs, nsegs))});
  hipEvent_t e0, e1;
  const bool timed = (flags & TSG_SEARCH_TIME_DEFER) && dc.defer_slot(e0, e1);
  const size_t tslot = timed ? dc.tring_used - 1 : 0;
  // workgroup stamps: timed queries, and every 16th query for the XCD split (the first 8 all)
  // full workgroup stamps only for the diagnostics that read them per workgroup (a timed query's
  // span comes from the count lines: each carries its workgroup's seen / end stamps' low 32 bits)
  static const bool dump_stamps = std::getenv("TSG_RES_DUMP") != nullptr;
  const bool stamp = (timed && dump_stamps) || (debug_xsplit() && (dc.res_xsamples < 8 || dc.res_qn % 16 == 0));
  dc.res_qn++;
  const uint32_t cs = kResCountStride;
  const size_t hdr = 256, cntb = align_up(size_t(W) * 4 * cs, 256), stb = align_up(size_t(W) * 8 * kResStampStride, 256);
  uint32_t *counts = nullptr;
  unsigned long long *qst = nullptr;
  const uint8_t *recs = nullptr;
  auto post = [&] {
    PA.seg_cap = dc.pool_seg;
    area.buf.ensure(res_area_bytes(W, PA.seg_cap));
    uint8_t *base = static_cast<uint8_t *>(area.buf.p);
    counts = reinterpret_cast<uint32_t *>(base + hdr);
    qst = reinterpret_cast<unsigned long long *>(base + hdr + cntb);
    recs = base + hdr + cntb + stb;
    PA.counts = counts;
    PA.recs = base + hdr + cntb + stb;
    PA.err = reinterpret_cast<uint32_t *>(base);
    PA.qstamps = stamp ? qst : nullptr;
    PA.cstride = cs;
    for (uint32_t w = 0; w < W; w++) counts[size_t(w) * cs] = kCountPending;
    if (stamp)  // (the stamps land after the counts: 0 = not yet)
      for (uint32_t x = 0; x < W; x++) qst[size_t(x) * kResStampStride] = qst[size_t(x) * kResStampStride + 1] = 0;
    if (rel.posted) dc.res_inflight.erase(rel.seq);
    rel.seq = ++dc.res_seq;
    rel.posted = true;
    dc.res_inflight[rel.seq] = uint32_t(ai);
    res_post(dc, rel.seq, kResSearch, &PA, &parts);
    dc.res_queries++;
  };
  // every workgroup's count (stored after its records), with dc.mu released; a launch that ended
  // first (it left on an idle timeout just as this query was posted) is launched again from the
  // oldest query not served (res_relaunch_inflight)
  auto wait = [&] {
    const auto t0 = std::chrono::steady_clock::now();
    const bool prof = prof_on();
    thread_local std::vector<uint8_t> seen;
    seen.assign(W, 0);
    uint32_t lo = 0, nseen = 0;
    const uint32_t seg = PA.seg_cap;
    static const bool prefetch = DeviceCtx::env_u32("TSG_RES_PREFETCH", 1, 0, 1) != 0;
    lk.unlock();
    for (uint32_t it = 1;; it++) {
      // counts not seen yet; a finished workgroup's records are pulled into this core's
      // caches while the others still run (the copy after the wait then hits them)
      for (uint32_t w = lo; w < W; w++) {
        if (seen[w]) {
          if (w == lo) lo++;
          continue;
        }
        const uint32_t c = __atomic_load_n(counts + size_t(w) * cs, __ATOMIC_ACQUIRE);
        if (c == kCountPending) continue;
        seen[w] = 1;
        if (prof && nseen == 0)
          prof_add("res.first_count", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        nseen++;
        if (w == lo) lo++;
        if (prefetch) {
          const uint8_t *p0 = recs + uint64_t(w) * seg * sizeof(MatchRec);
          for (uint64_t o = 0; o < uint64_t(std::min(c, seg)) * sizeof(MatchRec); o += 64) __builtin_prefetch(p0 + o);
          if (stamp) __builtin_prefetch(qst + uint64_t(w) * kResStampStride);  // (a timed query's stamps)
        }
      }
      if (lo == W) {
        if (prof)
          prof_add("res.last_count", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        if (stamp) {  // a timed query's stamps, stored after each workgroup's count (bounded: a missing one reads 0)
          const auto ts = std::chrono::steady_clock::now();
          for (uint32_t x = 0; x < W; x++)
            while ((__atomic_load_n(qst + size_t(x) * kResStampStride, __ATOMIC_ACQUIRE) == 0 ||
                    __atomic_load_n(qst + size_t(x) * kResStampStride + 1, __ATOMIC_ACQUIRE) == 0) &&
                   std::chrono::steady_clock::now() - ts < std::chrono::milliseconds(2))
              __builtin_ia32_pause();
        }
        lk.lock();
        return;
      }
      if ((it & 0xfffffu) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        lk.lock();
        fail(TSG_E_DEVICE, "resident search: no answer in 5 s");
      }
      if ((it & 255u) == 0) {
        lk.lock();
        if (__atomic_load_n(static_cast<uint32_t *>(dc.res_host.p), __ATOMIC_ACQUIRE))
          fail(TSG_E_DEVICE, "resident search: a mailbox slot never verified");
        res_relaunch_inflight(dc);
        lk.unlock();
      }
      __builtin_ia32_pause();
    }
  };
  auto scan = [&](uint64_t &total, uint32_t &maxc) {
    total = 0;
    maxc = 0;
    for (uint32_t w = 0; w < W; w++) {
      total += counts[size_t(w) * cs];
      maxc = std::max(maxc, counts[size_t(w) * cs]);
    }
  };
  uint64_t total = 0;
  uint32_t maxc = 0, reruns = 0;
  try {
    tr.mark("plan");
    post();
    tr.mark("search");
    wait();
    tr.mark("sync");
    scan(total, maxc);
    // a workgroup's records exceed its host segment: a larger segment and the query again; more
    // than its LDS regions hold: the other paths
    while (maxc > std::min(PA.seg_cap, rec_cap)) {
      if (maxc > rec_cap) {
        dc.pool_skip = 16;
        dc.pool_skip_key = pool_query_key(q);
        return 0;
      }
      uint32_t want = 2 * PA.seg_cap;
      while (want < maxc) want <<= 1;
      dc.pool_seg = std::min(want, rec_cap);
      post();
      wait();
      reruns++;
      scan(total, maxc);
    }
  } catch (...) {
    //  the launch may still write into this area: it is set aside until shutdown, the
    // launch is ended (bounded) and the next query starts a new one
    if (!lk.owns_lock()) lk.lock();
    dc.res_quarantine.push_back(area.buf);
    area.buf = DeviceCtx::ResArea().buf;
    try {
      resident_quit(dc);
    } catch (...) {
    }
    dc.res_alive = false;
    throw;
  }
  if (const uint32_t rj = __atomic_exchange_n(static_cast<uint32_t *>(dc.res_host.p) + kResRejectWord, 0u, __ATOMIC_ACQ_REL))
    dc.res_rejects += rj;
  if (dc.pool_seg > 32 && uint64_t(maxc) * 8 < dc.pool_seg) dc.pool_seg >>= 1;
  if (stamp) {
    if (debug_xsplit()) res_calibrate(dc, qst, PA, U, W);
  }
  if (timed) {  // the query's span on the device: first workgroup to see it .. last to finish
    // (from the count lines: the stamps' low 32 bits, 100 MHz: relative to workgroup 0's seen)
    const uint32_t ref = counts[1];
    int64_t dlo = INT64_MAX, dhi = INT64_MIN;
    for (uint32_t w = 0; w < W; w++) {
      dlo = std::min<int64_t>(dlo, int32_t(counts[size_t(w) * cs + 1] - ref));
      dhi = std::max<int64_t>(dhi, int32_t(counts[size_t(w) * cs + 2] - ref));
    }
    const unsigned long long span = dhi > dlo ? uint64_t(dhi - dlo) : 0;
    static const bool dump = std::getenv("TSG_RES_DUMP") != nullptr;
    if (dump) {  // spread of the workgroups' {seen, end} stamps (us after the first seen)
      unsigned long long lo = ~0ull;  // (the full stamps' first seen)
      for (uint32_t w = 0; w < W; w++) lo = std::min(lo, qst[size_t(w) * kResStampStride]);
      std::vector<double> sn(W), en(W);
      for (uint32_t w = 0; w < W; w++) {
        sn[w] = double(qst[size_t(w) * kResStampStride] - lo) / 100.0;
        en[w] = double(qst[size_t(w) * kResStampStride + 1] - lo) / 100.0;
      }
      static const bool raw = std::getenv("TSG_RES_DUMP")[0] == '2';
      if (raw) {  // every workgroup's end (0.01 us after the first seen), workgroup order
        std::string line = "[tsg] resident xsplit:";
        for (int x = 0; x < 8; x++) line += " " + std::to_string(PA.xsplit ? dc.res_xf[x] : 0.125);
        line += "\n[tsg] resident runs:";
        for (uint32_t w = 0; w < W; w++)
          line += " " + std::to_string(PA.xsplit ? PA.xn[w & 7] + ((w >> 3) < PA.xr[w & 7] ? 1u : 0u) : PA.wq + (w < PA.wr ? 1u : 0u));
        line += "\n[tsg] resident seen:";
        for (uint32_t w = 0; w < W; w++) line += " " + std::to_string(qst[size_t(w) * kResStampStride] - lo);
        line += "\n[tsg] resident ends:";
        for (uint32_t w = 0; w < W; w++) line += " " + std::to_string(qst[size_t(w) * kResStampStride + 1] - lo);
        line += "\n[tsg] resident counts:";
        for (uint32_t w = 0; w < W; w++) line += " " + std::to_string(counts[size_t(w) * cs]);
        std::fprintf(stderr, "%s\n", line.c_str());
      }
      std::sort(sn.begin(), sn.end());
      std::sort(en.begin(), en.end());
      std::fprintf(stderr, "[tsg] resident stamps us: seen p50 %.2f p90 %.2f max %.2f | end min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f\n",
                   sn[W / 2], sn[W * 9 / 10], sn[W - 1], en[0], en[W / 10], en[W / 2], en[W * 9 / 10], en[W - 1]);
    }
    if (dc.tring_res.size() < dc.tring_used) dc.tring_res.resize(dc.tring_used);
    dc.tring_aql[tslot] = -3;
    dc.tring_res[tslot] = span * 10ull;  // (100 MHz ticks)
  }
  out.kernel_ns = out.scan_ns = 0;
  out.reruns = reruns;
  out.resident = true;
  tr.mark("events");
  // records: the segments in workgroup order are the reference order (static runs, each
  // wave's matches in scan order); a limit keeps each block part's first L
  const uint32_t seg = PA.seg_cap;
  const auto *prec = reinterpret_cast<const SearchOut::Rec *>(recs);
  thread_local std::vector<uint32_t> pos;
  uint32_t max_idx = 0;
  for (const auto &sg : segs) max_idx = std::max(max_idx, sg.block_idx);
  pos.assign(size_t(max_idx) + 1, 0);
  for (uint32_t i = 0; i < PA.nsegs; i++) pos[segs[i].block_idx] = i;
  thread_local std::vector<uint64_t> per;
  per.assign(PA.nsegs, 0);
  out.recs.resize(total);
  uint64_t kept = 0;
  uint64_t run = 0, ps = ~0ull, cut = 0;
  for (uint32_t w = 0; w < W; w++) {
    const SearchOut::Rec *r = prec + uint64_t(w) * seg;
    for (uint32_t i = 0, c = counts[size_t(w) * cs]; i < c; i++) {
      const uint32_t bi = r[i].block_il & 0xffffffu;
      const uint64_t s_i = bi <= max_idx ? pos[bi] : 0;
      if (s_i != ps) {
        ps = s_i;
        run = 0;
        cut = limit ? std::min<uint64_t>(limit, segs[s_i].cap) : segs[s_i].cap;
      }
      if (run++ < cut) {
        out.recs[kept++] = r[i];
        per[s_i]++;
      }
    }
  }
  out.recs.resize(kept);
  for (uint32_t i = 0; i < PA.nsegs; i++)
    for (size_t bi = 0; bi < blocks.size(); bi++)
      if (blocks[bi].first == segs[i].block_idx) out.block_counts[bi] = per[i];
  out.scan_bytes += uint64_t(W) * 4 + kept * 32;
  if (has_dur && q.has_range)
    for (const auto &sg : segs) out.scan_bytes -= 4ull * (sg.n - sg.e0);
  tr.mark("post");
  return 1;
}

// One search_pool_kernel launch for a narrow search (every block scanned whole; a limit
// cuts each block's records to its first `cap` on the host). Returns false, with
// nothing written to `out`, when a workgroup found more matches than its record buffer
// holds: the caller then runs the segment / look-back path.
bool pool_search(DeviceCtx &dc, const std::vector<std::pair<uint32_t, Block *>> &blocks, const tsg_query &q,
                 uint32_t limit, uint32_t flags, const std::vector<ScanSeg> &segs, const std::vector<NarrowSeg> &nsegv,
                 const std::vector<std::array<uint32_t, 8>> &nbms,
                 const std::vector<std::array<uint8_t, kArgTerms>> &nbmi,
                 const std::vector<const DevBlockDesc *> &seg_desc, bool has_dur, Tracer &tr, SearchOut &out,
                 std::unique_lock<std::mutex> &lk) {
  hipStream_t s = dc.stream;
  const uint32_t nsegs = uint32_t(segs.size()), W = uint32_t(dc.num_cu);
  PoolArgs PA;
  std::memset(&PA, 0, sizeof PA);
  // limit L: each block's part needs its first L records only (ids are unique within a
  // block: the consumer takes at most L from it), so units keep their first L (parts start
  // on unit boundaries)
  PA.unit_cap = limit;
  for (const auto &sg : segs)
    if (sg.e0 % kPoolTile) PA.unit_cap = 0;
  uint32_t U = 0;
  for (uint32_t i = 0; i < nsegs; i++) {
    PoolBlk &b = PA.blk[i];
    const NarrowSeg &ns = nsegv[i];
    b.scan = ns.scan;
    for (uint32_t t = 0; t < q.nterms; t++) {
      b.col[t] = ns.ncol + uint64_t(ns.slot[t]) * ns.npad;
      b.bmi4 |= uint32_t(nbmi[i][t]) << (8 * t);
      b.nsets4 |= uint32_t(ns.nsets[t]) << (8 * t);
    }
    b.npad = ns.npad;
    b.nent = uint32_t(segs[i].n);
    b.ubase = U;
    b.block_idx = segs[i].block_idx;
    PA.desc[i] = seg_desc[i];
    PA.ubase[i] = U;
    PA.ebase[i] = uint32_t(segs[i].e0);  // (a multiple of kPoolTile)
    const uint64_t u = (segs[i].n - segs[i].e0 + kPoolTile - 1) / kPoolTile;
    if (uint64_t(U) + u >= (1ull << 31)) return false;
    U += uint32_t(u);
  }
  PA.ubase[nsegs] = U;
  for (size_t j = 0; j < nbms.size(); j++)
    for (int x = 0; x < 8; x++) PA.bms[j][x] = nbms[j][size_t(x)];
  // static runs: (100 - dyn)% of the units split evenly; the rest in dynamic chunks
  uint32_t S = uint32_t(uint64_t(U) * (100 - dc.pool_dyn_pct) / 100 / W);
  // small searches (a limit query's first wave, one block): every unit static. Their
  // refill triggers would all fall in the first two claim rounds, and chunks are
  // requested strictly in order: a chain of device-counter round trips
  if (S < dc.pool_small) S = uint32_t((uint64_t(U) + W - 1) / W);
  // units per dynamic claim: TSG_POOL_CHUNK (16), at most half a workgroup's static run
  uint32_t cs = dc.pool_chunk_shift;
  while (cs > 0 && (1u << cs) > std::max(1u, S / 2)) cs--;
  const uint32_t dyn_units = U > S * W ? U - S * W : 0u;
  while (((dyn_units + (1u << cs) - 1) >> cs) + 64 > kPoolChunks) cs++;
  PA.nsegs = nsegs;
  PA.units = U;
  PA.static_per_wg = S;
  PA.dyn0 = S * W;
  PA.chunk_shift = cs;
  PA.lookahead = std::min(dc.pool_lookahead, S);
  PA.has_min = q.has_min;
  PA.has_max = q.has_max;
  // duration bounds in the ds column's units (2 x whole ms + a remainder bit: devctx.hip):
  // dur >= m ms <=> ds >= 2m, dur <= M ms <=> ds <= 2M (callers: m, M <= kDs16MaxMs)
  PA.min32 = q.has_min ? uint32_t(2 * (q.min_ns / 1000000ull)) : 0u;
  PA.max32 = q.has_max ? uint32_t(2 * (q.max_ns / 1000000ull)) : 0u;
  PA.start_s = q.start_s;
  PA.end_s = q.end_s;
  // LDS: the record buffer is sized so that one workgroup takes more than half a CU. The
  // host segments are smaller (dc.pool_seg records per workgroup, adaptive): the records
  // of a sparse query stay on a few pages of pinned memory
  constexpr size_t kPoolLds = 96 << 10;
  const uint32_t rec_cap = std::min(dc.pool_rec, uint32_t(kPoolLds / sizeof(MatchRec)));
  if (uint64_t(W) * rec_cap > (1u << 20)) return false;  // (record slots are 20-bit in the host's sort keys)
  PA.rec_cap = rec_cap;
  const size_t hdr = 256, cntb = align_up(size_t(W) * 4, 256);
  if (dc.pool_head.ensure(256)) {  // then self-resetting
    HIP_OK(hipMemsetAsync(dc.pool_head.p, 0, dc.pool_head.cap, s));
    HIP_OK(hipStreamSynchronize(s));  // (launches may go to the AQL queue, which does not follow this stream)
  }
  if (!dc.aql_tried) {
    dc.aql_tried = true;
    dc.aql = aql_open(dc.ordinal);
  }
  unsigned *heads = static_cast<unsigned *>(dc.pool_head.p);
  static const bool want_stamps = std::getenv("TSG_STAMPS") != nullptr;
  if (want_stamps) {
    dc.stamps.ensure(size_t(W) * kStampSlots * 8);
    HIP_OK(hipMemsetAsync(dc.stamps.p, 0, size_t(W) * kStampSlots * 8, s));
    PA.stamps = static_cast<unsigned long long *>(dc.stamps.p);
  }
  const bool use_static = uint64_t(U) < uint64_t(dc.pool_static_units) * W;
  const PoolFn fn = use_static ? pick_static(q.nterms, has_dur, q.has_range, dc.pool_nt)
                               : pick_pool(q.nterms, has_dur, q.has_range, dc.pool_nt);
  if (!dc.pool_attr.count(reinterpret_cast<const void *>(fn))) {
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                               int(kPoolLds)));
    dc.pool_attr.insert(reinterpret_cast<const void *>(fn));
  }
  const uint32_t threads = 64 * dc.pool_waves;
  PA.nthreads = threads;
  PA.ngroups = W;
  PA.sq = U / (W * (threads / 64));
  PA.sr = U % (W * (threads / 64));
  PA.nbms = uint32_t(nbms.size());
  PA.wq = U / W;
  PA.wr = U % W;
  const bool time_all = flags & TSG_SEARCH_TIME_ALL, time_scan = flags & (TSG_SEARCH_TIME_SCAN | TSG_SEARCH_TIME_ALL);
  // the resident kernel serves the query when it can (the only context on the device, no
  // per-call HIP events or stamps asked for); otherwise the queue and the CUs are freed first
  // (and no other process has a context on the GPU: cotenant_others)
  if (dc.res_on && dc.aql && !want_stamps && !time_scan && (U + W - 1) / W <= kResMaxUnits &&
      contexts_on(dc.ordinal) == 1) {
    if (cotenant_others(dc) == 0) {
      const int r = resident_search(dc, lk, PA, segs, blocks, q, limit, flags, has_dur, kResThreads, W, rec_cap, tr, out);
      if (r >= 0) return r == 1;
    } else {
      dc.res_cotenant_queries++;
      out.path |= TSG_PATH_COTENANT;
    }
  }
  resident_quit(dc);
  dc.res_plain_queries++;
  hipEvent_t e0 = dc.es0, e1 = dc.es1;
  const bool defer = !time_scan && (flags & TSG_SEARCH_TIME_DEFER) && dc.defer_slot(e0, e1);
  uint32_t *counts = nullptr;
  const uint8_t *recs = nullptr;
  bool via_aql = false;  // the launch being waited for went to the AQL queue
  auto launch = [&](bool first) {
    PA.seg_cap = dc.pool_seg;
    dc.hres.ensure(hdr + cntb + size_t(W) * PA.seg_cap * sizeof(MatchRec));
    uint8_t *base = static_cast<uint8_t *>(dc.hres.p);
    counts = reinterpret_cast<uint32_t *>(base + hdr);
    recs = base + hdr + cntb;
    PA.counts = counts;
    PA.recs = base + hdr + cntb;
    PA.err = reinterpret_cast<uint32_t *>(base);
    *reinterpret_cast<volatile uint32_t *>(base) = 0;
    PA.head = heads + 32 * dc.pool_parity;
    PA.head_next = heads + 32 * (dc.pool_parity ^ 1u);
    std::fill_n(counts, W, kCountPending);  // (each workgroup stores its count last)
    if (first && time_all) HIP_OK(hipEventRecord(dc.ev0, s));
    // timing: the first launch on e0/e1 (scan time or a deferred pair), a rerun on er0/er1
    const bool timed = first ? (time_scan || defer) : time_scan;
    hipEvent_t t0 = first ? e0 : dc.er0, t1 = first ? e1 : dc.er1;
    AqlKernel ak;
    via_aql = false;
    // AQL for untimed launches and for deferred-timed first launches (timed by the queue's own
    // dispatch timestamps, as the untimed ones run); explicit per-call timing stays on HIP events
    const bool aql_timed = first && defer && !time_scan;
    if ((!timed || aql_timed) && !want_stamps && dc.aql)
      ak = aql_kernel(dc.aql, kernel_symbol(use_static, q.nterms, has_dur, q.has_range, dc.pool_nt).c_str(),
                      uint32_t(sizeof(PoolArgs)));
    if (ak.kobj) {
      // our own AQL packet (aql.hpp): only the argument words this launch's kernel reads
      thread_local std::vector<std::pair<uint32_t, uint32_t>> parts;
      parts.clear();
      parts.push_back({uint32_t(offsetof(PoolArgs, blk)), uint32_t(nsegs * sizeof(PoolBlk))});
      parts.push_back({uint32_t(offsetof(PoolArgs, desc)), uint32_t(nsegs * sizeof(PA.desc[0]))});
      if (!nbms.empty()) parts.push_back({uint32_t(offsetof(PoolArgs, bms)), uint32_t(nbms.size() * sizeof(PA.bms[0]))});
      parts.push_back({uint32_t(offsetof(PoolArgs, ubase)), uint32_t((nsegs + 1) * sizeof(PA.ubase[0]))});
      parts.push_back({uint32_t(offsetof(PoolArgs, ebase)), uint32_t(nsegs * sizeof(PA.ebase[0]))});
      parts.push_back({uint32_t(offsetof(PoolArgs, nsegs)), uint32_t(sizeof(PoolArgs) - offsetof(PoolArgs, nsegs))});
      const int ps = aql_dispatch(dc.aql, ak, W, threads, uint32_t(kPoolLds), &PA, parts, aql_timed);
      if (aql_timed) dc.tring_aql[dc.tring_used - 1] = ps >= 0 ? ps : -2;  // (the slot defer_slot took; -2: untimed)
      via_aql = true;
    } else if (timed && dc.ext_events) {  // stamped from the dispatch packet itself
      void *kargs[] = {&PA};
      HIP_OK(hipExtLaunchKernel(reinterpret_cast<const void *>(fn), dim3(W), dim3(threads), kargs, kPoolLds, s, t0,
                                t1, 0));
    } else {
      if (timed) HIP_OK(hipEventRecord(t0, s));
      fn<<<W, threads, kPoolLds, s>>>(PA);
      HIP_OK(hipGetLastError());
      if (timed) HIP_OK(hipEventRecord(t1, s));
    }
    if (first && time_all) HIP_OK(hipEventRecord(dc.ev1, s));
    if (!use_static) dc.pool_parity ^= 1u;  // (the static kernel claims nothing)
  };
  // completion: every workgroup's count (stored after its records completed, read with
  // acquire loads); finished segments are pulled into this core's caches meanwhile; the
  // stream is queried now and then so that a kernel that dies fails the search
  auto wait = [&] {
    thread_local std::vector<uint8_t> seen;
    seen.assign(W, 0);
    const uint32_t seg = PA.seg_cap;
    uint32_t lo = 0;
    for (uint32_t it = 1; lo < W; it++) {
      for (uint32_t w = lo; w < W; w++) {
        if (seen[w]) {
          if (w == lo) lo++;
          continue;
        }
        const uint32_t c = __atomic_load_n(counts + w, __ATOMIC_ACQUIRE);
        if (c == kCountPending) continue;
        seen[w] = 1;
        if (w == lo) lo++;
        const uint8_t *p0 = recs + uint64_t(w) * seg * sizeof(MatchRec);
        for (uint64_t o = 0; o < uint64_t(std::min(c, seg)) * sizeof(MatchRec); o += 64) __builtin_prefetch(p0 + o);
      }
      if (lo == W) break;
      if ((it & 255u) == 0) {
        const hipError_t e = via_aql ? (aql_done(dc.aql) ? hipSuccess : hipErrorNotReady) : hipStreamQuery(s);
        if (e == hipSuccess) {
          bool all = true;
          for (uint32_t w = 0; w < W && all; w++) all = __atomic_load_n(counts + w, __ATOMIC_ACQUIRE) != kCountPending;
          if (all) break;
          fail(TSG_E_DEVICE, "pool search kernel completed without storing every workgroup count");
        }
        if (e != hipErrorNotReady) HIP_OK(e);
      }
      __builtin_ia32_pause();
    }
  };
  auto scan_counts = [&](uint64_t &total, uint32_t &maxc) {
    if (__atomic_load_n(PA.err, __ATOMIC_ACQUIRE))
      fail(TSG_E_DEVICE, "pool search: a workgroup's chunk poll ran past its bound (claim protocol broken)");
    total = 0;
    maxc = 0;
    for (uint32_t w = 0; w < W; w++) {
      total += counts[w];
      maxc = std::max(maxc, counts[w]);
    }
  };
  tr.mark("plan");
  launch(true);
  tr.mark("search");
  wait();
  tr.mark("sync");
  if (want_stamps) print_stamps(dc, W, true);
  uint64_t total = 0;
  uint32_t maxc = 0;
  scan_counts(total, maxc);
  // A workgroup's count depends on which dynamic chunks it won, so a rerun can overflow
  // where the first launch did not: launch until every count fits its segment (segments
  // double each time, at most up to the LDS buffer), or leave for the other paths.
  uint32_t reruns = 0;
  float rerun_ms = 0;
  // (a workgroup keeps at most min(seg_cap, rec_cap) records: its LDS buffer can be the
  // smaller one, TSG_POOL_REC)
  if (maxc > std::min(PA.seg_cap, rec_cap)) {
    for (;;) {
      if (maxc > rec_cap) {  // dense: this query (and its next few searches) take the other paths
        dc.pool_skip = 16;
        dc.pool_skip_key = pool_query_key(q);
        return false;
      }
      if (maxc <= PA.seg_cap) break;
      uint32_t want = 2 * PA.seg_cap;  // (headroom: the next launch's split differs)
      while (want < maxc) want <<= 1;
      dc.pool_seg = std::min(want, rec_cap);
      // a rerun produces the records: its time counts too
      launch(false);
      wait();
      if (time_scan) {
        float ms = 0;
        HIP_OK(hipEventSynchronize(dc.er1));
        HIP_OK(hipEventElapsedTime(&ms, dc.er0, dc.er1));
        rerun_ms += ms;
      }
      reruns++;
      scan_counts(total, maxc);
    }
  } else if (dc.pool_seg > 32 && uint64_t(maxc) * 8 < dc.pool_seg) {
    dc.pool_seg >>= 1;  // sparse again: smaller segments from the next query on
  }
  const uint32_t seg = PA.seg_cap;
  float ms = 0, sms = 0;
  if (time_all) {
    HIP_OK(hipEventSynchronize(dc.ev1));
    HIP_OK(hipEventElapsedTime(&ms, dc.ev0, dc.ev1));
  }
  if (time_scan) {
    HIP_OK(hipEventSynchronize(e1));
    HIP_OK(hipEventElapsedTime(&sms, e0, e1));
  }
  out.kernel_ns = uint64_t(double(ms + (time_all ? rerun_ms : 0.f)) * 1e6);
  out.scan_ns = uint64_t(double(sms + rerun_ms) * 1e6);
  out.reruns = reruns;
  tr.mark("events");
  // records: the blocks' order in the launch, the entry index within a block (the
  // reference scan order) = the record's position in the launch's unit space. Ordered
  // by one bucket pass over that position (about one record per bucket) and an
  // insertion fix-up; a crowded bucket is sorted on its own.
  uint32_t max_idx = 0;
  for (const auto &sg : segs) max_idx = std::max(max_idx, sg.block_idx);
  thread_local std::vector<uint32_t> pos, bucket;
  pos.assign(size_t(max_idx) + 1, 0);
  for (uint32_t i = 0; i < nsegs; i++) pos[segs[i].block_idx] = i;
  thread_local std::vector<uint64_t> keys, sorted;
  keys.resize(total);
  sorted.resize(total);
  // keys straight from the pinned segments: position << 20 | record slot (w * seg + i);
  // the gather below reads the same lines again, from cache
  const auto *prec = reinterpret_cast<const SearchOut::Rec *>(recs);
  thread_local std::vector<uint64_t> per;
  per.assign(nsegs, 0);
  const uint64_t span = uint64_t(U) * kPoolTile;  // positions < span <= 2^31 * 512
  uint32_t lb = 6;
  while ((1ull << lb) < total && lb < 20) lb++;
  uint32_t sb = 0;
  while (((span - 1) >> sb) >= (1ull << lb)) sb++;  // bucket of the largest position < 2^lb
  bucket.assign((size_t(1) << lb) + 1, 0);
  uint64_t nrec = 0;
  for (uint32_t w = 0; w < W; w++)
    for (uint32_t i = 0; i < counts[w]; i++) {
      const uint64_t slot = uint64_t(w) * seg + i;  // (< 256 x 2048 < 2^20)
      const SearchOut::Rec &r = prec[slot];
      const uint32_t bi = r.block_il & 0xffffffu;
      const uint32_t ps = bi <= max_idx ? pos[bi] : 0;
      per[ps]++;
      const uint64_t at = uint64_t(PA.blk[ps].ubase) * kPoolTile + (r.entry - PA.ebase[ps]);
      keys[nrec++] = (at << 20) | slot;
      bucket[size_t(at >> sb) + 1]++;  // (bucket counts in the same pass)
    }
  tr.mark("post.keys");
  for (size_t b = 1; b < bucket.size(); b++) bucket[b] += bucket[b - 1];
  for (uint64_t i = 0; i < total; i++) sorted[bucket[size_t((keys[i] >> 20) >> sb)]++] = keys[i];
  // (bucket[b] is now the end of bucket b)
  for (size_t b = 0, lo = 0; b + 1 < bucket.size(); lo = bucket[b], b++) {
    const size_t hi = bucket[b];
    if (hi - lo <= 1) continue;
    if (hi - lo > 32) {
      std::sort(sorted.begin() + lo, sorted.begin() + hi);
      continue;
    }
    for (size_t i = lo + 1; i < hi; i++) {
      const uint64_t k = sorted[i];
      size_t j = i;
      while (j > lo && sorted[j - 1] > k) {
        sorted[j] = sorted[j - 1];
        j--;
      }
      sorted[j] = k;
    }
  }
  // limit L: each block's part keeps its first L matches in scan order (the records of a
  // part all lie in its range [e0, e1)); the sorted records of a block are contiguous, so
  // the cut keeps a prefix of each block's run
  tr.mark("post.sort");
  auto cut = [&](uint64_t i) { return limit ? std::min<uint64_t>(limit, segs[i].cap) : segs[i].cap; };
  out.recs.resize(total);
  uint64_t kept = 0;
  for (uint64_t i = 0, run = 0, ps = ~0ull, c = 0; i < total; i++) {
    const SearchOut::Rec &r = prec[sorted[i] & 0xfffffu];
    const uint32_t bi = r.block_il & 0xffffffu;
    const uint64_t seg_i = bi <= max_idx ? pos[bi] : 0;
    if (seg_i != ps) {
      ps = seg_i;
      run = 0;
      c = cut(seg_i);
    }
    if (run++ < c) out.recs[kept++] = r;
  }
  out.recs.resize(kept);
  for (uint32_t i = 0; i < nsegs; i++) {
    per[i] = std::min<uint64_t>(per[i], cut(i));
    for (size_t bi = 0; bi < blocks.size(); bi++)
      if (blocks[bi].first == segs[i].block_idx) out.block_counts[bi] = per[i];
  }
  out.scan_bytes += uint64_t(W) * 4 + kept * 32;  // + workgroup counts, + id/start/end of each record
  // (the caller counted 4 B of duration + 8 B of start / end per entry; these kernels read
  // the 4 B ds column (duration | span) + the 4 B start column when both filters are on)
  if (has_dur && q.has_range)
    for (const auto &sg : segs) out.scan_bytes -= 4ull * (sg.n - sg.e0);
  tr.mark("post");
  return true;
}

}  // namespace tsg
