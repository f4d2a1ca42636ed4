// engine.hip — MI355X (gfx950) search pipeline for Tempo backend search blocks.
//
// Per query, on each device, for the blocks resident there:
//   K1  dict_match      substring test of every term's needle against the block's
//                       value dictionary of that key -> value-set bitmap
//                       (bytes.Contains semantics of ContainsTag, searchdata_util.go:47-61)
//   K1b dict_sets       value matches -> value-set bitmap for multi-valued keys
//   K2  scan_compact    one pass over the resident columns: trace filters
//                       (pipeline.go:29-66) AND tag terms via bitmap lookups, then
//                       order-preserving compaction with a single-pass decoupled
//                       look-back (epoch-tagged 8-byte granules, agent scope)
//   K3  compact_regions limit mode only: per-block regions -> one contiguous list
// All kernels are HBM/L2-bound integer work; no MFMA (no dense contraction exists).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "devctx.hpp"

namespace tsg {

// ------------------------------------------------------------------------------------
// device-side descriptors (POD, copied H2D once per query)
struct DictJob {
  const uint8_t *bytes;
  const uint32_t *off;
  const uint32_t *set_off;
  const uint32_t *set_vals;
  uint32_t nvals, nsets;
  uint32_t needle_off, needle_len;
  uint32_t vmatch_base;  // u8 per value (non-identity jobs)
  uint32_t bm_base;      // u32 words
  uint32_t identity, pad;
};
struct ScanTerm {
  const void *col;
  const uint32_t *bm;  // global bitmap
  uint32_t width, nsets;
  uint32_t lds_off;    // word offset in LDS, or kNone -> read global
  uint32_t bm_words;
};
struct ScanSeg {
  uint64_t n;
  uint32_t first_tile, ntiles;
  const uint32_t *dur32;
  const uint64_t *dur64;
  const uint32_t *start_s, *end_s;
  const uint8_t *ids;
  const uint64_t *start_ns, *end_ns;
  uint64_t out_base, cap;
  uint32_t term0, nterms;
  uint32_t block_idx, lds_words;
};
struct MatchRec {  // == SearchOut::Rec
  uint8_t id[16];
  uint64_t start, end;
  uint64_t entry;
  uint32_t block, pad;
};
static_assert(sizeof(MatchRec) == 48, "record layout");
static_assert(sizeof(MatchRec) == sizeof(SearchOut::Rec), "record layout");

struct ScanParams {
  const ScanSeg *segs;
  const ScanTerm *terms;
  uint32_t nsegs, ntiles;
  uint32_t has_dur, need64, has_min, has_max;
  uint64_t min_ns, max_ns;
  uint32_t has_range, start_s, end_s, per_seg_chain;
  unsigned long long epoch;  // < 2^24
  unsigned long long ticket_base;
  unsigned long long *ticket;
  unsigned long long *gran;  // per global tile
  MatchRec *out;             // global-chain output
  uint64_t out_cap;
  MatchRec *regions;         // per-segment-chain output
  uint64_t *seg_counts;      // per segment total (written by its last tile)
  uint64_t *total;           // global-chain total (written by the last tile)
  uint32_t *err;             // look-back timeout flag
};

constexpr int kThreads = 256;
constexpr int kSteps = 4;                              // entries per thread = 4 x kSteps
constexpr int kTile = kThreads * 4 * kSteps;           // 4096 entries per tile
constexpr unsigned long long kStAgg = 1, kStInc = 2;
constexpr int kValBits = 38;
constexpr unsigned long long kValMask = (1ULL << kValBits) - 1;

__device__ __forceinline__ unsigned long long gran_make(unsigned long long epoch, unsigned long long st,
                                                        unsigned long long v) {
  return (epoch << 40) | (st << kValBits) | (v & kValMask);
}

// ------------------------------------------------------------------------------------
// K1: dictionary substring match
__device__ __forceinline__ bool dev_contains(const uint8_t *h, uint32_t hl, const uint8_t *nd, uint32_t nl) {
  if (nl == 0) return true;  // bytes.Contains(x, "") == true (pitfall P7)
  if (nl > hl) return false;
  const uint8_t f = nd[0];
  for (uint32_t i = 0; i + nl <= hl; i++) {
    if (h[i] != f) continue;
    uint32_t k = 1;
    while (k < nl && h[i + k] == nd[k]) k++;
    if (k == nl) return true;
  }
  return false;
}

__device__ __forceinline__ uint32_t find_job(const uint32_t *prefix, uint32_t njobs, uint64_t item) {
  uint32_t lo = 0, hi = njobs;  // largest j with prefix[j] <= item
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (prefix[mid] <= item) lo = mid;
    else hi = mid;
  }
  return lo;
}

// items: identity jobs -> one item per 32 values (writes a bitmap word directly);
//        other jobs    -> one item per value (writes vmatch)
extern "C" __global__ void __launch_bounds__(256) dict_match_kernel(const DictJob *jobs, const uint32_t *prefix, uint32_t njobs,
                                                         uint32_t total, const uint8_t *needles, uint8_t *vmatch,
                                                         uint32_t *bitmaps) {
  uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= total) return;
  uint32_t j = find_job(prefix, njobs, item);
  const DictJob jb = jobs[j];
  uint32_t local = item - prefix[j];
  const uint8_t *nd = needles + jb.needle_off;
  if (jb.identity) {
    uint32_t word = 0;
    uint32_t v0 = local * 32;
    for (uint32_t b = 0; b < 32 && v0 + b < jb.nvals; b++) {
      uint32_t v = v0 + b;
      uint32_t o0 = jb.off[v], o1 = jb.off[v + 1];
      if (dev_contains(jb.bytes + o0, o1 - o0, nd, jb.needle_len)) word |= 1u << b;
    }
    bitmaps[jb.bm_base + local] = word;
  } else {
    uint32_t v = local;
    uint32_t o0 = jb.off[v], o1 = jb.off[v + 1];
    vmatch[jb.vmatch_base + v] = dev_contains(jb.bytes + o0, o1 - o0, nd, jb.needle_len) ? 1 : 0;
  }
}

// K1b: per bitmap word of a non-identity job: set matches iff any of its values matches
extern "C" __global__ void __launch_bounds__(256) dict_sets_kernel(const DictJob *jobs, const uint32_t *set_jobs,
                                                        const uint32_t *prefix, uint32_t nsj, uint32_t total,
                                                        const uint8_t *vmatch, uint32_t *bitmaps) {
  uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= total) return;
  uint32_t q = find_job(prefix, nsj, item);
  const DictJob jb = jobs[set_jobs[q]];
  uint32_t w = item - prefix[q];
  uint32_t word = 0;
  for (uint32_t b = 0; b < 32; b++) {
    uint32_t s = w * 32 + b;
    if (s >= jb.nsets) break;
    for (uint32_t i = jb.set_off[s]; i < jb.set_off[s + 1]; i++)
      if (vmatch[jb.vmatch_base + jb.set_vals[i]]) {
        word |= 1u << b;
        break;
      }
  }
  bitmaps[jb.bm_base + w] = word;
}

// ------------------------------------------------------------------------------------
// K2: scan + order-preserving compaction
__device__ __forceinline__ void load4_col(const void *col, uint32_t width, uint64_t e, bool full, uint64_t n,
                                          uint32_t v[4]) {
  if (full) {
    if (width == 1) {
      uint32_t x = *reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(col) + e);
      v[0] = x & 0xff; v[1] = (x >> 8) & 0xff; v[2] = (x >> 16) & 0xff; v[3] = x >> 24;
    } else if (width == 2) {
      uint2 x = *reinterpret_cast<const uint2 *>(static_cast<const uint16_t *>(col) + e);
      v[0] = x.x & 0xffff; v[1] = x.x >> 16; v[2] = x.y & 0xffff; v[3] = x.y >> 16;
    } else {
      uint4 x = *reinterpret_cast<const uint4 *>(static_cast<const uint32_t *>(col) + e);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
  } else {
    for (int j = 0; j < 4; j++) {
      uint64_t i = e + j;
      if (i >= n) { v[j] = 0xffffffffu; continue; }
      if (width == 1) v[j] = static_cast<const uint8_t *>(col)[i];
      else if (width == 2) v[j] = static_cast<const uint16_t *>(col)[i];
      else v[j] = static_cast<const uint32_t *>(col)[i];
    }
  }
}

__device__ __forceinline__ uint4 load4_u32(const uint32_t *p, uint64_t e, bool full, uint64_t n) {
  if (full) return *reinterpret_cast<const uint4 *>(p + e);
  uint4 r;
  r.x = e < n ? p[e] : 0;
  r.y = e + 1 < n ? p[e + 1] : 0;
  r.z = e + 2 < n ? p[e + 2] : 0;
  r.w = e + 3 < n ? p[e + 3] : 0;
  return r;
}

__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    unsigned long long o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

extern "C" __global__ void __launch_bounds__(kThreads) scan_compact_kernel(ScanParams P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_bm[];
  __shared__ uint32_t s_tile, s_seg;
  __shared__ unsigned long long s_wsum[kThreads / 64];
  __shared__ unsigned long long s_excl;
  __shared__ uint32_t s_wcnt[kThreads / 64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    unsigned long long t = atomicAdd(P.ticket, 1ULL) - P.ticket_base;  // dynamic tile id: scan order
    uint32_t lo = 0, hi = P.nsegs;
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (P.segs[mid].first_tile <= t) lo = mid;
      else hi = mid;
    }
    s_tile = uint32_t(t);
    s_seg = lo;
  }
  __syncthreads();
  const uint32_t t = __builtin_amdgcn_readfirstlane(s_tile);
  const ScanSeg S = P.segs[__builtin_amdgcn_readfirstlane(s_seg)];
  const uint32_t seg_i = __builtin_amdgcn_readfirstlane(s_seg);
  const uint64_t n = S.n;
  const uint32_t local_tile = t - S.first_tile;
  const uint64_t tile0 = uint64_t(local_tile) * kTile;

  // stage small bitmaps in LDS
  for (uint32_t q = 0; q < S.nterms; q++) {
    const ScanTerm &T = P.terms[S.term0 + q];
    if (T.lds_off != 0xffffffffu)
      for (uint32_t w = tid; w < T.bm_words; w += kThreads) lds_bm[T.lds_off + w] = T.bm[w];
  }
  __syncthreads();

  // ---- predicate: 16 entries per thread, bit (4k + j) <-> entry tile0 + k*1024 + 4*tid + j
  uint32_t mask = 0xffffu;
  uint64_t ebase[kSteps];
  bool full[kSteps];
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    ebase[k] = tile0 + uint64_t(k) * (kThreads * 4) + uint64_t(tid) * 4;
    full[k] = ebase[k] + 4 <= n;
    for (int j = 0; j < 4; j++)
      if (ebase[k] + j >= n) mask &= ~(1u << (4 * k + j));
  }
  if (P.has_dur) {
    uint4 d[kSteps];
#pragma unroll
    for (int k = 0; k < kSteps; k++) d[k] = load4_u32(S.dur32, ebase[k], full[k], n);
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      uint32_t dv[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint64_t dd = dv[j];
        if (P.need64 && dv[j] == 0xffffffffu && ebase[k] + j < n) dd = S.dur64[ebase[k] + j];
        bool ok = (!P.has_min || dd >= P.min_ns) && (!P.has_max || dd <= P.max_ns);
        if (!ok) mask &= ~(1u << (4 * k + j));
      }
    }
  }
  if (P.has_range) {
    uint4 s[kSteps], e[kSteps];
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      s[k] = load4_u32(S.start_s, ebase[k], full[k], n);
      e[k] = load4_u32(S.end_s, ebase[k], full[k], n);
    }
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      uint32_t sv[4] = {s[k].x, s[k].y, s[k].z, s[k].w}, ev[4] = {e[k].x, e[k].y, e[k].z, e[k].w};
#pragma unroll
      for (int j = 0; j < 4; j++)  // req.Start <= endSec && req.End >= startSec (pipeline.go:59-66)
        if (!(P.start_s <= ev[j] && P.end_s >= sv[j])) mask &= ~(1u << (4 * k + j));
    }
  }
  for (uint32_t q = 0; q < S.nterms; q++) {
    const ScanTerm T = P.terms[S.term0 + q];
    uint32_t v[kSteps][4];
#pragma unroll
    for (int k = 0; k < kSteps; k++) load4_col(T.col, T.width, ebase[k], full[k], n, v[k]);
#pragma unroll
    for (int k = 0; k < kSteps; k++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t x = v[k][j];
        bool ok = x < T.nsets;  // all-ones = key absent
        if (ok) {
          uint32_t w = T.lds_off != 0xffffffffu ? lds_bm[T.lds_off + (x >> 5)] : T.bm[x >> 5];
          ok = (w >> (x & 31)) & 1u;
        }
        if (!ok) mask &= ~(1u << (4 * k + j));
      }
  }

  // ---- tile count
  uint32_t c = __popc(mask);
  uint32_t wc = c;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) wc += __shfl_xor(wc, d, 64);
  if (lane == 0) s_wcnt[wid] = wc;
  __syncthreads();
  uint32_t tile_count = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; w++) tile_count += s_wcnt[w];

  // ---- decoupled look-back (wave 0). Chain = this segment's tiles (limit mode) or all tiles.
  if (wid == 0) {
    const uint32_t chain0 = P.per_seg_chain ? S.first_tile : 0;
    unsigned long long excl = 0;
    if (t == chain0) {
      if (lane == 0)
        __hip_atomic_store(&P.gran[t], gran_make(P.epoch, kStInc, tile_count), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(&P.gran[t], gran_make(P.epoch, kStAgg, tile_count), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      int64_t end = int64_t(t);  // window (end-64, end]
      uint32_t spins = 0;
      for (;;) {
        int64_t j = end - 1 - lane;
        unsigned long long g;
        bool ready;
        if (j < int64_t(chain0)) {
          g = gran_make(P.epoch, kStInc, 0);  // chain boundary acts as an inclusive 0
          ready = true;
        } else {
          g = __hip_atomic_load(&P.gran[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ready = (g >> 40) == P.epoch;
        }
        // wait until every lane's predecessor has published (aggregate or inclusive)
        while (!__all(ready)) {
          if (++spins > (1u << 22)) {
            if (lane == 0) atomicOr(P.err, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if (!ready) {
            g = __hip_atomic_load(&P.gran[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ready = (g >> 40) == P.epoch;
          }
        }
        if (spins > (1u << 22)) break;
        unsigned long long st = (g >> kValBits) & 3ULL;
        unsigned long long incl_mask = __ballot(st == kStInc);
        int first = incl_mask ? __builtin_ctzll(incl_mask) : 64;  // nearest inclusive predecessor
        unsigned long long v = (lane <= first) ? (g & kValMask) : 0ULL;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
        excl += v;
        if (incl_mask) break;
        end -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(&P.gran[t], gran_make(P.epoch, kStInc, excl + tile_count), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_excl = excl;
      if (P.per_seg_chain && local_tile + 1 == S.ntiles) P.seg_counts[seg_i] = excl + tile_count;
      if (!P.per_seg_chain && t + 1 == P.ntiles) *P.total = excl + tile_count;
    }
  }
  __syncthreads();
  if (tile_count == 0) return;
  const unsigned long long excl = s_excl;

  // ---- intra-tile ranks in scan order (k, tid, j): scan 4 packed 16-bit per-step counts
  unsigned long long pc = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) pc |= (unsigned long long)__popc((mask >> (4 * k)) & 0xfu) << (16 * k);
  unsigned long long inc = wave_incl_scan_u64(pc, lane);
  if (lane == 63) s_wsum[wid] = inc;
  __syncthreads();
  unsigned long long before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; w++) {
    if (w < wid) before += s_wsum[w];
    tot += s_wsum[w];
  }
  unsigned long long mine = before + inc - pc;  // exclusive, per step field
  uint32_t step_base = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    uint32_t nib = (mask >> (4 * k)) & 0xfu;
    uint32_t r0 = step_base + uint32_t((mine >> (16 * k)) & 0xffff);
    step_base += uint32_t((tot >> (16 * k)) & 0xffff);
    uint32_t seen = 0;
    for (int j = 0; j < 4; j++) {
      if (!(nib & (1u << j))) continue;
      uint64_t rank = excl + r0 + seen++;
      MatchRec *dst;
      if (P.per_seg_chain) {
        if (rank >= S.cap) continue;
        dst = P.regions + S.out_base + rank;
      } else {
        if (rank >= P.out_cap) continue;
        dst = P.out + rank;
      }
      uint64_t ei = ebase[k] + j;
      const uint4 id = *reinterpret_cast<const uint4 *>(S.ids + ei * 16);
      uint4 *d4 = reinterpret_cast<uint4 *>(dst);
      d4[0] = id;
      uint64_t *d8 = reinterpret_cast<uint64_t *>(dst);
      d8[2] = S.start_ns[ei];
      d8[3] = S.end_ns[ei];
      d8[4] = ei;
      d8[5] = (unsigned long long)S.block_idx;
    }
  }
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// K3 (limit mode): per-segment regions -> contiguous output after the header
extern "C" __global__ void __launch_bounds__(256) compact_regions_kernel(const ScanSeg *segs, uint32_t nsegs,
                                                              const uint64_t *seg_counts, const MatchRec *regions,
                                                              MatchRec *out, uint64_t *total) {
  const uint32_t s = blockIdx.x;
  __shared__ unsigned long long s_base;
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (uint32_t i = 0; i < s; i++) b += umin64(seg_counts[i], segs[i].cap);
    s_base = b;
    if (s + 1 == nsegs) *total = b + umin64(seg_counts[s], segs[s].cap);
  }
  __syncthreads();
  uint64_t cnt = umin64(seg_counts[s], segs[s].cap);
  for (uint64_t i = threadIdx.x; i < cnt; i += blockDim.x) out[s_base + i] = regions[segs[s].out_base + i];
}

// ------------------------------------------------------------------------------------
// host side
int device_ordinal(const DeviceCtx &dc) { return dc.ordinal; }

void ctx_init(Ctx &c, const tsg_options *opts) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) fail(TSG_E_DEVICE, "no HIP device visible (libtsg has no CPU path)");
  std::vector<int> ords;
  if (opts && opts->devices && opts->num_devices > 0) {
    for (int i = 0; i < opts->num_devices; i++) ords.push_back(opts->devices[i]);
  } else {
    int m = (opts && opts->num_devices > 0) ? std::min(opts->num_devices, n) : n;
    for (int i = 0; i < m; i++) ords.push_back(i);
  }
  for (int o : ords) {
    if (o < 0 || o >= n) fail(TSG_E_INVALID, "device ordinal out of range");
    auto dc = std::make_unique<DeviceCtx>();
    dc->ordinal = o;
    HIP_OK(hipSetDevice(o));
    HIP_OK(hipStreamCreateWithFlags(&dc->stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreate(&dc->ev0));
    HIP_OK(hipEventCreate(&dc->ev1));
    HIP_OK(hipEventCreate(&dc->es0));
    HIP_OK(hipEventCreate(&dc->es1));
    dc->ticket.ensure(64);
    HIP_OK(hipMemset(dc->ticket.p, 0, 64));
    dc->err.ensure(64);
    HIP_OK(hipMemset(dc->err.p, 0, 64));
    c.devs.push_back(dc.release());
  }
}

void ctx_shutdown(Ctx &c) {
  for (auto &dc : c.devs) {
    (void)hipSetDevice(dc->ordinal);
    (void)hipStreamSynchronize(dc->stream);
    for (DevBuf *b : {&dc->desc, &dc->vmatch, &dc->bitmaps, &dc->gran, &dc->ticket, &dc->out, &dc->regions,
                      &dc->seg_counts, &dc->hdr, &dc->err})
      b->release();
    dc->hdesc.release();
    dc->hout.release();
    (void)hipEventDestroy(dc->ev0);
    (void)hipEventDestroy(dc->ev1);
    (void)hipEventDestroy(dc->es0);
    (void)hipEventDestroy(dc->es1);
    (void)hipStreamDestroy(dc->stream);
    delete dc;
  }
  c.devs.clear();
}

template <typename T>
static T *dev_upload(DevBlock &b, const T *src, size_t count, hipStream_t s) {
  void *p = nullptr;
  size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  HIP_OK(hipMalloc(&p, bytes));
  b.allocs.push_back(p);
  b.bytes += bytes;
  if (count) HIP_OK(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s));
  return static_cast<T *>(p);
}

void block_upload(Ctx &c, Block &b, int device_hint) {
  if (c.devs.empty()) fail(TSG_E_DEVICE, "no device");
  DeviceCtx &dc = *c.devs[size_t(std::max(device_hint, 0)) % c.devs.size()];
  b.dc = &dc;
  DevBlock &d = b.dev;
  const HostBlock &h = b.host;
  d.device = dc.ordinal;
  d.n = h.n;
  std::lock_guard<std::mutex> lk(dc.mu);
  HIP_OK(hipSetDevice(dc.ordinal));
  hipStream_t s = dc.stream;
  size_t n = h.n;
  std::vector<uint32_t> dur32(n), ss(n), es(n);
  std::vector<uint64_t> dur64(n);
  for (size_t i = 0; i < n; i++) {
    uint64_t dd = h.end[i] - h.start[i];  // uint64 wrap (pitfall P2)
    dur64[i] = dd;
    dur32[i] = dd >= 0xffffffffULL ? 0xffffffffu : uint32_t(dd);
    ss[i] = uint32_t(h.start[i] / 1000000000ULL);
    es[i] = uint32_t(h.end[i] / 1000000000ULL);
  }
  d.dur32 = dev_upload(d, dur32.data(), n, s);
  d.dur64 = dev_upload(d, dur64.data(), n, s);
  d.start_s = dev_upload(d, ss.data(), n, s);
  d.end_s = dev_upload(d, es.data(), n, s);
  d.ids = dev_upload(d, h.ids.data(), n * 16, s);
  d.start_ns = dev_upload(d, h.start.data(), n, s);
  d.end_ns = dev_upload(d, h.end.data(), n, s);
  // the staging vectors must outlive the async copies
  HIP_OK(hipStreamSynchronize(s));
  for (const KeyColumn &kc : h.keys) {
    DevKey k;
    k.name = kc.name;
    k.width = kc.width();
    k.nvals = kc.nvals();
    k.nsets = kc.nsets();
    k.identity = kc.identity;
    if (k.width == 1) {
      std::vector<uint8_t> col(n);
      for (size_t i = 0; i < n; i++) col[i] = kc.col[i] == kNone ? 0xff : uint8_t(kc.col[i]);
      k.col = dev_upload(d, col.data(), n, s);
      HIP_OK(hipStreamSynchronize(s));
    } else if (k.width == 2) {
      std::vector<uint16_t> col(n);
      for (size_t i = 0; i < n; i++) col[i] = kc.col[i] == kNone ? 0xffff : uint16_t(kc.col[i]);
      k.col = dev_upload(d, col.data(), n, s);
      HIP_OK(hipStreamSynchronize(s));
    } else {
      k.col = dev_upload(d, kc.col.data(), n, s);
    }
    k.dict_bytes = dev_upload(d, kc.dict_bytes.data(), kc.dict_bytes.size(), s);
    k.dict_off = dev_upload(d, kc.dict_off.data(), kc.dict_off.size(), s);
    k.dict_nbytes = kc.dict_bytes.size();
    if (!kc.identity) {
      k.set_off = dev_upload(d, kc.set_off.data(), kc.set_off.size(), s);
      k.set_vals = dev_upload(d, kc.set_vals.data(), kc.set_vals.size(), s);
    }
    d.keys.push_back(k);
  }
  HIP_OK(hipStreamSynchronize(s));
}

void block_free(Block &b) {
  if (!b.dc) return;
  std::lock_guard<std::mutex> lk(b.dc->mu);
  (void)hipSetDevice(b.dc->ordinal);
  (void)hipStreamSynchronize(b.dc->stream);
  for (void *p : b.dev.allocs) (void)hipFree(p);
  b.dev.allocs.clear();
  b.dc = nullptr;
}

static size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

void device_search(DeviceCtx &dc, const std::vector<std::pair<uint32_t, Block *>> &blocks, const tsg_query &q,
                   uint32_t limit, SearchOut &out) {
  std::lock_guard<std::mutex> lk(dc.mu);
  HIP_OK(hipSetDevice(dc.ordinal));
  hipStream_t s = dc.stream;

  // ---- plan: segments, terms, dictionary jobs
  std::vector<ScanSeg> segs;
  std::vector<ScanTerm> terms;
  std::vector<DictJob> jobs;
  std::vector<uint32_t> job_items(1, 0), set_jobs, set_items(1, 0);
  std::vector<uint8_t> needles;
  std::vector<uint32_t> needle_off(q.nterms);
  for (uint32_t t = 0; t < q.nterms; t++) {
    needle_off[t] = uint32_t(needles.size());
    needles.insert(needles.end(), q.values[t], q.values[t] + q.value_lens[t]);
  }
  uint32_t vmatch_total = 0, bm_total = 0, tiles = 0;
  uint64_t region_total = 0;
  uint64_t alg_bytes = 0, scan_bytes = 0;
  const bool has_dur = q.has_min || q.has_max;
  uint32_t max_lds_words = 0;
  constexpr uint32_t kLdsBudgetWords = 8192;  // 32 KiB per workgroup
  std::vector<uint32_t> term_bm_base;  // per ScanTerm: word base in the bitmap scratch
  for (auto &bp : blocks) {
    Block &b = *bp.second;
    const DevBlock &d = b.dev;
    if (d.n == 0) continue;
    // resolve every term's key first: a key absent from the block means FindTag fails
    // for every entry, so the block contributes no match (its metrics still count)
    std::vector<int> kidx(q.nterms);
    bool dead = false;
    for (uint32_t t = 0; t < q.nterms; t++) {
      std::string key(reinterpret_cast<const char *>(q.keys[t]), q.key_lens[t]);
      auto it = b.host.key_index.find(key);
      if (it == b.host.key_index.end()) {
        dead = true;
        break;
      }
      kidx[t] = it->second;
    }
    if (dead) continue;
    ScanSeg sg{};
    sg.n = d.n;
    sg.dur32 = d.dur32;
    sg.dur64 = d.dur64;
    sg.start_s = d.start_s;
    sg.end_s = d.end_s;
    sg.ids = d.ids;
    sg.start_ns = d.start_ns;
    sg.end_ns = d.end_ns;
    sg.block_idx = bp.first;
    sg.term0 = uint32_t(terms.size());
    uint32_t lds_words = 0;
    uint64_t per = (has_dur ? 4 : 0) + (q.has_range ? 8 : 0);
    for (uint32_t t = 0; t < q.nterms; t++) {
      const DevKey &k = d.keys[size_t(kidx[t])];
      DictJob jb{};
      jb.bytes = k.dict_bytes;
      jb.off = k.dict_off;
      jb.set_off = k.set_off;
      jb.set_vals = k.set_vals;
      jb.nvals = k.nvals;
      jb.nsets = k.nsets;
      jb.needle_off = needle_off[t];
      jb.needle_len = q.value_lens[t];
      jb.identity = k.identity ? 1 : 0;
      jb.bm_base = bm_total;
      uint32_t words = (k.nsets + 31) / 32;
      bm_total += words;
      if (k.identity) {
        job_items.push_back(job_items.back() + words);
      } else {
        jb.vmatch_base = vmatch_total;
        vmatch_total += k.nvals;
        job_items.push_back(job_items.back() + k.nvals);
        set_jobs.push_back(uint32_t(jobs.size()));
        set_items.push_back(set_items.back() + words);
      }
      jobs.push_back(jb);
      alg_bytes += k.dict_nbytes + 4ull * (k.nvals + 1) + 4ull * words;
      ScanTerm st{};
      st.col = k.col;
      st.width = uint32_t(k.width);
      st.nsets = k.nsets;
      st.bm_words = words;
      if (lds_words + words <= kLdsBudgetWords) {
        st.lds_off = lds_words;
        lds_words += words;
      } else {
        st.lds_off = 0xffffffffu;  // large dictionary: bitmap read from L2/MALL
      }
      terms.push_back(st);
      term_bm_base.push_back(jb.bm_base);
      per += uint64_t(k.width);
    }
    sg.nterms = q.nterms;
    sg.lds_words = lds_words;
    max_lds_words = std::max(max_lds_words, lds_words);
    sg.first_tile = tiles;
    sg.ntiles = uint32_t((d.n + kTile - 1) / kTile);
    tiles += sg.ntiles;
    if (limit) {
      sg.out_base = region_total;
      sg.cap = std::min<uint64_t>(limit, d.n);
      region_total += sg.cap;
    } else {
      sg.cap = d.n;
    }
    alg_bytes += d.n * per;
    scan_bytes += d.n * per;
    segs.push_back(sg);
  }
  out.recs.clear();
  out.block_counts.assign(blocks.size(), 0);
  out.device_bytes = alg_bytes;
  out.kernel_ns = 0;
  if (segs.empty() || q.exhaustive) return;

  // ---- scratch
  dc.bitmaps.ensure(std::max<size_t>(bm_total, 1) * 4);
  dc.vmatch.ensure(std::max<size_t>(vmatch_total, 1));
  if (dc.gran_tiles < tiles) {
    HIP_OK(hipStreamSynchronize(s));
    dc.gran.ensure(size_t(tiles) * 8 * 2);
    HIP_OK(hipMemsetAsync(dc.gran.p, 0, dc.gran.cap, s));
    dc.gran_tiles = dc.gran.cap / 8;
  }
  uint64_t n_total = 0;
  for (auto &sg : segs) n_total += sg.n;
  uint64_t out_cap = limit ? region_total : std::min<uint64_t>(n_total, 1u << 20);
  dc.out.ensure(std::max<size_t>(out_cap, 1) * sizeof(MatchRec));
  if (limit) dc.regions.ensure(std::max<size_t>(region_total, 1) * sizeof(MatchRec));
  dc.seg_counts.ensure(std::max<size_t>(segs.size(), 1) * 8);
  dc.hdr.ensure(64);
  for (size_t i = 0; i < terms.size(); i++) terms[i].bm = static_cast<const uint32_t *>(dc.bitmaps.p) + term_bm_base[i];

  // ---- descriptors -> one H2D copy
  size_t o_segs = 0, o_terms = align16(o_segs + segs.size() * sizeof(ScanSeg));
  size_t o_jobs = align16(o_terms + terms.size() * sizeof(ScanTerm));
  size_t o_jp = align16(o_jobs + jobs.size() * sizeof(DictJob));
  size_t o_sj = align16(o_jp + job_items.size() * 4);
  size_t o_sp = align16(o_sj + set_jobs.size() * 4);
  size_t o_nd = align16(o_sp + set_items.size() * 4);
  size_t total_desc = align16(o_nd + needles.size() + 1);
  dc.hdesc.ensure(total_desc);
  dc.desc.ensure(total_desc);
  auto *hd = static_cast<uint8_t *>(dc.hdesc.p);
  std::memcpy(hd + o_segs, segs.data(), segs.size() * sizeof(ScanSeg));
  std::memcpy(hd + o_terms, terms.data(), terms.size() * sizeof(ScanTerm));
  std::memcpy(hd + o_jobs, jobs.data(), jobs.size() * sizeof(DictJob));
  std::memcpy(hd + o_jp, job_items.data(), job_items.size() * 4);
  if (!set_jobs.empty()) std::memcpy(hd + o_sj, set_jobs.data(), set_jobs.size() * 4);
  std::memcpy(hd + o_sp, set_items.data(), set_items.size() * 4);
  if (!needles.empty()) std::memcpy(hd + o_nd, needles.data(), needles.size());
  auto *dd = static_cast<uint8_t *>(dc.desc.p);
  HIP_OK(hipMemcpyAsync(dd, hd, total_desc, hipMemcpyHostToDevice, s));

  HIP_OK(hipEventRecord(dc.ev0, s));
  uint32_t njob_items = job_items.back();
  if (njob_items) {
    dict_match_kernel<<<(njob_items + 255) / 256, 256, 0, s>>>(
        reinterpret_cast<const DictJob *>(dd + o_jobs), reinterpret_cast<const uint32_t *>(dd + o_jp),
        uint32_t(jobs.size()), njob_items, dd + o_nd, static_cast<uint8_t *>(dc.vmatch.p),
        static_cast<uint32_t *>(dc.bitmaps.p));
    HIP_OK(hipGetLastError());
  }
  if (set_items.back()) {
    dict_sets_kernel<<<(set_items.back() + 255) / 256, 256, 0, s>>>(
        reinterpret_cast<const DictJob *>(dd + o_jobs), reinterpret_cast<const uint32_t *>(dd + o_sj),
        reinterpret_cast<const uint32_t *>(dd + o_sp), uint32_t(set_jobs.size()), set_items.back(),
        static_cast<const uint8_t *>(dc.vmatch.p), static_cast<uint32_t *>(dc.bitmaps.p));
    HIP_OK(hipGetLastError());
  }
  dc.epoch = (dc.epoch + 1) & 0xffffffULL;
  if (dc.epoch == 0) dc.epoch = 1;
  ScanParams P{};
  P.segs = reinterpret_cast<const ScanSeg *>(dd + o_segs);
  P.terms = reinterpret_cast<const ScanTerm *>(dd + o_terms);
  P.nsegs = uint32_t(segs.size());
  P.ntiles = tiles;
  P.has_dur = has_dur;
  P.has_min = q.has_min;
  P.has_max = q.has_max;
  P.min_ns = q.min_ns;
  P.max_ns = q.max_ns;
  P.need64 = (q.has_min && q.min_ns >= 0xffffffffULL) || (q.has_max && q.max_ns >= 0xffffffffULL);
  P.has_range = q.has_range;
  P.start_s = q.start_s;
  P.end_s = q.end_s;
  P.per_seg_chain = limit ? 1 : 0;
  P.epoch = dc.epoch;
  P.ticket_base = dc.ticket_base;
  P.ticket = static_cast<unsigned long long *>(dc.ticket.p);
  P.gran = static_cast<unsigned long long *>(dc.gran.p);
  P.out = static_cast<MatchRec *>(dc.out.p);
  P.out_cap = out_cap;
  P.regions = static_cast<MatchRec *>(dc.regions.p);
  P.seg_counts = static_cast<uint64_t *>(dc.seg_counts.p);
  P.total = static_cast<uint64_t *>(dc.hdr.p);
  P.err = static_cast<uint32_t *>(dc.err.p);
  HIP_OK(hipEventRecord(dc.es0, s));
  scan_compact_kernel<<<tiles, kThreads, max_lds_words * 4, s>>>(P);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(dc.es1, s));
  dc.ticket_base += tiles;
  if (limit) {
    compact_regions_kernel<<<uint32_t(segs.size()), 256, 0, s>>>(
        reinterpret_cast<const ScanSeg *>(dd + o_segs), uint32_t(segs.size()),
        static_cast<const uint64_t *>(dc.seg_counts.p), static_cast<const MatchRec *>(dc.regions.p),
        static_cast<MatchRec *>(dc.out.p), static_cast<uint64_t *>(dc.hdr.p));
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipEventRecord(dc.ev1, s));

  // ---- results: header + a first slice in one round trip
  const size_t first = std::min<uint64_t>(out_cap, 4096);
  size_t hbytes = 64 + segs.size() * 8 + first * sizeof(MatchRec) + 64;
  dc.hout.ensure(hbytes);
  auto *ho = static_cast<uint8_t *>(dc.hout.p);
  HIP_OK(hipMemcpyAsync(ho, dc.hdr.p, 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(ho + 8, dc.err.p, 4, hipMemcpyDeviceToHost, s));
  if (limit) HIP_OK(hipMemcpyAsync(ho + 64, dc.seg_counts.p, segs.size() * 8, hipMemcpyDeviceToHost, s));
  uint8_t *hrec = ho + 64 + segs.size() * 8;
  hrec = reinterpret_cast<uint8_t *>((uintptr_t(hrec) + 15) & ~uintptr_t(15));
  if (first) HIP_OK(hipMemcpyAsync(hrec, dc.out.p, first * sizeof(MatchRec), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  uint64_t total;
  std::memcpy(&total, ho, 8);
  uint32_t errf;
  std::memcpy(&errf, ho + 8, 4);
  if (errf) {
    HIP_OK(hipMemset(dc.err.p, 0, 4));
    fail(TSG_E_DEVICE, "scan look-back timed out");
  }
  float ms = 0, sms = 0;
  HIP_OK(hipEventElapsedTime(&ms, dc.ev0, dc.ev1));
  HIP_OK(hipEventElapsedTime(&sms, dc.es0, dc.es1));
  out.kernel_ns = uint64_t(double(ms) * 1e6);
  out.scan_ns = uint64_t(double(sms) * 1e6);
  out.scan_bytes = scan_bytes + std::min<uint64_t>(total, out_cap) * (sizeof(MatchRec) + 32);
  if (!limit && total > out_cap) {
    // output capacity exceeded: grow and rerun once with room for every match
    dc.out.ensure(total * sizeof(MatchRec));
    HIP_OK(hipStreamSynchronize(s));
    dc.epoch = (dc.epoch + 1) & 0xffffffULL;
    if (dc.epoch == 0) dc.epoch = 1;
    P.epoch = dc.epoch;
    P.ticket_base = dc.ticket_base;
    P.out = static_cast<MatchRec *>(dc.out.p);
    P.out_cap = total;
    out_cap = total;
    HIP_OK(hipEventRecord(dc.ev0, s));
    scan_compact_kernel<<<tiles, kThreads, max_lds_words * 4, s>>>(P);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(dc.ev1, s));
    dc.ticket_base += tiles;
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipEventElapsedTime(&ms, dc.ev0, dc.ev1));
    out.kernel_ns += uint64_t(double(ms) * 1e6);
  }
  out.recs.resize(total);
  if (total <= first) {
    if (total) std::memcpy(out.recs.data(), hrec, total * sizeof(MatchRec));
  } else {
    HIP_OK(hipMemcpy(out.recs.data(), dc.out.p, total * sizeof(MatchRec), hipMemcpyDeviceToHost));
  }
  if (limit) {
    for (size_t i = 0; i < segs.size(); i++) {
      uint64_t c;
      std::memcpy(&c, ho + 64 + i * 8, 8);
      c = std::min<uint64_t>(c, segs[i].cap);
      // map seg -> caller block position
      for (size_t bi = 0; bi < blocks.size(); bi++)
        if (blocks[bi].first == segs[i].block_idx) out.block_counts[bi] = c;
    }
  }
}

}  // namespace tsg
