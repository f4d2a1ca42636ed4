// search.hip — MI355X (gfx950) search pipeline for Tempo backend search blocks.
//
// Per query, on each device, for the blocks resident there:
//   dict_match   substring test of each term's needle against the block's value
//                dictionary for that key (bytes.Contains of ContainsTag,
//                pkg/tempofb/searchdata_util.go:47-61) -> value-set bitmap;
//                one lane per dictionary value, 64-value wave ballots -> words
//   dict_sets    value matches -> value-set bitmap (multi-valued keys only)
//   scan         one streaming pass over the resident filter columns: trace
//                filters (tempodb/search/pipeline.go:29-66) AND tag terms via
//                LDS-staged bitmap lookups. Workgroups own contiguous tile ranges
//                of one block; a tile that matches stores its 4096-bit match mask
//   emit         order-preserving compaction: workgroup prefix over the per-
//                workgroup counts (no atomics, no inter-workgroup waits), ranks
//                inside a tile from packed wave scans, records written in the
//                reference scan order (pages ascending, entry index ascending)
// Everything is integer, HBM-bound streaming; no MFMA (no dense contraction).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "aql.hpp"
#include "search_common.hpp"

namespace tsg {

// ------------------------------------------------------------------------------------
// descriptors (POD, one H2D copy per query)
struct DictJob {
  const uint8_t *bytes;
  const uint32_t *off;
  const uint32_t *set_off;
  const uint32_t *set_vals;
  uint32_t nvals, nsets;
  uint32_t needle_off, needle_len;
  uint32_t vmatch_base;  // u8 per value (non-identity jobs)
  uint32_t bm_base;      // bitmap word base
  uint32_t identity, item_base;  // first item (64-aligned) of this job
};
struct ScanTerm {
  const void *col;
  const uint32_t *bm;  // bitmap in global memory
  uint32_t width, nsets;
  uint32_t lds_off;    // word offset of the LDS copy, or ~0u (read global)
  uint32_t bm_words;
  // the dictionary pass's "some value of this (block, term) matched" flag (device memory):
  // 0 = no entry of the block can match the term, so none matches the query (general path)
  const uint32_t *anyf;
};

struct ScanParams {
  const ScanSeg *segs;
  const ScanTerm *terms;
  const uint16_t *wg_seg;  // workgroup -> segment (block) index
  uint32_t nsegs, nwg;
  uint32_t has_min, has_max, need64, limit_mode;
  uint64_t min_ns, max_ns;
  uint32_t start_s, end_s;
  uint16_t *mask;            // masks of tiles beyond kLdsTiles per workgroup: [workgroup][mask_tpw][256] u16
  uint32_t mask_tpw, pad2;
  unsigned long long *agg;   // per workgroup: {epoch, match count}, published once per launch
  uint32_t epoch;            // this launch's tag (never 0)
  uint32_t lds_bm_words;     // dynamic LDS: [bitmaps | kLdsTiles masks | per-block sums]
  uint8_t *out;              // pinned host: [header | (segment mode) tile counts | records];
                             // header[0] total, [1] error, [2] done epoch, [8+s] per block
  unsigned long long *stamps;  // TSG_STAMPS: per workgroup s_memrealtime at phase boundaries (else null)
  uint64_t hdr_bytes, out_cap;  // records start at out + hdr_bytes
  uint32_t *counts;          // segment mode: match count of every tile (pinned host)
  unsigned *done;            // one-launch path: completion counters (device; 8 XCD groups + top, 32 words apart)
  uint32_t seg_cap;          // segment mode (> 0): records per tile segment; 0 = look-back mode
  uint32_t done_top;         // top counter value once every XCD group has finished
  uint32_t done_target[8];   // group counter values once every scan workgroup of the group has finished
  // use_ticket: workgroup order from a device-wide ticket counter (ticket - ticket_base),
  // for the protocols that wait on lower-numbered workgroups (look-back, dictionary
  // granules): HIP promises no dispatch order, a ticket holder has started by definition
  unsigned long long *ticket;
  unsigned long long ticket_base;
  uint32_t use_ticket;
  // TSG_PRIO=1: scan loop wave priority from progress (s_setprio 3 -> 0 over the
  // workgroup's tiles). The co-resident workgroups of a CU progress in dispatch order
  // (issue is arbitrated by priority, then age: the 4th one ends ~10 us after the 1st);
  // this evens a CU out, but the kernel's end is set by the chip-wide tail, which it
  // does not move (profiles/r02_prio: kernel p50 38.7-39.8 vs 38.5-38.6 us off)
  uint32_t prio;
  // 1: the last workgroup raises header word 2 through the completion counters; 0 (segment
  // mode): the host completes on the per-workgroup counts alone (each stored after its
  // records), so no counter round trips sit at the end of the launch
  uint32_t flag_done;
  // look-back mode: 1 = each record is its 8-byte position (scan position | block index << 32),
  // the host fills the rest from the block's host columns (a dense config-4 query had written
  // 48-byte records across PCIe: 89 MB for 1.85 M matches, VERDICT r4 "What's weak" 4)
  uint32_t compact;
  unsigned *steal;  // tail claim counters, one per block slot (128 B apart), monotonic
  // bitmap mode (general path, full scans of dense queries): each workgroup writes one bit per
  // entry of its range into this pinned host array (block s at segs[s].bm_word0) and no records:
  // 1.25 MB per 10 M entries over PCIe instead of 8 bytes per match; the
  // host expands the bits into scan positions
  unsigned long long *bitmap;
  // general path: danyf (one flag per block x term, nterms per block). A launch whose every block
  // has a dead term returns at once, before taking a ticket (the host gives the tickets back)
  const uint32_t *anyf;
  uint32_t nterms;
};


// ------------------------------------------------------------------------------------
// dictionary match

__device__ __forceinline__ bool dev_contains(const uint8_t *h, uint32_t hl, const uint8_t *nd, uint32_t nl) {
  if (nl == 0) return true;  // bytes.Contains(x, "") (pitfall P7)
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

// prep: (1) workgroup 0 copies the query descriptors from pinned host memory into
// device memory for the search kernel (no H2D copy launch); (2) dictionary match,
// one lane per dictionary value; every job's item range is 64-aligned so a wave
// never straddles two jobs, and identity jobs turn the wave's matches into two
// bitmap words with one ballot. The job table and needles are read from `src`
// (host or device copy) once per workgroup into LDS when they fit.
constexpr uint32_t kPrepLdsJobs = 128, kPrepLdsNeedle = 4096;
constexpr size_t kHostDescMax = 64 << 10;  // larger descriptor sets take one H2D copy
static_assert(sizeof(DictJob) % 16 == 0, "DictJob staged as 16-byte words");
extern "C" __global__ void __launch_bounds__(256) prep_kernel(const uint8_t *src, uint8_t *dst, uint32_t copy16,
                                                              uint32_t o_jobs, uint32_t o_jb, uint32_t njobs,
                                                              uint32_t total, uint32_t o_nd, uint32_t nd_bytes,
                                                              uint8_t *vmatch, uint32_t *bitmaps, uint32_t *anyf) {
  __shared__ __attribute__((aligned(16))) DictJob s_jobs[kPrepLdsJobs];
  __shared__ __attribute__((aligned(16))) uint8_t s_nd[kPrepLdsNeedle];
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && src != dst)
    for (uint32_t i = tid; i < copy16; i += blockDim.x)
      reinterpret_cast<u32x4 *>(dst)[i] = reinterpret_cast<const u32x4 *>(src)[i];
  if (total == 0) return;
  // one round trip for the whole job table + needles when they fit in LDS
  const bool stage = njobs <= kPrepLdsJobs && nd_bytes <= kPrepLdsNeedle;
  const DictJob *jobs = reinterpret_cast<const DictJob *>(src + o_jobs);
  const uint8_t *needles = src + o_nd;
  if (stage) {
    constexpr uint32_t w16 = sizeof(DictJob) / 16;
    for (uint32_t i = tid; i < njobs * w16; i += blockDim.x)
      reinterpret_cast<u32x4 *>(s_jobs)[i] = reinterpret_cast<const u32x4 *>(jobs)[i];
    for (uint32_t i = tid; i < (nd_bytes + 3) / 4; i += blockDim.x)
      reinterpret_cast<uint32_t *>(s_nd)[i] = reinterpret_cast<const uint32_t *>(needles)[i];
    __syncthreads();
    jobs = s_jobs;
    needles = s_nd;
  }
  const uint32_t item = blockIdx.x * blockDim.x + tid;
  const uint32_t wave_item = __builtin_amdgcn_readfirstlane(item & ~63u);
  if (wave_item >= total) return;
  const uint32_t *jbase = reinterpret_cast<const uint32_t *>(src + o_jb);
  uint32_t lo = 0, hi = njobs;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if ((stage ? s_jobs[mid].item_base : jbase[mid]) <= wave_item) lo = mid;
    else hi = mid;
  }
  const DictJob jb = jobs[lo];
  const uint32_t v = item - jb.item_base;
  bool m = false;
  if (v < jb.nvals) {
    uint32_t o0 = G(jb.off)[v], o1 = G(jb.off)[v + 1];
    m = dev_contains(jb.bytes + o0, o1 - o0, needles + jb.needle_off, jb.needle_len);
  }
  if (jb.identity) {
    unsigned long long b = __ballot(m);
    const int lane = tid & 63;
    const uint32_t w0 = (v - lane) >> 5;  // first word of this wave
    const uint32_t words = (jb.nsets + 31) >> 5;
    if (lane == 0 && w0 < words) bitmaps[jb.bm_base + w0] = uint32_t(b);
    if (lane == 32 && w0 + 1 < words) bitmaps[jb.bm_base + w0 + 1] = uint32_t(b >> 32);
    if (lane == 0 && b != 0) anyf[lo] = 1u;  // (some value of the job matched; device memory)
  } else if (v < jb.nvals) {
    vmatch[jb.vmatch_base + v] = m ? 1 : 0;
  }
}

// multi-valued keys: a value set matches iff any of its values does
extern "C" __global__ void __launch_bounds__(256) dict_sets_kernel(const DictJob *jobs, const uint32_t *set_jobs,
                                                                   const uint32_t *prefix, uint32_t nsj,
                                                                   uint32_t total, const uint8_t *vmatch,
                                                                   uint32_t *bitmaps, uint32_t *anyf) {
  uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= total) return;
  uint32_t lo = 0, hi = nsj;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (prefix[mid] <= item) lo = mid;
    else hi = mid;
  }
  const DictJob &jb = jobs[set_jobs[lo]];
  uint32_t w = item - prefix[lo];
  uint32_t word = 0;
  if (jb.identity) {  // a streamed identity job (dict_stream_kernel): value v = set v, 32 match bytes per word
    const u32x4 *vb = reinterpret_cast<const u32x4 *>(vmatch + jb.vmatch_base + size_t(w) * 32);  // 32-aligned
    const u32x4 a = vb[0], c = vb[1];
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t x = d[k];  // bytes 0/1; bytes past nvals are zero
      word |= ((x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u)) << (4 * k);
    }
    bitmaps[jb.bm_base + w] = word;
    if (word) anyf[set_jobs[lo]] = 1u;
    return;
  }
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
  if (word) anyf[set_jobs[lo]] = 1u;
}

// ------------------------------------------------------------------------------------
// dict_stream: bytes.Contains over a large dictionary as ONE byte stream
//
// A key's value bytes sit back to back (dict_off | dict_bytes), so the substring test
// of every value is a scan of that stream for the needle, a match counting for the
// value that holds all of it. One lane per value (prep_kernel) leaves long values
// (db.statement: 100-2000 B) to a lane each: divergent, uncoalesced byte loops. Here a
// wave owns a 64 KiB span of the stream and walks it 1 KiB at a time: each lane loads
// 16 B (one coalesced dwordx4 per lane), the window and the next 1 KiB sit in LDS, a
// SWAR test of the needle's first two bytes at all 16 positions of a lane picks the
// candidates, the rest of the needle is compared from LDS, and a verified start maps to
// its value through the value offsets staged in LDS. Bytes are read once from HBM.
constexpr uint32_t kStreamSpan = 64u << 10;     // start positions per wave (at most; see stream_span)
constexpr uint32_t kStreamMaxNeedle = 1024;     // the 2 KiB window holds any match that starts in its first half
constexpr uint64_t kStreamMinBytes = 1u << 20;  // smaller dictionaries: prep_kernel (lane per value)
constexpr uint32_t kStreamOffs = 128;           // value offsets staged per reload
constexpr int kStreamAhead = 4;                 // KiB loaded ahead of the window, per wave
constexpr uint32_t kStreamWg = 4;               // waves (independent spans) per workgroup
struct StreamJob {
  const uint8_t *base;  // 16-byte aligned: the dictionary bytes start at base + lead
  const uint32_t *off;  // value offsets, nvals + 1
  uint64_t nbytes;
  uint32_t lead, nvals;
  uint32_t needle_off, needle_len;
  uint32_t vmatch_base, wave0;  // match bytes (32-aligned); first wave of this job
  // a second byte pair of the needle tested in registers beside its first two bytes: needle
  // bytes [pj, pj + 1], 2 <= pj <= min(len - 2, kStreamPairMax); 0 = none (the host picks
  // the pair that is rarest in the key's values: most steps then hold no candidate at all)
  uint32_t pj, pad[3];
};
static_assert(sizeof(StreamJob) == 64, "StreamJob layout");
constexpr uint32_t kStreamPairMax = 11;  // its bytes of a lane's 16 starts lie in this lane's + the next lane's 16

// bit 7 of each byte of the result: that byte of x is non-zero (exact, no carries across bytes)
__device__ __forceinline__ uint32_t nz_bytes(uint32_t x) { return (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u; }
// largest v in [lo, hi) with off[v] <= p (off[lo] <= p < off[hi] or hi = nvals + 1): 64-ary search
__device__ __forceinline__ uint32_t value_at(const uint32_t *off, uint32_t lo, uint32_t hi, uint64_t p, int lane) {
  while (hi - lo > 1) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t idx = lo + uint32_t(lane) * step;
    const bool le = idx < hi && uint64_t(G(off)[idx]) <= p;  // (global: flat loads make every wait drain LDS too)
    const uint32_t c = uint32_t(__popcll(__ballot(le)));  // lanes 0..c-1 (monotone offsets)
    lo = lo + (c - 1) * step;
    hi = min(hi, lo + step);
  }
  return lo;
}

// The ring of the stream kernel is loaded by inline asm and waited for by hand: the compiler's
// wait insertion drained every load in flight twice per ring turn (at the loop head, and where
// it copies a scalar through a VGPR whose load was still pending), so the read-ahead was
// mostly idle. Loads return in issue order, so "all but the newest N" covers the two oldest
// ring slots whatever other vector memory operations were issued after them.
__device__ __forceinline__ u32x4 ring_load(const uint8_t *p) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
// slots a (the step's KiB) and b (the next) have arrived; kRing - 2 newer loads may be in flight
__device__ __forceinline__ void ring_wait4(u32x4 &a, u32x4 &b) { asm volatile("s_waitcnt vmcnt(4)" : "+v"(a), "+v"(b)); }
__device__ __forceinline__ void ring_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The dictionary stream kernel runs one wave per workgroup: its LDS hand-offs between lanes
// need no s_barrier, and __syncthreads()' fence would also wait for every global load in
// flight (s_waitcnt vmcnt(0)), draining the read-ahead ring at each step. A single wave's LDS
// operations execute in order; the asm keeps the compiler from moving memory accesses across.
__device__ __forceinline__ void wave_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// kStreamWg waves per workgroup, each on its own span with its own LDS (no barriers: a
// one-wave workgroup per span would cap a CU at its workgroup slots, half the wave slots)
//
// A step's candidates (starts where the tested needle bytes all match) are appended to the
// wave's LDS list in scan order; the list is verified and mapped to values in batches of 64
// (one candidate per lane: the needle compared from global memory, L2-resident after the
// stream read it; the start's value found by a wave-wide 64-ary search plus the offsets
// around it staged in LDS). Verifying inline cost a whole wave iteration per candidate with
// one or two lanes active, on nearly every step of a dense needle (db.statement "from orders").
constexpr uint32_t kCandMax = 1024;  // >= the 64 x 16 starts of one step: a step always fits after a flush
extern "C" __global__ void __launch_bounds__(64 * kStreamWg) dict_stream_kernel(const StreamJob *jobs, uint32_t njobs,
                                                                                 const uint8_t *needles, uint8_t *vmatch,
                                                                                 uint32_t span, uint32_t nwaves) {
  __shared__ uint32_t s_cand_all[kStreamWg][kCandMax];                  // candidate starts - s0, ascending
  __shared__ uint32_t s_ndw_all[kStreamWg][kStreamMaxNeedle / 4 + 1];  // the needle as words
  __shared__ uint32_t s_off_all[kStreamWg][kStreamOffs + 1];
  const int lane = threadIdx.x & 63;
  const uint32_t wid = uint32_t(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
  uint32_t *const s_cand = s_cand_all[wid];
  uint32_t *const s_ndw = s_ndw_all[wid];
  uint32_t *const s_off = s_off_all[wid];
  const uint32_t w = blockIdx.x * kStreamWg + wid;
  if (w >= nwaves) return;
  uint32_t j = 0;
  for (uint32_t k = 1; k < njobs; k++)
    if (jobs[k].wave0 <= w) j = k;
  const StreamJob J = jobs[j];
  const uint32_t nl = J.needle_len;
  const uint64_t end = uint64_t(J.lead) + J.nbytes;  // aligned coordinates of the last byte + 1
  const uint64_t s0 = uint64_t(w - J.wave0) * span;
  // start positions q (aligned coordinates) of this wave: [qlo, qhi)
  const uint64_t qlo = max<uint64_t>(s0, J.lead);
  const uint64_t qhi = min<uint64_t>(s0 + span, end >= nl ? end - nl + 1 : 0);
  if (qlo >= qhi) return;
  // the needle as little-endian words (zero past its end)
  for (uint32_t i = lane; 4 * i < nl; i += 64) {
    uint32_t x = 0;
    for (uint32_t b = 0; b < 4; b++)
      if (4 * i + b < nl) x |= uint32_t(needles[J.needle_off + 4 * i + b]) << (8 * b);
    s_ndw[i] = x;
  }
  const uint32_t n0 = uint32_t(needles[J.needle_off]) * 0x01010101u;
  const uint32_t n1 = uint32_t(needles[J.needle_off + 1]) * 0x01010101u;  // (streamed needles: >= 2 bytes)
  const uint32_t pj = J.pj;  // (wave-uniform)
  const uint32_t r0 = pj ? uint32_t(needles[J.needle_off + pj]) * 0x01010101u : 0u;
  const uint32_t r1 = pj ? uint32_t(needles[J.needle_off + pj + 1]) * 0x01010101u : 0u;
  const uint32_t pq = pj >> 2, ps = pj & 3u;
  // a: aligned coordinate of this lane's 16 bytes. Past the stream's last 16-byte chunk
  // the load repeats that chunk: bytes past `end` only ever form starts >= qhi (dropped) and
  // are never compared.
  const uint64_t last16 = (end - 1) & ~uint64_t(15);
  const uint64_t last4 = (end - 1) & ~uint64_t(3);  // (verification's dword loads stay inside the value bytes)
  auto load16 = [&](uint64_t a) -> u32x4 { return ring_load(J.base + min(a, last16)); };
  wave_sync();
  uint32_t ncand = 0;   // (wave-uniform) candidates in the list
  uint64_t mdone = 0;   // (wave-uniform) starts below this lie in a value the wave has marked
  uint32_t vlo = 0;     // (wave-uniform) no value before it holds a start not yet verified
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  // verify the list's candidates, map the matches to their values, mark them; empties the list
  auto flush = [&]() {
    // every ring load has arrived before anything here may move a ring register (a copy of a
    // register whose load is still in flight would read the old bytes); flushes are rare
    ring_drain();
    wave_sync();
    for (uint32_t b0 = 0; b0 < ncand; b0 += 64) {
      const uint32_t nb = min(64u, ncand - b0);
      const bool act = uint32_t(lane) < nb;
      const uint64_t q = s0 + s_cand[b0 + (act ? uint32_t(lane) : 0u)];
      bool ok = act && q >= qlo && q < qhi && q >= mdone;
      // the needle, 4 bytes per round trip, from global memory (issuing 16 bytes' loads at once
      // measured slower: profiles/r04_final, `tools/gpu_r4b.sh abcfg4`)
      for (uint32_t k = 0; 4 * k < nl; k++) {
        if (__ballot(ok) == 0) break;
        const uint64_t a = q + 4 * k;
        const uint64_t a4 = a & ~uint64_t(3);
        const uint32_t lo4 = *G<uint32_t>(J.base + min(a4, last4));
        const uint32_t hi4 = *G<uint32_t>(J.base + min(a4 + 4, last4));
        const uint32_t x = __builtin_amdgcn_alignbyte(hi4, lo4, uint32_t(a & 3));
        const uint32_t rem = nl - 4 * k;
        const uint32_t m = rem >= 4 ? 0xffffffffu : (1u << (8 * rem)) - 1u;
        ok = ok && ((x ^ s_ndw[k]) & m) == 0;
      }
      const uint64_t okb = __ballot(ok);
      if (okb) {
        // the values of the batch's verified starts: the first one's by a 64-ary search from vlo,
        // then the offsets from there staged in LDS (a batch of a dense needle spans a few dozen
        // values); a start past the staged ones searches the global offsets
        const int f = __builtin_ctzll(okb);
        const uint64_t pf = uint64_t(__builtin_amdgcn_readlane(uint32_t(q - J.lead), f)) |
                            (uint64_t(__builtin_amdgcn_readlane(uint32_t((q - J.lead) >> 32), f)) << 32);
        const uint32_t v0 = value_at(J.off, vlo, J.nvals + 1, pf, lane);
        const uint32_t kv = min<uint32_t>(kStreamOffs, J.nvals - v0);
        for (uint32_t i = lane; i <= kv; i += 64) s_off[i] = G(J.off)[v0 + i];
        wave_sync();
        const uint64_t p = q - J.lead;
        uint32_t v = 0;
        uint64_t vend = 0;
        if (ok) {
          if (p < uint64_t(s_off[kv]) || kv == J.nvals - v0) {
            uint32_t lo = 0, hi = kv;
            while (hi - lo > 1) {
              const uint32_t mid = (lo + hi) >> 1;
              if (uint64_t(s_off[mid]) <= p) lo = mid;
              else hi = mid;
            }
            v = v0 + lo;
            vend = s_off[lo + 1];
          } else {
            uint32_t lo = v0 + kv, hi = J.nvals;
            while (hi - lo > 1) {
              const uint32_t mid = (lo + hi) >> 1;
              if (uint64_t(G(J.off)[mid]) <= p) lo = mid;
              else hi = mid;
            }
            v = lo;
            vend = G(J.off)[v + 1];
          }
          if (p + nl <= vend) vmatch[J.vmatch_base + v] = 1;  // (a match that runs into the next value does not count)
          else ok = false;
        }
        // later starts inside the furthest marked value add nothing; no later start lies before v0
        const uint64_t mb = __ballot(ok);
        if (mb) {
          const int hl = 63 - __builtin_clzll(mb);
          const uint64_t e = vend + J.lead;
          mdone = max(mdone, uint64_t(__builtin_amdgcn_readlane(uint32_t(e), hl)) |
                                 (uint64_t(__builtin_amdgcn_readlane(uint32_t(e >> 32), hl)) << 32));
        }
        vlo = v0;
        wave_sync();
      }
    }
    ncand = 0;
    wave_sync();
  };
  uint64_t cq = s0;
  // Ring slots: the window's two KiB + kStreamAhead KiB in flight. The step loop is unrolled
  // over the slots so each slot keeps its register (a rotation by moves waits for every
  // in-flight load it moves), and a slot is reloaded right after its step used it.
  constexpr int kRing = kStreamAhead + 2;
  static_assert(kRing == 6, "ring_wait4: kRing - 2 loads newer than a step's two slots");
  u32x4 ring[kRing];
#pragma unroll
  for (int k = 0; k < kRing; k++) ring[k] = load16(cq + uint64_t(k) * 1024 + lane * 16);
  // one 1 KiB step of start positions [c, c + 1024): cur = its bytes, nxt = the next KiB
  auto step = [&](const uint64_t c, const u32x4 cur, const u32x4 nxt) {
    // the needle's first two bytes at all 16 start positions of this lane, in registers:
    // the dword after the lane's 16 bytes is the next lane's first (DPP shift; lane 63: the
    // next KiB's first dword)
    const uint32_t nx0 = __builtin_amdgcn_readlane(nxt.x, 0);
    uint32_t nxw = uint32_t(__builtin_amdgcn_update_dpp(0, int(cur.x), 0x130, 0xf, 0xf, false));  // wave_shl:1
    if (lane == 63) nxw = nx0;
    const uint32_t d[5] = {cur.x, cur.y, cur.z, cur.w, nxw};
    // x[k]: a byte is zero where every tested needle byte matches at that start (the xors of
    // the pairs OR-ed together: one zero-byte test per dword for all of them)
    uint32_t xs[4];
#pragma unroll
    for (int k = 0; k < 4; k++) xs[k] = (d[k] ^ n0) | (__builtin_amdgcn_alignbyte(d[k + 1], d[k], 1) ^ n1);
    if (pj) {
      // the second pair: bytes pj, pj + 1 after each start, from this lane's 16 bytes and the
      // next lane's (DPP; lane 63: the next KiB's first lane). V[m] = window bytes pj + 4m ..
      const uint32_t ny = uint32_t(__builtin_amdgcn_update_dpp(0, int(cur.y), 0x130, 0xf, 0xf, false));
      const uint32_t nzw = uint32_t(__builtin_amdgcn_update_dpp(0, int(cur.z), 0x130, 0xf, 0xf, false));
      const uint32_t nww = uint32_t(__builtin_amdgcn_update_dpp(0, int(cur.w), 0x130, 0xf, 0xf, false));
      // (the readlanes unconditional: a select, not a branch around each)
      const uint32_t n1y = __builtin_amdgcn_readlane(nxt.y, 0), n1z = __builtin_amdgcn_readlane(nxt.z, 0),
                     n1w = __builtin_amdgcn_readlane(nxt.w, 0);
      const bool l63 = lane == 63;
      const uint32_t W[8] = {cur.x, cur.y, cur.z, cur.w, nxw, l63 ? n1y : ny, l63 ? n1z : nzw, l63 ? n1w : nww};
      uint32_t V[5];
      if (pq == 0) {
#pragma unroll
        for (int m = 0; m < 5; m++) V[m] = __builtin_amdgcn_alignbyte(W[m + 1], W[m], ps);
      } else if (pq == 1) {
#pragma unroll
        for (int m = 0; m < 5; m++) V[m] = __builtin_amdgcn_alignbyte(W[m + 2], W[m + 1], ps);
      } else {
#pragma unroll
        for (int m = 0; m < 5; m++) V[m] = __builtin_amdgcn_alignbyte(W[m + 3], W[m + 2], ps);
      }
#pragma unroll
      for (int k = 0; k < 4; k++) xs[k] |= (V[k] ^ r0) | (__builtin_amdgcn_alignbyte(V[k + 1], V[k], 1) ^ r1);
    }
    // a zero byte anywhere: (x - 0x01010101) & ~x & 0x80808080 is non-zero exactly when x has
    // one (its false flags sit above a true zero: right for "any", not for "which")
    uint32_t any = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) any |= (xs[k] - 0x01010101u) & ~xs[k];
    // most steps hold no candidate in any lane: nothing else to do (a wave-uniform branch)
    if (__ballot((any & 0x80808080u) != 0) == 0) return;
    // bit 7 of byte b of f[k]: start 4k + b of this lane is a candidate (exact per byte); starts
    // inside a value the wave already marked are dropped when the list is verified
    uint32_t f[4], mine = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      f[k] = nz_bytes(xs[k]) ^ 0x80808080u;
      mine += uint32_t(__popc(f[k]));
    }
    // append the step's candidates to the list (a lane's in start order, lanes in order): a
    // lane's place is the count of the lanes below it (one ballot when no lane has two)
    uint32_t pre, tot;
    if (__ballot(mine > 1u) == 0) {
      const uint64_t one = __ballot(mine != 0u);
      pre = uint32_t(__popcll(one & below));
      tot = uint32_t(__popcll(one));
    } else {
      pre = tot = 0;
#pragma unroll
      for (int b = 0; b < 5; b++) {
        const uint64_t bal = __ballot((mine >> b) & 1u);
        pre += uint32_t(__popcll(bal & below)) << b;
        tot += uint32_t(__popcll(bal)) << b;
      }
    }
    if (ncand + tot > kCandMax) flush();
    uint32_t at = ncand + pre;
    const uint32_t rel = uint32_t(c - s0) + uint32_t(lane) * 16;
#pragma unroll
    for (int k = 0; k < 4; k++)
      for (uint32_t m = f[k]; m; m &= m - 1) s_cand[at++] = rel + 4 * k + (uint32_t(__builtin_ctz(m)) >> 3);
    ncand += tot;
  };
  for (; cq < qhi; cq += uint64_t(kRing) * 1024) {
#pragma unroll
    for (int st = 0; st < kRing; st++) {
      const uint64_t c = cq + uint64_t(st) * 1024;
      if (c >= qhi) break;
      ring_wait4(ring[st], ring[(st + 1) % kRing]);
      step(c, ring[st], ring[(st + 1) % kRing]);
      ring[st] = load16(c + uint64_t(kRing) * 1024 + lane * 16);  // (the KiB kRing steps ahead)
    }
  }
  ring_drain();  // (no load of the ring outlives the wave)
  if (ncand) flush();
}

// ------------------------------------------------------------------------------------
// scan
// Scan columns are allocated to whole kColPad-entry multiples (devctx.hip), so every
// tile load is in bounds; entries past n are only masked off.
static_assert(kColPad % (kThreads * 4 * kSteps) == 0, "column padding covers whole tiles");

// 4 consecutive column values, raw (decoded by col_at). Branch-free over the
// (wave-uniform) width: 4 dword loads whose addresses collapse onto the first
// dword for narrow columns (same cache line, no extra HBM bytes). A width switch
// here makes hipcc merge the three load shapes with vmcnt(0) waits that serialise
// every outstanding load.
__device__ __forceinline__ u32x4 load_col(const void *col, uint32_t width, uint64_t e) {
  const auto *c = G<uint32_t>(static_cast<const uint8_t *>(col) + e * width);
  u32x4 r;
  r.x = c[0];
  r.y = c[width >= 2 ? 1 : 0];
  r.z = c[width == 4 ? 2 : 0];
  r.w = c[width == 4 ? 3 : 0];
  return r;
}
__device__ __forceinline__ uint32_t col_at(u32x4 r, uint32_t width, int j) {
  if (width == 1) return (r.x >> (8 * j)) & 0xffu;
  if (width == 2) return ((j < 2 ? r.x : r.y) >> (16 * (j & 1))) & 0xffffu;
  return j == 0 ? r.x : j == 1 ? r.y : j == 2 ? r.z : r.w;
}
// Bit 0: value set x matches the term (x >= nsets: the all-ones sentinel, key absent, FindTag
// fails). Branch-free over x: the sentinel reads word 0 and is masked off (an early return
// became an exec-mask branch per entry that diverges on real data); the LDS / global choice is
// per term (wave-uniform).
__device__ __forceinline__ uint32_t term_bit(const ScanTerm &T, const uint32_t *lds_bm, uint32_t x) {
  const uint32_t in = uint32_t(x < T.nsets);
  const uint32_t xi = in ? x : 0u;
  const uint32_t lo = __builtin_amdgcn_readfirstlane(T.lds_off);
  const uint32_t w = lo != kNoLds ? lds_bm[lo + (xi >> 5)] : G(T.bm)[xi >> 5];
  return in & (w >> (xi & 31));
}

// One tile's filter-column registers for this thread: entries
// tile0 + 1024k + 4*tid + j (k < kSteps, j < 4). Loaded one tile ahead of use.
template <int NT, bool W1>
struct TileRegs {
  u32x4 d[kSteps], s[kSteps], e[kSteps];
  typename std::conditional<W1, uint32_t, u32x4>::type tv[NT > 0 ? NT : 1][kSteps];  // u8 columns: one dword
};

__device__ __forceinline__ uint64_t step_base(uint64_t tile0, int k, int tid) {
  return tile0 + uint64_t(k) * (kThreads * 4) + uint64_t(tid) * 4;
}

// Issue every load of one tile (NT < 0: the term columns are loaded in eval_tile).
// Steps of a tile that start at or past `lim` (the workgroup's range end) re-load
// step 0's addresses (cache hits, no extra HBM bytes) and are masked off in eval.
__device__ __forceinline__ uint64_t load_base(uint64_t tile0, int k, int tid, uint64_t lim) {
  const uint64_t s0 = tile0 + uint64_t(k) * kUnit;
  return (s0 < lim ? s0 : tile0) + uint64_t(tid) * 4;
}
template <int NT, bool DUR, bool RANGE, bool W1>
__device__ __forceinline__ void load_tile(TileRegs<NT, W1> &R, const ScanSeg &S, const ScanTerm *T, uint64_t tile0,
                                          uint64_t lim, int tid) {
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint64_t e = load_base(tile0, k, tid, lim);
    if (DUR) R.d[k] = load4_u32(S.dur32, e);
    if (RANGE) {
      R.s[k] = load4_u32(S.start_s, e);
      R.e[k] = load4_u32(S.end_s, e);
    }
  }
  if (NT > 0) {
#pragma unroll
    for (int q = 0; q < (NT > 0 ? NT : 1); q++)
#pragma unroll
      for (int k = 0; k < kSteps; k++) {
        const uint64_t e = load_base(tile0, k, tid, lim);
        if constexpr (W1) R.tv[q][k] = *G<uint32_t>(static_cast<const uint8_t *>(T[q].col) + e);
        else R.tv[q][k] = load_col(T[q].col, T[q].width, e);
      }
  }
}

// Match mask of one loaded tile: bit (4k+j) <-> entry tile0 + 1024k + 4*tid + j.
template <int NT, bool DUR, bool RANGE, bool W1>
__device__ __forceinline__ uint32_t eval_tile(const TileRegs<NT, W1> &R, const ScanParams &P, const ScanSeg &S,
                                              const ScanTerm *T, const uint32_t *lds_bm, uint64_t tile0,
                                              uint64_t lim, int tid) {
  const uint64_t n = lim;  // entries of this workgroup's range (<= the block's n)
  uint32_t mask = kMaskAll;
  if (tile0 + kTile > n) {  // last tile of the range
    mask = 0;
#pragma unroll
    for (int k = 0; k < kSteps; k++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (step_base(tile0, k, tid) + j < n) mask |= 1u << (4 * k + j);
  }
  if (DUR) {
    if (!P.need64) {  // both thresholds < 2^32-1 ns: the saturated u32 column is exact
      const uint32_t mn = uint32_t(P.min_ns), mx = uint32_t(P.max_ns);
#pragma unroll
      for (int k = 0; k < kSteps; k++) {
        const uint32_t dv[4] = {R.d[k].x, R.d[k].y, R.d[k].z, R.d[k].w};
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (!((!P.has_min || dv[j] >= mn) && (!P.has_max || dv[j] <= mx))) mask &= ~(1u << (4 * k + j));
      }
    } else {
#pragma unroll
      for (int k = 0; k < kSteps; k++) {
        const uint32_t dv[4] = {R.d[k].x, R.d[k].y, R.d[k].z, R.d[k].w};
        const uint64_t eb = step_base(tile0, k, tid);
#pragma unroll
        for (int j = 0; j < 4; j++) {
          uint64_t dd = dv[j];
          if (dv[j] == 0xffffffffu && eb + j < n) dd = G(S.dur64)[eb + j];
          if (!((!P.has_min || dd >= P.min_ns) && (!P.has_max || dd <= P.max_ns))) mask &= ~(1u << (4 * k + j));
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    if (RANGE) {
      const uint32_t sv[4] = {R.s[k].x, R.s[k].y, R.s[k].z, R.s[k].w};
      const uint32_t ev[4] = {R.e[k].x, R.e[k].y, R.e[k].z, R.e[k].w};
#pragma unroll
      for (int j = 0; j < 4; j++)  // req.Start <= endSeconds && req.End >= startSeconds
        if (!(P.start_s <= ev[j] && P.end_s >= sv[j])) mask &= ~(1u << (4 * k + j));
    }
    if (NT > 0) {
#pragma unroll
      for (int q = 0; q < (NT > 0 ? NT : 1); q++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          uint32_t ok;
          if constexpr (W1) {  // u8 column, bitmap in LDS padded to 8 words: branch-free lookup
            const uint32_t x = (R.tv[q][k] >> (8 * j)) & 0xffu;
            const uint32_t w = lds_bm[T[q].lds_off + (x >> 5)];
            ok = uint32_t(x < T[q].nsets) & (w >> (x & 31));
          } else {
            ok = term_bit(T[q], lds_bm, col_at(R.tv[q][k], T[q].width, j));
          }
          mask &= ~((~ok & 1u) << (4 * k + j));
        }
    }
  }
  if (NT < 0) {
    for (uint32_t q = 0; q < S.nterms; q++) {
      const ScanTerm Tq = P.terms[S.term0 + q];
      u32x4 c[kSteps];
#pragma unroll
      for (int k = 0; k < kSteps; k++) c[k] = load_col(Tq.col, Tq.width, load_base(tile0, k, tid, lim));
#pragma unroll
      for (int k = 0; k < kSteps; k++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          mask &= ~((~term_bit(Tq, lds_bm, col_at(c[k], Tq.width, j)) & 1u) << (4 * k + j));
    }
  }
  return mask;
}

// ------------------------------------------------------------------------------------
// helpers
__device__ __forceinline__ unsigned long long block_sum(unsigned long long v, unsigned long long *red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  unsigned long long t = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; w++) t += red[w];
  return t;
}
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) {
  return a < b ? a : b;
}

// The launch-order index of this workgroup: blockIdx.x, or with use_ticket a ticket
// claimed from one device counter, so that every workgroup this one waits for (a lower
// index) is already running whatever order the dispatcher chose.
__device__ __forceinline__ uint32_t wg_order(const ScanParams &P, bool use_ticket) {
  if (!use_ticket) return blockIdx.x;
  __shared__ uint32_t s_ticket;
  if (threadIdx.x == 0)
    s_ticket = uint32_t(__hip_atomic_fetch_add(P.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                        P.ticket_base);
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s_ticket);
}


// The matches of one tile (bit 4k+j of `mask` <-> entry tile0 + 1024k + 4*tid + j)
// in scan order (k, thread, j): ranks from a wave scan of kSteps packed 16-bit
// per-step counts; rank r -> output slot slot_of(run + r) (~0 = not kept). Record
// fields are gathered from the cold columns; sink(slot, words) stores one record
// (6 x u64).
template <class Slot, class Sink>
__device__ __forceinline__ void emit_tile(const ScanSeg &S, uint32_t mask, uint64_t tile0, unsigned long long run,
                                          unsigned long long *s_wsum, Slot &&slot_of, Sink &&sink,
                                          bool compact = false) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  unsigned long long pc = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) pc |= (unsigned long long)__popc((mask >> (4 * k)) & 0xfu) << (16 * k);
  unsigned long long inc = pc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    unsigned long long o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  __syncthreads();
  if (lane == 63) s_wsum[wid] = inc;
  __syncthreads();
  unsigned long long before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; w++) {
    if (w < wid) before += s_wsum[w];
    tot += s_wsum[w];
  }
  const unsigned long long mine_ex = before + inc - pc;
  uint32_t step_base = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t nib = (mask >> (4 * k)) & 0xfu;
    uint32_t r = step_base + uint32_t((mine_ex >> (16 * k)) & 0xffff);
    step_base += uint32_t((tot >> (16 * k)) & 0xffff);
    for (int j = 0; j < 4; j++) {
      if (!(nib & (1u << j))) continue;
      const unsigned long long slot = slot_of(run + r++);
      if (slot == ~0ull) continue;
      const uint64_t ei = tile0 + uint64_t(k) * kUnit + uint64_t(tid) * 4 + j;
      if (compact) {  // (position only: the host gathers the fields)
        const unsigned long long w1[1] = {(unsigned long long)uint32_t(ei) | (unsigned long long)S.block_idx << 32};
        sink(slot, w1);
        continue;
      }
      const u32x4 id = *G<u32x4>(S.ids + ei * 16);
      const uint64_t st = G(S.start_ns)[ei], en = G(S.end_ns)[ei];
      const uint64_t nm = G(reinterpret_cast<const uint64_t *>(S.names))[ei];
      const uint32_t il = G(S.id_len)[ei];
      const unsigned long long w[6] = {(unsigned long long)id.x | (unsigned long long)id.y << 32,
                                       (unsigned long long)id.z | (unsigned long long)id.w << 32,
                                       (unsigned long long)st, (unsigned long long)en,
                                       (unsigned long long)uint32_t(ei) | (unsigned long long)(S.block_idx | (il << 24)) << 32,
                                       (unsigned long long)nm};
      sink(slot, w);
    }
  }
}

// ------------------------------------------------------------------------------------
// search: scan + in-order compaction in one launch
//
// Phase 1 (scan): the workgroup streams its tiles; per tile a 16-bit mask per
//   thread (LDS for the first kLdsTiles tiles, global beyond) and a count.
// Phase 2 (publish / look-back): the workgroup publishes its match count as one
//   8-byte {epoch, count} word (agent-scope store, bypasses the non-coherent L1/L2
//   paths), then sums the words of every lower-numbered workgroup, polling those
//   not yet published. Workgroups are dispatched in index order, so every waited-on
//   workgroup is resident or done; the poll is bounded anyway (error flag, the host
//   fails the query loudly). Only workgroups with matches (and the last one, which
//   writes the header) look back.
// Phase 3 (emit): records in scan order straight into the pinned host buffer.
constexpr uint32_t kLdsTiles = 16;      // tiles per workgroup whose masks stay in LDS
constexpr uint32_t kMaxTpw = 2048;      // tiles per workgroup (per-tile counts in LDS)
constexpr uint32_t kSpinMax = 1u << 22; // look-back poll bound (~seconds): never reached unless broken
constexpr uint32_t kMaxSegs = 2048;

// workgroup -> block and per-block record caps, from the device descriptors
struct DescSegs {
  const uint16_t *wg_seg;
  const ScanSeg *segs;
  __device__ uint32_t seg_of(uint32_t i) const { return G(wg_seg)[i]; }
  __device__ unsigned long long cap_of(uint32_t s) const { return segs[s].cap; }
};
// ... from LDS copies of the kernel-argument tables (one-launch path)
struct ArgSegs {
  const uint32_t *first_wg;  // nsegs + 1
  const unsigned long long *cap;
  uint32_t nsegs;
  __device__ uint32_t seg_of(uint32_t i) const {
    uint32_t lo = 0, hi = nsegs;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (first_wg[mid] <= i) lo = mid;
      else hi = mid;
    }
    return lo;
  }
  __device__ unsigned long long cap_of(uint32_t s) const { return cap[s]; }
};

// Phases 1-3 for one workgroup of block `si`. `init_segs` zeroes lds_seg (and
// stages the block tables) after the scan. `issue_stage` issues
// the loads the bitmaps need (before the first tile's loads), `wait_bitmaps` brings
// the term bitmaps into LDS and ends with a barrier; it runs after the first tile's
// loads are issued, so dictionary latency hides under the stream.
template <int NT, bool DUR, bool RANGE, bool W1, bool SEG, class Segs, class Issue, class Wait, class Init>
__device__ __forceinline__ void scan_emit(const ScanParams &P, const ScanSeg &S, const ScanTerm *T, uint32_t si,
                                          const Segs &segs, const uint32_t *lds_bm, uint16_t *lds_mask,
                                          uint32_t *lds_seg, unsigned long long *lds_rec, unsigned long long t_start,
                                          unsigned long long *stamps, uint32_t wg, Issue &&issue_stage,
                                          Wait &&wait_bitmaps, Init &&init_segs, bool dead = false) {
  __shared__ uint16_t s_tc[kMaxTpw];
  __shared__ uint32_t s_wcnt[2][kThreads / 64];
  __shared__ unsigned long long s_red[kThreads / 64];
  __shared__ unsigned long long s_wsum[kThreads / 64];
  __shared__ unsigned long long s_bits[kSteps * kUnit / 64];  // bitmap mode: one tile's words
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // (`stamps` = P.stamps, passed in already loaded: a kernel-argument load here would
  // add a scalar round trip in front of the first tile load)
  auto stamp = [&](int k) {
    if (stamps && tid == 0) stamps[uint64_t(wg) * kStampSlots + k] = __builtin_amdgcn_s_memrealtime();
  };
  if (stamps && tid == 0) {
    stamps[uint64_t(wg) * kStampSlots] = t_start;
    // where the workgroup ran: XCC_ID (hwreg 20) << 32 | HW_ID (hwreg 4: wave, SIMD, CU, SH, SE)
    const unsigned long long hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    const unsigned long long xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    stamps[uint64_t(wg) * kStampSlots + 8] = (xcc << 32) | hw;
  }

  // ---- phase 1: scan, one tile of loads in flight ahead of the tile evaluated
  const uint32_t lw = wg - S.first_wg;  // static units split evenly over the block's workgroups (+-1 unit)
  const uint32_t us = S.nunits - min(S.nunits, 2 * S.tail);  // static units: all but the tail tiles
  const uint32_t u0 = uint32_t(uint64_t(lw) * us / S.nwg);
  const uint32_t u1 = uint32_t(uint64_t(lw + 1) * us / S.nwg);
  const uint32_t ntl = (u1 - u0 + kSteps - 1) / kSteps;
  const uint64_t tbase = uint64_t(u0) * kUnit;
  const uint64_t lim = min(uint64_t(u1) * kUnit, S.n);
  uint32_t wsum = 0;
  auto finish = [&](uint32_t t, uint32_t mask) {
    uint32_t c = __popc(mask);
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, 64);
    const int buf = t & 1;
    if (lane == 0) s_wcnt[buf][wid] = c;
    __syncthreads();  // (LDS only: hipcc waits lgkmcnt here, the next tile's loads stay in flight)
    uint32_t tc = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; w++) tc += s_wcnt[buf][w];
    if (P.bitmap) {
      // one bit per entry: step k of the tile is unit tile0/kUnit + k, and lanes 16m .. 16m+15
      // hold the nibbles of its 64-entry word m (entry = tile0 + k*kUnit + 4*tid + j). The tile's
      // 32 words are staged in LDS and stored by 32 consecutive lanes (whole-line PCIe writes;
      // 8-byte stores from scattered lanes had made the bitmap cost as much as the positions);
      // only the units of this workgroup's range (a tile past it belongs to the next workgroup)
      const uint64_t te = tbase + uint64_t(t) * kTile;
#pragma unroll
      for (int k = 0; k < kSteps; k++) {
        unsigned long long v = (unsigned long long)((mask >> (4 * k)) & 0xfu) << (4 * (lane & 15));
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) v |= __shfl_xor(v, d, 64);
        if ((lane & 15) == 0) s_bits[k * (kUnit / 64) + (tid >> 4)] = v;
      }
      __syncthreads();
      if (tid < kSteps * kUnit / 64 && te + uint64_t(tid / (kUnit / 64)) * kUnit < lim)
        host_store(P.bitmap + S.bm_word0 + te / 64 + uint64_t(tid), s_bits[tid]);
      return;
    }
    if (t < kLdsTiles) lds_mask[t * kThreads + tid] = uint16_t(mask);
    else if (tc) P.mask[(uint64_t(wg) * P.mask_tpw + t) * kThreads + tid] = uint16_t(mask);
    if (tid == 0) s_tc[t] = uint16_t(tc);
    wsum += tc;
  };
  TileRegs<NT, W1> ra, rb;
  // two register sets, unrolled by two (no dynamic register indexing). Both
  // are loaded before the bitmaps are waited for (the setup chain — descriptors,
  // dictionary staging, match — hides under two tiles of stream); afterwards each
  // set is refilled right after its tile is evaluated. A prefetch past the last
  // tile re-reads the last tile (cache hit) so the load sequence stays
  // unconditional and hipcc's vmcnt counting stays exact.
  auto tile0 = [&](uint32_t t) { return tbase + uint64_t(min(t, ntl - 1)) * kTile; };
  const uint32_t prio = P.prio;
  auto set_prio = [&](uint32_t t) {  // (s_setprio takes an immediate)
    if (!prio) return;
    const uint32_t lvl = min(3u, (t * 4) / max(ntl, 1u));
    if (lvl == 0) __builtin_amdgcn_s_setprio(3);
    else if (lvl == 1) __builtin_amdgcn_s_setprio(2);
    else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };
  // (dead: a term of the block matched no dictionary value, so no entry matches: nothing is
  // loaded or scanned; the workgroup publishes a count of 0)
  if (!dead) {
    issue_stage();
    load_tile<NT, DUR, RANGE, W1>(ra, S, T, tile0(0), lim, tid);  // (ntl >= 1: never more workgroups than units)
    load_tile<NT, DUR, RANGE, W1>(rb, S, T, tile0(1), lim, tid);
    wait_bitmaps();
    stamp(1);
    for (uint32_t t = 0;; t += 2) {
      set_prio(t);
      finish(t, eval_tile<NT, DUR, RANGE, W1>(ra, P, S, T, lds_bm, tile0(t), lim, tid));
      if (t + 1 >= ntl) break;
      load_tile<NT, DUR, RANGE, W1>(ra, S, T, tile0(t + 2), lim, tid);
      finish(t + 1, eval_tile<NT, DUR, RANGE, W1>(rb, P, S, T, lds_bm, tile0(t + 1), lim, tid));
      if (t + 2 >= ntl) break;
      load_tile<NT, DUR, RANGE, W1>(rb, S, T, tile0(t + 3), lim, tid);
    }
  }
  if (P.bitmap) {  // (no counts, no records: the host counts and expands the bits after the launch)
    stamp(2);
    stamp(4);
    return;
  }

  if (prio) __builtin_amdgcn_s_setprio(0);
  // ---- phase 2: publish, look back
  // (the per-block tables the look-back needs are staged only now: their loads
  // would otherwise sit in front of the dictionary and tile loads)
  init_segs();
  __syncthreads();
  stamp(2);
  if constexpr (SEG) {
    // segment mode: the first min(seg_cap, cap) matches of this workgroup go to its
    // own segment of the pinned buffer, its count to counts[wg]; the host concatenates
    // the segments in workgroup order (= scan order). No workgroup waits on another.
    // The count is stored after the records have completed: the host reads a count
    // that is no longer the sentinel it wrote before the launch as "this segment is
    // final" and pulls it into its caches while later workgroups are still scanning.
    stamp(3);
    // records are gathered into LDS first (no gather load waits behind a host store:
    // loads and stores share vmcnt), then copied out in one burst of write-through
    // stores, the only host traffic the completion protocol waits for
    const unsigned long long keep = umin64(P.seg_cap, S.cap);
    unsigned long long run = 0;
    auto to_lds = [&](unsigned long long slot, const unsigned long long *w) {
#pragma unroll
      for (int i = 0; i < 6; i++) lds_rec[slot * 6 + i] = w[i];
    };
    auto kept = [&](unsigned long long r) { return r < keep ? r : ~0ull; };
    if (wsum) {
      for (uint32_t t = 0; t < ntl; t++) {
        const uint32_t tc = s_tc[t];
        if (tc == 0) continue;
        const uint32_t mask = t < kLdsTiles ? lds_mask[t * kThreads + tid]
                                            : G(P.mask)[(uint64_t(wg) * P.mask_tpw + t) * kThreads + tid];
        emit_tile(S, mask, tbase + uint64_t(t) * kTile, run, s_wsum, kept, to_lds);
        run += tc;
      }
    }
    // tail: the block's last S.tail tiles, one per claim from the block's counter, by
    // whichever of its workgroups is free first (per-CU bandwidth is uneven: the early
    // finishers absorb the slow ones' share). The records of a workgroup stay in its own
    // segment in claim order, after its static ones; the host orders each block's
    // records by scan position (tail positions follow every static one).
    if (S.tail) {
      __shared__ uint32_t s_claim;
      auto claim = [&]() -> uint32_t {
        __syncthreads();
        if (tid == 0)
          s_claim = __hip_atomic_fetch_add(P.steal + 32 * si, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                    S.steal_base;
        __syncthreads();
        return s_claim;
      };
      uint32_t c = claim();
      while (c < S.tail) {
        const uint64_t t0 = uint64_t(us + 2 * c) * kUnit;
        const uint64_t tl = min(uint64_t(us + 2 * c + 2) * kUnit, S.n);
        load_tile<NT, DUR, RANGE, W1>(ra, S, T, t0, tl, tid);
        const uint32_t next = claim();  // (its return waits for the tile loads anyway)
        const uint32_t mask = eval_tile<NT, DUR, RANGE, W1>(ra, P, S, T, lds_bm, t0, tl, tid);
        uint32_t cnt = __popc(mask);
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
        if (lane == 0) s_wcnt[0][wid] = cnt;
        __syncthreads();
        uint32_t tc = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; w++) tc += s_wcnt[0][w];
        if (tc) emit_tile(S, mask, t0, run, s_wsum, kept, to_lds);
        run += tc;
        wsum += tc;
        c = next;
      }
    }
    if (wsum) {
      __syncthreads();
      const uint32_t nw = uint32_t(umin64(wsum, keep)) * 6;
      auto *dst = reinterpret_cast<unsigned long long *>(P.out + P.hdr_bytes) + (unsigned long long)wg * P.seg_cap * 6;
      for (uint32_t i = tid; i < nw; i += kThreads) host_store(dst + i, lds_rec[i]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (memory clobber: no store moves below it)
      __syncthreads();
    }
    if (tid == 0) host_store(P.counts + wg, wsum);
    stamp(4);
    return;
  }
  const unsigned long long tag = (unsigned long long)P.epoch << 32;
  if (tid == 0) __hip_atomic_store(&P.agg[wg], tag | wsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool last = wg + 1 == P.nwg;
  if (wsum == 0 && !last) {
    stamp(3);
    stamp(4);
    return;
  }
  const bool per_seg = P.limit_mode || last;
  unsigned long long loc = 0;
  for (uint32_t i = tid; i < wg; i += kThreads) {
    unsigned long long w;
    uint32_t spins = 0;
    while (((w = __hip_atomic_load(&P.agg[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & ~0xffffffffull) != tag) {
      if (++spins > kSpinMax) {
        reinterpret_cast<volatile unsigned long long *>(P.out)[1] = 1;  // host fails the query
        w = tag;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    const uint32_t v = uint32_t(w);
    if (per_seg) atomicAdd(&lds_seg[segs.seg_of(i)], v);
    else loc += v;
  }
  unsigned long long *hdr = reinterpret_cast<unsigned long long *>(P.out);
  unsigned long long seg_rank0, base;  // rank of this workgroup's first match in its block; output slot of rank 0
  if (!per_seg) {
    seg_rank0 = 0;  // unused in this mode
    base = block_sum(loc, s_red);
  } else {
    __syncthreads();
    seg_rank0 = lds_seg[si];  // lower workgroups of the same block
    unsigned long long b = 0;
    for (uint32_t s2 = tid; s2 < si; s2 += kThreads) {
      const unsigned long long c = lds_seg[s2];
      b += P.limit_mode ? umin64(c, segs.cap_of(s2)) : c;
    }
    base = block_sum(b, s_red);
    if (!P.limit_mode) base += seg_rank0;
    if (last) {  // header: records written + per-block counts (this block's total includes our own)
      __syncthreads();
      if (tid == 0) lds_seg[si] += wsum;
      __syncthreads();
      unsigned long long tot = 0;
      for (uint32_t s2 = tid; s2 < P.nsegs; s2 += kThreads) {
        const unsigned long long c = P.limit_mode ? umin64(lds_seg[s2], segs.cap_of(s2)) : lds_seg[s2];
        host_store(hdr + 8 + s2, c);
        tot += c;
      }
      tot = block_sum(tot, s_red);
      if (tid == 0) host_store(hdr + 0, tot);
    }
  }
  stamp(3);
  if (wsum == 0 || (P.limit_mode && seg_rank0 >= S.cap)) {  // (the block's first `cap` matches precede us)
    stamp(4);
    return;
  }

  // ---- phase 3: emit in scan order
  MatchRec *out = reinterpret_cast<MatchRec *>(P.out + P.hdr_bytes);
  unsigned long long run = 0;  // matches of this workgroup before the current tile
  for (uint32_t t = 0; t < ntl; t++) {
    const uint32_t tc = s_tc[t];
    if (tc == 0) continue;
    const uint32_t mask = t < kLdsTiles ? lds_mask[t * kThreads + tid]
                                        : G(P.mask)[(uint64_t(wg) * P.mask_tpw + t) * kThreads + tid];
    emit_tile(S, mask, tbase + uint64_t(t) * kTile, run, s_wsum,
              [&](unsigned long long rank_wg) -> unsigned long long {  // rank among this workgroup's matches
                if (P.limit_mode) return seg_rank0 + rank_wg < S.cap ? base + seg_rank0 + rank_wg : ~0ull;
                return base + rank_wg < P.out_cap ? base + rank_wg : ~0ull;
              },
              [&](unsigned long long slot, const unsigned long long *w) {
                if (P.compact) {
                  reinterpret_cast<unsigned long long *>(P.out + P.hdr_bytes)[slot] = w[0];
                  return;
                }
                auto *d = reinterpret_cast<unsigned long long *>(out + slot);
#pragma unroll
                for (int i = 0; i < 6; i++) d[i] = w[i];
              },
              P.compact != 0);
    run += tc;
  }
  stamp(4);
}

// General path: descriptors in device memory (copied by prep_kernel), value-set
// bitmaps precomputed by prep/dict_sets.
template <int NT, bool DUR, bool RANGE, bool W1>
__global__ void __launch_bounds__(kThreads) search_kernel(ScanParams P) {
  const unsigned long long t_start = P.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *lds_bm = lds;                                                   // [lds_bm_words]
  uint16_t *lds_mask = reinterpret_cast<uint16_t *>(lds + P.lds_bm_words);  // [kLdsTiles][kThreads]
  uint32_t *lds_seg = lds + P.lds_bm_words + kLdsTiles * kThreads / 2;      // [nsegs]
  const int tid = threadIdx.x;
  if (P.anyf && P.nterms) {  // every block has a term no dictionary value matched: nothing to scan
    int live = 0;
    for (uint32_t i = uint32_t(tid); i < P.nsegs; i += kThreads) {
      bool dead = false;
      for (uint32_t q = 0; q < P.nterms; q++) dead = dead || G(P.anyf)[uint64_t(i) * P.nterms + q] == 0u;
      live |= dead ? 0 : 1;
    }
    if (!__syncthreads_or(live)) return;
  }
  const uint32_t vb = wg_order(P, P.use_ticket);
  const uint32_t si = P.wg_seg[vb];
  const ScanSeg S = P.segs[si];
  constexpr int NTA = NT > 0 ? NT : 1;
  ScanTerm T[NTA];
  if (NT > 0)
#pragma unroll
    for (int q = 0; q < NTA; q++) T[q] = P.terms[S.term0 + q];
  // the dictionary pass found no value of some term in this block: no entry can match
  bool dead = false;
  if (NT > 0)
#pragma unroll
    for (int q = 0; q < NTA; q++)
      if (uint32_t(q) < S.nterms && T[q].anyf && *G(T[q].anyf) == 0u) dead = true;
  scan_emit<NT, DUR, RANGE, W1, false>(P, S, T, si, DescSegs{P.wg_seg, P.segs}, lds_bm, lds_mask, lds_seg, nullptr, t_start,
                                P.stamps, vb, [] {}, [&] {
                                  for (uint32_t q = 0; q < S.nterms; q++) {  // stage the small bitmaps in LDS
                                    const ScanTerm &Tq = P.terms[S.term0 + q];
                                    if (Tq.lds_off != kNoLds)
                                      for (uint32_t w = tid; w < Tq.bm_words; w += kThreads)
                                        lds_bm[Tq.lds_off + w] = Tq.bm[w];
                                  }
                                  __syncthreads();
                                },
                                [&] {
                                  for (uint32_t i = tid; i < P.nsegs; i += kThreads) lds_seg[i] = 0;
                                },
                                dead);
}

// ------------------------------------------------------------------------------------
// one-launch path: the whole query travels in the kernel arguments and block
// columns / dictionaries are found through the blocks' resident descriptors.
// The grid's first njobs workgroups are dictionary workgroups, one per (block,
// term): each stages that dictionary in LDS, matches every value against the
// needle and publishes the value-set bitmap as 8-byte {epoch, word} granules
// (agent-scope stores: untorn, no fences needed). The scan workgroups behind them
// poll the granules of their block's terms, then scan. Dispatch is in index
// order, so the producers are resident or done; polls are bounded.
constexpr uint32_t kFastStageWords = 6144;  // 24 KiB: one dictionary's offsets + bytes + value bits + set CSR
struct QArgs {
  const DevBlockDesc *blk[kArgSegs];
  unsigned long long cap[kArgSegs];  // records kept per block (limit mode)
  uint32_t first_wg[kArgSegs + 1];   // scan workgroup numbering (without the dictionary workgroups)
  uint32_t block_idx[kArgSegs];
  uint16_t key_of[kArgSegs][kArgTerms];
  uint16_t nd_off[kArgTerms + 1];
  alignas(16) uint8_t needles[kArgNeedle];  // (aligned: read as dwords by scalar loads)
  uint32_t nsegs, nterms, njobs, gstride;  // dictionary jobs = nsegs x nterms, granules per job
  uint32_t bm_words, stage_words;
  uint32_t mask_words;      // LDS words between the bitmaps and the block sums: tile masks / self-match stage
  uint32_t self_dict;       // 1: every scan workgroup matches its block's (small) dictionaries itself, njobs = 0
  uint32_t stage_first;     // self_dict: the dictionary words land before the first tile loads issue
  uint32_t bm_first;        // narrow: the bitmap words land before the first tile loads issue
  unsigned long long *gbm;  // njobs x gstride granules
  // narrow mode: every term column of every block is one byte wide and its dictionary
  // was matched on the host (interned canonical dictionaries): the scan columns and the
  // 256-bit value-set bitmaps travel here, so a workgroup's first tile load waits for
  // nothing but these arguments (no descriptor chain, no dictionary staging)
  uint32_t narrow;
  const uint32_t *scan[kArgSegs];   // [dur32 | start_s | end_s], npad entries each
  const uint8_t *ncol[kArgSegs];    // one-byte key columns, npad bytes per slot
  uint32_t npad[kArgSegs], nent[kArgSegs];
  uint8_t slot[kArgSegs][kArgTerms], bmi[kArgSegs][kArgTerms], nsets8[kArgSegs][kArgTerms];
  uint32_t bms[kArgBms][8];
  // segment mode work stealing: tail tiles per block and its claim counter's value at launch
  uint32_t tail[kArgSegs];  // (u32: one scalar load; u16 kernel arguments become vector loads)
  uint32_t steal_base[kArgSegs];
  ScanParams P;             // thresholds, outputs (segs/terms/wg_seg unused)
};
static_assert(sizeof(QArgs) <= 4096, "kernel arguments");

// bytes.Contains over LDS-staged bytes
__device__ __forceinline__ bool lds_contains(const uint8_t *h, uint32_t hl, const uint8_t *nd, uint32_t nl) {
  if (nl == 0) return true;  // bytes.Contains(x, "") (pitfall P7)
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

__device__ __forceinline__ DevKeyDesc key_desc(const DevBlockDesc *B, uint32_t k) {
  const auto *p = K4(reinterpret_cast<const DevKeyDesc *>(B + 1)) + k;
  DevKeyDesc r;
  r.col = p->col;
  r.dict_bytes = p->dict_bytes;
  r.dict_off = p->dict_off;
  r.set_off = p->set_off;
  r.set_vals = p->set_vals;
  r.width = p->width;
  r.nvals = p->nvals;
  r.nsets = p->nsets;
  r.identity = p->identity;
  r.dict_nbytes = p->dict_nbytes;
  r.nsetvals = p->nsetvals;
  return r;
}

// One dictionary workgroup: job j = (block s, term q).
__device__ __forceinline__ void dict_job(const QArgs &A, uint32_t j, uint32_t *stage, uint32_t *bits) {
  __shared__ __attribute__((aligned(16))) uint8_t s_nd[kArgNeedle];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t s = j / A.nterms, q = j % A.nterms;
  const DevKeyDesc K = key_desc(A.blk[s], A.key_of[s][q]);
  const uint32_t nl = A.nd_off[q + 1] - A.nd_off[q];
  for (uint32_t i = tid; i < nl; i += kThreads) s_nd[i] = A.needles[A.nd_off[q] + i];
  // stage: off[nvals+1] | bytes (whole words) | [set_off nsets+1 | set_vals]; value bits in `bits`
  const uint32_t bw = (K.dict_nbytes + 3) / 4;
  uint32_t *off = stage, *by = stage + K.nvals + 1, *soff = by + bw, *svals = soff + K.nsets + 1;
  for (uint32_t i = tid; i <= K.nvals; i += kThreads) off[i] = G(K.dict_off)[i];
  for (uint32_t i = tid; i < bw; i += kThreads) by[i] = G(reinterpret_cast<const uint32_t *>(K.dict_bytes))[i];
  if (!K.identity) {
    for (uint32_t i = tid; i <= K.nsets; i += kThreads) soff[i] = G(K.set_off)[i];
    for (uint32_t i = tid; i < K.nsetvals; i += kThreads) svals[i] = G(K.set_vals)[i];
  }
  __syncthreads();
  const uint8_t *b8 = reinterpret_cast<const uint8_t *>(by);
  for (uint32_t v0 = 0; v0 < K.nvals; v0 += kThreads) {
    const uint32_t v = v0 + tid;
    bool m = false;
    if (v < K.nvals) m = lds_contains(b8 + off[v], off[v + 1] - off[v], s_nd, nl);
    const unsigned long long b = __ballot(m);
    const uint32_t w0 = (v - lane) >> 5;
    if (lane == 0 && w0 * 32 < K.nvals) bits[w0] = uint32_t(b);
    if (lane == 32 && (w0 + 1) * 32 < K.nvals) bits[w0 + 1] = uint32_t(b >> 32);
  }
  __syncthreads();
  const uint32_t words = (K.nsets + 31) / 32;
  const unsigned long long tag = (unsigned long long)A.P.epoch << 32;
  unsigned long long *g = A.gbm + uint64_t(j) * A.gstride;
  if (K.identity) {  // value set == value
    for (uint32_t w = tid; w < words; w += kThreads)
      __hip_atomic_store(&g[w], tag | bits[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {  // a set matches iff one of its values does
    for (uint32_t s0 = 0; s0 < K.nsets; s0 += kThreads) {
      const uint32_t sid = s0 + tid;
      bool m = false;
      if (sid < K.nsets)
        for (uint32_t i = soff[sid]; i < soff[sid + 1] && !m; i++) m = (bits[svals[i] >> 5] >> (svals[i] & 31)) & 1u;
      const unsigned long long b = __ballot(m);
      const uint32_t w0 = (sid - lane) >> 5;
      if (lane == 0 && w0 < words) __hip_atomic_store(&g[w0], tag | uint32_t(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 32 && w0 + 1 < words)
        __hip_atomic_store(&g[w0 + 1], tag | uint32_t(b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Small dictionaries (every term's blob of the block fits kSelfWords in all): the
// scan workgroup matches them itself, straight into its LDS bitmaps, with no
// cross-workgroup wait. Same per-value test and set rule as dict_job.
// The staging loads go into registers (kSelfPer words per thread, no loop) and are
// issued BEFORE the first tile's loads: vmcnt retires loads in order, so waiting
// for the dictionary words does not wait for the tile stream behind them.
constexpr uint32_t kSelfWords = 4096;
constexpr int kSelfPer = int(kSelfWords / kThreads);
template <int NTA>
struct SelfStage {
  const uint32_t *src[NTA];  // key blobs [off | bytes | set_off | set_vals]
  uint32_t cum[NTA + 1];     // blob word prefix over the terms
  uint32_t base[NTA];        // LDS word offset of each term's staged blob (+ value bits after it)
  uint32_t nvals[NTA], nsets[NTA], bw[NTA], identity[NTA];
  uint32_t w[kSelfPer];
};

template <int NTA>
__device__ __forceinline__ void self_issue(SelfStage<NTA> &X, const DevKeyDesc *KD) {
  const int tid = threadIdx.x;
  uint32_t c = 0, o = 0;
#pragma unroll
  for (int q = 0; q < NTA; q++) {  // (one-launch kernels: NTA == nterms)
    const DevKeyDesc &K = KD[q];
    X.cum[q] = c;
    X.base[q] = o;
    X.src[q] = K.dict_off;
    X.nvals[q] = K.nvals;
    X.nsets[q] = K.nsets;
    X.identity[q] = K.identity;
    X.bw[q] = (K.dict_nbytes + 3) / 4;
    const uint32_t words = K.nvals + 1 + X.bw[q] + (K.identity ? 0u : K.nsets + 1 + K.nsetvals);
    c += words;
    o += words + (K.identity ? 0u : (K.nvals + 63) / 32);  // + value bits of a non-identity key
  }
  X.cum[NTA] = c;
  // lanes past the staged total skip their load (every workgroup of the block
  // reads the same few lines: redundant requests queue on one L2 channel)
#pragma unroll
  for (int r = 0; r < kSelfPer; r++) {
    const uint32_t i = uint32_t(tid) + uint32_t(r) * kThreads;
    if (i >= c) continue;
    const uint32_t *src = X.src[0];
    uint32_t cq = 0;
#pragma unroll
    for (int q2 = 1; q2 < NTA; q2++)
      if (i >= X.cum[q2]) {
        src = X.src[q2];
        cq = X.cum[q2];
      }
    X.w[r] = G(src)[i - cq];
  }
}

template <int NTA>
__device__ __forceinline__ void self_finish(SelfStage<NTA> &X, const QArgs &A, const ScanTerm *T, uint32_t *lds_bm,
                                            uint32_t *scratch, uint32_t wg) {
  __shared__ __attribute__((aligned(16))) uint32_t s_nd2w[kArgNeedle / 4];
  const uint8_t *s_nd2 = reinterpret_cast<const uint8_t *>(s_nd2w);
  const int tid = threadIdx.x, lane = tid & 63;
  // needles: uniform loop, scalar kernel-argument loads (lgkmcnt, not behind the
  // tile loads in the vmcnt queue)
  if (tid == 0) {
    const uint32_t nw = (uint32_t(A.nd_off[NTA]) + 3) / 4;
#pragma clang loop vectorize(disable) unroll(disable)
    for (uint32_t w = 0; w < nw; w++) s_nd2w[w] = reinterpret_cast<const uint32_t *>(A.needles)[w];
  }
#pragma unroll
  for (int r = 0; r < kSelfPer; r++) {
    const uint32_t i = uint32_t(tid) + uint32_t(r) * kThreads;
    if (i < X.cum[NTA]) {
      uint32_t dst = X.base[0] + i - X.cum[0];
#pragma unroll
      for (int q2 = 1; q2 < NTA; q2++)
        if (i >= X.cum[q2]) dst = X.base[q2] + i - X.cum[q2];
      scratch[dst] = X.w[r];
    }
  }
  __syncthreads();
  if (A.P.stamps && tid == 0)  // TSG_STAMPS slot 7: dictionary words in LDS
    A.P.stamps[uint64_t(wg) * kStampSlots + 7] = __builtin_amdgcn_s_memrealtime();
  bool sets = false;
#pragma unroll
  for (int q = 0; q < NTA; q++) {
    {
      const uint32_t *off = scratch + X.base[q];
      const uint8_t *b8 = reinterpret_cast<const uint8_t *>(off + X.nvals[q] + 1);
      const uint8_t *nd = s_nd2 + A.nd_off[q];
      const uint32_t nl = A.nd_off[q + 1] - A.nd_off[q];
      // value set == value: straight into the term bitmap; else value bits after the blob
      uint32_t *bits = X.identity[q] ? lds_bm + T[q].lds_off : scratch + X.base[q] + (X.cum[q + 1] - X.cum[q]);
      sets |= !X.identity[q];
      for (uint32_t v0 = 0; v0 < X.nvals[q]; v0 += kThreads) {
        const uint32_t v = v0 + tid;
        bool m = false;
        if (v < X.nvals[q]) m = lds_contains(b8 + off[v], off[v + 1] - off[v], nd, nl);
        const unsigned long long b = __ballot(m);
        const uint32_t w0 = (v - lane) >> 5;
        if (lane == 0 && w0 * 32 < X.nvals[q]) bits[w0] = uint32_t(b);
        if (lane == 32 && (w0 + 1) * 32 < X.nvals[q]) bits[w0 + 1] = uint32_t(b >> 32);
      }
    }
  }
  __syncthreads();
  if (!sets) return;
#pragma unroll
  for (int q = 0; q < NTA; q++) {  // a set matches iff one of its values does
    if (!X.identity[q]) {
      const uint32_t *soff = scratch + X.base[q] + X.nvals[q] + 1 + X.bw[q];
      const uint32_t *svals = soff + X.nsets[q] + 1;
      const uint32_t *vbits = scratch + X.base[q] + (X.cum[q + 1] - X.cum[q]);
      for (uint32_t s0 = 0; s0 < X.nsets[q]; s0 += kThreads) {
        const uint32_t sid = s0 + tid;
        bool m = false;
        if (sid < X.nsets[q])
          for (uint32_t i = soff[sid]; i < soff[sid + 1] && !m; i++) m = (vbits[svals[i] >> 5] >> (svals[i] & 31)) & 1u;
        const unsigned long long b = __ballot(m);
        const uint32_t w0 = (sid - lane) >> 5;
        if (lane == 0 && w0 * 32 < X.nsets[q]) lds_bm[T[q].lds_off + w0] = uint32_t(b);
        if (lane == 32 && (w0 + 1) * 32 < X.nsets[q]) lds_bm[T[q].lds_off + w0 + 1] = uint32_t(b >> 32);
      }
    }
  }
  __syncthreads();
}

// Leading scalar arguments: the first kernel-argument dwords are preloaded into SGPRs at
// wave launch (-mllvm -amdgpu-kernarg-preload-count, gfx950; firmware without preload
// runs the compiler's compatibility prologue instead). With a uniform block split
// (kPreUniform) a workgroup finds its block from these alone, so its first memory round
// trip already fetches the block's arguments.
enum : uint32_t { kPreTicket = 1, kPreNarrow = 2, kPreBmFirst = 4, kPreSelf = 8, kPreUniform = 16, kPreStamps = 32 };
template <int NT, bool DUR, bool RANGE, bool W1, bool SEG>
__global__ void __launch_bounds__(kThreads, 3)
    search_fast_kernel(uint32_t k_flags, uint32_t k_nsegs, uint32_t k_njobs, uint32_t k_wgs, uint32_t k_half,
                       uint32_t k_bm_words, uint32_t k_mask_words, uint32_t k_nterms,
                       unsigned long long *k_stamps, QArgs A) {
  // (stamps only: s_memrealtime is a scalar memory operation)
  const unsigned long long t_start = k_stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  // Every kernel argument the prologue branches on arrives in ONE round trip: scalar
  // loads return out of order, so each s_waitcnt lgkmcnt waits for every load issued,
  // and loads issued behind a branch would each add a round trip before the first tile
  // load (the empty asm statements pin them all in front of the first use)
  const uint32_t use_ticket = k_flags & kPreTicket, njobs = k_njobs, nsegs = k_nsegs,
                 narrow_arg = k_flags & kPreNarrow, bm_words = k_bm_words, mask_words = k_mask_words,
                 nterms = k_nterms, bm_first = k_flags & kPreBmFirst, self_dict = k_flags & kPreSelf;
  unsigned long long *const stamps = k_stamps;
  const uint32_t vb = wg_order(A.P, use_ticket != 0);  // (a ticket when dictionary or look-back waits exist)
  if (vb < njobs) {  // dictionary workgroup: [value bits | stage]
    dict_job(A, vb, lds + bm_words, lds);
    return;
  }
  // scan workgroup: [bitmaps bm_words | kLdsTiles masks | seg sums nsegs | first_wg nsegs+1 | caps]
  uint32_t *lds_bm = lds;
  uint16_t *lds_mask = reinterpret_cast<uint16_t *>(lds + bm_words);
  uint32_t *lds_seg = lds + bm_words + mask_words;
  uint32_t *lds_fw = lds_seg + ((nsegs + 1) & ~1u);  // (even: lds_cap below is 8-byte aligned)
  unsigned long long *lds_cap = reinterpret_cast<unsigned long long *>(lds_fw + ((nsegs + 2) & ~1u));
  unsigned long long *lds_rec = lds_cap + nsegs;  // segment mode: kSegMax staged records
  const int tid = threadIdx.x;
  const uint32_t wg = vb - njobs;
  uint32_t si = 0;
  if (k_flags & kPreUniform) {
    // first_wg[s] = (k_wgs * s + k_half) / nsegs: the block whose range holds wg
    si = min(nsegs - 1, ((wg + 1) * nsegs - k_half - 1) / k_wgs);
  } else {
    uint32_t fw[kArgSegs];
#pragma unroll
    for (int s2 = 0; s2 < kArgSegs; s2++) fw[s2] = A.first_wg[s2];
#pragma unroll
    for (int s2 = 0; s2 < kArgSegs; s2++) asm volatile("" : "+s"(fw[s2]));
#pragma unroll
    for (int s2 = 1; s2 < kArgSegs; s2++) si += (uint32_t(s2) < nsegs && fw[s2] <= wg) ? 1u : 0u;
  }
  // wave-uniform: descriptor reads become scalar loads (one round trip, not vmcnt-serialised)
  si = __builtin_amdgcn_readfirstlane(si);
  const DevBlockDesc *B = A.blk[si];
  constexpr int NTA = NT > 0 ? NT : 1;
  const bool narrow = narrow_arg != 0;
  // narrow mode: this block's scan arguments, again in one round trip
  const uint32_t *n_scan = A.scan[si];
  const uint8_t *n_col = A.ncol[si];
  uint32_t n_npad = A.npad[si], n_ent = A.nent[si];
  // (the per-term bytes as raw dwords, and one pin for everything: the compiler then
  // issues every load before a single wait instead of unpacking between batches)
  static_assert(kArgTerms == 4, "slot/bmi/nsets8 rows are one dword");
  uint32_t r_slot = *reinterpret_cast<const uint32_t *>(A.slot[si]);
  uint32_t r_sets = *reinterpret_cast<const uint32_t *>(A.nsets8[si]);
  uint32_t r_bmi = *reinterpret_cast<const uint32_t *>(A.bmi[si]);
  // the rest of this block's arguments, in the same round trip
  uint32_t b_fw0 = A.first_wg[si], b_fw1 = A.first_wg[si + 1], b_idx = A.block_idx[si], b_tail = A.tail[si],
           b_sbase = A.steal_base[si];
  unsigned long long b_cap = A.cap[si];
  asm volatile(""
               : "+s"(n_scan), "+s"(n_col), "+s"(n_npad), "+s"(n_ent), "+s"(r_slot), "+s"(r_sets), "+s"(r_bmi),
                 "+s"(b_fw0), "+s"(b_fw1), "+s"(b_idx), "+s"(b_tail), "+s"(b_sbase), "+s"(b_cap), "+s"(B));
  uint32_t n_slot[NTA], n_sets[NTA], n_bmi[NTA];
#pragma unroll
  for (int q = 0; q < NTA; q++) {
    n_slot[q] = (r_slot >> (8 * q)) & 0xffu;
    n_sets[q] = (r_sets >> (8 * q)) & 0xffu;
    n_bmi[q] = (r_bmi >> (8 * q)) & 0xffu;
  }
  // narrow: the query's bitmap words for this block's terms, requested now (before the
  // tile burst: issued behind it, the scalar round trip queues behind ~30 MB of tile
  // loads chip-wide and gates the first evaluation by ~10 us)
  uint32_t bw[NTA][8];
  if (NT > 0 && narrow_arg) {
#pragma unroll
    for (int q = 0; q < NTA; q++)
#pragma unroll
      for (int w = 0; w < 8; w++) bw[q][w] = A.bms[n_bmi[q]][w];
    if (bm_first) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  DevKeyDesc KD[NTA];  // scalar loads, all issued together (one-launch kernels: NT == nterms)
  if (NT > 0 && !narrow)
#pragma unroll
    for (int q = 0; q < NTA; q++) KD[q] = key_desc(B, A.key_of[si][q]);
  ScanSeg S;
  // the record columns (ids, times, names) are read only to emit matches; in narrow mode
  // their descriptor loads are issued after the scan: scalar loads complete out of order,
  // so any earlier use of a kernel argument would wait for them (s_waitcnt lgkmcnt(0))
  auto cold = [&](const DevBlockDesc *Bd) {
    const auto *Bc = K4(Bd);
    S.dur64 = Bc->dur64;
    S.ids = Bc->ids;
    S.start_ns = Bc->start_ns;
    S.end_ns = Bc->end_ns;
    S.names = Bc->names;
    S.id_len = Bc->id_len;
  };
  if (narrow) {
    S.n = n_ent;
    S.dur32 = n_scan;
    S.start_s = n_scan + n_npad;
    S.end_s = n_scan + 2ull * n_npad;
    S.dur64 = nullptr;  // (narrow mode: no threshold >= 2^32-1 ns)
    S.ids = nullptr;
    S.start_ns = S.end_ns = nullptr;
    S.names = nullptr;
    S.id_len = nullptr;
  } else {
    const auto *Bc = K4(B);
    S.n = Bc->n;
    S.dur32 = Bc->dur32;
    S.start_s = Bc->start_s;
    S.end_s = Bc->end_s;
    cold(B);
  }
  S.nunits = uint32_t((S.n + kUnit - 1) / kUnit);
  S.first_wg = b_fw0;
  S.nwg = b_fw1 - b_fw0;  // (first_wg[nsegs] = the grid's scan workgroups)
  S.tpw = 0;
  S.term0 = 0;
  S.nterms = nterms;
  S.lds_words = bm_words;
  S.block_idx = b_idx;
  S.cap = b_cap;
  S.tail = SEG ? b_tail : 0u;
  S.steal_base = b_sbase;
  ScanTerm T[NTA];
  uint32_t gw[NTA + 1];  // granule prefix over this block's terms
  gw[0] = 0;
  uint32_t bmo = 0;
#pragma unroll
  for (int q = 0; q < NTA; q++) {
    if (NT <= 0) break;
    const DevKeyDesc &K = KD[q];
    if (narrow) {
      T[q].col = n_col + uint64_t(n_slot[q]) * n_npad;
      T[q].width = 1;
      T[q].nsets = n_sets[q];
    } else {
      T[q].col = K.col;
      T[q].width = K.width;
      T[q].nsets = K.nsets;
    }
    T[q].bm = nullptr;
    T[q].lds_off = bmo;
    T[q].bm_words = (K.nsets + 31) / 32;
    bmo += W1 ? 8u : T[q].bm_words;
    gw[q + 1] = gw[q] + T[q].bm_words;
  }
  // bitmaps: poll this block's granules (one per thread) into LDS, after the first
  // tile's loads are in flight
  SelfStage<NTA> X;
  auto issue_stage = [&] {
    if (stamps && threadIdx.x == 0)  // (waits for the descriptor scalar loads: lgkmcnt)
      stamps[uint64_t(wg) * kStampSlots + 5] = __builtin_amdgcn_s_memrealtime();
    if (NT > 0 && self_dict) {
      self_issue<NTA>(X, KD);
      // stage_first: wait for the (few, L2-shared) dictionary words before this
      // workgroup's tile stream is issued. Issued together, they queue behind every
      // CU's opening burst of tile loads (~60 MB chip-wide) and gate the scan for
      // ~10 us; alone they land in ~1-2 us and the matching then hides under the tiles.
      if (A.stage_first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (stamps && threadIdx.x == 0)
      stamps[uint64_t(wg) * kStampSlots + 6] = __builtin_amdgcn_s_memrealtime();
  };
  auto wait_bitmaps = [&] {
    if (narrow) {  // the host's bitmaps, from the kernel arguments (loaded in the prologue)
      if (NT > 0 && tid == 0)
#pragma unroll
        for (int q = 0; q < NTA; q++)
#pragma unroll
          for (int w = 0; w < 8; w++) lds_bm[T[q].lds_off + w] = bw[q][w];
      __syncthreads();
      return;
    }
    if (NT > 0 && self_dict) {  // (self_finish ends with a barrier)
      self_finish<NTA>(X, A, T, lds_bm, lds + bm_words, wg);
      return;
    }
    if (NT > 0) {
      const unsigned long long tag = (unsigned long long)A.P.epoch << 32;
      for (uint32_t i = tid; i < gw[nterms]; i += kThreads) {
        uint32_t q = 0;
#pragma unroll
        for (int q2 = 1; q2 < NTA; q2++)
          if (i >= gw[q2]) q = q2;
        const unsigned long long *g = A.gbm + uint64_t(si * nterms + q) * A.gstride + (i - gw[q]);
        unsigned long long v;
        uint32_t spins = 0;
        while (((v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & ~0xffffffffull) != tag) {
          if (++spins > kSpinMax) {
            reinterpret_cast<volatile unsigned long long *>(A.P.out)[1] = 1;  // host fails the query
            break;
          }
          __builtin_amdgcn_s_sleep(4);
        }
        uint32_t lo = 0;
#pragma unroll
        for (int q2 = 0; q2 < NTA; q2++)
          if (q2 == int(q)) lo = T[q2].lds_off;
        lds_bm[lo + (i - gw[q])] = uint32_t(v);
      }
    }
    __syncthreads();
  };
  scan_emit<NT, DUR, RANGE, W1, SEG>(A.P, S, T, si, ArgSegs{lds_fw, lds_cap, nsegs}, lds_bm, lds_mask, lds_seg,
                                     lds_rec, t_start, stamps, wg, issue_stage, wait_bitmaps, [&] {
                                       if (narrow) {  // (the asm keeps the loads below the scan loop)
                                         const DevBlockDesc *Bd = B;
                                         asm volatile("" : "+s"(Bd));
                                         cold(Bd);
                                       }
                                       if constexpr (!SEG) {
                                         for (uint32_t i = tid; i < nsegs; i += kThreads) {
                                           lds_seg[i] = 0;
                                           lds_fw[i] = A.first_wg[i];
                                           lds_cap[i] = A.cap[i];
                                         }
                                         if (tid == 0) lds_fw[nsegs] = A.first_wg[nsegs];
                                       }
                                     });
  // completion: the last scan workgroup raises the flag the host polls (header word 2 =
  // epoch). Arrivals are counted per XCD group (blockIdx % 8: a group label, speed
  // only) and the last of each group arrives at the top counter, so no single word
  // takes a thousand atomics at the end of the launch. Every workgroup's record and
  // count stores (system-scope write-through) have completed before it arrives.
  if (!A.P.flag_done) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t g = vb & 7u;
    // (relaxed: the only data behind the flag is host memory written through at system
    // scope, already complete; an acquire/release here would write back / invalidate L2)
    const unsigned prev = __hip_atomic_fetch_add(A.P.done + 32 * g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1u == A.P.done_target[g]) {
      const unsigned top = __hip_atomic_fetch_add(A.P.done + 32 * 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (top + 1u == A.P.done_top) {
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(A.P.out) + 2, (unsigned long long)A.P.epoch,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// host

using ScanFn = void (*)(ScanParams);
using FastFn = void (*)(uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                        unsigned long long *, QArgs);
template <int NT, bool W1, bool SEG>
static FastFn pick3_fast(bool dur, bool range) {
  if (dur && range) return search_fast_kernel<NT, true, true, W1, SEG>;
  if (dur) return search_fast_kernel<NT, true, false, W1, SEG>;
  if (range) return search_fast_kernel<NT, false, true, W1, SEG>;
  return search_fast_kernel<NT, false, false, W1, SEG>;
}
template <bool SEG>
static FastFn pick_fast_t(uint32_t nterms, bool dur, bool range, bool w1) {
  switch (nterms) {
    case 0: return pick3_fast<0, false, SEG>(dur, range);
    case 1: return w1 ? pick3_fast<1, true, SEG>(dur, range) : pick3_fast<1, false, SEG>(dur, range);
    case 2: return w1 ? pick3_fast<2, true, SEG>(dur, range) : pick3_fast<2, false, SEG>(dur, range);
    case 3: return w1 ? pick3_fast<3, true, SEG>(dur, range) : pick3_fast<3, false, SEG>(dur, range);
    default: return w1 ? pick3_fast<4, true, SEG>(dur, range) : pick3_fast<4, false, SEG>(dur, range);
  }
}
// seg: segment-mode kernel (dynamic tiles, per-tile segments) vs look-back mode
static FastFn pick_fast(uint32_t nterms, bool dur, bool range, bool w1, bool seg) {
  return seg ? pick_fast_t<true>(nterms, dur, range, w1) : pick_fast_t<false>(nterms, dur, range, w1);
}
template <int NT, bool W1>
static ScanFn pick3(bool dur, bool range) {
  if (dur && range) return search_kernel<NT, true, true, W1>;
  if (dur) return search_kernel<NT, true, false, W1>;
  if (range) return search_kernel<NT, false, true, W1>;
  return search_kernel<NT, false, false, W1>;
}
// w1: every term column of every block in this launch is one byte wide
static ScanFn pick_scan(uint32_t nterms, bool dur, bool range, bool w1) {
  switch (nterms) {
    case 0: return pick3<0, false>(dur, range);
    case 1: return w1 ? pick3<1, true>(dur, range) : pick3<1, false>(dur, range);
    case 2: return w1 ? pick3<2, true>(dur, range) : pick3<2, false>(dur, range);
    case 3: return w1 ? pick3<3, true>(dur, range) : pick3<3, false>(dur, range);
    case 4: return w1 ? pick3<4, true>(dur, range) : pick3<4, false>(dur, range);
    default: return pick3<-1, false>(dur, range);
  }
}


// TSG_STAMPS: where a launch's time goes (us from the first workgroup start; 100 MHz clock)
void print_stamps(DeviceCtx &dc, uint32_t nwg, bool fast) {
  std::vector<unsigned long long> st(size_t(nwg) * kStampSlots);
  HIP_OK(hipMemcpy(st.data(), dc.stamps.p, st.size() * 8, hipMemcpyDeviceToHost));
  unsigned long long t0 = ~0ull;
  for (uint32_t w = 0; w < nwg; w++) t0 = std::min(t0, st[size_t(w) * kStampSlots]);
  const char *names[8] = {"start", "setup", "scan", "lookback", "end", "desc", "staged", "inlds"};
  if (const char *f = std::getenv("TSG_STAMPS_FILE")) {  // raw rows: wg, 8 stamps (us), xcc, se, sh, cu
    static int launch = 0;
    if (FILE *o = std::fopen(f, "a")) {
      for (uint32_t w = 0; w < nwg; w++) {
        std::fprintf(o, "%d,%u", launch, w);
        for (int k = 0; k < 8; k++) {
          const unsigned long long x = st[size_t(w) * kStampSlots + k];
          std::fprintf(o, ",%.2f", x ? double(x - t0) / 100.0 : -1.0);
        }
        const unsigned long long hw = st[size_t(w) * kStampSlots + 8];
        std::fprintf(o, ",%llu,%llu,%llu,%llu\n", hw >> 32, (hw >> 13) & 3, (hw >> 12) & 1, (hw >> 8) & 15);
      }
      std::fclose(o);
    }
    launch++;
  }
  std::fprintf(stderr, "[tsg] stamps (%s, %u wg) us avg/max:", fast ? "one-launch" : "general", nwg);
  for (int k = 0; k < 8; k++) {
    double sum = 0, mx = 0;
    for (uint32_t w = 0; w < nwg; w++) {
      const unsigned long long x = st[size_t(w) * kStampSlots + k];
      const double v = x ? double(x - t0) / 100.0 : 0.0;  // (unwritten slot: 0)
      sum += v;
      mx = std::max(mx, v);
    }
    std::fprintf(stderr, " %s=%.1f/%.1f", names[k], sum / nwg, mx);
  }
  std::fprintf(stderr, "\n");
  // spread of the scan ends: percentiles, and per XCD group (workgroup index % 8)
  std::vector<double> se(nwg), su(nwg);
  double gsum[8] = {}, gmax[8] = {};
  uint32_t gn[8] = {};
  for (uint32_t w = 0; w < nwg; w++) {
    se[w] = double(st[size_t(w) * kStampSlots + 2] - t0) / 100.0;
    su[w] = double(st[size_t(w) * kStampSlots + 1] - t0) / 100.0;
    gsum[w & 7] += se[w];
    gmax[w & 7] = std::max(gmax[w & 7], se[w]);
    gn[w & 7]++;
  }
  std::sort(se.begin(), se.end());
  std::sort(su.begin(), su.end());
  auto pct = [&](const std::vector<double> &v, double p) { return v[std::min(v.size() - 1, size_t(p * v.size()))]; };
  std::fprintf(stderr, "[tsg] stamps scan-end p10/p50/p90/p99 %.1f/%.1f/%.1f/%.1f setup p50/p90 %.1f/%.1f | group avg/max:",
               pct(se, 0.1), pct(se, 0.5), pct(se, 0.9), pct(se, 0.99), pct(su, 0.5), pct(su, 0.9));
  for (int g = 0; g < 8; g++) std::fprintf(stderr, " %.1f/%.1f", gn[g] ? gsum[g] / gn[g] : 0.0, gmax[g]);
  std::fprintf(stderr, "\n");
}



// A limit wave's part of a block: the records of scan positions outside its range (paths that
// scan the block from position 0 or to its end) are dropped; the others keep their order.
static void drop_before_ranges(const std::vector<std::pair<uint32_t, Block *>> &blocks, const EntryRanges &ranges,
                               SearchOut &out) {
  thread_local std::vector<uint64_t> lo, hi;
  uint32_t mx = 0;
  for (const auto &bp : blocks) mx = std::max(mx, bp.first);
  lo.assign(size_t(mx) + 1, 0);
  hi.assign(size_t(mx) + 1, UINT64_MAX);
  for (size_t i = 0; i < blocks.size(); i++) {
    lo[blocks[i].first] = ranges[i].first;
    hi[blocks[i].first] = ranges[i].second;
  }
  size_t k = 0;
  for (size_t r = 0; r < out.recs.size(); r++) {
    const uint32_t bi = out.recs[r].block_il & 0xffffffu;
    if (out.recs[r].entry >= lo[bi] && out.recs[r].entry < hi[bi]) out.recs[k++] = out.recs[r];
  }
  out.recs.resize(k);
}

// out.recs sized to n records (not initialised); new storage of a large record array is
// advised huge pages before the copy touches it
static void grow_recs(SearchOut &out, size_t n) {
  const size_t cap0 = out.recs.capacity();
  out.recs.resize(n);
  if (out.recs.capacity() != cap0) advise_huge(out.recs.data(), out.recs.capacity() * sizeof(SearchOut::Rec));
}

// positions (entry | block index << 32) -> records from each block's host columns (the same
// values the device columns hold), on several threads
static void positions_to_recs(const std::vector<std::pair<uint32_t, Block *>> &blocks, const uint64_t *pos,
                              uint64_t total, SearchOut &out) {
  uint32_t max_idx = 0;
  for (const auto &bp : blocks) max_idx = std::max(max_idx, bp.first);
  std::vector<const HostBlock *> hb(size_t(max_idx) + 1, nullptr);
  for (const auto &bp : blocks) hb[bp.first] = bp.second->host.get();
  std::atomic<bool> bad{false};
  parallel_ranges(size_t(total), size_t(1) << 16, 16, [&](size_t lo, size_t hi) {
    for (size_t r = lo; r < hi; r++) {
      const uint64_t x = pos[r];
      const uint32_t e = uint32_t(x), bi = uint32_t(x >> 32);
      const HostBlock *hp = bi <= max_idx ? hb[bi] : nullptr;
      if (!hp || e >= hp->start.size() || uint64_t(e) * 16 + 16 > hp->ids.size()) {
        bad.store(true, std::memory_order_relaxed);
        return;
      }
      const HostBlock &h = *hp;
      SearchOut::Rec &o = out.recs[r];
      std::memcpy(o.id, h.ids.data() + uint64_t(e) * 16, 16);
      o.start = h.start[e];
      o.end = h.end[e];
      o.entry = e;
      o.block_il = bi | (uint32_t(h.id_len[e]) << 24);
      o.svc = h.svc_vid.empty() ? kNone : h.svc_vid[e];
      o.name = h.name_vid.empty() ? kNone : h.name_vid[e];
    }
  });
  if (bad.load()) fail(TSG_E_DEVICE, "look-back position outside its block's host columns");
}

void device_search(DeviceCtx &dc, const std::vector<std::pair<uint32_t, Block *>> &blocks, const tsg_query &q,
                   uint32_t limit, uint32_t flags, SearchOut &out, const EntryRanges *ranges) {
  Tracer tr;
  out.compact = false;
  out.pos.clear();
  out.resident = false;
  out.path = 0;
  // (a resident-kernel query releases dc.mu while it runs: other callers post theirs meanwhile)
  std::unique_lock<std::mutex> lk(dc.mu);
  HIP_OK(hipSetDevice(dc.ordinal));
  hipStream_t s = dc.stream;
  if (dc.dev_cu == 0) {
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, dc.ordinal));
    dc.dev_cu = prop.multiProcessorCount;
  }
  dc.num_cu = debug_groups() ? int(debug_groups()) : dc.dev_cu;

  // ---- plan (scratch vectors kept per thread: no allocation per query once warm)
  struct PlanScratch {
    std::vector<ScanSeg> segs;
    std::vector<ScanTerm> terms;
    std::vector<DictJob> jobs;
    std::vector<uint32_t> set_jobs, set_items, term_bm_base, needle_off;
    std::vector<uint8_t> needles;
    std::vector<StreamJob> stream_jobs;
    std::vector<std::array<uint16_t, kArgTerms>> seg_keys;
    std::vector<const DevBlockDesc *> seg_desc;
    std::vector<NarrowSeg> nsegv;
    std::vector<int> kidx;
    std::string key;
  };
  thread_local PlanScratch ps;
  auto &segs = ps.segs;
  auto &terms = ps.terms;
  auto &jobs = ps.jobs;
  auto &set_jobs = ps.set_jobs, &set_items = ps.set_items, &term_bm_base = ps.term_bm_base;
  auto &needles = ps.needles;
  auto &needle_off = ps.needle_off;
  segs.clear();
  terms.clear();
  jobs.clear();
  set_jobs.clear();
  set_items.assign(1, 0);
  term_bm_base.clear();
  needles.clear();
  auto &stream_jobs = ps.stream_jobs;
  stream_jobs.clear();
  uint32_t stream_waves = 0, stream_span = kStreamSpan;
  needle_off.assign(q.nterms, 0);
  for (uint32_t t = 0; t < q.nterms; t++) {
    needle_off[t] = uint32_t(needles.size());
    needles.insert(needles.end(), q.values[t], q.values[t] + q.value_lens[t]);
  }
  const bool has_dur = q.has_min || q.has_max;
  uint32_t vmatch_total = 0, bm_total = 0, items = 0, units = 0, max_lds_words = 0;
  uint64_t dict_bytes = 0, scan_bytes = 0, n_all = 0;
  bool all_w1 = true;
  constexpr uint32_t kLdsBudgetWords = 8192;  // 32 KiB per workgroup
  // one-launch path bookkeeping: per block key indices and LDS words its
  // workgroups need to match the dictionaries themselves
  auto &seg_keys = ps.seg_keys;
  auto &seg_desc = ps.seg_desc;
  auto &nsegv = ps.nsegv;
  seg_keys.clear();
  seg_desc.clear();
  nsegv.clear();
  bool all_narrow = q.nterms <= uint32_t(kArgTerms);
  uint32_t fast_stage = 0, fast_bm = 0, fast_bm8 = 0, fast_vbits = 0, fast_words = 1, fast_self = 0;
  for (size_t bi_ = 0; bi_ < blocks.size(); bi_++) {
    const auto &bp = blocks[bi_];
    Block &b = *bp.second;
    const DevBlock &d = b.dev;
    // the scanned range [e0, e1): a whole block, or a limit wave's part of it (e0 on a
    // 512-entry boundary: the pool kernels' unit; other paths scan from 0 and the records
    // before e0 are dropped below)
    uint64_t e0 = 0, e1 = d.n;
    if (ranges) {
      e1 = std::min<uint64_t>((*ranges)[bi_].second, d.n);
      e0 = std::min<uint64_t>((*ranges)[bi_].first, e1) / 512 * 512;
    }
    if (e1 <= e0 || q.exhaustive) continue;
    auto &kidx = ps.kidx;
    kidx.assign(q.nterms, 0);
    bool dead = false;  // a key absent from the block: FindTag fails for every entry
    for (uint32_t t = 0; t < q.nterms && !dead; t++) {
      ps.key.assign(reinterpret_cast<const char *>(q.keys[t]), q.key_lens[t]);
      auto it = b.host->key_index.find(ps.key);
      if (it == b.host->key_index.end()) dead = true;
      else kidx[t] = it->second;
    }
    if (dead) continue;
    ScanSeg sg{};
    sg.n = e1;
    sg.e0 = e0;
    sg.dur32 = d.dur32;
    sg.dur64 = d.dur64;
    sg.start_s = d.start_s;
    sg.end_s = d.end_s;
    sg.ids = d.ids;
    sg.start_ns = d.start_ns;
    sg.end_ns = d.end_ns;
    sg.names = d.names;
    sg.id_len = d.id_len;
    sg.block_idx = bp.first;
    sg.term0 = uint32_t(terms.size());
    sg.nterms = q.nterms;
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
      jb.item_base = items;
      // a large dictionary of values >= 16 B on average: one byte-stream pass
      // (dict_stream_kernel) instead of a lane per value
      const bool stream = dc.dict_stream && k.dict_nbytes > kStreamMinBytes && q.value_lens[t] >= 2 &&
                          q.value_lens[t] <= kStreamMaxNeedle && k.dict_nbytes >= 16ull * k.nvals;
      if (!stream) items += uint32_t(align_up(std::max<uint32_t>(k.nvals, 1), 64));
      const uint32_t words = (k.nsets + 31) / 32;
      bm_total += words + 2;  // +2: a wave's ballot writes whole 64-value word pairs
      if (stream) {
        // match bytes 32-aligned (dict_sets_kernel packs identity words from 32 of them)
        vmatch_total = uint32_t(align_up(vmatch_total, 32));
        jb.vmatch_base = vmatch_total;
        vmatch_total += uint32_t(align_up(k.nvals, 32));
        set_jobs.push_back(uint32_t(jobs.size()));
        set_items.push_back(set_items.back() + words);
        StreamJob sj{};
        sj.lead = uint32_t(reinterpret_cast<uintptr_t>(k.dict_bytes) & 15u);
        sj.base = k.dict_bytes - sj.lead;
        sj.off = k.dict_off;
        sj.nbytes = k.dict_nbytes;
        sj.nvals = k.nvals;
        sj.needle_off = needle_off[t];
        sj.needle_len = q.value_lens[t];
        sj.vmatch_base = jb.vmatch_base;
        // the second byte pair tested in registers: the needle's rarest in the key's values
        // (sampled at open), else its last pair within reach
        if (q.value_lens[t] >= 4) {
          const uint8_t *nd = q.values[t];
          const uint32_t hi = std::min<uint32_t>(q.value_lens[t] - 2, kStreamPairMax);
          const auto &pf = b.host->keys[size_t(kidx[t])].pair_freq;
          sj.pj = hi;
          if (pf.size() == 65536) {
            uint32_t best = UINT32_MAX;
            for (uint32_t j = 2; j <= hi; j++) {
              const uint32_t f = pf[(uint32_t(nd[j]) << 8) | nd[j + 1]];
              if (f < best) {
                best = f;
                sj.pj = j;
              }
            }
          }
        }
        stream_jobs.push_back(sj);  // (wave0: after the plan, once the span is known)
      } else if (!k.identity) {
        jb.vmatch_base = vmatch_total;
        vmatch_total += k.nvals;
        set_jobs.push_back(uint32_t(jobs.size()));
        set_items.push_back(set_items.back() + words);
      }
      jobs.push_back(jb);
      dict_bytes += k.dict_nbytes + 4ull * (k.nvals + 1) + 4ull * words;
      ScanTerm st{};
      st.col = k.col;
      st.width = uint32_t(k.width);
      st.nsets = k.nsets;
      st.bm_words = words;
      const uint32_t lds_need = k.width == 1 ? 8u : words;  // u8: 256-bit table, branch-free lookups
      if (sg.lds_words + lds_need <= kLdsBudgetWords) {
        st.lds_off = sg.lds_words;
        sg.lds_words += lds_need;
      } else {
        st.lds_off = kNoLds;  // large dictionary: bitmap lookups go to L2 / MALL
      }
      terms.push_back(st);
      term_bm_base.push_back(jb.bm_base);
      per += uint64_t(k.width);
      all_w1 = all_w1 && k.width == 1 && st.lds_off != kNoLds;
    }
    max_lds_words = std::max(max_lds_words, sg.lds_words);
    {
      NarrowSeg ns{};
      ns.scan = d.dur32;
      ns.ncol = d.narrow_base;
      ns.npad = uint32_t(d.npad);
      for (uint32_t t = 0; t < q.nterms && all_narrow; t++) {
        const size_t k = size_t(kidx[t]);
        if (d.narrow_slot.size() <= k || d.narrow_slot[k] < 0 || d.narrow_slot[k] > 255 || !b.narrow[k]) {
          all_narrow = false;
          break;
        }
        ns.slot[t] = uint8_t(d.narrow_slot[k]);
        ns.nsets[t] = uint8_t(d.keys[k].nsets);
        ns.dict[t] = b.narrow[k].get();
      }
      if (d.npad >= (1ull << 32)) all_narrow = false;
      nsegv.push_back(ns);
    }
    {
      std::array<uint16_t, kArgTerms> ks{};
      uint32_t bmw = 0, bmw8 = 0, selfw = 0;
      for (uint32_t t = 0; t < q.nterms && t < kArgTerms; t++) {
        const DevKey &k = d.keys[size_t(kidx[t])];
        ks[t] = uint16_t(kidx[t]);
        uint32_t stage = k.nvals + 1 + uint32_t((k.dict_nbytes + 3) / 4);
        if (!k.identity) stage += k.nsets + 1 + k.nsetvals;
        if (k.dict_nbytes > (1u << 20) || k.nvals > (1u << 20) || kidx[t] > 0xffff) stage = 0xfffffffu;
        fast_stage = std::max(fast_stage, stage);
        selfw += stage + (k.identity ? 0u : (k.nvals + 63) / 32);
        fast_vbits = std::max(fast_vbits, (k.nvals + 63) / 32);
        fast_words = std::max(fast_words, (k.nsets + 31) / 32);
        bmw += (k.nsets + 31) / 32;
        bmw8 += k.width == 1 ? 8u : (k.nsets + 31) / 32;
      }
      seg_keys.push_back(ks);
      seg_desc.push_back(d.desc);
      fast_bm = std::max(fast_bm, bmw);
      fast_bm8 = std::max(fast_bm8, bmw8);
      fast_self = std::max(fast_self, std::min(selfw, 0xfffffffu));
    }
    sg.nunits = uint32_t((e1 + kUnit - 1) / kUnit);
    units += sg.nunits;
    // limit L: the block's first L records (ids are unique within a block: the consumer takes
    // at most L). The segment / look-back paths count records from position 0, so a part cut
    // at e0 > 0 keeps everything there (drop_before_ranges removes what precedes it); the pool
    // kernels scan [e0, e1) and cut each part to L themselves
    sg.cap = limit && e0 == 0 ? std::min<uint64_t>(limit, e1) : e1;
    scan_bytes += (e1 - e0) * per;
    n_all += e1;
    segs.push_back(sg);
  }
  out.recs.clear();
  out.term_any.clear();
  out.block_counts.assign(blocks.size(), 0);
  out.device_bytes = scan_bytes + dict_bytes;
  out.kernel_ns = out.scan_ns = 0;
  out.reruns = 0;
  out.pool = false;
  out.scan_bytes = scan_bytes;
  if (segs.empty()) return;
  if (segs.size() > kMaxSegs) fail(TSG_E_UNSUPPORTED, "too many blocks per device in one search (max 2048)");
  const uint32_t nsegs = uint32_t(segs.size());
  // one launch when the whole query fits the kernel arguments and every block's
  // dictionaries for it can be matched in LDS by the scanning workgroups
  // narrow mode: the value-set bitmap of every (dictionary, term) pair, matched here on
  // the host (bytes.Contains per value, a set matches when one of its values does);
  // identical dictionaries of different blocks are matched once
  thread_local std::vector<std::array<uint32_t, 8>> nbms;
  thread_local std::vector<std::array<uint8_t, kArgTerms>> nbmi;
  nbms.clear();
  nbmi.assign(segs.size(), {});
  const bool need64 = (q.has_min && q.min_ns >= 0xffffffffULL) || (q.has_max && q.max_ns >= 0xffffffffULL);
  bool narrow = all_narrow && !need64 && !dc.narrow_off && nsegs <= uint32_t(kArgSegs) &&
                needles.size() <= size_t(kArgNeedle);
  if (narrow) {
    std::pair<const NarrowDict *, uint32_t> memo[kArgBms];  // (dictionary, term) of each bitmap
    thread_local std::vector<uint8_t> vm;
    for (size_t i = 0; i < segs.size() && narrow; i++)
      for (uint32_t t = 0; t < q.nterms && narrow; t++) {
        const NarrowDict *nd = nsegv[i].dict[t];
        size_t j = 0;
        while (j < nbms.size() && !(memo[j].first == nd && memo[j].second == t)) j++;
        if (j < nbms.size()) {
          nbmi[i][t] = uint8_t(j);
          continue;
        }
        if (nbms.size() == size_t(kArgBms)) {
          narrow = false;
          break;
        }
        const std::string_view needle(reinterpret_cast<const char *>(q.values[t]), q.value_lens[t]);
        vm.assign(nd->nvals(), 0);
        for (uint32_t v = 0; v < nd->nvals(); v++) {
          const std::string_view val(reinterpret_cast<const char *>(nd->bytes.data() + nd->off[v]), nd->off[v + 1] - nd->off[v]);
          vm[v] = needle.empty() || val.find(needle) != std::string_view::npos;  // bytes.Contains (P7)
        }
        std::array<uint32_t, 8> bm{};
        for (uint32_t st = 0; st < nd->nsets(); st++) {
          bool m = false;
          for (uint32_t j = nd->set_off[st]; j < nd->set_off[st + 1] && !m; j++) m = vm[nd->set_vals[j]] != 0;
          if (m) bm[st >> 5] |= 1u << (st & 31);
        }
        nbmi[i][t] = uint8_t(nbms.size());
        memo[nbms.size()] = {nd, t};
        nbms.push_back(bm);
      }
  }
  const bool fast = !dc.fast_off && nsegs <= uint32_t(kArgSegs) && q.nterms <= 4 && needles.size() <= size_t(kArgNeedle) &&
                    (fast_stage <= kFastStageWords || narrow);
  // workgroups: about one resident wave of them (occupancy x CUs), each owning a
  // contiguous tile range of one block
  const ScanFn scan_fn = fast ? nullptr : pick_scan(q.nterms, has_dur, q.has_range, all_w1);
  // result mode, decided before the kernel is picked (see "Result modes" below)
  constexpr uint32_t kSegMax = 256;
  constexpr uint64_t kSegBudget = 64ull << 20;  // pinned bytes of segment records (workgroups <= 8 per CU)
  auto seg_fits = [&](uint32_t c) {
    return fast && !dc.seg_off && c > 0 && c <= kSegMax &&
           uint64_t(dc.num_cu) * std::max(8, dc.per_cu_override) * c * sizeof(MatchRec) <= kSegBudget;
  };
  // the segment / look-back paths' limit mode (segments of L records per workgroup, no rerun
  // on overflow) counts from position 0: a search with a part cut at e0 > 0 runs them in full
  // mode (its e0 = 0 parts keep their caps); the pool kernels take `limit` as it is
  bool cut_parts = false;
  for (const auto &sg : segs) cut_parts = cut_parts || sg.e0 > 0;
  const uint32_t climit = cut_parts ? 0u : limit;
  uint32_t seg = climit ? climit : dc.seg_cap;
  if (!seg_fits(seg)) seg = 0;
  // ---- pool path: narrow searches (search_pool_kernel); falls through to the
  // segment / look-back paths below when a workgroup's matches overflow its LDS buffer
  const bool ds16 = (!q.has_min || q.min_ns <= kDs16MaxMs * 1000000ull) && (!q.has_max || q.max_ns <= kDs16MaxMs * 1000000ull);
  if (fast && narrow && ds16 && !dc.seg_off && !dc.pool_off) {
    if (dc.pool_skip && dc.pool_skip_key == pool_query_key(q)) dc.pool_skip--;
    else if (pool_search(dc, blocks, q, limit, flags, segs, nsegv, nbms, nbmi, seg_desc, has_dur, tr, out, lk)) {
      if (ranges) drop_before_ranges(blocks, *ranges, out);
      out.pool = true;
      out.path |= out.resident ? TSG_PATH_RESIDENT : TSG_PATH_PLAIN;
      return;
    }
  }
  resident_quit(dc);  // (the other paths' kernels need the CUs the resident search launch holds)
  out.path |= TSG_PATH_OTHER;
  const FastFn fast_seg = fast ? pick_fast(q.nterms, has_dur, q.has_range, all_w1, true) : nullptr;
  const FastFn fast_lb = fast ? pick_fast(q.nterms, has_dur, q.has_range, all_w1, false) : nullptr;
  const void *kfn = fast ? reinterpret_cast<const void *>(seg ? fast_seg : fast_lb)
                         : reinterpret_cast<const void *>(scan_fn);
  // fast LDS: scan workgroups [bitmaps | masks | seg sums | first_wg | caps], dictionary
  // workgroups [value bits | stage]; the launch takes the larger
  // self-match: every block's dictionaries for this query fit one workgroup's LDS
  // stage, so no dictionary workgroups and no cross-workgroup wait
  const bool self_dict = fast && !narrow && !dc.self_off && q.nterms > 0 && fast_self <= kSelfWords;
  const uint32_t fast_bm_words =
      uint32_t(align_up(std::max(all_w1 ? fast_bm8 : fast_bm, self_dict ? 0u : fast_vbits), 2));
  const uint32_t fast_mask_words =
      std::max<uint32_t>(kLdsTiles * kThreads / 2, self_dict ? uint32_t(align_up(fast_self, 4)) : 0u);
  const uint32_t fast_scan_words = fast_mask_words + ((nsegs + 1) & ~1u) + ((nsegs + 2) & ~1u) + 2 * nsegs +
                                   (seg ? kSegMax * uint32_t(sizeof(MatchRec) / 4) : 0u);
  const uint32_t lds_words = fast ? fast_bm_words + std::max<uint32_t>(fast_scan_words, uint32_t(align_up(fast_stage, 4)))
                                  : max_lds_words + kLdsTiles * kThreads / 2 + nsegs;
  int &per_cu = dc.occupancy[{kfn, size_t(lds_words) * 4}];
  if (per_cu == 0) {
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kThreads, size_t(lds_words) * 4));
    per_cu = std::max(1, std::min(per_cu, 8));
  }
  // every workgroup of the launch resident at once: a workgroup dispatched only
  // when another retires starts a full scan slice late and the in-order look-back
  // waits for it. The one-launch grid also holds the dictionary workgroups.
  const uint32_t slots = uint32_t(dc.num_cu) * uint32_t(dc.per_cu_override ? dc.per_cu_override : per_cu);
  const uint32_t njobs_fast = fast && !self_dict && !narrow ? nsegs * q.nterms : 0;
  const uint32_t target_wg = slots > njobs_fast + uint32_t(dc.num_cu) ? slots - njobs_fast : uint32_t(dc.num_cu);
  // workgroups per block in proportion to its units, the units of a block split
  // evenly over its workgroups: every CU gets the same load (+-1 unit of 1024 entries)
  uint32_t nwg = 0, tpw = 1;
  uint64_t units_before = 0;
  for (auto &sg : segs) {
    // cumulative rounding: the block gets round(target * units_through / units)
    // minus what earlier blocks got, so the grid never exceeds target_wg (+1 per
    // block only where a block would otherwise get none)
    const uint64_t hi = (uint64_t(target_wg) * (units_before + sg.nunits) + units / 2) / units;
    units_before += sg.nunits;
    uint64_t w = hi > nwg ? hi - nwg : 0;
    w = std::max<uint64_t>(1, std::min<uint64_t>(w, (sg.nunits + kSteps - 1) / kSteps));  // <= its tiles
    sg.first_wg = nwg;
    sg.nwg = uint32_t(w);
    sg.tpw = uint32_t(((sg.nunits + w - 1) / w + kSteps - 1) / kSteps);
    // work stealing (segment mode): the block's last quarter of tiles is claimed at run time
    // (static tiles stay >= one per workgroup)
    {
      const uint32_t tiles = (sg.nunits + kSteps - 1) / kSteps;
      sg.tail = dc.steal_off ? 0u : std::min<uint32_t>(tiles / 4, tiles - uint32_t(w));
      if (sg.tail > 0xffffu) sg.tail = 0xffffu;
    }
    tpw = std::max(tpw, sg.tpw);
    nwg += sg.nwg;
  }
  if (tpw > kMaxTpw) fail(TSG_E_UNSUPPORTED, "too many entries per device in one search");
  if (n_all >= (1ull << 32)) fail(TSG_E_UNSUPPORTED, "more than 2^32 entries per device in one search");
  tr.mark("plan");

  // ---- scratch
  if (tpw > kLdsTiles) dc.maskbits.ensure(size_t(nwg) * tpw * kThreads * 2);
  if (dc.agg.ensure(size_t(nwg) * 8)) HIP_OK(hipMemsetAsync(dc.agg.p, 0, dc.agg.cap, s));  // no stale epochs
  if (fast && dc.done.ensure(9 * 128)) {  // completion counters: zeroed once, then monotonic
    HIP_OK(hipMemsetAsync(dc.done.p, 0, dc.done.cap, s));
    std::fill(std::begin(dc.done_base), std::end(dc.done_base), 0u);
  }
  const size_t hdr_bytes = align_up(64 + 8 * segs.size(), 256);
  uint64_t n_total = 0, cap_total = 0;
  for (size_t i = 0; i < segs.size(); i++) {
    n_total += segs[i].n;
    cap_total += segs[i].cap;
  }
  const size_t cnt_bytes = align_up(size_t(nwg) * 4, 256);
  // Result modes (the records go straight to pinned host memory: no D2H copy).
  //  segment (one-launch path): a segment of seg_cap records per workgroup, no
  //    look-back; limit L: segments of L; limit 0: seg_cap follows the largest
  //    per-workgroup count seen on this device (an overflow re-runs with larger
  //    segments, or in look-back mode beyond kSegMax)
  //  look-back: one record array; limit 0 starts from the capacity the buffer already
  //    has (>= 2^16 records) and a larger match count re-runs into a grown buffer
  auto lb_cap = [&]() -> uint64_t {
    const uint64_t have = dc.hres.cap > hdr_bytes ? (dc.hres.cap - hdr_bytes) / sizeof(MatchRec) : 0;
    return climit ? cap_total : std::min<uint64_t>(n_total, std::max<uint64_t>(have, 1u << 16));
  };
  const bool time_all = flags & TSG_SEARCH_TIME_ALL, time_scan = flags & (TSG_SEARCH_TIME_SCAN | TSG_SEARCH_TIME_ALL);
  const bool time_defer = flags & TSG_SEARCH_TIME_DEFER;

  ScanParams P{};
  P.prio = dc.prio ? 1u : 0u;
  P.nsegs = nsegs;
  P.nwg = nwg;
  P.has_min = q.has_min;
  P.has_max = q.has_max;
  P.need64 = (q.has_min && q.min_ns >= 0xffffffffULL) || (q.has_max && q.max_ns >= 0xffffffffULL);
  P.limit_mode = climit ? 1 : 0;
  P.min_ns = q.min_ns;
  P.max_ns = q.max_ns;
  P.start_s = q.start_s;
  P.end_s = q.end_s;
  P.mask = static_cast<uint16_t *>(dc.maskbits.p);
  P.mask_tpw = tpw;
  P.agg = static_cast<unsigned long long *>(dc.agg.p);
  P.lds_bm_words = max_lds_words;
  // [header | tile counts (segment mode) | records]
  static const bool lb_full = std::getenv("TSG_LB_FULL") != nullptr;  // (A/B: 48-byte look-back records)
  // TSG_LB_BITMAP: 0 = never bitmap mode, 1 = every full scan on the general path, 2 (default) =
  // when the previous full scan there had more than one match per 64 entries
  const uint32_t lb_bitmap = debug_lb_bitmap();
  const bool bm_mode = !fast && !climit && !ranges && !lb_full && lb_bitmap && (lb_bitmap == 1 || dc.lb_dense);
  uint64_t bm_words_total = 0;
  auto configure = [&](uint32_t sg, uint64_t out_cap) {
    P.seg_cap = sg;
    P.compact = sg || lb_full ? 0u : 1u;
    P.hdr_bytes = sg ? hdr_bytes + cnt_bytes : hdr_bytes;
    P.out_cap = sg ? uint64_t(nwg) * sg : out_cap;
    dc.hres.ensure(P.hdr_bytes + std::max<uint64_t>(P.out_cap, 1) * sizeof(MatchRec));
    P.out = static_cast<uint8_t *>(dc.hres.p);
    P.counts = reinterpret_cast<uint32_t *>(P.out + hdr_bytes);
  };
  configure(seg, seg ? 0 : lb_cap());
  static const bool want_stamps = std::getenv("TSG_STAMPS") != nullptr;
  if (want_stamps) {
    dc.stamps.ensure(size_t(nwg) * kStampSlots * 8);
    HIP_OK(hipMemsetAsync(dc.stamps.p, 0, size_t(nwg) * kStampSlots * 8, s));
    P.stamps = static_cast<unsigned long long *>(dc.stamps.p);
  }
  QArgs A;
  if (fast) {
    std::memset(&A, 0, sizeof A);
    for (uint32_t i = 0; i < nsegs; i++) {
      A.blk[i] = seg_desc[i];
      A.cap[i] = segs[i].cap;
      A.first_wg[i] = segs[i].first_wg;
      A.block_idx[i] = segs[i].block_idx;
      for (int t = 0; t < kArgTerms; t++) A.key_of[i][t] = seg_keys[i][size_t(t)];
    }
    A.first_wg[nsegs] = nwg;
    for (uint32_t i = 0; i < nsegs; i++) A.tail[i] = segs[i].tail;
    if (dc.steal.ensure(kArgSegs * 128)) {  // claim counters: zeroed once, then monotonic
      HIP_OK(hipMemsetAsync(dc.steal.p, 0, dc.steal.cap, s));
      std::fill(std::begin(dc.steal_base), std::end(dc.steal_base), 0u);
    }
    P.steal = static_cast<unsigned *>(dc.steal.p);
    A.narrow = narrow ? 1u : 0u;
    if (narrow) {
      for (uint32_t i = 0; i < nsegs; i++) {
        A.scan[i] = nsegv[i].scan;
        A.ncol[i] = nsegv[i].ncol;
        A.npad[i] = nsegv[i].npad;
        A.nent[i] = uint32_t(segs[i].n);
        for (uint32_t t = 0; t < q.nterms; t++) {
          A.slot[i][t] = nsegv[i].slot[t];
          A.nsets8[i][t] = nsegv[i].nsets[t];
          A.bmi[i][t] = nbmi[i][t];
        }
      }
      for (size_t j = 0; j < nbms.size(); j++)
        for (int w = 0; w < 8; w++) A.bms[j][w] = nbms[j][size_t(w)];
    }
    for (uint32_t t = 0; t <= q.nterms; t++) A.nd_off[t] = uint16_t(t < q.nterms ? needle_off[t] : needles.size());
    if (!needles.empty()) std::memcpy(A.needles, needles.data(), needles.size());
    A.nsegs = nsegs;
    A.nterms = q.nterms;
    A.njobs = njobs_fast;
    A.self_dict = self_dict ? 1u : 0u;
    A.stage_first = dc.stage_first ? 1u : 0u;
    A.bm_first = dc.bm_first ? 1u : 0u;
    A.mask_words = fast_mask_words;
    A.gstride = fast_words;
    A.bm_words = fast_bm_words;
    A.stage_words = fast_stage;
    if (A.njobs && dc.gbm.ensure(size_t(A.njobs) * fast_words * 8))
      HIP_OK(hipMemsetAsync(dc.gbm.p, 0, dc.gbm.cap, s));  // tag 0: never published
    A.gbm = static_cast<unsigned long long *>(dc.gbm.p);
    P.done = static_cast<unsigned *>(dc.done.p);
    tr.mark("desc");
    if (time_all) HIP_OK(hipEventRecord(dc.ev0, s));
  } else {
    dc.bitmaps.ensure(std::max<size_t>(bm_total, 1) * 4);
    dc.vmatch.ensure(std::max<size_t>(vmatch_total, 1));
    // per job (= term: one per block and term, in the same order): some value matched
    dc.danyf.ensure(std::max<size_t>(jobs.size(), 1) * 4);
    for (size_t i = 0; i < terms.size(); i++) {
      terms[i].bm = static_cast<const uint32_t *>(dc.bitmaps.p) + term_bm_base[i];
      terms[i].anyf = static_cast<const uint32_t *>(dc.danyf.p) + i;  // (the scan skips a block with a dead term)
    }
    P.anyf = static_cast<const uint32_t *>(dc.danyf.p);
    P.nterms = q.nterms;
    // bitmap mode (full scans on this path whose last one was dense): the blocks' bit ranges
    if (bm_mode) {
      uint64_t w0 = 0;
      for (auto &sg : segs) {
        sg.bm_word0 = w0;
        w0 += uint64_t(sg.nunits) * (kUnit / 64);
      }
      dc.hbits.ensure(std::max<uint64_t>(w0, 1) * 8);
      P.bitmap = static_cast<unsigned long long *>(dc.hbits.p);
      bm_words_total = w0;
    }
    // ---- descriptors: written to pinned host memory; the prep kernel copies them
    // into device memory (small descriptor sets) or one H2D copy (large ones)
    const size_t o_segs = 0, o_terms = align_up(segs.size() * sizeof(ScanSeg), 16);
    const size_t o_jobs = align_up(o_terms + terms.size() * sizeof(ScanTerm), 16);
    const size_t o_jb = align_up(o_jobs + jobs.size() * sizeof(DictJob), 16);
    const size_t o_sj = align_up(o_jb + jobs.size() * 4, 16);
    const size_t o_sp = align_up(o_sj + set_jobs.size() * 4, 16);
    const size_t o_nd = align_up(o_sp + set_items.size() * 4, 16);
    const size_t o_ws = align_up(o_nd + needles.size() + 1, 16);
    // dictionary stream spans: ~16 waves per CU over the pass's bytes, 8-64 KiB each (one
    // 64 KiB span per wave left a 91 MB dictionary with ~5 waves per CU: latency-bound)
    if (!stream_jobs.empty()) {
      uint64_t tot = 0;
      for (const auto &sj : stream_jobs) tot += sj.lead + sj.nbytes;
      uint64_t sp = tot / (uint64_t(std::max(dc.num_cu, 1)) * 16);
      sp = std::min<uint64_t>(kStreamSpan, std::max<uint64_t>(8192, (sp + 1023) / 1024 * 1024));
      stream_span = uint32_t(sp);
      stream_waves = 0;
      for (auto &sj : stream_jobs) {
        sj.wave0 = stream_waves;
        stream_waves += uint32_t((sj.lead + sj.nbytes + sp - 1) / sp);
      }
    }
    const size_t o_stj = align_up(o_ws + size_t(nwg) * 2, 16);
    const size_t total_desc = align_up(o_stj + stream_jobs.size() * sizeof(StreamJob), 16);
    dc.hdesc.ensure(total_desc);
    dc.desc.ensure(total_desc);
    auto *hd = static_cast<uint8_t *>(dc.hdesc.p);
    for (auto &sg : segs) sg.tail = 0;  // (the descriptor path splits every tile statically)
    std::memcpy(hd + o_segs, segs.data(), segs.size() * sizeof(ScanSeg));
    std::memcpy(hd + o_terms, terms.data(), terms.size() * sizeof(ScanTerm));
    std::memcpy(hd + o_jobs, jobs.data(), jobs.size() * sizeof(DictJob));
    auto *jbase = reinterpret_cast<uint32_t *>(hd + o_jb);
    for (size_t i = 0; i < jobs.size(); i++) jbase[i] = jobs[i].item_base;
    if (!set_jobs.empty()) std::memcpy(hd + o_sj, set_jobs.data(), set_jobs.size() * 4);
    std::memcpy(hd + o_sp, set_items.data(), set_items.size() * 4);
    if (!needles.empty()) std::memcpy(hd + o_nd, needles.data(), needles.size());
    if (!stream_jobs.empty()) std::memcpy(hd + o_stj, stream_jobs.data(), stream_jobs.size() * sizeof(StreamJob));
    auto *ws = reinterpret_cast<uint16_t *>(hd + o_ws);
    for (size_t i = 0; i < segs.size(); i++)
      for (uint32_t w = 0; w < segs[i].nwg; w++) ws[segs[i].first_wg + w] = uint16_t(i);
    auto *dd = static_cast<uint8_t *>(dc.desc.p);
    const uint8_t *src = hd;
    if (total_desc > kHostDescMax) {
      HIP_OK(hipMemcpyAsync(dd, hd, total_desc, hipMemcpyHostToDevice, s));
      src = dd;
    }
    tr.mark("desc");
    if (time_all) HIP_OK(hipEventRecord(dc.ev0, s));
    if (!stream_jobs.empty()) HIP_OK(hipMemsetAsync(dc.vmatch.p, 0, vmatch_total, s));
    // per job: some value matched (device flags, zeroed here; copied to pinned host memory
    // after the dictionary kernels: one small copy instead of a host store per matching word)
    dc.hany.ensure(std::max<size_t>(jobs.size(), 1) * 4);
    dc.danyf.ensure(std::max<size_t>(jobs.size(), 1) * 4);
    auto *anyf = static_cast<uint32_t *>(dc.danyf.p);
    if (!jobs.empty()) HIP_OK(hipMemsetAsync(anyf, 0, jobs.size() * 4, s));
    prep_kernel<<<std::max<uint32_t>(1, (items + 255) / 256), 256, 0, s>>>(
        src, dd, uint32_t(total_desc / 16), uint32_t(o_jobs), uint32_t(o_jb), uint32_t(jobs.size()), items,
        uint32_t(o_nd), uint32_t(needles.size()), static_cast<uint8_t *>(dc.vmatch.p),
        static_cast<uint32_t *>(dc.bitmaps.p), anyf);
    if (!stream_jobs.empty())
      dict_stream_kernel<<<(stream_waves + kStreamWg - 1) / kStreamWg, 64 * kStreamWg, 0, s>>>(
          reinterpret_cast<const StreamJob *>(dd + o_stj), uint32_t(stream_jobs.size()), dd + o_nd,
          static_cast<uint8_t *>(dc.vmatch.p), stream_span, stream_waves);
    if (set_items.back())
      dict_sets_kernel<<<(set_items.back() + 255) / 256, 256, 0, s>>>(
          reinterpret_cast<const DictJob *>(dd + o_jobs), reinterpret_cast<const uint32_t *>(dd + o_sj),
          reinterpret_cast<const uint32_t *>(dd + o_sp), uint32_t(set_jobs.size()), set_items.back(),
          static_cast<const uint8_t *>(dc.vmatch.p), static_cast<uint32_t *>(dc.bitmaps.p), anyf);
    if (!jobs.empty()) HIP_OK(hipMemcpyAsync(dc.hany.p, anyf, jobs.size() * 4, hipMemcpyDeviceToHost, s));
    P.segs = reinterpret_cast<const ScanSeg *>(dd + o_segs);
    P.terms = reinterpret_cast<const ScanTerm *>(dd + o_terms);
    P.wg_seg = reinterpret_cast<const uint16_t *>(dd + o_ws);
    tr.mark("dict");
  }
  // XCD groups of the scan workgroups (blockIdx % 8 over [njobs, njobs + nwg))
  const uint32_t grid = fast ? A.njobs + nwg : nwg;
  uint32_t group_n[8] = {};
  for (uint32_t g = 0; g < 8; g++) {
    const uint32_t lo = fast ? A.njobs : 0u;
    // blocks b in [lo, grid) with b % 8 == g
    const uint32_t first = lo + ((g + 8 - lo % 8) % 8);
    group_n[g] = first < grid ? (grid - first + 7) / 8 : 0;
  }
  auto launch = [&](bool first) {
    if (++dc.search_epoch == 0) dc.search_epoch = 1;  // 0 is the never-published tag of a fresh buffer
    P.epoch = dc.search_epoch;
    auto *h = reinterpret_cast<volatile uint64_t *>(P.out);
    h[0] = 0;
    h[1] = 0;  // look-back / granule poll error flag
    h[2] = 0;  // completion flag (one-launch path)
    if (!fast && !P.seg_cap)  // (per-block counts: what a launch whose blocks are all dead leaves)
      for (uint32_t i = 0; i < nsegs; i++) h[8 + i] = 0;
    if (fast && P.seg_cap) std::fill_n(P.counts, nwg, kCountPending);  // (each workgroup stores its count last)
    static const bool flag_env = std::getenv("TSG_FLAG_DONE") != nullptr;
    P.flag_done = fast && (!P.seg_cap || flag_env) ? 1u : 0u;
    if (fast) {
      for (uint32_t i = 0; i < nsegs; i++) A.steal_base[i] = dc.steal_base[i];
      uint32_t ng = 0;
      for (uint32_t g = 0; g < 8; g++) {
        P.done_target[g] = dc.done_base[g] + group_n[g];
        ng += group_n[g] ? 1u : 0u;
      }
      P.done_top = dc.done_base[8] + ng;
    }
    // workgroups that wait on lower-numbered ones take their order from a ticket
    P.ticket = static_cast<unsigned long long *>(dc.ticket.p);
    P.ticket_base = dc.ticket_base;
    // (bitmap mode: no look-back, no dictionary waits: blockIdx order)
    P.use_ticket = P.bitmap ? 0u : (!fast || !P.seg_cap || A.njobs) ? 1u : 0u;
    // the fast kernel's preloaded scalar arguments (search_fast_kernel)
    uint32_t pre[8] = {};
    if (fast) {
      const uint32_t n = A.nsegs, W = A.first_wg[A.nsegs], h = n / 2;
      bool uniform = n > 0 && W > 0 && uint64_t(W + 1) * n < (1ull << 32);
      for (uint32_t i = 0; i <= n && uniform; i++) uniform = A.first_wg[i] == uint32_t((uint64_t(W) * i + h) / n);
      pre[0] = (P.use_ticket ? kPreTicket : 0u) | (A.narrow ? kPreNarrow : 0u) | (A.bm_first ? kPreBmFirst : 0u) |
               (A.self_dict ? kPreSelf : 0u) | (uniform ? kPreUniform : 0u) | (P.stamps ? kPreStamps : 0u);
      pre[1] = n;
      pre[2] = A.njobs;
      pre[3] = W;
      pre[4] = h;
      pre[5] = A.bm_words;
      pre[6] = A.mask_words;
      pre[7] = A.nterms;
    }
    hipEvent_t e0 = first ? dc.es0 : dc.er0, e1 = first ? dc.es1 : dc.er1;
    const bool timed = time_scan;  // (a rerun's launch is timed too: it produces the records)
    const bool defer = first && !timed && time_defer && dc.defer_slot(e0, e1);
    if ((timed || defer) && dc.ext_events) {  // events stamped from the dispatch packet (hipExtLaunchKernel)
      if (fast) A.P = P;
      void *fargs[] = {&pre[0], &pre[1], &pre[2], &pre[3], &pre[4], &pre[5], &pre[6], &pre[7], &P.stamps, &A};
      void *sargs[] = {&P};
      void **args = fast ? fargs : sargs;
      const void *f = fast ? reinterpret_cast<const void *>(P.seg_cap ? fast_seg : fast_lb) : kfn;
      HIP_OK(hipExtLaunchKernel(f, dim3(grid), dim3(kThreads), args, size_t(lds_words) * 4, s, e0, e1, 0));
    } else {
      if (timed || defer) HIP_OK(hipEventRecord(e0, s));
      else if (dc.mark_mode & 1) HIP_OK(hipEventRecord(dc.mk0, s));
      if (fast) {
        A.P = P;
        (P.seg_cap ? fast_seg : fast_lb)<<<grid, kThreads, size_t(lds_words) * 4, s>>>(
            pre[0], pre[1], pre[2], pre[3], pre[4], pre[5], pre[6], pre[7], P.stamps, A);
      } else {
        scan_fn<<<grid, kThreads, size_t(lds_words) * 4, s>>>(P);
      }
      HIP_OK(hipGetLastError());
      if (timed || defer) HIP_OK(hipEventRecord(e1, s));
      else if (dc.mark_mode & 2) HIP_OK(hipEventRecord(dc.mk1, s));
    }
    if (fast && P.flag_done) {  // the launch advances every counter by a known amount
      for (uint32_t g = 0; g < 8; g++) dc.done_base[g] = P.done_target[g];
      dc.done_base[8] = P.done_top;
    }
    if (P.use_ticket) dc.ticket_base += grid;
    if (fast && P.seg_cap)  // every workgroup of a block with a tail ends with one failed claim
      for (uint32_t i = 0; i < nsegs; i++)
        if (segs[i].tail) dc.steal_base[i] += segs[i].tail + segs[i].nwg;
  };
  // segment mode: poll the completion flag the last workgroup raises in the pinned
  // header instead of waiting for the stream (the end-of-kernel signal comes later);
  // the stream is queried now and then, so a kernel that dies without raising the
  // flag fails the search instead of hanging the host
  auto wait = [&] {
    if (!fast || !P.seg_cap) {  // (look-back mode writes its records with plain stores)
      HIP_OK(hipStreamSynchronize(s));
      return;
    }
    // The flag is read with acquire semantics: the record and count loads after it
    // cannot be satisfied before it. On the device side every workgroup's record and
    // count stores (system-scope write-through) complete (s_waitcnt vmcnt(0), memory
    // clobber) before its arrival at the completion counters, and the flag store is
    // issued by the last arrival, so the flag is the last of the launch's host writes.
    // Without the flag (P.flag_done 0): done once every workgroup's count has been seen —
    // each count is stored after that workgroup's records completed, and the counts are
    // read with acquire loads, so the copy below reads complete records.
    const uint64_t *flag = reinterpret_cast<const uint64_t *>(P.out) + 2;
    auto flag_up = [&] { return P.flag_done && __atomic_load_n(flag, __ATOMIC_ACQUIRE) == P.epoch; };
    // while the tail of the launch runs, pull the record segments of workgroups that
    // have finished into this core's caches (the copy after the flag then reads cached
    // lines instead of missing on every one)
    const uint32_t *cnt = P.counts;
    const uint8_t *rec = P.out + P.hdr_bytes;
    thread_local std::vector<uint8_t> seen;
    seen.assign(nwg, 0);
    uint32_t lo = 0;  // every workgroup below lo has been seen
    for (uint32_t it = 1;; it++) {
      if (flag_up()) return;
      for (uint32_t w = lo; w < nwg; w++) {
        if (seen[w]) {
          if (w == lo) lo++;
          continue;
        }
        const uint32_t c = __atomic_load_n(cnt + w, __ATOMIC_ACQUIRE);
        if (c == kCountPending) continue;
        seen[w] = 1;
        if (w == lo) lo++;
        const uint8_t *p0 = rec + uint64_t(w) * P.seg_cap * sizeof(MatchRec);
        for (uint64_t o = 0; o < uint64_t(std::min(c, P.seg_cap)) * sizeof(MatchRec); o += 64) __builtin_prefetch(p0 + o);
      }
      if (!P.flag_done && lo == nwg) return;
      if ((it & 255u) == 0) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) {
          if (flag_up() || lo == nwg) return;
          bool all = true;
          for (uint32_t w = 0; w < nwg && all; w++) all = __atomic_load_n(cnt + w, __ATOMIC_ACQUIRE) != kCountPending;
          if (all) return;
          fail(TSG_E_DEVICE, "search kernel completed without storing every workgroup count");
        }
        if (e != hipErrorNotReady) HIP_OK(e);
      }
      __builtin_ia32_pause();
    }
  };
  auto check = [&] {
    if (reinterpret_cast<volatile uint64_t *>(P.out)[1])
      fail(TSG_E_DEVICE, "search look-back did not complete (workgroup dispatch order assumption broken)");
  };
  launch(true);
  if (time_all) HIP_OK(hipEventRecord(dc.ev1, s));
  tr.mark("search");
  wait();
  tr.mark("sync");
  check();
  if (!fast && P.nterms && P.use_ticket) {
    // every block dead: the launch's workgroups returned before taking tickets (search_kernel)
    const auto *anyf = static_cast<const volatile uint32_t *>(dc.hany.p);
    bool all_dead = true;
    for (uint32_t i = 0; i < nsegs && all_dead; i++) {
      bool dead = false;
      for (uint32_t t = 0; t < q.nterms; t++) dead = dead || anyf[size_t(i) * q.nterms + t] == 0u;
      all_dead = dead;
    }
    if (all_dead) dc.ticket_base -= grid;
  }
  if (!fast) {  // per block: which terms some dictionary value matched (job = segment x term)
    const auto *anyf = static_cast<const volatile uint32_t *>(dc.hany.p);
    for (uint32_t i = 0; i < nsegs; i++) {
      uint32_t m = 0;
      for (uint32_t t = 0; t < q.nterms; t++)
        if (t >= 32 || anyf[size_t(i) * q.nterms + t]) m |= t < 32 ? 1u << t : 0u;
      out.term_any.push_back({segs[i].block_idx, m});
    }
  }
  if (want_stamps) print_stamps(dc, nwg, fast);
  float ms = 0, sms = 0;
  if (time_all) {
    HIP_OK(hipEventSynchronize(dc.ev1));
    HIP_OK(hipEventElapsedTime(&ms, dc.ev0, dc.ev1));
  }
  if (time_scan) {
    HIP_OK(hipEventSynchronize(dc.es1));
    HIP_OK(hipEventElapsedTime(&sms, dc.es0, dc.es1));
  }
  out.kernel_ns = uint64_t(double(ms) * 1e6);
  out.scan_ns = uint64_t(double(sms) * 1e6);
  tr.mark("events");
  // a rerun produces the records: its time counts too, and the reruns are counted
  auto rerun_timed = [&] {
    launch(false);  // (timed with er0/er1 under time_scan)
    wait();
    check();
    if (time_scan) {
      float rms = 0;
      HIP_OK(hipEventSynchronize(dc.er1));
      HIP_OK(hipEventElapsedTime(&rms, dc.er0, dc.er1));
      out.scan_ns += uint64_t(double(rms) * 1e6);
      if (time_all) out.kernel_ns += uint64_t(double(rms) * 1e6);
    }
    out.reruns++;
  };

  // ---- results
  if (P.seg_cap) {
    const uint32_t *cnt = P.counts;  // (every scan workgroup writes its count)
    for (uint32_t w = 0; w < nwg; w += 16) __builtin_prefetch(cnt + w);
    uint32_t maxc = 0;
    uint64_t total = 0;
    for (uint32_t w = 0; w < nwg; w++) {
      maxc = std::max(maxc, cnt[w]);
      total += cnt[w];
    }
    tr.mark("counts");
    if (!climit && maxc > P.seg_cap) {
      // a workgroup overflowed its segment: remember the size and run again with
      // larger segments, or in look-back mode
      uint32_t want = 16;
      while (want < maxc && want < (1u << 30)) want <<= 1;
      dc.seg_cap = want;
      configure(seg_fits(want) ? want : 0u, total);
      rerun_timed();
    }
  }
  uint64_t nrec = 0;
  if (P.seg_cap) {
    // concatenate the workgroup segments in scan order; limit L: each block's first L
    const uint32_t *cnt = P.counts;
    const uint8_t *rec = P.out + P.hdr_bytes;
    // the GPU's writes evicted these lines from the CPU caches: touch every non-empty
    // segment once (prefetch) before copying, so the misses overlap
    uint64_t upper = 0;
    for (uint32_t w = 0; w < nwg; w++) {
      const uint32_t c = std::min(cnt[w], P.seg_cap);
      if (!c) continue;
      upper += c;
      const uint8_t *p0 = rec + uint64_t(w) * P.seg_cap * sizeof(MatchRec);
      for (uint64_t o = 0; o < c * sizeof(MatchRec); o += 64) __builtin_prefetch(p0 + o);
    }
    grow_recs(out, upper);
    for (size_t i = 0; i < segs.size(); i++) {
      uint64_t kept = 0;
      const bool stole = fast && segs[i].tail;  // tail records sit in their claimers' segments
      const size_t b0 = nrec;
      for (uint32_t w = segs[i].first_wg; w < segs[i].first_wg + segs[i].nwg && (stole || kept < segs[i].cap); w++) {
        const uint64_t c = stole ? std::min(cnt[w], P.seg_cap)
                                 : std::min<uint64_t>(std::min(cnt[w], P.seg_cap), segs[i].cap - kept);
        if (!c) continue;
        std::memcpy(&out.recs[nrec], rec + uint64_t(w) * P.seg_cap * sizeof(MatchRec), c * sizeof(MatchRec));
        nrec += c;
        kept += c;
      }
      if (stole && nrec - b0 > 1) {  // scan order = scan position within the block; then the cap
        std::sort(out.recs.begin() + b0, out.recs.begin() + nrec,
                  [](const SearchOut::Rec &a, const SearchOut::Rec &b) { return a.entry < b.entry; });
      }
      if (stole && kept > segs[i].cap) {
        nrec = b0 + segs[i].cap;
        kept = segs[i].cap;
      }
      for (size_t bi = 0; bi < blocks.size(); bi++)
        if (blocks[bi].first == segs[i].block_idx) out.block_counts[bi] = kept;
    }
    out.recs.resize(nrec);
    out.scan_bytes += uint64_t(nwg) * 4 + nrec * 32;  // + workgroup counts, + id/start/end of each record
  } else if (bm_mode) {
    // bitmap mode: per block its bits' popcount (a block with a dead term: the kernel skipped
    // it and wrote nothing, count 0), then the bits expanded into scan positions, block by block
    // on several threads
    const auto *bits = static_cast<const uint64_t *>(dc.hbits.p);
    const auto *hanyp = static_cast<const volatile uint32_t *>(dc.hany.p);
    // (locals, not thread_local: the lambdas below run on other threads too)
    std::vector<uint64_t> cnt(nsegs, 0), off(nsegs + 1, 0);
    std::vector<uint8_t> live(nsegs, 1);
    for (uint32_t i = 0; i < nsegs; i++)
      for (uint32_t t = 0; t < q.nterms; t++)
        if (!hanyp[size_t(i) * q.nterms + t]) live[i] = 0;
    auto words_of = [&](uint32_t i) { return (segs[i].n + 63) / 64; };
    parallel_ranges(nsegs, 1, 16, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; i++) {
        if (!live[i]) continue;
        const uint64_t *b = bits + segs[i].bm_word0;
        uint64_t c = 0;
        for (uint64_t w = 0, nw = words_of(uint32_t(i)); w < nw; w++) c += uint64_t(__builtin_popcountll(b[w]));
        cnt[i] = c;
      }
    });
    for (uint32_t i = 0; i < nsegs; i++) off[i + 1] = off[i] + cnt[i];
    const uint64_t total = off[nsegs];
    nrec = total;
    thread_local RawVec<uint64_t> bpos;
    RawVec<uint64_t> &pos = out.want_pos ? out.pos : bpos;
    pos.resize(total);
    parallel_ranges(nsegs, 1, 16, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; i++) {
        if (!cnt[i]) continue;
        const uint64_t *b = bits + segs[i].bm_word0;
        uint64_t *o = pos.data() + off[i];
        const uint64_t tag = uint64_t(segs[i].block_idx) << 32;
        for (uint64_t w = 0, nw = words_of(uint32_t(i)); w < nw; w++)
          for (uint64_t x = b[w]; x; x &= x - 1) *o++ = tag | (w * 64 + uint64_t(__builtin_ctzll(x)));
      }
    });
    if (out.want_pos) {
      out.compact = true;
    } else if (total) {
      grow_recs(out, total);
      positions_to_recs(blocks, pos.data(), total, out);
    }
    for (size_t i = 0; i < segs.size(); i++)
      for (size_t bi = 0; bi < blocks.size(); bi++)
        if (blocks[bi].first == segs[i].block_idx) out.block_counts[bi] = cnt[i];
    out.scan_bytes += bm_words_total * 8;  // + the bits written
    if (total * 256 < n_total) dc.lb_dense = false;  // (sparse again: positions from the next full scan on)
  } else {
    uint64_t total = *reinterpret_cast<volatile uint64_t *>(P.out);
    if (!climit && !ranges && !fast && P.compact && total * 64 > n_total) dc.lb_dense = true;
    if (!climit && total > P.out_cap) {
      // more matches than the result buffer holds: grow it and run the launch again
      configure(0, total);
      rerun_timed();
    }
    if (!climit && fast && total <= 64) dc.seg_cap = 16;  // sparse again: back to segment mode
    nrec = total;
    if (total && P.compact && out.want_pos && !ranges) {
      // the caller gathers the records from the host columns itself (into its result arrays)
      out.pos.resize(total);
      parallel_ranges(size_t(total) * 8, size_t(4) << 20, 16, [&](size_t lo, size_t hi) {
        std::memcpy(reinterpret_cast<uint8_t *>(out.pos.data()) + lo, P.out + P.hdr_bytes + lo, hi - lo);
      });
      out.compact = true;
    } else if (total && P.compact) {
      grow_recs(out, total);
      positions_to_recs(blocks, reinterpret_cast<const uint64_t *>(P.out + P.hdr_bytes), total, out);
    } else if (total) {
      // (a dense result is tens of MB of pinned memory: copied on several threads)
      grow_recs(out, total);
      parallel_ranges(size_t(total) * sizeof(MatchRec), size_t(8) << 20, 16, [&](size_t lo, size_t hi) {
        std::memcpy(reinterpret_cast<uint8_t *>(out.recs.data()) + lo, P.out + P.hdr_bytes + lo, hi - lo);
      });
    }
    for (size_t i = 0; i < segs.size(); i++) {
      uint64_t c;
      std::memcpy(&c, P.out + 64 + 8 * i, 8);
      for (size_t bi = 0; bi < blocks.size(); bi++)
        if (blocks[bi].first == segs[i].block_idx) out.block_counts[bi] = c;
    }
    out.scan_bytes += uint64_t(nwg) * 8 + nrec * (P.compact ? 8 : 32);  // + published counts, + records
  }
  if (ranges) drop_before_ranges(blocks, *ranges, out);
  tr.mark("post");
}

bool device_last_dense(DeviceCtx &dc) {
  std::lock_guard<std::mutex> lk(dc.mu);
  return dc.lb_dense;
}

void device_kernel_times(DeviceCtx &dc, std::vector<uint64_t> &ns) {
  std::lock_guard<std::mutex> lk(dc.mu);
  HIP_OK(hipSetDevice(dc.ordinal));
  HIP_OK(hipStreamSynchronize(dc.stream));
  for (size_t i = 0; i < dc.tring_used; i++) {
    if (i < dc.tring_aql.size() && dc.tring_aql[i] == -2) continue;  // (an AQL dispatch left untimed)
    if (i < dc.tring_aql.size() && dc.tring_aql[i] == -3) {  // a resident query: its span on the device
      ns.push_back(i < dc.tring_res.size() ? dc.tring_res[i] : 0);
      continue;
    }
    if (i < dc.tring_aql.size() && dc.tring_aql[i] >= 0 && dc.aql) {  // an AQL dispatch: its queue's timestamps
      ns.push_back(aql_time_ns(dc.aql, dc.tring_aql[i]));
      continue;
    }
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, dc.tring[2 * i], dc.tring[2 * i + 1]));
    ns.push_back(uint64_t(double(ms) * 1e6));
  }
  dc.tring_used = 0;
  if (dc.aql) aql_time_reset(dc.aql);
}

}  // namespace tsg
