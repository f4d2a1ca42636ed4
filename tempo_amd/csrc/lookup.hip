// lookup.hip — batched trace-ID lookup against v2 trace blocks on MI355X.
//
// Per probe id (one lane), for every block resident on the device, in block order:
//   includeBlock's id range check          tempodb/tempodb.go:492-511 (time window and
//                                          blockID shard range are per block: host)
//   bloom shard = FNV-1-32(id) % shards    tempodb/encoding/common/bloom.go:83-93
//   willf/bloom Test: 2 murmur3-x64-128 hashes (id, id||0x01), k probes
//                                          vendor/github.com/willf/bloom/bloom.go:94-124,182-190
//   index lower_bound over record ids      tempodb/encoding/v2/index_reader.go:85-114
// The id's hashes are computed once and reused across all blocks. Hits are
// emitted sorted by (id, block) with a count pass + decoupled look-back offsets
// and a write pass (the write pass recomputes: ALU is cheap, HBM is not).
//
// Bloom slabs. The k probe positions of an id depend only on (m, k) and its hashes,
// not on the block, so blocks whose blooms share (m, k, bitlen, shards) — every
// block a given config writes for a given object estimate — are probed together:
// per call their blooms are transposed into one table, slab[shard][bit] = a J-bit
// vector (bit j = block j's bloom bit). An id then costs k loads of J/8 bytes for
// the whole slab (J <= 256 blocks: 7 x 32 B for the default k), AND-ed, instead of
// up to k random loads per block; the surviving bits are the bloom-positive blocks.
// 200 blocks x 1 M probes: ~0.45 GB of slab reads instead of ~19 GB of bloom reads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "devctx.hpp"

namespace tsg {

struct LkBlock {
  const uint64_t *bloom;  // shards x words
  uint64_t words;         // words per shard
  uint64_t m, k, bitlen;  // per-block bloom parameters (shards are uniform within a block)
  uint64_t m_magic;       // floor(2^64 / m) for the Barrett reduction
  const uint8_t *rec_ids; // records x 16
  const uint64_t *rec_start;
  const uint32_t *rec_len;
  uint32_t shards, records;
  uint32_t min_len, max_len;
  uint32_t block_idx, dir_bits;
  const uint32_t *dir;    // index directory (V2Block::d_dir) or null
  uint64_t pfx[2], pmask[2];  // the records' common id prefix (dir_cp bytes, big-endian halves) and its mask
  uint64_t mn[2], mx[2];      // min_id / max_id zero-padded to 16 bytes, big-endian halves
  uint32_t dir_cp, pad;
};

struct LkSlab {
  const uint32_t *T;               // [shards][bitlen][W] u32
  uint64_t m, k, bitlen, m_magic;  // shared bloom parameters of the members
  uint32_t shards, W, J, first;    // W u32 per position; J members at slab_blk[first..]
};

struct LkParams {
  const LkBlock *blocks;
  uint32_t nblocks;
  const LkSlab *slabs;       // slab-probed blocks
  uint32_t nslabs, ndirect;
  const uint32_t *slab_blk;  // member block ordinals of every slab, in block order
  const uint32_t *direct;    // block ordinals probed one by one (ascending)
  const uint8_t *ids;
  uint64_t nids;
  uint32_t pair;  // slab probes two at a time (TSG_LK_PAIR=1; default one at a time)
  uint32_t smaj;  // kept hits slot-major, (block, record) pairs at hit_b as uint2 (hit j of id i at
                  // j * nids + i: a wave's stores of its ids' first hits land in adjacent words), or
                  // id-major in hit_b / hit_r (i * kHitK + j, TSG_LK_SLOTMAJOR=0)
  unsigned long long epoch, ticket_base;
  unsigned long long *ticket, *gran;
  uint64_t *offsets;  // per id: first output slot
  uint64_t *total;
  uint32_t *err;
  // the count pass keeps each id's first kHitK hits (block ordinal, record): the write
  // pass copies them instead of probing every block again (more hits: it re-probes)
  uint32_t *hit_cnt, *hit_b;
  int32_t *hit_r;
  // write pass
  uint32_t *o_id, *o_block;
  int32_t *o_rec;
  uint64_t *o_start;
  uint32_t *o_len;
  // the write pass places its columns itself (o_* = obase + total x column offsets, total read
  // from the count pass's *total), so the host need not read the total between the passes; a
  // total above ocap (or a count pass that failed) writes nothing and the host relaunches
  uint8_t *obase;
  uint64_t ocap;
};

__device__ __forceinline__ uint64_t d_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t d_fmix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
// murmur3 x64-128 (murmur128.go:62-200) of 16 bytes (one block, no tail) and of
// 17 bytes (one block + 1-byte tail 0x01): the block rounds are shared.
__device__ __forceinline__ void d_hashes(const uint64_t a, const uint64_t b, uint64_t h[4]) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 0, h2 = 0;
  h1 ^= d_rotl(a * c1, 31) * c2;
  h1 = (d_rotl(h1, 27) + h2) * 5 + 0x52dce729;
  h2 ^= d_rotl(b * c2, 33) * c1;
  h2 = (d_rotl(h2, 31) + h1) * 5 + 0x38495ab5;
  // Sum128 over 16 bytes
  {
    uint64_t x1 = h1 ^ 16, x2 = h2 ^ 16;
    x1 += x2;
    x2 += x1;
    x1 = d_fmix(x1);
    x2 = d_fmix(x2);
    x1 += x2;
    x2 += x1;
    h[0] = x1;
    h[1] = x2;
  }
  // Sum128 over 17 bytes: tail k1 = 0x01
  {
    uint64_t y1 = h1 ^ (d_rotl(1ULL * c1, 31) * c2), y2 = h2;
    y1 ^= 17;
    y2 ^= 17;
    y1 += y2;
    y2 += y1;
    y1 = d_fmix(y1);
    y2 = d_fmix(y2);
    y1 += y2;
    y2 += y1;
    h[2] = y1;
    h[3] = y2;
  }
}
__device__ __forceinline__ uint64_t d_mod(uint64_t x, uint64_t m, uint64_t magic) {
  uint64_t q = __umul64hi(x, magic);
  uint64_t r = x - q * m;
  while (r >= m) r -= m;
  return r;
}

// includeBlock's id range + index lower_bound: first record with
// bytes.Compare(rec.ID, id) >= 0 (pkg/sort/search.go:5-24), a hit if < TotalRecords.
// With a directory the search starts in the id's bucket: every record of an earlier
// bucket is below the id and every record of a later one above it, so the lower bound
// lies in [dir[b], dir[b+1]] — the same record sort.Search finds over the whole index,
// after ~2 line fetches instead of the ~6 bottom levels of a 1.6 MB binary search
// that miss L2 (trace ids are uniform hashes: a handful of records per bucket).
__device__ __forceinline__ uint64_t d_bswap64(uint64_t x) { return __builtin_bswap64(x); }
// bytes.Compare of two 16-byte ids held as big-endian halves
__device__ __forceinline__ int d_cmp128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
  if (ah != bh) return ah < bh ? -1 : 1;
  if (al != bl) return al < bl ? -1 : 1;
  return 0;
}
__device__ __forceinline__ int32_t d_post(const LkBlock &B, const uint8_t *id) {
  // the id as a 128-bit big-endian number (constant byte indices: stays in registers)
  uint64_t ihi = 0, ilo = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    ihi = (ihi << 8) | id[q];
    ilo = (ilo << 8) | id[8 + q];
  }
  // bytes.Compare(id, min/max) with the meta ids zero-padded to 16 bytes: equal padded
  // means equal first len bytes, and then the 16-byte id is the longer, greater one
  int cmin = d_cmp128(ihi, ilo, B.mn[0], B.mn[1]);
  if (cmin == 0 && B.min_len < 16) cmin = 1;
  int cmax = d_cmp128(ihi, ilo, B.mx[0], B.mx[1]);
  if (cmax == 0 && B.max_len < 16) cmax = 1;
  if (cmin < 0 || cmax > 0) return -1;
  uint32_t lo = 0, hi = B.records;
  if (B.dir) {
    const uint64_t mhi = B.pmask[0], mlo = B.pmask[1];
    const uint64_t ph = B.pfx[0], pl = B.pfx[1];
    if ((ihi & mhi) != ph) return (ihi & mhi) < ph ? (B.records ? 0 : -1) : -1;  // below / above every record
    if ((ilo & mlo) != pl) return (ilo & mlo) < pl ? (B.records ? 0 : -1) : -1;
    const uint32_t s = 8 * B.dir_cp;  // the 32 id bits after the prefix
    const uint64_t top = s == 0 ? ihi : s < 64 ? (ihi << s) | (ilo >> (64 - s)) : ilo << (s - 64);
    const uint32_t bk = uint32_t(top >> 32) >> (32 - B.dir_bits);
    lo = B.dir[bk];
    hi = B.dir[bk + 1];
  }
  while (lo < hi) {  // (a record is one 16-byte load)
    const uint32_t mid = (lo + hi) >> 1;
    const uint4 v = *reinterpret_cast<const uint4 *>(B.rec_ids + uint64_t(mid) * 16);
    const uint64_t rh = d_bswap64(uint64_t(v.x) | uint64_t(v.y) << 32), rl = d_bswap64(uint64_t(v.z) | uint64_t(v.w) << 32);
    if (d_cmp128(rh, rl, ihi, ilo) < 0) lo = mid + 1;
    else hi = mid;
  }
  return lo < B.records ? int32_t(lo) : -1;
}

// evaluates one (id, block) against the block's own bloom: record index (>= 0) on a
// hit, -1 otherwise (the range check and the bloom are both required: order is free)
__device__ __forceinline__ int32_t d_probe(const LkBlock &B, const uint8_t *id, uint32_t fnv, const uint64_t h[4]) {
  uint32_t shard = fnv % B.shards;
  const uint64_t *w = B.bloom + uint64_t(shard) * B.words;
  for (uint64_t i = 0; i < B.k; i++) {
    uint64_t loc = d_mod(h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) / 2)], B.m, B.m_magic);
    if (loc >= B.bitlen) return -1;
    if (!((w[loc >> 6] >> (loc & 63)) & 1ULL)) return -1;
  }
  return d_post(B, id);
}

// Calls f(block ordinal, record) for every hit of one id: slab members first (each
// slab in block order), then the directly probed blocks. Not globally block-ordered
// when several sources interleave: the write pass sorts each id's range.
template <class F>
__device__ __forceinline__ void for_each_hit(const LkParams &P, const uint8_t *id, uint32_t fnv, const uint64_t h[4], F &&f) {
  for (uint32_t si = 0; si < P.nslabs; si++) {
    const LkSlab &S = P.slabs[si];
    const uint32_t W = S.W;
    const uint32_t *base = S.T + uint64_t(fnv % S.shards) * S.bitlen * W;
    uint32_t v[8];
#pragma unroll
    for (int q = 0; q < 8; q++)  // (columns past J are zero in the table too)
      v[q] = uint32_t(q) * 32 >= S.J ? 0u : uint32_t(q + 1) * 32 <= S.J ? ~0u : (1u << (S.J % 32)) - 1u;
    // Probes go out two at a time with an early exit after each pair (issuing all k loads
    // up front needs ~130 VGPRs, and at 3 waves/SIMD the count pass measured 2.35 ms vs
    // 1.74 ms for the one-at-a-time chain, config 5). A pair's second position repeats the
    // first past k: AND is idempotent. P.pair = 0: the one-at-a-time chain.
    if (P.pair) {
      for (uint64_t i = 0; i < S.k; i += 2) {
        const uint64_t i1 = i + 1 < S.k ? i + 1 : i;
        const uint64_t l0 = d_mod(h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) / 2)], S.m, S.m_magic);
        const uint64_t l1 = d_mod(h[i1 % 2] + i1 * h[2 + (((i1 + (i1 % 2)) % 4) / 2)], S.m, S.m_magic);
        if (l0 >= S.bitlen || l1 >= S.bitlen) {
#pragma unroll
          for (int q = 0; q < 8; q++) v[q] = 0;
          break;
        }
        const uint32_t *p0 = base + l0 * W, *p1 = base + l1 * W;
        if (W == 8) {
          const uint4 a0 = *reinterpret_cast<const uint4 *>(p0), b0 = *reinterpret_cast<const uint4 *>(p0 + 4);
          const uint4 a1 = *reinterpret_cast<const uint4 *>(p1), b1 = *reinterpret_cast<const uint4 *>(p1 + 4);
          v[0] &= a0.x & a1.x; v[1] &= a0.y & a1.y; v[2] &= a0.z & a1.z; v[3] &= a0.w & a1.w;
          v[4] &= b0.x & b1.x; v[5] &= b0.y & b1.y; v[6] &= b0.z & b1.z; v[7] &= b0.w & b1.w;
        } else if (W == 4) {
          const uint4 a0 = *reinterpret_cast<const uint4 *>(p0), a1 = *reinterpret_cast<const uint4 *>(p1);
          v[0] &= a0.x & a1.x; v[1] &= a0.y & a1.y; v[2] &= a0.z & a1.z; v[3] &= a0.w & a1.w;
        } else if (W == 2) {
          const uint2 a0 = *reinterpret_cast<const uint2 *>(p0), a1 = *reinterpret_cast<const uint2 *>(p1);
          v[0] &= a0.x & a1.x; v[1] &= a0.y & a1.y;
        } else {
          v[0] &= p0[0] & p1[0];
        }
        uint32_t any = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) any |= v[q];
        if (!any) break;
      }
    } else
    for (uint64_t i = 0; i < S.k; i++) {
      uint64_t loc = d_mod(h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) / 2)], S.m, S.m_magic);
      if (loc >= S.bitlen) {
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = 0;
        break;
      }
      const uint32_t *p = base + loc * W;
      if (W == 8) {
        uint4 a = *reinterpret_cast<const uint4 *>(p), b = *reinterpret_cast<const uint4 *>(p + 4);
        v[0] &= a.x; v[1] &= a.y; v[2] &= a.z; v[3] &= a.w;
        v[4] &= b.x; v[5] &= b.y; v[6] &= b.z; v[7] &= b.w;
      } else if (W == 4) {
        uint4 a = *reinterpret_cast<const uint4 *>(p);
        v[0] &= a.x; v[1] &= a.y; v[2] &= a.z; v[3] &= a.w;
      } else if (W == 2) {
        uint2 a = *reinterpret_cast<const uint2 *>(p);
        v[0] &= a.x; v[1] &= a.y;
      } else {
        v[0] &= p[0];
      }
      uint32_t any = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) any |= v[q];
      if (!any) break;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      uint32_t x = v[q];
      while (x) {
        const uint32_t j = uint32_t(q) * 32 + uint32_t(__builtin_ctz(x));
        x &= x - 1;
        const uint32_t b = P.slab_blk[S.first + j];
        const int32_t r = d_post(P.blocks[b], id);
        if (r >= 0) f(b, r);
      }
    }
  }
  for (uint32_t di = 0; di < P.ndirect; di++) {
    const uint32_t b = P.direct[di];
    const int32_t r = d_probe(P.blocks[b], id, fnv, h);
    if (r >= 0) f(b, r);
  }
}

// slab[s][pos][jc] bit j = bloom bit pos of shard s of member jc*32+j. One thread per
// (shard, 64-bit word, 32-member column): 32 words in registers, 64 positions out.
struct TrParams {
  const uint64_t *const *bloom;  // member bloom words (shards x words), J entries
  uint32_t *T;
  uint64_t words, bitlen;
  uint32_t shards, W, J;
};
extern "C" __global__ void __launch_bounds__(256) lookup_transpose_kernel(TrParams P) {
  const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint32_t jc = uint32_t(g % P.W);
  const uint64_t rest = g / P.W;
  const uint64_t w = rest % P.words, s = rest / P.words;
  if (s >= P.shards) return;
  uint64_t x[32];
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const uint32_t mj = jc * 32 + uint32_t(j);
    x[j] = mj < P.J ? P.bloom[mj][s * P.words + w] : 0ULL;
  }
  uint32_t *out = P.T + (s * P.bitlen + w * 64) * P.W + jc;
  const uint32_t nq = uint32_t(min<uint64_t>(64, P.bitlen - w * 64));
  for (uint32_t q = 0; q < nq; q++) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) o |= uint32_t((x[j] >> q) & 1ULL) << j;
    out[uint64_t(q) * P.W] = o;
  }
}

// The same table, the 32 x 64 bit block of a thread transposed as two 32 x 32 bit matrices with
// log2(32) = 5 rounds of masked swaps (each round swaps the off-diagonal j x j blocks of every
// 2j x 2j block), ~400 ALU ops per 1024 bits instead of one shift-and-or per bit.
__device__ __forceinline__ void d_tr32(uint32_t (&A)[32]) {
  uint32_t m = 0x0000FFFFu;
#pragma unroll
  for (int j = 16; j; j >>= 1, m ^= (m << j)) {
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 2 * j)
#pragma unroll
      for (int k = k0; k < k0 + j; k++) {
        const uint32_t t = ((A[k] >> j) ^ A[k + j]) & m;
        A[k + j] ^= t;
        A[k] ^= t << j;
      }
  }
}
extern "C" __global__ void __launch_bounds__(256) lookup_transpose2_kernel(TrParams P) {
  const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint32_t jc = uint32_t(g % P.W);
  const uint64_t rest = g / P.W;
  const uint64_t w = rest % P.words, s = rest / P.words;
  if (s >= P.shards) return;
  uint32_t lo[32], hi[32];
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const uint32_t mj = jc * 32 + uint32_t(j);
    const uint64_t x = mj < P.J ? P.bloom[mj][s * P.words + w] : 0ULL;
    lo[j] = uint32_t(x);
    hi[j] = uint32_t(x >> 32);
  }
  d_tr32(lo);
  d_tr32(hi);
  uint32_t *out = P.T + (s * P.bitlen + w * 64) * P.W + jc;
  const uint32_t nq = uint32_t(min<uint64_t>(64, P.bitlen - w * 64));
#pragma unroll
  for (int q = 0; q < 32; q++)
    if (uint32_t(q) < nq) out[uint64_t(q) * P.W] = lo[q];
#pragma unroll
  for (int q = 0; q < 32; q++)
    if (uint32_t(q) + 32 < nq) out[uint64_t(q + 32) * P.W] = hi[q];
}

constexpr int kLkThreads = 256;
constexpr uint32_t kHitK = 4;
constexpr unsigned long long kGAgg = 1, kGInc = 2;

__device__ __forceinline__ void d_id_hash(const uint8_t *id, uint32_t &fnv, uint64_t h[4]) {
  uint32_t f = 2166136261u;
  for (int i = 0; i < 16; i++) f = (f * 16777619u) ^ id[i];
  fnv = f;
  uint64_t a, b;
  memcpy(&a, id, 8);
  memcpy(&b, id + 8, 8);
  d_hashes(a, b, h);
}

template <bool NT>
__device__ __forceinline__ void lookup_count_body(const LkParams &P) {
  __shared__ uint32_t s_tile;
  __shared__ unsigned long long s_w[kLkThreads / 64], s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) s_tile = uint32_t(atomicAdd(P.ticket, 1ULL) - P.ticket_base);
  __syncthreads();
  const uint32_t t = __builtin_amdgcn_readfirstlane(s_tile);
  const uint64_t i = uint64_t(t) * kLkThreads + tid;
  uint32_t cnt = 0;
  if (i < P.nids) {
    uint8_t id[16];
    if (NT) {  // (streamed once: kept out of L2, which holds what it can of the slab table)
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(P.ids) + i);
#pragma unroll
      for (int q = 0; q < 16; q++) id[q] = uint8_t(w[q / 4] >> (8 * (q % 4)));
    } else {
      memcpy(id, P.ids + i * 16, 16);
    }
    uint32_t fnv;
    uint64_t h[4];
    d_id_hash(id, fnv, h);
    for_each_hit(P, id, fnv, h, [&](uint32_t b, int32_t r) {
      if (cnt < kHitK) {
        if (P.smaj) {  // (block and record in one 8-byte store)
          reinterpret_cast<uint2 *>(P.hit_b)[uint64_t(cnt) * P.nids + i] = make_uint2(b, uint32_t(r));
        } else {
          P.hit_b[i * kHitK + cnt] = b;
          P.hit_r[i * kHitK + cnt] = r;
        }
      }
      cnt++;
    });
    if (NT) __builtin_nontemporal_store(cnt, P.hit_cnt + i);
    else P.hit_cnt[i] = cnt;
  }
  // block scan of counts
  unsigned long long v = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    unsigned long long o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  if (lane == 63) s_w[wid] = v;
  __syncthreads();
  unsigned long long before = 0, tot = 0;
  for (int w = 0; w < kLkThreads / 64; w++) {
    if (w < wid) before += s_w[w];
    tot += s_w[w];
  }
  if (wid == 0) {
    unsigned long long excl = 0;
    auto mk = [&](unsigned long long st, unsigned long long val) { return (P.epoch << 40) | (st << 38) | val; };
    if (t == 0) {
      if (lane == 0) __hip_atomic_store(&P.gran[t], mk(kGInc, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&P.gran[t], mk(kGAgg, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t end = t;
      uint32_t spins = 0;
      bool timeout = false;
      for (;;) {
        int64_t j = end - 1 - lane;
        unsigned long long g = j < 0 ? mk(kGInc, 0) : __hip_atomic_load(&P.gran[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ready = (g >> 40) == P.epoch;
        while (!__all(ready)) {
          if (++spins > (1u << 22)) {
            timeout = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if (!ready) {
            g = __hip_atomic_load(&P.gran[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ready = (g >> 40) == P.epoch;
          }
        }
        if (timeout) {
          if (lane == 0) atomicOr(P.err, 1u);
          break;
        }
        unsigned long long im = __ballot(((g >> 38) & 3ULL) == kGInc);
        int first = im ? __builtin_ctzll(im) : 64;
        unsigned long long x = lane <= first ? (g & ((1ULL << 38) - 1)) : 0ULL;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
        excl += x;
        if (im) break;
        end -= 64;
      }
      if (lane == 0) __hip_atomic_store(&P.gran[t], mk(kGInc, excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_excl = excl;
      if (uint64_t(t + 1) * kLkThreads >= P.nids) *P.total = excl + tot;
    }
  }
  __syncthreads();
  if (i < P.nids) {
    if (NT) __builtin_nontemporal_store(uint64_t(s_excl + before + v - cnt), P.offsets + i);
    else P.offsets[i] = s_excl + before + v - cnt;
  }
}
extern "C" __global__ void __launch_bounds__(kLkThreads) lookup_count_kernel(LkParams P) { lookup_count_body<false>(P); }
// the same pass at more waves per SIMD: 72 VGPRs and 7 waves, no spills (the default; config 5
// 2.07 vs 2.12-2.13 ms per call at 6 waves, 2.13 at 8 waves with 48 B of spills per lane —
// profiles/r06_lookup; TSG_LK_OCC=6 / 8 select the others)
extern "C" __global__ void __launch_bounds__(kLkThreads) __attribute__((amdgpu_waves_per_eu(7)))
lookup_count_kernel_w7(LkParams P) {
  lookup_count_body<false>(P);
}
// ids loaded and counts / offsets stored non-temporally (experiment, TSG_LK_OCC=17)
extern "C" __global__ void __launch_bounds__(kLkThreads) __attribute__((amdgpu_waves_per_eu(7)))
lookup_count_kernel_w7nt(LkParams P) {
  lookup_count_body<true>(P);
}
extern "C" __global__ void __launch_bounds__(kLkThreads) __attribute__((amdgpu_waves_per_eu(8)))
lookup_count_kernel_w8(LkParams P) {
  lookup_count_body<false>(P);
}

extern "C" __global__ void __launch_bounds__(kLkThreads) lookup_write_kernel(LkParams P) {
  const uint64_t i = uint64_t(blockIdx.x) * kLkThreads + threadIdx.x;
  if (i >= P.nids) return;
  if (P.obase) {
    const uint64_t total = __builtin_amdgcn_readfirstlane(uint32_t(*P.total)) |
                           uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(*P.total >> 32))) << 32;
    if (total > P.ocap || *P.err) return;
    P.o_start = reinterpret_cast<uint64_t *>(P.obase);
    P.o_id = reinterpret_cast<uint32_t *>(P.obase + total * 8);
    P.o_block = reinterpret_cast<uint32_t *>(P.obase + total * 12);
    P.o_rec = reinterpret_cast<int32_t *>(P.obase + total * 16);
    P.o_len = reinterpret_cast<uint32_t *>(P.obase + total * 20);
  }
  const uint32_t cnt = P.hit_cnt[i];
  const uint64_t o0 = P.offsets[i];
  if (cnt <= kHitK) {  // every hit was kept by the count pass: sort by block, copy
    uint32_t hb[kHitK];
    int32_t hr[kHitK];
    for (uint32_t j = 0; j < cnt; j++) {
      if (P.smaj) {
        const uint2 br = reinterpret_cast<const uint2 *>(P.hit_b)[uint64_t(j) * P.nids + i];
        hb[j] = br.x;
        hr[j] = int32_t(br.y);
      } else {
        hb[j] = P.hit_b[i * kHitK + j];
        hr[j] = P.hit_r[i * kHitK + j];
      }
      for (uint32_t q = j; q > 0 && hb[q - 1] > hb[q]; q--) {
        uint32_t tb = hb[q]; hb[q] = hb[q - 1]; hb[q - 1] = tb;
        int32_t tr = hr[q]; hr[q] = hr[q - 1]; hr[q - 1] = tr;
      }
    }
    for (uint32_t j = 0; j < cnt; j++) {
      const LkBlock &B = P.blocks[hb[j]];
      const int32_t r = hr[j];
      P.o_id[o0 + j] = uint32_t(i);
      P.o_block[o0 + j] = B.block_idx;
      P.o_rec[o0 + j] = r;
      P.o_start[o0 + j] = B.rec_start[r];
      P.o_len[o0 + j] = B.rec_len[r];
    }
    return;
  }
  uint8_t id[16];
  memcpy(id, P.ids + i * 16, 16);
  uint32_t fnv;
  uint64_t h[4];
  d_id_hash(id, fnv, h);
  uint64_t o = o0;
  for_each_hit(P, id, fnv, h, [&](uint32_t b, int32_t r) {
    const LkBlock &B = P.blocks[b];
    P.o_id[o] = uint32_t(i);
    P.o_block[o] = B.block_idx;
    P.o_rec[o] = r;
    P.o_start[o] = B.rec_start[r];
    P.o_len[o] = B.rec_len[r];
    o++;
  });
  // sources interleave in block order: insertion sort of this id's range by block
  for (uint64_t a = o0 + 1; a < o; a++) {
    const uint32_t kb = P.o_block[a];
    const int32_t kr = P.o_rec[a];
    const uint64_t ks = P.o_start[a];
    const uint32_t kl = P.o_len[a];
    uint64_t q = a;
    for (; q > o0 && P.o_block[q - 1] > kb; q--) {
      P.o_block[q] = P.o_block[q - 1];
      P.o_rec[q] = P.o_rec[q - 1];
      P.o_start[q] = P.o_start[q - 1];
      P.o_len[q] = P.o_len[q - 1];
    }
    P.o_block[q] = kb;
    P.o_rec[q] = kr;
    P.o_start[q] = ks;
    P.o_len[q] = kl;
  }
}

// ------------------------------------------------------------------------------------
// host
static void *dalloc(V2Block &b, size_t bytes) {
  void *p = nullptr;
  HIP_OK(hipMalloc(&p, std::max<size_t>(bytes, 16)));
  b.allocs.push_back(p);
  return p;
}

void v2block_open(Ctx &c, V2Block &b, const std::string &dir, int device_hint) {
  if (c.devs.empty()) fail(TSG_E_DEVICE, "no device");
  DeviceCtx &dc = *c.devs[size_t(std::max(device_hint, 0)) % c.devs.size()];
  b.dc = &dc;
  b.device = device_ordinal(dc);
  std::vector<uint8_t> meta;
  if (!read_file(dir + "/meta.json", meta)) fail(TSG_E_NOT_FOUND, "meta.json not found");
  std::string js(meta.begin(), meta.end());
  auto field = [&](const char *name) -> std::string {
    std::string pat = std::string("\"") + name + "\"";
    size_t p = js.find(pat);
    if (p == std::string::npos) return "";
    p += pat.size();
    while (p < js.size() && (js[p] == ':' || js[p] == ' ')) p++;
    if (js[p] == '"') {
      size_t e = js.find('"', p + 1);
      return js.substr(p + 1, e - p - 1);
    }
    size_t e = p;
    while (e < js.size() && js[e] != ',' && js[e] != '}') e++;
    return js.substr(p, e - p);
  };
  auto b64 = [](const std::string &s) {
    std::vector<uint8_t> o;
    uint32_t acc = 0;
    int bits = 0;
    for (char ch : s) {
      int v = (ch >= 'A' && ch <= 'Z') ? ch - 'A' : (ch >= 'a' && ch <= 'z') ? ch - 'a' + 26
              : (ch >= '0' && ch <= '9') ? ch - '0' + 52 : ch == '+' ? 62 : ch == '/' ? 63 : -1;
      if (v < 0) continue;
      acc = (acc << 6) | uint32_t(v);
      bits += 6;
      if (bits >= 8) {
        bits -= 8;
        o.push_back(uint8_t(acc >> bits));
      }
    }
    return o;
  };
  auto rfc3339 = [](const std::string &s) -> int64_t {  // time.Time.Unix()
    int Y, M, D, h, mi, se;
    if (std::sscanf(s.c_str(), "%d-%d-%dT%d:%d:%d", &Y, &M, &D, &h, &mi, &se) != 6) return 0;
    size_t p = s.find('T') + 9;
    if (p < s.size() && s[p] == '.')
      do p++; while (p < s.size() && s[p] >= '0' && s[p] <= '9');
    int64_t off = 0;
    if (p < s.size() && (s[p] == '+' || s[p] == '-')) {
      int oh = 0, om = 0;
      std::sscanf(s.c_str() + p + 1, "%d:%d", &oh, &om);
      off = (oh * 3600 + om * 60) * (s[p] == '-' ? -1 : 1);
    }
    int64_t y = Y - (M <= 2);
    int64_t era = (y >= 0 ? y : y - 399) / 400;
    unsigned yoe = unsigned(y - era * 400);
    unsigned doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
    unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    int64_t days = era * 146097 + int64_t(doe) - 719468;
    return days * 86400 + h * 3600 + mi * 60 + se - off;
  };
  b.min_id = b64(field("minID"));
  b.max_id = b64(field("maxID"));
  if (b.min_id.size() > 16 || b.max_id.size() > 16) fail(TSG_E_UNSUPPORTED, "min/max id longer than 16 bytes");
  b.start_unix = rfc3339(field("startTime"));
  b.end_unix = rfc3339(field("endTime"));
  {
    std::string u = field("blockID");
    int nib = 0;
    std::memset(b.block_id, 0, 16);
    for (char ch : u) {
      int v = (ch >= '0' && ch <= '9') ? ch - '0' : (ch >= 'a' && ch <= 'f') ? ch - 'a' + 10
              : (ch >= 'A' && ch <= 'F') ? ch - 'A' + 10 : -1;
      if (v < 0 || nib >= 32) continue;
      b.block_id[nib / 2] |= uint8_t(nib % 2 == 0 ? v << 4 : v);
      nib++;
    }
  }
  std::string enc = field("encoding");
  std::string ips = field("indexPageSize"), tr = field("totalRecords"), bs = field("bloomShards");
  uint32_t page_size = ips.empty() ? 0 : uint32_t(std::stoul(ips));
  b.total_records = tr.empty() ? 0 : uint32_t(std::stoul(tr));
  uint32_t shards = bs.empty() ? 0 : uint32_t(std::stoul(bs));
  b.shards = shards ? shards : 10;  // ValidateShardCount (bloom.go:88-93)
  // blooms (big-endian willf serialisation)
  std::vector<uint64_t> words;
  for (uint32_t s = 0; s < b.shards; s++) {
    std::vector<uint8_t> f;
    if (!read_file(dir + "/bloom-" + std::to_string(s), f)) fail(TSG_E_IO, "bloom shard missing");
    if (f.size() < 24) fail(TSG_E_CORRUPT, "bloom too small");
    uint64_t m = be64(f.data()), k = be64(f.data() + 8), bitlen = be64(f.data() + 16);
    uint64_t nw = (bitlen + 63) / 64;
    if (24 + nw * 8 > f.size()) fail(TSG_E_CORRUPT, "bloom truncated");
    if (m == 0) fail(TSG_E_CORRUPT, "bloom m == 0");
    if (s == 0) {
      b.bloom_m = m;
      b.bloom_k = k;
      b.bloom_bitlen = bitlen;
      b.bloom_words = nw;
    } else if (m != b.bloom_m || k != b.bloom_k || bitlen != b.bloom_bitlen) {
      fail(TSG_E_UNSUPPORTED, "bloom shards with differing parameters");
    }
    for (uint64_t w = 0; w < nw; w++) words.push_back(be64(f.data() + 24 + 8 * w));
  }
  std::vector<uint8_t> idx;
  if (!read_file(dir + "/index", idx)) fail(TSG_E_IO, "index missing");
  std::vector<IndexRecord> recs = read_index(idx.data(), idx.size(), page_size, b.total_records);
  std::vector<uint8_t> rid(recs.size() * 16);
  std::vector<uint64_t> rs(recs.size());
  std::vector<uint32_t> rl(recs.size());
  for (size_t i = 0; i < recs.size(); i++) {
    std::memcpy(&rid[i * 16], recs[i].id, 16);
    rs[i] = recs[i].start;
    rl[i] = recs[i].length;
  }
  // index directory (d_post): only over a sorted index (the writer's invariant; an
  // unsorted one keeps the plain binary search, whose answer the directory would not
  // reproduce). TSG_LK_DIR=0 turns it off.
  std::vector<uint32_t> rdir;
  static const bool dir_on = [] {
    const char *e = std::getenv("TSG_LK_DIR");
    return !e || std::atoi(e) != 0;
  }();
  const size_t n = recs.size();
  bool sorted = n == b.total_records;
  for (size_t i = 1; i < n && sorted; i++) sorted = std::memcmp(&rid[(i - 1) * 16], &rid[i * 16], 16) <= 0;
  if (dir_on && sorted && n >= 64) {
    uint32_t cp = 0;
    while (cp < 12 && rid[cp] == rid[(n - 1) * 16 + cp]) cp++;  // (sorted: every record shares it)
    uint32_t bits = 0;
    while ((size_t(2) << bits) <= n / 4 && bits < 20) bits++;  // ~4 records per bucket
    bits = std::max(bits, 1u);
    rdir.assign((size_t(1) << bits) + 1, uint32_t(n));
    auto bucket = [&](size_t r) {
      uint32_t key = 0;
      for (uint32_t q = 0; q < 4; q++) key = (key << 8) | rid[r * 16 + cp + q];
      return key >> (32 - bits);
    };
    size_t bk = 0;
    for (size_t r = 0; r < n; r++) {
      const size_t k = bucket(r);
      while (bk <= k) rdir[bk++] = uint32_t(r);
    }
    b.dir_bits = bits;
    b.dir_cp = cp;
    std::memcpy(b.dir_prefix, rid.data(), cp);
  }
  std::lock_guard<std::mutex> lk(dc.mu);
  HIP_OK(hipSetDevice(dc.ordinal));
  auto up = [&](const void *src, size_t bytes) {
    void *p = dalloc(b, bytes);
    if (bytes) HIP_OK(hipMemcpy(p, src, bytes, hipMemcpyHostToDevice));
    return p;
  };
  b.d_bloom = static_cast<uint64_t *>(up(words.data(), words.size() * 8));
  b.d_rec_ids = static_cast<uint8_t *>(up(rid.data(), rid.size()));
  b.d_rec_start = static_cast<uint64_t *>(up(rs.data(), rs.size() * 8));
  b.d_rec_len = static_cast<uint32_t *>(up(rl.data(), rl.size() * 4));
  if (!rdir.empty()) b.d_dir = static_cast<uint32_t *>(up(rdir.data(), rdir.size() * 4));
  // the data file for findOne on the device (pages stay compressed in HBM)
  b.enc = enc.empty() ? -1 : parse_encoding(enc);
  std::vector<uint8_t> data;
  if (!std::getenv("TSG_V2_NO_DATA") && read_file(dir + "/data", data)) {
    b.d_data = static_cast<const uint8_t *>(up(data.data(), data.size()));
    b.data_len = data.size();
  }
}

void v2block_free(V2Block &b) {
  if (!b.dc) return;
  std::lock_guard<std::mutex> lk(b.dc->mu);
  (void)hipSetDevice(b.dc->ordinal);
  (void)hipStreamSynchronize(b.dc->stream);
  for (void *p : b.allocs) (void)hipFree(p);
  b.allocs.clear();
  b.dc = nullptr;
}

// The caller's probe ids to the device. Pinned memory (registered or hipHostMalloc'd) goes by
// DMA as it is; a pageable buffer through two pinned staging chunks, the host's copy of chunk
// i + 1 (on several threads) overlapping chunk i's DMA (a pageable hipMemcpy of 160 MB of ids
// ran at a third of the link's rate, VERDICT r4 "What's weak" 5).
static void upload_ids(DeviceCtx &dc, uint8_t *dst, const uint8_t *src, size_t bytes, hipStream_t s) {
  if (!bytes) return;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, src) == hipSuccess && at.type == hipMemoryTypeHost) {
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return;
  }
  (void)hipGetLastError();  // (an unregistered pointer's lookup error)
  constexpr size_t kChunk = size_t(32) << 20;
  if (bytes <= (size_t(4) << 20)) {  // (small: one pageable copy)
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return;
  }
  dc.lkstage.ensure(2 * kChunk);
  for (auto &e : dc.lk_ev)
    if (!e) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  auto *base = static_cast<uint8_t *>(dc.lkstage.p);
  for (size_t off = 0, i = 0; off < bytes; off += kChunk, i++) {
    const size_t n = std::min(kChunk, bytes - off);
    uint8_t *stage = base + (i & 1) * kChunk;
    if (i >= 2) HIP_OK(hipEventSynchronize(dc.lk_ev[i & 1]));  // (the DMA that read this half is done)
    parallel_ranges(n, size_t(2) << 20, 8, [&](size_t lo, size_t hi) { std::memcpy(stage + lo, src + off + lo, hi - lo); });
    HIP_OK(hipMemcpyAsync(dst + off, stage, n, hipMemcpyHostToDevice, s));
    HIP_OK(hipEventRecord(dc.lk_ev[i & 1], s));
  }
}

void device_lookup(DeviceCtx &dc, const std::vector<std::pair<uint32_t, V2Block *>> &blocks, const uint8_t (*ids)[16],
                   size_t nids, const tsg_lookup_opts *opts, LookupOut &out) {
  std::lock_guard<std::mutex> lk(dc.mu);
  resident_quit(dc);  // (the resident search launch holds every CU's LDS)
  HIP_OK(hipSetDevice(dc.ordinal));
  hipStream_t s = dc.stream;
  // per-block prefilter that does not depend on the id (tempodb.go:497-509)
  std::vector<LkBlock> lb;
  for (auto &bp : blocks) {
    const V2Block &b = *bp.second;
    if (opts && opts->time_start != 0 && opts->time_end != 0)
      if (b.start_unix >= int64_t(opts->time_end) || b.end_unix <= int64_t(opts->time_start)) continue;
    if (opts && opts->block_start && opts->block_end)
      if (bytes_compare(b.block_id, 16, opts->block_start, 16) < 0 || bytes_compare(b.block_id, 16, opts->block_end, 16) > 0)
        continue;
    LkBlock k{};
    k.bloom = b.d_bloom;
    k.words = b.bloom_words;
    k.m = b.bloom_m;
    k.k = b.bloom_k;
    k.bitlen = b.bloom_bitlen;
    k.m_magic = uint64_t(~0ULL / k.m);  // floor((2^64-1)/m), m >= 1 (v2block_open): d_mod corrects by <= 2 steps
    k.rec_ids = b.d_rec_ids;
    k.rec_start = b.d_rec_start;
    k.rec_len = b.d_rec_len;
    k.shards = b.shards;
    k.records = b.total_records;
    k.min_len = uint32_t(b.min_id.size());
    for (uint32_t q = 0; q < 16; q++) {
      k.mn[q / 8] |= uint64_t(q < b.min_id.size() ? b.min_id[q] : 0u) << (56 - 8 * (q % 8));
      k.mx[q / 8] |= uint64_t(q < b.max_id.size() ? b.max_id[q] : 0u) << (56 - 8 * (q % 8));
    }
    k.max_len = uint32_t(b.max_id.size());
    k.block_idx = bp.first;
    if (b.d_dir) {
      k.dir = b.d_dir;
      k.dir_bits = b.dir_bits;
      k.dir_cp = b.dir_cp;
      for (uint32_t q = 0; q < 16; q++) {  // big-endian halves of the prefix and its mask
        const uint64_t byte = q < b.dir_cp ? b.dir_prefix[q] : 0u, m = q < b.dir_cp ? 0xffu : 0u;
        k.pfx[q / 8] |= byte << (56 - 8 * (q % 8));
        k.pmask[q / 8] |= m << (56 - 8 * (q % 8));
      }
    }
    lb.push_back(k);
  }
  out = LookupOut();
  if (nids == 0 || lb.empty()) return;
  uint32_t tiles = uint32_t((nids + kLkThreads - 1) / kLkThreads);

  // ---- slabs: blocks with identical bloom parameters, up to 256 per slab, when the
  // probes they save outweigh building the table (TSG_LK_SLAB=0/1 forces it off/on)
  const char *slab_env = std::getenv("TSG_LK_SLAB");
  const int slab_mode = slab_env ? std::atoi(slab_env) : -1;
  std::vector<LkSlab> slabs;
  std::vector<uint32_t> slab_blk, direct;
  std::vector<std::vector<uint32_t>> members;  // per slab: lb ordinals
  {
    std::vector<bool> used(lb.size(), false);
    for (size_t a = 0; a < lb.size(); a++) {
      if (used[a]) continue;
      std::vector<uint32_t> grp;
      for (size_t b = a; b < lb.size(); b++)
        if (!used[b] && lb[b].m == lb[a].m && lb[b].k == lb[a].k && lb[b].bitlen == lb[a].bitlen &&
            lb[b].shards == lb[a].shards && lb[b].words == lb[a].words) {
          grp.push_back(uint32_t(b));
          used[b] = true;
        }
      for (size_t g0 = 0; g0 < grp.size(); g0 += 256) {
        std::vector<uint32_t> part(grp.begin() + long(g0), grp.begin() + long(std::min(grp.size(), g0 + 256)));
        const uint64_t J = part.size();
        const uint32_t W = J <= 32 ? 1 : J <= 64 ? 2 : J <= 128 ? 4 : 8;
        const double table = double(lb[a].shards) * double(lb[a].bitlen) * W * 4;
        const double blooms = double(J) * lb[a].shards * lb[a].words * 8;
        const bool use = slab_mode == 1 ? true : slab_mode == 0 ? false
                                                : (J >= 2 && double(nids) * double(J) * 96.0 >= 2.0 * (table + blooms));
        if (!use) {
          for (uint32_t b : part) direct.push_back(b);
          continue;
        }
        LkSlab sl{};
        sl.m = lb[a].m;
        sl.k = lb[a].k;
        sl.bitlen = lb[a].bitlen;
        sl.m_magic = lb[a].m_magic;
        sl.shards = lb[a].shards;
        sl.W = W;
        sl.J = uint32_t(J);
        sl.first = uint32_t(slab_blk.size());
        for (uint32_t b : part) slab_blk.push_back(b);
        slabs.push_back(sl);
        members.push_back(part);
      }
    }
    std::sort(direct.begin(), direct.end());
  }
  std::vector<size_t> slab_off(slabs.size());
  size_t slab_bytes = 0;
  for (size_t i = 0; i < slabs.size(); i++) {
    slab_off[i] = slab_bytes;
    slab_bytes += (size_t(slabs[i].shards) * slabs[i].bitlen * slabs[i].W * 4 + 255) & ~size_t(255);
  }
  if (slab_bytes) dc.lkslab.ensure(slab_bytes);
  for (size_t i = 0; i < slabs.size(); i++)
    slabs[i].T = reinterpret_cast<const uint32_t *>(static_cast<uint8_t *>(dc.lkslab.p) + slab_off[i]);

  // descriptor area: LkBlock[] | LkSlab[] | slab_blk[] | direct[] | member bloom ptrs | ids
  auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
  const size_t o_slab = al(lb.size() * sizeof(LkBlock));
  const size_t o_sblk = o_slab + al(slabs.size() * sizeof(LkSlab));
  const size_t o_dir = o_sblk + al(slab_blk.size() * 4);
  const size_t o_bptr = o_dir + al(direct.size() * 4);
  const size_t desc_bytes = o_bptr + al(slab_blk.size() * 8);
  dc.desc.ensure(desc_bytes + nids * 16);
  dc.hdesc.ensure(desc_bytes);
  auto *hd = static_cast<uint8_t *>(dc.hdesc.p);
  std::memcpy(hd, lb.data(), lb.size() * sizeof(LkBlock));
  if (!slabs.empty()) std::memcpy(hd + o_slab, slabs.data(), slabs.size() * sizeof(LkSlab));
  if (!slab_blk.empty()) std::memcpy(hd + o_sblk, slab_blk.data(), slab_blk.size() * 4);
  if (!direct.empty()) std::memcpy(hd + o_dir, direct.data(), direct.size() * 4);
  for (size_t i = 0; i < slab_blk.size(); i++) {
    const uint64_t *bp = lb[slab_blk[i]].bloom;
    std::memcpy(hd + o_bptr + i * 8, &bp, 8);
  }
  auto *dd = static_cast<uint8_t *>(dc.desc.p);
  HIP_OK(hipMemcpyAsync(dd, hd, desc_bytes, hipMemcpyHostToDevice, s));
  upload_ids(dc, dd + desc_bytes, reinterpret_cast<const uint8_t *>(ids), nids * 16, s);
  if (dc.gran_tiles < tiles) {
    HIP_OK(hipStreamSynchronize(s));
    dc.gran.ensure(size_t(tiles) * 8 * 2);
    HIP_OK(hipMemsetAsync(dc.gran.p, 0, dc.gran.cap, s));
    dc.gran_tiles = dc.gran.cap / 8;
  }
  dc.vmatch.ensure(nids * 8);  // per-id offsets
  dc.hdr.ensure(64);
  dc.epoch = (dc.epoch + 1) & 0xffffffULL;
  if (dc.epoch == 0) dc.epoch = 1;
  LkParams P{};
  P.blocks = reinterpret_cast<const LkBlock *>(dd);
  P.nblocks = uint32_t(lb.size());
  P.slabs = reinterpret_cast<const LkSlab *>(dd + o_slab);
  P.nslabs = uint32_t(slabs.size());
  P.slab_blk = reinterpret_cast<const uint32_t *>(dd + o_sblk);
  P.direct = reinterpret_cast<const uint32_t *>(dd + o_dir);
  P.ndirect = uint32_t(direct.size());
  P.ids = dd + desc_bytes;
  P.nids = nids;
  static const uint32_t pair = [] {
    const char *e = std::getenv("TSG_LK_PAIR");
    return e ? uint32_t(std::atoi(e) != 0) : 0u;  // (pairs: 2.18 vs 2.15 ms per config-5 step, profiles/r03_lookup)
  }();
  P.pair = pair;
  static const uint32_t smaj = [] {
    const char *e = std::getenv("TSG_LK_SLOTMAJOR");
    return e ? uint32_t(std::atoi(e) != 0) : 1u;
  }();
  P.smaj = smaj;
  P.epoch = dc.epoch;
  P.ticket_base = dc.ticket_base;
  P.ticket = static_cast<unsigned long long *>(dc.ticket.p);
  P.gran = static_cast<unsigned long long *>(dc.gran.p);
  P.offsets = static_cast<uint64_t *>(dc.vmatch.p);
  P.total = static_cast<uint64_t *>(dc.hdr.p);
  P.err = static_cast<uint32_t *>(dc.err.p);
  dc.lkhits.ensure((std::max<uint64_t>(nids, 1) + 1) * (4 + kHitK * 8));
  P.hit_cnt = static_cast<uint32_t *>(dc.lkhits.p);
  P.hit_b = P.hit_cnt + ((nids + 1) & ~uint64_t(1));  // (8-byte aligned: the slot-major uint2 pairs)
  P.hit_r = reinterpret_cast<int32_t *>(P.hit_b + nids * kHitK);
  HIP_OK(hipEventRecord(dc.ev0, s));
  for (size_t i = 0; i < slabs.size(); i++) {  // (inside the timed region: built per call)
    TrParams tp{};
    tp.bloom = reinterpret_cast<const uint64_t *const *>(dd + o_bptr + size_t(slabs[i].first) * 8);
    tp.T = const_cast<uint32_t *>(slabs[i].T);
    tp.words = lb[members[i][0]].words;
    tp.bitlen = slabs[i].bitlen;
    tp.shards = slabs[i].shards;
    tp.W = slabs[i].W;
    tp.J = slabs[i].J;
    if (tp.words * 64 < tp.bitlen) fail(TSG_E_CORRUPT, "bloom shorter than its bit length");
    const uint64_t threads = uint64_t(tp.shards) * tp.words * tp.W;
    static const bool tr_bits = [] {  // (TSG_LK_TR=1: the bit-at-a-time transpose)
      const char *e = std::getenv("TSG_LK_TR");
      return e && std::atoi(e) == 1;
    }();
    if (tr_bits) lookup_transpose_kernel<<<uint32_t((threads + 255) / 256), 256, 0, s>>>(tp);
    else lookup_transpose2_kernel<<<uint32_t((threads + 255) / 256), 256, 0, s>>>(tp);
    HIP_OK(hipGetLastError());
  }
  static const int occ = [] {
    const char *e = std::getenv("TSG_LK_OCC");
    return e ? std::atoi(e) : 7;
  }();
  if (occ == 8) lookup_count_kernel_w8<<<tiles, kLkThreads, 0, s>>>(P);
  else if (occ == 6) lookup_count_kernel<<<tiles, kLkThreads, 0, s>>>(P);
  else if (occ == 17) lookup_count_kernel_w7nt<<<tiles, kLkThreads, 0, s>>>(P);
  else lookup_count_kernel_w7<<<tiles, kLkThreads, 0, s>>>(P);
  HIP_OK(hipGetLastError());
  dc.ticket_base += tiles;
  // The write pass follows at once, its columns sized on the device for up to ocap hits (one
  // per id, or what the output buffer already holds): no host round trip between the passes.
  const size_t per = 4 + 4 + 4 + 8 + 4;
  static const bool host_sized = [] {  // (TSG_LK_HOSTSIZE=1: the round-5 order, the total read first)
    const char *e = std::getenv("TSG_LK_HOSTSIZE");
    return e && std::atoi(e) != 0;
  }();
  uint64_t want = std::max<uint64_t>(nids, 1);
  if (host_sized) {
    uint64_t t0 = 0;
    HIP_OK(hipMemcpyAsync(&t0, dc.hdr.p, 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    want = std::max<uint64_t>(want, t0);
  }
  dc.out.ensure(want * per + 64);
  P.obase = static_cast<uint8_t *>(dc.out.p);
  P.ocap = (dc.out.cap - 64) / per;
  static const uint64_t cap_test = [] {  // (test hook: TSG_LK_OCAP=n caps the first write pass's
    const char *e = std::getenv("TSG_LK_OCAP");  // columns at n hits, so the relaunch runs)
    return e ? uint64_t(std::strtoull(e, nullptr, 10)) : ~0ULL;
  }();
  P.ocap = std::min<uint64_t>(P.ocap, cap_test);
  lookup_write_kernel<<<tiles, kLkThreads, 0, s>>>(P);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(dc.ev1, s));
  uint64_t total = 0;
  uint32_t errf = 0;
  HIP_OK(hipMemcpyAsync(&total, dc.hdr.p, 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(&errf, dc.err.p, 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (errf) {
    HIP_OK(hipMemset(dc.err.p, 0, 4));
    fail(TSG_E_DEVICE, "lookup look-back timed out");
  }
  if (total > P.ocap) {  // more hits than the columns held: grow them and write again
    dc.out.ensure(total * per + 64);
    P.obase = static_cast<uint8_t *>(dc.out.p);
    P.ocap = (dc.out.cap - 64) / per;
    lookup_write_kernel<<<tiles, kLkThreads, 0, s>>>(P);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(dc.ev1, s));
  }
  auto *ob = static_cast<uint8_t *>(dc.out.p);
  P.o_start = reinterpret_cast<uint64_t *>(ob);
  P.o_id = reinterpret_cast<uint32_t *>(ob + total * 8);
  P.o_block = reinterpret_cast<uint32_t *>(ob + total * 12);
  P.o_rec = reinterpret_cast<int32_t *>(ob + total * 16);
  P.o_len = reinterpret_cast<uint32_t *>(ob + total * 20);
  out.id_idx.resize(total);
  out.block_idx.resize(total);
  out.rec.resize(total);
  out.start.resize(total);
  out.len.resize(total);
  if (total) {
    HIP_OK(hipMemcpyAsync(out.start.data(), P.o_start, total * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(out.id_idx.data(), P.o_id, total * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(out.block_idx.data(), P.o_block, total * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(out.rec.data(), P.o_rec, total * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(out.len.data(), P.o_len, total * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_OK(hipStreamSynchronize(s));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, dc.ev0, dc.ev1));
  out.kernel_ns = uint64_t(double(ms) * 1e6);
}

}  // namespace tsg
