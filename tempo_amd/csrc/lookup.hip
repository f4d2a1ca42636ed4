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
  uint8_t min_id[16], max_id[16];
  uint32_t min_len, max_len;
  uint32_t block_idx, pad;
};

struct LkParams {
  const LkBlock *blocks;
  uint32_t nblocks;
  const uint8_t *ids;
  uint64_t nids;
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
__device__ __forceinline__ int d_cmp16(const uint8_t *a, const uint8_t *b, uint32_t bl) {  // bytes.Compare(a[16], b)
  uint32_t n = bl < 16 ? bl : 16;
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 16 == bl ? 0 : (16 < bl ? -1 : 1);
}

// evaluates one (id, block): returns record index (>= 0) on a hit, -1 otherwise
__device__ __forceinline__ int32_t d_probe(const LkBlock &B, const uint8_t *id, uint32_t fnv, const uint64_t h[4]) {
  if (d_cmp16(id, B.min_id, B.min_len) < 0 || d_cmp16(id, B.max_id, B.max_len) > 0) return -1;
  uint32_t shard = fnv % B.shards;
  const uint64_t *w = B.bloom + uint64_t(shard) * B.words;
  for (uint64_t i = 0; i < B.k; i++) {
    uint64_t loc = d_mod(h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) / 2)], B.m, B.m_magic);
    if (loc >= B.bitlen) return -1;
    if (!((w[loc >> 6] >> (loc & 63)) & 1ULL)) return -1;
  }
  // lower_bound: first record with bytes.Compare(rec.ID, id) >= 0 (pkg/sort/search.go:5-24)
  uint32_t lo = 0, hi = B.records;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    const uint8_t *r = B.rec_ids + uint64_t(mid) * 16;
    int c = 0;
    for (int q = 0; q < 16 && c == 0; q++)
      if (r[q] != id[q]) c = r[q] < id[q] ? -1 : 1;
    if (c < 0) lo = mid + 1;
    else hi = mid;
  }
  return lo < B.records ? int32_t(lo) : -1;
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

extern "C" __global__ void __launch_bounds__(kLkThreads) lookup_count_kernel(LkParams P) {
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
    memcpy(id, P.ids + i * 16, 16);
    uint32_t fnv;
    uint64_t h[4];
    d_id_hash(id, fnv, h);
    for (uint32_t b = 0; b < P.nblocks; b++) {
      const int32_t r = d_probe(P.blocks[b], id, fnv, h);
      if (r < 0) continue;
      if (cnt < kHitK) {
        P.hit_b[i * kHitK + cnt] = b;
        P.hit_r[i * kHitK + cnt] = r;
      }
      cnt++;
    }
    P.hit_cnt[i] = cnt;
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
  if (i < P.nids) P.offsets[i] = s_excl + before + v - cnt;
}

extern "C" __global__ void __launch_bounds__(kLkThreads) lookup_write_kernel(LkParams P) {
  const uint64_t i = uint64_t(blockIdx.x) * kLkThreads + threadIdx.x;
  if (i >= P.nids) return;
  const uint32_t cnt = P.hit_cnt[i];
  if (cnt <= kHitK) {  // every hit was kept by the count pass, in block order
    uint64_t o = P.offsets[i];
    for (uint32_t j = 0; j < cnt; j++, o++) {
      const LkBlock &B = P.blocks[P.hit_b[i * kHitK + j]];
      const int32_t r = P.hit_r[i * kHitK + j];
      P.o_id[o] = uint32_t(i);
      P.o_block[o] = B.block_idx;
      P.o_rec[o] = r;
      P.o_start[o] = B.rec_start[r];
      P.o_len[o] = B.rec_len[r];
    }
    return;
  }
  uint8_t id[16];
  memcpy(id, P.ids + i * 16, 16);
  uint32_t fnv;
  uint64_t h[4];
  d_id_hash(id, fnv, h);
  uint64_t o = P.offsets[i];
  for (uint32_t b = 0; b < P.nblocks; b++) {
    const LkBlock &B = P.blocks[b];
    int32_t r = d_probe(B, id, fnv, h);
    if (r < 0) continue;
    P.o_id[o] = uint32_t(i);
    P.o_block[o] = B.block_idx;
    P.o_rec[o] = r;
    P.o_start[o] = B.rec_start[r];
    P.o_len[o] = B.rec_len[r];
    o++;
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

void device_lookup(DeviceCtx &dc, const std::vector<std::pair<uint32_t, V2Block *>> &blocks, const uint8_t (*ids)[16],
                   size_t nids, const tsg_lookup_opts *opts, LookupOut &out) {
  std::lock_guard<std::mutex> lk(dc.mu);
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
    std::memcpy(k.min_id, b.min_id.data(), b.min_id.size());
    std::memcpy(k.max_id, b.max_id.data(), b.max_id.size());
    k.min_len = uint32_t(b.min_id.size());
    k.max_len = uint32_t(b.max_id.size());
    k.block_idx = bp.first;
    lb.push_back(k);
  }
  out = LookupOut();
  if (nids == 0 || lb.empty()) return;
  uint32_t tiles = uint32_t((nids + kLkThreads - 1) / kLkThreads);
  size_t desc_bytes = (lb.size() * sizeof(LkBlock) + 15) & ~size_t(15);
  dc.desc.ensure(desc_bytes + nids * 16);
  dc.hdesc.ensure(desc_bytes);
  std::memcpy(dc.hdesc.p, lb.data(), lb.size() * sizeof(LkBlock));
  auto *dd = static_cast<uint8_t *>(dc.desc.p);
  HIP_OK(hipMemcpyAsync(dd, dc.hdesc.p, lb.size() * sizeof(LkBlock), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(dd + desc_bytes, ids, nids * 16, hipMemcpyHostToDevice, s));
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
  P.ids = dd + desc_bytes;
  P.nids = nids;
  P.epoch = dc.epoch;
  P.ticket_base = dc.ticket_base;
  P.ticket = static_cast<unsigned long long *>(dc.ticket.p);
  P.gran = static_cast<unsigned long long *>(dc.gran.p);
  P.offsets = static_cast<uint64_t *>(dc.vmatch.p);
  P.total = static_cast<uint64_t *>(dc.hdr.p);
  P.err = static_cast<uint32_t *>(dc.err.p);
  dc.lkhits.ensure(std::max<uint64_t>(nids, 1) * (4 + kHitK * 8));
  P.hit_cnt = static_cast<uint32_t *>(dc.lkhits.p);
  P.hit_b = P.hit_cnt + nids;
  P.hit_r = reinterpret_cast<int32_t *>(P.hit_b + nids * kHitK);
  HIP_OK(hipEventRecord(dc.ev0, s));
  lookup_count_kernel<<<tiles, kLkThreads, 0, s>>>(P);
  HIP_OK(hipGetLastError());
  dc.ticket_base += tiles;
  uint64_t total = 0;
  uint32_t errf = 0;
  HIP_OK(hipMemcpyAsync(&total, dc.hdr.p, 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(&errf, dc.err.p, 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (errf) {
    HIP_OK(hipMemset(dc.err.p, 0, 4));
    fail(TSG_E_DEVICE, "lookup look-back timed out");
  }
  size_t per = 4 + 4 + 4 + 8 + 4;
  dc.out.ensure(std::max<uint64_t>(total, 1) * per + 64);
  auto *ob = static_cast<uint8_t *>(dc.out.p);
  P.o_start = reinterpret_cast<uint64_t *>(ob);
  P.o_id = reinterpret_cast<uint32_t *>(ob + total * 8);
  P.o_block = reinterpret_cast<uint32_t *>(ob + total * 12);
  P.o_rec = reinterpret_cast<int32_t *>(ob + total * 16);
  P.o_len = reinterpret_cast<uint32_t *>(ob + total * 20);
  lookup_write_kernel<<<tiles, kLkThreads, 0, s>>>(P);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(dc.ev1, s));
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
