// proto_scan.hip — proto-object backend search on the device.
//
// proto_scan_kernel evaluates, for every object of the searched page range, what
// ObjectDecoder.Matches + trace.MatchesProto decide for it (pkg/model/v2/object_decoder.go:57-89,
// pkg/model/v1/object_decoder.go, pkg/model/trace/matches.go:33-116), over the columns the
// loader built (proto.cpp): one lane per object, one 64-object ballot per wave, two bits
// per object (match, error) written as 64-bit words. The host then replays
// BackendBlock.Search's loop (tempodb/encoding/v2/backend_block.go:185-202, :211-231) over
// those bits: metrics per object, MaxBytes skips, the first error, the limit break, and
// the paged iterator's chunked page reads (iterator_paged.go:62-131).
//
// Bound: HBM, ~(24 + Σ term column width) B per object + term bitmaps (L2-resident).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "devctx.hpp"
#include "proto.hpp"

namespace tsg {

std::vector<uint32_t> proto_term_bitmap(const ProtoBlock &b, const std::string &key, std::string_view v, bool &present);
void proto_load_host(ProtoBlock &b, const std::string &dir);

constexpr int kPThreads = 256;
constexpr int kPTerms = 16;

struct PTerm {
  const uint8_t *col;     // value-set id per object (width bytes, all-ones = key absent); null = key not in block
  const uint32_t *bm;     // value-set bitmap of this term
  uint32_t width, pad;
};

struct PArgs {
  const uint32_t *fr_start, *fr_end, *st_sec, *en_sec, *dur_ms, *obj_len;
  const uint8_t *flags;
  uint32_t t0, t1, v2, nterms;
  uint32_t start, end, min_ms, max_ms, max_bytes, pad;
  unsigned long long *out;  // [2 * words]: match bits, then error bits (bit i = object t0 + i)
  uint32_t words, pad2;
  PTerm terms[kPTerms];
};

__global__ void __launch_bounds__(kPThreads) proto_scan_kernel(PArgs A) {
  const uint32_t i = A.t0 + blockIdx.x * kPThreads + threadIdx.x;
  bool m = false, e = false;
  if (i < A.t1) {
    const uint32_t len = A.obj_len[i];
    const bool skipped = A.max_bytes && len > A.max_bytes;  // search(): SkippedTraces, no Matches
    if (!skipped) {
      const uint8_t fl = A.flags[i];
      bool pass = true;
      if (A.v2) {
        if (fl & PF_HDRBAD) {  // FastRange: stripStartEnd error
          e = true;
          pass = false;
        } else {
          const uint32_t s = A.fr_start[i], en = A.fr_end[i];
          if (!(A.start <= en && A.end >= s)) pass = false;
          const uint32_t d = en - s;  // (uint32 wrap, as the reference)
          if (A.max_ms && d > A.max_ms / 1000 + 1) pass = false;
          if (A.min_ms && d < A.min_ms / 1000) pass = false;
        }
      }
      if (pass && (fl & PF_BAD)) {  // PrepareForRead: proto.Unmarshal error
        e = true;
        pass = false;
      }
      if (pass) {
        for (uint32_t q = 0; q < A.nterms && pass; q++) {
          const PTerm &T = A.terms[q];
          if (!T.col) {
            pass = false;
            break;
          }
          uint32_t sid;
          if (T.width == 1) {
            sid = T.col[i];
            sid = sid == 0xffu ? 0xffffffffu : sid;
          } else if (T.width == 2) {
            sid = reinterpret_cast<const uint16_t *>(T.col)[i];
            sid = sid == 0xffffu ? 0xffffffffu : sid;
          } else {
            sid = reinterpret_cast<const uint32_t *>(T.col)[i];
          }
          pass = sid != 0xffffffffu && ((T.bm[sid >> 5] >> (sid & 31)) & 1u);
        }
        if (pass) {
          const uint32_t dms = A.dur_ms[i];
          if (A.max_ms && A.max_ms < dms) pass = false;
          if (A.min_ms && A.min_ms > dms) pass = false;
          if (!(A.start <= A.en_sec[i] && A.end >= A.st_sec[i])) pass = false;
        }
        m = pass;
      }
    }
  }
  const unsigned long long bm = __ballot(m), be = __ballot(e);
  const uint32_t w = (blockIdx.x * kPThreads + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0 && w < A.words) {
    A.out[w] = bm;
    A.out[A.words + w] = be;
  }
}

static void *palloc(ProtoBlock &b, size_t bytes) {
  void *p = nullptr;
  HIP_OK(hipMalloc(&p, std::max<size_t>(bytes, 16)));
  b.allocs.push_back(p);
  b.device_bytes += bytes;
  return p;
}

void proto_block_open(Ctx &c, ProtoBlock &b, const std::string &dir, int device_hint) {
  if (c.devs.empty()) fail(TSG_E_DEVICE, "no device");
  proto_load_host(b, dir);
  DeviceCtx &dc = *c.devs[size_t(std::max(device_hint, 0)) % c.devs.size()];
  b.dc = &dc;
  std::lock_guard<std::mutex> lk(dc.mu);
  HIP_OK(hipSetDevice(dc.ordinal));
  const size_t n = b.n;
  auto *u = static_cast<uint32_t *>(palloc(b, n * 6 * 4));
  const std::vector<uint32_t> *cols[6] = {&b.fr_start, &b.fr_end, &b.st_sec, &b.en_sec, &b.dur_ms, &b.obj_len};
  for (int k = 0; k < 6; k++)
    if (n) HIP_OK(hipMemcpy(u + k * n, cols[k]->data(), n * 4, hipMemcpyHostToDevice));
  b.d_u32 = u;
  auto *fl = static_cast<uint8_t *>(palloc(b, n));
  if (n) HIP_OK(hipMemcpy(fl, b.flags.data(), n, hipMemcpyHostToDevice));
  b.d_flags = fl;
  for (ProtoKey &K : b.keys) {
    auto *p = static_cast<uint8_t *>(palloc(b, K.col.size()));
    if (!K.col.empty()) HIP_OK(hipMemcpy(p, K.col.data(), K.col.size(), hipMemcpyHostToDevice));
    K.d_col = p;
    std::vector<uint8_t>().swap(K.col);
  }
}

void proto_block_free(ProtoBlock &b) {
  if (!b.dc) return;
  std::lock_guard<std::mutex> lk(b.dc->mu);
  (void)hipSetDevice(b.dc->ordinal);
  (void)hipStreamSynchronize(b.dc->stream);
  for (void *p : b.allocs) (void)hipFree(p);
  b.allocs.clear();
  b.dc = nullptr;
}

void proto_search(ProtoBlock &b, const tsg_proto_request &req, ProtoOut &out) {
  out = ProtoOut();
  if (!b.dc) fail(TSG_E_INVALID, "proto block not resident");
  if (req.ntags > kPTerms) fail(TSG_E_UNSUPPORTED, "more than 16 tags in one proto search");
  const uint32_t npages = uint32_t(b.page_len.size());
  const uint32_t chunk = req.chunk_size_bytes ? req.chunk_size_bytes : 1000000u;  // DefaultSearchOptions
  // TotalPages > 0: partialIterator(StartPage, TotalPages); else Iterator() from page 0
  const uint32_t start_page = req.total_pages ? req.start_page : 0;
  const uint64_t maxp = req.total_pages ? uint64_t(start_page) + req.total_pages : ~0ULL;
  // objects of the searched page range (the kernel covers them; the host walk stops early)
  const uint32_t p0 = std::min(start_page, npages);
  const uint32_t p1 = uint32_t(std::min<uint64_t>(npages, maxp));
  const uint32_t t0 = b.page_first[p0], t1 = p1 > p0 ? b.page_first[p1] : t0;
  // query terms: map semantics (one value per key: the last one given wins)
  std::vector<std::pair<std::string, std::string>> tags;
  for (uint32_t q = 0; q < req.ntags; q++) {
    std::string k(req.keys[q], req.key_lens[q]), v(req.values[q], req.value_lens[q]);
    bool dup = false;
    for (auto &kv : tags)
      if (kv.first == k) {
        kv.second = v;
        dup = true;
      }
    if (!dup) tags.emplace_back(k, v);
  }
  std::vector<uint32_t> bmw;
  std::vector<size_t> bm_at(tags.size(), 0);
  std::vector<int> key_of(tags.size(), -1);
  for (size_t q = 0; q < tags.size(); q++) {
    bool present;
    std::vector<uint32_t> bm = proto_term_bitmap(b, tags[q].first, tags[q].second, present);
    if (!present) continue;
    key_of[q] = int(b.key_index.at(tags[q].first));
    bm_at[q] = bmw.size();
    bmw.insert(bmw.end(), bm.begin(), bm.end());
  }
  DeviceCtx &dc = *b.dc;
  std::vector<unsigned long long> bits;
  const uint32_t words = (t1 - t0 + 63) / 64;
  {
    std::lock_guard<std::mutex> lk(dc.mu);
    resident_quit(dc);  // (the resident search launch holds every CU's LDS)
    HIP_OK(hipSetDevice(dc.ordinal));
    hipStream_t s = dc.stream;
    if (t1 > t0) {
      dc.pbm.ensure(std::max<size_t>(bmw.size(), 1) * 4);
      dc.pout.ensure(size_t(words) * 16);
      if (!bmw.empty()) HIP_OK(hipMemcpyAsync(dc.pbm.p, bmw.data(), bmw.size() * 4, hipMemcpyHostToDevice, s));
      PArgs A{};
      const size_t n = b.n;
      A.fr_start = b.d_u32;
      A.fr_end = b.d_u32 + n;
      A.st_sec = b.d_u32 + 2 * n;
      A.en_sec = b.d_u32 + 3 * n;
      A.dur_ms = b.d_u32 + 4 * n;
      A.obj_len = b.d_u32 + 5 * n;
      A.flags = b.d_flags;
      A.t0 = t0;
      A.t1 = t1;
      A.v2 = b.v2;
      A.nterms = uint32_t(tags.size());
      A.start = req.start;
      A.end = req.end;
      A.min_ms = req.min_duration_ms;
      A.max_ms = req.max_duration_ms;
      A.max_bytes = req.max_bytes;
      A.out = static_cast<unsigned long long *>(dc.pout.p);
      A.words = words;
      for (size_t q = 0; q < tags.size(); q++) {
        if (key_of[q] < 0) continue;  // (col null: the key is in no object of the block)
        const ProtoKey &K = b.keys[size_t(key_of[q])];
        A.terms[q].col = K.d_col;
        A.terms[q].width = K.width;
        A.terms[q].bm = static_cast<const uint32_t *>(dc.pbm.p) + bm_at[q];
      }
      HIP_OK(hipEventRecord(dc.ev0, s));
      proto_scan_kernel<<<(t1 - t0 + kPThreads - 1) / kPThreads, kPThreads, 0, s>>>(A);
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(dc.ev1, s));
      bits.resize(size_t(words) * 2);
      HIP_OK(hipMemcpyAsync(bits.data(), dc.pout.p, bits.size() * 8, hipMemcpyDeviceToHost, s));
      HIP_OK(hipStreamSynchronize(s));
      float ms = 0;
      HIP_OK(hipEventElapsedTime(&ms, dc.ev0, dc.ev1));
      out.kernel_ns = uint64_t(double(ms) * 1e6);
    }
  }
  // BackendBlock.Search's loop over the paged iterator
  auto bit = [&](uint32_t i, int which) {
    const uint32_t r = i - t0;
    return (bits[size_t(which) * words + (r >> 6)] >> (r & 63)) & 1ULL;
  };
  auto fail_at = [&](int code, const std::string &m) {
    out.status = code;
    out.error = m;
    out.traces.clear();
  };
  const uint32_t limit = req.limit;
  uint64_t cur = start_page;
  for (;;) {
    if (cur >= maxp) return;                    // io.EOF
    auto at = [&](uint64_t r) -> int {          // indexReader.At: 1 record, 0 nil, -1 error
      if (r >= b.total_records) return 0;
      if (r >= b.index_err_at) return -1;
      return 1;
    };
    int a = at(cur);
    if (a < 0) return fail_at(TSG_E_CORRUPT, "error reading index record " + std::to_string(cur));
    if (a == 0) return;
    // gather a chunk: at least one record, then while it fits and is inside the range
    std::vector<uint32_t> chunk_pages;
    uint64_t length = 0;
    while (a > 0) {
      if ((length + b.page_len[cur] > chunk || cur >= maxp) && !chunk_pages.empty()) break;
      chunk_pages.push_back(uint32_t(cur));
      length += b.page_len[cur];
      cur++;
      a = at(cur);
      if (a < 0) return fail_at(TSG_E_CORRUPT, "error getting next record " + std::to_string(cur));
    }
    for (uint32_t p : chunk_pages)
      if (b.page_status[p] == PP_DECODE) return fail_at(TSG_E_CORRUPT, "error reading objects for records (page " + std::to_string(p) + ")");
    for (uint32_t p : chunk_pages) {
      for (uint32_t i = b.page_first[p]; i < b.page_first[p + 1]; i++) {
        out.inspected_traces++;
        out.inspected_bytes += b.obj_len[i];
        if (req.max_bytes && b.obj_len[i] > req.max_bytes) {
          out.skipped_traces++;
        } else if (bit(i, 1)) {
          return fail_at(TSG_E_CORRUPT, "object " + std::to_string(i) + ": trace decode failed");
        } else if (bit(i, 0)) {
          out.traces.push_back(i);
        }
        if (out.traces.size() >= limit) return;  // (limit 0: after the first object)
      }
      if (b.page_status[p] == PP_FRAMING)
        return fail_at(TSG_E_CORRUPT, "error unmarshalling active page " + std::to_string(p));
    }
  }
}

}  // namespace tsg
