// host_stub.cpp — TEST INFRASTRUCTURE ONLY (never linked into libtsg.so): the HIP-side entry
// points of libtsg (devctx.hip, search.hip, pool.hip, lookup.hip, find.hip, proto_scan.hip)
// replaced by a host stand-in, so that libtsg's host code — the C ABI (capi.cpp: the coalescer
// and its leaders, the result holders, the limit waves, tsg_search_batch's workers), the
// loader, the writer, the merge — runs under AddressSanitizer / UBSan and ThreadSanitizer on a
// machine without a GPU (tests/sanitize/Makefile, tests/test_sanitizers.py).
//
// The stand-in "device" does not search: device_search marks entry e of a block as a match when
// a hash of (e, the query) falls below 1/32 (capped, ranged and ordered as the real path hands
// them over), so that concurrent callers with different queries get different, checkable
// records. tsg_init fails with TSG_E_DEVICE (as without a GPU) unless TSG_STUB_DEVICES=n is set.
#include <algorithm>
#include <chrono>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../../tempo_amd/csrc/block.hpp"
#include "../../tempo_amd/csrc/devctx.hpp"
#include "../../tempo_amd/csrc/engine.hpp"
#include "../../tempo_amd/csrc/proto.hpp"

namespace tsg {

void ctx_init(Ctx &c, const tsg_options *opts) {
  const char *e = std::getenv("TSG_STUB_DEVICES");
  const int n = e ? std::atoi(e) : 0;
  if (n <= 0) fail(TSG_E_DEVICE, "no HIP device visible (libtsg has no CPU path)");
  const int m = opts && opts->num_devices > 0 ? opts->num_devices : n;
  for (int i = 0; i < m; i++) {
    auto *dc = new DeviceCtx();
    dc->ordinal = opts && opts->devices ? opts->devices[i] : i;
    dc->num_cu = dc->dev_cu = 256;
    c.devs.push_back(dc);
  }
}
void ctx_shutdown(Ctx &c) {
  for (DeviceCtx *dc : c.devs) delete dc;
  c.devs.clear();
}
void block_upload(Ctx &c, Block &b, int device_hint) {
  if (c.devs.empty()) fail(TSG_E_DEVICE, "no device");
  b.dc = c.devs[size_t(std::max(device_hint, 0)) % c.devs.size()];
  b.dev = DevBlock();
  b.dev.n = b.host->n;
}
void block_clone(Ctx &c, const Block &src, Block &dst, int device_hint) {
  dst.host = src.host;
  block_upload(c, dst, device_hint);
}
void block_free(Block &b) { b.dc = nullptr; }

static uint64_t query_hash(const tsg_query &q) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ q.nterms ^ (uint64_t(q.has_min) << 8) ^ (q.min_ns * 31) ^ (q.max_ns * 131);
  for (uint32_t t = 0; t < q.nterms; t++) {
    h ^= xxhash64(q.values[t], q.value_lens[t]) + 0x632BE59BD9B4E019ull * (t + 1);
    h ^= xxhash64(q.keys[t], q.key_lens[t]) * 3;
  }
  return h;
}
// TSG_STUB_ONE_IN: one entry in n matches (default 32); TSG_STUB_SLEEP_US: the stand-in device
// time (default 20 + 0..63 us by query); both for tools/host_prof.py's host-cost runs
static uint64_t stub_env(const char *name, uint64_t dflt) {
  const char *e = std::getenv(name);
  return e ? std::strtoull(e, nullptr, 10) : dflt;
}
bool stub_match(const tsg_query &q, uint64_t e) {  // (also called by the stress driver)
  static const uint64_t one_in = std::max<uint64_t>(1, stub_env("TSG_STUB_ONE_IN", 32));
  uint64_t x = (e + 1) * 0xD6E8FEB86659FD93ull ^ query_hash(q);
  x ^= x >> 32;
  x *= 0xD6E8FEB86659FD93ull;
  x ^= x >> 29;
  return x % one_in == 0;
}

void device_search(DeviceCtx &dc, const std::vector<std::pair<uint32_t, Block *>> &blocks, const tsg_query &q,
                   uint32_t limit, uint32_t flags, SearchOut &out, const EntryRanges *ranges) {
  (void)flags;
  std::unique_lock<std::mutex> lk(dc.mu);
  out.recs.clear();
  out.term_any.clear();
  out.compact = false;
  out.pos.clear();
  out.block_counts.assign(blocks.size(), 0);
  out.device_bytes = out.kernel_ns = out.scan_ns = out.scan_bytes = 0;
  out.reruns = 0;
  out.pool = true;  // (entry ranges are honoured: the limit waves may cut blocks)
  out.resident = false;
  out.path = TSG_PATH_PLAIN;
  if (q.exhaustive) return;
  for (size_t i = 0; i < blocks.size(); i++) {
    const HostBlock &h = *blocks[i].second->host;
    uint64_t e0 = 0, e1 = h.n;
    if (ranges) {
      e1 = std::min<uint64_t>((*ranges)[i].second, h.n);
      e0 = std::min<uint64_t>((*ranges)[i].first, e1) / 512 * 512;
    }
    uint64_t kept = 0;
    // (TSG_STUB_CACHE=1, tools/host_prof.py: a block's matches are found once per query, so that
    // the stand-in device costs nothing per search; the host's share is what is measured)
    static const bool cache = stub_env("TSG_STUB_CACHE", 0) != 0;
    const std::vector<uint32_t> *hit = nullptr;
    if (cache) {
      static std::mutex mu;
      static std::map<std::pair<const HostBlock *, uint64_t>, std::vector<uint32_t>> memo;
      std::lock_guard<std::mutex> g(mu);
      auto &v = memo[{&h, query_hash(q)}];
      if (v.empty()) {
        for (uint64_t e = 0; e < h.n; e++)
          if (stub_match(q, e)) v.push_back(uint32_t(e));
        v.push_back(UINT32_MAX);
      }
      hit = &v;
    }
    size_t hi = 0;
    for (uint64_t e = e0; e < e1 && (!limit || kept < limit); e++) {
      if (hit) {
        while ((*hit)[hi] < e) hi++;
        if ((*hit)[hi] >= e1) break;
        e = (*hit)[hi];
      } else if (!stub_match(q, e)) {
        continue;
      }
      SearchOut::Rec r;
      std::memcpy(r.id, h.ids.data() + e * 16, 16);
      r.start = h.start[e];
      r.end = h.end[e];
      r.entry = uint32_t(e);
      r.block_il = blocks[i].first | (uint32_t(h.id_len[e]) << 24);
      r.svc = h.svc_vid.empty() ? kNone : h.svc_vid[e];
      r.name = h.name_vid.empty() ? kNone : h.name_vid[e];
      out.recs.push_back(r);
      kept++;
    }
    out.block_counts[i] = kept;
    out.scan_bytes += (e1 - e0) * 11;
  }
  out.device_bytes = out.scan_bytes;
  // the device's time, with dc.mu released as the resident path releases it: other callers
  // plan meanwhile (the interleavings ThreadSanitizer sees)
  lk.unlock();
  static const uint64_t sleep_us = stub_env("TSG_STUB_SLEEP_US", ~0ull);
  const uint64_t us = sleep_us == ~0ull ? 20 + (query_hash(q) & 63) : sleep_us;
  if (us) std::this_thread::sleep_for(std::chrono::microseconds(us));
}

int device_numa_node(const DeviceCtx &) { return -1; }
int device_ordinal(const DeviceCtx &dc) { return dc.ordinal; }
void device_counters(DeviceCtx &dc, uint64_t out[8]) {
  std::lock_guard<std::mutex> lk(dc.mu);
  for (int i = 0; i < 8; i++) out[i] = 0;
}
void device_kernel_times(DeviceCtx &, std::vector<uint64_t> &ns) { ns.clear(); }
bool device_last_dense(DeviceCtx &) { return true; }
uint64_t resident_batch_begin(DeviceCtx &) { return 0; }
uint64_t resident_batch_end(DeviceCtx &, uint64_t) { return 0; }
int debug_set(const char *name, int64_t) {
  return name && (!std::strcmp(name, "res_torn") || !std::strcmp(name, "groups") || !std::strcmp(name, "xsplit") ||
                  !std::strcmp(name, "lb_bitmap"))
             ? TSG_OK
             : TSG_E_INVALID;
}
void *pinned_get(size_t bytes) {
  void *p = std::malloc(bytes ? bytes : 1);
  if (!p) throw std::bad_alloc();
  return p;
}
void pinned_put(void *p, size_t) { std::free(p); }
void v2block_open(Ctx &, V2Block &, const std::string &, int) { fail(TSG_E_UNSUPPORTED, "host stub: no v2 blocks"); }
void v2block_free(V2Block &) {}
void device_lookup(DeviceCtx &, const std::vector<std::pair<uint32_t, V2Block *>> &, const uint8_t (*)[16], size_t,
                   const tsg_lookup_opts *, LookupOut &) {
  fail(TSG_E_UNSUPPORTED, "host stub: no lookup");
}
void device_find(DeviceCtx &, const std::vector<std::pair<uint32_t, V2Block *>> &, const uint8_t (*)[16], size_t,
                 const tsg_lookup_opts *, FindOut &) {
  fail(TSG_E_UNSUPPORTED, "host stub: no find");
}
void proto_block_open(Ctx &, ProtoBlock &, const std::string &, int) { fail(TSG_E_UNSUPPORTED, "host stub: no proto blocks"); }
void proto_block_free(ProtoBlock &) {}
void proto_search(ProtoBlock &, const tsg_proto_request &, ProtoOut &) { fail(TSG_E_UNSUPPORTED, "host stub: no proto search"); }

}  // namespace tsg
