// devctx.hpp — per-device context shared by the search and lookup pipelines.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <utility>

#include "engine.hpp"

namespace tsg {
struct Aql;  // aql.hpp

#define HIP_OK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) ::tsg::fail(TSG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {  // true when (re)allocated
    if (n <= cap) return false;
    if (p) HIP_OK(hipFree(p));
    size_t c = std::max(n, cap * 2);
    HIP_OK(hipMalloc(&p, c));
    cap = c;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};
struct HostBuf {
  void *p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) HIP_OK(hipHostFree(p));
    size_t c = std::max(n, cap * 2);
    HIP_OK(hipHostMalloc(&p, c, flags));
    cap = c;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct DeviceCtx {
  int ordinal = 0;
  int num_cu = 0;   // the CUs search launches plan for: dev_cu, or the "groups" test hook
  int dev_cu = 0;   // the device's
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, es0 = nullptr, es1 = nullptr;
  hipEvent_t mk0 = nullptr, mk1 = nullptr;  // untimed markers around a launch
  hipEvent_t er0 = nullptr, er1 = nullptr;  // timing of rerun launches
  // search kernels timed by events stamped from their own dispatch packet
  // (hipExtLaunchKernel start/stop events: what rocprofv3's kernel trace measures);
  // TSG_EXT_EVENTS=0: marker events recorded on the stream before and after the launch
  bool ext_events = [] {
    const char *e = std::getenv("TSG_EXT_EVENTS");
    return !e || std::atoi(e) != 0;
  }();
  // TSG_MARK (default 0, experiment): bit 0 = an untimed marker event recorded right
  // before each search launch, bit 1 = one right after it. An apparent 16 us/step gain
  // was NUMA placement of the polling thread (profiles/r01_host); with the thread on the
  // GPU's node a marker costs ~2-3 us per step.
  bool stage_first = [] {  // TSG_STAGE_FIRST=0/1: dictionary words before the tile stream
    const char *e = std::getenv("TSG_STAGE_FIRST");
    return e ? std::atoi(e) != 0 : false;
  }();
  bool prio = [] {  // TSG_PRIO=1: progress-ordered wave priority in the scan loop (default off)
    const char *e = std::getenv("TSG_PRIO");
    return e ? std::atoi(e) != 0 : false;
  }();
  bool bm_first = [] {  // TSG_BM_FIRST=0/1: narrow bitmap words before the tile stream
    const char *e = std::getenv("TSG_BM_FIRST");
    return e ? std::atoi(e) != 0 : false;
  }();
  int mark_mode = [] {
    const char *e = std::getenv("TSG_MARK");
    return e ? std::atoi(e) : 0;
  }();
  std::mutex mu;
  // search scratch: descriptors, dictionary matches, value-set bitmaps, match
  // bitmasks (one bit per entry of tiles that matched), per-tile / per-workgroup
  // counts, [header | records] output. lookup reuses desc/gran/ticket/out/hdr/err.
  DevBuf desc, vmatch, bitmaps, gran, ticket, out, regions, seg_counts, hdr, err;
  DevBuf maskbits, agg, stamps, gbm, lkhits;
  DevBuf lkslab, lkslabdesc;  // lookup: transposed bloom slabs + their member tables
  DevBuf pbm, pout;  // proto search: term bitmaps, per-object match/error bits
  DevBuf fpages, fhits, fres, farena, fcrc, fdst, foff;  // device findOne (find.hip)
  HostBuf hdesc, hout;
  // lookup: pinned staging of the caller's (pageable) probe ids, two chunks in turn: the host
  // copies one while the other's DMA runs (lookup.hip upload_ids)
  HostBuf lkstage;
  hipEvent_t lk_ev[2] = {nullptr, nullptr};
  // search results, written by the emit kernel directly (coherent: the kernel's
  // stores go over the fabric, visible to the host once the stream is synchronised)
  HostBuf hres{nullptr, 0, hipHostMallocMapped | hipHostMallocCoherent};
  // per dictionary job of a general-path search: 1 once some value of it matched (prep /
  // dict_sets kernels set danyf in device memory; one copy here; read after the sync)
  HostBuf hany{nullptr, 0, hipHostMallocMapped | hipHostMallocCoherent};
  DevBuf danyf;  // (the device-side flags hany is copied from)
  // look-back bitmap mode (search.hip): one bit per scanned entry, written by the scan kernel;
  // lb_dense: the last full scan on the general path had more than one match per 64 entries
  HostBuf hbits{nullptr, 0, hipHostMallocMapped | hipHostMallocCoherent};
  bool lb_dense = false;
  unsigned long long epoch = 0, ticket_base = 0;  // lookup launches
  uint32_t search_epoch = 0;
  bool fast_off = std::getenv("TSG_NO_FAST") != nullptr;  // force the general (prep + search) path
  bool self_off = std::getenv("TSG_NO_SELF_DICT") != nullptr;  // one-launch path: always use dictionary workgroups
  bool narrow_off = std::getenv("TSG_NO_NARROW") != nullptr;  // one-launch path: never host-matched narrow dictionaries
  std::map<std::pair<const void *, size_t>, int> occupancy;  // (kernel, dynamic LDS) -> blocks per CU  // search launches: tag of the published workgroup counts
  size_t gran_tiles = 0;
  // one-launch search path: per-XCD-group completion counters + top counter, 128 B
  // apart; monotonic: a launch advances each by an amount the host knows, mirrored
  // in done_base
  DevBuf done;
  uint32_t done_base[9] = {};
  // segment-mode work stealing: per block slot claim counters (128 B apart), monotonic;
  // steal_base mirrors each one's value at the next launch. Opt-in (TSG_STEAL=1): on
  // MI355X the static split's kernel p50 was equal or better (profiles/r02_steal)
  DevBuf steal;
  uint32_t steal_base[32] = {};
  bool steal_off = std::getenv("TSG_STEAL") == nullptr;
  uint32_t seg_cap = 16;                                  // segment-mode records per workgroup (limit 0), adaptive
  bool seg_off = std::getenv("TSG_NO_SEG") != nullptr;    // one-launch path: always look-back mode
  // pool path (search_pool_kernel: narrow full scans, one workgroup per CU). TSG_NO_POOL=1
  // disables it; TSG_POOL_DYN = percent of the units claimed dynamically (default 20),
  // TSG_POOL_CHUNK = log2 units per dynamic claim (4), TSG_POOL_LOOK = claims of lookahead (8),
  // TSG_POOL_WAVES = waves per workgroup (16)
  bool pool_off = std::getenv("TSG_NO_POOL") != nullptr;
  uint32_t pool_skip = 0;  // searches of query pool_skip_key left to skip the pool after a record-buffer overflow
  uint64_t pool_skip_key = 0;
  static uint32_t env_u32(const char *name, uint32_t dflt, uint32_t lo, uint32_t hi) {
    const char *e = std::getenv(name);
    if (!e) return dflt;
    const long v = std::atol(e);
    return v < long(lo) ? lo : v > long(hi) ? hi : uint32_t(v);
  }
  uint32_t pool_dyn_pct = env_u32("TSG_POOL_DYN", 20, 0, 100);
  uint32_t pool_chunk_shift = env_u32("TSG_POOL_CHUNK", 4, 0, 10);
  uint32_t pool_lookahead = env_u32("TSG_POOL_LOOK", 8, 0, 1024);  // (32: kernel p50 +1.5 us, profiles/r02_pool)
  uint32_t pool_waves = env_u32("TSG_POOL_WAVES", 16, 2, 16);  // waves per workgroup (one workgroup per CU)
  // TSG_POOL_NT=0: default-policy stream loads (non-temporal measured faster: kernel p50
  // 32.8 vs 34.5 us, profiles/r02_pool)
  bool pool_nt = env_u32("TSG_POOL_NT", 1, 0, 1) != 0;
  uint32_t pool_rec = env_u32("TSG_POOL_REC", 1u << 20, 1, 1u << 20);  // TSG_POOL_REC: LDS records per workgroup below the 2048 that fit (tests)
  // TSG_POOL_SMALL: a search whose static run would be below this many units per
  // workgroup is split statically whole (no device-counter claims); 0 keeps the dynamic
  // tail at every size (tests)
  uint32_t pool_small = env_u32("TSG_POOL_SMALL", 32, 0, 1u << 20);
  uint32_t pool_seg = 32;  // host segment records per workgroup (adaptive: grows on overflow, halves when sparse)
  // Launches below TSG_POOL_STATIC_UNITS units per workgroup (default 32: ~4 M entries, a
  // limit query's waves, one block) run the static-run kernel (search_static_kernel: its
  // first loads go out before anything is staged; limit-wave kernel 16.4 vs 18.3 us);
  // larger ones the claim-based pool kernel, whose dynamic tail evens the CUs out (config-3
  // share 287 vs 319 us, profiles/r03_ab). 0: always the pool kernel; a huge value: always static.
  uint32_t pool_static_units = env_u32("TSG_POOL_STATIC_UNITS", 32, 0, 1u << 30);
  // large dictionaries matched as one byte stream (dict_stream_kernel); 0: a lane per value
  bool dict_stream = env_u32("TSG_DICT_STREAM", 1, 0, 1) != 0;
  DevBuf pool_head;  // two dynamic-chunk counters (128 B apart): a launch uses one, zeroes the other
  // untimed narrow-search launches as AQL packets on a queue of our own (aql.hpp); opened at
  // the first narrow search, nullptr when unavailable (TSG_AQL=0: always through HIP)
  Aql *aql = nullptr;
  bool aql_tried = false;
  uint32_t pool_parity = 0;
  // resident search kernel (pool.hip search_resident_kernel; TSG_RESIDENT=0 turns it off): the
  // mailbox (uncached device memory: doorbell page + slots), the live launch, and the memory
  // epoch its launch saw (block uploads / frees bump mem_epoch: the next query relaunches, so
  // the launch's acquire fence sees the new columns and descriptors as any launch does)
  bool res_on = env_u32("TSG_RESIDENT", 1, 0, 1) != 0;
  // (TSG_RESIDENT_IDLE_US, read at each launch: the idle timeout in us, default 10000)
  uint64_t res_launches = 0, res_queries = 0, res_relaunches = 0, res_quits = 0;  // tsg_device_counters
  uint8_t *res_mem = nullptr;
  uint32_t res_seq = 0;  // last posted sequence number
  bool res_alive = false;
  std::string res_kernel;
  uint64_t res_epoch = 0, mem_epoch = 0;
  HostBuf res_host{nullptr, 0, hipHostMallocMapped | hipHostMallocCoherent};  // [0..63] error word, then query stamps
  // XCD-weighted split (TSG_RES_XSPLIT=0: even runs): each XCD's share of a query's units, from the
  // workgroups' measured {seen, end} stamps (pool.hip res_calibrate); samples taken so far
  double res_xf[8] = {0.125, 0.125, 0.125, 0.125, 0.125, 0.125, 0.125, 0.125};
  uint32_t res_xsamples = 0;
  uint64_t res_qn = 0;
  // slot reads the kernel rejected (check mismatch), queries the plain launches served because
  // another process shares the device, plain-launch narrow queries (tsg_device_counters [4..6])
  uint64_t res_rejects = 0, res_cotenant_queries = 0, res_plain_queries = 0;
  int res_cotenant = -1;          // other processes with a libtsg context on this device (-1: not checked)
  uint32_t res_cotenant_gen = ~0u;  // the shared generation word's value at that check
  uint32_t *cot_gen = nullptr;      // the GPU's shared generation word (pool.hip cotenant_register)
  std::string cot_dir, cot_prefix;
  std::vector<HostBuf> res_quarantine;  // result areas a failed resident query may still write into (kept to shutdown)
  // queries in flight on the resident launch (concurrent callers release mu while theirs run):
  // each holds a result area (pool.hip res_area_bytes); seq -> area index
  struct ResArea {
    HostBuf buf{nullptr, 0, hipHostMallocMapped | hipHostMallocCoherent};
    bool busy = false;
    uint32_t W = 0;
    std::string sym;  // the kernel that serves it (a relaunch after an idle exit uses it)
  };
  std::vector<ResArea> res_areas;
  std::map<uint32_t, uint32_t> res_inflight;
  uint32_t res_threads = 0, res_groups = 0;  // the live launch's shape
  bool res_profile_next = false;  // tsg_search_batch: the next resident launch gets dispatch timestamps
  int res_profile_slot = -1;      // ... its AQL profiling slot
  std::set<const void *> pool_attr;  // pool kernels whose dynamic LDS limit has been raised
  // TSG_PER_CU=k (1..16): scan workgroups per CU in the grid plan instead of the
  // occupancy (k above it oversubscribes: later workgroups start as earlier ones retire)
  int per_cu_override = [] {
    const char *e = std::getenv("TSG_PER_CU");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= 16 ? v : 0;
  }();
  // TSG_SEARCH_TIME_DEFER: event pairs recorded around search kernels, read by tsg_kernel_times
  std::vector<hipEvent_t> tring;
  std::vector<int> tring_aql;  // per deferred slot: its AQL profiling slot, -1 (the event pair), -3 (tring_res)
  std::vector<uint64_t> tring_res;  // per deferred slot served by the resident kernel: its span (ns)
  size_t tring_used = 0;
  bool defer_slot(hipEvent_t &a, hipEvent_t &b) {
    constexpr size_t kMaxDeferred = 4096;
    if (tring_used == kMaxDeferred) return false;
    if (2 * tring_used == tring.size()) {
      hipEvent_t e0, e1;
      HIP_OK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
      HIP_OK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
      tring.push_back(e0);
      tring.push_back(e1);
    }
    a = tring[2 * tring_used];
    b = tring[2 * tring_used + 1];
    if (tring_aql.size() <= tring_used) tring_aql.resize(tring_used + 1);
    tring_aql[tring_used] = -1;
    tring_used++;
    return true;
  }
};



int device_numa_node(const DeviceCtx &dc);
// pool.hip: end the device's resident search launch, if any (before other kernels use the
// device, at shutdown, or when another context opens on the same device)
void resident_quit(DeviceCtx &dc);
void resident_release(DeviceCtx &dc);  // (shutdown: quit, then free the mailbox)
// contexts open on a device ordinal (a resident launch only when this context is the only one);
// context_opened ends the resident launches of the other contexts on the device
int contexts_on(int ordinal);
void context_opened(DeviceCtx &dc);
void context_closed(DeviceCtx &dc);
}  // namespace tsg
