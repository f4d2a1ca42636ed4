// capi.cpp — the extern "C" boundary of libtsg (include/tsg.h). Every entry point
// catches C++ exceptions and maps them to TSG_* codes + the thread-local
// tsg_last_error() text. The search itself only ever runs on a HIP device:
// there is no CPU fallback behind this ABI (the Go shim keeps its own CPU path).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <list>
#include <set>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include <execinfo.h>
#include <sys/syscall.h>
#include <fcntl.h>
#include <csignal>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "block.hpp"
#include "common.hpp"
#include "engine.hpp"
#include "park.hpp"
#include "proto.hpp"
#include "writer.hpp"

// One persistent host thread per device for multi-device calls: a search or lookup whose
// blocks span devices hands each further device's part to that device's worker (the caller
// runs the first device's part itself) instead of starting a thread per device per call.
// Short critical sections concurrent searches share (the coalescer's queue, the result-holder
// pool) take a ParkLock (park.hpp): a bounded spin, then the futex — a contended std::mutex
// parks at once and its wake-up costs tens of microseconds, an unbounded spin keeps a
// preempted holder off its CPU.
using SpinLock = tsg::ParkLock;

struct DevWorker {
  std::mutex m;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  bool stop = false;
  std::thread th;
  DevWorker() : th([this] { run(); }) {}
  ~DevWorker() {
    {
      std::lock_guard<std::mutex> lk(m);
      stop = true;
    }
    cv.notify_all();
    th.join();
  }
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        f = std::move(q.front());
        q.pop_front();
      }
      f();
    }
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(m);
      q.push_back(std::move(f));
    }
    cv.notify_one();
  }
};
// Completion of a set of submitted parts.
struct Latch {
  std::mutex m;
  std::condition_variable cv;
  size_t left;
  explicit Latch(size_t n) : left(n) {}
  void done() {
    std::lock_guard<std::mutex> lk(m);
    if (--left == 0) cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return left == 0; });
  }
};

struct tsg_ctx {
  tsg::Ctx c;
  std::mutex wmu;
  std::unordered_map<const void *, std::unique_ptr<DevWorker>> workers;  // per DeviceCtx
  DevWorker &worker(const void *dc) {
    std::lock_guard<std::mutex> lk(wmu);
    auto &w = workers[dc];
    if (!w) w = std::make_unique<DevWorker>();
    return *w;
  }
  // Runs part(i) for i in [0, n): part 0 on the calling thread, the others on the workers
  // of key(i)'s device; exceptions are collected and the first rethrown.
  template <class Key, class Part>
  void fan_out(size_t n, Key &&key, Part &&part) {
    if (n == 1) {
      part(size_t(0));
      return;
    }
    std::vector<std::exception_ptr> errs(n);
    Latch latch(n - 1);
    for (size_t i = 1; i < n; i++)
      worker(key(i)).submit([&, i] {
        try {
          part(i);
        } catch (...) {
          errs[i] = std::current_exception();
        }
        latch.done();
      });
    try {
      part(size_t(0));
    } catch (...) {
      errs[0] = std::current_exception();
    }
    latch.wait();
    for (auto &e : errs)
      if (e) std::rethrow_exception(e);
  }
  // tsg_cancel (cooperative, like BackendSearchBlock.Search's per-page sr.Quit()): a search
  // with a query id registers it while it runs and checks for a cancel between device
  // chunks and waves. A cancel for a running id marks it; for an id whose search finished
  // less than kLateNs ago (the usual timeout race: the cancel lands just after the search
  // returned) it is dropped, so it cannot fail a later search that reuses the id; any other
  // cancel is kept for kPendingNs (one that overtakes its search start, also for a reused id)
  // and then expires.
  std::mutex cmu;
  std::unordered_map<uint64_t, int> active;        // id -> searches running with it
  std::unordered_set<uint64_t> cancelled;          // marks on running ids
  std::unordered_map<uint64_t, uint64_t> pending;  // id -> time of a cancel before its search
  std::unordered_map<uint64_t, uint64_t> recent;   // id -> when its last search finished (FIFO, bounded)
  std::deque<uint64_t> recent_order;
  static constexpr uint64_t kPendingNs = 10'000'000'000ull;
  static constexpr uint64_t kLateNs = 1'000'000'000ull;
  static uint64_t now_ns() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch())
                        .count());
  }
  void cancel(uint64_t qid) {
    std::lock_guard<std::mutex> lk(cmu);
    if (active.count(qid)) {
      cancelled.insert(qid);
    } else {
      auto r = recent.find(qid);
      if (r != recent.end() && now_ns() - r->second < kLateNs) return;  // late cancel of a finished search
      if (pending.size() >= 4096) {  // expire, then bound
        const uint64_t t = now_ns();
        for (auto it = pending.begin(); it != pending.end();) it = t - it->second > kPendingNs ? pending.erase(it) : ++it;
        if (pending.size() >= 4096) pending.erase(pending.begin());
      }
      pending[qid] = now_ns();
    }
  }
  void begin(uint64_t qid) {
    if (!qid) return;
    std::lock_guard<std::mutex> lk(cmu);
    active[qid]++;
    auto it = pending.find(qid);
    if (it != pending.end()) {
      if (now_ns() - it->second <= kPendingNs) cancelled.insert(qid);
      pending.erase(it);
    }
  }
  bool is_cancelled(uint64_t qid) {
    if (!qid) return false;
    std::lock_guard<std::mutex> lk(cmu);
    return cancelled.count(qid) != 0;
  }
  void forget(uint64_t qid) {
    if (!qid) return;
    std::lock_guard<std::mutex> lk(cmu);
    auto it = active.find(qid);
    if (it != active.end() && --it->second == 0) {
      active.erase(it);
      cancelled.erase(qid);
    }
    auto r = recent.emplace(qid, 0);
    r.first->second = now_ns();
    if (r.second) {
      recent_order.push_back(qid);
      while (recent_order.size() > 4096) {
        recent.erase(recent_order.front());
        recent_order.pop_front();
      }
    }
  }
  // Coalescer (group commit) for concurrent searches on one device. The ingester's
  // searchLocalBlocks starts a goroutine per block and each calls Search on its own
  // (modules/ingester/instance_search.go:164-185), so the shim makes one tsg_search per
  // block. A call whose device part is one launch queues it on the device; one queued
  // caller (the leader) waits a short window for callers still filtering headers, then runs
  // every queued part with an equal query as ONE launch and hands each caller the records
  // of its own blocks. A lone caller runs at once (nobody is approaching).
  struct CoalReq {
    const std::vector<std::pair<uint32_t, tsg::Block *>> *list;
    const tsg_query *q;
    uint32_t limit, flags;
    tsg::SearchOut *out;
    std::atomic<bool> done{false};
    std::atomic<bool> taken{false};  // in a leader's batch (set under the coalescer's lock)
    std::exception_ptr err;
  };
  struct Coalescer {
    SpinLock m;
    std::vector<CoalReq *> pending;
    // leaders running device searches at once (TSG_COAL_LEADERS, default 4): queries that
    // differ run side by side — the resident kernel serves them back to back — while the
    // requests of one query still join one leader's launch
    std::atomic<int> leaders{0};
    // waiters spin (bounded, and only while the host has CPUs to spare), then park on `park`
    // until the leader hands off (park.hpp: an oversubscribed host must not run a spinning
    // waiter instead of the leader)
    tsg::EpochPark park;
    std::atomic<int> spinning{0};
    // searches with a block on this device that have not reached their device stage yet:
    // the leader waits (bounded) for them to queue
    std::atomic<int> approaching{0};
    void wake() { park.notify(); }
  };
  // one per device, created at tsg_init (read without a lock afterwards)
  std::vector<std::pair<const void *, std::unique_ptr<Coalescer>>> coal;
  Coalescer &coalescer(const void *dc) {
    for (auto &x : coal)
      if (x.first == dc) return *x.second;
    throw std::logic_error("coalescer: unknown device");
  }
};
// A search on its way to the device stage, counted on the coalescer of every device its
// blocks are on (Coalescer::approaching), until leave().
struct Approach {
  static constexpr int kMaxDev = 16;
  std::atomic<int> *cnt[kMaxDev];
  int ncnt = 0;
  std::atomic<bool> left{false};
  void add(std::atomic<int> *c) {
    for (int i = 0; i < ncnt; i++)
      if (cnt[i] == c) return;
    if (ncnt == kMaxDev) return;
    cnt[ncnt++] = c;
    c->fetch_add(1, std::memory_order_acq_rel);
  }
  void leave() {
    if (!left.exchange(true, std::memory_order_acq_rel))
      for (int i = 0; i < ncnt; i++) cnt[i]->fetch_sub(1, std::memory_order_acq_rel);
  }
  ~Approach() { leave(); }
};
struct tsg_block {
  tsg::Block b;
  tsg_ctx *ctx = nullptr;
};
struct tsg_proto_block {
  tsg_ctx *ctx = nullptr;
  tsg::ProtoBlock b;
};
struct tsg_v2block {
  tsg::V2Block b;
};

namespace tsg {
tsg_pipeline *pipeline_new(const tsg_request &req);
bool pipeline_matches_block(const tsg_query &q, const uint8_t *hdr, size_t len);
bool pipeline_matches_block_indexed(const tsg_query &q, const HostBlock &h, uint32_t *defer = nullptr);
bool pipeline_matches_stream_header(const tsg_query &q, uint64_t min_dur, uint64_t max_dur,
                                    const std::map<std::string, std::set<std::string>> &tags);

static thread_local std::string g_last_error;
void set_last_error(const std::string &m) { g_last_error = m; }

template <typename F>
static int guard(F &&f) {
  try {
    f();
    return TSG_OK;
  } catch (const Error &e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc &) {
    set_last_error("out of memory");
    return TSG_E_OOM;
  } catch (const std::exception &e) {
    set_last_error(e.what());
    return TSG_E_INVALID;
  }
}

// Holder behind tsg_result: owns the arrays the public struct points into.
struct ResultHolder {
  tsg_result pub{};
  // (RawVec: a result of millions of records is written once, never zero-filled first)
  RawVec<uint8_t> ids, id_len;
  RawVec<uint64_t> start, end, entry;
  RawVec<uint32_t> dur, block, svc_len, name_len;
  RawVec<uint64_t> svc_off, name_off;  // into `arena` (one allocation for every name)
  char *arena = nullptr;  // (grown by hand: no zero-fill, no per-name insert)
  size_t arena_size = 0, arena_cap = 0;
  ResultHolder() = default;
  ResultHolder(const ResultHolder &) = delete;
  ResultHolder &operator=(const ResultHolder &) = delete;
  ~ResultHolder() { std::free(arena); }
  void arena_grow(size_t need) {
    const size_t cap = std::max<size_t>({need, 2 * arena_cap, 4096});
    char *p = static_cast<char *>(std::realloc(arena, cap));
    if (!p) throw std::bad_alloc();
    arena = p;
    arena_cap = cap;
  }
  RawVec<const char *> svc_p, name_p;
  bool ptrs_ready = false;  // svc_p / name_p filled with the records (the arena was final before them)
  std::vector<int32_t> bstatus;      // per caller block
  std::vector<std::string> berr_s;
  std::vector<const char *> berr;
  void set_blocks(size_t nb) {
    bstatus.assign(nb, TSG_OK);
    berr_s.assign(nb, std::string());
  }
  void reserve(size_t n) {
    ids.reserve(16 * n);
    for (auto *v : {&start, &end, &entry, &svc_off, &name_off}) v->reserve(n);
    for (auto *v : {&dur, &block, &svc_len, &name_len}) v->reserve(n);
    id_len.reserve(n);
    if (24 * n > arena_cap) arena_grow(24 * n);
  }
  // names are interned by source: every name comes from a block's host dictionary (or an
  // earlier result), so one dictionary value is copied into the arena once per result and
  // records share its offset (a dense result's arena stays small, and a packed transport
  // can ship the arena as it is)
  struct InternSlot {
    const char *p;
    uint32_t l;
    uint64_t off;
  };
  // slots of an earlier result (another generation) count as empty: a reused holder starts a
  // result in O(1) instead of clearing the table (a query over 10 blocks interns ~1 000 names)
  std::vector<InternSlot> intern;
  std::vector<uint32_t> intern_gen;
  uint32_t gen = 1;
  size_t intern_used = 0;
  uint64_t intern_lookup(const char *p, size_t l) {
    if (intern.empty()) {
      intern.assign(4096, InternSlot{nullptr, 0, 0});
      intern_gen.assign(4096, 0);
    }
    if (2 * (intern_used + 1) > intern.size()) {  // grow: rehash this generation's slots
      std::vector<InternSlot> old;
      std::vector<uint32_t> og;
      old.swap(intern);
      og.swap(intern_gen);
      intern.assign(2 * old.size(), InternSlot{nullptr, 0, 0});
      intern_gen.assign(2 * old.size(), 0);
      intern_used = 0;
      for (size_t i = 0; i < old.size(); i++)
        if (og[i] == gen) intern_insert(old[i].p, old[i].l, old[i].off);
    }
    const size_t mask = intern.size() - 1;
    size_t h = (uintptr_t(p) * 0x9E3779B97F4A7C15ull ^ l) >> 7;
    for (;; h++) {
      InternSlot &x = intern[h & mask];
      if (intern_gen[h & mask] != gen) {
        x = InternSlot{p, uint32_t(l), arena_size};
        intern_gen[h & mask] = gen;
        intern_used++;
        if (arena_size + l > arena_cap) arena_grow(arena_size + l);
        std::memcpy(arena + arena_size, p, l);
        arena_size += l;
        return x.off;
      }
      if (x.p == p && x.l == l) return x.off;
    }
  }
  void intern_insert(const char *p, uint32_t l, uint64_t off) {
    const size_t mask = intern.size() - 1;
    size_t h = (uintptr_t(p) * 0x9E3779B97F4A7C15ull ^ l) >> 7;
    while (intern_gen[h & mask] == gen) h++;
    intern[h & mask] = InternSlot{p, l, off};
    intern_gen[h & mask] = gen;
    intern_used++;
  }
  void set_str(RawVec<uint64_t> &off, RawVec<uint32_t> &len, size_t i, const char *p, size_t l) {
    len[i] = uint32_t(l);
    off[i] = l ? intern_lookup(p, l) : 0;
  }
  // The record loop's names come from one block's root.service.name / root.name dictionaries
  // at a time: a direct-indexed cache per column (value id -> arena offset and length) in
  // front of the pointer-keyed intern table, started afresh for every block (vid_block)
  static constexpr size_t kVcMax = 1 << 16;
  struct VcSlot {
    uint32_t gen, len;
    uint64_t off;
  };
  std::vector<VcSlot> vc[2];
  uint32_t vc_gen = 0;
  void vid_block(size_t nsvc, size_t nname) {
    if (++vc_gen == 0) {
      for (auto &c : vc) std::fill(c.begin(), c.end(), VcSlot{0, 0, 0});
      vc_gen = 1;
    }
    if (nsvc <= kVcMax && vc[0].size() < nsvc) vc[0].resize(nsvc, VcSlot{0, 0, 0});
    if (nname <= kVcMax && vc[1].size() < nname) vc[1].resize(nname, VcSlot{0, 0, 0});
  }
  // record i's name of column c (0 root service, 1 root name): value `vid` of key `key` of h
  void set_vid(int c, size_t i, const HostBlock &h, int key, uint32_t vid) {
    RawVec<uint64_t> &off = c ? name_off : svc_off;
    RawVec<uint32_t> &len = c ? name_len : svc_len;
    if (key < 0 || vid == kNone) {
      len[i] = 0;
      off[i] = 0;
      return;
    }
    VcSlot *slot = vid < vc[c].size() ? &vc[c][vid] : nullptr;
    if (slot && slot->gen == vc_gen) {
      len[i] = slot->len;
      off[i] = slot->off;
      return;
    }
    const std::string_view v = h.dict_value(key, vid);
    len[i] = uint32_t(v.size());
    if (v.empty()) {
      off[i] = 0;
    } else if (small_names) {  // (appended: the per-block cache above is the only dedupe)
      if (arena_size + v.size() > arena_cap) arena_grow(arena_size + v.size());
      std::memcpy(arena + arena_size, v.data(), v.size());
      off[i] = arena_size;
      arena_size += v.size();
    } else {
      off[i] = intern_lookup(v.data(), v.size());
    }
    if (slot) *slot = VcSlot{vc_gen, uint32_t(v.size()), off[i]};
  }
  // A result of few records skips the intern table: its names go to the arena as the records
  // meet them (deduped per block by the value-id cache). The table's probe was ~1/3 of the host
  // time of a 500-record search (tools/host_prof.py); what it saves — a dense result's arena
  // holding each distinct name once — does not arise below a few thousand records.
  bool small_names = false;
  size_t size() const { return start.size(); }
  void resize(size_t n) {
    ids.resize(16 * n);
    for (auto *v : {&start, &end, &entry, &svc_off, &name_off}) v->resize(n);
    for (auto *v : {&dur, &block, &svc_len, &name_len}) v->resize(n);
    id_len.resize(n);
  }
  void set_rec(size_t i, const uint8_t *id, uint8_t il, uint64_t s, uint64_t e, uint32_t b, uint64_t en) {
    std::memcpy(&ids[16 * i], id, 16);
    id_len[i] = il;
    start[i] = s;
    end[i] = e;
    dur[i] = uint32_t((e - s) / 1000000ULL);  // util.go:33
    block[i] = b;
    entry[i] = en;
  }
  void set(size_t i, const uint8_t *id, uint8_t il, uint64_t s, uint64_t e, uint32_t b, uint64_t en, const char *sv,
           size_t svl, const char *nm, size_t nml) {
    set_rec(i, id, il, s, e, b, en);
    set_str(svc_off, svc_len, i, sv, svl);
    set_str(name_off, name_len, i, nm, nml);
  }
  void push(const uint8_t *id, uint8_t il, uint64_t s, uint64_t e, uint32_t b, uint64_t en, const char *sv,
            size_t svl, const char *nm, size_t nml) {
    const size_t i = size();
    resize(i + 1);
    set(i, id, il, s, e, b, en, sv, svl, nm, nml);
  }
  void clear() {  // (for reuse: sizes to zero, capacities kept)
    pub = tsg_result{};
    ids.clear();
    id_len.clear();
    for (auto *v : {&start, &end, &entry, &svc_off, &name_off}) v->clear();
    for (auto *v : {&dur, &block, &svc_len, &name_len}) v->clear();
    arena_size = 0;
    if (intern_used && ++gen == 0) {  // (wrapped: clear once)
      std::fill(intern_gen.begin(), intern_gen.end(), 0u);
      gen = 1;
    }
    intern_used = 0;
    svc_p.clear();
    name_p.clear();
    ptrs_ready = false;
    small_names = false;
    bstatus.clear();
    berr_s.clear();
    berr.clear();
  }
  const char *svc(size_t i) const { return arena + svc_off[i]; }
  const char *name(size_t i) const { return arena + name_off[i]; }
  void finalize() {
    const size_t n = start.size();
    if (!ptrs_ready || svc_p.size() != n || name_p.size() != n) {
      svc_p.resize(n);
      name_p.resize(n);
      parallel_ranges(n, size_t(1) << 18, 16, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; i++) {
          svc_p[i] = svc(i);
          name_p[i] = name(i);
        }
      });
    }
    pub.n = n;
    pub.trace_id = reinterpret_cast<const uint8_t(*)[16]>(ids.data());
    pub.trace_id_len = id_len.data();
    pub.start_ns = start.data();
    pub.end_ns = end.data();
    pub.duration_ms = dur.data();
    pub.block_idx = block.data();
    pub.entry_idx = entry.data();
    pub.root_service = svc_p.data();
    pub.root_service_len = svc_len.data();
    pub.root_name = name_p.data();
    pub.root_name_len = name_len.data();
    pub.names = arena ? arena : "";
    pub.names_len = arena_size;
    pub.root_service_off = svc_off.data();
    pub.root_name_off = name_off.data();
    berr.resize(bstatus.size());
    for (size_t i = 0; i < bstatus.size(); i++) berr[i] = bstatus[i] ? berr_s[i].c_str() : nullptr;
    pub.nblocks = bstatus.size();
    pub.block_status = bstatus.data();
    pub.block_error = berr.data();
  }
};
static_assert(offsetof(ResultHolder, pub) == 0, "pub first");

// Result holders are recycled (a query per ~60 us allocates a dozen arrays and a name
// arena; reusing them keeps allocation and first-touch page faults off the step)
struct HolderPool {
  SpinLock mu;
  std::vector<ResultHolder *> free;
  ~HolderPool() {
    for (auto *h : free) delete h;
  }
};
static HolderPool &holder_pool() {
  static HolderPool *p = new HolderPool();  // (leaked on purpose: results may be freed at exit)
  return *p;
}
static ResultHolder *acquire_holder() {
  HolderPool &hp = holder_pool();
  {
    std::lock_guard<SpinLock> lk(hp.mu);
    if (!hp.free.empty()) {
      ResultHolder *h = hp.free.back();
      hp.free.pop_back();
      return h;
    }
  }
  return new ResultHolder();
}
static void release_holder(ResultHolder *h) {
  if (!h) return;
  HolderPool &hp = holder_pool();
  // large holders (a dense result of millions of records: their pages stay faulted in for
  // the next such query) are kept too, at most 2 of them
  constexpr size_t kSmall = size_t(1) << 20, kBig = size_t(1) << 25;
  const size_t cap = h->start.capacity();
  if (h->arena_cap <= (256u << 20) && cap <= kBig) {
    h->clear();
    std::lock_guard<SpinLock> lk(hp.mu);
    size_t big = 0;
    for (auto *x : hp.free) big += x->start.capacity() > kSmall;
    if (hp.free.size() < 16 && (cap <= kSmall || big < 2)) {
      hp.free.push_back(h);
      return;
    }
  }
  delete h;
}
struct HolderRelease {
  void operator()(ResultHolder *h) const { release_holder(h); }
};

struct LookupHolder {
  tsg_lookup_result pub{};
  LookupOut o;
};
static_assert(offsetof(LookupHolder, pub) == 0, "pub first");
struct FindHolder {
  tsg_find_result pub{};
  FindOut o;
};
static_assert(offsetof(FindHolder, pub) == 0, "pub first");

struct ProtoHolder {
  tsg_proto_result pub{};
  std::vector<uint8_t> ids;
  std::vector<uint32_t> id_off, dur, obj, id_len, svc_len, root_len;
  std::vector<uint64_t> start;
  std::vector<std::string> svc, root;
  std::vector<const char *> svc_p, root_p;
};
static_assert(offsetof(ProtoHolder, pub) == 0, "pub first");

static std::string join(const char *dir, const char *name) { return std::string(dir) + "/" + name; }

template <class Decode>
static void open_common(tsg_ctx *ctx, Decode &&decode, int device_hint, tsg_block **out) {
  auto *b = new tsg_block();
  b->ctx = ctx;
  try {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    decode(*b->b.host);
    const auto t1 = clk::now();
    if (b->b.host->has_meta) block_upload(ctx->c, b->b, device_hint);
    if (prof_on()) {
      prof_add("open.decode", std::chrono::duration<double, std::micro>(t1 - t0).count());
      prof_add("open.upload", std::chrono::duration<double, std::micro>(clk::now() - t1).count());
    }
  } catch (...) {
    block_free(b->b);
    delete b;
    throw;
  }
  // the device holds the columns now; keep only what the host needs (names, header, pages,
  // and the per-entry result columns ids, id_len, start, end, svc_vid, name_vid — 41 bytes
  // per entry — that a dense result's scan positions are gathered from: search.hip
  // "positions -> records", fill_records_direct; kept as columns: at the densities where the
  // gather matters each column is read as a near-sequential stream, which 48-byte rows per
  // entry were not (twice the gather time in cfg4's statement+url query)
  for (size_t k = 0; k < b->b.host->keys.size(); k++) {
    auto &kc = b->b.host->keys[k];
    std::vector<uint32_t>().swap(kc.col);
    if (int(k) != b->b.host->svc_key && int(k) != b->b.host->name_key) {
      Bytes().swap(kc.dict_bytes);
      std::vector<uint32_t>().swap(kc.dict_off);
      std::vector<uint32_t>().swap(kc.set_vals);
      kc.set_off.resize(1);
    }
  }
  *out = b;
}

}  // namespace tsg

using namespace tsg;

extern "C" {

const char *tsg_last_error(void) { return g_last_error.c_str(); }
int tsg_abi_version(void) { return TSG_ABI_VERSION; }
void tsg_free(void *p) { std::free(p); }

// TSG_SEGV_TRACE=1 (diagnostics): a fault in the process prints the native stack (libtsg's
// frames as module + offset: addr2line on the same libtsg.so resolves them), then dies as before
static void segv_trace(int sig) {
  void *frames[64];
  const int n = backtrace(frames, 64);
  static const char msg[] = "[tsg] fatal signal, native stack:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

// ... and SIGUSR2 sent to one thread (pthread_kill: a test's hung caller) prints that thread's
// native stack and lets it go on
static void stack_dump(int) {
  void *frames[64];
  const int n = backtrace(frames, 64);
  char msg[64];
  const int l = std::snprintf(msg, sizeof msg, "[tsg] thread %ld native stack:\n", long(syscall(SYS_gettid)));
  (void)!write(2, msg, size_t(l));
  backtrace_symbols_fd(frames, n, 2);
}

int tsg_init(const tsg_options *opts, tsg_ctx **out) {
  if (!out) return TSG_E_INVALID;
  static const bool segv = [] {
    if (!std::getenv("TSG_SEGV_TRACE")) return false;
    void *f[2];
    (void)backtrace(f, 2);  // (loads the unwinder now, not inside a handler)
    signal(SIGSEGV, segv_trace);
    signal(SIGBUS, segv_trace);
    signal(SIGUSR2, stack_dump);
    return true;
  }();
  (void)segv;
  return guard([&] {
    auto *c = new tsg_ctx();
    try {
      ctx_init(c->c, opts);
      for (auto *dc : c->c.devs) c->coal.emplace_back(dc, std::make_unique<tsg_ctx::Coalescer>());
    } catch (...) {
      ctx_shutdown(c->c);
      delete c;
      throw;
    }
    *out = c;
  });
}
void tsg_shutdown(tsg_ctx *ctx) {
  if (!ctx) return;
  {
    std::lock_guard<std::mutex> lk(ctx->wmu);
    ctx->workers.clear();  // (joins the device workers: idle, no call is in flight)
  }
  ctx_shutdown(ctx->c);
  delete ctx;
}
int tsg_device_count(tsg_ctx *ctx) { return ctx ? int(ctx->c.devs.size()) : 0; }
int tsg_device_numa_node(tsg_ctx *ctx, int dev) {
  if (!ctx || dev < 0 || size_t(dev) >= ctx->c.devs.size()) return -1;
  return device_numa_node(*ctx->c.devs[size_t(dev)]);
}
int tsg_device_counters(tsg_ctx *ctx, int dev, uint64_t *out, size_t n) {
  if (!ctx || !out || dev < 0 || size_t(dev) >= ctx->c.devs.size()) return TSG_E_INVALID;
  return guard([&] {
    uint64_t c[8];
    device_counters(*ctx->c.devs[size_t(dev)], c);
    for (size_t i = 0; i < n; i++) out[i] = i < 8 ? c[i] : 0;
  });
}
int tsg_cancel(tsg_ctx *ctx, uint64_t qid) {
  if (!ctx || !qid) return TSG_E_INVALID;
  ctx->cancel(qid);
  return TSG_OK;
}

int tsg_pipeline_new(const tsg_request *req, tsg_pipeline **out) {
  if (!req || !out) return TSG_E_INVALID;
  return guard([&] { *out = pipeline_new(*req); });
}
const tsg_query *tsg_pipeline_query(const tsg_pipeline *p);
void tsg_pipeline_free(tsg_pipeline *p);

int tsg_pipeline_matches_header(const tsg_query *q, const uint8_t *header, size_t len, int *matches) {
  if (!q || !header || !matches) return TSG_E_INVALID;
  return guard([&] { *matches = pipeline_matches_block(*q, header, len) ? 1 : 0; });
}

// A read-only private mapping of a whole file, pages populated up front (the page data is
// only read while the block decodes: no copy of it into a heap buffer, no zero fill)
struct MappedFile {
  const uint8_t *p = nullptr;
  size_t n = 0;
  void *m = MAP_FAILED;
  std::vector<uint8_t> heap;  // (empty files, or a file the kernel will not map: read instead)
  bool open(const std::string &path) {
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      if (errno == ENOENT) return false;
      fail(TSG_E_IO, "open " + path + ": " + std::strerror(errno));
    }
    struct stat st;
    if (fstat(fd, &st) == 0 && st.st_size > 0)
      m = mmap(nullptr, size_t(st.st_size), PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    ::close(fd);
    if (m != MAP_FAILED) {
      p = static_cast<const uint8_t *>(m);
      n = size_t(st.st_size);
      return true;
    }
    if (!read_file(path, heap)) return false;
    p = heap.data();
    n = heap.size();
    return true;
  }
  ~MappedFile() {
    if (m != MAP_FAILED) munmap(m, n);
  }
};

int tsg_block_open(tsg_ctx *ctx, const char *dir, int device_hint, tsg_block **out) {
  if (!ctx || !dir || !out) return TSG_E_INVALID;
  return guard([&] {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    std::vector<uint8_t> meta, index;
    Bytes header;
    MappedFile data;
    if (!read_file(join(dir, "search.meta.json"), meta)) fail(TSG_E_NOT_FOUND, "search.meta.json not found");
    if (!read_file(join(dir, "search-header"), header)) fail(TSG_E_IO, "search-header missing");
    if (!read_file(join(dir, "search-index"), index)) fail(TSG_E_IO, "search-index missing");
    if (!data.open(join(dir, "search"))) fail(TSG_E_IO, "search missing");
    if (prof_on()) prof_add("open.read", std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    open_common(ctx, [&](HostBlock &h) {
      decode_search_block(meta.data(), meta.size(), true, std::move(header), index.data(), index.size(), data.p,
                          data.n, 0, h);
    }, device_hint, out);
  });
}
int tsg_block_open_pages(tsg_ctx *ctx, const char *dir, uint32_t first_page, uint32_t npages, int device_hint,
                         tsg_block **out) {
  if (!ctx || !dir || !out || !npages) return TSG_E_INVALID;
  return guard([&] {
    std::vector<uint8_t> meta, index;
    Bytes header;
    MappedFile data;
    if (!read_file(join(dir, "search.meta.json"), meta)) fail(TSG_E_NOT_FOUND, "search.meta.json not found");
    if (!read_file(join(dir, "search-header"), header)) fail(TSG_E_IO, "search-header missing");
    if (!read_file(join(dir, "search-index"), index)) fail(TSG_E_IO, "search-index missing");
    if (!data.open(join(dir, "search"))) fail(TSG_E_IO, "search missing");
    open_common(ctx, [&](HostBlock &h) {
      decode_search_block(meta.data(), meta.size(), true, std::move(header), index.data(), index.size(), data.p,
                          data.n, 0, h, first_page, npages);
    }, device_hint, out);
  });
}
int tsg_block_open_mem(tsg_ctx *ctx, const uint8_t *meta, size_t ml, const uint8_t *header, size_t hl,
                       const uint8_t *index, size_t il, const uint8_t *data, size_t dl, int device_hint,
                       tsg_block **out) {
  if (!ctx || !out) return TSG_E_INVALID;
  return guard([&] {
    if (!meta) fail(TSG_E_NOT_FOUND, "search.meta.json not provided");
    Bytes hv(header, header + hl);
    open_common(ctx, [&](HostBlock &h) { decode_search_block(meta, ml, true, std::move(hv), index, il, data, dl, 0, h); },
                device_hint, out);
  });
}
int tsg_wal_block_open(tsg_ctx *ctx, const char *path, int device_hint, tsg_block **out) {
  if (!ctx || !path || !out) return TSG_E_INVALID;
  return guard([&] {
    std::string p(path), version;
    const size_t slash = p.find_last_of('/');
    const int enc = parse_wal_filename(slash == std::string::npos ? p : p.substr(slash + 1), version);
    std::vector<uint8_t> data;
    if (!read_file(p, data)) fail(TSG_E_IO, "wal file missing");
    open_common(ctx, [&](HostBlock &h) { decode_wal_search_block(data.data(), data.size(), enc, h); }, device_hint, out);
  });
}
int tsg_wal_block_open_mem(tsg_ctx *ctx, const uint8_t *data, size_t len, int encoding, int device_hint,
                           tsg_block **out) {
  if (!ctx || (len && !data) || !out) return TSG_E_INVALID;
  return guard([&] {
    open_common(ctx, [&](HostBlock &h) { decode_wal_search_block(data, len, encoding, h); }, device_hint, out);
  });
}
int tsg_live_block_open_mem(tsg_ctx *ctx, const uint8_t *bytes, const uint64_t *seg_off, size_t nsegs,
                            const uint64_t *trace_seg, size_t ntraces, int device_hint, tsg_block **out) {
  if (!ctx || !out || !trace_seg || (nsegs && (!bytes || !seg_off)) || ntraces > 0xffffffffu) return TSG_E_INVALID;
  return guard([&] {
    static const uint64_t zero = 0;
    const uint64_t *so = nsegs ? seg_off : &zero;
    open_common(ctx, [&](HostBlock &h) { decode_live_block(bytes, so, nsegs, trace_seg, uint32_t(ntraces), h); },
                device_hint, out);
  });
}
int tsg_block_clone(tsg_ctx *ctx, const tsg_block *src, int device_hint, tsg_block **out) {
  if (!ctx || !src || !out) return TSG_E_INVALID;
  return guard([&] {
    auto *b = new tsg_block();
    b->ctx = ctx;
    try {
      if (src->b.host->has_meta) block_clone(ctx->c, src->b, b->b, device_hint);
      else b->b.host = src->b.host;
    } catch (...) {
      block_free(b->b);
      delete b;
      throw;
    }
    *out = b;
  });
}
void tsg_block_close(tsg_block *b) {
  if (!b) return;
  block_free(b->b);
  delete b;
}
int tsg_block_info_get(const tsg_block *b, tsg_block_info *o) {
  if (!b || !o) return TSG_E_INVALID;
  const HostBlock &h = *b->b.host;
  o->entries = h.n;
  o->pages = h.page_entries.size();
  o->keys = h.keys.size();
  o->header_bytes = h.header.size();
  o->fb_bytes = h.fb_bytes;
  o->device_bytes = b->b.dev.bytes;
  o->min_dur_ns = h.min_dur;
  o->max_dur_ns = h.max_dur;
  o->device = b->b.dev.device;
  o->encoding = h.meta.encoding;
  o->streaming = h.streaming ? 1 : 0;
  o->partial = h.partial ? 1 : 0;
  o->stop_status = h.stop_status;
  o->index_truncated = h.index_truncated ? 1 : 0;
  o->live = h.live ? 1 : 0;
  o->hdr_deferred = 0;
  for (uint8_t d : h.hdr_defer) o->hdr_deferred += d ? 1 : 0;
  o->traces = h.live ? h.ntraces() : h.n;
  return TSG_OK;
}

static void pack_strings(const std::vector<std::string> &v, uint8_t **out, size_t *len, size_t *n) {
  size_t total = 0;
  for (auto &s : v) total += 4 + s.size();
  auto *p = static_cast<uint8_t *>(std::malloc(total ? total : 1));
  size_t o = 0;
  for (auto &s : v) {
    uint32_t l = uint32_t(s.size());
    std::memcpy(p + o, &l, 4);
    std::memcpy(p + o + 4, s.data(), s.size());
    o += 4 + s.size();
  }
  *out = p;
  *len = total;
  *n = v.size();
}

// SearchableBlock.Tags / TagValues of one block into a set (sorted, unique):
// BackendSearchBlock (backend_search_block.go:145-181) on the header rollup,
// StreamingSearchBlock (streaming_search_block.go:97-116) on the replayed mutable header,
// live traces (instance_search.go:191-200, 229-240) on every segment.
static void block_tags_into(const tsg_block *b, std::set<std::string> &keys) {
  const HostBlock &h = *b->b.host;
  if (h.live) {  // every KeyValues key of every segment (with or without values)
    for (const auto &kc : h.keys) keys.insert(kc.name);
    return;
  }
  if (h.streaming) {
    for (auto &kv : h.stream_tags) keys.insert(kv.first);
    return;
  }
  if (!h.has_meta) fail(TSG_E_NOT_FOUND, "search-header does not exist");
  const auto &hb = h.header;
  FbTable t = FbTable::root(hb.data(), hb.size());
  uint16_t o = t.field(kHdrTags);
  uint32_t cnt = o ? t.vector_len(o) : 0, st = o ? t.vector_start(o) : 0;
  FbTable kv{hb.data(), hb.size(), 0};
  for (uint32_t i = 0; i < cnt; i++) {
    kv.pos = t.indirect(st + 4 * i);
    uint16_t ko = kv.field(kKvKey);
    keys.insert(std::string(ko ? kv.byte_vector(kv.pos + ko) : std::string_view()));
  }
}
static void block_tag_values_into(const tsg_block *b, std::string_view key, std::set<std::string> &vals) {
  const HostBlock &h = *b->b.host;
  if (h.live || h.streaming) {
    auto it = h.stream_tags.find(std::string(key));
    if (it != h.stream_tags.end()) vals.insert(it->second.begin(), it->second.end());
    return;
  }
  if (!h.has_meta) fail(TSG_E_NOT_FOUND, "search-header does not exist");
  const auto &hb = h.header;
  FbTable t = FbTable::root(hb.data(), hb.size());
  uint16_t o = t.field(kHdrTags);
  uint32_t cnt = o ? t.vector_len(o) : 0, st = o ? t.vector_start(o) : 0;
  FbTable kv{hb.data(), hb.size(), 0};
  uint32_t i = 0, j = cnt;  // FindTag binary search (searchdata_util.go:63-100)
  bool found = false;
  while (i < j) {
    uint32_t m = (i + j) >> 1;
    kv.pos = t.indirect(st + 4 * m);
    uint16_t ko = kv.field(kKvKey);
    std::string_view kk = ko ? kv.byte_vector(kv.pos + ko) : std::string_view();
    int c = bytes_compare(reinterpret_cast<const uint8_t *>(kk.data()), kk.size(),
                          reinterpret_cast<const uint8_t *>(key.data()), key.size());
    if (c == 0) {
      found = true;
      break;
    }
    if (c < 0) j = m;
    else i = m + 1;
  }
  if (!found) return;
  uint16_t vo = kv.field(kKvValue);
  uint32_t vn = vo ? kv.vector_len(vo) : 0, vs = vo ? kv.vector_start(vo) : 0;
  for (uint32_t q = 0; q < vn; q++) vals.insert(std::string(kv.byte_vector(vs + 4 * q)));
}
static void pack_set(const std::set<std::string> &v, uint8_t **out, size_t *len, size_t *n) {
  pack_strings(std::vector<std::string>(v.begin(), v.end()), out, len, n);
}

int tsg_block_tags(const tsg_block *b, uint8_t **out, size_t *len, size_t *n) {
  if (!b || !out || !len || !n) return TSG_E_INVALID;
  return guard([&] {
    std::set<std::string> keys;
    block_tags_into(b, keys);
    pack_set(keys, out, len, n);
  });
}
int tsg_block_tag_values(const tsg_block *b, const uint8_t *key, size_t klen, uint8_t **out, size_t *len,
                         size_t *n) {
  if (!b || !out || !len || !n || (klen && !key)) return TSG_E_INVALID;
  return guard([&] {
    std::set<std::string> vals;
    block_tag_values_into(b, std::string_view(reinterpret_cast<const char *>(key), klen), vals);
    pack_set(vals, out, len, n);
  });
}
// instance.SearchTags (instance_search.go:187-215): live traces, then WAL and local blocks
int tsg_search_tags(tsg_block *const *blocks, size_t nblocks, uint8_t **out, size_t *len, size_t *n) {
  if ((nblocks && !blocks) || !out || !len || !n) return TSG_E_INVALID;
  return guard([&] {
    std::set<std::string> keys;
    for (int pass = 0; pass < 2; pass++)
      for (size_t i = 0; i < nblocks; i++)
        if (blocks[i]->b.host->live == (pass == 0)) block_tags_into(blocks[i], keys);
    pack_set(keys, out, len, n);
  });
}
// instance.SearchTagValues (instance_search.go:217-273) with util.MapSizeWithinLimit
// (pkg/util/map_size.go:4-11) after the live traces and after every block
int tsg_search_tag_values(tsg_block *const *blocks, size_t nblocks, const uint8_t *key, size_t klen,
                          int64_t max_bytes, uint8_t **out, size_t *len, size_t *n) {
  if ((nblocks && !blocks) || (klen && !key) || !out || !len || !n) return TSG_E_INVALID;
  return guard([&] {
    const std::string_view k(reinterpret_cast<const char *>(key), klen);
    std::set<std::string> vals;
    for (int pass = 0; pass < 2; pass++) {
      for (size_t i = 0; i < nblocks; i++)
        if (blocks[i]->b.host->live == (pass == 0)) block_tag_values_into(blocks[i], k, vals);
      if (max_bytes >= 0) {
        int64_t size = 0;
        for (const auto &v : vals) size += int64_t(v.size());
        if (!(size < max_bytes)) {  // "exceeded limit": an empty response
          vals.clear();
          break;
        }
      }
    }
    pack_set(vals, out, len, n);
  });
}

static bool same_query(const tsg_query &a, const tsg_query &b) {
  if (&a == &b) return true;
  if (a.nterms != b.nterms || a.has_min != b.has_min || a.has_max != b.has_max || a.has_range != b.has_range ||
      a.exhaustive != b.exhaustive || a.min_ns != b.min_ns || a.max_ns != b.max_ns || a.start_s != b.start_s ||
      a.end_s != b.end_s)
    return false;
  for (uint32_t t = 0; t < a.nterms; t++)
    if (a.key_lens[t] != b.key_lens[t] || a.value_lens[t] != b.value_lens[t] ||
        std::memcmp(a.keys[t], b.keys[t], a.key_lens[t]) != 0 ||
        std::memcmp(a.values[t], b.values[t], a.value_lens[t]) != 0)
      return false;
  return true;
}

// How long a coalesced caller spins before it parks (TSG_WAIT_SPIN_US, default 40 µs: about
// a limit query's launch, so that on a host with CPUs to spare the hand-off costs no wake-up).
static uint64_t wait_spin_ns() {
  static const uint64_t ns = [] {
    const char *e = std::getenv("TSG_WAIT_SPIN_US");
    return uint64_t(e ? std::max(0, std::atoi(e)) : 40) * 1000ull;
  }();
  return ns;
}

// tsg_search_batch's worker threads: their searches skip the coalescer (each item is its own
// query; the resident kernel serves the items' queries back to back instead)
static thread_local bool tl_batch_item = false;

// device_search through the device's coalescer (tsg_ctx::Coalescer). TSG_COALESCE=0 turns
// it off; TSG_COALESCE_US (default 30) bounds the leader's wait for approaching callers.
static void coalesced_search(tsg_ctx *ctx, DeviceCtx *dc, const std::vector<std::pair<uint32_t, Block *>> &list,
                             const tsg_query &q, uint32_t limit, uint32_t flags, SearchOut &out, Approach &ap) {
  static const bool on = [] {
    const char *e = std::getenv("TSG_COALESCE");
    return !e || std::atoi(e) != 0;
  }();
  static const uint64_t window_ns = [] {
    const char *e = std::getenv("TSG_COALESCE_US");
    return uint64_t(e ? std::max(0, std::atoi(e)) : 30) * 1000ull;
  }();
  static const int max_leaders = [] {
    const char *e = std::getenv("TSG_COAL_LEADERS");
    return e ? std::max(1, std::min(64, std::atoi(e))) : 4;
  }();
  constexpr size_t kBatchBlocks = 32;  // one launch's kernel-argument capacity
  if (!on || tl_batch_item) {
    ap.leave();
    device_search(*dc, list, q, limit, flags, out);
    return;
  }
  tsg_ctx::Coalescer &c = ctx->coalescer(dc);
  tsg_ctx::CoalReq r;
  r.list = &list;
  r.q = &q;
  r.limit = limit;
  r.flags = flags;
  r.out = &out;
  {
    std::lock_guard<SpinLock> lk(c.m);
    c.pending.push_back(&r);
  }
  ap.leave();
  const auto t_wait = std::chrono::steady_clock::now();
  bool spun = false;
  for (;;) {
    if (r.done.load(std::memory_order_acquire)) break;
    int cur = c.leaders.load(std::memory_order_relaxed);
    if (r.taken.load(std::memory_order_acquire) || cur >= max_leaders ||
        !c.leaders.compare_exchange_strong(cur, cur + 1, std::memory_order_acq_rel)) {
      // A waiter: the leader hands off by setting `done` (or clearing `busy`) and bumping the
      // park epoch. Spin once, for at most spin_ns and only while fewer waiters spin than the
      // caller's CPUs leave room for beside the leader; then park (bounded re-checks).
      const uint32_t e = c.park.read();
      auto ready = [&] {
        return r.done.load(std::memory_order_acquire) ||
               (!r.taken.load(std::memory_order_acquire) && c.leaders.load(std::memory_order_acquire) < max_leaders);
      };
      if (ready()) continue;
      if (!spun) {
        spun = true;
        const int cpus = tsg::host_threads_now();
        if (c.spinning.fetch_add(1, std::memory_order_acq_rel) + 2 < cpus && tsg::spin_for(wait_spin_ns(), ready)) {
          c.spinning.fetch_sub(1, std::memory_order_acq_rel);
          continue;
        }
        c.spinning.fetch_sub(1, std::memory_order_acq_rel);
      }
      const auto tp = std::chrono::steady_clock::now();
      const bool woke = c.park.wait(e, 5'000'000);
      if (prof_on()) {
        prof_add("coal.park_us", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tp).count());
        if (!woke) prof_add("coal.park_timeout", 1.0);
      }
      continue;
    }
    if (r.done.load(std::memory_order_acquire)) {  // served while we took the lead
      c.leaders.fetch_sub(1, std::memory_order_acq_rel);
      c.wake();
      break;
    }
    // leader: give callers still on their way a moment to queue (bounded)
    const bool prof = prof_on();
    const auto t_lead = std::chrono::steady_clock::now();
    if (prof) prof_add("coal.lead_after_us", std::chrono::duration<double, std::micro>(t_lead - t_wait).count());
    if (window_ns) tsg::spin_for(window_ns, [&] { return c.approaching.load(std::memory_order_acquire) <= 0; });
    // the batch: this caller's part first, then every queued part with the same query,
    // per-block limit and flags, up to one launch's blocks
    thread_local std::vector<tsg_ctx::CoalReq *> batch;
    thread_local std::vector<std::pair<uint32_t, Block *>> blist;
    thread_local std::vector<std::pair<uint32_t, uint32_t>> owner;  // batch position -> (request, caller index)
    batch.clear();
    blist.clear();
    owner.clear();
    bool own_taken = false;
    {
      std::lock_guard<SpinLock> lk(c.m);
      // (another leader may have taken this request into its batch already: then it serves it)
      own_taken = std::find(c.pending.begin(), c.pending.end(), &r) == c.pending.end();
      size_t nb = 0;
      auto take = [&](size_t k) {
        tsg_ctx::CoalReq *x = c.pending[k];
        x->taken.store(true, std::memory_order_release);
        for (const auto &p : *x->list) {
          owner.push_back({uint32_t(batch.size()), p.first});
          blist.push_back({uint32_t(blist.size()), p.second});
        }
        nb += x->list->size();
        batch.push_back(x);
        c.pending[k] = nullptr;
      };
      for (size_t k = 0; k < c.pending.size() && !own_taken; k++)
        if (c.pending[k] == &r) take(k);
      for (size_t k = 0; k < c.pending.size() && !own_taken; k++) {
        tsg_ctx::CoalReq *x = c.pending[k];
        if (!x || x->limit != limit || x->flags != flags || nb + x->list->size() > kBatchBlocks ||
            !same_query(*x->q, q))
          continue;
        take(k);
      }
      c.pending.erase(std::remove(c.pending.begin(), c.pending.end(), nullptr), c.pending.end());
    }
    if (own_taken) {  // a waiter again, for the leader that took it
      c.leaders.fetch_sub(1, std::memory_order_acq_rel);
      c.wake();
      spun = false;
      continue;
    }
    if (prof) {
      prof_add("coal.window_us", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_lead).count());
      prof_add("coal.batch_callers", double(batch.size()));
    }
    if (batch.size() == 1) {  // alone: straight into the caller's output
      try {
        device_search(*dc, list, q, limit, flags, out);
      } catch (...) {
        r.err = std::current_exception();
      }
      r.done.store(true, std::memory_order_release);
      c.leaders.fetch_sub(1, std::memory_order_acq_rel);
      c.wake();
      break;
    }
    thread_local SearchOut bout;
    bout.want_pos = false;  // (the batch's records are split among the callers below)
    std::exception_ptr err;
    try {
      device_search(*dc, blist, q, limit, flags, bout);
    } catch (...) {
      err = std::current_exception();
    }
    if (err) {
      // the batched launch failed (device memory, a device error): each caller's part runs
      // on its own, so that one caller's failure is not every caller's
      for (auto *x : batch) {
        try {
          device_search(*dc, *x->list, *x->q, limit, flags, *x->out);
        } catch (...) {
          x->err = std::current_exception();
        }
        x->done.store(true, std::memory_order_release);
      }
      c.leaders.fetch_sub(1, std::memory_order_acq_rel);
      c.wake();
      break;
    }
    // each caller: its blocks' records (the batch's are grouped by position, in order), its
    // share of the algorithmic bytes (by entries), the launch's device time
    uint64_t n_all = 0;
    for (const auto &p : blist) n_all += p.second->host->n;
    for (size_t k = 0; k < batch.size(); k++) {
      SearchOut &o = *batch[k]->out;
      o.recs.clear();
      o.block_counts.clear();
      uint64_t n_mine = 0;
      for (const auto &p : *batch[k]->list) n_mine += p.second->host->n;
      const double share = n_all ? double(n_mine) / double(n_all) : 0.0;
      o.device_bytes = uint64_t(double(bout.device_bytes) * share);
      o.scan_bytes = uint64_t(double(bout.scan_bytes) * share);
      o.kernel_ns = bout.kernel_ns;
      o.scan_ns = bout.scan_ns;
      o.reruns = batch[k] == &r ? bout.reruns : 0;
      o.pool = bout.pool;
      o.path = bout.path;
      o.term_any.clear();
    }
    for (const auto &rec : bout.recs) {
      const auto &ow = owner[rec.block_il & 0xffffffu];
      SearchOut::Rec x = rec;
      x.block_il = (rec.block_il & 0xff000000u) | ow.second;
      batch[ow.first]->out->recs.push_back(x);
    }
    for (const auto &ta : bout.term_any) {
      const auto &ow = owner[ta.first];
      batch[ow.first]->out->term_any.push_back({ow.second, ta.second});
    }
    for (auto *x : batch) x->done.store(true, std::memory_order_release);
    c.leaders.fetch_sub(1, std::memory_order_acq_rel);
    c.wake();
    if (prof) prof_add("coal.lead_total_us", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_lead).count());
    break;
  }
  if (prof_on()) prof_add("coal.call_us", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_wait).count());
  if (r.err) std::rethrow_exception(r.err);
}

// Distinct trace ids for the consumer's limit count: open addressing over the 16-byte
// ids (no allocation per insert; a search reuses its thread's table).
struct IdSet {
  std::vector<uint64_t> key;  // two words per slot
  std::vector<uint8_t> used;
  size_t n = 0;
  void clear() {
    if (n) std::fill(used.begin(), used.end(), uint8_t(0));
    n = 0;
  }
  size_t size() const { return n; }
  bool insert(const uint8_t *id) {
    if ((n + 1) * 2 > used.size()) grow();
    uint64_t a, b;
    std::memcpy(&a, id, 8);
    std::memcpy(&b, id + 8, 8);
    return put(a, b);
  }

 private:
  bool put(uint64_t a, uint64_t b) {
    const size_t mask = used.size() - 1;
    uint64_t h = (a ^ (b * 0x9e3779b97f4a7c15ull)) * 0xff51afd7ed558ccdull;
    h ^= h >> 29;
    for (size_t i = size_t(h) & mask;; i = (i + 1) & mask) {
      if (!used[i]) {
        used[i] = 1;
        key[2 * i] = a;
        key[2 * i + 1] = b;
        n++;
        return true;
      }
      if (key[2 * i] == a && key[2 * i + 1] == b) return false;
    }
  }
  void grow() {
    std::vector<uint64_t> ok;
    std::vector<uint8_t> ou;
    ok.swap(key);
    ou.swap(used);
    const size_t cap = std::max<size_t>(64, ou.size() * 2);
    key.assign(2 * cap, 0);
    used.assign(cap, 0);
    n = 0;
    for (size_t i = 0; i < ou.size(); i++)
      if (ou[i]) put(ok[2 * i], ok[2 * i + 1]);
  }
};

// Record `x` (entry | block index << 32, a compact device output) of block h from its host
// columns (the ones the device columns were uploaded from).
static inline SearchOut::Rec rec_from_pos(const HostBlock &h, uint64_t x) {
  const uint32_t e = uint32_t(x);
  if (e >= h.start.size() || uint64_t(e) * 16 + 16 > h.ids.size())
    fail(TSG_E_DEVICE, "device position outside its block's host columns");
  SearchOut::Rec r;
  std::memcpy(r.id, h.ids.data() + uint64_t(e) * 16, 16);
  r.start = h.start[e];
  r.end = h.end[e];
  r.entry = e;
  r.block_il = uint32_t(x >> 32) | (uint32_t(h.id_len[e]) << 24);
  r.svc = h.svc_vid.empty() ? kNone : h.svc_vid[e];
  r.name = h.name_vid.empty() ? kNone : h.name_vid[e];
  return r;
}

// Per distinct HostBlock: its root.service.name / root.name values' arena offsets and lengths
// by value id (every value interned up front: the arena is final before any record is written).
struct FillNames {
  struct Names {
    const HostBlock *h;
    std::vector<uint64_t> off[2];
    std::vector<uint32_t> len[2];
  };
  std::vector<Names> tabs;
  std::vector<int> tab_of;  // per caller block: its table (-1: none)
};
// Tables for the caller blocks i with use[i]; false when the names are many next to `nrec`
// records (or the blocks many distinct ones): the per-thread arena path is used then.
static bool fill_names(ResultHolder &res, tsg_block *const *blocks, size_t nblocks, size_t nrec,
                       const std::vector<uint8_t> &use, FillNames &fn) {
  auto &tabs = fn.tabs;
  tabs.clear();
  fn.tab_of.assign(nblocks, -1);
  size_t nvals = 0;
  for (size_t i = 0; i < nblocks; i++) {
    if (!use[i]) continue;
    const HostBlock *h = blocks[i]->b.host.get();
    int t = -1;
    for (size_t k = 0; k < tabs.size() && t < 0; k++)
      if (tabs[k].h == h) t = int(k);
    if (t < 0) {
      if (tabs.size() >= 64) return false;  // (many distinct blocks: the per-thread path)
      t = int(tabs.size());
      tabs.push_back(FillNames::Names{h, {}, {}});
      for (int c = 0; c < 2; c++) {
        const int key = c ? h->name_key : h->svc_key;
        nvals += key >= 0 ? h->keys[size_t(key)].nvals() : 0;
      }
    }
    fn.tab_of[i] = t;
  }
  if (nvals * 4 > nrec + 4096) return false;
  const auto t_names = std::chrono::steady_clock::now();
  for (auto &tb : tabs)
    for (int c = 0; c < 2; c++) {
      const int key = c ? tb.h->name_key : tb.h->svc_key;
      const size_t nv = key >= 0 ? tb.h->keys[size_t(key)].nvals() : 0;
      tb.off[c].resize(nv);
      tb.len[c].resize(nv);
      for (size_t v = 0; v < nv; v++) {
        const std::string_view x = tb.h->dict_value(key, uint32_t(v));
        tb.len[c][v] = uint32_t(x.size());
        tb.off[c][v] = x.empty() ? 0 : res.intern_lookup(x.data(), x.size());
      }
    }
  if (prof_on())
    prof_add("fill.names", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_names).count());
  return true;
}

// Output records [o_begin, o_end) (record o of block i: obase[i] <= o < obase[i + 1]) on nt
// threads, names from fn (fill_names done; the arena no longer grows); the result arrays
// hold o_end records.
static void fill_direct_range(ResultHolder &res, tsg_block *const *blocks,
                              const std::vector<std::pair<const SearchOut::Rec *, size_t>> &per_block,
                              const std::vector<const uint64_t *> &per_pos, const std::vector<size_t> &obase,
                              size_t o_begin, size_t o_end, size_t nt, const FillNames &fn) {
  using Names = FillNames::Names;
  const auto &tabs = fn.tabs;
  const auto &tab_of = fn.tab_of;
  const size_t nout = o_end - o_begin;
  if (!nout) return;
  res.svc_p.resize(o_end);
  res.name_p.resize(o_end);
  const char *const arena = res.arena ? res.arena : "";
  std::atomic<bool> bad{false};
  const bool prof = prof_on();
  static const bool passes = [] {  // TSG_FILL_PASSES=0: positions gathered record by record (A/B)
    const char *e = std::getenv("TSG_FILL_PASSES");
    return !e || std::atoi(e) != 0;
  }();
  static const bool nts = [] {  // TSG_FILL_NT=0: the passes with plain stores (A/B)
    const char *e = std::getenv("TSG_FILL_NT");
    return !e || std::atoi(e) != 0;
  }();
  const auto t_par = std::chrono::steady_clock::now();
  // a name column's (offset, length, pointer) for value id v of table c
  auto put_name = [&](const Names &tb, int c, uint32_t v, size_t o) {
    uint64_t off = 0;
    uint32_t len = 0;
    if (v != kNone && v < tb.off[c].size()) {
      off = tb.off[c][v];
      len = tb.len[c][v];
    }
    (c ? res.name_off : res.svc_off)[o] = off;
    (c ? res.name_len : res.svc_len)[o] = len;
    (c ? res.name_p : res.svc_p)[o] = arena + off;
  };
  // Each thread takes a contiguous output range and walks it block run by block run. A run of
  // scan positions is filled in column passes (each pass: the positions, one or two source
  // columns, its own outputs — a record-at-a-time gather kept 6 input and 12 output streams
  // open per thread: 4.2 vs 2.9 ms for config 4's 1.85 M records, tools/probe/fill_probe.cpp);
  // a run of device records is copied record by record (one input stream).
  parallel_ranges(nt, 1, int(nt), [&](size_t t0, size_t t1) {
    for (size_t t = t0; t < t1; t++) {
      const size_t o0 = o_begin + nout * t / nt, o1 = o_begin + nout * (t + 1) / nt;
      if (o0 >= o1) continue;
      size_t i = size_t(std::upper_bound(obase.begin(), obase.end(), o0) - obase.begin()) - 1;
      for (size_t r0 = o0; r0 < o1; i++) {
        if (r0 >= obase[i + 1]) continue;
        const size_t r1 = std::min(o1, obase[i + 1]);
        const HostBlock &h = *blocks[i]->b.host;
        const Names &tb = tabs[size_t(tab_of[i])];
        const uint64_t *pp = per_pos[i] ? per_pos[i] - obase[i] : nullptr;
        if (pp && !passes) {
          for (size_t o = r0; o < r1; o++) {
            const uint32_t e = uint32_t(pp[o]);
            if (e >= h.start.size() || uint64_t(e) * 16 + 16 > h.ids.size()) {
              bad.store(true, std::memory_order_relaxed);
              return;
            }
            std::memcpy(&res.ids[16 * o], h.ids.data() + uint64_t(e) * 16, 16);
            const uint64_t st = h.start[e], en = h.end[e];
            res.start[o] = st;
            res.end[o] = en;
            res.dur[o] = uint32_t((en - st) / 1000000ULL);  // util.go:33
            res.id_len[o] = h.id_len[e];
            res.entry[o] = e;
            res.block[o] = uint32_t(i);
            put_name(tb, 0, h.svc_vid.empty() ? kNone : h.svc_vid[e], o);
            put_name(tb, 1, h.name_vid.empty() ? kNone : h.name_vid[e], o);
          }
        } else if (pp && nts) {  // the same passes with non-temporal stores (no read for ownership)
          typedef long long v2di __attribute__((vector_size(16)));
          for (size_t o = r0; o < r1; o++) {
            const uint32_t e = uint32_t(pp[o]);
            if (e >= h.start.size() || uint64_t(e) * 16 + 16 > h.ids.size()) {
              bad.store(true, std::memory_order_relaxed);
              return;
            }
            v2di v;
            std::memcpy(&v, h.ids.data() + uint64_t(e) * 16, 16);
            __builtin_nontemporal_store(v, reinterpret_cast<v2di *>(&res.ids[16 * o]));
          }
          for (size_t o = r0; o < r1; o++) {
            const uint32_t e = uint32_t(pp[o]);
            const uint64_t st = h.start[e], en = h.end[e];
            __builtin_nontemporal_store(st, &res.start[o]);
            __builtin_nontemporal_store(en, &res.end[o]);
            __builtin_nontemporal_store(uint32_t((en - st) / 1000000ULL), &res.dur[o]);  // util.go:33
          }
          for (size_t o = r0; o < r1; o++) {
            const uint32_t e = uint32_t(pp[o]);
            res.id_len[o] = h.id_len[e];
            __builtin_nontemporal_store(uint64_t(e), &res.entry[o]);
            __builtin_nontemporal_store(uint32_t(i), &res.block[o]);
          }
          for (int c = 0; c < 2; c++) {
            const std::vector<uint32_t> &vid = c ? h.name_vid : h.svc_vid;
            uint64_t *offp = c ? res.name_off.data() : res.svc_off.data();
            uint32_t *lenp = c ? res.name_len.data() : res.svc_len.data();
            const char **ptrp = c ? res.name_p.data() : res.svc_p.data();
            for (size_t o = r0; o < r1; o++) {
              const uint32_t v = vid.empty() ? kNone : vid[uint32_t(pp[o])];
              uint64_t off = 0;
              uint32_t len = 0;
              if (v != kNone && v < tb.off[c].size()) {
                off = tb.off[c][v];
                len = tb.len[c][v];
              }
              __builtin_nontemporal_store(off, &offp[o]);
              __builtin_nontemporal_store(len, &lenp[o]);
              __builtin_nontemporal_store(arena + off, &ptrp[o]);
            }
          }
          __builtin_ia32_sfence();
        } else if (pp) {
          for (size_t o = r0; o < r1; o++) {
            const uint32_t e = uint32_t(pp[o]);
            if (e >= h.start.size() || uint64_t(e) * 16 + 16 > h.ids.size()) {
              bad.store(true, std::memory_order_relaxed);
              return;
            }
            std::memcpy(&res.ids[16 * o], h.ids.data() + uint64_t(e) * 16, 16);
          }
          for (size_t o = r0; o < r1; o++) {
            const uint32_t e = uint32_t(pp[o]);
            const uint64_t st = h.start[e], en = h.end[e];
            res.start[o] = st;
            res.end[o] = en;
            res.dur[o] = uint32_t((en - st) / 1000000ULL);  // util.go:33
          }
          for (size_t o = r0; o < r1; o++) {
            const uint32_t e = uint32_t(pp[o]);
            res.id_len[o] = h.id_len[e];
            res.entry[o] = e;
            res.block[o] = uint32_t(i);
          }
          for (size_t o = r0; o < r1; o++) put_name(tb, 0, h.svc_vid.empty() ? kNone : h.svc_vid[uint32_t(pp[o])], o);
          for (size_t o = r0; o < r1; o++) put_name(tb, 1, h.name_vid.empty() ? kNone : h.name_vid[uint32_t(pp[o])], o);
        } else {
          const SearchOut::Rec *rb = per_block[i].first - obase[i];
          for (size_t o = r0; o < r1; o++) {
            const SearchOut::Rec &r = rb[o];
            std::memcpy(&res.ids[16 * o], r.id, 16);
            res.id_len[o] = uint8_t(r.block_il >> 24);
            res.start[o] = r.start;
            res.end[o] = r.end;
            res.dur[o] = uint32_t((r.end - r.start) / 1000000ULL);  // util.go:33
            res.block[o] = uint32_t(i);
            res.entry[o] = r.entry;
            put_name(tb, 0, r.svc, o);
            put_name(tb, 1, r.name, o);
          }
        }
        r0 = r1;
      }
    }
  });
  if (prof)
    prof_add("fill.records", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_par).count());
  if (bad.load()) fail(TSG_E_DEVICE, "device position outside its block's host columns");
  res.ptrs_ready = true;
}

// Result arrays of a large full scan whose names are few next to its records: every value of
// the root.service.name / root.name dictionaries of the blocks with records is interned first
// (one arena, final before any record is written), then the records are written on several
// threads, names and their pointers by value id from the per-block tables (no hash probe per
// name, no offset fix-up pass, no pointer pass in finalize). Records of a block with per_pos
// are gathered from its host columns; the others copied from per_block. (Non-temporal stores
// were tried: 12 output streams per thread overflow the write-combining buffers, 3x slower.)
static bool fill_records_direct(ResultHolder &res, tsg_block *const *blocks,
                                const std::vector<std::pair<const SearchOut::Rec *, size_t>> &per_block,
                                const std::vector<const uint64_t *> &per_pos, const std::vector<size_t> &obase,
                                size_t nout, size_t nt) {
  thread_local FillNames fn_tl;
  FillNames &fn = fn_tl;
  const size_t nblocks = obase.size() - 1;
  thread_local std::vector<uint8_t> use;
  use.assign(nblocks, 0);
  for (size_t i = 0; i < nblocks; i++) use[i] = obase[i + 1] > obase[i];
  if (!fill_names(res, blocks, nblocks, nout, use, fn)) return false;
  fill_direct_range(res, blocks, per_block, per_pos, obase, 0, nout, nt, fn);
  return true;
}

// Result arrays of a large full scan on several threads: output record o of block i is
// per_block[i].first[o - obase[i]], or position per_pos[i][o - obase[i]] gathered from block
// i's host columns. Names few next to the records: fill_records_direct. Otherwise each thread
// interns its names into an arena of its own (a name = a block dictionary value, interned by
// address); the arenas are then placed one after another and each thread's name offsets
// shifted by its arena's place.
static void fill_records_parallel(ResultHolder &res, tsg_block *const *blocks,
                                  const std::vector<std::pair<const SearchOut::Rec *, size_t>> &per_block,
                                  const std::vector<const uint64_t *> &per_pos,
                                  const std::vector<size_t> &obase, size_t nout) {
  const size_t hw = size_t(host_threads_now());
  const size_t nt = std::max<size_t>(1, std::min<size_t>({16, hw, nout / 32768}));
  static const bool rows_path = std::getenv("TSG_FILL_INTERN") == nullptr;  // (A/B: the per-thread arenas)
  if (rows_path && fill_records_direct(res, blocks, per_block, per_pos, obase, nout, nt)) return;
  struct Local {
    std::vector<ResultHolder::InternSlot> tab;
    size_t used = 0;
    std::string arena;
    uint64_t get(const char *p, size_t l) {
      if (2 * (used + 1) > tab.size()) {  // grow: rehash
        std::vector<ResultHolder::InternSlot> old;
        old.swap(tab);
        tab.assign(std::max<size_t>(256, 2 * old.size()), ResultHolder::InternSlot{nullptr, 0, 0});
        used = 0;
        for (const auto &x : old)
          if (x.p) put(x);
      }
      const size_t mask = tab.size() - 1;
      for (size_t h = (uintptr_t(p) * 0x9E3779B97F4A7C15ull ^ l) >> 7;; h++) {
        auto &x = tab[h & mask];
        if (!x.p) {
          x = ResultHolder::InternSlot{p, uint32_t(l), arena.size()};
          used++;
          arena.append(p, l);
          return x.off;
        }
        if (x.p == p && x.l == l) return x.off;
      }
    }
    void put(const ResultHolder::InternSlot &s) {
      const size_t mask = tab.size() - 1;
      size_t h = (uintptr_t(s.p) * 0x9E3779B97F4A7C15ull ^ s.l) >> 7;
      while (tab[h & mask].p) h++;
      tab[h & mask] = s;
      used++;
    }
  };
  std::vector<Local> loc(nt);
  std::atomic<bool> bad{false};
  // a name's arena offset by its dictionary value id, per thread and block, where the block's
  // names are few next to its records (an array index instead of a hash probe per name)
  auto dense_ok = [&](size_t i, int key) {
    if (key < 0) return false;
    const uint64_t recs = obase[i + 1] - obase[i];
    return uint64_t(blocks[i]->b.host->keys[size_t(key)].nvals()) * 4 <= recs / nt + 1024;
  };
  auto range = [&](size_t t, size_t &o0, size_t &o1) {
    o0 = nout * t / nt;
    o1 = nout * (t + 1) / nt;
  };
  parallel_ranges(nt, 1, int(nt), [&](size_t t0, size_t t1) {
    for (size_t t = t0; t < t1; t++) {
      size_t o0, o1;
      range(t, o0, o1);
      if (o0 >= o1) continue;
      Local &L = loc[t];
      size_t i = size_t(std::upper_bound(obase.begin(), obase.end(), o0) - obase.begin()) - 1;
      std::vector<uint64_t> dsvc, dname;  // value id -> arena offset + 1 (0: not yet), this block
      size_t dblock = ~size_t(0);
      bool dsv = false, dnm = false;
      auto name_off = [&](std::vector<uint64_t> &dense, bool use, uint32_t vid, std::string_view v) -> uint64_t {
        if (!use) return L.get(v.data(), v.size());
        uint64_t &x = dense[vid];
        if (!x) x = L.get(v.data(), v.size()) + 1;
        return x - 1;
      };
      for (size_t o = o0; o < o1; o++) {
        while (o >= obase[i + 1]) i++;
        const HostBlock &h = *blocks[i]->b.host;
        if (i != dblock) {
          dblock = i;
          dsv = dense_ok(i, h.svc_key);
          dnm = dense_ok(i, h.name_key);
          if (dsv) dsvc.assign(h.keys[size_t(h.svc_key)].nvals(), 0);
          if (dnm) dname.assign(h.keys[size_t(h.name_key)].nvals(), 0);
        }
        uint32_t svc, name;
        if (const uint64_t *pp = per_pos[i]) {
          const uint32_t e = uint32_t(pp[o - obase[i]]);
          if (e >= h.start.size() || uint64_t(e) * 16 + 16 > h.ids.size()) {
            bad.store(true, std::memory_order_relaxed);
            return;
          }
          std::memcpy(&res.ids[16 * o], h.ids.data() + uint64_t(e) * 16, 16);
          res.id_len[o] = h.id_len[e];
          const uint64_t st = h.start[e], en = h.end[e];
          res.start[o] = st;
          res.end[o] = en;
          res.dur[o] = uint32_t((en - st) / 1000000ULL);  // util.go:33
          res.entry[o] = e;
          svc = h.svc_vid.empty() ? kNone : h.svc_vid[e];
          name = h.name_vid.empty() ? kNone : h.name_vid[e];
        } else {
          const SearchOut::Rec *r = per_block[i].first + (o - obase[i]);
          std::memcpy(&res.ids[16 * o], r->id, 16);
          res.id_len[o] = uint8_t(r->block_il >> 24);
          res.start[o] = r->start;
          res.end[o] = r->end;
          res.dur[o] = uint32_t((r->end - r->start) / 1000000ULL);  // util.go:33
          res.entry[o] = r->entry;
          svc = r->svc;
          name = r->name;
        }
        res.block[o] = uint32_t(i);
        std::string_view sv, nm;
        if (h.svc_key >= 0 && svc != kNone) sv = h.dict_value(h.svc_key, svc);
        if (h.name_key >= 0 && name != kNone) nm = h.dict_value(h.name_key, name);
        res.svc_len[o] = uint32_t(sv.size());
        res.svc_off[o] = sv.empty() ? 0 : name_off(dsvc, dsv, svc, sv);
        res.name_len[o] = uint32_t(nm.size());
        res.name_off[o] = nm.empty() ? 0 : name_off(dname, dnm, name, nm);
      }
    }
  });
  if (bad.load()) fail(TSG_E_DEVICE, "device position outside its block's host columns");
  std::vector<uint64_t> base(nt + 1, 0);
  for (size_t t = 0; t < nt; t++) base[t + 1] = base[t] + loc[t].arena.size();
  if (base[nt] > res.arena_cap) res.arena_grow(base[nt]);
  res.arena_size = base[nt];
  parallel_ranges(nt, 1, int(nt), [&](size_t t0, size_t t1) {
    for (size_t t = t0; t < t1; t++) {
      if (!loc[t].arena.empty()) std::memcpy(res.arena + base[t], loc[t].arena.data(), loc[t].arena.size());
      size_t o0, o1;
      range(t, o0, o1);
      if (!base[t]) continue;
      for (size_t o = o0; o < o1; o++) {
        if (res.svc_len[o]) res.svc_off[o] += base[t];
        if (res.name_len[o]) res.name_off[o] += base[t];
      }
    }
  });
}

int tsg_search(tsg_ctx *ctx, tsg_block *const *blocks, size_t nblocks, const tsg_query *q,
               const tsg_search_opts *opts, tsg_result **out) {
  if (!ctx || !q || !out || (nblocks && !blocks)) return TSG_E_INVALID;
  // TSG_CHUNK_BLOCKS: blocks per device launch (default 32 = the one-launch path's
  // kernel-argument capacity; 0 = one launch for all, the descriptor path beyond 32)
  static const size_t kChunk = [] {
    const char *e = std::getenv("TSG_CHUNK_BLOCKS");
    return e ? size_t(std::atoll(e)) : size_t(32);
  }();
  static const bool trace = std::getenv("TSG_TRACE") != nullptr || prof_on();
  using clk = std::chrono::steady_clock;
  const clk::time_point t_in = trace ? clk::now() : clk::time_point();
  const uint64_t qid = opts ? opts->query_id : 0;
  ctx->begin(qid);
  Approach approach;
  for (size_t i = 0; i < nblocks; i++)
    if (blocks && blocks[i] && blocks[i]->b.dc) approach.add(&ctx->coalescer(blocks[i]->b.dc).approaching);
  struct Forget {  // the id is done with once this search returns, cancelled or not
    tsg_ctx *c;
    uint64_t q;
    ~Forget() { c->forget(q); }
  } forget_qid{ctx, qid};
  auto check_cancel = [&] {
    if (ctx->is_cancelled(qid)) fail(TSG_E_CANCELLED, "search cancelled (tsg_cancel)");
  };
  return guard([&] {
    check_cancel();
    const uint32_t limit = opts ? opts->limit : 0;
    const uint32_t flags = opts ? opts->flags : 0;
    auto *res = acquire_holder();
    std::unique_ptr<ResultHolder, HolderRelease> guard_res(res);
    tsg_metrics &m = res->pub.metrics;
    std::memset(&m, 0, sizeof m);
    res->set_blocks(nblocks);
    // block filter on the host (header), device work grouped per device
    // (per-query scratch kept per thread: no allocations once warm)
    thread_local std::vector<int> state;
    state.assign(nblocks, 0);  // 0 no meta, 1 skipped, 2 inspected
    // MatchesBlock terms left to the device dictionary pass (HostBlock::hdr_defer) per block,
    // and what the pass found (term_any: -1 = not reported); resolved when the consumer
    // reaches the block
    thread_local std::vector<uint32_t> defer;
    thread_local std::vector<int64_t> anym;
    defer.assign(nblocks, 0);
    anym.assign(nblocks, -1);
    bool any_live = false;
    for (size_t i = 0; i < nblocks; i++) {
      Block &b = blocks[i]->b;
      if (!b.host->has_meta) continue;
      if (b.host->live) {  // searchLiveTraces: no block filter
        state[i] = 2;
        any_live = true;
        continue;
      }
      bool ok = b.host->streaming
                    ? pipeline_matches_stream_header(*q, b.host->min_dur, b.host->max_dur, b.host->stream_tags)
                    : b.host->hdr_index ? pipeline_matches_block_indexed(*q, *b.host, &defer[i])
                                        : pipeline_matches_block(*q, b.host->header.data(), b.host->header.size());
      state[i] = ok ? 2 : 1;
    }
    auto note_any = [&](const SearchOut &o) {
      for (const auto &ta : o.term_any)
        if (ta.first < nblocks) anym[ta.first] = int64_t(ta.second);
    };
    // Blocks [b0, b1) on their devices, one device_search per device (concurrently).
    // device outputs: a deque keeps them in place (per_block points into their records);
    // entries are reused across queries, their record vectors keep their capacity
    thread_local std::deque<SearchOut> outs;
    size_t outs_used = 0;
    thread_local std::vector<std::pair<const SearchOut::Rec *, size_t>> per_block;
    per_block.assign(nblocks, {nullptr, 0});
    thread_local std::vector<const uint64_t *> per_pos;  // block i's scan positions (compact device output)
    per_pos.assign(nblocks, nullptr);
    size_t nrec = 0;
    // Blocks [b0, b1) (live_only: just the live ones) searched whole, each block capped at
    // dlimit records. Live blocks are never capped: a trace's result combines all its
    // matching segments (a limit search runs them on their own, below)
    auto search_range = [&](size_t b0, size_t b1, bool live_only, uint32_t dlimit) {
      // blocks per device, in first-seen device order (a handful of devices: linear search)
      std::vector<std::pair<DeviceCtx *, std::vector<std::pair<uint32_t, Block *>>>> per_dev;
      for (size_t i = b0; i < b1; i++) {
        if (state[i] != 2 || !blocks[i]->b.dc) continue;
        if (live_only && !blocks[i]->b.host->live) continue;
        DeviceCtx *dc = blocks[i]->b.dc;
        size_t d = 0;
        while (d < per_dev.size() && per_dev[d].first != dc) d++;
        if (d == per_dev.size()) per_dev.push_back({dc, {}});
        per_dev[d].second.push_back({uint32_t(i), &blocks[i]->b});
      }
      std::vector<SearchOut *> slots;
      for (size_t d = 0; d < per_dev.size(); d++) {
        if (outs_used == outs.size()) outs.emplace_back();
        slots.push_back(&outs[outs_used++]);
      }
      auto work = [&](size_t slot) {
        DeviceCtx *dc = per_dev[slot].first;
        const auto &list = per_dev[slot].second;
        // chunks of at most kChunk blocks, one launch each (the one-launch path
        // carries 32 blocks in its kernel arguments); cancellation is checked
        // before every chunk
        const size_t nl = list.size(), step = kChunk ? kChunk : nl;
        SearchOut &o = *slots[slot];
        // a whole-block full scan (no cap, no live block) takes scan positions: the records
        // are gathered from the host columns straight into the result arrays
        o.want_pos = !dlimit && !live_only && !any_live && nl <= step;
        if (nl <= step) {  // one chunk: the device's list as it is (coalesced with concurrent callers)
          check_cancel();
          coalesced_search(ctx, dc, list, *q, dlimit, flags, o, approach);
          return;
        }
        approach.leave();
        for (size_t c0 = 0; c0 < nl; c0 += step) {
          check_cancel();
          const std::vector<std::pair<uint32_t, Block *>> part(list.begin() + c0,
                                                               list.begin() + std::min(nl, c0 + step));
          if (c0 == 0) {
            device_search(*dc, part, *q, dlimit, flags, o);
            continue;
          }
          SearchOut more;
          device_search(*dc, part, *q, dlimit, flags, more);
          o.recs.insert(o.recs.end(), more.recs.begin(), more.recs.end());
          o.term_any.insert(o.term_any.end(), more.term_any.begin(), more.term_any.end());
          o.device_bytes += more.device_bytes;
          o.kernel_ns += more.kernel_ns;
          o.scan_ns += more.scan_ns;
          o.scan_bytes += more.scan_bytes;
          o.reruns += more.reruns;
          o.path |= more.path;
        }
      };
      if (per_dev.empty()) approach.leave();
      if (!per_dev.empty()) ctx->fan_out(per_dev.size(), [&](size_t i) { return per_dev[i].first; }, work);
      // per block match lists in scan order (each device's records are grouped by block already)
      uint64_t wave_k = 0, wave_s = 0;  // devices run concurrently: a wave takes its slowest
      for (size_t d = 0; d < slots.size(); d++) {
        SearchOut *o = slots[d];
        note_any(*o);
        m.device_bytes_read += o->device_bytes;
        m.reruns += o->reruns;
        m.path |= o->path;
        wave_k = std::max<uint64_t>(wave_k, o->kernel_ns);
        wave_s = std::max<uint64_t>(wave_s, o->scan_ns);
        m.scan_bytes += o->scan_bytes;
        const auto &list = per_dev[d].second;
        if (o->compact) {  // positions in list order, o->block_counts per list entry
          uint64_t sum = 0;
          for (uint64_t c : o->block_counts) sum += c;
          if (o->block_counts.size() != list.size() || sum != o->pos.size())
            fail(TSG_E_DEVICE, "device positions do not match their per-block counts");
          size_t r = 0;
          for (size_t x = 0; x < list.size(); x++) {
            if (o->block_counts[x]) {
              per_block[list[x].first] = {nullptr, size_t(o->block_counts[x])};
              per_pos[list[x].first] = o->pos.data() + r;
            }
            r += size_t(o->block_counts[x]);
          }
          nrec += o->pos.size();
          continue;
        }
        const auto &recs = o->recs;
        // the device's per-block counts (its list order = record order) when they describe
        // these records; otherwise one pass over the records' block indices
        if (o->block_counts.size() == list.size()) {
          uint64_t sum = 0;
          for (uint64_t c : o->block_counts) sum += c;
          if (sum == recs.size()) {
            size_t r = 0;
            for (size_t x = 0; x < list.size(); x++) {
              if (o->block_counts[x]) per_block[list[x].first] = {recs.data() + r, size_t(o->block_counts[x])};
              r += size_t(o->block_counts[x]);
            }
            nrec += recs.size();
            continue;
          }
        }
        for (size_t r = 0; r < recs.size();) {
          const uint32_t bi = recs[r].block_il & 0xffffffu;
          size_t e = r;
          while (e < recs.size() && (recs[e].block_il & 0xffffffu) == bi) e++;
          per_block[bi] = {&recs[r], e - r};
          r = e;
        }
        nrec += recs.size();
      }
      m.kernel_ns += wave_k;
      m.scan_kernel_ns += wave_s;
    };
    // searchLiveTraces' per-trace results: the block's matching rows (segments) come in row
    // order = trace order; consecutive rows of one trace fold into one result with
    // CombineSearchResults (tempodb/search/util.go:40-62)
    struct LiveRec {
      uint32_t trace;
      uint8_t id[16];
      uint8_t il;
      uint64_t start, end;
      uint32_t dur;
      uint64_t row;
      std::string_view sv, nm;
    };
    thread_local std::vector<LiveRec> live_recs;
    auto rec_names = [&](const HostBlock &h, const SearchOut::Rec *r, std::string_view &sv, std::string_view &nm) {
      sv = nm = std::string_view();
      if (h.svc_key >= 0 && r->svc != kNone) sv = h.dict_value(h.svc_key, r->svc);
      if (h.name_key >= 0 && r->name != kNone) nm = h.dict_value(h.name_key, r->name);
    };
    auto combine_live = [&](size_t i, const SearchOut::Rec *recs, size_t nr) {
      live_recs.clear();
      const HostBlock &h = *blocks[i]->b.host;
      static const uint8_t zero[16] = {};
      for (size_t ri = 0; ri < nr; ri++) {
        const SearchOut::Rec *r = recs + ri;
        const uint32_t t = h.row_trace[r->entry];
        std::string_view sv, nm;
        rec_names(h, r, sv, nm);
        const uint32_t dur = uint32_t((r->end - r->start) / 1000000ULL);  // util.go:33
        if (!live_recs.empty() && live_recs.back().trace == t) {
          LiveRec &x = live_recs.back();
          if (std::memcmp(x.id, zero, 16) == 0) {  // existing.TraceID == "" (all-zero ids trim to "")
            std::memcpy(x.id, r->id, 16);
            x.il = uint8_t(r->block_il >> 24);
          }
          if (x.sv.empty()) x.sv = sv;
          if (x.nm.empty()) x.nm = nm;
          if (x.start > r->start) x.start = r->start;
          if (x.dur < dur) x.dur = dur;
          continue;
        }
        LiveRec x;
        x.trace = t;
        std::memcpy(x.id, r->id, 16);
        x.il = uint8_t(r->block_il >> 24);
        x.start = r->start;
        x.end = r->end;
        x.dur = dur;
        x.row = r->entry;
        x.sv = sv;
        x.nm = nm;
        live_recs.push_back(x);
      }
    };
    // Early exit (limit > 0): the consumer stops at the L-th distinct id in
    // block order, so nothing behind that point is needed. The blocks' entries form one
    // sequence (blocks in caller order, scan order inside); progressive waves search its next
    // stretch — the first TSG_LIMIT_WAVE0 entries (2^20: a 512-entry unit for every other wave
    // of the chip; 2^21 took 1.3 us more of kernel and 3.7 us more of step on the limit-20 leg,
    // profiles/r04_final), then a stretch sized by the selectivity seen so far (x1.5 the entries the missing
    // ids need at that rate, at least 4x the last wave) — cutting blocks on unit boundaries,
    // until the consumer stops inside what has been searched. A block's records over its
    // parts are its records in scan order, so the result is the one-wave result. Live blocks
    // are never cut (a trace's segments combine), and once a search leaves the pool kernels
    // (which take the cut ranges on the device) the waves cut at block boundaries only.
    static const uint64_t kWave0 = [] {
      const char *e = std::getenv("TSG_LIMIT_WAVE0");
      return e ? std::max<uint64_t>(512, uint64_t(std::atoll(e))) : uint64_t(1) << 20;
    }();
    // A limit search whose blocks hold at most one first wave's entries is one launch with
    // per-block caps (concurrent callers coalesce: the shim's per-block calls); larger ones,
    // and any with a live block, take the waves.
    uint64_t inspect_entries = 0;
    for (size_t i = 0; i < nblocks; i++)
      if (state[i] == 2 && blocks[i]->b.dc && !blocks[i]->b.host->live) inspect_entries += blocks[i]->b.host->n;
    // IDs the caller's consumer took before these blocks (tsg_search_opts.seen_ids)
    const uint8_t(*seen)[16] = opts && opts->nseen ? opts->seen_ids : nullptr;
    const uint64_t nseen = seen ? opts->nseen : 0;
    auto seed = [&](IdSet &ids) {
      for (uint64_t i = 0; i < nseen; i++) ids.insert(seen[i]);
    };
    thread_local std::vector<size_t> obase;
    // caller blocks [i0, i1): MatchesBlock's deferred terms resolved, metrics, and the output
    // offsets of their records (obase[i + 1]); returns the records they hold
    auto account = [&](size_t i0, size_t i1) {
      for (size_t i = i0; i < i1; i++) {
        const HostBlock &h = *blocks[i]->b.host;
        size_t k = 0;
        if (state[i] != 0) {
          if (!h.part_tail) m.bytes_inspected += h.header.size();
          if (state[i] == 2 && defer[i])  // (as in the consumer below)
            state[i] = anym[i] >= 0 ? ((defer[i] & ~uint32_t(anym[i])) ? 1 : 2)
                                    : (pipeline_matches_block_indexed(*q, h) ? 2 : 1);
          if (state[i] == 1) {
            if (!h.part_tail) m.blocks_skipped++;
          } else {
            if (!h.part_tail) m.blocks_inspected++;
            k = per_block[i].second;
            m.traces_inspected += uint32_t(h.n);
            m.bytes_inspected += h.fb_bytes;
            if (h.stop_status) {
              res->bstatus[i] = h.stop_status;
              res->berr_s[i] = h.stop_msg;
            }
          }
        }
        obase[i + 1] = obase[i] + k;
      }
      return obase[i1] - obase[i0];
    };
    // ---- pipelined full scan. A full scan whose device work is long (the dictionary pass over
    // large dictionaries: config 4's statement queries, ~2.5 ms) and whose results are dense
    // runs as consecutive launches of TSG_PIPE_BLOCKS blocks on a producer thread while this
    // thread assembles the result arrays of the launches already done: the host's gather of
    // 1.85 M records (2.4-3.5 ms on 16 CPUs) overlaps the device instead of following it.
    // Same records in the same order and the same metrics as one launch (caller block order,
    // each block's records in scan order).
    bool pipelined = false;
    std::vector<std::vector<std::pair<uint32_t, Block *>>> pchunks;
    DeviceCtx *pdev = nullptr;
    auto pipelined_plan = [&]() -> bool {
      if (nseen) return false;
      // the blocks, one device (the plain fan-out otherwise), before anything costlier
      thread_local std::vector<std::pair<uint32_t, Block *>> list;
      list.clear();
      for (size_t i = 0; i < nblocks; i++) {
        if (state[i] != 2 || !blocks[i]->b.dc) continue;
        Block &b = blocks[i]->b;
        if (pdev && b.dc != pdev) return false;
        pdev = b.dc;
        list.push_back({uint32_t(i), &b});
      }
      if (list.size() < 2 || list.size() > kChunk) return false;
      // (a sparse result has nothing for the host to fill while the device works: one launch
      // — six launches of an absent needle had cost 93 us of scan kernels; TSG_PIPE_SPARSE=1
      // pipelines whatever the last full scan's density. Checked before the dictionary sizes:
      // their per-block key lookups had cost every sparse full scan ~1 us of host time)
      const char *e3 = std::getenv("TSG_PIPE_SPARSE");
      if (!(e3 && std::atoi(e3)) && !device_last_dense(*pdev)) return false;
      // (read per query: a test turns it on for small blocks)
      const char *e1 = std::getenv("TSG_PIPE_DICT_MB"), *e2 = std::getenv("TSG_PIPE_BLOCKS");
      const uint64_t kPipeDict = uint64_t(e1 ? std::atoll(e1) : 2048) << 20;  // wide-term dictionary bytes, all blocks
      const size_t kPipeBlocks = size_t(std::max(1, e2 ? std::atoi(e2) : 2));
      if (!kPipeDict) return false;
      uint64_t dict = 0;
      for (const auto &bp : list)
        for (uint32_t t = 0; t < q->nterms; t++) {
          const auto it = bp.second->host->key_index.find(
              std::string(reinterpret_cast<const char *>(q->keys[t]), q->key_lens[t]));
          if (it == bp.second->host->key_index.end() || size_t(it->second) >= bp.second->dev.keys.size()) continue;
          const DevKey &k = bp.second->dev.keys[size_t(it->second)];
          if (k.width != 1) dict += k.dict_nbytes;
        }
      if (dict < kPipeDict) return false;
      // one block in the last launch (its result fill is the part nothing overlaps) and in the
      // first (the host starts filling sooner); kPipeBlocks per launch between them
      const size_t nl = list.size();
      const size_t edge = kPipeBlocks > 1 && nl >= kPipeBlocks + 2 ? 1 : kPipeBlocks;
      size_t c0 = 0;
      while (c0 < nl) {
        const size_t left = nl - c0;
        const size_t take = c0 == 0 ? edge : left <= edge ? left : std::min(kPipeBlocks, left - edge);
        pchunks.emplace_back(list.begin() + c0, list.begin() + c0 + take);
        c0 += take;
      }
      approach.leave();
      return true;
    };
    auto pipelined_run = [&]() -> size_t {
      const size_t nc = pchunks.size();
      while (outs.size() < outs_used + nc) outs.emplace_back();
      std::vector<SearchOut *> po(nc);
      for (size_t c = 0; c < nc; c++) {
        po[c] = &outs[outs_used++];
        po[c]->want_pos = true;
      }
      std::atomic<uint32_t> done{0};
      std::atomic<bool> failed{false}, pstop{false};
      tsg::EpochPark pk;
      std::exception_ptr perr;
      // the producer: one device_search per chunk, back to back
      std::thread producer([&] {
        try {
          for (size_t c = 0; c < nc && !pstop.load(std::memory_order_acquire); c++) {
            if (ctx->is_cancelled(qid)) fail(TSG_E_CANCELLED, "search cancelled (tsg_cancel)");
            device_search(*pdev, pchunks[c], *q, 0, flags, *po[c]);
            done.store(uint32_t(c + 1), std::memory_order_release);
            pk.notify();
          }
        } catch (...) {
          perr = std::current_exception();
          failed.store(true, std::memory_order_release);
          pk.notify();
        }
      });
      struct Join {  // (an early exit here stops the producer after its current launch)
        std::thread &t;
        std::atomic<bool> &stop;
        ~Join() {
          stop.store(true, std::memory_order_release);
          if (t.joinable()) t.join();
        }
      } join{producer, pstop};
      // every name of the inspected blocks interned first (the arena is final before any
      // record is written); the arrays reserved for every entry (virtual: touched as filled)
      thread_local FillNames fn_tl;
      FillNames &fn = fn_tl;
      thread_local std::vector<uint8_t> use;
      use.assign(nblocks, 0);
      uint64_t ent = 0;
      for (const auto &ch : pchunks)
        for (const auto &bp : ch) {
          use[bp.first] = 1;
          ent += bp.second->host->n;
        }
      const bool direct = fill_names(*res, blocks, nblocks, size_t(ent / 8), use, fn);
      res->reserve(size_t(ent));
      res->svc_p.reserve(size_t(ent));
      res->name_p.reserve(size_t(ent));
      obase.assign(nblocks + 1, 0);
      size_t next_i = 0, filled = 0;
      const size_t hw = size_t(host_threads_now());
      for (size_t c = 0; c < nc; c++) {
        // wait for chunk c (the producer runs on another CPU: a short spin, then park)
        auto ready = [&] { return done.load(std::memory_order_acquire) > c || failed.load(std::memory_order_acquire); };
        while (!ready()) {
          const uint32_t e = pk.read();
          if (!tsg::spin_for(20'000, ready)) pk.wait(e, 100'000'000);
        }
        if (done.load(std::memory_order_acquire) <= c) {  // the producer failed
          producer.join();
          std::rethrow_exception(perr);
        }
        SearchOut &o = *po[c];
        note_any(o);
        m.device_bytes_read += o.device_bytes;
        m.reruns += o.reruns;
        m.path |= o.path;
        m.kernel_ns += o.kernel_ns;
        m.scan_kernel_ns += o.scan_ns;
        m.scan_bytes += o.scan_bytes;
        const auto &list = pchunks[c];
        // this launch's records per block (its list order = record order)
        uint64_t sum = 0;
        for (uint64_t x : o.block_counts) sum += x;
        const size_t nr = o.compact ? o.pos.size() : o.recs.size();
        if (o.block_counts.size() == list.size() && sum == nr) {
          size_t r = 0;
          for (size_t x = 0; x < list.size(); x++) {
            const size_t cnt = size_t(o.block_counts[x]);
            per_block[list[x].first] = {o.compact ? nullptr : o.recs.data() + r, cnt};
            per_pos[list[x].first] = o.compact && cnt ? o.pos.data() + r : nullptr;
            r += cnt;
          }
        } else if (!o.compact) {  // (records grouped by block already: one pass over their block indices)
          for (size_t r = 0; r < nr;) {
            const uint32_t bi = o.recs[r].block_il & 0xffffffu;
            size_t e = r;
            while (e < nr && (o.recs[e].block_il & 0xffffffu) == bi) e++;
            if (bi < nblocks) per_block[bi] = {&o.recs[r], e - r};
            r = e;
          }
        } else {
          fail(TSG_E_DEVICE, "device positions do not match their per-block counts");
        }
        nrec += nr;
        // the caller blocks up to this launch's last one (the ones between were not searched)
        const size_t i1 = c + 1 < nc ? size_t(list.back().first) + 1 : nblocks;
        account(next_i, i1);
        next_i = i1;
        const size_t o_end = obase[i1];
        for (size_t j = i1 + 1; j <= nblocks; j++) obase[j] = o_end;  // (monotone: the fill's binary search)
        if (o_end > filled) {
          res->resize(o_end);
          // (one CPU of the job's share stays with the producer, which polls the device)
          const size_t nt = std::max<size_t>(1, std::min<size_t>({15, hw > 1 ? hw - 1 : 1, (o_end - filled) / 16384}));
          if (direct) {
            fill_direct_range(*res, blocks, per_block, per_pos, obase, filled, o_end, nt, fn);
          } else {  // (many names: record by record, interned through the result's table)
            for (size_t i = 0; i < i1; i++) {
              if (obase[i + 1] <= std::max(obase[i], filled)) continue;
              const HostBlock &h = *blocks[i]->b.host;
              res->vid_block(h.svc_key >= 0 ? h.keys[size_t(h.svc_key)].nvals() : 0,
                             h.name_key >= 0 ? h.keys[size_t(h.name_key)].nvals() : 0);
              for (size_t oo = std::max(obase[i], filled); oo < obase[i + 1]; oo++) {
                const size_t ri = oo - obase[i];
                const SearchOut::Rec rr = per_pos[i] ? rec_from_pos(h, per_pos[i][ri]) : per_block[i].first[ri];
                res->set_rec(oo, rr.id, uint8_t(rr.block_il >> 24), rr.start, rr.end, uint32_t(i), rr.entry);
                res->set_vid(0, oo, h, h.svc_key, rr.svc);
                res->set_vid(1, oo, h, h.name_key, rr.name);
              }
            }
            res->ptrs_ready = false;
          }
          filled = o_end;
        }
        check_cancel();
      }
      if (!direct) res->ptrs_ready = false;
      if (prof_on()) prof_add("pipe.chunks", double(nc));
      return filled;
    };

    if (limit && (any_live || inspect_entries > kWave0 || nseen)) {
      thread_local std::vector<std::vector<SearchOut::Rec>> acc;  // per block: its records so far
      if (acc.size() < nblocks) acc.resize(nblocks);
      for (size_t i = 0; i < nblocks; i++) acc[i].clear();
      // live blocks first, whole and uncapped (a trace's result combines all its segments;
      // one live block no longer lifts the other blocks' caps or the waves)
      if (any_live) {
        search_range(0, nblocks, true, 0);
        for (size_t i = 0; i < nblocks; i++)
          if (blocks[i]->b.host->live) acc[i].assign(per_block[i].first, per_block[i].first + per_block[i].second);
        nrec = 0;
      }
      approach.leave();
      thread_local IdSet distinct_w;
      distinct_w.clear();
      seed(distinct_w);
      bool stop = distinct_w.size() >= limit, cut_ok = true;
      size_t cb = 0;     // cursor: next block ...
      uint64_t ce = 0;   // ... and its next scan position
      uint64_t wave = kWave0, scanned = 0, matched = 0;
      thread_local std::deque<SearchOut> wouts;
      while (!stop) {
        while (cb < nblocks && (state[cb] != 2 || !blocks[cb]->b.dc ||
                                (!blocks[cb]->b.host->live && ce >= blocks[cb]->b.host->n))) {
          cb++;
          ce = 0;
        }
        if (cb >= nblocks) break;
        check_cancel();
        // this wave's parts, grouped per device (first-seen device order)
        std::vector<DeviceCtx *> devs;
        std::vector<std::vector<std::pair<uint32_t, Block *>>> lists;
        std::vector<EntryRanges> rngs;
        std::vector<std::pair<size_t, uint64_t>> order;  // (block, end) of the parts in sequence order
        uint64_t want = wave;
        while (want > 0 && cb < nblocks) {
          if (state[cb] != 2 || !blocks[cb]->b.dc) {
            cb++;
            ce = 0;
            continue;
          }
          if (blocks[cb]->b.host->live) {  // (searched above: its place in the sequence)
            order.push_back({cb, UINT64_MAX});
            cb++;
            ce = 0;
            continue;
          }
          const uint64_t n = blocks[cb]->b.host->n;
          uint64_t e1 = n;
          if (cut_ok && n - ce > want) e1 = std::min(n, (ce + want + 511) / 512 * 512);
          DeviceCtx *dc = blocks[cb]->b.dc;
          size_t d = 0;
          while (d < devs.size() && devs[d] != dc) d++;
          if (d == devs.size()) {
            devs.push_back(dc);
            lists.emplace_back();
            rngs.emplace_back();
          }
          lists[d].push_back({uint32_t(cb), &blocks[cb]->b});
          rngs[d].push_back({ce, e1});
          order.push_back({cb, e1});
          want -= std::min(want, e1 - ce);
          scanned += e1 - ce;
          if (e1 >= n) {
            cb++;
            ce = 0;
          } else {
            ce = e1;
          }
        }
        while (wouts.size() < devs.size()) wouts.emplace_back();
        // (the parts run on the devices' worker threads: a thread_local named inside the lambda
        // would be the worker's own; this reference is the caller's)
        std::deque<SearchOut> &wo = wouts;
        std::vector<uint8_t> used_pool(devs.size(), 0);
        if (!devs.empty())
        ctx->fan_out(devs.size(), [&](size_t i) { return devs[i]; },
                     [&](size_t i) {
                       SearchOut &o = wo[i];
                       o.recs.clear();
                       o.term_any.clear();
                       o.path = 0;
                       // (a part list longer than one launch's 32 blocks: whole blocks by chunks)
                       const size_t nl = lists[i].size(), step = kChunk ? kChunk : nl;
                       for (size_t c0 = 0; c0 < nl; c0 += step) {
                         const size_t c1 = std::min(nl, c0 + step);
                         const std::vector<std::pair<uint32_t, Block *>> part(lists[i].begin() + c0,
                                                                              lists[i].begin() + c1);
                         const EntryRanges pr(rngs[i].begin() + c0, rngs[i].begin() + c1);
                         SearchOut more;
                         // (each part keeps its first `limit` records: ids are unique within a
                         // block, so the consumer takes at most that many from a block)
                         device_search(*devs[i], part, *q, limit, flags, more, &pr);
                         o.recs.insert(o.recs.end(), more.recs.begin(), more.recs.end());
                         o.term_any.insert(o.term_any.end(), more.term_any.begin(), more.term_any.end());
                         o.device_bytes += more.device_bytes;
                         o.kernel_ns += more.kernel_ns;
                         o.scan_ns += more.scan_ns;
                         o.scan_bytes += more.scan_bytes;
                         o.reruns += more.reruns;
                         o.path |= more.path;
                         used_pool[i] = used_pool[i] || more.pool;
                       }
                     });
        uint64_t wk = 0, ws = 0;
        for (size_t i = 0; i < devs.size(); i++) {
          SearchOut &o = wouts[i];
          note_any(o);
          m.device_bytes_read += o.device_bytes;
          m.scan_bytes += o.scan_bytes;
          m.reruns += o.reruns;
          m.path |= o.path;
          wk = std::max<uint64_t>(wk, o.kernel_ns);
          ws = std::max<uint64_t>(ws, o.scan_ns);
          for (const auto &r : o.recs) acc[r.block_il & 0xffffffu].push_back(r);
          o.device_bytes = o.kernel_ns = o.scan_ns = o.scan_bytes = 0;
          o.reruns = 0;
          if (!used_pool[i]) cut_ok = false;  // (the other paths scan a block from 0: cut at block ends)
        }
        m.kernel_ns += wk;
        m.scan_kernel_ns += ws;
        // the consumer over the stretch just searched (its parts in sequence order)
        for (size_t k = 0; k < order.size() && !stop; k++) {
          const size_t bi = order[k].first;
          const auto &v = acc[bi];
          if (blocks[bi]->b.host->live) {  // its per-trace results, as the final consumer counts them
            combine_live(bi, v.data(), v.size());
            for (size_t x = 0; x < live_recs.size() && !stop; x++)
              if (distinct_w.insert(live_recs[x].id) && distinct_w.size() >= limit) stop = true;
            continue;
          }
          for (size_t ri = 0; ri < v.size() && !stop; ri++) {
            if (v[ri].entry >= order[k].second) break;
            if (distinct_w.insert(v[ri].id) && distinct_w.size() >= limit)
              stop = true;
          }
        }
        if (stop) break;
        // (records of a block over its parts: the check above re-walks a block's earlier
        // parts; distinct ids are a set, so only new ones count)
        matched = distinct_w.size();
        const uint64_t need = limit - matched;
        uint64_t next = 4 * wave;
        if (matched > 0) {
          const double est = double(need) * double(scanned) / double(matched) * 1.5;
          next = std::max<uint64_t>(next, uint64_t(std::min(est, 1e18)));
        }
        wave = next;
      }
      for (size_t i = 0; i < nblocks; i++) {
        per_block[i] = {acc[i].data(), acc[i].size()};
        per_pos[i] = nullptr;
        nrec += acc[i].size();
      }
    } else if (!limit && !any_live && pipelined_plan()) {
      pipelined = true;
    } else {
      search_range(0, nblocks, false, limit);  // (limit > 0 here: no live block)
      check_cancel();
    }
    const clk::time_point t_dev = trace ? clk::now() : clk::time_point();
    if (!pipelined) {
      res->reserve(nrec);
      res->small_names = nrec <= 4096;
      res->resize(nrec);
    }
    const clk::time_point t_res = trace ? clk::now() : clk::time_point();
    size_t nout = 0;
    // A large full scan (no limit, no live block: every record of every inspected block is
    // kept, nothing to consume) is assembled on several threads; otherwise one thread
    // consumes in caller block order (deterministic refinement of instance.Search)
    const bool par = !pipelined && !limit && !any_live && nrec >= (size_t(1) << 16);
    if (pipelined) {
      nout = pipelined_run();
    } else if (par) {
      obase.assign(nblocks + 1, 0);
      account(0, nblocks);
      nout = obase[nblocks];
      fill_records_parallel(*res, blocks, per_block, per_pos, obase, nout);
    }
    // consume in caller block order (deterministic refinement of instance.Search)
    thread_local IdSet distinct;
    distinct.clear();
    seed(distinct);
    bool stopped = limit && distinct.size() >= limit;
    for (size_t i = 0; i < nblocks && !stopped && !par && !pipelined; i++) {
      const HostBlock &h = *blocks[i]->b.host;
      if (state[i] == 0) continue;  // meta missing: no-op (backend_search_block.go:191-203)
      if (h.live) {  // searchLiveTraces (instance_search.go:99-128)
        combine_live(i, per_block[i].first, per_block[i].second);
        uint64_t stop_trace = UINT64_MAX;
        for (const LiveRec &x : live_recs) {
          res->set(nout, x.id, x.il, x.start, x.end, uint32_t(i), x.trace, x.sv.data(), x.sv.size(), x.nm.data(),
                   x.nm.size());
          res->dur[nout++] = x.dur;
          if (limit) {
            distinct.insert(x.id);
            if (distinct.size() >= limit) {
              stopped = true;
              stop_trace = x.trace;
              break;
            }
          }
        }
        // AddTraceInspected(1) and the segments' bytes for every trace visited: all of
        // them, or those up to the one whose result closed the consumer
        const uint64_t nt = stopped ? stop_trace + 1 : h.ntraces();
        m.traces_inspected += uint32_t(nt);
        m.bytes_inspected += h.trace_bytes0[nt];
        continue;
      }
      if (!h.part_tail) m.bytes_inspected += h.header.size();  // (a page range after page 0: not again)
      if (state[i] == 2 && defer[i]) {
        // MatchesBlock's deferred terms: a key whose values all miss the needle skips the
        // block (its scan found nothing: the term's bitmap is empty). Not reported (the block
        // never reached a dictionary pass): the host scans the header's values itself.
        if (anym[i] >= 0) state[i] = (defer[i] & ~uint32_t(anym[i])) ? 1 : 2;
        else state[i] = pipeline_matches_block_indexed(*q, h) ? 2 : 1;
      }
      if (state[i] == 1) {
        if (!h.part_tail) m.blocks_skipped++;
        continue;
      }
      if (!h.part_tail) m.blocks_inspected++;
      uint64_t stop_entry = UINT64_MAX;
      if (per_block[i].second)
        res->vid_block(h.svc_key >= 0 ? h.keys[size_t(h.svc_key)].nvals() : 0,
                       h.name_key >= 0 ? h.keys[size_t(h.name_key)].nvals() : 0);
      for (size_t ri = 0; ri < per_block[i].second; ri++) {
        SearchOut::Rec rp;
        const SearchOut::Rec *r = &rp;
        if (per_pos[i]) rp = rec_from_pos(h, per_pos[i][ri]);
        else r = per_block[i].first + ri;
        res->set_rec(nout, r->id, uint8_t(r->block_il >> 24), r->start, r->end, uint32_t(i), r->entry);
        res->set_vid(0, nout, h, h.svc_key, r->svc);
        res->set_vid(1, nout++, h, h.name_key, r->name);
        if (limit) {
          distinct.insert(r->id);
          if (distinct.size() >= limit) {
            stopped = true;
            stop_entry = r->entry;
            break;
          }
        }
      }
      if (!stopped) {
        m.traces_inspected += uint32_t(h.n);
        m.bytes_inspected += h.fb_bytes;
        if (h.stop_status) {  // the damaged page is reached: Search returns its error
          res->bstatus[i] = h.stop_status;
          res->berr_s[i] = h.stop_msg;
        }
      } else {
        // pages up to and including the stop page; entries up to and including the match
        m.traces_inspected += uint32_t(stop_entry + 1);
        for (size_t p = 0; p < h.page_first.size() && h.page_first[p] <= stop_entry; p++)
          m.bytes_inspected += h.page_fb_bytes[p];
      }
    }
    const clk::time_point t_fin = trace ? clk::now() : clk::time_point();
    res->resize(nout);
    res->finalize();
    *out = &guard_res.release()->pub;
    if (prof_on()) {
      const clk::time_point t_end = clk::now();
      prof_add("tsg_search.results.finalize", std::chrono::duration<double, std::micro>(t_end - t_fin).count());
      prof_add("tsg_search.results.alloc", std::chrono::duration<double, std::micro>(t_res - t_dev).count());
      prof_add("tsg_search.results.records", std::chrono::duration<double, std::micro>(t_fin - t_res).count());
      prof_add("tsg_search.device", std::chrono::duration<double, std::micro>(t_dev - t_in).count());
      prof_add("tsg_search.results", std::chrono::duration<double, std::micro>(t_end - t_dev).count());
    } else if (trace) {
      const clk::time_point t_end = clk::now();
      std::fprintf(stderr, "[tsg] tsg_search us: device=%.1f results=%.1f total=%.1f\n",
                   std::chrono::duration<double, std::micro>(t_dev - t_in).count(),
                   std::chrono::duration<double, std::micro>(t_end - t_dev).count(),
                   std::chrono::duration<double, std::micro>(t_end - t_in).count());
    }
  });
}
void tsg_result_free(tsg_result *r) {
  if (prof_on()) {
    const auto t0 = std::chrono::steady_clock::now();
    release_holder(reinterpret_cast<ResultHolder *>(r));
    prof_add("result_free", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    return;
  }
  release_holder(reinterpret_cast<ResultHolder *>(r));
}

int tsg_search_batch(tsg_ctx *ctx, const tsg_search_item *items, size_t n, uint32_t depth, tsg_result **outs,
                     uint64_t *device_ns) {
  if (!ctx || (n && (!items || !outs))) return TSG_E_INVALID;
  if (device_ns) *device_ns = 0;
  for (size_t i = 0; i < n; i++) outs[i] = nullptr;
  if (!n) return TSG_OK;
  // the devices the items' blocks live on: each starts a fresh resident launch with dispatch
  // timestamps (the batch's device time), ended after the last item
  std::vector<DeviceCtx *> devs;
  for (size_t i = 0; i < n; i++)
    for (size_t b = 0; b < items[i].nblocks; b++) {
      const tsg_block *blk = items[i].blocks ? items[i].blocks[b] : nullptr;
      if (blk && blk->b.dc && std::find(devs.begin(), devs.end(), blk->b.dc) == devs.end()) devs.push_back(blk->b.dc);
    }
  std::vector<uint64_t> before(devs.size());
  const int rc0 = guard([&] {
    for (size_t d = 0; d < devs.size(); d++) before[d] = resident_batch_begin(*devs[d]);
  });
  if (rc0) return rc0;
  const size_t nt = std::min<size_t>(n, depth ? depth : 16);
  std::atomic<size_t> next{0};
  std::vector<int> rcs(n, TSG_OK);
  std::vector<std::string> errs(n);
  auto run = [&] {
    tl_batch_item = true;
    for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) {
      const tsg_search_item &it = items[i];
      rcs[i] = tsg_search(ctx, it.blocks, it.nblocks, it.query, &it.opts, &outs[i]);
      if (rcs[i]) {
        errs[i] = tsg_last_error();
        outs[i] = nullptr;
      }
    }
    tl_batch_item = false;
  };
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; t++) th.emplace_back(run);
  run();
  for (auto &t : th) t.join();
  uint64_t dns = 0;
  const int rc1 = guard([&] {
    for (size_t d = 0; d < devs.size(); d++) dns = std::max(dns, resident_batch_end(*devs[d], before[d]));
  });
  if (device_ns) *device_ns = dns;
  for (size_t i = 0; i < n; i++)
    if (rcs[i]) {
      set_last_error(errs[i]);
      return rcs[i];
    }
  return rc1;
}
int tsg_debug_set(const char *name, int64_t value) { return debug_set(name, value); }

int tsg_kernel_times(tsg_ctx *ctx, uint64_t *ns, size_t cap, size_t *n) {
  if (!ctx || !n || (cap && !ns)) return TSG_E_INVALID;
  return guard([&] {
    std::vector<uint64_t> v;
    for (DeviceCtx *dc : ctx->c.devs) device_kernel_times(*dc, v);
    const size_t k = std::min(cap, v.size());
    if (k) std::memcpy(ns, v.data(), k * sizeof(uint64_t));
    *n = k;
  });
}

int tsg_results_combine(const tsg_result *in, uint32_t max_results, tsg_result **out) {
  if (!in || !out) return TSG_E_INVALID;
  return guard([&] {
    if (max_results == 0) max_results = 20;  // instance_search.go:24-28
    auto *res = new ResultHolder();
    std::unique_ptr<ResultHolder> gr(res);
    struct F {
      uint64_t first;
      size_t idx;  // index into res arrays
    };
    std::unordered_map<std::string, size_t> map;
    std::vector<F> order;
    for (uint64_t i = 0; i < in->n; i++) {
      std::string key(reinterpret_cast<const char *>(in->trace_id[i]), 16);
      auto it = map.find(key);
      if (it != map.end()) {  // CombineSearchResults (util.go:40-62)
        size_t e = it->second;
        if (res->svc_len[e] == 0) res->set_str(res->svc_off, res->svc_len, e, in->root_service[i], in->root_service_len[i]);
        if (res->name_len[e] == 0) res->set_str(res->name_off, res->name_len, e, in->root_name[i], in->root_name_len[i]);
        if (res->start[e] > in->start_ns[i]) res->start[e] = in->start_ns[i];
        if (res->dur[e] < in->duration_ms[i]) res->dur[e] = in->duration_ms[i];
      } else {
        map.emplace(key, res->start.size());
        order.push_back({i, res->start.size()});
        res->push(in->trace_id[i], in->trace_id_len[i], in->start_ns[i], in->end_ns[i], in->block_idx[i],
                  in->entry_idx[i], in->root_service[i], in->root_service_len[i], in->root_name[i],
                  in->root_name_len[i]);
        res->dur.back() = in->duration_ms[i];
      }
      if (map.size() >= max_results) break;
    }
    // sort by StartTimeUnixNano descending; ties by first occurrence
    std::stable_sort(order.begin(), order.end(),
                     [&](const F &a, const F &b) { return res->start[a.idx] > res->start[b.idx]; });
    auto *fin = new ResultHolder();
    std::unique_ptr<ResultHolder> gf(fin);
    for (auto &f : order) {
      size_t e = f.idx;
      fin->push(&res->ids[e * 16], res->id_len[e], res->start[e], res->end[e], res->block[e], res->entry[e],
                res->svc(e), res->svc_len[e], res->name(e), res->name_len[e]);
      fin->dur.back() = res->dur[e];
    }
    fin->pub.metrics = in->metrics;
    fin->set_blocks(size_t(in->nblocks));
    for (uint64_t i = 0; i < in->nblocks; i++) {
      fin->bstatus[i] = in->block_status[i];
      if (in->block_error[i]) fin->berr_s[i] = in->block_error[i];
    }
    fin->finalize();
    *out = &gf.release()->pub;
  });
}

// ---- v2 lookup -----------------------------------------------------------------------
int tsg_v2block_open(tsg_ctx *ctx, const char *dir, int device_hint, tsg_v2block **out) {
  if (!ctx || !dir || !out) return TSG_E_INVALID;
  return guard([&] {
    auto *b = new tsg_v2block();
    try {
      v2block_open(ctx->c, b->b, dir, device_hint);
    } catch (...) {
      v2block_free(b->b);
      delete b;
      throw;
    }
    *out = b;
  });
}
void tsg_v2block_close(tsg_v2block *b) {
  if (!b) return;
  v2block_free(b->b);
  delete b;
}
// Blocks on several devices: each device probes every id against its own blocks (the
// block fan-out of tempodb.Find, tempodb/tempodb.go:335-350), concurrently, and the
// per-device hit lists (each sorted by (id, block)) are merged into one (id, block) order.
extern "C++" {
template <class Out, class Run>
static void per_device_merge(tsg_ctx *ctx, tsg_v2block *const *blocks, size_t nblocks, Out &out, Run &&run,
                             void (*append)(Out &, const Out &, size_t)) {
  std::vector<DeviceCtx *> order;
  std::unordered_map<DeviceCtx *, std::vector<std::pair<uint32_t, V2Block *>>> per_dev;
  for (size_t i = 0; i < nblocks; i++) {
    DeviceCtx *dc = blocks[i]->b.dc;
    if (!per_dev.count(dc)) order.push_back(dc);
    per_dev[dc].push_back({uint32_t(i), &blocks[i]->b});
  }
  if (order.size() <= 1) {
    if (!order.empty()) run(*order[0], per_dev[order[0]], out);
    return;
  }
  std::vector<Out> parts(order.size());
  ctx->fan_out(order.size(), [&](size_t d) { return order[d]; },
               [&](size_t d) { run(*order[d], per_dev[order[d]], parts[d]); });
  // k-way merge by (id_idx, block_idx)
  std::vector<size_t> pos(parts.size(), 0);
  out = Out();
  out.kernel_ns = 0;
  for (auto &p : parts) out.kernel_ns = std::max(out.kernel_ns, p.kernel_ns);
  for (;;) {
    size_t best = parts.size();
    for (size_t d = 0; d < parts.size(); d++) {
      if (pos[d] >= parts[d].id_idx.size()) continue;
      if (best == parts.size() ||
          std::make_pair(parts[d].id_idx[pos[d]], parts[d].block_idx[pos[d]]) <
              std::make_pair(parts[best].id_idx[pos[best]], parts[best].block_idx[pos[best]]))
        best = d;
    }
    if (best == parts.size()) break;
    append(out, parts[best], pos[best]++);
  }
}
static void lk_append(LookupOut &o, const LookupOut &p, size_t i) {
  o.id_idx.push_back(p.id_idx[i]);
  o.block_idx.push_back(p.block_idx[i]);
  o.rec.push_back(p.rec[i]);
  o.start.push_back(p.start[i]);
  o.len.push_back(p.len[i]);
}
static void find_append(FindOut &o, const FindOut &p, size_t i) {
  o.id_idx.push_back(p.id_idx[i]);
  o.block_idx.push_back(p.block_idx[i]);
  o.status.push_back(p.status[i]);
  o.obj_off.push_back(o.bytes.size());
  o.obj_len.push_back(p.obj_len[i]);
  if (p.status[i] == TSG_OK)
    o.bytes.insert(o.bytes.end(), p.bytes.begin() + long(p.obj_off[i]), p.bytes.begin() + long(p.obj_off[i] + p.obj_len[i]));
}
}  // extern "C++"

int tsg_lookup_ids(tsg_ctx *ctx, tsg_v2block *const *blocks, size_t nblocks, const uint8_t (*ids)[16], size_t nids,
                   const tsg_lookup_opts *opts, tsg_lookup_result **out) {
  if (!ctx || !out || (nblocks && !blocks) || (nids && !ids)) return TSG_E_INVALID;
  return guard([&] {
    auto *h = new LookupHolder();
    std::unique_ptr<LookupHolder> g(h);
    per_device_merge(ctx, blocks, nblocks, h->o,
                     [&](DeviceCtx &dc, const std::vector<std::pair<uint32_t, V2Block *>> &list, LookupOut &o) {
                       device_lookup(dc, list, ids, nids, opts, o);
                     },
                     lk_append);
    h->pub.n = h->o.id_idx.size();
    h->pub.id_idx = h->o.id_idx.data();
    h->pub.block_idx = h->o.block_idx.data();
    h->pub.record_idx = h->o.rec.data();
    h->pub.record_start = h->o.start.data();
    h->pub.record_length = h->o.len.data();
    h->pub.kernel_ns = h->o.kernel_ns;
    *out = &g.release()->pub;
  });
}
void tsg_lookup_result_free(tsg_lookup_result *r) { delete reinterpret_cast<LookupHolder *>(r); }

int tsg_find_ids(tsg_ctx *ctx, tsg_v2block *const *blocks, size_t nblocks, const uint8_t (*ids)[16], size_t nids,
                 const tsg_lookup_opts *opts, tsg_find_result **out) {
  if (!ctx || !out || (nblocks && !blocks) || (nids && !ids)) return TSG_E_INVALID;
  return guard([&] {
    auto *h = new FindHolder();
    std::unique_ptr<FindHolder> g(h);
    per_device_merge(ctx, blocks, nblocks, h->o,
                     [&](DeviceCtx &dc, const std::vector<std::pair<uint32_t, V2Block *>> &list, FindOut &o) {
                       device_find(dc, list, ids, nids, opts, o);
                     },
                     find_append);
    h->pub.n = h->o.id_idx.size();
    h->pub.id_idx = h->o.id_idx.data();
    h->pub.block_idx = h->o.block_idx.data();
    h->pub.status = h->o.status.data();
    h->pub.obj_off = h->o.obj_off.data();
    h->pub.obj_len = h->o.obj_len.data();
    h->pub.obj_bytes = h->o.bytes.data();
    h->pub.kernel_ns = h->o.kernel_ns;
    *out = &g.release()->pub;
  });
}
void tsg_find_result_free(tsg_find_result *r) { delete reinterpret_cast<FindHolder *>(r); }

// ---- writer ---------------------------------------------------------------------------
int tsg_write_search_block(const char *dir, const uint8_t *entries, size_t len, int encoding, uint32_t page_size) {
  if (!dir || (len && !entries)) return TSG_E_INVALID;
  return guard([&] { write_search_block(dir, parse_entries(entries, len), encoding, page_size); });
}
int tsg_write_wal_search(const char *path, const uint8_t *entries, size_t len, int encoding) {
  if (!path || (len && !entries)) return TSG_E_INVALID;
  return guard([&] { write_wal_search(path, parse_entries(entries, len), encoding); });
}
int tsg_fb_search_entry(const uint8_t *entry, size_t len, uint8_t **out, size_t *out_len) {
  if (!entry || !out || !out_len) return TSG_E_INVALID;
  return guard([&] {
    auto es = parse_entries(entry, len);
    if (es.size() != 1) fail(TSG_E_INVALID, "expected exactly one entry");
    auto b = fb_search_entry_bytes(es[0]);
    *out = static_cast<uint8_t *>(std::malloc(b.size()));
    std::memcpy(*out, b.data(), b.size());
    *out_len = b.size();
  });
}
int tsg_fb_search_header(const uint8_t *entries, size_t len, uint8_t **out, size_t *out_len) {
  if (!out || !out_len) return TSG_E_INVALID;
  return guard([&] {
    HeaderBuilder h;
    for (auto &e : parse_entries(entries, len)) h.add_entry(e);
    auto b = h.to_bytes();
    *out = static_cast<uint8_t *>(std::malloc(b.size()));
    std::memcpy(*out, b.data(), b.size());
    *out_len = b.size();
  });
}
int tsg_synth_search_block(const char *dir, uint64_t n, uint64_t seed, int profile, int encoding,
                           uint32_t page_size) {
  if (!dir) return TSG_E_INVALID;
  return guard([&] { synth_search_block(dir, n, seed, profile, encoding, page_size); });
}
int tsg_synth_v2_block(const char *dir, uint64_t n, uint64_t seed, uint8_t (*ids_out)[16]) {
  if (!dir) return TSG_E_INVALID;
  return guard([&] { synth_v2_block(dir, n, seed, ids_out); });
}

int tsg_write_v2_block(const char *dir, const uint8_t (*ids)[16], const uint8_t *objs, const uint64_t *obj_off,
                       size_t n, int encoding, const char *data_encoding, uint32_t index_downsample_bytes) {
  if (!dir || (n && (!ids || !objs || !obj_off))) return TSG_E_INVALID;
  return guard([&] {
    for (size_t i = 1; i < n; i++)
      if (bytes_compare(ids[i - 1], 16, ids[i], 16) >= 0) fail(TSG_E_INVALID, "ids must be strictly ascending");
    std::vector<std::vector<uint8_t>> o(n ? n : 1);
    for (size_t i = 0; i < n; i++) o[i].assign(objs + obj_off[i], objs + obj_off[i + 1]);
    V2Params prm;
    prm.encoding = encoding;
    prm.data_encoding = data_encoding ? data_encoding : "v2";
    if (index_downsample_bytes) prm.index_downsample_bytes = index_downsample_bytes;
    for (int k = 0; k < 16; k++) prm.block_id[k] = uint8_t(0x11 * (k + 1));
    prm.block_id[6] = (prm.block_id[6] & 0x0f) | 0x40;
    write_v2_block(dir, ids, o, n, prm);
  });
}

int tsg_proto_block_open(tsg_ctx *ctx, const char *dir, int device_hint, tsg_proto_block **out) {
  if (!ctx || !dir || !out) return TSG_E_INVALID;
  return guard([&] {
    auto *b = new tsg_proto_block();
    b->ctx = ctx;
    try {
      proto_block_open(ctx->c, b->b, dir, device_hint);
    } catch (...) {
      proto_block_free(b->b);
      delete b;
      throw;
    }
    *out = b;
  });
}
void tsg_proto_block_close(tsg_proto_block *b) {
  if (!b) return;
  proto_block_free(b->b);
  delete b;
}
int tsg_proto_block_info(const tsg_proto_block *b, uint64_t out[4]) {
  if (!b || !out) return TSG_E_INVALID;
  out[0] = b->b.n;
  out[1] = b->b.page_len.size();
  out[2] = b->b.keys.size();
  out[3] = b->b.device_bytes;
  return TSG_OK;
}
int tsg_proto_search(tsg_ctx *ctx, tsg_proto_block *b, const tsg_proto_request *req, tsg_proto_result **out) {
  if (!ctx || !b || !req || !out || (req->ntags && (!req->keys || !req->key_lens || !req->values || !req->value_lens)))
    return TSG_E_INVALID;
  *out = nullptr;
  return guard([&] {
    ProtoOut o;
    proto_search(b->b, *req, o);
    if (o.status != TSG_OK) fail(o.status, o.error);
    auto *h = new ProtoHolder();
    std::unique_ptr<ProtoHolder> g(h);
    const ProtoBlock &pb = b->b;
    for (uint32_t i : o.traces) {
      h->id_off.push_back(uint32_t(h->ids.size()));
      h->id_len.push_back(pb.id_len[i]);
      h->ids.insert(h->ids.end(), pb.ids.begin() + pb.id_off[i], pb.ids.begin() + pb.id_off[i] + pb.id_len[i]);
      h->svc.emplace_back(pb.names, pb.svc_off[i], pb.svc_len[i]);
      h->root.emplace_back(pb.names, pb.root_off[i], pb.root_len[i]);
      h->start.push_back(pb.start_ns[i]);
      h->dur.push_back(pb.dur_ms[i]);
      h->obj.push_back(i);
    }
    for (size_t i = 0; i < h->svc.size(); i++) {
      h->svc_p.push_back(h->svc[i].c_str());
      h->root_p.push_back(h->root[i].c_str());
      h->svc_len.push_back(uint32_t(h->svc[i].size()));
      h->root_len.push_back(uint32_t(h->root[i].size()));
    }
    tsg_proto_result &r = h->pub;
    r.n = uint32_t(o.traces.size());
    r.trace_ids = h->ids.data();
    r.trace_id_off = h->id_off.data();
    r.trace_id_len = h->id_len.data();
    r.root_service_name = h->svc_p.data();
    r.root_trace_name = h->root_p.data();
    r.root_service_name_len = h->svc_len.data();
    r.root_trace_name_len = h->root_len.data();
    r.start_time_unix_nano = h->start.data();
    r.duration_ms = h->dur.data();
    r.object_idx = h->obj.data();
    r.inspected_traces = o.inspected_traces;
    r.inspected_bytes = o.inspected_bytes;
    r.skipped_traces = o.skipped_traces;
    r.kernel_ns = o.kernel_ns;
    *out = &g.release()->pub;
  });
}
void tsg_proto_result_free(tsg_proto_result *r) { delete reinterpret_cast<ProtoHolder *>(r); }

int tsg_go_parse(int kind, const char *s, size_t n, double *f, int64_t *i) {
  if (!s && n) return TSG_E_INVALID;
  std::string_view v(s ? s : "", n);
  if (kind == 0) {
    int64_t x = 0;
    const bool ok = go_parse_int(v, x);
    if (ok && i) *i = x;
    return ok;
  }
  if (kind == 1) {
    double x = 0;
    const bool ok = go_parse_float(v, x);
    if (ok && f) *f = x;
    return ok;
  }
  if (kind == 2) {
    bool x = false;
    const bool ok = go_parse_bool(v, x);
    if (ok && i) *i = x;
    return ok;
  }
  return TSG_E_INVALID;
}

}  // extern "C"
