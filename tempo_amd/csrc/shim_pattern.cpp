// shim_pattern.cpp — the Go shim's call pattern for the ingester, in C (bench / test
// driver, built to tempo_amd/libtsg_shim_pattern.so next to libtsg; not part of the ABI).
//
// instance.searchLocalBlocks starts one goroutine per block and each calls
// BackendSearchBlock.Search on its own (modules/ingester/instance_search.go:164-185); the
// shim turns each into one tsg_search over that block with the request's
// limit (Pipeline.Query carries it) and a tsg_result_free. Goroutines run on OS threads without a global lock, so the pattern is
// driven from C threads here (Python threads would serialise on the GIL between calls).
// One thread per block, kept across queries (Go reuses its OS threads); a query ends when
// every block's call has returned.
//
// Idle threads wait the way goroutines do: parked, not spinning (a goroutine blocked on a
// channel or a WaitGroup holds no CPU). A short bounded spin first (park.hpp), then the futex:
// with more threads than CPUs, spinning idlers kept the one thread with work — the coalesced
// launch's leader — off a CPU until the scheduler's next tick (10 ms steps).
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "park.hpp"
#include "tsg.h"

namespace {
// FNV-1a 64 over one block's ordered records (caller-set position, then per record its scan
// position, id and start): the per-round digest is the sum over the set's blocks, so it does
// not depend on which thread finished first.
uint64_t fnv(uint64_t h, const void *p, size_t n) {
  const auto *b = static_cast<const uint8_t *>(p);
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
  return h;
}
uint64_t result_digest(uint32_t pos, const tsg_result *r) {
  uint64_t h = fnv(0xcbf29ce484222325ull, &pos, 4);
  for (uint64_t i = 0; i < r->n; i++) {
    h = fnv(h, &r->entry_idx[i], 8);
    h = fnv(h, r->trace_id[i], 16);
    h = fnv(h, &r->start_ns[i], 8);
  }
  return h;
}
}  // namespace

extern "C" {
// rounds queries over nsets block sets of nblocks blocks each (blocks[s * nblocks + i]);
// query r searches set r % nsets. round_ns[r] = wall time of query r (all calls issued at
// once, until the last returned); matches[r] = records over all blocks of query r; digest[r]
// (optional) = the sum over blocks i of result_digest(i, block i's result). limit: the
// request's limit passed per block (tsg_search_opts.limit; the ingester's default is 20, 0 =
// every match). Returns the first non-zero tsg_search code (the round's other calls still
// complete).
int tsgx_shim_pattern(tsg_ctx *ctx, tsg_block *const *blocks, size_t nblocks, size_t nsets, const tsg_query *q,
                      uint32_t limit, uint32_t rounds, uint64_t *round_ns, uint64_t *matches, uint64_t *digest) {
  if (!ctx || !q || !blocks || !nblocks || !nsets || !round_ns || !matches) return TSG_E_INVALID;
  constexpr uint64_t kSpinNs = 20000;  // an idle thread's spin before it parks
  tsg::EpochPark go;                    // epoch = query generation
  std::atomic<uint32_t> left{0};        // calls of the current query still running (futex word)
  std::atomic<int> main_parked{0};
  std::atomic<uint64_t> nmatch{0}, dsum{0};
  std::atomic<int> first_err{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  th.reserve(nblocks);
  for (size_t i = 0; i < nblocks; i++)
    th.emplace_back([&, i] {
      uint32_t seen = 0;
      for (;;) {
        uint32_t g;
        while ((g = go.read()) == seen && !stop.load(std::memory_order_acquire)) {
          if (tsg::spin_for(kSpinNs, [&] { return go.read() != seen || stop.load(std::memory_order_acquire); }))
            continue;
          go.wait(seen, 100'000'000);
        }
        if (stop.load(std::memory_order_acquire)) return;
        seen = g;
        tsg_search_opts o{};
        o.limit = limit;
        tsg_result *r = nullptr;
        const int rc = tsg_search(ctx, &blocks[((g - 1) % nsets) * nblocks + i], 1, q, &o, &r);
        if (rc == TSG_OK) {
          nmatch.fetch_add(r->n, std::memory_order_relaxed);
          if (digest) dsum.fetch_add(result_digest(uint32_t(i), r), std::memory_order_relaxed);
          tsg_result_free(r);
        } else {
          int z = 0;
          first_err.compare_exchange_strong(z, rc);
        }
        if (left.fetch_sub(1, std::memory_order_seq_cst) == 1 && main_parked.load(std::memory_order_seq_cst))
          tsg::futex_wake_u32(&left);
      }
    });
  for (uint32_t r = 0; r < rounds; r++) {
    nmatch.store(0);
    dsum.store(0);
    left.store(uint32_t(nblocks), std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    go.notify();
    // the caller waits like a WaitGroup: a short spin, then parked until the last call wakes it
    if (!tsg::spin_for(kSpinNs, [&] { return left.load(std::memory_order_acquire) == 0; })) {
      main_parked.store(1, std::memory_order_seq_cst);
      for (uint32_t v; (v = left.load(std::memory_order_seq_cst)) != 0;) tsg::futex_wait_u32(&left, v, 100'000'000);
      main_parked.store(0, std::memory_order_relaxed);
    }
    round_ns[r] = uint64_t(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
    matches[r] = nmatch.load();
    if (digest) digest[r] = dsum.load();
  }
  stop.store(true, std::memory_order_release);
  go.notify();
  for (auto &t : th) t.join();
  return first_err.load();
}
}
