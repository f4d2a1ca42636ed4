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
#include <atomic>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

#include "tsg.h"

extern "C" {
// rounds queries over nsets block sets of nblocks blocks each (blocks[s * nblocks + i]);
// query r searches set r % nsets. round_ns[r] = wall time of query r (all calls issued at
// once, until the last returned); matches[r] = records over all blocks of query r. limit: the
// request's limit passed per block (tsg_search_opts.limit; the ingester's default is 20, 0 =
// every match). Returns the first non-zero tsg_search code (the round's other calls still
// complete).
int tsgx_shim_pattern(tsg_ctx *ctx, tsg_block *const *blocks, size_t nblocks, size_t nsets, const tsg_query *q,
                      uint32_t limit, uint32_t rounds, uint64_t *round_ns, uint64_t *matches) {
  if (!ctx || !q || !blocks || !nblocks || !nsets || !round_ns || !matches) return TSG_E_INVALID;
  std::atomic<uint32_t> gen{0};
  std::atomic<size_t> left{0};
  std::atomic<uint64_t> nmatch{0};
  std::atomic<int> first_err{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  th.reserve(nblocks);
  for (size_t i = 0; i < nblocks; i++)
    th.emplace_back([&, i] {
      uint32_t seen = 0;
      for (;;) {
        uint32_t g;
        while ((g = gen.load(std::memory_order_acquire)) == seen && !stop.load(std::memory_order_acquire))
          __builtin_ia32_pause();
        if (stop.load(std::memory_order_acquire)) return;
        seen = g;
        tsg_search_opts o{};
        o.limit = limit;
        tsg_result *r = nullptr;
        const int rc = tsg_search(ctx, &blocks[((g - 1) % nsets) * nblocks + i], 1, q, &o, &r);
        if (rc == TSG_OK) {
          nmatch.fetch_add(r->n, std::memory_order_relaxed);
          tsg_result_free(r);
        } else {
          int z = 0;
          first_err.compare_exchange_strong(z, rc);
        }
        left.fetch_sub(1, std::memory_order_acq_rel);
      }
    });
  for (uint32_t r = 0; r < rounds; r++) {
    nmatch.store(0);
    left.store(nblocks, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    gen.fetch_add(1, std::memory_order_acq_rel);
    while (left.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    round_ns[r] = uint64_t(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
    matches[r] = nmatch.load();
  }
  stop.store(true, std::memory_order_release);
  for (auto &t : th) t.join();
  return first_err.load();
}
}
