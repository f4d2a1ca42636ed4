// san_coal.cpp — TEST INFRASTRUCTURE ONLY: libtsg's C ABI under ThreadSanitizer (and ASan), with
// the device replaced by tests/sanitize/host_stub.cpp (tests/test_sanitizers.py).
//
// Many threads call tsg_search at once — one block per call with one query (the Go shim's
// per-block calls, which the coalescer merges into one launch), block sets spread over two stub
// devices (the per-device fan-out), limit queries through the progressive waves
// (TSG_LIMIT_WAVE0=4096), tsg_search_batch (its worker threads skip the coalescer) — and every
// result is compared with the same search run alone first. The coalescer's leaders and waiters
// (park.hpp: futex parking, the epoch word, the three-state lock), the result-holder pool and
// the wave consumer run under the sanitizer; the packed responses go through tsg_wire_merge.
// Usage: san_coal <tmpdir> <threads> <rounds>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "tsg.h"

namespace tsg {
void synth_search_block(const std::string &dir, uint64_t n, uint64_t seed, int profile, int enc, uint32_t page_size);
}

static uint64_t digest(const tsg_result *r) {
  uint64_t h = 1469598103934665603ull ^ r->n;
  for (uint64_t i = 0; i < r->n; i++) {
    for (int k = 0; k < 16; k++) h = (h ^ r->trace_id[i][k]) * 1099511628211ull;
    h = (h ^ r->block_idx[i]) * 1099511628211ull;
    h = (h ^ r->entry_idx[i]) * 1099511628211ull;
    h = (h ^ r->start_ns[i]) * 1099511628211ull;
    h = (h ^ r->root_service_len[i]) * 1099511628211ull;
  }
  h ^= uint64_t(r->metrics.traces_inspected) << 20 ^ r->metrics.bytes_inspected;
  return h;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  const std::string tmp = argv[1];
  const int nthreads = std::atoi(argv[2]), rounds = std::atoi(argv[3]);
  setenv("TSG_STUB_DEVICES", "2", 1);
  setenv("TSG_LIMIT_WAVE0", "4096", 1);
  tsg_ctx *ctx = nullptr;
  if (tsg_init(nullptr, &ctx) != TSG_OK) {
    std::fprintf(stderr, "tsg_init: %s\n", tsg_last_error());
    return 1;
  }
  constexpr int kBlocks = 6;
  std::vector<tsg_block *> blocks(kBlocks);
  for (int b = 0; b < kBlocks; b++) {
    const std::string dir = tmp + "/c" + std::to_string(b);
    tsg::synth_search_block(dir, 6000 + 1500 * uint64_t(b), 300 + uint64_t(b), 0, 6, 16 << 10);
    if (tsg_block_open(ctx, dir.c_str(), b % 2, &blocks[size_t(b)]) != TSG_OK) {
      std::fprintf(stderr, "open: %s\n", tsg_last_error());
      return 1;
    }
  }
  const char *vals[] = {"svc-07", "svc-03", "svc-11"};
  std::vector<tsg_pipeline *> pipes;
  for (const char *v : vals) {
    const uint8_t *k[] = {reinterpret_cast<const uint8_t *>("service.name")};
    const uint8_t *vv[] = {reinterpret_cast<const uint8_t *>(v)};
    const uint32_t kl[] = {12}, vl[] = {uint32_t(std::strlen(v))};
    tsg_request req{};
    req.ntags = 1;
    req.tag_keys = k;
    req.tag_key_lens = kl;
    req.tag_values = vv;
    req.tag_value_lens = vl;
    tsg_pipeline *p = nullptr;
    if (tsg_pipeline_new(&req, &p) != TSG_OK) return 1;
    pipes.push_back(p);
  }
  // the cases: (query, first block, block count, limit)
  std::vector<std::tuple<int, int, int, uint32_t>> cases;
  for (int q = 0; q < 3; q++)
    for (int b = 0; b < kBlocks; b++) {
      cases.emplace_back(q, b, 1, 0);   // per-block calls (coalesced)
      cases.emplace_back(q, b, 1, 20);  // the shim's limit-20 per block
    }
  for (int q = 0; q < 3; q++) {
    cases.emplace_back(q, 0, kBlocks, 0);
    cases.emplace_back(q, 0, kBlocks, 7);
    cases.emplace_back(q, 1, 4, 50);
  }
  auto run = [&](size_t c, uint64_t *dg, uint64_t *n) -> int {
    const auto &[q, b0, nb, lim] = cases[c];
    tsg_search_opts o{};
    o.limit = lim;
    tsg_result *r = nullptr;
    const int rc = tsg_search(ctx, blocks.data() + b0, size_t(nb), tsg_pipeline_query(pipes[size_t(q)]), &o, &r);
    if (rc) return rc;
    *dg = digest(r);
    *n = r->n;
    tsg_result_free(r);
    return 0;
  };
  std::vector<uint64_t> exp(cases.size()), expn(cases.size());
  for (size_t c = 0; c < cases.size(); c++)
    if (run(c, &exp[c], &expn[c])) {
      std::fprintf(stderr, "case %zu: %s\n", c, tsg_last_error());
      return 1;
    }
  std::atomic<int> bad{0}, calls{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++)
    th.emplace_back([&, t] {
      std::mt19937_64 rng(uint64_t(t) * 7919 + 1);
      for (int r = 0; r < rounds; r++) {
        if (t % 4 == 3 && r % 5 == 0) {  // a batch: its items run on worker threads, past the coalescer
          std::vector<tsg_search_item> items;
          std::vector<size_t> which;
          for (int i = 0; i < 6; i++) {
            const size_t c = size_t(rng() % cases.size());
            const auto &[q, b0, nb, lim] = cases[c];
            tsg_search_item it{};
            it.blocks = blocks.data() + b0;
            it.nblocks = size_t(nb);
            it.query = tsg_pipeline_query(pipes[size_t(q)]);
            it.opts.limit = lim;
            items.push_back(it);
            which.push_back(c);
          }
          std::vector<tsg_result *> outs(items.size());
          uint64_t dns = 0;
          if (tsg_search_batch(ctx, items.data(), items.size(), 3, outs.data(), &dns) != TSG_OK) {
            bad++;
            continue;
          }
          for (size_t i = 0; i < items.size(); i++) {
            if (digest(outs[i]) != exp[which[i]]) bad++;
            tsg_result_free(outs[i]);
          }
          calls += int(items.size());
          continue;
        }
        // the shim pattern: the same query on each block at once from this thread's share
        const size_t c = size_t(rng() % cases.size());
        uint64_t dg = 0, n = 0;
        if (run(c, &dg, &n) || dg != exp[c] || n != expn[c]) bad++;
        calls++;
      }
    });
  for (auto &x : th) x.join();
  // the frontend's merge over packed responses (tsg_result_pack / tsg_wire_merge)
  std::vector<uint8_t *> wires;
  std::vector<size_t> lens;
  for (int b = 0; b < kBlocks; b++) {
    tsg_search_opts o{};
    tsg_result *r = nullptr;
    if (tsg_search(ctx, blocks.data() + b, 1, tsg_pipeline_query(pipes[0]), &o, &r) != TSG_OK) return 1;
    uint8_t *w = nullptr;
    size_t wl = 0;
    if (tsg_result_pack(r, &w, &wl) != TSG_OK) return 1;
    wires.push_back(w);
    lens.push_back(wl);
    tsg_result_free(r);
  }
  size_t need = 0;
  tsg_wire_merge(wires.data(), lens.data(), wires.size(), 20, kBlocks, nullptr, 0, &need);
  std::vector<uint8_t> merged(need + 64);
  size_t got = 0;
  if (tsg_wire_merge(wires.data(), lens.data(), wires.size(), 20, kBlocks, merged.data(), merged.size(), &got) != TSG_OK)
    bad++;
  for (uint8_t *w : wires) tsg_free(w);
  for (auto *b : blocks) tsg_block_close(b);
  for (auto *p : pipes) tsg_pipeline_free(p);
  tsg_shutdown(ctx);
  std::printf("san_coal: %d calls, %zu cases, %d mismatches; merge %zu bytes\n", calls.load(), cases.size(), bad.load(), got);
  return bad.load() ? 1 : 0;
}
