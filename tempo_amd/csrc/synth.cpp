// synth.cpp — seeded synthetic trace-search data (SURVEY.md §8 d). Tag vocabulary
// follows what the distributor extracts (modules/distributor/search_data.go:28-113):
// lowercase keys, string values, root.service.name / root.name of the root span.
// Entries are generated directly in ascending trace-id order and streamed through
// SearchBlockWriter, so a 1 M-entry block never exists as a whole in memory.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "common.hpp"
#include "writer.hpp"

namespace tsg {

namespace {
struct SplitMix {
  uint64_t s;
  explicit SplitMix(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return next() % n; }
  double unit() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
  double normal() {
    double u1 = unit(), u2 = unit();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

const char *kMethods[] = {"get", "post", "put", "delete", "patch", "head", "options", "connect"};
const char *kKinds[] = {"client", "server", "internal", "producer", "consumer"};
const char *kPlans[] = {"free", "pro", "team", "enterprise"};
const char *kWords[] = {"users", "orders", "items", "carts", "payments", "sessions", "accounts", "invoices",
                        "products", "reviews", "search", "shipping", "tokens", "events", "metrics", "auth"};
const char *kTables[] = {"users", "orders", "line_items", "carts", "payments", "sessions", "accounts", "inventory"};

std::string fmt(const char *f, uint64_t v) {
  char b[64];
  std::snprintf(b, sizeof b, f, (unsigned long long)v);
  return b;
}

void gen_tags(SplitMix &r, int profile, TagMap &t) {
  uint64_t svc = r.below(50);
  std::string s = fmt("svc-%02llu", svc);
  t["service.name"].insert(s);
  t["root.service.name"].insert(s);
  t["root.name"].insert(fmt("op-%03llu", r.below(500)));
  uint64_t nn = 1 + r.below(5);
  for (uint64_t i = 0; i < nn; i++) t["name"].insert(fmt("span-%04llu", r.below(2000)));
  uint64_t sc = r.below(100);
  t["status.code"].insert(sc < 90 ? "0" : (sc < 95 ? "1" : "2"));
  t["http.method"].insert(kMethods[r.below(8)]);
  t["http.status_code"].insert(fmt("%llu", 200 + r.below(40) * 7));
  {
    std::string url = "/api/v1/";
    uint64_t segs = 2 + r.below(6);
    for (uint64_t i = 0; i < segs; i++) {
      url += kWords[r.below(16)];
      url += '/';
      url += std::to_string(r.below(1000000));
      url += '/';
    }
    url += "?q=" + std::to_string(r.next() % 100000000000ULL);
    if (url.size() > 200) url.resize(200);
    t["http.url"].insert(url);
  }
  if (profile == 1) {
    std::string st = "select ";
    uint64_t target = 100 + r.below(1901);
    while (st.size() < target) {
      st += "c";
      st += std::to_string(r.below(100));
      st += ", ";
      if (r.below(8) == 0) {
        st += "from ";
        st += kTables[r.below(8)];
        st += " where id = ";
        st += std::to_string(r.below(10000000));
        st += " and ";
      }
    }
    st.resize(target);
    t["db.statement"].insert(st);
  }
  t["k8s.namespace"].insert(fmt("ns-%02llu", r.below(20)));
  t["k8s.pod.name"].insert(fmt("pod-%04llu", r.below(1000)));
  t["cluster"].insert(fmt("cluster-%llu", r.below(5)));
  t["region"].insert(fmt("region-%llu", r.below(10)));
  t["host.name"].insert(fmt("host-%03llu", r.below(500)));
  t["component"].insert(fmt("comp-%02llu", r.below(30)));
  t["peer.service"].insert(fmt("peer-%02llu", r.below(50)));
  t["span.kind"].insert(kKinds[r.below(5)]);
  t["error"].insert(sc >= 95 ? "true" : "false");
  t["user.id"].insert(fmt("user-%06llu", r.below(100000)));
  t["tenant.plan"].insert(kPlans[r.below(4)]);
}
}  // namespace

void synth_search_block(const std::string &dir, uint64_t n, uint64_t seed, int profile, int enc, uint32_t page_size) {
  SplitMix r(0x7e3a0ULL + seed);
  std::vector<std::array<uint8_t, 16>> ids(n);
  for (auto &id : ids) {
    uint64_t a = r.next(), b = r.next();
    std::memcpy(id.data(), &a, 8);
    std::memcpy(id.data() + 8, &b, 8);
  }
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  const uint64_t T0 = 1700000000ULL * 1000000000ULL;
  SearchBlockWriter w(dir, enc, page_size);
  SearchEntryIn e;
  for (size_t i = 0; i < ids.size(); i++) {
    SplitMix er(seed * 0x9E3779B97F4A7C15ULL ^ (i + 1) * 0xD1B54A32D192ED03ULL);
    e.id.assign(ids[i].begin(), ids[i].end());
    e.start = T0 + er.below(3600ULL * 1000000000ULL);
    double d = std::exp(std::log(50e6) + 1.5 * er.normal());  // median 50 ms, sigma 1.5
    d = std::min(std::max(d, 1e3), 60e9);
    e.end = e.start + uint64_t(d);
    if (er.below(1000) == 0) e.end = 0;  // 0.1 %: missing end (pitfalls P1/P2)
    e.tags.clear();
    gen_tags(er, profile, e.tags);
    w.append(e);
  }
  w.finish();
}

void synth_v2_block(const std::string &dir, uint64_t n, uint64_t seed, uint8_t (*ids_out)[16]) {
  SplitMix r(0xb10c0ULL + seed);
  std::vector<std::array<uint8_t, 16>> ids(n);
  for (auto &id : ids) {
    uint64_t a = r.next(), b = r.next();
    std::memcpy(id.data(), &a, 8);
    std::memcpy(id.data() + 8, &b, 8);
  }
  std::sort(ids.begin(), ids.end());
  std::vector<std::vector<uint8_t>> objs(16);
  for (size_t i = 0; i < objs.size(); i++) objs[i].assign(64 + 16 * i, uint8_t(i));
  V2Params prm;
  uint64_t a = r.next(), b = r.next();
  std::memcpy(prm.block_id, &a, 8);
  std::memcpy(prm.block_id + 8, &b, 8);
  prm.block_id[6] = (prm.block_id[6] & 0x0f) | 0x40;
  prm.start_unix = 1700000000 + int64_t(seed % 100) * 3600;
  prm.end_unix = prm.start_unix + 3600;
  write_v2_block(dir, reinterpret_cast<const uint8_t(*)[16]>(ids.data()), objs, ids.size(), prm);
  if (ids_out) std::memcpy(ids_out, ids.data(), ids.size() * 16);
}

}  // namespace tsg
