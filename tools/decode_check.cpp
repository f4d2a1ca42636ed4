// Host-only check of the columnar decoder (no device): decodes a block and
// prints per-key dictionary stats. Build: g++ -O2 -std=c++17 tools/decode_check.cpp
//   -Itempo_amd/csrc -Iinclude -Ltempo_amd -ltsg -Wl,-rpath,$PWD/tempo_amd
#include <cstdio>
#include "block.hpp"
int main(int argc, char **argv) {
  using namespace tsg;
  std::string d = argv[1];
  std::vector<uint8_t> m, h, i, s;
  read_file(d + "/search.meta.json", m); read_file(d + "/search-header", h);
  read_file(d + "/search-index", i); read_file(d + "/search", s);
  HostBlock hb;
  try {
    decode_search_block(m.data(), m.size(), true, h, i.data(), i.size(), s.data(), s.size(), 0, hb);
  } catch (Error &e) { printf("error %d %s\n", e.code, e.what()); return 1; }
  printf("n=%lu pages=%zu fb=%lu keys=%zu min=%lu max=%lu\n", hb.n, hb.page_entries.size(), hb.fb_bytes,
         hb.keys.size(), hb.min_dur, hb.max_dur);
  for (auto &k : hb.keys) {
    size_t present = 0; for (auto c : k.col) present += c != kNone;
    printf("  %-20s vals=%u sets=%u width=%d identity=%d present=%zu\n", k.name.c_str(), k.nvals(), k.nsets(), k.width(), k.identity, present);
  }
  if (hb.svc_key >= 0) printf("entry0 svc=%.*s\n", (int)hb.dict_value(hb.svc_key, hb.svc_vid[0]).size(), hb.dict_value(hb.svc_key, hb.svc_vid[0]).data());
  return 0;
}
