// pipeline.cpp — host mirror of search.NewSearchPipeline (tempodb/search/pipeline.go:26-140)
// and of Pipeline.MatchesBlock (:172-183) for the block prefilter, which runs on the
// host against the on-disk search-header (pitfall P1: never recomputed values).
#include <cstring>
#include <string>
#include <vector>

#include "block.hpp"
#include "common.hpp"

struct tsg_pipeline {
  std::vector<std::string> keys, values;
  std::vector<const uint8_t *> kp, vp;
  std::vector<uint32_t> kl, vl;
  tsg_query q{};
};

namespace tsg {

static bool eq(std::string_view a, const char *b) { return a == b; }

tsg_pipeline *pipeline_new(const tsg_request &req) {
  auto *p = new tsg_pipeline();
  if (req.min_duration_ms > 0) {  // pipeline.go:29-42
    p->q.has_min = 1;
    p->q.min_ns = uint64_t(req.min_duration_ms) * 1000000ULL;
  }
  if (req.max_duration_ms > 0) {  // :44-57
    p->q.has_max = 1;
    p->q.max_ns = uint64_t(req.max_duration_ms) * 1000000ULL;
  }
  if (req.start != 0 && req.end != 0) {  // :59-66
    p->q.has_range = 1;
    p->q.start_s = req.start;
    p->q.end_s = req.end;
  }
  for (uint32_t i = 0; i < req.ntags; i++) {
    std::string_view k(reinterpret_cast<const char *>(req.tag_keys[i]), req.tag_key_lens[i]);
    std::string_view v(reinterpret_cast<const char *>(req.tag_values[i]), req.tag_value_lens[i]);
    // rewriteTagLookup (pipeline.go:108-140); matched on the request bytes before ToLower
    if (eq(k, "x-dbg-exhaustive")) {  // SecretExhaustiveSearchTag
      p->q.exhaustive = 1;
      continue;
    }
    std::string nk(k), nv(v);
    if (eq(k, "error")) {  // trace.ErrorTag
      if (eq(v, "true")) { nk = "status.code"; nv = "2"; }
    } else if (eq(k, "status.code")) {  // trace.StatusCodeMapping (pkg/model/trace/matches.go:27-31)
      if (eq(v, "unset")) { nv = "0"; }
      else if (eq(v, "ok")) { nv = "1"; }
      else if (eq(v, "error")) { nv = "2"; }
    }
    p->keys.push_back(go_to_lower(nk));  // pipeline.go:82-83
    p->values.push_back(go_to_lower(nv));
  }
  for (size_t i = 0; i < p->keys.size(); i++) {
    p->kp.push_back(reinterpret_cast<const uint8_t *>(p->keys[i].data()));
    p->vp.push_back(reinterpret_cast<const uint8_t *>(p->values[i].data()));
    p->kl.push_back(uint32_t(p->keys[i].size()));
    p->vl.push_back(uint32_t(p->values[i].size()));
  }
  p->q.nterms = uint32_t(p->keys.size());
  p->q.keys = p->kp.data();
  p->q.values = p->vp.data();
  p->q.key_lens = p->kl.data();
  p->q.value_lens = p->vl.data();
  return p;
}

bool pipeline_matches_block(const tsg_query &q, const uint8_t *hdr, size_t len) {
  FbTable h = FbTable::root(hdr, len);
  if (q.has_min && !(h.u64(kHdrMax) >= q.min_ns)) return false;  // pipeline.go:38-41
  if (q.has_max && !(h.u64(kHdrMin) <= q.max_ns)) return false;  // :53-56
  for (uint32_t t = 0; t < q.nterms; t++) {
    std::string_view k(reinterpret_cast<const char *>(q.keys[t]), q.key_lens[t]);
    std::string_view v(reinterpret_cast<const char *>(q.values[t]), q.value_lens[t]);
    if (!fb_contains_tag(h, kHdrTags, k, v)) return false;
  }
  return true;
}

// The same predicate over the header walked at open (HostBlock::hdr_*): the same binary
// search over the keys in the header's order (searchdata_util.go:63-100, reversed
// comparator) and the same bytes.Contains over the found key's values.
// defer != nullptr: a term whose key's header values are the block's (large) dictionary
// (HostBlock::hdr_defer) is not scanned here; its bit is set in *defer and the caller takes
// "some value contains the needle" from the device dictionary pass (tsg_search).
bool pipeline_matches_block_indexed(const tsg_query &q, const HostBlock &h, uint32_t *defer) {
  if (defer) *defer = 0;
  if (q.has_min && !(h.max_dur >= q.min_ns)) return false;  // pipeline.go:38-41
  if (q.has_max && !(h.min_dur <= q.max_ns)) return false;  // :53-56
  const uint32_t n = uint32_t(h.hdr_keys.size());
  for (uint32_t t = 0; t < q.nterms; t++) {
    const uint8_t *k = q.keys[t];
    const size_t kl = q.key_lens[t];
    std::string_view v(reinterpret_cast<const char *>(q.values[t]), q.value_lens[t]);
    uint32_t i = 0, j = n, at = n;
    while (i < j) {
      const uint32_t m = (i + j) >> 1;
      const std::string_view key = h.hdr_keys[m];
      const int c = bytes_compare(reinterpret_cast<const uint8_t *>(key.data()), key.size(), k, kl);
      if (c == 0) {
        at = m;
        break;
      }
      if (c < 0) j = m;
      else i = m + 1;
    }
    if (at == n) return false;
    if (defer && t < 32 && !q.exhaustive && at < h.hdr_defer.size() && h.hdr_defer[at]) {
      *defer |= 1u << t;
      continue;
    }
    bool any = false;
    for (uint32_t x = h.hdr_val0[at]; x < h.hdr_val0[at + 1] && !any; x++)
      any = v.empty() || h.hdr_vals[x].find(v) != std::string_view::npos;  // bytes.Contains
    if (!any) return false;
  }
  return true;
}

// MatchesBlock on a StreamingSearchBlock's SearchBlockHeaderMutable
// (streaming_search_block.go:127-134): the same duration filters, but the tag filter is
// SearchDataMap.Contains (searchdatamap.go:43-49): the EXACT value must be present,
// not a substring of one (the backend header's ContainsTag).
bool pipeline_matches_stream_header(const tsg_query &q, uint64_t min_dur, uint64_t max_dur,
                                    const std::map<std::string, std::set<std::string>> &tags) {
  if (q.has_min && !(max_dur >= q.min_ns)) return false;
  if (q.has_max && !(min_dur <= q.max_ns)) return false;
  for (uint32_t t = 0; t < q.nterms; t++) {
    auto it = tags.find(std::string(reinterpret_cast<const char *>(q.keys[t]), q.key_lens[t]));
    if (it == tags.end()) return false;
    if (!it->second.count(std::string(reinterpret_cast<const char *>(q.values[t]), q.value_lens[t]))) return false;
  }
  return true;
}

}  // namespace tsg

extern "C" {
const tsg_query *tsg_pipeline_query(const tsg_pipeline *p) { return p ? &p->q : nullptr; }
void tsg_pipeline_free(tsg_pipeline *p) { delete p; }
}
