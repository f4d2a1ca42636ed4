// writer.hpp — block writers and synthetic data (tooling, not the search path).
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace tsg {

// SearchDataMap: key -> set of values (pkg/tempofb/searchdatamap.go:13)
using TagMap = std::map<std::string, std::set<std::string>>;
// The same map accumulated over many entries (page and block-header rollups): hashed,
// sorted once when written (write_search_data_map orders keys and values as Go does).
using TagRollup = std::unordered_map<std::string, std::unordered_set<std::string>>;

struct SearchEntryIn {
  std::vector<uint8_t> id;
  uint64_t start = 0, end = 0;
  TagMap tags;
};

struct HeaderBuilder {  // SearchBlockHeaderMutable
  TagRollup tags;
  uint64_t min_dur = 0, max_dur = 0;
  void add_entry(const SearchEntryIn &e);
  std::vector<uint8_t> to_bytes() const;
};

std::vector<SearchEntryIn> parse_entries(const uint8_t *p, size_t n);
std::vector<uint8_t> fb_search_entry_bytes(const SearchEntryIn &e);
void write_search_block(const std::string &dir, std::vector<SearchEntryIn> entries, int enc, uint32_t page_size);
void write_wal_search(const std::string &path, const std::vector<SearchEntryIn> &entries, int enc);

// Streaming form of NewBackendSearchBlock: entries must arrive in strictly
// ascending trace-id order (what the deduping WAL iterator yields).
class SearchBlockWriter {
 public:
  SearchBlockWriter(const std::string &dir, int enc, uint32_t page_size);
  ~SearchBlockWriter();
  void append(const SearchEntryIn &e);
  void finish();

 private:
  struct Impl;
  Impl *p_;
};

struct V2Params {
  double bloom_fp = 0.01;                 // modules/storage/config.go:47
  uint64_t bloom_shard_bytes = 100 * 1024; // :48
  uint32_t index_downsample_bytes = 1024 * 1024;  // :49
  uint32_t index_page_bytes = 250 * 1024;  // :50
  int encoding = 0;
  uint8_t block_id[16] = {0};
  int64_t start_unix = 1700000000, end_unix = 1700003600;
  std::string data_encoding = "v2";  // meta dataEncoding: the object format (pkg/model/{v1,v2})
};
void bloom_estimate(uint64_t n, double fp, uint64_t &m, uint64_t &k);
uint32_t bloom_shard_count(double fp, uint64_t shard_size, uint64_t n);
void write_v2_block(const std::string &dir, const uint8_t (*ids)[16], const std::vector<std::vector<uint8_t>> &objs,
                    uint64_t n, const V2Params &prm);

// synth.cpp
void synth_search_block(const std::string &dir, uint64_t n, uint64_t seed, int profile, int enc, uint32_t page_size);
void synth_v2_block(const std::string &dir, uint64_t n, uint64_t seed, uint8_t (*ids_out)[16]);

}  // namespace tsg
