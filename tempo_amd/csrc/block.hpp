// block.hpp — on-disk formats (read side) and the host half of the columnar
// loader: a backend search block decoded ONCE into per-key dictionaries,
// value-set ids and per-entry columns, ready to upload to HBM.
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"

namespace tsg {

// ---- flatbuffer table access (vendor/github.com/google/flatbuffers/go/table.go:14-57),
// bounds-checked: a malformed buffer raises TSG_E_CORRUPT instead of reading past it.
struct FbTable {
  const uint8_t *b = nullptr;
  size_t n = 0;
  uint32_t pos = 0;

  void need(uint64_t off, uint64_t len) const {
    if (off + len > n) fail(TSG_E_CORRUPT, "flatbuffer offset out of range");
  }
  uint16_t field(uint16_t vto) const {  // Table.Offset
    need(pos, 4);
    int64_t vt = int64_t(pos) - int32_t(le32(b + pos));
    if (vt < 0) fail(TSG_E_CORRUPT, "flatbuffer vtable out of range");
    need(uint64_t(vt), 2);
    uint16_t vlen = le16(b + vt);
    if (vto < vlen) {
      need(uint64_t(vt) + vto, 2);
      return le16(b + vt + vto);
    }
    return 0;
  }
  uint32_t indirect(uint32_t off) const {
    need(off, 4);
    return off + le32(b + off);
  }
  uint32_t vector_len(uint16_t o) const {
    uint32_t off = indirect(pos + o);
    need(off, 4);
    return le32(b + off);
  }
  uint32_t vector_start(uint16_t o) const { return indirect(pos + o) + 4; }
  std::string_view byte_vector(uint32_t off) const {  // Table.ByteVector
    off = indirect(off);
    need(off, 4);
    uint32_t l = le32(b + off);
    need(uint64_t(off) + 4, l);
    return {reinterpret_cast<const char *>(b + off + 4), l};
  }
  uint64_t u64(uint16_t vto) const {
    uint16_t o = field(vto);
    if (!o) return 0;
    need(uint64_t(pos) + o, 8);
    return le64(b + pos + o);
  }
  static FbTable root(const uint8_t *b, size_t n) {
    FbTable t;
    t.b = b;
    t.n = n;
    t.need(0, 4);
    t.pos = le32(b);
    return t;
  }
};

// tempofb vtable slots (pkg/tempofb/{SearchEntry,SearchPage,SearchBlockHeader,KeyValues}.go)
enum : uint16_t {
  kEntryId = 4, kEntryTags = 6, kEntryStart = 8, kEntryEnd = 10,
  kPageTags = 4, kPageEntries = 6,
  kHdrTags = 4, kHdrMin = 6, kHdrMax = 8,
  kKvKey = 4, kKvValue = 6,
};

// FindTag + ContainsTag over any [KeyValues] vector (pkg/tempofb/searchdata_util.go:47-100).
bool fb_contains_tag(const FbTable &t, uint16_t tags_vto, std::string_view k, std::string_view v);
struct HostBlock;
void index_header(HostBlock &hb);  // fills hdr_keys / hdr_vals / hdr_val0 (block.cpp)

// ---- search.meta.json (tempodb/search/block_meta.go:11-43) ----------------------
struct SearchMeta {
  std::string version;
  int encoding = -1;
  uint32_t index_page_size = 0, index_records = 0;
};
SearchMeta parse_search_meta(const uint8_t *p, size_t n);

// ---- v2 index (tempodb/encoding/v2/index_reader.go) -------------------------------
struct IndexRecord {
  uint8_t id[16];
  uint64_t start;
  uint32_t length;
};
// indexReader.At for i = 0, 1, ... (index_reader.go:42-82,116-143): page checksum
// (xxhash64) verified, all-zero record rejected. prefix == nullptr: any failure throws
// TSG_E_CORRUPT (the trace-ID lookup path, where Find returns the error). Otherwise the
// records before the first failing At(i) are returned and *prefix is set to true when
// one failed: BackendSearchBlock.Search drops At's error (`record, _ := ir.At(ctx, i)`,
// backend_search_block.go:252-255) and ends the block there without an error.
std::vector<IndexRecord> read_index(const uint8_t *p, size_t n, uint32_t page_size, uint32_t total,
                                    bool *prefix = nullptr);
// dataReader.Read of one record + decompression (data_reader.go:45-125).
void read_data_page(const uint8_t *file, size_t flen, const IndexRecord &r, int enc, std::vector<uint8_t> &out);
int zstd_host_decode(const uint8_t *src, size_t n, std::vector<uint8_t> &out);  // zstd_host.cpp

// ---- the decoded block ------------------------------------------------------------
static constexpr uint32_t kNone = 0xFFFFFFFFu;

struct KeyColumn {
  std::string name;
  // value dictionary (distinct values of this key in the block, first-seen order)
  Bytes dict_bytes;  // (no zero fill on resize: config 4 holds ~1 GB here)
  std::vector<uint32_t> dict_off;  // nvals + 1
  // value sets (the distinct value vectors of this key's KeyValues tables)
  std::vector<uint32_t> set_off;   // nsets + 1
  std::vector<uint32_t> set_vals;  // value ids, in vector order (descending bytes)
  bool identity = true;            // every set is {v} with set id == value id
  std::vector<uint32_t> col;       // per entry: set id or kNone (key absent)
  // large dictionaries (> kDeferMinBytes): counts of each adjacent byte pair (b0 << 8 | b1) in
  // a sample of the value bytes; the dictionary stream pass tests a needle's rarest pair
  std::vector<uint32_t> pair_freq;
  // during the load only (large dictionaries): each value's xxhash64, for verify_header_dicts
  std::vector<uint64_t> dict_vh;
  uint32_t nvals() const { return uint32_t(dict_off.size() - 1); }
  uint32_t nsets() const { return uint32_t(set_off.size() - 1); }
  int width() const { return nsets() < 255 ? 1 : (nsets() < 65535 ? 2 : 4); }
};

struct HostBlock {
  bool has_meta = false;
  // WAL (StreamingSearchBlock) form: one entry per "page", no on-disk header; the
  // header is the SearchBlockHeaderMutable rebuilt during replay (exact-value Contains)
  bool streaming = false;
  bool partial = false;  // replay stopped at a damaged page (the reference's warning)
  // Backend blocks with damage: a failing index record ends the block silently (its
  // pages are not resident; index_truncated = true). A damaged data page k (read, page
  // framing, decompression, object framing, flatbuffer bounds) keeps pages [0, k)
  // resident and stop_status / stop_msg is the error the reference's Search returns
  // after their matches (backend_search_block.go:258-266); 0 = none.
  bool index_truncated = false;
  // a page range of the block (tsg_block_open_pages: one rank's share of a large block): index
  // records [part_first_page, +n). part_tail: the range does not start at page 0, so its
  // searches count neither the header's bytes nor the block as inspected / skipped (the range
  // at page 0 does: the ranges' metrics sum to the whole block's); scan positions are inside
  // the range
  uint32_t part_first_page = 0;
  bool part_tail = false;
  int stop_status = 0;
  std::string stop_msg;
  // WAL blocks: the mutable header's (key -> values) map (Tags / TagValues / block filter).
  // Live blocks: per key the values FindTag reaches in some segment (TagValues).
  std::map<std::string, std::set<std::string>> stream_tags;
  // Live traces (instance.searchLiveTraces, modules/ingester/instance_search.go:83-130): one
  // row per search-data segment, rows in trace order; trace t = rows [trace_row0[t],
  // trace_row0[t+1]) (a trace may have none), trace_bytes0 = prefix sums of the segments'
  // lengths (bytesInspected). No header: searched without a block filter.
  bool live = false;
  std::vector<uint32_t> row_trace;
  std::vector<uint64_t> trace_row0, trace_bytes0;
  uint32_t ntraces() const { return trace_row0.empty() ? 0u : uint32_t(trace_row0.size() - 1); }
  SearchMeta meta;
  Bytes header;  // raw search-header flatbuffer (kept for MatchesBlock/Tags)
  uint64_t min_dur = 0, max_dur = 0;
  // the header's tag table walked once at open (MatchesBlock per query without decoding
  // the flatbuffer again): keys in the header's own order, each key's values (CSR), views
  // into `header`. hdr_index false: a header that did not walk cleanly (the per-query
  // flatbuffer path then fails the search exactly where the reference's reader would)
  std::vector<std::string_view> hdr_keys, hdr_vals;
  std::vector<uint32_t> hdr_val0;
  bool hdr_index = false;
  // per header key (hdr_keys order): 1 = the key's value list is the block's dictionary for
  // that key (same values, compared byte for byte at open: verify_header_dicts)
  // and the dictionary is large (> kDeferMinBytes). MatchesBlock's "any header value of the
  // key contains the needle" is then the device dictionary pass's "any dictionary value
  // matched", and the host does not scan the values (24 ms per query on config 4)
  std::vector<uint8_t> hdr_defer;
  uint64_t n = 0;
  std::vector<uint32_t> page_entries;  // EntriesLength per page
  std::vector<uint64_t> page_fb_bytes; // flatbuffer bytes per page (bytesInspected)
  std::vector<uint64_t> page_first;    // scan position of each page's first entry
  uint64_t fb_bytes = 0;
  // per entry (scan order)
  std::vector<uint8_t> ids;     // n * 16, right aligned
  std::vector<uint8_t> id_len;  // n
  std::vector<uint64_t> start, end;
  std::vector<uint32_t> svc_vid, name_vid;  // Value(0) of root.service.name / root.name
  int svc_key = -1, name_key = -1;
  std::vector<KeyColumn> keys;
  std::unordered_map<std::string, int> key_index;

  std::string_view dict_value(int key, uint32_t vid) const {
    const KeyColumn &k = keys[size_t(key)];
    return {reinterpret_cast<const char *>(k.dict_bytes.data() + k.dict_off[vid]), k.dict_off[vid + 1] - k.dict_off[vid]};
  }
};

// Dictionaries above this size take MatchesBlock's tag test from the device (hdr_defer).
constexpr uint64_t kDeferMinBytes = 1u << 20;
// Fills hdr_defer (block.cpp): a large key's header values are exactly its dictionary values
// (equal counts; each header value found byte for byte, no dictionary value twice), checked on
// up to nthreads threads.
void verify_header_dicts(HostBlock &hb, int nthreads);

// Reads + decodes a block (meta missing -> has_meta=false, TSG_OK). nthreads <= 0: all cores.
// first_page / npages: only those index records (npages UINT32_MAX = to the end).
void decode_search_block(const uint8_t *meta, size_t meta_len, bool meta_present, Bytes header,
                         const uint8_t *index, size_t index_len, const uint8_t *data, size_t data_len, int nthreads,
                         HostBlock &out, uint32_t first_page = 0, uint32_t npages = 0xFFFFFFFFu);

// newStreamingSearchBlockFromWALReplay + the deduping iterator of its Search
// (tempodb/search/rescan_blocks.go:74-107, tempodb/wal/replay.go:15-71,
// streaming_search_block.go:118-175, iterator_deduping.go, data_combiner.go):
// pages replayed in file order (header AddEntry per page), records sorted by id,
// equal ids combined, each resulting entry one scan position whose bytesInspected
// is its object length.
void decode_wal_search_block(const uint8_t *file, size_t len, int enc, HostBlock &out);
// Live traces: segment i = bytes[seg_off[i], seg_off[i+1]) (a SearchEntry flatbuffer as the
// distributor wrote it), trace t = segments [trace_seg[t], trace_seg[t+1]). Every segment is
// one row (its own Matches, pitfall P3 resolved per table as for WAL entries).
void decode_live_block(const uint8_t *bytes, const uint64_t *seg_off, uint64_t nsegs, const uint64_t *trace_seg,
                       uint32_t ntraces, HostBlock &out);
// wal.ParseFilename (tempodb/wal/wal.go:179-219): blockID:tenant:version:encoding[:dataEncoding]
int parse_wal_filename(const std::string &name, std::string &version);

}  // namespace tsg
