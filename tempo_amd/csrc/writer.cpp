// writer.cpp — search-block and v2 trace-block writers (tooling for synthetic
// data and test fixtures; not on the search path).
//
// Restates, in order of the call chain:
//   NewBackendSearchBlock          tempodb/search/backend_search_block.go:28-129
//   backendSearchBlockWriter       tempodb/search/backend_search_block_writer.go:17-101
//   BufferedAppenderGeneric        tempodb/encoding/v2/appender_buffered_generic.go:11-97
//   SearchPageBuilder              pkg/tempofb/search_page_builder.go:5-66
//   SearchEntryMutable.WriteToBuilder pkg/tempofb/search_entry_mutable.go:48-60
//   WriteSearchDataMap/writeKeyValues pkg/tempofb/searchdatamap.go:71-152
//   SearchBlockHeaderMutable       pkg/tempofb/SearchBlockHeader_util.go:13-75
//   dataWriter / object / page     tempodb/encoding/v2/data_writer.go:25-93, object.go:25-48, page.go:110-146
//   indexWriter                    tempodb/encoding/v2/index_writer.go:25-77
//   StreamingBlock (v2 data, bloom, meta) tempodb/encoding/v2/streaming_block.go, common/bloom.go
#include "writer.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <ctime>
#include <map>
#include <set>
#include <type_traits>
#include <unordered_map>

#include "common.hpp"
#include "fbbuilder.hpp"

namespace tsg {

// ---- SearchDataMap / writeKeyValues -------------------------------------------
template <class Values>
static uint32_t write_key_values(FBBuilder &b, const std::string &key_in, const Values &vals_in,
                                 std::unordered_map<uint64_t, uint32_t> *cache) {
  if (vals_in.empty()) return 0;  // searchdatamap.go:104-106
  std::string key = go_to_lower(key_in);
  std::vector<std::string> values;
  values.reserve(vals_in.size());
  for (auto &v : vals_in) values.push_back(go_to_lower(v));
  std::sort(values.begin(), values.end());
  uint64_t ce = 0;
  if (cache) {
    XXH64Stream h;
    h.write(key.data(), key.size());
    for (auto &v : values) {
      uint8_t z = 0;
      h.write(&z, 1);
      h.write(v.data(), v.size());
    }
    ce = h.sum();
    auto it = cache->find(ce);
    if (it != cache->end()) return it->second;
  }
  uint32_t ko = b.create_shared_string(key);
  std::vector<uint32_t> vs(values.size());
  for (size_t i = 0; i < values.size(); i++) vs[i] = b.create_shared_string(values[i]);
  b.start_vector(4, vs.size(), 4);  // KeyValuesStartValueVector
  for (uint32_t o : vs) b.prepend_uoffset(o);
  uint32_t vv = b.end_vector(vs.size());
  b.start_object(2);  // KeyValuesStart
  b.prepend_uoffset_slot(0, ko, 0);
  b.prepend_uoffset_slot(1, vv, 0);
  uint32_t off = b.end_object();
  if (cache) (*cache)[ce] = off;
  return off;
}

template <class Map>
static uint32_t write_search_data_map(FBBuilder &b, const Map &d, std::unordered_map<uint64_t, uint32_t> *cache) {
  // keys sorted bytewise like sort.Strings (a std::map already is; a rollup is sorted here)
  std::vector<const typename Map::value_type *> kvs;
  kvs.reserve(d.size());
  for (auto &kv : d) kvs.push_back(&kv);
  if (!std::is_same<Map, TagMap>::value)
    std::sort(kvs.begin(), kvs.end(), [](auto *a, auto *b) { return a->first < b->first; });
  std::vector<uint32_t> offs;
  offs.reserve(d.size());
  for (auto *kv : kvs) offs.push_back(write_key_values(b, kv->first, kv->second, cache));
  b.start_vector(4, offs.size(), 4);  // SearchEntryStartTagsVector
  for (uint32_t o : offs) b.prepend_uoffset(o);
  return b.end_vector(offs.size());
}

static uint32_t write_entry(FBBuilder &b, const SearchEntryIn &e, std::unordered_map<uint64_t, uint32_t> *cache) {
  // SearchEntryMutable.WriteToBuilder: CreateByteString(id), tags, start/end, tags
  uint32_t ido;
  {
    std::string_view id(reinterpret_cast<const char *>(e.id.data()), e.id.size());
    ido = b.create_string(id);
  }
  uint32_t to = write_search_data_map(b, e.tags, cache);
  b.start_object(4);
  b.prepend_uoffset_slot(0, ido, 0);
  b.prepend_u64_slot(2, e.start, 0);
  b.prepend_u64_slot(3, e.end, 0);
  b.prepend_uoffset_slot(1, to, 0);
  return b.end_object();
}

std::vector<uint8_t> fb_search_entry_bytes(const SearchEntryIn &e) {
  FBBuilder b(2048);
  uint32_t off = write_entry(b, e, nullptr);
  b.finish(off);
  return b.finished_bytes();
}

// SearchBlockHeaderMutable
void HeaderBuilder::add_entry(const SearchEntryIn &e) {
  for (auto &kv : e.tags)
    for (auto &v : kv.second) tags[kv.first].insert(v);
  uint64_t dur = e.end - e.start;
  if (min_dur == 0 || dur < min_dur) min_dur = dur;  // SearchBlockHeader_util.go:37-40 (quirk P1)
  if (dur > max_dur) max_dur = dur;
}
std::vector<uint8_t> HeaderBuilder::to_bytes() const {
  FBBuilder b(1024);
  uint32_t t = write_search_data_map(b, tags, nullptr);
  b.start_object(3);
  b.prepend_u64_slot(1, min_dur, 0);
  b.prepend_u64_slot(2, max_dur, 0);
  b.prepend_uoffset_slot(0, t, 0);
  uint32_t o = b.end_object();
  b.finish(o);
  return b.finished_bytes();
}

// ---- v2 data pages ------------------------------------------------------------
// object: [u32 totalLength][u32 idLength][id][obj] (object.go:25-48)
static void marshal_object(std::vector<uint8_t> &o, const uint8_t *id, size_t idl, const uint8_t *obj, size_t n) {
  put_le32(o, uint32_t(n + idl + 8));
  put_le32(o, uint32_t(idl));
  o.insert(o.end(), id, id + idl);
  o.insert(o.end(), obj, obj + n);
}
// CutPage: compress the object buffer, page = [u32 total][u16 0][payload] (page.go:110-146)
static size_t cut_data_page(std::vector<uint8_t> &file, const std::vector<uint8_t> &objects, int enc) {
  std::vector<uint8_t> payload;
  if (enc == 6) snappy_framed_encode(objects.data(), objects.size(), payload);
  else if (enc == 0) payload = objects;
  else fail(TSG_E_UNSUPPORTED_ENCODING, std::string("writer: unsupported encoding ") + encoding_name(enc));
  uint32_t total = uint32_t(payload.size() + 6);
  put_le32(file, total);
  put_le16(file, 0);
  file.insert(file.end(), payload.begin(), payload.end());
  return total;
}

// StreamingSearchBlock.Append per entry (streaming_search_block.go:80-95): one
// SearchEntry flatbuffer per page, the page's object keyed by the entry's id, pages in
// append order (v2.Appender: Write + CutPage).
void write_wal_search(const std::string &path, const std::vector<SearchEntryIn> &entries, int enc) {
  std::vector<uint8_t> file, obj;
  for (const auto &e : entries) {
    const std::vector<uint8_t> fb = fb_search_entry_bytes(e);
    obj.clear();
    marshal_object(obj, e.id.data(), e.id.size(), fb.data(), fb.size());
    cut_data_page(file, obj, enc);
  }
  FILE *f = std::fopen(path.c_str(), "wb");
  if (!f) fail(TSG_E_IO, "cannot create " + path);
  const size_t w = file.empty() ? 0 : std::fwrite(file.data(), 1, file.size(), f);
  std::fclose(f);
  if (w != file.size()) fail(TSG_E_IO, "short write " + path);
}

struct Record {
  std::vector<uint8_t> id;
  uint64_t start = 0;
  uint32_t length = 0;
};

// indexWriter.Write (index_writer.go:25-77)
static std::vector<uint8_t> write_index(const std::vector<Record> &recs, uint32_t page_size) {
  size_t rpp = (page_size - 8 - 6) / 28;
  if (rpp == 0) fail(TSG_E_INVALID, "index page too small");
  size_t pages = (recs.size() + rpp - 1) / rpp;
  std::vector<uint8_t> out(pages * page_size, 0);
  for (size_t p = 0; p < pages; p++) {
    uint8_t *pg = out.data() + p * page_size;
    uint8_t *data = pg + 14;
    size_t n = std::min(rpp, recs.size() - p * rpp);
    for (size_t i = 0; i < n; i++) {
      const Record &r = recs[p * rpp + i];
      if (r.id.size() != 16) fail(TSG_E_INVALID, "ids must be 128 bit");  // MarshalRecordsToBuffer
      std::memcpy(data + 28 * i, r.id.data(), 16);
      std::memcpy(data + 28 * i + 16, &r.start, 8);
      std::memcpy(data + 28 * i + 24, &r.length, 4);
    }
    uint64_t cs = xxhash64(data, page_size - 14);
    uint32_t tl = page_size;
    uint16_t hl = 8;
    std::memcpy(pg, &tl, 4);
    std::memcpy(pg + 4, &hl, 2);
    std::memcpy(pg + 6, &cs, 8);
  }
  return out;
}

// ---- NewBackendSearchBlock ----------------------------------------------------------
struct SearchBlockWriter::Impl {
  std::string dir;
  int enc;
  uint32_t page_size;
  HeaderBuilder header;
  FBBuilder b{1024};
  TagRollup all_tags;
  std::vector<uint32_t> page_entries;
  std::unordered_map<uint64_t, uint32_t> kvcache;
  std::vector<uint8_t> file;
  std::vector<Record> records;
  Record cur;
  bool have_cur = false;
  uint64_t cur_offset = 0;
  long cur_bytes = 0;
  std::vector<uint8_t> last_id;
  bool any = false;

  size_t cut_page() {
    // SearchPageBuilder.Finish (search_page_builder.go:35-59)
    b.start_vector(4, page_entries.size(), 4);
    for (uint32_t e : page_entries) b.prepend_uoffset(e);
    uint32_t ev = b.end_vector(page_entries.size());
    uint32_t to = write_search_data_map(b, all_tags, &kvcache);
    b.start_object(2);
    b.prepend_uoffset_slot(1, ev, 0);
    b.prepend_uoffset_slot(0, to, 0);
    uint32_t root = b.end_object();
    b.finish(root);
    // dw.Write(uuid.Nil[:], buf) + dw.CutPage (backend_search_block_writer.go:67-80)
    std::vector<uint8_t> obj;
    static const uint8_t nil_id[16] = {0};
    marshal_object(obj, nil_id, 16, b.data(), b.size());
    size_t flushed = cut_data_page(file, obj, enc);
    // SearchPageBuilder.Reset
    b.reset();
    page_entries.clear();
    all_tags.clear();
    kvcache.clear();
    return flushed;
  }
  void flush() {  // BufferedAppenderGeneric.flush (appender_buffered_generic.go:78-97)
    if (!have_cur) return;
    size_t n = cut_page();
    cur_offset += n;
    cur.length += uint32_t(n);
    records.push_back(cur);
    have_cur = false;
    cur_bytes = 0;
  }
};

SearchBlockWriter::SearchBlockWriter(const std::string &dir, int enc, uint32_t page_size) : p_(new Impl) {
  if (enc != 0 && enc != 6) fail(TSG_E_UNSUPPORTED_ENCODING, "writer supports none/snappy");
  p_->dir = dir;
  p_->enc = enc;
  p_->page_size = page_size ? page_size : 2 * 1024 * 1024;  // defaultBackendSearchBlockPageSize
}
SearchBlockWriter::~SearchBlockWriter() { delete p_; }

void SearchBlockWriter::append(const SearchEntryIn &e) {
  Impl &w = *p_;
  if (w.any && bytes_compare(e.id.data(), e.id.size(), w.last_id.data(), w.last_id.size()) <= 0)
    fail(TSG_E_INVALID, "writer input must be strictly ascending by trace id");
  w.any = true;
  w.last_id = e.id;
  w.header.add_entry(e);
  // SearchPageBuilder.AddData (search_page_builder.go:20-33)
  for (auto &kv : e.tags)
    for (auto &v : kv.second) w.all_tags[kv.first].insert(v);
  uint32_t old = w.b.offset();
  uint32_t off = write_entry(w.b, e, &w.kvcache);
  w.page_entries.push_back(off);
  long written = long(off) - long(old);
  // BufferedAppenderGeneric.Append (appender_buffered_generic.go:38-61)
  if (!w.have_cur) {
    w.cur = Record();
    w.cur.start = w.cur_offset;
    w.have_cur = true;
  }
  w.cur_bytes += written;
  w.cur.id = e.id;
  if (w.cur_bytes > long(w.page_size)) w.flush();
}

void SearchBlockWriter::finish() {
  Impl &w = *p_;
  w.flush();
  std::vector<uint8_t> index = write_index(w.records, 100 * 1024);
  std::vector<uint8_t> hb = w.header.to_bytes();
  char meta[256];
  std::snprintf(meta, sizeof meta, "{\"version\":\"v2\",\"encoding\":\"%s\",\"indexPageSize\":%u,\"indexRecords\":%zu}",
                encoding_name(w.enc), 100u * 1024u, w.records.size());
  make_dirs(w.dir);
  write_file(w.dir + "/search", w.file.data(), w.file.size());
  write_file(w.dir + "/search-index", index.data(), index.size());
  write_file(w.dir + "/search-header", hb.data(), hb.size());
  write_file(w.dir + "/search.meta.json", reinterpret_cast<const uint8_t *>(meta), std::strlen(meta));
}

void write_search_block(const std::string &dir, std::vector<SearchEntryIn> entries, int enc, uint32_t page_size) {
  // streaming block iterator order: ascending id, deduped (iterator_deduping.go)
  std::sort(entries.begin(), entries.end(), [](const SearchEntryIn &a, const SearchEntryIn &b) {
    return bytes_compare(a.id.data(), a.id.size(), b.id.data(), b.id.size()) < 0;
  });
  SearchBlockWriter w(dir, enc, page_size);
  for (auto &e : entries) w.append(e);
  w.finish();
}

// ---- entry wire format --------------------------------------------------------
std::vector<SearchEntryIn> parse_entries(const uint8_t *p, size_t n) {
  std::vector<SearchEntryIn> out;
  size_t i = 0;
  auto need = [&](size_t k) {
    if (n - i < k) fail(TSG_E_INVALID, "entry list truncated");
  };
  while (i < n) {
    SearchEntryIn e;
    need(4);
    uint32_t idl = le32(p + i);
    i += 4;
    need(idl);
    e.id.assign(p + i, p + i + idl);
    i += idl;
    need(20);
    e.start = le64(p + i);
    e.end = le64(p + i + 8);
    uint32_t nt = le32(p + i + 16);
    i += 20;
    for (uint32_t t = 0; t < nt; t++) {
      need(4);
      uint32_t kl = le32(p + i);
      i += 4;
      need(kl);
      std::string k(reinterpret_cast<const char *>(p + i), kl);
      i += kl;
      need(4);
      uint32_t vl = le32(p + i);
      i += 4;
      need(vl);
      std::string v(reinterpret_cast<const char *>(p + i), vl);
      i += vl;
      e.tags[k].insert(v);  // SearchEntryMutable.AddTag
    }
    out.push_back(std::move(e));
  }
  return out;
}

// ---- v2 trace block (StreamingBlock.AddObject/Complete, NewBloom) ------------------
void bloom_estimate(uint64_t n, double fp, uint64_t &m, uint64_t &k) {
  // willf/bloom EstimateParameters (bloom.go:120-124)
  m = uint64_t(std::ceil(-1.0 * double(n) * std::log(fp) / std::pow(std::log(2.0), 2.0)));
  k = uint64_t(std::ceil(std::log(2.0) * double(m) / double(n)));
}
uint32_t bloom_shard_count(double fp, uint64_t shard_size, uint64_t n) {
  uint64_t m, k;
  bloom_estimate(n, fp, m, k);
  double sc = std::ceil(double(m) / (double(shard_size) * 8.0));  // common/bloom.go:30-31
  uint64_t c = uint64_t(sc);
  if (c < 1) c = 1;
  if (c > 1000) c = 1000;
  return uint32_t(c);
}

static std::string b64(const uint8_t *p, size_t n) {
  static const char *T = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string o;
  for (size_t i = 0; i < n; i += 3) {
    uint32_t v = uint32_t(p[i]) << 16;
    if (i + 1 < n) v |= uint32_t(p[i + 1]) << 8;
    if (i + 2 < n) v |= p[i + 2];
    o.push_back(T[(v >> 18) & 63]);
    o.push_back(T[(v >> 12) & 63]);
    o.push_back(i + 1 < n ? T[(v >> 6) & 63] : '=');
    o.push_back(i + 2 < n ? T[v & 63] : '=');
  }
  return o;
}

void write_v2_block(const std::string &dir, const uint8_t (*ids)[16], const std::vector<std::vector<uint8_t>> &objs,
                    uint64_t n, const V2Params &prm) {
  // bloom
  uint64_t m, k;
  bloom_estimate(n ? n : 1, prm.bloom_fp, m, k);
  uint32_t shards = bloom_shard_count(prm.bloom_fp, prm.bloom_shard_bytes, n ? n : 1);
  uint64_t sm = prm.bloom_shard_bytes * 8;  // bloom.New(shardSize*8, k)
  if (k < 1) k = 1;
  uint64_t words = (sm + 63) / 64;
  std::vector<std::vector<uint64_t>> bits(shards, std::vector<uint64_t>(words, 0));
  // data pages (bufferedAppender, indexDownsample)
  std::vector<uint8_t> file, objbuf;
  std::vector<Record> records;
  Record cur;
  bool have = false;
  uint64_t off = 0;
  long cb = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t *id = ids[i];
    size_t before = objbuf.size();
    const auto &o = objs[i % objs.size()];
    marshal_object(objbuf, id, 16, o.data(), o.size());
    long written = long(objbuf.size() - before);
    if (!have) {
      cur = Record();
      cur.start = off;
      have = true;
    }
    cb += written;
    cur.id.assign(id, id + 16);
    if (cb > long(prm.index_downsample_bytes)) {
      size_t f = cut_data_page(file, objbuf, prm.encoding);
      objbuf.clear();
      off += f;
      cur.length += uint32_t(f);
      records.push_back(cur);
      have = false;
      cb = 0;
    }
    // bloom.Add (bloom.go:~140): shard by FNV-1, k locations of the murmur3 base hashes
    uint32_t s = fnv1_32(id, 16) % shards;
    uint64_t h[4];
    murmur3_128(id, 16, h[0], h[1]);
    uint8_t tmp[17];
    std::memcpy(tmp, id, 16);
    tmp[16] = 1;
    murmur3_128(tmp, 17, h[2], h[3]);
    for (uint64_t j = 0; j < k; j++) {
      uint64_t loc = (h[j % 2] + j * h[2 + (((j + (j % 2)) % 4) / 2)]) % sm;
      bits[s][loc >> 6] |= 1ULL << (loc & 63);
    }
  }
  if (have) {
    size_t f = cut_data_page(file, objbuf, prm.encoding);
    off += f;
    cur.length += uint32_t(f);
    records.push_back(cur);
  }
  std::vector<uint8_t> index = write_index(records, prm.index_page_bytes);
  make_dirs(dir);
  write_file(dir + "/data", file.data(), file.size());
  write_file(dir + "/index", index.data(), index.size());
  for (uint32_t s = 0; s < shards; s++) {
    std::vector<uint8_t> bb;
    put_be64(bb, sm);
    put_be64(bb, k);
    put_be64(bb, sm);
    for (uint64_t w : bits[s]) put_be64(bb, w);
    char name[32];
    std::snprintf(name, sizeof name, "/bloom-%u", s);
    write_file(dir + name, bb.data(), bb.size());
  }
  // meta.json (backend.BlockMeta)
  std::string min_id = n ? b64(ids[0], 16) : "", max_id = n ? b64(ids[n - 1], 16) : "";
  auto fmt_time = [](int64_t t) {
    time_t tt = time_t(t);
    struct tm g;
    gmtime_r(&tt, &g);
    char b[64];
    std::strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%SZ", &g);
    return std::string(b);
  };
  char bid[40];
  const uint8_t *u = prm.block_id;
  std::snprintf(bid, sizeof bid, "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", u[0], u[1],
                u[2], u[3], u[4], u[5], u[6], u[7], u[8], u[9], u[10], u[11], u[12], u[13], u[14], u[15]);
  std::string meta = std::string("{\"format\":\"v2\",\"blockID\":\"") + bid + "\",\"minID\":\"" + min_id +
                     "\",\"maxID\":\"" + max_id + "\",\"tenantID\":\"single-tenant\",\"startTime\":\"" +
                     fmt_time(prm.start_unix) + "\",\"endTime\":\"" + fmt_time(prm.end_unix) +
                     "\",\"totalObjects\":" + std::to_string(n) + ",\"size\":" + std::to_string(file.size()) +
                     ",\"compactionLevel\":0,\"encoding\":\"" + encoding_name(prm.encoding) +
                     "\",\"indexPageSize\":" + std::to_string(prm.index_page_bytes) +
                     ",\"totalRecords\":" + std::to_string(records.size()) +
                     ",\"dataEncoding\":\"" + prm.data_encoding + "\",\"bloomShards\":" + std::to_string(shards) + "}";
  write_file(dir + "/meta.json", reinterpret_cast<const uint8_t *>(meta.data()), meta.size());
}

}  // namespace tsg
