// block.cpp — read side of the on-disk formats and the host half of the columnar
// loader. Each data page is decoded exactly once (parallel over pages); the
// flatbuffer is walked once per distinct KeyValues table (tables are shared
// between entries of a page by writeKeyValues' cache, searchdatamap.go:115-128).
#include "block.hpp"

#include <algorithm>
#include <cctype>

#include "writer.hpp"
#include <atomic>
#include <chrono>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>

namespace tsg {

// ---- ContainsTag ------------------------------------------------------------------
bool fb_contains_tag(const FbTable &t, uint16_t tags_vto, std::string_view k, std::string_view v) {
  uint16_t o = t.field(tags_vto);
  uint32_t n = o ? t.vector_len(o) : 0;
  uint32_t start = o ? t.vector_start(o) : 0;
  uint32_t i = 0, j = n;
  FbTable kv{t.b, t.n, 0};
  bool found = false;
  while (i < j) {  // binarySearch with the reversed comparator (searchdata_util.go:63-100)
    uint32_t h = (i + j) >> 1;
    kv.pos = t.indirect(start + 4 * h);
    uint16_t ko = kv.field(kKvKey);
    std::string_view key = ko ? kv.byte_vector(kv.pos + ko) : std::string_view();
    int c = bytes_compare(reinterpret_cast<const uint8_t *>(key.data()), key.size(),
                          reinterpret_cast<const uint8_t *>(k.data()), k.size());
    if (c == 0) {
      found = true;
      break;
    }
    if (c < 0) j = h;
    else i = h + 1;
  }
  if (!found) return false;
  uint16_t vo = kv.field(kKvValue);
  if (!vo) return false;
  uint32_t vn = kv.vector_len(vo), vs = kv.vector_start(vo);
  for (uint32_t q = 0; q < vn; q++) {
    std::string_view val = kv.byte_vector(vs + 4 * q);
    if (v.empty() || val.find(v) != std::string_view::npos) return true;  // bytes.Contains
  }
  return false;
}

// The header's tag table as views (the same walk fb_contains_tag does per query).
void index_header(HostBlock &hb) {
  hb.hdr_keys.clear();
  hb.hdr_vals.clear();
  hb.hdr_val0.assign(1, 0);
  hb.hdr_index = false;
  try {
    FbTable t = FbTable::root(hb.header.data(), hb.header.size());
    const uint16_t o = t.field(kHdrTags);
    const uint32_t n = o ? t.vector_len(o) : 0;
    const uint32_t start = o ? t.vector_start(o) : 0;
    FbTable kv{t.b, t.n, 0};
    for (uint32_t h = 0; h < n; h++) {
      kv.pos = t.indirect(start + 4 * h);
      const uint16_t ko = kv.field(kKvKey);
      hb.hdr_keys.push_back(ko ? kv.byte_vector(kv.pos + ko) : std::string_view());
      const uint16_t vo = kv.field(kKvValue);
      if (vo) {
        const uint32_t vn = kv.vector_len(vo), vs = kv.vector_start(vo);
        for (uint32_t q = 0; q < vn; q++) hb.hdr_vals.push_back(kv.byte_vector(vs + 4 * q));
      }
      hb.hdr_val0.push_back(uint32_t(hb.hdr_vals.size()));
    }
    hb.hdr_index = true;
  } catch (...) {
    hb.hdr_keys.clear();
    hb.hdr_vals.clear();
    hb.hdr_val0.assign(1, 0);
  }
}

// ---- meta ---------------------------------------------------------------------------
static bool json_field(std::string_view js, const char *name, std::string_view &val) {
  std::string pat = std::string("\"") + name + "\"";
  size_t p = js.find(pat);
  if (p == std::string_view::npos) return false;
  p += pat.size();
  while (p < js.size() && (js[p] == ' ' || js[p] == ':')) p++;
  size_t e = p;
  if (p < js.size() && js[p] == '"') {
    e = js.find('"', p + 1);
    if (e == std::string_view::npos) return false;
    val = js.substr(p + 1, e - p - 1);
    return true;
  }
  while (e < js.size() && js[e] != ',' && js[e] != '}') e++;
  val = js.substr(p, e - p);
  return true;
}
SearchMeta parse_search_meta(const uint8_t *p, size_t n) {
  std::string_view js(reinterpret_cast<const char *>(p), n), v;
  SearchMeta m;
  if (json_field(js, "version", v)) m.version = std::string(v);
  if (json_field(js, "encoding", v)) m.encoding = parse_encoding(v);
  if (json_field(js, "indexPageSize", v)) m.index_page_size = json_u32(v, "indexPageSize");
  if (json_field(js, "indexRecords", v)) m.index_records = json_u32(v, "indexRecords");
  return m;
}

// ---- v2 pages -------------------------------------------------------------------------
// unmarshalPageFromBytes (page.go:30-57)
static void unmarshal_page(const uint8_t *b, size_t n, size_t hdr_len, const uint8_t *&hdr, const uint8_t *&data,
                           size_t &dlen) {
  if (n < 6 + hdr_len) fail(TSG_E_CORRUPT, "page too small");
  uint32_t total = le32(b);
  uint16_t hl = le16(b + 4);
  if (hl > n - 6) fail(TSG_E_CORRUPT, "page header length out of range");
  if (hl != hdr_len) fail(TSG_E_CORRUPT, "unexpected page header length");
  hdr = b + 6;
  int64_t want = int64_t(total) - int64_t(6 + hdr_len);
  if (want < 0 || uint64_t(want) != n - 6 - hl) fail(TSG_E_CORRUPT, "page length mismatch");
  data = b + 6 + hl;
  dlen = n - 6 - hl;
}

std::vector<IndexRecord> read_index(const uint8_t *p, size_t n, uint32_t page_size, uint32_t total, bool *prefix) {
  std::vector<IndexRecord> out;
  if (prefix) *prefix = false;
  if (total == 0) return out;
  try {
    if (page_size < 14 + 28) fail(TSG_E_CORRUPT, "index page too small for one record");
    uint32_t rpp = (page_size - 8 - 6) / 28;  // objectsPerPage (page.go:175-182)
    out.reserve(total);
    for (uint32_t pidx = 0; uint64_t(pidx) * rpp < total; pidx++) {
      // getPage: ReadAt of one whole page (a short read is an error), framing, checksum
      uint64_t off = uint64_t(pidx) * page_size;
      if (off + page_size > n) fail(TSG_E_CORRUPT, "index truncated");
      const uint8_t *hdr, *data;
      size_t dlen;
      unmarshal_page(p + off, page_size, 8, hdr, data, dlen);
      if (le64(hdr) != xxhash64(data, dlen)) fail(TSG_E_CORRUPT, "mismatched index page checksum");
      for (uint32_t r = 0; r < rpp && uint64_t(pidx) * rpp + r < total; r++) {
        if ((r + 1) * 28 > dlen) fail(TSG_E_CORRUPT, "index record out of bounds");
        const uint8_t *rec = data + r * 28;
        bool zero = true;
        for (int k = 0; k < 28 && zero; k++) zero = rec[k] == 0;
        if (zero) fail(TSG_E_CORRUPT, "unexpected zero value index record");
        IndexRecord ir;
        std::memcpy(ir.id, rec, 16);
        ir.start = le64(rec + 16);
        ir.length = le32(rec + 24);
        out.push_back(ir);
      }
    }
  } catch (const Error &) {
    if (!prefix) throw;
    *prefix = true;  // At(i) failed: the records before i are what Search visits
  }
  return out;
}

void read_data_page(const uint8_t *file, size_t flen, const IndexRecord &r, int enc, std::vector<uint8_t> &out) {
  if (r.start + r.length > flen) fail(TSG_E_CORRUPT, "record out of bounds of data file");
  const uint8_t *hdr, *payload;
  size_t pl;
  unmarshal_page(file + r.start, r.length, 0, hdr, payload, pl);
  if (enc == 0) out.assign(payload, payload + pl);
  else if (enc == 6) snappy_framed_decode(payload, pl, out);
  else if (enc == 7) {
    const int st = zstd_host_decode(payload, pl, out);
    if (st != TSG_OK) fail(st, "zstd page decode failed");
  } else fail(TSG_E_UNSUPPORTED_ENCODING, std::string("unsupported page encoding ") + encoding_name(enc));
}

// ---- page parse ---------------------------------------------------------------------------
namespace {
struct PageKV {
  std::string_view key;
  std::vector<std::string_view> vals;
};
struct PageParse {
  std::vector<uint8_t> buf;
  uint64_t fb_bytes = 0;
  uint32_t nentries = 0;
  std::vector<PageKV> kvs;
  std::vector<uint32_t> id_off;  // into buf
  std::vector<uint8_t> id_len;
  std::vector<uint64_t> start, end;
  std::vector<uint32_t> tag_begin;  // nentries + 1
  std::vector<uint32_t> tag_kv;     // the entry's KeyValues tables, vector order (SearchEntry.Get)
  std::vector<uint32_t> tag_res;    // per table: the table FindTag(its key) lands on, or kNone
  int err = 0;
  std::string msg;
};

// One SearchEntry table -> pp (id, times, tag tables). Which table a term on key k
// reads is what FindTag's binarySearch over this entry's vector finds for k
// (searchdata_util.go:63-100), resolved here once per table: for keys unique and
// strictly descending (backend blocks, pitfall P3) that is the table itself; WAL
// entries written from mixed-case keys may be out of order or repeat a key, and then
// a key can resolve to another table with the same key, or to none (the reference's
// search misses it). Exact-key lookup of the resolved table is then the reference.
void parse_entry(const FbTable &e, const uint8_t *fb, uint32_t fb_base, PageParse &pp,
                 std::unordered_map<uint32_t, uint32_t> &memo) {
  FbTable kv{e.b, e.n, 0};
  uint16_t io = e.field(kEntryId);
  std::string_view id = io ? e.byte_vector(e.pos + io) : std::string_view();
  if (id.size() > 16) fail(TSG_E_UNSUPPORTED, "trace id longer than 16 bytes");
  pp.id_off.push_back(uint32_t(reinterpret_cast<const uint8_t *>(id.data()) - fb) + fb_base);
  pp.id_len.push_back(uint8_t(id.size()));
  pp.start.push_back(e.u64(kEntryStart));
  pp.end.push_back(e.u64(kEntryEnd));
  uint16_t to = e.field(kEntryTags);
  uint32_t nt = to ? e.vector_len(to) : 0, ts = to ? e.vector_start(to) : 0;
  const size_t t0 = pp.tag_kv.size();
  bool ordered = true;
  for (uint32_t t = 0; t < nt; t++) {
    uint32_t pos = e.indirect(ts + 4 * t);
    auto it = memo.find(pos);
    uint32_t idx;
    if (it == memo.end()) {
      kv.pos = pos;
      PageKV p;
      uint16_t ko = kv.field(kKvKey);
      p.key = ko ? kv.byte_vector(kv.pos + ko) : std::string_view();
      uint16_t vo = kv.field(kKvValue);
      uint32_t vn = vo ? kv.vector_len(vo) : 0, vs = vo ? kv.vector_start(vo) : 0;
      p.vals.reserve(vn);
      for (uint32_t q = 0; q < vn; q++) p.vals.push_back(kv.byte_vector(vs + 4 * q));
      idx = uint32_t(pp.kvs.size());
      pp.kvs.push_back(std::move(p));
      memo.emplace(pos, idx);
    } else {
      idx = it->second;
    }
    if (t > 0 && !(pp.kvs[pp.tag_kv.back()].key > pp.kvs[idx].key)) ordered = false;
    pp.tag_kv.push_back(idx);
  }
  for (uint32_t t = 0; t < nt; t++) {
    if (ordered) {
      pp.tag_res.push_back(pp.tag_kv[t0 + t]);
      continue;
    }
    const std::string_view k = pp.kvs[pp.tag_kv[t0 + t]].key;
    uint32_t i = 0, j = nt, found = kNone;
    while (i < j) {
      const uint32_t h = (i + j) >> 1;
      const std::string_view hk = pp.kvs[pp.tag_kv[t0 + h]].key;
      const int c = bytes_compare(reinterpret_cast<const uint8_t *>(hk.data()), hk.size(),
                                  reinterpret_cast<const uint8_t *>(k.data()), k.size());
      if (c == 0) {
        found = pp.tag_kv[t0 + h];
        break;
      }
      if (c < 0) j = h;
      else i = h + 1;
    }
    pp.tag_res.push_back(found);
  }
  pp.tag_begin.push_back(uint32_t(pp.tag_kv.size()));
}

struct KeyBuild {
  std::unordered_map<std::string, uint32_t> vmap;
  std::unordered_map<std::string, uint32_t> smap;
};
}  // namespace


// Appends one parsed page to the block: its KeyValues tables resolved to (key, value
// set) ids, then its entries' columns (scan order = pages ascending, entry index ascending).
static void merge_page(HostBlock &hb, std::vector<KeyBuild> &kb, PageParse &pp) {
  uint64_t base = hb.n;
  hb.page_entries.push_back(pp.nentries);
  hb.page_fb_bytes.push_back(pp.fb_bytes);
  hb.page_first.push_back(base);
  hb.fb_bytes += pp.fb_bytes;
  // resolve the page's KeyValues tables to (key, set)
  std::vector<std::pair<int, uint32_t>> res(pp.kvs.size());
  for (size_t q = 0; q < pp.kvs.size(); q++) {
    const PageKV &p = pp.kvs[q];
    std::string key(p.key);
    auto ki = hb.key_index.find(key);
    int k;
    if (ki == hb.key_index.end()) {
      k = int(hb.keys.size());
      hb.key_index.emplace(key, k);
      KeyColumn kc;
      kc.name = key;
      kc.dict_off.push_back(0);
      kc.set_off.push_back(0);
      hb.keys.push_back(std::move(kc));
      kb.emplace_back();
      if (key == "root.service.name") hb.svc_key = k;
      if (key == "root.name") hb.name_key = k;
    } else {
      k = ki->second;
    }
    KeyColumn &kc = hb.keys[size_t(k)];
    KeyBuild &b = kb[size_t(k)];
    std::string skey;
    skey.reserve(4 * p.vals.size());
    uint32_t first_vid = kNone;
    for (auto &v : p.vals) {
      std::string vs(v);
      auto vi = b.vmap.find(vs);
      uint32_t vid;
      if (vi == b.vmap.end()) {
        vid = kc.nvals();
        kc.dict_bytes.insert(kc.dict_bytes.end(), v.begin(), v.end());
        kc.dict_off.push_back(uint32_t(kc.dict_bytes.size()));
        if (kc.dict_bytes.size() > 0xF0000000u) fail(TSG_E_UNSUPPORTED, "dictionary too large");
        b.vmap.emplace(std::move(vs), vid);
      } else {
        vid = vi->second;
      }
      if (first_vid == kNone) first_vid = vid;
      skey.append(reinterpret_cast<const char *>(&vid), 4);
    }
    auto si = b.smap.find(skey);
    uint32_t sid;
    if (si == b.smap.end()) {
      sid = kc.nsets();
      for (auto &v : p.vals) kc.set_vals.push_back(b.vmap[std::string(v)]);
      kc.set_off.push_back(uint32_t(kc.set_vals.size()));
      if (p.vals.size() != 1 || sid != first_vid) kc.identity = false;
      b.smap.emplace(std::move(skey), sid);
    } else {
      sid = si->second;
    }
    res[q] = {k, sid};
  }
  // entries
  uint64_t n1 = base + pp.nentries;
  for (auto &kc : hb.keys) kc.col.resize(n1, kNone);
  hb.ids.resize(n1 * 16, 0);
  hb.id_len.resize(n1);
  hb.start.resize(n1);
  hb.end.resize(n1);
  hb.svc_vid.resize(n1, kNone);
  hb.name_vid.resize(n1, kNone);
  for (uint32_t j = 0; j < pp.nentries; j++) {
    uint64_t e = base + j;
    uint8_t il = pp.id_len[j];
    std::memcpy(&hb.ids[e * 16 + 16 - il], pp.buf.data() + pp.id_off[j], il);
    hb.id_len[e] = il;
    hb.start[e] = pp.start[j];
    hb.end[e] = pp.end[j];
    bool svc_done = false, name_done = false;
    for (uint32_t t = pp.tag_begin[j]; t < pp.tag_begin[j + 1]; t++) {
      auto [k, sid] = res[pp.tag_kv[t]];
      KeyColumn &kc = hb.keys[size_t(k)];
      if (pp.tag_res[t] != kNone) kc.col[e] = res[pp.tag_res[t]].second;
      // SearchEntry.Get: first key match in vector order, Value(0) (searchdata_util.go:10-23)
      if (k == hb.svc_key && !svc_done) {
        svc_done = true;
        if (kc.set_off[sid + 1] > kc.set_off[sid]) hb.svc_vid[e] = kc.set_vals[kc.set_off[sid]];
      }
      if (k == hb.name_key && !name_done) {
        name_done = true;
        if (kc.set_off[sid + 1] > kc.set_off[sid]) hb.name_vid[e] = kc.set_vals[kc.set_off[sid]];
      }
    }
  }
  hb.n = n1;
}

// Narrow keys (fewer than 255 value sets: one-byte columns) get a canonical numbering:
// values in byte order, value sets in order of their (renumbered) value lists. Blocks
// holding the same values for a key then hold byte-identical dictionaries, which the
// engine interns once per context and matches once per query on the host (the one-launch
// search path takes the resulting 256-bit set bitmaps in its kernel arguments).
// Ids are internal; scan order, set membership and Value(0) are unchanged.
static void canonicalize_narrow_keys(HostBlock &hb) {
  for (size_t k = 0; k < hb.keys.size(); k++) {
    KeyColumn &kc = hb.keys[k];
    if (kc.width() != 1) continue;
    const uint32_t nv = kc.nvals(), ns = kc.nsets();
    std::vector<uint32_t> vord(nv);
    for (uint32_t i = 0; i < nv; i++) vord[i] = i;
    std::sort(vord.begin(), vord.end(), [&](uint32_t a, uint32_t b) {
      std::string_view x = hb.dict_value(int(k), a), y = hb.dict_value(int(k), b);
      return x < y;
    });
    std::vector<uint32_t> vnew(nv);
    for (uint32_t i = 0; i < nv; i++) vnew[vord[i]] = i;
    Bytes bytes;
    std::vector<uint32_t> off(1, 0);
    for (uint32_t i = 0; i < nv; i++) {
      std::string_view v = hb.dict_value(int(k), vord[i]);
      bytes.insert(bytes.end(), v.begin(), v.end());
      off.push_back(uint32_t(bytes.size()));
    }
    std::vector<std::vector<uint32_t>> sets(ns);
    for (uint32_t sidx = 0; sidx < ns; sidx++)
      for (uint32_t i = kc.set_off[sidx]; i < kc.set_off[sidx + 1]; i++) sets[sidx].push_back(vnew[kc.set_vals[i]]);
    std::vector<uint32_t> sord(ns);
    for (uint32_t i = 0; i < ns; i++) sord[i] = i;
    std::sort(sord.begin(), sord.end(), [&](uint32_t a, uint32_t b) { return sets[a] < sets[b]; });
    std::vector<uint32_t> snew(ns), set_off(1, 0), set_vals;
    for (uint32_t i = 0; i < ns; i++) {
      snew[sord[i]] = i;
      set_vals.insert(set_vals.end(), sets[sord[i]].begin(), sets[sord[i]].end());
      set_off.push_back(uint32_t(set_vals.size()));
    }
    kc.dict_bytes.swap(bytes);
    kc.dict_off.swap(off);
    kc.set_off.swap(set_off);
    kc.set_vals.swap(set_vals);
    for (auto &c : kc.col)
      if (c != kNone) c = snew[c];
    if (int(k) == hb.svc_key)
      for (auto &v : hb.svc_vid)
        if (v != kNone) v = vnew[v];
    if (int(k) == hb.name_key)
      for (auto &v : hb.name_vid)
        if (v != kNone) v = vnew[v];
  }
}

// ---- the columnar loader of a backend block: three parallel phases -------------------
// A. per page (threads over pages): decompress, walk the entries once, collect the page's
//    distinct KeyValues tables (the writer shares a table between the entries of a page,
//    searchdata.go:115-128) with their values' hashes, resolve each entry's FindTag target.
// B. per key (threads over keys): intern the key's values and value sets over the pages in
//    order (first-seen ids), no allocation per value: values are views into the page buffers.
// C. per page again: the entries' columns (ids, times, value-set id per key, root names).
// Keys are numbered in name order. Values, sets and entries keep the scan order (pages
// ascending, entry index ascending); the first damaged page ends the block as in
// BackendSearchBlock.Search (backend_search_block.go:258-266).
namespace {
inline uint64_t hash_bytes(const void *p, size_t n) { return xxhash64(static_cast<const uint8_t *>(p), n); }
inline uint64_t mix_set(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

struct KeyNames {  // provisional key ids, shared by the page workers (a handful of keys)
  std::mutex mu;
  std::vector<std::string> names;
  std::unordered_map<std::string, uint32_t> ids;
  uint32_t get(std::string_view k) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = ids.find(std::string(k));
    if (it != ids.end()) return it->second;
    const uint32_t id = uint32_t(names.size());
    names.emplace_back(k);
    ids.emplace(names.back(), id);
    return id;
  }
};
struct KeyCache {  // per worker: key bytes -> provisional id, no lock once seen
  struct E {
    uint64_t h;
    std::string k;
    uint32_t id;
  };
  std::vector<E> e;
  uint32_t get(KeyNames &kn, std::string_view k) {
    const uint64_t h = hash_bytes(k.data(), k.size());
    for (const auto &x : e)
      if (x.h == h && x.k == k) return x.id;
    const uint32_t id = kn.get(k);
    e.push_back({h, std::string(k), id});
    return id;
  }
};

struct LPage {
  std::vector<uint8_t> buf;
  uint64_t fb_bytes = 0;
  uint32_t n = 0;
  int err = 0;
  std::string msg;
  std::vector<uint32_t> id_off;
  std::vector<uint8_t> id_len;
  std::vector<uint64_t> start, end;
  std::vector<uint32_t> tag0;     // n + 1: entry j's tag references [tag0[j], tag0[j+1])
  std::vector<uint32_t> tag_kv;   // per reference: its own table (SearchEntry.Get walks these)
  std::vector<uint32_t> tag_res;  // per reference: the table FindTag lands on for its key, or kNone
  std::vector<uint32_t> kv_key;   // per distinct table: provisional key id
  std::vector<uint32_t> kv_v0;    // tables + 1: its values [kv_v0[t], kv_v0[t+1]) in vals
  std::vector<std::string_view> vals;
  std::vector<uint64_t> vhash;
  std::vector<uint32_t> vloc;     // phase B: per value reference, its id in its hash shard
  std::vector<uint32_t> kv_sid;   // phase B: the table's value set id within its key
  std::vector<uint64_t> kv_shash; // phase B: a multi-valued table's set hash
  std::vector<uint32_t> bykey, bykey0;  // tables grouped by provisional key (CSR)
  struct KStat {  // per provisional key: its tables in this page, their values and value bytes
    uint64_t tables = 0, refs = 0, bytes = 0;
    bool multi = false;  // some table holds no value or several
  };
  std::vector<KStat> kstat;
};

// open addressing: table position -> page-local table index (reset per page)
// A page's tables by their position in the page's flatbuffer: tables start on 4-byte words,
// so position / 4 indexes a direct table (one 8-byte slot per word of the page: {page
// generation, index + 1}; a new page only bumps the generation). A hash of the position had
// scattered the lookups of neighbouring tables over the whole table (a cache miss per tag
// reference); word order keeps an entry's tables, written next to each other, on few lines.
struct PosMap {
  std::vector<uint64_t> slot;
  uint32_t gen = 0;
  void reset(size_t fb_bytes) {
    const size_t need = fb_bytes / 4 + 1;
    if (slot.size() < need) {
      slot.assign(need, 0);
      gen = 0;
    }
    if (++gen == 0) {  // (wrapped: clear once)
      std::fill(slot.begin(), slot.end(), 0);
      gen = 1;
    }
  }
  // index of the table at `pos`, or records `fresh` for it and returns kNone
  uint32_t find_or_put(uint32_t pos, uint32_t fresh) {
    const size_t i = pos >> 2;
    if (i >= slot.size()) fail(TSG_E_CORRUPT, "flatbuffer table position out of range");
    uint64_t &x = slot[i];
    if (uint32_t(x >> 32) == gen) return uint32_t(x) - 1;
    x = (uint64_t(gen) << 32) | (uint64_t(fresh) + 1);
    return kNone;
  }
};

// per worker: the sizes of its previous page (pages of a block are alike: reserving them up
// front saves the vectors' regrowth copies)
struct PageHint {
  size_t tables = 0, vals = 0, refs = 0;
};

void parse_lpage(const uint8_t *data, size_t dlen, int enc, const IndexRecord &rec, KeyNames &kn, KeyCache &kc,
                 PosMap &pm, PageHint &hint, LPage &pp) {
  read_data_page(data, dlen, rec, enc, pp.buf);
  // object.UnmarshalAndAdvanceBuffer (object.go:82-113): [u32 total][u32 idLen][id][obj]
  if (pp.buf.size() < 8) fail(TSG_E_CORRUPT, "object header truncated");
  const uint32_t total = le32(pp.buf.data()), il = le32(pp.buf.data() + 4);
  if (total < 8 || pp.buf.size() - 8 < total - 8 || il > total - 8) fail(TSG_E_CORRUPT, "object out of bounds");
  const uint8_t *fb = pp.buf.data() + 8 + il;
  const size_t fbn = total - 8 - il;
  const uint32_t fb_base = uint32_t(fb - pp.buf.data());
  pp.fb_bytes = fbn;
  FbTable page = FbTable::root(fb, fbn);
  const uint16_t eo = page.field(kPageEntries);
  pp.n = eo ? page.vector_len(eo) : 0;
  const uint32_t es = eo ? page.vector_start(eo) : 0;
  pp.id_off.resize(pp.n);
  pp.id_len.resize(pp.n);
  pp.start.resize(pp.n);
  pp.end.resize(pp.n);
  pp.tag0.assign(1, 0);
  pp.tag0.reserve(pp.n + 1);
  const size_t want_refs = hint.refs ? hint.refs + hint.refs / 4 : size_t(pp.n) * 20;
  pp.tag_kv.reserve(want_refs);
  pp.tag_res.reserve(want_refs);
  pp.kv_v0.assign(1, 0);
  if (hint.tables) {
    pp.kv_key.reserve(hint.tables + hint.tables / 4);
    pp.kv_v0.reserve(hint.tables + hint.tables / 4 + 1);
    pp.vals.reserve(hint.vals + hint.vals / 4);
    pp.vhash.reserve(hint.vals + hint.vals / 4);
  }
  pm.reset(fbn);
  std::vector<std::pair<uint32_t, uint32_t>> kpos_ids;  // key string position -> key id
  FbTable e{fb, fbn, 0}, kv{fb, fbn, 0};
  for (uint32_t j = 0; j < pp.n; j++) {
    e.pos = page.indirect(es + 4 * j);
    const uint16_t io = e.field(kEntryId);
    const std::string_view id = io ? e.byte_vector(e.pos + io) : std::string_view();
    if (id.size() > 16) fail(TSG_E_UNSUPPORTED, "trace id longer than 16 bytes");
    pp.id_off[j] = uint32_t(reinterpret_cast<const uint8_t *>(id.data()) - fb) + fb_base;
    pp.id_len[j] = uint8_t(id.size());
    pp.start[j] = e.u64(kEntryStart);
    pp.end[j] = e.u64(kEntryEnd);
    const uint16_t to = e.field(kEntryTags);
    const uint32_t nt = to ? e.vector_len(to) : 0, ts = to ? e.vector_start(to) : 0;
    const size_t t0 = pp.tag_kv.size();
    bool ordered = true;
    std::string_view prev;
    for (uint32_t t = 0; t < nt; t++) {
      const uint32_t pos = e.indirect(ts + 4 * t);
      uint32_t idx = pm.find_or_put(pos, uint32_t(pp.kv_key.size()));
      std::string_view key;
      if (idx == kNone) {  // a table not seen in this page yet
        idx = uint32_t(pp.kv_key.size());
        kv.pos = pos;
        const uint16_t ko = kv.field(kKvKey);
        key = ko ? kv.byte_vector(kv.pos + ko) : std::string_view();
        // the page's strings are shared (one copy of a key per page): key id by string position
        const uint32_t kpos = ko ? kv.indirect(kv.pos + ko) : 0u;
        uint32_t kid = kNone;
        for (const auto &x : kpos_ids)
          if (x.first == kpos) {
            kid = x.second;
            break;
          }
        if (kid == kNone) {
          kid = kc.get(kn, key);
          kpos_ids.push_back({kpos, kid});
        }
        pp.kv_key.push_back(kid);
        const uint16_t vo = kv.field(kKvValue);
        const uint32_t vn = vo ? kv.vector_len(vo) : 0, vs = vo ? kv.vector_start(vo) : 0;
        if (kid >= pp.kstat.size()) pp.kstat.resize(size_t(kid) + 1);
        LPage::KStat &ks = pp.kstat[kid];
        ks.tables++;
        ks.refs += vn;
        ks.multi = ks.multi || vn != 1;
        for (uint32_t q = 0; q < vn; q++) {
          const std::string_view v = kv.byte_vector(vs + 4 * q);
          ks.bytes += v.size();
          pp.vals.push_back(v);
          pp.vhash.push_back(hash_bytes(v.data(), v.size()));
        }
        pp.kv_v0.push_back(uint32_t(pp.vals.size()));
      } else {
        kv.pos = pos;
        const uint16_t ko = kv.field(kKvKey);
        key = ko ? kv.byte_vector(kv.pos + ko) : std::string_view();
      }
      // backend blocks hold keys unique and strictly descending (pitfall P3); otherwise
      // FindTag's binary search is emulated below
      if (t > 0 && !(prev > key)) ordered = false;
      prev = key;
      pp.tag_kv.push_back(idx);
    }
    if (ordered) {
      pp.tag_res.insert(pp.tag_res.end(), pp.tag_kv.begin() + long(t0), pp.tag_kv.end());
    } else {
      auto key_of = [&](uint32_t x) {
        kv.pos = e.indirect(ts + 4 * x);
        const uint16_t ko = kv.field(kKvKey);
        return ko ? kv.byte_vector(kv.pos + ko) : std::string_view();
      };
      for (uint32_t t = 0; t < nt; t++) {
        const std::string_view k = key_of(t);
        uint32_t i = 0, jj = nt, found = kNone;
        while (i < jj) {  // binarySearch, reversed comparator (searchdata_util.go:63-100)
          const uint32_t h = (i + jj) >> 1;
          const std::string_view hk = key_of(h);
          const int c = bytes_compare(reinterpret_cast<const uint8_t *>(hk.data()), hk.size(),
                                      reinterpret_cast<const uint8_t *>(k.data()), k.size());
          if (c == 0) {
            found = pp.tag_kv[t0 + h];
            break;
          }
          if (c < 0) jj = h;
          else i = h + 1;
        }
        pp.tag_res.push_back(found);
      }
    }
    pp.tag0.push_back(uint32_t(pp.tag_kv.size()));
  }
  pp.kv_sid.assign(pp.kv_key.size(), kNone);
  hint.tables = pp.kv_key.size();
  hint.vals = pp.vals.size();
  hint.refs = pp.tag_kv.size();
}

// Phase B tables. A key's values are interned in hash shards (shard = top hash bits), each
// by its own thread in page order; a value's id is its shard's base + its index there.
struct ValueShard {
  std::vector<uint8_t> bytes;
  std::vector<uint32_t> off{0};
  std::vector<uint64_t> slot;  // (hash high 32) << 32 | (local + 1)
  std::vector<uint64_t> vh;    // per local id: its hash
  size_t used = 0;
  static size_t probe0(uint64_t h, size_t mask) { return size_t(h ^ (h >> 29)) & mask; }
  void reserve(size_t nv, size_t nb) {
    size_t c = 256;
    while (c < 2 * nv + 2) c <<= 1;
    slot.assign(c, 0);
    vh.reserve(nv);
    off.reserve(nv + 1);
    bytes.reserve(nb);
  }
  uint32_t get(std::string_view v, uint64_t h) {
    if (2 * (used + 1) > slot.size()) grow();
    const size_t mask = slot.size() - 1;
    for (size_t i = probe0(h, mask);; i = (i + 1) & mask) {
      const uint64_t x = slot[i];
      if (!x) {
        const uint32_t id = uint32_t(off.size() - 1);
        bytes.insert(bytes.end(), v.begin(), v.end());
        off.push_back(uint32_t(bytes.size()));
        vh.push_back(h);
        slot[i] = (h & 0xffffffff00000000ull) | (uint64_t(id) + 1);
        used++;
        return id;
      }
      if ((x >> 32) == (h >> 32)) {
        const uint32_t id = uint32_t(x) - 1;
        if (vh[id] == h && off[id + 1] - off[id] == v.size() && std::memcmp(bytes.data() + off[id], v.data(), v.size()) == 0)
          return id;
      }
    }
  }
  void grow() {
    std::vector<uint64_t> old;
    old.swap(slot);
    slot.assign(std::max<size_t>(256, old.size() * 2), 0);
    const size_t mask = slot.size() - 1;
    for (uint64_t x : old) {
      if (!x) continue;
      size_t i = probe0(vh[uint32_t(x) - 1], mask);
      while (slot[i]) i = (i + 1) & mask;
      slot[i] = x;
    }
  }
};
// A multi-valued key's value sets (vectors of value ids), interned in page order.
struct SetIntern {
  KeyColumn *kc;
  std::vector<uint64_t> slot, sh;
  size_t used = 0;
  void reserve(size_t ns) {
    size_t c = 256;
    while (c < 2 * ns + 2) c <<= 1;
    slot.assign(c, 0);
    sh.reserve(ns);
  }
  uint32_t get(const uint32_t *vids, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    for (size_t i = 0; i < n; i++) {
      h = (h ^ vids[i]) * 0xff51afd7ed558ccdull;
      h ^= h >> 32;
    }
    if (2 * (used + 1) > slot.size()) grow();
    const size_t mask = slot.size() - 1;
    for (size_t i = ValueShard::probe0(h, mask);; i = (i + 1) & mask) {
      const uint64_t x = slot[i];
      if (!x) {
        const uint32_t sid = kc->nsets();
        kc->set_vals.insert(kc->set_vals.end(), vids, vids + n);
        kc->set_off.push_back(uint32_t(kc->set_vals.size()));
        if (n != 1 || sid != vids[0]) kc->identity = false;
        sh.push_back(h);
        slot[i] = (h & 0xffffffff00000000ull) | (uint64_t(sid) + 1);
        used++;
        return sid;
      }
      if ((x >> 32) == (h >> 32)) {
        const uint32_t sid = uint32_t(x) - 1;
        if (sh[sid] == h && kc->set_off[sid + 1] - kc->set_off[sid] == n &&
            std::equal(vids, vids + n, kc->set_vals.begin() + kc->set_off[sid]))
          return sid;
      }
    }
  }
  void grow() {
    std::vector<uint64_t> old;
    old.swap(slot);
    slot.assign(std::max<size_t>(256, old.size() * 2), 0);
    const size_t mask = slot.size() - 1;
    for (uint64_t x : old) {
      if (!x) continue;
      size_t i = ValueShard::probe0(sh[uint32_t(x) - 1], mask);
      while (slot[i]) i = (i + 1) & mask;
      slot[i] = x;
    }
  }
};

// Search blocks this process is decoding right now. A decode that was not given a thread
// count sizes each of its parallel phases to its share of the CPUs at that moment: blocks
// opened together (a querier's or the bench's concurrent opens) then split the CPUs instead
// of each starting a thread per CPU (measured: 8 blocks on 8 CPUs, 0.57 -> 0.71 GB/s).
std::atomic<int> g_decoding{0};
thread_local bool t_share = false;
int phase_threads(int nthreads) {
  if (!t_share) return nthreads;
  const int a = std::max(1, g_decoding.load(std::memory_order_relaxed));
  return std::max(1, std::min(nthreads, (host_threads_now() + a - 1) / a));
}

// runs f(i) for i in [0, n) on up to nthreads threads, items taken in order from a counter
template <class F>
void for_each_index(size_t n, int nthreads, F &&f) {
  nthreads = phase_threads(nthreads);
  std::atomic<size_t> next{0};
  std::mutex emu;
  std::exception_ptr err;
  auto work = [&] {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) break;
      try {
        f(i);
      } catch (...) {
        std::lock_guard<std::mutex> lk(emu);
        if (!err) err = std::current_exception();
        next.store(n);
      }
    }
  };
  const size_t nt = std::min<size_t>(size_t(std::max(1, nthreads)), n);
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto &x : th) x.join();
  if (err) std::rethrow_exception(err);
}
}  // namespace

static void load_pages(HostBlock &hb, const std::vector<IndexRecord> &recs, const uint8_t *data, size_t data_len,
                       int nthreads) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  // ---- A: pages
  std::vector<LPage> pages(recs.size());
  KeyNames kn;
  std::vector<KeyCache> caches(size_t(std::max(1, nthreads)));
  std::atomic<size_t> next{0};
  {
    auto work = [&](size_t w) {
      PosMap pm;
      PageHint hint;
      for (;;) {
        const size_t i = next.fetch_add(1);
        if (i >= pages.size()) break;
        LPage &pp = pages[i];
        try {
          parse_lpage(data, data_len, hb.meta.encoding, recs[i], kn, caches[w], pm, hint, pp);
        } catch (const Error &e) {
          pp.err = e.code;
          pp.msg = e.what();
        }
      }
    };
    const size_t nt = std::min<size_t>(size_t(std::max(1, phase_threads(nthreads))), std::max<size_t>(1, pages.size()));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; t++) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
  }
  // the first damaged page ends the block: the pages before it stay, and its error is what
  // Search returns once it gets there
  size_t np = pages.size();
  for (size_t i = 0; i < pages.size(); i++)
    if (pages[i].err) {
      hb.stop_status = pages[i].err;
      hb.stop_msg = pages[i].msg;
      np = i;
      break;
    }
  const auto t1 = clk::now();
  // keys (only those of the kept pages) in name order; tables grouped per key
  const size_t nk0 = kn.names.size();
  std::vector<uint8_t> used(nk0, 0);
  for (size_t i = 0; i < np; i++)
    for (uint32_t k : pages[i].kv_key) used[k] = 1;
  std::vector<uint32_t> ord;
  for (uint32_t k = 0; k < nk0; k++)
    if (used[k]) ord.push_back(k);
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return kn.names[a] < kn.names[b]; });
  std::vector<uint32_t> final_of(nk0, kNone);
  hb.keys.clear();
  hb.key_index.clear();
  hb.keys.resize(ord.size());
  for (size_t f = 0; f < ord.size(); f++) {
    final_of[ord[f]] = uint32_t(f);
    KeyColumn &kc = hb.keys[f];
    kc.name = kn.names[ord[f]];
    kc.dict_off.assign(1, 0);
    kc.set_off.assign(1, 0);
    hb.key_index.emplace(kc.name, int(f));
    if (kc.name == "root.service.name") hb.svc_key = int(f);
    if (kc.name == "root.name") hb.name_key = int(f);
  }
  const size_t nk = ord.size();
  for_each_index(np, nthreads, [&](size_t i) {
    LPage &pp = pages[i];
    for (auto &k : pp.kv_key) k = final_of[k];
    pp.bykey0.assign(nk + 1, 0);
    for (uint32_t k : pp.kv_key) pp.bykey0[k + 1]++;
    for (size_t k = 0; k < nk; k++) pp.bykey0[k + 1] += pp.bykey0[k];
    pp.bykey.resize(pp.kv_key.size());
    std::vector<uint32_t> at(pp.bykey0.begin(), pp.bykey0.end() - 1);
    for (uint32_t t = 0; t < pp.kv_key.size(); t++) pp.bykey[at[pp.kv_key[t]]++] = t;
  });
  const auto t2 = clk::now();
  // ---- B: values (hash shards, parallel) and value sets per key
  {
    struct KInfo {
      uint64_t tables = 0, refs = 0, bytes = 0;
      bool single = true;  // every table of the key holds exactly one value: set id = value id
      uint32_t P = 1;      // value shards
    };
    std::vector<KInfo> kin(nk);
    for (size_t k = 0; k < nk; k++) {  // (the pages counted their keys' tables as they parsed)
      KInfo &I = kin[k];
      const uint32_t pk = ord[k];
      for (size_t i = 0; i < np; i++) {
        const LPage &pp = pages[i];
        if (pk >= pp.kstat.size()) continue;
        const LPage::KStat &ks = pp.kstat[pk];
        I.tables += ks.tables;
        I.refs += ks.refs;
        I.bytes += ks.bytes;
        I.single = I.single && !ks.multi;
      }
      while (I.P < 16 && I.refs / I.P > 65536) I.P <<= 1;
    }
    auto shard_of = [](uint64_t h, uint32_t P) { return uint32_t(h >> 48) & (P - 1); };
    // each shard's value references (page << 32 | value), in page order: one pass per key
    std::vector<std::vector<std::vector<uint64_t>>> refs(nk);
    for_each_index(nk, nthreads, [&](size_t k) {
      const uint32_t P = kin[k].P;
      refs[k].resize(P);
      for (auto &r : refs[k]) r.reserve(size_t(kin[k].refs / P + kin[k].refs / (4 * P) + 16));
      for (size_t i = 0; i < np; i++) {
        const LPage &pp = pages[i];
        for (uint32_t b = pp.bykey0[k]; b < pp.bykey0[k + 1]; b++) {
          const uint32_t t = pp.bykey[b];
          for (uint32_t v = pp.kv_v0[t]; v < pp.kv_v0[t + 1]; v++)
            refs[k][shard_of(pp.vhash[v], P)].push_back((uint64_t(i) << 32) | v);
        }
      }
    });
    for_each_index(np, nthreads, [&](size_t i) { pages[i].vloc.resize(pages[i].vals.size()); });
    const auto tb1 = clk::now();
    std::vector<std::vector<ValueShard>> shards(nk);
    std::vector<std::pair<uint32_t, uint32_t>> jobs;  // (key, shard), heaviest first
    for (uint32_t k = 0; k < nk; k++) {
      shards[k].resize(kin[k].P);
      for (uint32_t x = 0; x < kin[k].P; x++) jobs.push_back({k, x});
    }
    std::sort(jobs.begin(), jobs.end(), [&](const auto &a, const auto &b) {
      return kin[a.first].refs / kin[a.first].P > kin[b.first].refs / kin[b.first].P;
    });
    for_each_index(jobs.size(), nthreads, [&](size_t j) {
      const uint32_t k = jobs[j].first, x = jobs[j].second, P = kin[k].P;
      ValueShard &S = shards[k][x];
      const auto &R = refs[k][x];
      S.reserve(R.size(), size_t(kin[k].bytes / P + kin[k].bytes / (4 * P)));
      // A reference's page-level entries (its string view, hash and id slot: arrays shared by
      // every key of the page, so consecutive references of one key are a line or more apart)
      // and the value bytes they point to were evicted long ago: the entries are prefetched 32
      // references ahead, the bytes 16 ahead (their view is in cache by then), the slots 8
      // ahead, so the misses of consecutive references overlap (one dependent DRAM round trip
      // per entry each before: ~150-250 ns per reference)
      const size_t nr = R.size();
      const size_t mask = S.slot.size() - 1;
      for (size_t q = 0; q < nr; q++) {
        if (q + 32 < nr) {
          const uint64_t rc = R[q + 32];
          const LPage &pc = pages[size_t(rc >> 32)];
          const uint32_t vc = uint32_t(rc);
          __builtin_prefetch(pc.vals.data() + vc);
          __builtin_prefetch(pc.vhash.data() + vc);
          __builtin_prefetch(pc.vloc.data() + vc, 1);
        }
        if (q + 16 < nr) {
          const uint64_t ra = R[q + 16];
          const LPage &pa = pages[size_t(ra >> 32)];
          __builtin_prefetch(pa.vals[uint32_t(ra)].data());
        }
        if (q + 8 < nr && S.slot.size() - 1 == mask) {
          const uint64_t rb = R[q + 8];
          const LPage &pb = pages[size_t(rb >> 32)];
          __builtin_prefetch(&S.slot[ValueShard::probe0(pb.vhash[uint32_t(rb)], mask)]);
        }
        const uint64_t r = R[q];
        LPage &pp = pages[size_t(r >> 32)];
        const uint32_t v = uint32_t(r);
        pp.vloc[v] = S.get(pp.vals[v], pp.vhash[v]);
      }
      S.slot = std::vector<uint64_t>();
      std::vector<uint64_t>().swap(refs[k][x]);
    });
    const auto tb2 = clk::now();
    // each key's dictionary: its shards one after another
    std::vector<std::vector<uint32_t>> vbase(nk);
    for_each_index(nk, nthreads, [&](size_t k) {
      KeyColumn &kc = hb.keys[k];
      uint64_t nv = 0, nb = 0;
      vbase[k].resize(kin[k].P);
      for (uint32_t x = 0; x < kin[k].P; x++) {
        vbase[k][x] = uint32_t(nv);
        nv += shards[k][x].off.size() - 1;
        nb += shards[k][x].bytes.size();
      }
      if (nb > 0xF0000000u) fail(TSG_E_UNSUPPORTED, "dictionary too large");
      kc.dict_bytes.resize(nb);  // (not zero-filled: the shards' copies below write every byte)
      advise_huge(kc.dict_bytes.data(), nb);
      kc.dict_off.resize(nv + 1);
      kc.dict_off[nv] = uint32_t(nb);
      if (nb > kDeferMinBytes) kc.dict_vh.resize(nv);  // (kept for verify_header_dicts)
    });
    for_each_index(jobs.size(), nthreads, [&](size_t j) {
      const uint32_t k = jobs[j].first, x = jobs[j].second;
      const ValueShard &S = shards[k][x];
      KeyColumn &kc = hb.keys[k];
      uint64_t b0 = 0;
      for (uint32_t y = 0; y < x; y++) b0 += shards[k][y].bytes.size();
      if (!S.bytes.empty()) std::memcpy(kc.dict_bytes.data() + b0, S.bytes.data(), S.bytes.size());
      for (size_t i = 0; i + 1 < S.off.size(); i++) kc.dict_off[vbase[k][x] + i] = uint32_t(b0 + S.off[i]);
      if (!kc.dict_vh.empty()) std::copy(S.vh.begin(), S.vh.end(), kc.dict_vh.begin() + vbase[k][x]);
    });
    shards.clear();
    const auto tb3 = clk::now();
    // value sets: a single-valued key's set of value v is v (identity); other keys intern
    // their value-id vectors in page order
    for_each_index(nk, nthreads, [&](size_t k) {
      KeyColumn &kc = hb.keys[k];
      const uint32_t P = kin[k].P;
      const std::vector<uint32_t> &vb = vbase[k];
      if (kin[k].single) {
        const uint32_t nv = kc.nvals();
        kc.identity = true;
        kc.set_off.resize(size_t(nv) + 1);
        kc.set_vals.resize(nv);
        for (uint32_t v = 0; v <= nv; v++) kc.set_off[v] = v;
        for (uint32_t v = 0; v < nv; v++) kc.set_vals[v] = v;
        for (size_t i = 0; i < np; i++) {
          LPage &pp = pages[i];
          for (uint32_t b = pp.bykey0[k]; b < pp.bykey0[k + 1]; b++) {
            const uint32_t t = pp.bykey[b], v = pp.kv_v0[t];
            pp.kv_sid[t] = vb[shard_of(pp.vhash[v], P)] + pp.vloc[v];
          }
        }
        return;
      }
      kc.identity = false;  // (some table holds no value or several)
    });
    // multi-valued keys: the value-id vectors interned in hash shards as well
    auto vid_of = [&](const LPage &pp, uint32_t k, uint32_t v) {
      return vbase[k][shard_of(pp.vhash[v], kin[k].P)] + pp.vloc[v];
    };
    auto set_hash = [&](const LPage &pp, uint32_t k, uint32_t t) {
      const uint32_t n = pp.kv_v0[t + 1] - pp.kv_v0[t];
      uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
      for (uint32_t v = pp.kv_v0[t]; v < pp.kv_v0[t + 1]; v++) {
        h = (h ^ vid_of(pp, k, v)) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
      }
      return mix_set(h);
    };
    std::vector<uint32_t> SP(nk, 1);
    std::vector<std::vector<std::vector<uint64_t>>> srefs(nk);  // per set shard: page << 32 | table
    bool any_multi = false;
    for (size_t k = 0; k < nk; k++) any_multi = any_multi || !kin[k].single;
    if (any_multi)  // each multi-valued table's set hash, computed once (kv_shash)
      for_each_index(np, nthreads, [&](size_t i) { pages[i].kv_shash.resize(pages[i].kv_key.size()); });
    for_each_index(nk, nthreads, [&](size_t k) {
      if (kin[k].single) return;
      while (SP[k] < 16 && kin[k].tables / SP[k] > 65536) SP[k] <<= 1;
      srefs[k].resize(SP[k]);
      for (auto &r : srefs[k]) r.reserve(size_t(kin[k].tables / SP[k] + kin[k].tables / (4 * SP[k]) + 16));
      for (size_t i = 0; i < np; i++) {
        LPage &pp = pages[i];
        for (uint32_t b = pp.bykey0[k]; b < pp.bykey0[k + 1]; b++) {
          const uint32_t t = pp.bykey[b];
          const uint64_t h = set_hash(pp, uint32_t(k), t);
          pp.kv_shash[t] = h;
          srefs[k][shard_of(h, SP[k])].push_back((uint64_t(i) << 32) | t);
        }
      }
    });
    struct SetShard {
      std::vector<uint32_t> vals, off{0};
      std::vector<uint64_t> slot, sh;
      size_t used = 0;
    };
    std::vector<std::vector<SetShard>> sshards(nk);
    std::vector<std::pair<uint32_t, uint32_t>> sjobs;
    for (uint32_t k = 0; k < nk; k++) {
      if (kin[k].single) continue;
      sshards[k].resize(SP[k]);
      for (uint32_t x = 0; x < SP[k]; x++) sjobs.push_back({k, x});
    }
    for_each_index(sjobs.size(), nthreads, [&](size_t j) {
      const uint32_t k = sjobs[j].first, x = sjobs[j].second;
      SetShard &S = sshards[k][x];
      const auto &R = srefs[k][x];
      size_t c = 256;
      while (c < 2 * R.size() + 2) c <<= 1;
      S.slot.assign(c, 0);
      const size_t mask = c - 1;
      std::vector<uint32_t> tmp;
      for (size_t q = 0; q < R.size(); q++) {
        if (q + 32 < R.size()) {  // (the table's value range and set hash, 32 references ahead)
          const LPage &pa = pages[size_t(R[q + 32] >> 32)];
          const uint32_t ta = uint32_t(R[q + 32]);
          __builtin_prefetch(&pa.kv_v0[ta]);
          __builtin_prefetch(&pa.kv_shash[ta]);
          __builtin_prefetch(&pa.kv_sid[ta], 1);
        }
        if (q + 16 < R.size()) {  // (its values' hashes and ids, 16 ahead: the range is in cache)
          const LPage &pb = pages[size_t(R[q + 16] >> 32)];
          const uint32_t v0 = pb.kv_v0[uint32_t(R[q + 16])];
          __builtin_prefetch(pb.vhash.data() + v0);
          __builtin_prefetch(pb.vloc.data() + v0);
        }
        const uint64_t r = R[q];
        LPage &pp = pages[size_t(r >> 32)];
        const uint32_t t = uint32_t(r);
        tmp.clear();
        for (uint32_t v = pp.kv_v0[t]; v < pp.kv_v0[t + 1]; v++) tmp.push_back(vid_of(pp, k, v));
        const uint64_t h = pp.kv_shash[t];
        uint32_t sid = kNone;
        for (size_t i = ValueShard::probe0(h, mask);; i = (i + 1) & mask) {
          const uint64_t xs = S.slot[i];
          if (!xs) {
            sid = uint32_t(S.off.size() - 1);
            S.vals.insert(S.vals.end(), tmp.begin(), tmp.end());
            S.off.push_back(uint32_t(S.vals.size()));
            S.sh.push_back(h);
            S.slot[i] = (h & 0xffffffff00000000ull) | (uint64_t(sid) + 1);
            break;
          }
          if ((xs >> 32) == (h >> 32)) {
            const uint32_t y = uint32_t(xs) - 1;
            if (S.sh[y] == h && S.off[y + 1] - S.off[y] == tmp.size() &&
                std::equal(tmp.begin(), tmp.end(), S.vals.begin() + S.off[y])) {
              sid = y;
              break;
            }
          }
        }
        pp.kv_sid[t] = sid;  // (local to the shard until the bases are added)
      }
      S.slot = std::vector<uint64_t>();
    });
    // each multi-valued key's sets: its shards one after another; table set ids shifted
    std::vector<std::vector<uint32_t>> sbase(nk);
    for_each_index(nk, nthreads, [&](size_t k) {
      if (kin[k].single) return;
      KeyColumn &kc = hb.keys[k];
      uint64_t ns = 0, nvals = 0;
      sbase[k].resize(SP[k]);
      for (uint32_t x = 0; x < SP[k]; x++) {
        sbase[k][x] = uint32_t(ns);
        ns += sshards[k][x].off.size() - 1;
        nvals += sshards[k][x].vals.size();
      }
      kc.set_vals.resize(nvals);
      kc.set_off.resize(ns + 1);
      uint64_t vo = 0;
      for (uint32_t x = 0; x < SP[k]; x++) {
        const SetShard &S = sshards[k][x];
        std::copy(S.vals.begin(), S.vals.end(), kc.set_vals.begin() + long(vo));
        for (size_t i = 0; i + 1 < S.off.size(); i++) kc.set_off[sbase[k][x] + i] = uint32_t(vo + S.off[i]);
        vo += S.vals.size();
      }
      kc.set_off[ns] = uint32_t(vo);
      for (size_t i = 0; i < np; i++) {
        LPage &pp = pages[i];
        for (uint32_t b = pp.bykey0[k]; b < pp.bykey0[k + 1]; b++) {
          const uint32_t t = pp.bykey[b];
          pp.kv_sid[t] += sbase[k][shard_of(pp.kv_shash[t], SP[k])];
        }
      }
    });
    if (prof_on()) {
      const auto tb4 = clk::now();
      prof_add("load.b.stats", std::chrono::duration<double, std::micro>(tb1 - t2).count());
      prof_add("load.b.values", std::chrono::duration<double, std::micro>(tb2 - tb1).count());
      prof_add("load.b.dict", std::chrono::duration<double, std::micro>(tb3 - tb2).count());
      prof_add("load.b.sets", std::chrono::duration<double, std::micro>(tb4 - tb3).count());
    }
  }
  const auto t3 = clk::now();
  // ---- C: entry columns
  std::vector<uint64_t> base(np + 1, 0);
  for (size_t i = 0; i < np; i++) {
    base[i + 1] = base[i] + pages[i].n;
    hb.page_entries.push_back(pages[i].n);
    hb.page_fb_bytes.push_back(pages[i].fb_bytes);
    hb.page_first.push_back(base[i]);
    hb.fb_bytes += pages[i].fb_bytes;
  }
  const uint64_t n = base[np];
  hb.n = n;
  hb.ids.assign(n * 16, 0);
  hb.id_len.resize(n);
  hb.start.resize(n);
  hb.end.resize(n);
  hb.svc_vid.assign(n, kNone);
  hb.name_vid.assign(n, kNone);
  for_each_index(nk, nthreads, [&](size_t k) { hb.keys[k].col.assign(n, kNone); });
  for_each_index(np, nthreads, [&](size_t i) {
    const LPage &pp = pages[i];
    for (uint32_t j = 0; j < pp.n; j++) {
      const uint64_t e = base[i] + j;
      const uint8_t il = pp.id_len[j];
      std::memcpy(&hb.ids[e * 16 + 16 - il], pp.buf.data() + pp.id_off[j], il);
      hb.id_len[e] = il;
      hb.start[e] = pp.start[j];
      hb.end[e] = pp.end[j];
      bool svc_done = false, name_done = false;
      for (uint32_t r = pp.tag0[j]; r < pp.tag0[j + 1]; r++) {
        const uint32_t t = pp.tag_kv[r];
        const uint32_t k = pp.kv_key[t];
        if (pp.tag_res[r] != kNone) hb.keys[k].col[e] = pp.kv_sid[pp.tag_res[r]];
        // SearchEntry.Get: the first table of the key in vector order, Value(0)
        // (searchdata_util.go:10-23)
        if (int(k) == hb.svc_key && !svc_done) {
          svc_done = true;
          if (pp.kv_v0[t + 1] > pp.kv_v0[t]) {
            const KeyColumn &kc = hb.keys[k];
            hb.svc_vid[e] = kc.set_vals[kc.set_off[pp.kv_sid[t]]];
          }
        }
        if (int(k) == hb.name_key && !name_done) {
          name_done = true;
          if (pp.kv_v0[t + 1] > pp.kv_v0[t]) {
            const KeyColumn &kc = hb.keys[k];
            hb.name_vid[e] = kc.set_vals[kc.set_off[pp.kv_sid[t]]];
          }
        }
      }
    }
  });
  if (prof_on()) {
    const auto t4 = clk::now();
    prof_add("load.pages", std::chrono::duration<double, std::micro>(t1 - t0).count());
    prof_add("load.group", std::chrono::duration<double, std::micro>(t2 - t1).count());
    prof_add("load.intern", std::chrono::duration<double, std::micro>(t3 - t2).count());
    prof_add("load.columns", std::chrono::duration<double, std::micro>(t4 - t3).count());
  }
}

void decode_search_block(const uint8_t *meta, size_t meta_len, bool meta_present, Bytes header,
                         const uint8_t *index, size_t index_len, const uint8_t *data, size_t data_len, int nthreads,
                         HostBlock &hb, uint32_t first_page, uint32_t npages) {
  struct Share {  // (this decode counts in g_decoding; its phases take their share when auto-sized)
    bool prev;
    explicit Share(bool on) : prev(t_share) {
      t_share = on;
      g_decoding.fetch_add(1);
    }
    ~Share() {
      g_decoding.fetch_sub(1);
      t_share = prev;
    }
  } share(nthreads <= 0);
  if (!meta_present) {
    hb.has_meta = false;
    return;
  }
  hb.has_meta = true;
  hb.meta = parse_search_meta(meta, meta_len);
  if (hb.meta.version != "v2") fail(TSG_E_UNSUPPORTED_ENCODING, "unsupported search block version " + hb.meta.version);
  if (hb.meta.encoding != 0 && hb.meta.encoding != 6)
    fail(TSG_E_UNSUPPORTED_ENCODING, std::string("search encoding not supported: ") + encoding_name(hb.meta.encoding));
  hb.header = std::move(header);
  {
    FbTable h = FbTable::root(hb.header.data(), hb.header.size());
    hb.min_dur = h.u64(kHdrMin);
    hb.max_dur = h.u64(kHdrMax);
  }
  const auto th0 = std::chrono::steady_clock::now();
  index_header(hb);
  if (prof_on())
    prof_add("load.hdr", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - th0).count());
  std::vector<IndexRecord> recs =
      read_index(index, index_len, hb.meta.index_page_size, hb.meta.index_records, &hb.index_truncated);
  if (first_page > 0 || npages < recs.size()) {  // a page range (records past a damaged one are gone already)
    const size_t a = std::min<size_t>(first_page, recs.size());
    const size_t b = a + std::min<size_t>(npages, recs.size() - a);
    recs = std::vector<IndexRecord>(recs.begin() + ptrdiff_t(a), recs.begin() + ptrdiff_t(b));
    hb.part_first_page = first_page;
    hb.part_tail = first_page > 0;
  }
  if (nthreads <= 0) nthreads = host_threads();
  nthreads = std::min<int>(nthreads, 64);

  using clk = std::chrono::steady_clock;
  const bool prof = prof_on();
  load_pages(hb, recs, data, data_len, nthreads);
  const auto tc0 = clk::now();
  canonicalize_narrow_keys(hb);
  const auto tc1 = clk::now();
  verify_header_dicts(hb, nthreads);
  // byte-pair counts of the large dictionaries: 64 windows of 16 KiB spread over the bytes
  for_each_index(hb.keys.size(), nthreads, [&](size_t k) {
    KeyColumn &kc = hb.keys[k];
    const size_t nb = kc.dict_bytes.size();
    if (nb <= kDeferMinBytes) return;
    kc.pair_freq.assign(65536, 0);
    constexpr size_t kWin = 16384, kWins = 64;
    for (size_t w = 0; w < kWins; w++) {
      const size_t a = (nb - kWin) / (kWins - 1) * w;
      const uint8_t *p = kc.dict_bytes.data() + a;
      for (size_t i = 0; i + 1 < kWin; i++) kc.pair_freq[(uint32_t(p[i]) << 8) | p[i + 1]]++;
    }
  });
  if (prof) {
    prof_add("load.canon", std::chrono::duration<double, std::micro>(tc1 - tc0).count());
    prof_add("load.verify", std::chrono::duration<double, std::micro>(clk::now() - tc1).count());
  }
}

// ---- header values == dictionary (hdr_defer) -------------------------------------------
// A large key's header values are deferred to the device pass only when they are exactly the
// block's dictionary values: equal counts, and every header value found byte for byte in the
// dictionary, no dictionary value found twice (the dictionary's values are distinct, so this
// is a bijection). The dictionary side is keyed by the xxhash64 each value was interned with
// (KeyColumn::dict_vh: no second pass over its bytes); a header value's hash only picks the
// candidates, the bytes decide (the earlier count + multiset-hash test rested on
// the hash alone). TSG_VERIFY_HASH_BITS (tests only) keeps that many low bits of the hash, so
// that unequal values collide and the byte comparison is what separates them.
void verify_header_dicts(HostBlock &hb, int nthreads) {
  hb.hdr_defer.assign(hb.hdr_keys.size(), 0);
  if (!hb.hdr_index) return;
  if (nthreads <= 0) nthreads = host_threads();
  nthreads = std::max(1, std::min(phase_threads(nthreads), 32));
  uint64_t mask = ~0ull;
  if (const char *e = std::getenv("TSG_VERIFY_HASH_BITS")) {
    const int bits = std::atoi(e);
    if (bits >= 0 && bits < 64) mask = (1ull << bits) - 1;
  }
  auto mix = [](uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    return h;
  };
  for (size_t hk = 0; hk < hb.hdr_keys.size(); hk++) {
    auto it = hb.key_index.find(std::string(hb.hdr_keys[hk]));
    if (it == hb.key_index.end()) continue;
    const int key = it->second;
    const KeyColumn &kc = hb.keys[size_t(key)];
    if (kc.dict_bytes.size() <= kDeferMinBytes) continue;
    const uint32_t v0 = hb.hdr_val0[hk], v1 = hb.hdr_val0[hk + 1];
    const uint32_t n = kc.nvals();
    if (v1 - v0 != n || kc.dict_vh.size() != n) continue;
    // open addressing over the dictionary's value ids by (masked) hash: a slot holds the hash's
    // high 32 bits and the id + 1 (a probe compares the tag before it touches the dictionary),
    // filled on nt threads with compare-and-swap
    size_t cap = 16;
    while (cap < 2 * size_t(n)) cap <<= 1;
    std::unique_ptr<std::atomic<uint64_t>[]> slot(new std::atomic<uint64_t>[cap]());
    const size_t nt = std::max<size_t>(1, std::min<size_t>(size_t(nthreads), n / 4096));
    auto par = [&](auto &&f) {
      std::vector<std::thread> th;
      for (size_t t = 1; t < nt; t++) th.emplace_back(f, t);
      f(size_t(0));
      for (auto &x : th) x.join();
    };
    par([&](size_t t) {
      const size_t lo = size_t(n) * t / nt, hi = size_t(n) * (t + 1) / nt;
      for (size_t d = lo; d < hi; d++) {
        const uint64_t m = mix(kc.dict_vh[d] & mask);
        const uint64_t v = (m & 0xffffffff00000000ull) | (uint64_t(d) + 1);
        for (size_t i = m & (cap - 1);; i = (i + 1) & (cap - 1)) {
          uint64_t cur = 0;
          if (slot[i].compare_exchange_strong(cur, v, std::memory_order_relaxed)) break;
        }
      }
    });
    std::unique_ptr<std::atomic<uint8_t>[]> used(new std::atomic<uint8_t>[n]());
    std::atomic<bool> ok{true};
    // header values in batches of kB: their hashes and slots first (prefetched), then the
    // candidates' offsets (prefetched), then the bytes: the misses of a batch overlap instead of
    // following one another (≈ 5 dependent cache misses per value before: 200 ms per block for
    // config 2's 1 M http.url values)
    constexpr size_t kB = 32;
    par([&](size_t t) {
      const size_t lo = size_t(n) * t / nt, hi = size_t(n) * (t + 1) / nt;
      uint64_t hm[kB];
      uint32_t cand[kB];
      for (size_t j0 = lo; j0 < hi && ok.load(std::memory_order_relaxed); j0 += kB) {
        const size_t nb = std::min(kB, hi - j0);
        for (size_t q = 0; q < nb; q++) {
          const std::string_view v = hb.hdr_vals[v0 + j0 + q];
          hm[q] = mix(xxhash64(reinterpret_cast<const uint8_t *>(v.data()), v.size()) & mask);
          __builtin_prefetch(&slot[hm[q] & (cap - 1)]);
        }
        for (size_t q = 0; q < nb; q++) {  // the first slot whose tag matches (the usual answer)
          cand[q] = kNone;
          for (size_t i = hm[q] & (cap - 1);; i = (i + 1) & (cap - 1)) {
            const uint64_t x = slot[i].load(std::memory_order_relaxed);
            if (!x) break;
            if ((x >> 32) == (hm[q] >> 32)) {
              cand[q] = uint32_t(x) - 1;
              break;
            }
          }
          if (cand[q] != kNone) {
            __builtin_prefetch(&kc.dict_off[cand[q]]);
            __builtin_prefetch(&used[cand[q]]);
          }
        }
        for (size_t q = 0; q < nb; q++)
          if (cand[q] != kNone) __builtin_prefetch(kc.dict_bytes.data() + kc.dict_off[cand[q]]);
        for (size_t q = 0; q < nb; q++) {
          const std::string_view v = hb.hdr_vals[v0 + j0 + q];
          bool found = false;
          if (cand[q] != kNone && hb.dict_value(key, cand[q]) == v) {
            found = !used[cand[q]].exchange(1, std::memory_order_relaxed);  // (a second copy: not the dictionary)
          } else {
            // the rest of the chain: every slot with this tag, bytes compared
            for (size_t i = hm[q] & (cap - 1);; i = (i + 1) & (cap - 1)) {
              const uint64_t x = slot[i].load(std::memory_order_relaxed);
              if (!x) break;
              const uint32_t d = uint32_t(x) - 1;
              if ((x >> 32) != (hm[q] >> 32) || d == cand[q] || hb.dict_value(key, d) != v) continue;
              found = !used[d].exchange(1, std::memory_order_relaxed);
              break;
            }
          }
          if (!found) ok.store(false, std::memory_order_relaxed);
        }
      }
    });
    hb.hdr_defer[hk] = ok.load() ? 1 : 0;
  }
  for (auto &kc : hb.keys) std::vector<uint64_t>().swap(kc.dict_vh);
}

}  // namespace tsg

namespace tsg {

int parse_wal_filename(const std::string &name, std::string &version) {
  std::vector<std::string> parts;
  size_t p = 0;
  for (;;) {
    size_t q = name.find(':', p);
    parts.push_back(name.substr(p, q == std::string::npos ? std::string::npos : q - p));
    if (q == std::string::npos) break;
    p = q + 1;
  }
  if (parts.size() != 4 && parts.size() != 5) fail(TSG_E_INVALID, "unable to parse " + name + ". unexpected number of segments");
  const std::string &u = parts[0];  // uuid.Parse: the canonical 36-character form
  bool uuid_ok = u.size() == 36;
  for (size_t i = 0; i < u.size() && uuid_ok; i++)
    uuid_ok = (i == 8 || i == 13 || i == 18 || i == 23) ? u[i] == '-' : std::isxdigit(uint8_t(u[i])) != 0;
  if (!uuid_ok) fail(TSG_E_INVALID, "unable to parse " + name + ". error parsing uuid");
  if (parts[1].empty()) fail(TSG_E_INVALID, "unable to parse " + name + ". missing fields");
  version = parts[2];
  if (version != "v2") fail(TSG_E_UNSUPPORTED_ENCODING, "unable to parse " + name + ". error parsing version");
  const int enc = parse_encoding(parts[3]);
  if (enc < 0) fail(TSG_E_INVALID, "unable to parse " + name + ". error parsing encoding");
  return enc;
}

namespace {
// SearchEntryMutable fields accumulated by DataCombiner.Combine (data_combiner.go:11-44)
void combine_into(SearchEntryIn &d, const std::vector<uint8_t> &obj) {
  FbTable e = FbTable::root(obj.data(), obj.size());
  uint16_t to = e.field(kEntryTags);
  uint32_t nt = to ? e.vector_len(to) : 0, ts = to ? e.vector_start(to) : 0;
  FbTable kv{obj.data(), obj.size(), 0};
  for (uint32_t t = 0; t < nt; t++) {
    kv.pos = e.indirect(ts + 4 * t);
    uint16_t ko = kv.field(kKvKey);
    std::string key(ko ? kv.byte_vector(kv.pos + ko) : std::string_view());
    uint16_t vo = kv.field(kKvValue);
    uint32_t vn = vo ? kv.vector_len(vo) : 0, vs = vo ? kv.vector_start(vo) : 0;
    for (uint32_t q = 0; q < vn; q++) d.tags[key].insert(std::string(kv.byte_vector(vs + 4 * q)));  // AddTag
  }
  const uint64_t st = e.u64(kEntryStart), en = e.u64(kEntryEnd);
  if (st > 0 && (d.start == 0 || d.start > st)) d.start = st;  // SetStartTimeUnixNano
  if (en > 0 && en > d.end) d.end = en;                         // SetEndTimeUnixNano
  uint16_t io = e.field(kEntryId);
  std::string_view id = io ? e.byte_vector(e.pos + io) : std::string_view();
  d.id.assign(id.begin(), id.end());  // data.TraceID = sd.Id()
}

// SearchBlockHeaderMutable.AddEntry (SearchBlockHeader_util.go:21-43)
void header_add_entry(HostBlock &hb, const uint8_t *obj, size_t n) {
  FbTable e = FbTable::root(obj, n);
  uint16_t to = e.field(kEntryTags);
  uint32_t nt = to ? e.vector_len(to) : 0, ts = to ? e.vector_start(to) : 0;
  FbTable kv{obj, n, 0};
  for (uint32_t t = 0; t < nt; t++) {
    kv.pos = e.indirect(ts + 4 * t);
    uint16_t ko = kv.field(kKvKey);
    std::string key(ko ? kv.byte_vector(kv.pos + ko) : std::string_view());
    uint16_t vo = kv.field(kKvValue);
    uint32_t vn = vo ? kv.vector_len(vo) : 0, vs = vo ? kv.vector_start(vo) : 0;
    for (uint32_t q = 0; q < vn; q++) hb.stream_tags[key].insert(std::string(kv.byte_vector(vs + 4 * q)));
  }
  const uint64_t dur = e.u64(kEntryEnd) - e.u64(kEntryStart);  // uint64 wrap (P2)
  if (hb.min_dur == 0 || dur < hb.min_dur) hb.min_dur = dur;    // quirk P1
  if (dur > hb.max_dur) hb.max_dur = dur;
}
}  // namespace

void decode_wal_search_block(const uint8_t *file, size_t len, int enc, HostBlock &hb) {
  hb = HostBlock();
  hb.has_meta = true;
  hb.streaming = true;
  hb.meta.version = "v2";
  hb.meta.encoding = enc;
  if (enc != 0 && enc != 6)
    fail(TSG_E_UNSUPPORTED_ENCODING, std::string("search encoding not supported: ") + encoding_name(enc));
  struct Rec {
    std::string id;
    std::vector<uint8_t> obj;
  };
  std::vector<Rec> recs;
  // ReplayWALAndGetRecords: pages in file order until EOF; a damaged page ends the
  // replay with a warning and keeps the records before it
  std::vector<uint8_t> buf;
  for (size_t off = 0; off < len;) {
    try {
      if (len - off < 6) fail(TSG_E_CORRUPT, "truncated page header");
      const uint32_t total = le32(file + off);
      if (total < 6 || total > len - off) fail(TSG_E_CORRUPT, "truncated page");
      const uint8_t *hdr, *payload;
      size_t pl;
      unmarshal_page(file + off, total, 0, hdr, payload, pl);
      if (enc == 0) buf.assign(payload, payload + pl);
      else snappy_framed_decode(payload, pl, buf);
      // exactly one object per page: [u32 total][u32 idLen][id][obj], then EOF
      if (buf.size() < 8) fail(TSG_E_CORRUPT, "object header truncated");
      const uint32_t ot = le32(buf.data()), il = le32(buf.data() + 4);
      if (ot < 8 || ot - 8 > buf.size() - 8 || il > ot - 8) fail(TSG_E_CORRUPT, "object out of bounds");
      if (buf.size() != ot) fail(TSG_E_CORRUPT, "expected EOF after the page's object");
      Rec r;
      r.id.assign(reinterpret_cast<const char *>(buf.data() + 8), il);
      r.obj.assign(buf.data() + 8 + il, buf.data() + ot);
      header_add_entry(hb, r.obj.data(), r.obj.size());  // handleObj
      recs.push_back(std::move(r));
      off += total;
    } catch (const Error &) {
      hb.partial = true;
      break;
    }
  }
  if (recs.empty()) fail(TSG_E_NOT_FOUND, "empty wal file");  // RescanBlocks drops it
  // common.SortRecords (bytes order of ids; equal ids combine order-independently)
  std::stable_sort(recs.begin(), recs.end(), [](const Rec &a, const Rec &b) { return a.id < b.id; });
  std::vector<KeyBuild> kb;
  PageParse pp;
  for (size_t i = 0; i < recs.size();) {
    size_t j = i + 1;
    while (j < recs.size() && recs[j].id == recs[i].id) j++;
    pp = PageParse();
    if (j - i == 1) {
      pp.buf = std::move(recs[i].obj);
    } else {  // dedupingIterator -> DataCombiner.Combine -> SearchEntryMutable.ToBytes
      SearchEntryIn d;
      for (size_t k = i; k < j; k++)
        if (!recs[k].obj.empty()) combine_into(d, recs[k].obj);
      pp.buf = fb_search_entry_bytes(d);
    }
    pp.fb_bytes = pp.buf.size();  // sr.AddBytesInspected(len(obj))
    pp.nentries = 1;
    pp.tag_begin.push_back(0);
    FbTable e = FbTable::root(pp.buf.data(), pp.buf.size());
    std::unordered_map<uint32_t, uint32_t> memo;
    parse_entry(e, pp.buf.data(), 0, pp, memo);
    merge_page(hb, kb, pp);
    i = j;
  }
  for (auto &kc : hb.keys) kc.col.resize(hb.n, kNone);
  canonicalize_narrow_keys(hb);
}

void decode_live_block(const uint8_t *bytes, const uint64_t *seg_off, uint64_t nsegs, const uint64_t *trace_seg,
                       uint32_t ntraces, HostBlock &hb) {
  hb = HostBlock();
  hb.has_meta = true;
  hb.live = true;
  hb.meta.version = "v2";
  hb.meta.encoding = 0;
  if (trace_seg[0] != 0 || trace_seg[ntraces] != nsegs) fail(TSG_E_INVALID, "trace_seg must run from 0 to nsegs");
  for (uint32_t t = 0; t < ntraces; t++)
    if (trace_seg[t] > trace_seg[t + 1]) fail(TSG_E_INVALID, "trace_seg must be non-decreasing");
  for (uint64_t i = 0; i < nsegs; i++)
    if (seg_off[i] > seg_off[i + 1]) fail(TSG_E_INVALID, "seg_off must be non-decreasing");
  hb.trace_row0.assign(size_t(ntraces) + 1, 0);
  hb.trace_bytes0.assign(size_t(ntraces) + 1, 0);
  hb.row_trace.reserve(nsegs);
  std::vector<KeyBuild> kb;
  PageParse pp;
  for (uint32_t t = 0; t < ntraces; t++) {
    uint64_t tb = 0;
    for (uint64_t i = trace_seg[t]; i < trace_seg[t + 1]; i++) {
      const uint64_t len = seg_off[i + 1] - seg_off[i];
      // (entry.Reset reads the root offset: a segment shorter than 4 bytes panics the reference)
      if (len < 4) fail(TSG_E_CORRUPT, "live segment shorter than a flatbuffer root offset");
      pp = PageParse();
      pp.buf.assign(bytes + seg_off[i], bytes + seg_off[i + 1]);
      pp.fb_bytes = len;  // sr.AddBytesInspected(len(s))
      pp.nentries = 1;
      pp.tag_begin.push_back(0);
      FbTable e = FbTable::root(pp.buf.data(), pp.buf.size());
      std::unordered_map<uint32_t, uint32_t> memo;
      parse_entry(e, pp.buf.data(), 0, pp, memo);
      merge_page(hb, kb, pp);
      hb.row_trace.push_back(t);
      tb += len;
    }
    hb.trace_row0[t + 1] = hb.n;
    hb.trace_bytes0[t + 1] = hb.trace_bytes0[t] + tb;
  }
  for (auto &kc : hb.keys) kc.col.resize(hb.n, kNone);
  // TagValues (instance_search.go:229-240): FindTag on every segment. A row's key column
  // holds the set FindTag lands on for that key, so the values are those of the sets used.
  for (size_t k = 0; k < hb.keys.size(); k++) {
    const KeyColumn &kc = hb.keys[k];
    std::vector<uint8_t> used(kc.nsets(), 0);
    for (uint32_t c : kc.col)
      if (c != kNone) used[c] = 1;
    auto &dst = hb.stream_tags[kc.name];
    for (uint32_t s = 0; s < kc.nsets(); s++)
      if (used[s])
        for (uint32_t j = kc.set_off[s]; j < kc.set_off[s + 1]; j++) dst.insert(std::string(hb.dict_value(int(k), kc.set_vals[j])));
  }
  canonicalize_narrow_keys(hb);
}

}  // namespace tsg
