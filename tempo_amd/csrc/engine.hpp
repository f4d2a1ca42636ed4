// engine.hpp — device side of libtsg: per-device context, resident blocks and the
// search / lookup pipelines. The kernels live in engine.hip.
#pragma once
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "block.hpp"

namespace tsg {

// Scan columns (dur32, start_s, end_s, term value-set columns) are allocated to a
// multiple of kColPad entries so the scan kernels load whole tiles unconditionally.
constexpr uint64_t kColPad = 4096;

struct DevKey {
  std::string name;
  int width = 4;
  uint32_t nsetvals = 0;
  void *col = nullptr;  // n entries of `width` bytes; all-ones = key absent
  uint8_t *dict_bytes = nullptr;
  uint32_t *dict_off = nullptr;
  uint32_t nvals = 0;
  uint32_t *set_off = nullptr, *set_vals = nullptr;
  uint32_t nsets = 0;
  bool identity = true;
  uint64_t dict_nbytes = 0;
};

// Resident descriptors (device memory, written once at upload): the one-launch
// search path finds a block's columns and dictionaries through these.
struct DevKeyDesc {  // 64 B
  const void *col;
  const uint8_t *dict_bytes;  // allocation padded to whole words
  // dict_off starts the key's contiguous blob [dict_off | dict_bytes | set_off | set_vals]
  const uint32_t *dict_off, *set_off, *set_vals;
  uint32_t width, nvals, nsets, identity;
  uint32_t dict_nbytes, nsetvals;
};
struct DevBlockDesc {  // 128 B, followed by nkeys DevKeyDesc
  uint64_t n;
  const uint32_t *dur32;
  const uint64_t *dur64;
  const uint32_t *start_s, *end_s;
  const uint8_t *ids;
  const uint64_t *start_ns, *end_ns;
  const uint32_t *names;  // per entry: {root.service.name value id, root.name value id}, ~0u = absent
  const uint8_t *id_len;
  uint32_t nkeys, pad[11];
};
static_assert(sizeof(DevKeyDesc) == 64 && sizeof(DevBlockDesc) == 128, "descriptor layout");

// The dictionary of a narrow key (< 255 value sets, one-byte column) in canonical form
// (block.cpp canonicalize_narrow_keys), interned per context: blocks with the same
// values share one. A query matches it on the host once and hands the one-launch kernel
// the 256-bit value-set bitmap.
struct NarrowDict {
  std::vector<uint8_t> bytes;
  std::vector<uint32_t> off;                // nvals + 1
  std::vector<uint32_t> set_off, set_vals;  // value sets (CSR over value ids)
  bool identity = true;
  uint32_t nvals() const { return uint32_t(off.size() - 1); }
  uint32_t nsets() const { return uint32_t(set_off.size() - 1); }
  bool operator==(const NarrowDict &o) const {
    return bytes == o.bytes && off == o.off && set_off == o.set_off && set_vals == o.set_vals && identity == o.identity;
  }
};

// One backend search block resident in HBM (DESIGN.md "Data layout in HBM").
struct DevBlock {
  int device = 0;
  uint64_t n = 0;
  uint32_t *dur32 = nullptr;   // min(end-start, 2^32-1) (uint64 wrap kept, pitfall P2)
  uint64_t *dur64 = nullptr;   // exact end-start, read only when a threshold >= 2^32-1
  uint32_t *start_s = nullptr; // uint32(start/1e9)
  uint32_t *end_s = nullptr;   // uint32(end/1e9)
  uint8_t *ids = nullptr;      // n x 16, right aligned
  uint64_t *start_ns = nullptr, *end_ns = nullptr;
  uint32_t *names = nullptr;   // n x {svc vid, name vid}: record fields resolved on the host
  uint8_t *id_len = nullptr;
  const DevBlockDesc *desc = nullptr;
  // dur32 | start_s | end_s share one allocation, `npad` entries each; the one-byte key
  // columns share another, `npad` bytes per slot (narrow_slot[k], -1 for wider keys)
  uint64_t npad = 0;
  const uint8_t *narrow_base = nullptr;
  std::vector<int> narrow_slot;
  std::vector<DevKey> keys;
  uint64_t bytes = 0;
  std::vector<void *> allocs;
  std::vector<size_t> alloc_bytes;  // (same order as allocs)
};

struct DeviceCtx;

struct Block {
  // dictionaries/metadata kept on the host (names, header, page table); immutable after
  // open, shared by clones (tsg_block_clone copies only the device side)
  std::shared_ptr<HostBlock> host = std::make_shared<HostBlock>();
  DevBlock dev;
  DeviceCtx *dc = nullptr;
  std::vector<std::shared_ptr<const NarrowDict>> narrow;  // per key: interned dictionary (narrow keys)
};

struct Ctx {
  std::vector<DeviceCtx *> devs;  // owned; freed by ctx_shutdown
  std::mutex mu;
  std::mutex dmu;  // narrow-dictionary intern table (content hash -> live dictionaries)
  std::unordered_map<uint64_t, std::vector<std::weak_ptr<const NarrowDict>>> dicts;
};

void ctx_init(Ctx &c, const tsg_options *opts);
void ctx_shutdown(Ctx &c);
void block_upload(Ctx &c, Block &b, int device_hint);
// A second resident copy of an open block on device_hint's device (device-to-device
// copies of every column and dictionary, a descriptor of its own; host metadata shared
// by value): replicas for load balancing across GPUs, or disjoint copies of one data set.
void block_clone(Ctx &c, const Block &src, Block &dst, int device_hint);
void block_free(Block &b);

struct SearchOut {
  struct Rec {
    Rec() {}  // (not zero-filled: record arrays are resized to millions, then written once)
    uint8_t id[16];
    uint64_t start, end;
    uint32_t entry;
    uint32_t block_il;  // block index | id length << 24
    uint32_t svc, name; // value ids of root.service.name / root.name (~0u = absent)
  };
  std::vector<Rec> recs;  // ordered (before the limit cut across blocks)
  // A caller that takes scan positions (want_pos, set before device_search: a full scan whose
  // records are gathered from the blocks' host columns straight into the result arrays) may
  // get them instead of recs: compact set, pos[i] = entry | block index << 32, in record order
  bool want_pos = false, compact = false;
  RawVec<uint64_t> pos;
  std::vector<uint64_t> block_counts;
  uint64_t device_bytes = 0, kernel_ns = 0;
  uint64_t scan_ns = 0, scan_bytes = 0;
  uint32_t reruns = 0;  // extra launches after a record overflow (timed into scan_ns / kernel_ns when timing)
  bool pool = false;    // served by the pool kernels (they search entry ranges on the device)
  bool resident = false;  // served by the resident search kernel
  uint32_t path = 0;      // TSG_PATH_* bits of the kernels that served it (tsg_metrics.path)
  // (block index, term mask) for the blocks whose dictionaries the device pass matched
  // (prep / dict_stream / dict_sets): bit t clear = no value of the block's key for term t
  // contains the needle. MatchesBlock's tag half for keys with HostBlock::hdr_defer.
  std::vector<std::pair<uint32_t, uint32_t>> term_any;
};
// Runs the device pipeline for a set of (block index, block) pairs that share
// one device. limit 0 = every match; limit L = each block's first L matches.
int device_numa_node(const DeviceCtx &dc);
// ranges (optional, one per entry of `blocks`): search only scan positions [first, second)
// of that block (a limit query's progressive waves, tsg_search); records outside are dropped.
using EntryRanges = std::vector<std::pair<uint64_t, uint64_t>>;
void device_search(DeviceCtx &dc, const std::vector<std::pair<uint32_t, Block *>> &blocks, const tsg_query &q,
                   uint32_t limit, uint32_t flags, SearchOut &out, const EntryRanges *ranges = nullptr);

// ---- v2 lookup ---------------------------------------------------------------------
struct V2Block {
  int device = 0;
  DeviceCtx *dc = nullptr;
  // host meta
  uint8_t block_id[16];
  std::vector<uint8_t> min_id, max_id;
  int64_t start_unix = 0, end_unix = 0;
  uint32_t shards = 0;
  uint32_t total_records = 0;
  uint64_t bloom_m = 0, bloom_k = 0, bloom_bitlen = 0, bloom_words = 0;  // common across shards
  bool uniform = true;
  std::vector<uint64_t> shard_m, shard_k, shard_bitlen;
  // device
  uint64_t *d_bloom = nullptr;  // shards x words (host-endian u64)
  uint8_t *d_rec_ids = nullptr; // total_records x 16
  uint64_t *d_rec_start = nullptr;
  uint32_t *d_rec_len = nullptr;
  // index directory (lookup.hip d_post): the records share their first dir_cp id bytes
  // (dir_prefix); dir[b] = first record whose next 32 id bits, top dir_bits of them, are
  // >= b (2^dir_bits + 1 entries). Null when the index is short or not sorted.
  uint32_t *d_dir = nullptr;
  uint32_t dir_bits = 0, dir_cp = 0;
  uint8_t dir_prefix[16] = {};
  uint64_t *d_shard_m = nullptr, *d_shard_k = nullptr, *d_shard_bitlen = nullptr, *d_shard_woff = nullptr;
  // the data file (compressed pages) resident for findOne on the device; enc = meta.json
  // "encoding" (backend.Encoding)
  const uint8_t *d_data = nullptr;
  uint64_t data_len = 0;
  int enc = -1;
  std::vector<void *> allocs;
};
void v2block_open(Ctx &c, V2Block &b, const std::string &dir, int device_hint);
void v2block_free(V2Block &b);
// Pinned host memory, cached across calls (devctx.hip): a lookup's hit columns are copied
// from the device straight into it (no staging copy, no zero fill) and handed to the caller in
// its tsg_lookup_result; freed blocks go back to the cache for the next call.
void *pinned_get(size_t bytes);
void pinned_put(void *p, size_t bytes);
template <class T>
struct PinnedAlloc {
  using value_type = T;
  PinnedAlloc() = default;
  template <class U>
  PinnedAlloc(const PinnedAlloc<U> &) {}
  T *allocate(size_t n) { return static_cast<T *>(pinned_get(n * sizeof(T))); }
  void deallocate(T *p, size_t n) { pinned_put(p, n * sizeof(T)); }
  template <class U>
  void construct(U *p) {
    ::new (static_cast<void *>(p)) U;  // default-initialised: resize() writes nothing
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
  }
  template <class U>
  bool operator==(const PinnedAlloc<U> &) const { return true; }
  template <class U>
  bool operator!=(const PinnedAlloc<U> &) const { return false; }
};
template <class T>
using PinnedVec = std::vector<T, PinnedAlloc<T>>;
struct LookupOut {
  PinnedVec<uint32_t> id_idx, block_idx;
  PinnedVec<int32_t> rec;
  PinnedVec<uint64_t> start;
  PinnedVec<uint32_t> len;
  uint64_t kernel_ns = 0;
};
void device_lookup(DeviceCtx &dc, const std::vector<std::pair<uint32_t, V2Block *>> &blocks, const uint8_t (*ids)[16],
                   size_t nids, const tsg_lookup_opts *opts, LookupOut &out);
// tempodb.Find per (id, block): the lookup, then findOne on the device (find.hip)
struct FindOut {
  std::vector<uint32_t> id_idx, block_idx;
  std::vector<int32_t> status;      // TSG_OK found, TSG_E_NOT_FOUND, or the page's error
  std::vector<uint64_t> obj_off;    // into bytes
  std::vector<uint32_t> obj_len;
  std::vector<uint8_t> bytes;
  uint64_t kernel_ns = 0;
};
void device_find(DeviceCtx &dc, const std::vector<std::pair<uint32_t, V2Block *>> &blocks, const uint8_t (*ids)[16],
                 size_t nids, const tsg_lookup_opts *opts, FindOut &out);

int device_ordinal(const DeviceCtx &dc);
// resident search counters: launches, queries served, relaunches after an idle-exit race, quits
void device_counters(DeviceCtx &dc, uint64_t out[8]);
// The last full scan on the device's dictionary-pass path had more than one match per 64
// entries (search.hip: its next full scans there return bitmaps; tsg_search pipelines them)
bool device_last_dense(DeviceCtx &dc);
// Durations of the TSG_SEARCH_TIME_DEFER launches since the last call (waits for the stream).
void device_kernel_times(DeviceCtx &dc, std::vector<uint64_t> &ns);
// tsg_search_batch (pool.hip): begin ends the device's resident launch and gives the next one
// dispatch timestamps (returns the launch count so far); end ends that launch and returns its
// dispatch duration (ns) when exactly one launch served the batch's resident queries, else 0
uint64_t resident_batch_begin(DeviceCtx &dc);
uint64_t resident_batch_end(DeviceCtx &dc, uint64_t launches_before);
// test hooks (tsg_debug_set): "res_torn", "groups" (search launches plan for this many CUs:
// e.g. 8 makes a resident query of 6 M entries run > 1536 units per workgroup), "xsplit"
// (0/1: the resident kernel's XCD-weighted split; default TSG_RES_XSPLIT, 0)
int debug_set(const char *name, int64_t value);
uint32_t debug_groups();
uint32_t debug_lb_bitmap();  // "lb_bitmap": 0 never / 1 always / 2 auto (TSG_LB_BITMAP, default 2)
bool debug_xsplit();

}  // namespace tsg
