// devctx.hip — device contexts, HBM residency of search blocks (host code using the
// HIP runtime; the search kernels are in search.hip, the lookup kernels in lookup.hip).
#include <cctype>
#include <cstdio>
#include <string>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <new>
#include <unordered_map>

#include "aql.hpp"
#include "devctx.hpp"

namespace tsg {

int device_ordinal(const DeviceCtx &dc) { return dc.ordinal; }

// ---- cached pinned host blocks (PinnedAlloc) ----------------------------------------------
// A block is reused for a request of at least half its size; sizes round up to 1 MiB. At most
// kPinnedCache bytes stay cached (pinning and unpinning hundreds of MB costs milliseconds).
static std::mutex g_pin_mu;
static std::multimap<size_t, void *> g_pin_free;  // capacity -> block
static size_t g_pin_cached = 0;
static std::unordered_map<void *, size_t> g_pin_cap;
constexpr size_t kPinnedCache = size_t(2) << 30;
void *pinned_get(size_t bytes) {
  if (bytes == 0) bytes = 1;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_free.lower_bound(bytes);
    if (it != g_pin_free.end() && it->first / 2 <= bytes) {
      void *p = it->second;
      g_pin_cached -= it->first;
      g_pin_free.erase(it);
      return p;
    }
  }
  const size_t cap = (bytes + (size_t(1) << 20) - 1) & ~((size_t(1) << 20) - 1);
  void *p = nullptr;
  if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess || !p) throw std::bad_alloc();
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_cap[p] = cap;
  return p;
}
void pinned_put(void *p, size_t) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  const size_t cap = g_pin_cap[p];
  g_pin_free.emplace(cap, p);
  g_pin_cached += cap;
  while (g_pin_cached > kPinnedCache && !g_pin_free.empty()) {  // (the smallest go first)
    auto it = g_pin_free.begin();
    g_pin_cached -= it->first;
    g_pin_cap.erase(it->second);
    (void)hipHostFree(it->second);
    g_pin_free.erase(it);
  }
}
void device_counters(DeviceCtx &dc, uint64_t out[8]) {
  std::lock_guard<std::mutex> lk(dc.mu);
  out[0] = dc.res_launches;
  out[1] = dc.res_queries;
  out[2] = dc.res_relaunches;
  out[3] = dc.res_quits;
  out[4] = dc.res_rejects;
  out[5] = dc.res_cotenant_queries;
  out[6] = dc.res_plain_queries;
  out[7] = dc.res_xsamples;
}

void ctx_init(Ctx &c, const tsg_options *opts) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) fail(TSG_E_DEVICE, "no HIP device visible (libtsg has no CPU path)");
  std::vector<int> ords;
  if (opts && opts->devices && opts->num_devices > 0) {
    for (int i = 0; i < opts->num_devices; i++) ords.push_back(opts->devices[i]);
  } else {
    int m = (opts && opts->num_devices > 0) ? std::min(opts->num_devices, n) : n;
    for (int i = 0; i < m; i++) ords.push_back(i);
  }
  for (int o : ords) {
    if (o < 0 || o >= n) fail(TSG_E_INVALID, "device ordinal out of range");
    auto dc = std::make_unique<DeviceCtx>();
    dc->ordinal = o;
    HIP_OK(hipSetDevice(o));
    HIP_OK(hipStreamCreateWithFlags(&dc->stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreate(&dc->ev0));
    HIP_OK(hipEventCreate(&dc->ev1));
    // scan timing events: no system-scope fence (no L2 writeback between kernels)
    HIP_OK(hipEventCreateWithFlags(&dc->es0, hipEventDisableSystemFence));
    HIP_OK(hipEventCreateWithFlags(&dc->es1, hipEventDisableSystemFence));
    HIP_OK(hipEventCreateWithFlags(&dc->er0, hipEventDisableSystemFence));  // (rerun launches)
    HIP_OK(hipEventCreateWithFlags(&dc->er1, hipEventDisableSystemFence));
    HIP_OK(hipEventCreateWithFlags(&dc->mk0, hipEventDisableTiming | hipEventDisableSystemFence));
    HIP_OK(hipEventCreateWithFlags(&dc->mk1, hipEventDisableTiming | hipEventDisableSystemFence));
    dc->ticket.ensure(64);
    HIP_OK(hipMemset(dc->ticket.p, 0, 64));
    dc->err.ensure(64);
    HIP_OK(hipMemset(dc->err.p, 0, 64));
    context_opened(*dc);
    c.devs.push_back(dc.release());
  }
}

void ctx_shutdown(Ctx &c) {
  for (auto &dc : c.devs) {
    (void)hipSetDevice(dc->ordinal);
    (void)hipStreamSynchronize(dc->stream);
    context_closed(*dc);
    try {
      std::lock_guard<std::mutex> lk(dc->mu);
      resident_release(*dc);  // (its launch leaves before the queue is closed)
    } catch (...) {
    }
    aql_close(dc->aql);  // (waits for its queue to drain)
    dc->aql = nullptr;
    for (DevBuf *b : {&dc->desc, &dc->vmatch, &dc->bitmaps, &dc->gran, &dc->ticket, &dc->out, &dc->regions,
                      &dc->seg_counts, &dc->hdr, &dc->err, &dc->maskbits, &dc->agg, &dc->stamps, &dc->gbm, &dc->lkhits,
                      &dc->done, &dc->steal, &dc->fpages, &dc->fhits, &dc->fres, &dc->farena, &dc->fcrc, &dc->fdst, &dc->foff,
                      &dc->danyf, &dc->pool_head, &dc->lkslab, &dc->lkslabdesc, &dc->pbm, &dc->pout})
      b->release();
    for (hipEvent_t e : dc->tring) (void)hipEventDestroy(e);
    dc->hdesc.release();
    dc->hout.release();
    dc->lkstage.release();
    for (auto &e : dc->lk_ev)
      if (e) (void)hipEventDestroy(e);
    dc->hres.release();
    dc->hany.release();
    dc->hbits.release();
    (void)hipEventDestroy(dc->ev0);
    (void)hipEventDestroy(dc->ev1);
    (void)hipEventDestroy(dc->es0);
    (void)hipEventDestroy(dc->mk0);
    (void)hipEventDestroy(dc->er0);
    (void)hipEventDestroy(dc->er1);
    (void)hipEventDestroy(dc->mk1);
    (void)hipEventDestroy(dc->es1);
    (void)hipStreamDestroy(dc->stream);
    delete dc;
  }
  c.devs.clear();
}

// pad_to: allocate a multiple of that many elements (scan columns: kColPad) and
// zero the tail, so whole-tile loads past the last entry stay in bounds.
template <typename T>
static T *dev_upload(DevBlock &b, const T *src, size_t count, hipStream_t s, size_t pad_to = 1) {
  void *p = nullptr;
  const size_t elems = (count + pad_to - 1) / pad_to * pad_to;
  // whole 16-byte words: kernels may read a dictionary's last bytes as a word
  size_t bytes = std::max<size_t>((elems * sizeof(T) + 15) / 16 * 16, 16);
  HIP_OK(hipMalloc(&p, bytes));
  b.allocs.push_back(p);
  b.alloc_bytes.push_back(bytes);
  b.bytes += bytes;
  if (count) HIP_OK(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s));
  if (bytes > count * sizeof(T))
    HIP_OK(hipMemsetAsync(static_cast<uint8_t *>(p) + count * sizeof(T), 0, bytes - count * sizeof(T), s));
  return static_cast<T *>(p);
}

// count zeroed elements (whole 16-byte words), filled by the caller's copies
template <typename T>
static T *dev_zeroed(DevBlock &b, size_t count, hipStream_t s) {
  void *p = nullptr;
  const size_t bytes = std::max<size_t>((count * sizeof(T) + 15) / 16 * 16, 16);
  HIP_OK(hipMalloc(&p, bytes));
  b.allocs.push_back(p);
  b.alloc_bytes.push_back(bytes);
  b.bytes += bytes;
  HIP_OK(hipMemsetAsync(p, 0, bytes, s));
  return static_cast<T *>(p);
}

static void upload_desc(DevBlock &d, hipStream_t s);

// One interned copy per distinct narrow dictionary (content-equal dictionaries of
// different blocks share it; entries of closed blocks expire).
static std::shared_ptr<const NarrowDict> intern_narrow(Ctx &c, NarrowDict &&nd) {
  auto hv = [](const auto &v) { return xxhash64(reinterpret_cast<const uint8_t *>(v.data()), v.size() * sizeof(v[0])); };
  const uint64_t h = hv(nd.bytes) ^ (hv(nd.off) * 31) ^ (hv(nd.set_off) * 131) ^ (hv(nd.set_vals) * 1313);
  std::lock_guard<std::mutex> lk(c.dmu);
  auto &vec = c.dicts[h];
  vec.erase(std::remove_if(vec.begin(), vec.end(), [](const auto &w) { return w.expired(); }), vec.end());
  for (auto &w : vec)
    if (auto p = w.lock())
      if (*p == nd) return p;
  auto p = std::make_shared<const NarrowDict>(std::move(nd));
  vec.push_back(p);
  return p;
}

void block_upload(Ctx &c, Block &b, int device_hint) {
  if (c.devs.empty()) fail(TSG_E_DEVICE, "no device");
  DeviceCtx &dc = *c.devs[size_t(std::max(device_hint, 0)) % c.devs.size()];
  b.dc = &dc;
  DevBlock &d = b.dev;
  const HostBlock &h = *b.host;
  d.device = dc.ordinal;
  d.n = h.n;
  size_t n = h.n;
  // Every host-side array is built first, without the device lock (blocks opened together
  // prepare theirs concurrently); the lock is held for the allocations and copies only.
  // [dur32 | start_s | end_s | ds], npad entries each (whole tiles: kColPad), one allocation.
  // ds, the pool kernels' compact form of the other three (4 B where they read 12):
  //   bits 0..15  D16 = 2 * floor(dur / 1 ms) + (dur % 1 ms != 0), saturated at 0xffff: for whole-
  //               ms bounds m, M <= kDs16MaxMs, dur >= m ms <=> D16 >= 2m and dur <= M ms <=> D16 <= 2M
  //               (a saturated entry has dur >= 32767 ms: above every such M, not below any m)
  //   bits 16..31 end_s - start_s when it fits below 0xffff, else 0xffff (the kernel then reads end_s)
  const size_t npad = (std::max<size_t>(n, 1) + kColPad - 1) / kColPad * kColPad;
  d.npad = npad;
  std::vector<uint32_t> scan(4 * npad, 0);
  std::vector<uint64_t> dur64(n);
  for (size_t i = 0; i < n; i++) {
    uint64_t dd = h.end[i] - h.start[i];  // uint64 wrap (pitfall P2)
    dur64[i] = dd;
    scan[i] = dd >= 0xffffffffULL ? 0xffffffffu : uint32_t(dd);
    const uint32_t ss = uint32_t(h.start[i] / 1000000000ULL), es = uint32_t(h.end[i] / 1000000000ULL);
    scan[npad + i] = ss;
    scan[2 * npad + i] = es;
    const uint64_t q = dd / 1000000ULL;
    const uint64_t d16 = q >= 0x8000ULL ? 0xffffULL : std::min<uint64_t>(2 * q + (dd % 1000000ULL != 0), 0xffffULL);
    const uint32_t span = es - ss;  // (uint32: an end before the start wraps to a large value)
    scan[3 * npad + i] = uint32_t(d16) | (span < 0xffffu ? span : 0xffffu) << 16;
  }
  // one-byte key columns: one allocation, npad bytes per narrow key
  d.narrow_slot.assign(h.keys.size(), -1);
  int nn = 0;
  for (size_t k = 0; k < h.keys.size(); k++)
    if (h.keys[k].width() == 1) d.narrow_slot[k] = nn++;
  std::vector<uint8_t> ncol(std::max<size_t>(size_t(nn), 1) * npad, 0xff);
  for (size_t k = 0; k < h.keys.size(); k++) {
    if (d.narrow_slot[k] < 0) continue;
    uint8_t *dst = ncol.data() + size_t(d.narrow_slot[k]) * npad;
    const auto &col = h.keys[k].col;
    for (size_t i = 0; i < n; i++) dst[i] = col[i] == kNone ? 0xff : uint8_t(col[i]);
  }
  b.narrow.assign(h.keys.size(), nullptr);
  for (size_t k = 0; k < h.keys.size(); k++) {
    if (d.narrow_slot[k] < 0) continue;
    const KeyColumn &kc = h.keys[k];
    NarrowDict nd;
    nd.bytes.assign(kc.dict_bytes.begin(), kc.dict_bytes.end());
    nd.off = kc.dict_off;
    nd.set_off = kc.set_off;
    nd.set_vals = kc.set_vals;
    nd.identity = kc.identity;
    b.narrow[k] = intern_narrow(c, std::move(nd));
  }
  std::vector<uint32_t> names(2 * n);
  for (size_t i = 0; i < n; i++) {
    names[2 * i] = h.svc_vid.empty() ? kNone : h.svc_vid[i];
    names[2 * i + 1] = h.name_vid.empty() ? kNone : h.name_vid[i];
  }
  // per key: its 16-bit column (width 2) and one contiguous blob in the order a workgroup
  // stages it into LDS: [value offsets nvals+1 | value bytes (whole words) | set offsets
  // nsets+1 | set values] (set arrays only for non-identity keys). The blob is assembled on
  // the device from the key's own arrays (config 4's statement dictionary is ~1 GB: building
  // it on the host first was a zero fill and a copy of that much)
  const size_t nk = h.keys.size();
  std::vector<std::vector<uint16_t>> col16(nk);
  for (size_t k = 0; k < nk; k++) {
    const KeyColumn &kc = h.keys[k];
    if (kc.width() == 2) {
      col16[k].resize(n);
      for (size_t i = 0; i < n; i++) col16[k][i] = kc.col[i] == kNone ? 0xffff : uint16_t(kc.col[i]);
    }
  }

  std::lock_guard<std::mutex> lk(dc.mu);
  dc.mem_epoch++;  // (a resident search launch relaunches before it reads new columns)
  // the resident launch holds every CU: the stream work below (the zero fill of the dictionary
  // blobs is a kernel) would wait for its idle exit
  resident_quit(dc);
  HIP_OK(hipSetDevice(dc.ordinal));
  hipStream_t s = dc.stream;
  d.dur32 = dev_upload(d, scan.data(), scan.size(), s);
  d.start_s = d.dur32 + npad;
  d.end_s = d.dur32 + 2 * npad;
  d.dur64 = dev_upload(d, dur64.data(), n, s);
  d.narrow_base = dev_upload(d, ncol.data(), ncol.size(), s);
  d.ids = dev_upload(d, h.ids.data(), n * 16, s);
  d.start_ns = dev_upload(d, h.start.data(), n, s);
  d.end_ns = dev_upload(d, h.end.data(), n, s);
  d.names = dev_upload(d, names.data(), 2 * n, s);
  d.id_len = dev_upload(d, h.id_len.data(), n, s);
  for (size_t kk = 0; kk < nk; kk++) {
    const KeyColumn &kc = h.keys[kk];
    DevKey k;
    k.name = kc.name;
    k.width = kc.width();
    k.nvals = kc.nvals();
    k.nsets = kc.nsets();
    k.identity = kc.identity;
    if (k.width == 1) {
      k.col = const_cast<uint8_t *>(d.narrow_base) + size_t(d.narrow_slot[kk]) * npad;
    } else if (k.width == 2) {
      k.col = dev_upload(d, col16[kk].data(), n, s, kColPad);
    } else {
      k.col = dev_upload(d, kc.col.data(), n, s, kColPad);
    }
    const size_t bw = (kc.dict_bytes.size() + 3) / 4;
    const size_t nso = kc.identity ? 0 : kc.set_off.size(), nsv = kc.identity ? 0 : kc.set_vals.size();
    uint32_t *dblob = dev_zeroed<uint32_t>(d, kc.dict_off.size() + bw + nso + nsv, s);
    auto put = [&](uint32_t *dst, const void *src, size_t bytes) {
      if (bytes) HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    };
    put(dblob, kc.dict_off.data(), kc.dict_off.size() * 4);
    put(dblob + kc.dict_off.size(), kc.dict_bytes.data(), kc.dict_bytes.size());
    if (nso) put(dblob + kc.dict_off.size() + bw, kc.set_off.data(), nso * 4);
    if (nsv) put(dblob + kc.dict_off.size() + bw + nso, kc.set_vals.data(), nsv * 4);
    k.dict_off = dblob;
    k.dict_bytes = reinterpret_cast<uint8_t *>(dblob + kc.dict_off.size());
    k.dict_nbytes = kc.dict_bytes.size();
    if (!kc.identity) {
      k.set_off = dblob + kc.dict_off.size() + bw;
      k.set_vals = k.set_off + nso;
      k.nsetvals = uint32_t(nsv);
    }
    d.keys.push_back(k);
  }
  // the staging vectors must outlive the async copies
  HIP_OK(hipStreamSynchronize(s));
  upload_desc(d, s);
}

// resident descriptor (one-launch search path): the block's column and dictionary pointers
static void upload_desc(DevBlock &d, hipStream_t s) {
  const uint64_t n = d.n;
  std::vector<uint8_t> desc(sizeof(DevBlockDesc) + d.keys.size() * sizeof(DevKeyDesc));
  auto *bd = reinterpret_cast<DevBlockDesc *>(desc.data());
  bd->n = n;
  bd->dur32 = d.dur32;
  bd->dur64 = d.dur64;
  bd->start_s = d.start_s;
  bd->end_s = d.end_s;
  bd->ids = d.ids;
  bd->start_ns = d.start_ns;
  bd->end_ns = d.end_ns;
  bd->names = d.names;
  bd->id_len = d.id_len;
  bd->nkeys = uint32_t(d.keys.size());
  auto *kd = reinterpret_cast<DevKeyDesc *>(bd + 1);
  for (size_t i = 0; i < d.keys.size(); i++) {
    const DevKey &k = d.keys[i];
    kd[i].col = k.col;
    kd[i].dict_bytes = k.dict_bytes;
    kd[i].dict_off = k.dict_off;
    kd[i].set_off = k.set_off;
    kd[i].set_vals = k.set_vals;
    kd[i].width = uint32_t(k.width);
    kd[i].nvals = k.nvals;
    kd[i].nsets = k.nsets;
    kd[i].identity = k.identity ? 1u : 0u;
    kd[i].dict_nbytes = uint32_t(std::min<uint64_t>(k.dict_nbytes, 0xffffffffu));
    kd[i].nsetvals = k.nsetvals;
  }
  d.desc = reinterpret_cast<const DevBlockDesc *>(dev_upload(d, desc.data(), desc.size(), s));
  HIP_OK(hipStreamSynchronize(s));
}

void block_clone(Ctx &c, const Block &src, Block &dst, int device_hint) {
  if (c.devs.empty()) fail(TSG_E_DEVICE, "no device");
  if (!src.dc) fail(TSG_E_INVALID, "block_clone: source block is not resident");
  DeviceCtx &dc = *c.devs[size_t(std::max(device_hint, 0)) % c.devs.size()];
  dst.host = src.host;  // (shared: the host side is immutable after open)
  dst.dc = &dc;
  DevBlock &d = dst.dev;
  const DevBlock &o = src.dev;
  d = DevBlock();
  d.device = dc.ordinal;
  d.n = o.n;
  std::lock_guard<std::mutex> lk(dc.mu);
  dc.mem_epoch++;
  resident_quit(dc);  // (as block_upload)
  HIP_OK(hipSetDevice(dc.ordinal));
  // the descriptor allocation (last) is rebuilt, every other one copied
  const size_t ncopy = o.allocs.empty() ? 0 : o.allocs.size() - 1;
  for (size_t i = 0; i < ncopy; i++) {
    void *p = nullptr;
    HIP_OK(hipMalloc(&p, o.alloc_bytes[i]));
    d.allocs.push_back(p);
    d.alloc_bytes.push_back(o.alloc_bytes[i]);
    d.bytes += o.alloc_bytes[i];
    // (hipMemcpyPeer semantics: a plain device-to-device copy works across devices too)
    HIP_OK(hipMemcpyAsync(p, o.allocs[i], o.alloc_bytes[i], hipMemcpyDeviceToDevice, dc.stream));
  }
  auto xl = [&](const void *q) -> void * {  // source pointer -> the same byte of the copy
    if (!q) return nullptr;
    for (size_t i = 0; i < ncopy; i++) {
      const uint8_t *a = static_cast<const uint8_t *>(o.allocs[i]);
      if (static_cast<const uint8_t *>(q) >= a && static_cast<const uint8_t *>(q) < a + o.alloc_bytes[i])
        return static_cast<uint8_t *>(d.allocs[i]) + (static_cast<const uint8_t *>(q) - a);
    }
    fail(TSG_E_INVALID, "block_clone: pointer outside the block's allocations");
  };
  d.dur32 = static_cast<uint32_t *>(xl(o.dur32));
  d.dur64 = static_cast<uint64_t *>(xl(o.dur64));
  d.start_s = static_cast<uint32_t *>(xl(o.start_s));
  d.end_s = static_cast<uint32_t *>(xl(o.end_s));
  d.ids = static_cast<uint8_t *>(xl(o.ids));
  d.start_ns = static_cast<uint64_t *>(xl(o.start_ns));
  d.end_ns = static_cast<uint64_t *>(xl(o.end_ns));
  d.names = static_cast<uint32_t *>(xl(o.names));
  d.id_len = static_cast<uint8_t *>(xl(o.id_len));
  d.npad = o.npad;
  d.narrow_base = static_cast<const uint8_t *>(xl(o.narrow_base));
  d.narrow_slot = o.narrow_slot;
  dst.narrow = src.narrow;
  for (const DevKey &k0 : o.keys) {
    DevKey k = k0;
    k.col = xl(k0.col);
    k.dict_off = static_cast<uint32_t *>(xl(k0.dict_off));
    k.dict_bytes = static_cast<uint8_t *>(xl(k0.dict_bytes));
    k.set_off = static_cast<uint32_t *>(xl(k0.set_off));
    k.set_vals = static_cast<uint32_t *>(xl(k0.set_vals));
    d.keys.push_back(k);
  }
  upload_desc(d, dc.stream);
}

void block_free(Block &b) {
  if (!b.dc) return;
  std::lock_guard<std::mutex> lk(b.dc->mu);
  b.dc->mem_epoch++;
  try {
    resident_quit(*b.dc);  // (no launch reads the columns after they are freed)
  } catch (...) {
  }
  (void)hipSetDevice(b.dc->ordinal);
  (void)hipStreamSynchronize(b.dc->stream);
  for (void *p : b.dev.allocs) (void)hipFree(p);
  b.dev.allocs.clear();
  b.dc = nullptr;
}

}  // namespace tsg

namespace tsg {
int device_numa_node(const DeviceCtx &dc) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, dc.ordinal) != hipSuccess) return -1;
  for (char *c = bus; *c; c++) *c = char(std::tolower(uint8_t(*c)));
  std::FILE *f = std::fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}
}  // namespace tsg
