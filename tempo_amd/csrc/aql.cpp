// aql.cpp — see aql.hpp.
#include "aql.hpp"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <mutex>
#include <string>
#include <unordered_map>

namespace tsg {

static constexpr uint32_t kSlotsDecl = 64;
struct Aql {
  hsa_agent_t agent{};
  hsa_queue_t *queue = nullptr;
  hsa_code_object_reader_t reader{};
  hsa_executable_t exe{};
  std::string code;
  uint8_t *kargs = nullptr;  // kSlots x kSlotBytes of device memory the host writes through the BAR
  uint32_t next = 0;
  // completion signals: a ring for the plain dispatches (one per dispatch, set to 1 before it;
  // reused kSlots dispatches later) and one per profiled dispatch until aql_time_reset
  hsa_signal_t ring[kSlotsDecl]{};
  std::vector<hsa_signal_t> prof;
  size_t prof_used = 0;
  hsa_signal_t last{0};
  double ns_per_tick = 1.0;
  std::unordered_map<std::string, AqlKernel> kernels;
  // the HDP flush register (hsa_amd_hdp_flush_t): host writes through the BAR pass the GPU's
  // host data path, which buffers them; a write to this register pushes them to memory
  volatile uint32_t *hdp_flush = nullptr;
};

static constexpr uint32_t kSlots = 64, kSlotBytes = 8192;

static bool trace_on() {
  static const bool t = std::getenv("TSG_TRACE") != nullptr;
  return t;
}
static void note(const char *what) {
  if (trace_on()) std::fprintf(stderr, "[tsg] aql: %s (HIP launches instead)\n", what);
}

static std::string lib_dir() {
  Dl_info info{};
  if (!dladdr(reinterpret_cast<void *>(&aql_open), &info) || !info.dli_fname) return ".";
  std::string p(info.dli_fname);
  const size_t k = p.rfind('/');
  return k == std::string::npos ? "." : p.substr(0, k);
}

Aql *aql_open(int hip_ordinal) {
  const char *e = std::getenv("TSG_AQL");
  if (e && std::atoi(e) == 0) return nullptr;
  // (TSG_POOL_CO: another build of the same kernels, for A/B measurements)
  const char *alt = std::getenv("TSG_POOL_CO");
  std::ifstream in(alt && *alt ? std::string(alt) : lib_dir() + "/libtsg_pool.co", std::ios::binary);
  if (!in) {
    note("no libtsg_pool.co beside libtsg.so");
    return nullptr;
  }
  auto *a = new Aql;
  a->code.assign((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  int bus = -1, dev = -1, dom = -1;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, hip_ordinal) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, hip_ordinal) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, hip_ordinal) != hipSuccess) {
    note("no PCI location for the device");
    delete a;
    return nullptr;
  }
  auto fail = [&](const char *what) -> Aql * {
    note(what);
    aql_close(a);
    return nullptr;
  };
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    delete a;
    note("hsa_init");
    return nullptr;
  }
  struct Find {
    uint32_t bdf;
    hsa_agent_t agent;
    bool found;
  } f{uint32_t((bus << 8) | (dev << 3)), {}, false};
  hsa_iterate_agents([](hsa_agent_t ag, void *d) {
    auto *F = static_cast<Find *>(d);
    hsa_device_type_t t;
    if (hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
      return HSA_STATUS_SUCCESS;
    uint32_t bdf = 0;
    if (hsa_agent_get_info(ag, hsa_agent_info_t(HSA_AMD_AGENT_INFO_BDFID), &bdf) == HSA_STATUS_SUCCESS && bdf == F->bdf) {
      F->agent = ag;
      F->found = true;
      return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
  }, &f);
  if (!f.found) return fail("no HSA agent at the device's PCI location");
  a->agent = f.agent;
  // the argument slots are written by the host through the BAR: only a large-BAR device maps
  // all of VRAM for the host; otherwise HIP launches
  int large_bar = 0;
  if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, hip_ordinal) != hipSuccess || !large_bar)
    return fail("not a large-BAR device (argument slots not host-writable)");
  hsa_amd_hdp_flush_t hdp{};
  if (hsa_agent_get_info(a->agent, hsa_agent_info_t(HSA_AMD_AGENT_INFO_HDP_FLUSH), &hdp) == HSA_STATUS_SUCCESS)
    a->hdp_flush = hdp.HDP_MEM_FLUSH_CNTL;
  if (hsa_code_object_reader_create_from_memory(a->code.data(), a->code.size(), &a->reader) != HSA_STATUS_SUCCESS)
    return fail("code object reader");
  if (hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &a->exe) !=
      HSA_STATUS_SUCCESS)
    return fail("executable");
  if (hsa_executable_load_agent_code_object(a->exe, a->agent, a->reader, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
      hsa_executable_freeze(a->exe, nullptr) != HSA_STATUS_SUCCESS)
    return fail("code object load");
  if (hsa_queue_create(a->agent, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &a->queue) !=
      HSA_STATUS_SUCCESS)
    return fail("queue");
  for (auto &sg : a->ring)
    if (hsa_signal_create(0, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) return fail("signal");
  if (hsa_amd_profiling_set_profiler_enabled(a->queue, 1) != HSA_STATUS_SUCCESS) return fail("queue profiling");
  uint64_t freq = 0;
  if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq) == HSA_STATUS_SUCCESS && freq)
    a->ns_per_tick = 1e9 / double(freq);
  // argument slots in device memory (as HIP keeps kernel arguments), written through the BAR;
  // zeroed once (the kernels read only the parts a launch writes)
  void *p = nullptr;
  if (hipExtMallocWithFlags(&p, size_t(kSlots) * kSlotBytes, hipDeviceMallocUncached) != hipSuccess)
    return fail("argument slots");
  a->kargs = static_cast<uint8_t *>(p);
  if (hipMemset(p, 0, size_t(kSlots) * kSlotBytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fail("argument slots init");
  return a;
}

void aql_close(Aql *a) {
  if (!a) return;
  if (a->queue) {  // every packet processed (bounded: ~1 s)
    for (int i = 0; i < 1000000 && hsa_queue_load_read_index_scacquire(a->queue) <
                                       hsa_queue_load_write_index_relaxed(a->queue); i++) {
      struct timespec ts{0, 1000};
      nanosleep(&ts, nullptr);
    }
  }
  if (a->kargs) (void)hipFree(a->kargs);
  for (auto &sg : a->ring)
    if (sg.handle) hsa_signal_destroy(sg);
  for (auto &sg : a->prof) hsa_signal_destroy(sg);
  if (a->queue) hsa_queue_destroy(a->queue);
  if (a->exe.handle) hsa_executable_destroy(a->exe);
  if (a->reader.handle) hsa_code_object_reader_destroy(a->reader);
  delete a;
}

AqlKernel aql_kernel(Aql *a, const char *name, uint32_t max_kernarg) {
  if (!a) return {};
  auto it = a->kernels.find(name);
  if (it != a->kernels.end()) return it->second;
  AqlKernel k;
  hsa_executable_symbol_t sym;
  const std::string kd = std::string(name) + ".kd";
  if (hsa_executable_get_symbol_by_name(a->exe, kd.c_str(), &a->agent, &sym) == HSA_STATUS_SUCCESS) {
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.kobj);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg);
    // the slot holds the kernel's own argument struct and nothing else: a kernel that reads
    // implicit arguments (blockDim / gridDim, printf: hidden arguments past the struct under
    // code object v5) would read unwritten bytes, so it launches through HIP
    if (k.kernarg > kSlotBytes || k.kernarg > max_kernarg) {
      k.kobj = 0;
      note("kernel reads implicit arguments (kernarg segment larger than its argument struct)");
    }
  } else {
    note("kernel symbol missing from the code object");
  }
  a->kernels.emplace(name, k);
  return k;
}

int aql_dispatch(Aql *a, const AqlKernel &k, uint32_t grid, uint32_t block, uint32_t dyn_lds, const void *args,
                 const std::vector<std::pair<uint32_t, uint32_t>> &parts, bool profiled) {
  static_assert(kSlotsDecl == kSlots, "signal ring = argument slots");
  const uint32_t si = a->next++ % kSlots;
  uint8_t *slot = a->kargs + size_t(si) * kSlotBytes;
  int pslot = -1;
  hsa_signal_t sig = a->ring[si];
  if (profiled) {
    constexpr size_t kMaxProf = 4096;
    if (a->prof_used == a->prof.size() && a->prof.size() < kMaxProf) {
      hsa_signal_t x{};
      if (hsa_signal_create(0, 0, nullptr, &x) == HSA_STATUS_SUCCESS) a->prof.push_back(x);
    }
    if (a->prof_used < a->prof.size()) {
      pslot = int(a->prof_used++);
      sig = a->prof[size_t(pslot)];
    }
  }
  const auto *src = static_cast<const uint8_t *>(args);
  uint32_t last = 0;
  for (const auto &pt : parts) {
    std::memcpy(slot + pt.first, src + pt.first, pt.second);
    last = pt.first + pt.second;
  }
  // The argument words must be in device memory before the kernel's waves load them. The
  // BAR stores are write-combined (sfence drains them onto the bus); on the device they pass
  // the host data path (HDP), which buffers host writes, and the doorbell reaches the command
  // processor on another path. Default (TSG_AQL_FENCE=hdp): write the HDP flush register and
  // read it back — the read returns after the flush, so every argument word is in memory
  // before the doorbell is rung (HIP flushes the same way before a launch whose
  // arguments live in device memory). `readback`: read the last argument word back instead;
  // `sfence`: posted-write order only (opt-in, measured faster, not guaranteed).
  static const int mode = [] {
    const char *e = std::getenv("TSG_AQL_FENCE");
    if (e && !std::strcmp(e, "sfence")) return 0;
    if (e && !std::strcmp(e, "readback")) return 1;
    if (const char *r = std::getenv("TSG_AQL_READBACK"); r && std::atoi(r) != 0) return 1;
    return 2;
  }();
  __builtin_ia32_sfence();
  if (mode == 2 && a->hdp_flush) {
    *a->hdp_flush = 1u;
    (void)*a->hdp_flush;
  } else if (mode >= 1) {
    (void)*reinterpret_cast<volatile uint32_t *>(slot + ((last - 1) & ~3u));
  }
  hsa_queue_t *q = a->queue;
  const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
  while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
  }  // (never: every launch completes before its caller returns)
  auto *pk = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx & (q->size - 1));
  pk->workgroup_size_x = uint16_t(block);
  pk->workgroup_size_y = 1;
  pk->workgroup_size_z = 1;
  pk->reserved0 = 0;
  pk->grid_size_x = grid * block;
  pk->grid_size_y = 1;
  pk->grid_size_z = 1;
  pk->private_segment_size = k.priv;
  pk->group_segment_size = k.group + dyn_lds;
  pk->kernel_object = k.kobj;
  pk->kernarg_address = slot;
  pk->reserved2 = 0;
  // (a signal of this dispatch's own: one shared signal reset to 1 here could be taken to 0 by
  // the previous dispatch's late completion while this one still runs)
  hsa_signal_store_relaxed(sig, 1);
  pk->completion_signal = sig;
  a->last = sig;
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  // agent-scope fences: the argument slots are uncached device memory, the search kernels
  // write their host results with system-scope stores of their own (a system-scope acquire
  // would also invalidate the L2 at every launch)
  static const int scope = [] {
    const char *e = std::getenv("TSG_AQL_SCOPE");
    return e ? std::atoi(e) : int(HSA_FENCE_SCOPE_AGENT);
  }();
  const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                       (scope << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                       (scope << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  __atomic_store_n(reinterpret_cast<uint32_t *>(pk), uint32_t(hdr) | (uint32_t(setup) << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, hsa_signal_value_t(idx));
  return pslot;
}

void aql_hdp_flush(Aql *a) {
  if (a && a->hdp_flush) *a->hdp_flush = 1u;
}

bool aql_done(Aql *a) { return !a->last.handle || hsa_signal_load_scacquire(a->last) <= 0; }

uint64_t aql_time_ns(Aql *a, int slot) {
  if (slot < 0 || size_t(slot) >= a->prof_used) return 0;
  const hsa_signal_t sg = a->prof[size_t(slot)];
  for (int i = 0; i < 1000000 && hsa_signal_load_scacquire(sg) > 0; i++) {
    struct timespec ts{0, 1000};
    nanosleep(&ts, nullptr);
  }
  hsa_amd_profiling_dispatch_time_t t{};
  if (hsa_amd_profiling_get_dispatch_time(a->agent, sg, &t) != HSA_STATUS_SUCCESS || t.end < t.start) return 0;
  return uint64_t(double(t.end - t.start) * a->ns_per_tick);
}
void aql_time_reset(Aql *a) { a->prof_used = 0; }

}  // namespace tsg
