// Host cost of one kernel launch with a ~3.9 KB by-value argument block (the pool search
// kernel's shape: 256 x 1024 threads, 96 KiB dynamic LDS), three ways: the <<<>>> launch,
// hipModuleLaunchKernel with the argument buffer passed whole, and an AQL packet written
// straight onto an HSA queue (the kernel loaded from this file's code object). Each launch
// is followed by a poll of a pinned-memory flag the last workgroup stores (as the search
// does), so `call` is the API's host time and `seen` is launch start -> flag seen.
// Build: see tools/probe/build.sh.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

struct BigArgs {
  unsigned *flag;
  unsigned val, pad;
  unsigned words[960];
};
static_assert(sizeof(BigArgs) <= 4096, "args");

extern "C" __global__ void __launch_bounds__(1024) probe_kernel(BigArgs A) {
  extern __shared__ unsigned lds[];
  if (threadIdx.x == 0) lds[0] = A.words[blockIdx.x % 960];
  __syncthreads();
  if (threadIdx.x == 0 && lds[0] != 0xdeadbeefu) __hip_atomic_store(A.flag + blockIdx.x, A.val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)
#define HK(x) do { hsa_status_t e = (x); if (e != HSA_STATUS_SUCCESS) { std::fprintf(stderr, "%s: %d\n", #x, int(e)); std::exit(1); } } while (0)
using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }
static void report(const char *name, std::vector<double> &c, std::vector<double> &s) {
  std::sort(c.begin(), c.end());
  std::sort(s.begin(), s.end());
  std::printf("%-8s call p50 %.2f p90 %.2f us | seen p50 %.2f p90 %.2f us\n", name, c[c.size() / 2], c[c.size() * 9 / 10],
              s[s.size() / 2], s[s.size() * 9 / 10]);
}

int main(int argc, char **argv) {
  const int N = 400, W = 256, LDS = 96 << 10;
  unsigned *flag;
  CK(hipHostMalloc(reinterpret_cast<void **>(&flag), W * 4, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(flag, 0, W * 4);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hipFuncSetAttribute(reinterpret_cast<const void *>(probe_kernel), hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  BigArgs A;
  std::memset(&A, 0, sizeof A);
  A.flag = flag;
  auto wait_all = [&](unsigned v) {
    for (int w = 0; w < W; w++)
      while (__atomic_load_n(flag + w, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
  };
  unsigned val = 0;
  // (a) <<<>>>
  {
    std::vector<double> c, sn;
    for (int i = 0; i < N + 20; i++) {
      A.val = ++val;
      auto t0 = clk::now();
      probe_kernel<<<W, 1024, LDS, s>>>(A);
      auto t1 = clk::now();
      wait_all(val);
      auto t2 = clk::now();
      if (i >= 20) { c.push_back(us(t0, t1)); sn.push_back(us(t0, t2)); }
    }
    CK(hipStreamSynchronize(s));
    report("chevron", c, sn);
  }
  // (b) hipModuleLaunchKernel, argument buffer whole
  {
    hipFunction_t f;
    CK(hipGetFuncBySymbol(&f, reinterpret_cast<const void *>(probe_kernel)));
    std::vector<double> c, sn;
    for (int i = 0; i < N + 20; i++) {
      A.val = ++val;
      size_t sz = sizeof A;
      void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &A, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
      auto t0 = clk::now();
      CK(hipModuleLaunchKernel(f, W, 1, 1, 1024, 1, 1, LDS, s, nullptr, extra));
      auto t1 = clk::now();
      wait_all(val);
      auto t2 = clk::now();
      if (i >= 20) { c.push_back(us(t0, t1)); sn.push_back(us(t0, t2)); }
    }
    CK(hipStreamSynchronize(s));
    report("module", c, sn);
  }
  // (c) AQL packet on an HSA queue of our own
  if (argc > 1) {
    std::ifstream in(argv[1], std::ios::binary);
    std::string co((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    HK(hsa_init());
    hsa_agent_t gpu{};
    HK(hsa_iterate_agents([](hsa_agent_t a, void *d) {
      hsa_device_type_t t;
      hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
      if (t == HSA_DEVICE_TYPE_GPU) { *static_cast<hsa_agent_t *>(d) = a; return HSA_STATUS_INFO_BREAK; }
      return HSA_STATUS_SUCCESS;
    }, &gpu) == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR);
    hsa_code_object_reader_t rd;
    HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
    hsa_executable_t ex;
    HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
    HK(hsa_executable_load_agent_code_object(ex, gpu, rd, nullptr, nullptr));
    HK(hsa_executable_freeze(ex, nullptr));
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(ex, "probe_kernel.kd", &gpu, &sym));
    uint64_t kobj;
    uint32_t kas, gss, pss;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kas));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &gss));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &pss));
    std::printf("hsa kernel: kernarg %u group %u private %u\n", kas, gss, pss);
    hsa_queue_t *q;
    HK(hsa_queue_create(gpu, 256, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    // kernarg pool: the agent's kernarg-capable fine-grained pool
    hsa_amd_memory_pool_t kpool{};
    struct PF { hsa_amd_memory_pool_t *p; hsa_agent_t a; };
    HK(hsa_amd_agent_iterate_memory_pools(gpu, [](hsa_amd_memory_pool_t p, void *d) { (void)p; (void)d; return HSA_STATUS_SUCCESS; }, nullptr));
    hsa_agent_t cpu{};
    hsa_iterate_agents([](hsa_agent_t a, void *d) {
      hsa_device_type_t t;
      hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
      if (t == HSA_DEVICE_TYPE_CPU) { *static_cast<hsa_agent_t *>(d) = a; return HSA_STATUS_INFO_BREAK; }
      return HSA_STATUS_SUCCESS;
    }, &cpu);
    PF pf{&kpool, cpu};
    hsa_amd_agent_iterate_memory_pools(cpu, [](hsa_amd_memory_pool_t p, void *d) {
      uint32_t flags = 0;
      hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
      if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) { *static_cast<PF *>(d)->p = p; return HSA_STATUS_INFO_BREAK; }
      return HSA_STATUS_SUCCESS;
    }, &pf);
    const int NK = 64;
    void *kargs;
    const bool devk = std::getenv("PROBE_HOSTK") == nullptr;
    if (devk) {  // kernel arguments in VRAM, written by the host through the BAR (as HIP does)
      CK(hipExtMallocWithFlags(&kargs, size_t(NK) * 4096, hipDeviceMallocUncached));
    } else {
      HK(hsa_amd_memory_pool_allocate(kpool, size_t(NK) * 4096, 0, &kargs));
      HK(hsa_amd_agents_allow_access(1, &gpu, nullptr, kargs));
    }
    std::printf("kernarg in %s\n", devk ? "device memory" : "host memory");
    hsa_signal_t done;
    HK(hsa_signal_create(0, 0, nullptr, &done));
    std::vector<double> c, sn;
    const uint64_t mask = q->size - 1;
    for (int i = 0; i < N + 20; i++) {
      A.val = ++val;
      auto t0 = clk::now();
      void *ka = static_cast<char *>(kargs) + size_t(i % NK) * 4096;
      std::memcpy(ka, &A, sizeof A);
      if (devk) {  // the writes reach VRAM before the packet: read one back
        (void)*static_cast<volatile uint32_t *>(static_cast<void *>(static_cast<char *>(ka) + sizeof A - 4));
      }
      const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
      auto *pk = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx & mask);
      pk->setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
      pk->workgroup_size_x = 1024;
      pk->workgroup_size_y = 1;
      pk->workgroup_size_z = 1;
      pk->reserved0 = 0;
      pk->grid_size_x = W * 1024;
      pk->grid_size_y = 1;
      pk->grid_size_z = 1;
      pk->private_segment_size = pss;
      pk->group_segment_size = gss + LDS;
      pk->kernel_object = kobj;
      pk->kernarg_address = ka;
      pk->reserved2 = 0;
      pk->completion_signal = hsa_signal_t{0};
      const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                           (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                           (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
      __atomic_store_n(reinterpret_cast<uint32_t *>(pk), uint32_t(hdr) | (uint32_t(pk->setup) << 16), __ATOMIC_RELEASE);
      hsa_signal_store_screlease(q->doorbell_signal, int64_t(idx));
      auto t1 = clk::now();
      wait_all(val);
      auto t2 = clk::now();
      if (i >= 20) { c.push_back(us(t0, t1)); sn.push_back(us(t0, t2)); }
    }
    report("aql", c, sn);
    hsa_signal_destroy(done);
    hsa_queue_destroy(q);
    if (devk) CK(hipFree(kargs)); else hsa_amd_memory_pool_free(kargs);
    hsa_executable_destroy(ex);
    hsa_code_object_reader_destroy(rd);
  }
  CK(hipHostFree(flag));
  return 0;
}
