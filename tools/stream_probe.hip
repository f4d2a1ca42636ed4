// stream_probe.hip — the read-bandwidth ceiling the search scan is measured against:
// a read-only streaming kernel (dwordx4 per lane, a few loads in flight per lane,
// one workgroup per resident slot, contiguous per-workgroup ranges like the scan)
// over a buffer that is either MALL-resident (<= 256 MiB, re-read back to back) or
// HBM-resident (larger). Prints one JSON line per size.
//   hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o build/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int INFLIGHT>
__global__ void __launch_bounds__(256) stream_read(const u32x4 *p, size_t n16, unsigned *sink) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t b = blockIdx.x * per, e = b + per < n16 ? b + per : n16;
  unsigned acc = 0;
  for (size_t i = b + threadIdx.x; i < e; i += 256 * INFLIGHT) {
    u32x4 v[INFLIGHT];
#pragma unroll
    for (int k = 0; k < INFLIGHT; k++) {
      const size_t j = i + size_t(k) * 256;
      v[k] = j < e ? p[j] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < INFLIGHT; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // keep the loads
}

int main(int argc, char **argv) {
  int cu = 0;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t sizes[] = {150ull << 20, 600ull << 20};
  unsigned *sink;
  CK(hipMalloc(&sink, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (size_t bytes : sizes) {
    void *buf;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 1, bytes));
    for (int wpc : {2, 4, 8}) {
      const int grid = cu * wpc;
      float best = 1e30f, sum = 0;
      const int reps = 30;
      for (int r = 0; r < reps + 3; r++) {
        CK(hipEventRecord(a));
        stream_read<4><<<grid, 256>>>(static_cast<const u32x4 *>(buf), bytes / 16, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 3) {
          sum += ms;
          best = ms < best ? ms : best;
        }
      }
      const float avg = sum / reps;
      std::printf("{\"bytes\": %zu, \"wg_per_cu\": %d, \"avg_us\": %.2f, \"best_us\": %.2f, \"avg_gbps\": %.1f}\n",
                  bytes, wpc, avg * 1e3, best * 1e3, bytes / (avg * 1e6));
    }
    CK(hipFree(buf));
  }
  return 0;
}
