// aql.hpp — kernel dispatch straight onto an HSA queue of our own (AQL packets), for the
// narrow search kernels whose per-query launch is on the step's critical path.
//
// The HIP launch call costs ~3.1-3.6 us of host time per launch (tools/probe/launch_probe.hip:
// <<<>>> and hipModuleLaunchKernel alike); writing the packet ourselves costs the copy of the
// argument words into device memory plus a few stores. The kernels come from a code object
// of pool.hip built beside libtsg.so (libtsg_pool.co) and read no implicit kernel argument.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace tsg {

struct Aql;
struct AqlKernel {
  uint64_t kobj = 0;  // 0: not available
  uint32_t group = 0, priv = 0, kernarg = 0;
};
// The device's dispatcher (hip_ordinal = the HIP device), or nullptr when unavailable:
// TSG_AQL=0, no code object, or any HSA call failing (then the caller launches through HIP).
Aql *aql_open(int hip_ordinal);
void aql_close(Aql *a);
// a kernel of the code object by its symbol name (without ".kd"); kobj = 0 (launch through
// HIP) when its kernarg segment is larger than max_kernarg, the size of its argument struct
AqlKernel aql_kernel(Aql *a, const char *name, uint32_t max_kernarg);
// One dispatch of grid x block threads with dyn_lds bytes of dynamic LDS. The kernel's
// argument block is assembled in a device-memory slot from `parts` (offset, bytes) of `args`
// (only the parts the kernel reads for this launch: the rest of the slot is stale).
// profiled = true: the dispatch's start / end are recorded (the queue's profiling timestamps,
// what rocprofv3's kernel trace reports) and the return value names them for aql_time_ns
// (-1 when no profiling slot is free); otherwise -1.
int aql_dispatch(Aql *a, const AqlKernel &k, uint32_t grid, uint32_t block, uint32_t dyn_lds, const void *args,
                 const std::vector<std::pair<uint32_t, uint32_t>> &parts, bool profiled = false);
// Host writes to device memory through the BAR pass the host data path (HDP), which buffers
// them: a posted write of the HDP flush register pushes them on (no read-back: the reader on
// the device verifies what it reads). No-op without the register.
void aql_hdp_flush(Aql *a);
// true once the last dispatch has completed (its own completion signal: dispatches on the
// queue complete in order; for a caller's liveness check while it polls the kernel's words)
bool aql_done(Aql *a);
// a profiled dispatch's duration (ns; 0 if it has not completed); aql_time_reset frees the slots
uint64_t aql_time_ns(Aql *a, int slot);
void aql_time_reset(Aql *a);

}  // namespace tsg
