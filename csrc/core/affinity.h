// CPU placement of native threads.
//
// The control loop's cost per poll is mostly cache traffic: request/response buffers, socket
// state and the kernel's TCP path. On a chiplet CPU (EPYC: one L3 per 8-core CCD) a worker
// whose thread migrates across CCDs, or whose peers run on another CCD, pays cross-die cache
// transfers on every request. Pinning each worker (and, in the benchmark, its fake endpoints)
// to one L3 domain keeps that traffic inside one CCD -- the CPU-side analogue of keeping a
// GPU kernel's tiles in one XCD's L2. The CPU lists come from the caller (Runner::set_cpus,
// the worker-process fleet's per-worker lists, the fakes' set_cpus); the CLI pins nothing by
// default, and bench.py confines a multi-rank job's ranks to CPU slices at the process level.
#pragma once

#include <vector>

namespace ksa {

using CpuList = std::vector<int>;

// Restricts the calling thread to `cpus` (no-op when empty). False if the kernel refused.
bool pin_current_thread(const CpuList& cpus);

}  // namespace ksa
