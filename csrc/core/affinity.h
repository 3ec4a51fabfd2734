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

#include <cstdint>
#include <string>
#include <vector>

namespace ksa {

using CpuList = std::vector<int>;

// Restricts the calling thread to `cpus` (no-op when empty). False if the kernel refused.
bool pin_current_thread(const CpuList& cpus);

// The CFS bandwidth limit of this process's cgroup: `quota_ns` of CPU per `period_ns` (a pod's
// limits.cpu: 100m is 10 ms per 100 ms). quota_ns == 0: no limit, or none found.
struct CpuQuota {
  int64_t quota_ns = 0;
  int64_t period_ns = 0;
  bool limited() const { return quota_ns > 0 && period_ns > 0; }
};
// cgroup v2 cpu.max ("max 100000" or "10000 100000", microseconds).
CpuQuota parse_cpu_max(const std::string& text);
// cgroup v1 cpu.cfs_quota_us (-1: unlimited) and cpu.cfs_period_us.
CpuQuota parse_cfs_quota(const std::string& quota_us, const std::string& period_us);
// Reads the calling process's limit: the cgroup named by /proc/self/cgroup under `root` (v2
// cpu.max, else the v1 cpu controller's cfs files), then `root`'s own files (a container with
// its own cgroup namespace sees its cgroup at the root).
CpuQuota read_cpu_quota(const std::string& root = "/sys/fs/cgroup");

}  // namespace ksa
