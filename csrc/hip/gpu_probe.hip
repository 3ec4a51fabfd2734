// MI355X node probe: GPU inventory + an on-device health check.
//
// The reference has no GPU code. The MI355X specialisation of this build is
// that the scaled Deployment is GPU-worker pods on an 8x MI355X node, so --max-pods defaults
// to 8; `--gpu-aware-max=local` (an extension, off by default) caps max-pods at the number of
// healthy GPUs this probe finds when the autoscaler runs on the GPU node itself (sidecar).
//
// The health check exercises what a worker pod needs from the device before the autoscaler
// counts it: HBM writes + reads over a large buffer and a grid that spans every CU.
//   * fill kernel:   16-byte vector stores of a position-derived pattern (HBM write path);
//   * verify kernel: 16-byte vector loads, per-lane checksum, 64-lane wave reduction with
//                    DPP-free __shfl_xor (wave64), one 64-bit atomic per wave.
// Grid = 8 x 256 CUs x 4 workgroups (>> 256, so all 8 XCDs participate); each workgroup
// strides over the buffer, so the grid size is independent of the buffer size and every
// wave reaches the exit (no persistent loop without a bound).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace {

constexpr int kBlock = 256;                // 4 waves of 64
constexpr int kGridBlocks = 8 * 256 * 4;   // XCDs x CUs-per-chip x blocks-per-CU (upper bound)

thread_local std::string g_last_error;

__host__ __device__ inline uint32_t mix32(uint64_t i) {
  uint64_t x = i * 0x9E3779B97F4A7C15ULL;
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ULL;
  x ^= x >> 32;
  return static_cast<uint32_t>(x);
}

__global__ __launch_bounds__(kBlock) void fill_kernel(uint4* __restrict__ buf, uint64_t n_vec) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t v = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < n_vec; v += stride) {
    const uint64_t e = v * 4;
    buf[v] = make_uint4(mix32(e), mix32(e + 1), mix32(e + 2), mix32(e + 3));
  }
}

__global__ __launch_bounds__(kBlock) void verify_kernel(const uint4* __restrict__ buf, uint64_t n_vec,
                                                        unsigned long long* __restrict__ sum,
                                                        unsigned long long* __restrict__ mismatches) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  unsigned long long acc = 0, bad = 0;
  for (uint64_t v = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < n_vec; v += stride) {
    const uint4 x = buf[v];
    const uint64_t e = v * 4;
    acc += static_cast<unsigned long long>(x.x) + x.y + x.z + x.w;
    bad += (x.x != mix32(e)) + (x.y != mix32(e + 1)) + (x.z != mix32(e + 2)) + (x.w != mix32(e + 3));
  }
  // wave64 butterfly reduction
  for (int off = 32; off > 0; off >>= 1) {
    acc += __shfl_xor(acc, off, 64);
    bad += __shfl_xor(bad, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(sum, acc);
    if (bad) atomicAdd(mismatches, bad);
  }
}

bool check(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

}  // namespace

extern "C" {

struct ksa_gpu_info {
  char name[256];
  char arch[64];
  int32_t compute_units;
  int32_t clock_khz;
  int32_t warp_size;
  int32_t pci_bus_id;
  int32_t pci_device_id;
  int32_t lds_bytes_per_block;
  int64_t total_mem_bytes;
  int64_t free_mem_bytes;
};

struct ksa_gpu_health {
  uint64_t bytes;
  uint64_t checksum;
  uint64_t expected_checksum;
  uint64_t mismatches;
  double fill_ms;
  double verify_ms;
  double write_gbps;
  double read_gbps;
};

const char* ksa_gpu_last_error() { return g_last_error.c_str(); }

int ksa_gpu_device_count() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) return 0;
  if (!check(e, "hipGetDeviceCount")) return -1;
  return n;
}

int ksa_gpu_get_info(int dev, ksa_gpu_info* out) {
  std::memset(out, 0, sizeof *out);
  hipDeviceProp_t p;
  if (!check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties")) return -1;
  std::snprintf(out->name, sizeof out->name, "%s", p.name);
  std::snprintf(out->arch, sizeof out->arch, "%s", p.gcnArchName);
  out->compute_units = p.multiProcessorCount;
  out->clock_khz = p.clockRate;
  out->warp_size = p.warpSize;
  out->pci_bus_id = p.pciBusID;
  out->pci_device_id = p.pciDeviceID;
  out->lds_bytes_per_block = static_cast<int32_t>(p.sharedMemPerBlock);
  out->total_mem_bytes = static_cast<int64_t>(p.totalGlobalMem);
  if (!check(hipSetDevice(dev), "hipSetDevice")) return -1;
  size_t free_b = 0, total_b = 0;
  if (!check(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo")) return -1;
  out->free_mem_bytes = static_cast<int64_t>(free_b);
  return 0;
}

// Writes then verifies `bytes` (rounded down to 16 B) of device memory on `dev`.
int ksa_gpu_health_check(int dev, uint64_t bytes, ksa_gpu_health* out) {
  std::memset(out, 0, sizeof *out);
  const uint64_t n_vec = bytes / sizeof(uint4);
  if (n_vec == 0) {
    g_last_error = "health check buffer too small";
    return -1;
  }
  if (!check(hipSetDevice(dev), "hipSetDevice")) return -1;
  uint4* buf = nullptr;
  unsigned long long* counters = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  int rc = -1;
  do {
    if (!check(hipMalloc(&buf, n_vec * sizeof(uint4)), "hipMalloc")) break;
    if (!check(hipMalloc(&counters, 2 * sizeof(unsigned long long)), "hipMalloc")) break;
    if (!check(hipMemset(counters, 0, 2 * sizeof(unsigned long long)), "hipMemset")) break;
    for (auto& e : ev)
      if (!check(hipEventCreate(&e), "hipEventCreate")) break;
    uint64_t want_blocks = (n_vec + kBlock - 1) / kBlock;
    int grid = static_cast<int>(want_blocks < static_cast<uint64_t>(kGridBlocks) ? want_blocks : kGridBlocks);
    hipEventRecord(ev[0], nullptr);
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(kBlock), 0, nullptr, buf, n_vec);
    if (!check(hipGetLastError(), "fill_kernel launch")) break;
    hipEventRecord(ev[1], nullptr);
    hipLaunchKernelGGL(verify_kernel, dim3(grid), dim3(kBlock), 0, nullptr, buf, n_vec, counters, counters + 1);
    if (!check(hipGetLastError(), "verify_kernel launch")) break;
    hipEventRecord(ev[2], nullptr);
    if (!check(hipEventSynchronize(ev[2]), "hipEventSynchronize")) break;
    unsigned long long host[2] = {0, 0};
    if (!check(hipMemcpy(host, counters, sizeof host, hipMemcpyDeviceToHost), "hipMemcpy")) break;
    float f_ms = 0, v_ms = 0;
    hipEventElapsedTime(&f_ms, ev[0], ev[1]);
    hipEventElapsedTime(&v_ms, ev[1], ev[2]);
    // Host reference of the checksum (mod 2^64).
    unsigned long long expect = 0;
    for (uint64_t e = 0; e < n_vec * 4; ++e) expect += mix32(e);
    out->bytes = n_vec * sizeof(uint4);
    out->checksum = host[0];
    out->expected_checksum = expect;
    out->mismatches = host[1];
    out->fill_ms = f_ms;
    out->verify_ms = v_ms;
    out->write_gbps = f_ms > 0 ? out->bytes / (f_ms * 1e6) : 0;
    out->read_gbps = v_ms > 0 ? out->bytes / (v_ms * 1e6) : 0;
    rc = (host[1] == 0 && host[0] == expect) ? 0 : 1;
    if (rc) g_last_error = "device memory verification failed";
  } while (false);
  for (auto& e : ev)
    if (e) hipEventDestroy(e);
  if (buf) hipFree(buf);
  if (counters) hipFree(counters);
  return rc;
}

}  // extern "C"
