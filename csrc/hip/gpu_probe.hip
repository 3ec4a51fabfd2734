// MI355X node probe: GPU inventory + an HBM write/verify health check.
//
// The reference has no GPU code. The MI355X specialisation of this build is
// that the scaled Deployment is GPU-worker pods on an 8x MI355X node, so --max-pods defaults
// to 8; `--gpu-aware-max=local` (an extension, off by default) caps max-pods at the number of
// GPUs that pass this probe when the autoscaler runs on the GPU node itself (sidecar).
//
// The health check is a streaming HBM pass, so it is written to run at HBM speed on CDNA4:
//   * fill:   every lane stores 4 x 16 B per iteration with nontemporal stores (no L2 pollution),
//             a 32-bit address-derived pattern (one v_mul_lo_u32 per dword), and accumulates the
//             checksum of what it *intended* to write;
//   * verify: 8 x 16 B nontemporal loads in flight per lane per iteration (128 B/lane, 64 KiB per
//             CU with 4 waves x 2 workgroups), compares each dword against the pattern and sums
//             what it *read*;
//   * both:   wave64 butterfly (__shfl_xor) -> LDS across the 4 waves -> ONE 64-bit atomic per
//             workgroup; grid = CUs x 2 workgroups of 256 threads (512 workgroups over all 8 XCDs),
//             grid-stride so every wave reaches the exit whatever the buffer size. 2/CU with deep
//             unrolling beat 4, 8 and 16/CU in the tune_probe sweep (fewer waves contending for
//             the same channels, same bytes in flight);
//   * timing: one untimed warm-up launch of each kernel, then best-of-`reps` with hipEvents over a
//             buffer >= the 256 MiB Infinity Cache, so the numbers are HBM numbers.
// Healthy <=> zero mismatches AND read checksum == written checksum.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace {

constexpr int kBlock = 256;  // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kUnrollFill = 4;    // 16-byte stores per lane per iteration
constexpr int kUnrollVerify = 8;  // 16-byte loads in flight per lane per iteration
constexpr int kBlocksPerCu = 2;   // measured best in round 1 (variant sweep; git history: r01_tune_probe.jsonl)

thread_local std::string g_last_error;

// Native clang vector (HIP's uint4 is a struct, which the nontemporal builtins reject).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pattern(uint64_t e, uint32_t seed) {
  return (static_cast<uint32_t>(e) * 0x9E3779B1u) ^ static_cast<uint32_t>(e >> 32) ^ seed;
}

__device__ __forceinline__ void block_reduce_add(unsigned long long a, unsigned long long b,
                                                 unsigned long long* __restrict__ out_a,
                                                 unsigned long long* __restrict__ out_b) {
  __shared__ unsigned long long sa[kWaves], sb[kWaves];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sa[wave] = a;
    sb[wave] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long ta = 0, tb = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      ta += sa[w];
      tb += sb[w];
    }
    if (out_a) atomicAdd(out_a, ta);
    if (out_b && tb) atomicAdd(out_b, tb);
  }
}

__device__ __forceinline__ u32x4 pattern4(uint64_t v, uint32_t seed) {
  const uint64_t e = v * 4;
  return u32x4{pattern(e, seed), pattern(e + 1, seed), pattern(e + 2, seed), pattern(e + 3, seed)};
}

__global__ __launch_bounds__(kBlock) void fill_kernel(u32x4* __restrict__ buf, uint64_t n_vec, uint32_t seed,
                                                      unsigned long long* __restrict__ sum) {
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * kBlock;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  unsigned long long acc = 0;
  uint64_t v = tid;
  // main body: kUnroll independent 16-B stores per lane per iteration, lanes coalesced per store
  for (; v + (kUnrollFill - 1) * nthreads < n_vec; v += kUnrollFill * nthreads) {
#pragma unroll
    for (int u = 0; u < kUnrollFill; ++u) {
      const uint64_t w = v + u * nthreads;
      const u32x4 x = pattern4(w, seed);
      acc += static_cast<unsigned long long>(x.x) + x.y + x.z + x.w;
      __builtin_nontemporal_store(x, buf + w);
    }
  }
  for (; v < n_vec; v += nthreads) {
    const u32x4 x = pattern4(v, seed);
    acc += static_cast<unsigned long long>(x.x) + x.y + x.z + x.w;
    __builtin_nontemporal_store(x, buf + v);
  }
  block_reduce_add(acc, 0, sum, nullptr);
}

__global__ __launch_bounds__(kBlock) void verify_kernel(const u32x4* __restrict__ buf, uint64_t n_vec, uint32_t seed,
                                                        unsigned long long* __restrict__ sum,
                                                        unsigned long long* __restrict__ mismatches) {
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * kBlock;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  unsigned long long acc = 0, bad = 0;
  uint64_t v = tid;
  for (; v + (kUnrollVerify - 1) * nthreads < n_vec; v += kUnrollVerify * nthreads) {
    u32x4 x[kUnrollVerify];
#pragma unroll
    for (int u = 0; u < kUnrollVerify; ++u) x[u] = __builtin_nontemporal_load(buf + v + u * nthreads);  // all in flight
#pragma unroll
    for (int u = 0; u < kUnrollVerify; ++u) {
      const u32x4 p = pattern4(v + u * nthreads, seed);
      acc += static_cast<unsigned long long>(x[u].x) + x[u].y + x[u].z + x[u].w;
      bad += (x[u].x != p.x) + (x[u].y != p.y) + (x[u].z != p.z) + (x[u].w != p.w);
    }
  }
  for (; v < n_vec; v += nthreads) {
    const u32x4 x = __builtin_nontemporal_load(buf + v);
    const u32x4 p = pattern4(v, seed);
    acc += static_cast<unsigned long long>(x.x) + x.y + x.z + x.w;
    bad += (x.x != p.x) + (x.y != p.y) + (x.z != p.z) + (x.w != p.w);
  }
  block_reduce_add(acc, bad, sum, mismatches);
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
  uint64_t checksum;           // sum of dwords read back by verify_kernel
  uint64_t expected_checksum;  // sum of dwords fill_kernel intended to write
  uint64_t mismatches;
  double fill_ms;    // best of `reps`
  double verify_ms;  // best of `reps`
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
  std::snprintf(out->name, sizeof out->name, "%s", p.name[0] ? p.name : "AMD Instinct GPU");
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

// Writes then verifies `bytes` (rounded down to 16 B) of device memory on `dev`, `reps` timed
// passes of each kernel after one warm-up. Returns 0 healthy, 1 verification failure, -1 error.
int ksa_gpu_health_check_ex(int dev, uint64_t bytes, int reps, ksa_gpu_health* out) {
  std::memset(out, 0, sizeof *out);
  const uint64_t n_vec = bytes / sizeof(u32x4);
  if (n_vec == 0) {
    g_last_error = "health check buffer too small";
    return -1;
  }
  if (reps < 1) reps = 1;
  if (!check(hipSetDevice(dev), "hipSetDevice")) return -1;
  hipDeviceProp_t p;
  if (!check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties")) return -1;
  u32x4* buf = nullptr;
  unsigned long long* counters = nullptr;  // [0] written sum, [1] read sum, [2] mismatches
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = -1;
  const uint32_t seed = 0xA5C3u;
  do {
    if (!check(hipMalloc(&buf, n_vec * sizeof(u32x4)), "hipMalloc")) break;
    if (!check(hipMalloc(&counters, 3 * sizeof(unsigned long long)), "hipMalloc")) break;
    if (!check(hipEventCreate(&e0), "hipEventCreate") || !check(hipEventCreate(&e1), "hipEventCreate")) break;
    const uint64_t want = (n_vec + kBlock - 1) / kBlock;
    const uint64_t cap = static_cast<uint64_t>(p.multiProcessorCount > 0 ? p.multiProcessorCount : 256) * kBlocksPerCu;
    const int grid = static_cast<int>(want < cap ? want : cap);
    float best_fill = 1e30f, best_verify = 1e30f;
    bool ok = true;
    for (int r = 0; r <= reps && ok; ++r) {  // r == 0 is the untimed warm-up
      ok = check(hipMemset(counters, 0, 3 * sizeof(unsigned long long)), "hipMemset");
      if (!ok) break;
      if (!(ok = check(hipEventRecord(e0, nullptr), "hipEventRecord"))) break;
      hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(kBlock), 0, nullptr, buf, n_vec, seed, counters);
      ok = check(hipGetLastError(), "fill_kernel launch");
      ok = ok && check(hipEventRecord(e1, nullptr), "hipEventRecord");
      ok = ok && check(hipEventSynchronize(e1), "hipEventSynchronize");
      float ms = 0;
      ok = ok && check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
      if (!ok) break;
      if (r > 0 && ms < best_fill) best_fill = ms;
      if (!(ok = check(hipEventRecord(e0, nullptr), "hipEventRecord"))) break;
      hipLaunchKernelGGL(verify_kernel, dim3(grid), dim3(kBlock), 0, nullptr, buf, n_vec, seed, counters + 1,
                         counters + 2);
      ok = check(hipGetLastError(), "verify_kernel launch");
      ok = ok && check(hipEventRecord(e1, nullptr), "hipEventRecord");
      ok = ok && check(hipEventSynchronize(e1), "hipEventSynchronize");
      ok = ok && check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
      if (ok && r > 0 && ms < best_verify) best_verify = ms;
    }
    if (!ok) break;
    unsigned long long host[3] = {0, 0, 0};
    if (!check(hipMemcpy(host, counters, sizeof host, hipMemcpyDeviceToHost), "hipMemcpy")) break;
    out->bytes = n_vec * sizeof(u32x4);
    out->expected_checksum = host[0];
    out->checksum = host[1];
    out->mismatches = host[2];
    out->fill_ms = best_fill;
    out->verify_ms = best_verify;
    out->write_gbps = best_fill > 0 ? out->bytes / (best_fill * 1e6) : 0;
    out->read_gbps = best_verify > 0 ? out->bytes / (best_verify * 1e6) : 0;
    rc = (host[2] == 0 && host[0] == host[1]) ? 0 : 1;
    if (rc) g_last_error = "device memory verification failed";
  } while (false);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (buf) (void)hipFree(buf);
  if (counters) (void)hipFree(counters);
  return rc;
}

int ksa_gpu_health_check(int dev, uint64_t bytes, ksa_gpu_health* out) {
  return ksa_gpu_health_check_ex(dev, bytes, 3, out);
}

}  // extern "C"
