// Variant sweep for the HBM probe's fill/verify kernels (tuning tool, not shipped in the .so).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 csrc/tools/tune_probe.hip -o build/tune_probe
// Prints one line per (kernel, store/load kind, blocks per CU, unroll) with the best-of-N GB/s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

// A failed HIP call ends the probe with its error (a tuning run must not print made-up numbers).
#define CHECK(call)                                                                   \
  do {                                                                                \
    const hipError_t e_ = (call);                                                     \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));          \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pattern(uint64_t e) { return (static_cast<uint32_t>(e) * 0x9E3779B1u) ^ static_cast<uint32_t>(e >> 32); }
__device__ __forceinline__ u32x4 pattern4(uint64_t v) {
  const uint64_t e = v * 4;
  return u32x4{pattern(e), pattern(e + 1), pattern(e + 2), pattern(e + 3)};
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void fill(u32x4* __restrict__ buf, uint64_t n, unsigned long long* sum) {
  const uint64_t nt = static_cast<uint64_t>(gridDim.x) * 256;
  uint64_t v = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  unsigned long long acc = 0;
  for (; v + (U - 1) * nt < n; v += U * nt) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4 x = pattern4(v + u * nt);
      acc += static_cast<unsigned long long>(x.x) + x.y + x.z + x.w;
      if (NT) __builtin_nontemporal_store(x, buf + v + u * nt);
      else buf[v + u * nt] = x;
    }
  }
  for (; v < n; v += nt) {
    const u32x4 x = pattern4(v);
    acc += static_cast<unsigned long long>(x.x) + x.y + x.z + x.w;
    buf[v] = x;
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(sum, acc);
}

// SUM: also accumulate the 64-bit checksum of what was read (what the shipped probe does).
template <int U, bool NT, bool SUM = false>
__global__ __launch_bounds__(256) void verify(const u32x4* __restrict__ buf, uint64_t n, unsigned long long* bad_out) {
  const uint64_t nt = static_cast<uint64_t>(gridDim.x) * 256;
  uint64_t v = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  unsigned long long bad = 0, acc = 0;
  for (; v + (U - 1) * nt < n; v += U * nt) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = NT ? __builtin_nontemporal_load(buf + v + u * nt) : buf[v + u * nt];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4 p = pattern4(v + u * nt);
      if (SUM) acc += static_cast<unsigned long long>(x[u].x) + x[u].y + x[u].z + x[u].w;
      bad += (x[u].x != p.x) + (x[u].y != p.y) + (x[u].z != p.z) + (x[u].w != p.w);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    bad += __shfl_xor(bad, off, 64);
    if (SUM) acc += __shfl_xor(acc, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (bad) atomicAdd(bad_out, bad);
    if (SUM) atomicAdd(bad_out + 1, acc);
  }
}

template <class K>
float best_ms(K launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r <= reps; ++r) {
    CHECK(hipEventRecord(a, nullptr));
    launch();
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(b, nullptr));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (r > 0 && ms < best) best = ms;
  }
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return best;
}

template <int U, bool NT, bool SUM = false>
void run(u32x4* buf, uint64_t n, unsigned long long* ctr, int cus, int bpc) {
  const int grid = cus * bpc;
  const double bytes = static_cast<double>(n) * 16;
  float f = best_ms([&] { hipLaunchKernelGGL((fill<U, NT>), dim3(grid), dim3(256), 0, nullptr, buf, n, ctr); }, 5);
  float v = best_ms([&] { hipLaunchKernelGGL((verify<U, NT, SUM>), dim3(grid), dim3(256), 0, nullptr, buf, n, ctr + 1); }, 5);
  unsigned long long h[3];
  CHECK(hipMemcpy(h, ctr, sizeof h, hipMemcpyDeviceToHost));
  std::printf("{\"unroll\":%d,\"nontemporal\":%s,\"checksum\":%s,\"blocks_per_cu\":%d,\"write_GBps\":%.1f,\"read_verify_GBps\":%.1f,\"mismatches\":%llu}\n",
              U, NT ? "true" : "false", SUM ? "true" : "false", bpc, bytes / (f * 1e6), bytes / (v * 1e6), h[1]);
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const uint64_t bytes = 2ull << 30;
  const uint64_t n = bytes / 16;
  u32x4* buf;
  unsigned long long* ctr;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&ctr, 32));
  CHECK(hipMemset(ctr, 0, 32));
  for (int bpc : {2, 4, 8}) {
    run<4, true>(buf, n, ctr, p.multiProcessorCount, bpc);
    run<8, true>(buf, n, ctr, p.multiProcessorCount, bpc);
    run<4, true, true>(buf, n, ctr, p.multiProcessorCount, bpc);
    run<8, true, true>(buf, n, ctr, p.multiProcessorCount, bpc);
    run<16, true, true>(buf, n, ctr, p.multiProcessorCount, bpc);
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(ctr));
  return 0;
}
