// gfx950 what-if policy sweep: one candidate configuration per lane.
//
// Each lane runs ksa_sim::simulate (csrc/sim/policy_sim.h: the reference's decision rules,
// bit-identical to the CPU path and the Python oracle) over the same queue-depth trace. The
// work is a branchy integer state machine -- no matrix math, so no MFMA -- and the layout is
// chosen for that:
//   * parameters and results are structure-of-arrays ([field][config]), so the 64 lanes of a
//     wave load and store each field as one contiguous 512-byte (int64) segment;
//   * the trace (segment start times + depths) is staged once per workgroup into dynamically
//     sized LDS when it fits (kLdsTraceBytes = 32 KiB: 2048 int64 segments), so the per-poll depth lookups --
//     every lane walks its own forward-only cursor -- hit LDS; longer traces are read from
//     global memory (lanes advance through it nearly in lockstep, so L1/L2 serve them) and then
//     no LDS is allocated at all, leaving occupancy to the VGPR budget;
//   * no 64-bit integer division per poll: the backlog metric divides once per replica run, and
//     the poll-to-poll interval in ms is picked from six precomputed floors (policy_sim.h);
//   * sweeps whose periods and latencies are whole milliseconds (ksa_sim::ms_path_ok: the grids
//     and latency models one writes by hand) run ksa_sim::simulate_ms, on 32-bit millisecond
//     clocks with a 32-bit trace (8 B per segment, so 4096 segments fit the same 32 KiB of LDS);
//     the same results, without the per-poll 64-bit compares, adds and products;
//   * the host orders configurations with the poll period outermost, so neighbouring lanes share
//     trip counts and a wave's lanes retire together (less divergence at the loop exit);
//   * grid-stride loop over configurations; the grid is one resident wave of workgroups
//     (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs: 74 VGPRs -> 6 waves/SIMD -> 6
//     workgroups of 256 per CU, 1536 over the 8 XCDs), so no workgroup waits for a second round
//     (a fixed CUs x 8 grid cost 10% in that tail). Forcing 7 waves/SIMD spills and is slower;
//     every lane's loop is bounded by horizon / max(poll, sqs latency) and ksa_sim::kMaxPolls.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../sim/policy_sim.h"
#include "device_arena.h"

namespace {

constexpr int kBlock = 256;
constexpr int kLdsTraceBytes = 32 * 1024;  // trace staged in LDS up to this size (-> 5 WG/CU)

thread_local std::string g_sweep_error;

enum : int { kPoll = 0, kUpCool, kDownCool, kUpMsgs, kDownMsgs, kUpPods, kDownPods, kMaxPods, kMinPods, kNumParams };
enum : int { kPodMs = 0, kBacklog, kFirstUp, kNumOut64 };
enum : int { kUps = 0, kDowns, kNoopUps, kNoopDowns, kFinal, kMaxRep, kPolls, kNumOut32 };

#ifndef KSA_SWEEP_WAVES_PER_EU
#define KSA_SWEEP_WAVES_PER_EU 6
#endif

// The grid-stride loop over configurations. The trace pointer is the LDS copy or the global
// array, chosen per launch, so the loads are flat: specialising them into ds_read and
// global_load copies of the loop (two inlined calls) measured slower on the global path (24.5 vs
// 22.5 ms, profiles/r03u_sweep_ab.jsonl) and equal from LDS.
template <bool kMs, bool kSkip, class T>
__device__ __forceinline__ void sweep_lanes(const int64_t* __restrict__ params, int64_t m, const ksa_sim::Latency& lat,
                                            const T* __restrict__ t, const T* __restrict__ d, int32_t n, int32_t init,
                                            int64_t horizon, int64_t* __restrict__ out64, int32_t* __restrict__ out32) {
  const ksa_sim::MsLatency lat_ms = ksa_sim::ms_latency(lat);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < m; i += stride) {
    ksa_sim::Params p;
    p.poll_ns = params[kPoll * m + i];
    p.up_cool_ns = params[kUpCool * m + i];
    p.down_cool_ns = params[kDownCool * m + i];
    p.up_msgs = params[kUpMsgs * m + i];
    p.down_msgs = params[kDownMsgs * m + i];
    p.up_pods = params[kUpPods * m + i];
    p.down_pods = params[kDownPods * m + i];
    p.max_pods = params[kMaxPods * m + i];
    p.min_pods = params[kMinPods * m + i];
    ksa_sim::Result r;
    if constexpr (kMs)
      r = ksa_sim::simulate_ms<kSkip>(p, lat_ms, t, d, n, init, horizon);
    else
      r = ksa_sim::simulate<kSkip>(p, lat, t, d, n, init, horizon);
    out64[kPodMs * m + i] = r.pod_ms;
    out64[kBacklog * m + i] = r.backlog;
    out64[kFirstUp * m + i] = r.first_up_ns;
    out32[kUps * m + i] = r.ups;
    out32[kDowns * m + i] = r.downs;
    out32[kNoopUps * m + i] = r.noop_ups;
    out32[kNoopDowns * m + i] = r.noop_downs;
    out32[kFinal * m + i] = r.final_replicas;
    out32[kMaxRep * m + i] = r.max_replicas;
    out32[kPolls * m + i] = r.polls;
  }
}

// kMs: ksa_sim::simulate_ms over a 32-bit trace (T = int32_t; the host checked ms_path_ok), else
// ksa_sim::simulate over the int64 trace. kSkip: the steady-stretch skip (ksa_sim::skip_pays), a
// separate instantiation because its code costs registers and time where no stretch forms.
template <bool kMs, bool kSkip, class T>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KSA_SWEEP_WAVES_PER_EU))) void sweep_kernel(
    const int64_t* __restrict__ params, int64_t m, ksa_sim::Latency lat, const T* __restrict__ g_t,
    const T* __restrict__ g_d, int32_t n, int32_t init, int64_t horizon, int64_t* __restrict__ out64,
    int32_t* __restrict__ out32, bool in_lds) {
  // Dynamic LDS: 2 x sizeof(T) per segment when the host stages the trace (in_lds), none
  // otherwise -- a static allocation would cap occupancy even for traces read from global memory.
  extern __shared__ int64_t s_lds[];
  T* s_t = reinterpret_cast<T*>(s_lds);
  T* s_d = s_t + (in_lds ? n : 0);
  if (in_lds) {
    for (int i = threadIdx.x; i < n; i += kBlock) {
      s_t[i] = g_t[i];
      s_d[i] = g_d[i];
    }
    __syncthreads();
  }
  sweep_lanes<kMs, kSkip>(params, m, lat, in_lds ? static_cast<const T*>(s_t) : g_t, in_lds ? static_cast<const T*>(s_d) : g_d, n,
                   init, horizon, out64, out32);
}

bool ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  g_sweep_error = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

// Launches one path's kernel on the arena's stream. The grid is one resident wave of workgroups
// (KSA_SWEEP_GRID: "tiles" = one workgroup per 256 configurations, or N x resident).
template <bool kMs, bool kSkip, class T>
bool launch(const ksa_gpu::DeviceArena& ar, const int64_t* d_p, int64_t m, const ksa_sim::Latency& lat, const T* d_t,
            const T* d_d, int32_t n, int32_t init, int64_t horizon_ns, int64_t* d_o64, int32_t* d_o32) {
  const int64_t want = (m + kBlock - 1) / kBlock;
  const size_t trace_bytes = 2 * static_cast<size_t>(n) * sizeof(T);
  size_t cap_bytes = kLdsTraceBytes;
  if (const char* c = std::getenv("KSA_SWEEP_LDS_BYTES"))  // tuning knob: the staging cap (A/B)
    cap_bytes = std::min<size_t>(static_cast<size_t>(std::max(0, std::atoi(c))), 64 * 1024);
  const size_t lds = trace_bytes <= cap_bytes ? trace_bytes : 0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sweep_kernel<kMs, kSkip, T>, kBlock, lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  int64_t cap = static_cast<int64_t>(ar.cus) * per_cu;
  if (const char* g = std::getenv("KSA_SWEEP_GRID")) cap = std::strcmp(g, "tiles") == 0 ? want : cap * std::max(1, std::atoi(g));
  const int grid = static_cast<int>(want < cap ? want : cap);
  hipLaunchKernelGGL((sweep_kernel<kMs, kSkip, T>), dim3(grid), dim3(kBlock), lds, ar.stream, d_p, m, lat, d_t, d_d, n, init,
                     horizon_ns, d_o64, d_o32, lds > 0);
  return ok(hipGetLastError(), "sweep_kernel launch");
}

}  // namespace

extern "C" {

const char* ksa_sweep_last_error() { return g_sweep_error.c_str(); }

// params: [9][m] int64 (poll, up_cool, down_cool, up_msgs, down_msgs, up_pods, down_pods, max, min)
// out64:  [3][m] int64 (pod_ms, backlog, first_up_ns); out32: [7][m] int32 (ups, downs, noop_ups,
// noop_downs, final, max_replicas, polls). latency: {sqs, get, update} ns. arith bits 0-1: 0 runs
// the millisecond clock when ksa_sim::ms_path_ok holds, 1 forces the nanosecond one; bits 2-3: the
// steady-stretch skip, 0 when ksa_sim::skip_pays, 1 always, 2 never (same results). *ms_used
// reports the choices: bit 0 the ms clock, bit 1 the skip. Returns 0 on success.
int ksa_sweep_gpu(int dev, const int64_t* trace_t, const int64_t* trace_d, int32_t n, int32_t init_replicas,
                  int64_t horizon_ns, const int64_t* latency, const int64_t* params, int64_t m, int64_t* out64,
                  int32_t* out32, double* kernel_ms, int32_t arith, int32_t* ms_used) {
  if (n < 1 || trace_t[0] != 0) {
    g_sweep_error = "trace must have at least one segment starting at t=0";
    return -1;
  }
  for (int k = 0; k < 3; ++k) {
    if (latency[k] < 0 || latency[k] > ksa_sim::kMaxLatencyNs) {
      g_sweep_error = "latencies must be within [0, 1 h]";
      return -1;
    }
  }
  if (m <= 0) return 0;
  const bool ms = (arith & 3) == 0 && ksa_sim::ms_path_ok(trace_t, trace_d, n, horizon_ns, latency, params, m);
  const int skip_mode = (arith >> 2) & 3;
  const bool skip = skip_mode == 1 || (skip_mode == 0 && ksa_sim::skip_pays(trace_t, n, horizon_ns, latency, params, m, ms ? 4 : 5));
  if (ms_used) *ms_used = (ms ? 1 : 0) | (skip ? 2 : 0);
  // the trace in the chosen path's element type
  std::vector<int32_t> t32, d32;
  const size_t elem = ms ? sizeof(int32_t) : sizeof(int64_t);
  const void* h_t = trace_t;
  const void* h_d = trace_d;
  if (ms) {
    t32.resize(n);
    d32.resize(n);
    ksa_sim::narrow_policy_trace(trace_t, trace_d, n, t32.data(), d32.data());
    h_t = t32.data();
    h_d = d32.data();
  }
  ksa_gpu::DeviceArena* ar = ksa_gpu::device_arena(dev, &g_sweep_error);
  if (!ar) return -1;
  std::lock_guard<std::mutex> lock(ar->mu);
  if (!ok(hipSetDevice(dev), "hipSetDevice")) return -1;
  void *d_t = nullptr, *d_d = nullptr, *d_p = nullptr, *d_o64 = nullptr, *d_o32 = nullptr;
  if (!ok(ar->get(0, n * elem, &d_t), "hipMalloc") || !ok(ar->get(1, n * elem, &d_d), "hipMalloc") ||
      !ok(ar->get(2, kNumParams * m * sizeof(int64_t), &d_p), "hipMalloc") ||
      !ok(ar->get(3, kNumOut64 * m * sizeof(int64_t), &d_o64), "hipMalloc") ||
      !ok(ar->get(4, kNumOut32 * m * sizeof(int32_t), &d_o32), "hipMalloc"))
    return -1;
  hipStream_t st = ar->stream;
  const ksa_gpu::StreamDrain drain{st};  // also on the error paths: t32 / d32 die with this frame
  if (!ok(hipMemcpyAsync(d_t, h_t, n * elem, hipMemcpyHostToDevice, st), "hipMemcpyAsync") ||
      !ok(hipMemcpyAsync(d_d, h_d, n * elem, hipMemcpyHostToDevice, st), "hipMemcpyAsync") ||
      !ok(hipMemcpyAsync(d_p, params, kNumParams * m * sizeof(int64_t), hipMemcpyHostToDevice, st), "hipMemcpyAsync"))
    return -1;
  const ksa_sim::Latency lat{latency[0], latency[1], latency[2]};
  const int64_t* p = static_cast<const int64_t*>(d_p);
  int64_t* o64 = static_cast<int64_t*>(d_o64);
  int32_t* o32 = static_cast<int32_t*>(d_o32);
  if (!ok(hipEventRecord(ar->e0, st), "hipEventRecord")) return -1;
  const auto* g_t32 = static_cast<const int32_t*>(d_t);
  const auto* g_d32 = static_cast<const int32_t*>(d_d);
  const auto* g_t64 = static_cast<const int64_t*>(d_t);
  const auto* g_d64 = static_cast<const int64_t*>(d_d);
  const bool launched =
      ms ? (skip ? launch<true, true>(*ar, p, m, lat, g_t32, g_d32, n, init_replicas, horizon_ns, o64, o32)
                 : launch<true, false>(*ar, p, m, lat, g_t32, g_d32, n, init_replicas, horizon_ns, o64, o32))
         : (skip ? launch<false, true>(*ar, p, m, lat, g_t64, g_d64, n, init_replicas, horizon_ns, o64, o32)
                 : launch<false, false>(*ar, p, m, lat, g_t64, g_d64, n, init_replicas, horizon_ns, o64, o32));
  if (!launched) return -1;
  if (!ok(hipEventRecord(ar->e1, st), "hipEventRecord")) return -1;
  if (!ok(hipMemcpyAsync(out64, o64, kNumOut64 * m * sizeof(int64_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync") ||
      !ok(hipMemcpyAsync(out32, o32, kNumOut32 * m * sizeof(int32_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync"))
    return -1;
  if (!ok(hipStreamSynchronize(st), "hipStreamSynchronize")) return -1;
  float ms_elapsed = 0;
  if (!ok(hipEventElapsedTime(&ms_elapsed, ar->e0, ar->e1), "hipEventElapsedTime")) return -1;
  if (kernel_ms) *kernel_ms = ms_elapsed;
  return 0;
}

}  // extern "C"
