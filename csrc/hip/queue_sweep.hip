// gfx950 closed-loop what-if sweep: one (configuration, seed) per lane.
//
// Each lane runs ksa_sim::simulate_queue (csrc/sim/queue_sim.h): the reference's decision rules
// driving a queue that the replicas drain, with random arrivals from a counter-based stream
// (integer-only, bit-identical to the CPU path). Lane l simulates configuration l / seeds with
// seed l % seeds, so a wave holds consecutive seeds of one configuration. Layout as the open-loop
// kernel (policy_sweep.hip): parameters [9][m] int64 (structure of arrays, read once per lane),
// outputs [field][m * seeds]; the arrival-rate trace is read from global memory through a
// register-resident cursor (queue_sim.h RateCursor), one segment ahead, so a poll inside a segment
// makes no trace load. The grid is one resident wave of workgroups
// (occupancy API x CUs) with a grid-stride loop; every lane's loop is bounded by the horizon
// and ksa_sim::kMaxPolls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../sim/queue_sim.h"
#include "device_arena.h"

namespace {

constexpr int kBlock = 256;

// Minimum resident waves per SIMD the register allocator must allow (0: compiler's choice).
// Measured on an MI355X (768k lanes x 24 h, same box): compiler's choice 107 VGPRs / 4 waves
// 182.7 ms; 5 waves (96 VGPRs, 24 B scratch) 171.1 ms; 6 waves (80 VGPRs, 92 B scratch) 188.5 ms.
// Round 2 (register rate cursor + sqrt memo, 24000 x 32 lanes x 24 h): 5 waves 125.6 ms vs 4 waves
// 131.3 ms. Round 3 (one-hash sampler, SatArith): 5 waves 109.1 ms (84 B scratch) vs 4 waves
// 111.2 ms (122 VGPRs, none); FastArith fits 96 VGPRs at 5 waves with no scratch (68.2 ms,
// profiles/r03h_queue). The millisecond-clock kernel (77 VGPRs, 6 waves at a floor of 5): a floor
// of 7 (72 VGPRs, 12 B scratch outside the poll loop) 55.7 ms vs 61.4-62.6 ms, a floor of 8
// (64 VGPRs, 60 B scratch) 60.1 ms (profiles/r03ai_queue_ab.jsonl).
#ifndef KSA_QUEUE_WAVES_PER_EU
#define KSA_QUEUE_WAVES_PER_EU 5
#endif
#ifndef KSA_QUEUE_FAST_WAVES_PER_EU
#define KSA_QUEUE_FAST_WAVES_PER_EU KSA_QUEUE_WAVES_PER_EU
#endif
#ifndef KSA_QUEUE_MS_WAVES_PER_EU
#define KSA_QUEUE_MS_WAVES_PER_EU 7
#endif
enum : int { kPoll = 0, kUpCool, kDownCool, kUpMsgs, kDownMsgs, kUpPods, kDownPods, kMaxPods, kMinPods, kNumParams };
enum : int { kPodMs = 0, kBacklogMsgMs, kViolationMs, kPeakBacklog, kArrived, kServed, kFinalBacklog, kNumOut64 };
enum : int { kUps = 0, kDowns, kFinal, kMaxRep, kPolls, kNumOut32 };

thread_local std::string g_queue_error;

// A: ksa_sim::FastArith (T = uint32_t, the host proved the sweep's bounds: fast_path_ok) or
// ksa_sim::SatArith (T = int64_t).
template <class A, class T, bool kMs>
__global__ __launch_bounds__(kBlock)
#if KSA_QUEUE_WAVES_PER_EU > 0 && KSA_QUEUE_FAST_WAVES_PER_EU > 0 && KSA_QUEUE_MS_WAVES_PER_EU > 0
__attribute__((amdgpu_waves_per_eu(kMs ? KSA_QUEUE_MS_WAVES_PER_EU
                                       : A::kExact ? KSA_QUEUE_FAST_WAVES_PER_EU : KSA_QUEUE_WAVES_PER_EU)))
#endif
void queue_sweep_kernel(const int64_t* __restrict__ params, int64_t m, int32_t seeds, uint64_t seed0,
                        ksa_sim::Latency lat, ksa_sim::QueueModel model, const T* __restrict__ t_ms,
                        const T* __restrict__ rate_milli, int32_t n, int32_t init, int64_t horizon,
                        int64_t* __restrict__ out64, int32_t* __restrict__ out32) {
  const int64_t lanes = m * seeds;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t l = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; l < lanes; l += stride) {
    const int64_t i = l / seeds;
    const int32_t s = static_cast<int32_t>(l - i * seeds);
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
    ksa_sim::QueueResult r;
    if constexpr (kMs)
      r = ksa_sim::simulate_queue_ms(p, lat, model, t_ms, rate_milli, n, init, horizon, seed0 + static_cast<uint64_t>(s));
    else
      r = ksa_sim::simulate_queue<A>(p, lat, model, t_ms, rate_milli, n, init, horizon, seed0 + static_cast<uint64_t>(s));
    out64[kPodMs * lanes + l] = r.pod_ms;
    out64[kBacklogMsgMs * lanes + l] = r.backlog_msg_ms;
    out64[kViolationMs * lanes + l] = r.violation_ms;
    out64[kPeakBacklog * lanes + l] = r.peak_backlog;
    out64[kArrived * lanes + l] = r.arrived;
    out64[kServed * lanes + l] = r.served;
    out64[kFinalBacklog * lanes + l] = r.final_backlog;
    out32[kUps * lanes + l] = r.ups;
    out32[kDowns * lanes + l] = r.downs;
    out32[kFinal * lanes + l] = r.final_replicas;
    out32[kMaxRep * lanes + l] = r.max_replicas;
    out32[kPolls * lanes + l] = r.polls;
  }
}

bool ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  g_queue_error = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

// Launches one arithmetic's kernel on the arena's stream; the grid is one resident wave of
// workgroups.
template <class A, class T, bool kMs = false>
bool launch(const ksa_gpu::DeviceArena& ar, const int64_t* d_p, int64_t m, int32_t seeds, uint64_t seed0,
            const ksa_sim::Latency& lat, const ksa_sim::QueueModel& qm, const T* d_t, const T* d_r, int32_t n,
            int32_t init, int64_t horizon_ns, int64_t* d_o64, int32_t* d_o32) {
  const int64_t lanes = m * seeds;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, queue_sweep_kernel<A, T, kMs>, kBlock, 0) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t want = (lanes + kBlock - 1) / kBlock;
  const int grid = static_cast<int>(std::min<int64_t>(want, static_cast<int64_t>(ar.cus) * per_cu));
  hipLaunchKernelGGL((queue_sweep_kernel<A, T, kMs>), dim3(grid), dim3(kBlock), 0, ar.stream, d_p, m, seeds, seed0, lat, qm,
                     d_t, d_r, n, init, horizon_ns, d_o64, d_o32);
  return ok(hipGetLastError(), "queue_sweep_kernel launch");
}

}  // namespace

extern "C" {

const char* ksa_queue_sweep_last_error() { return g_queue_error.c_str(); }

// trace: n segments (t_ms ascending from 0, rate in msgs/s x1000); model: {service_milli,
// startup_ns, slo_backlog, init_backlog}; latency {sqs, get, update} ns; params [9][m];
// out64 [7][m*seeds] (pod_ms, backlog_msg_ms, violation_ms, peak_backlog, arrived, served,
// final_backlog); out32 [5][m*seeds] (ups, downs, final, max_replicas, polls). arith: 0 picks
// FastArith when ksa_sim::fast_path_ok holds, with the decisions on the millisecond clock when
// ksa_sim::ms_clock_ok holds too; 1 forces SatArith; 2 allows FastArith but not the ms clock.
// *fast_used reports the choice: bit 0 FastArith, bit 1 the millisecond clock.
// 0 on success.
int ksa_queue_sweep_gpu(int dev, const int64_t* t_ms, const int64_t* rate_milli, int32_t n, int32_t init_replicas,
                        int64_t horizon_ns, const int64_t* latency, const int64_t* model, const int64_t* params,
                        int64_t m, int32_t seeds, uint64_t seed0, int64_t* out64, int32_t* out32, double* kernel_ms,
                        int32_t arith, int32_t* fast_used) {
  if (n < 1 || t_ms[0] != 0) {
    g_queue_error = "arrival trace must have at least one segment starting at t=0";
    return -1;
  }
  if (seeds < 1) {
    g_queue_error = "seeds must be >= 1";
    return -1;
  }
  for (int k = 0; k < 3; ++k)
    if (latency[k] < 0 || latency[k] > ksa_sim::kMaxLatencyNs) {
      g_queue_error = "latencies must be within [0, 1 h]";
      return -1;
    }
  const int64_t lanes = m * seeds;
  if (lanes <= 0) return 0;
  const ksa_sim::QueueModel qm{model[0], model[1], model[2], model[3]};
  const bool fast = arith != 1 && ksa_sim::fast_path_ok(t_ms, rate_milli, n, qm, init_replicas, horizon_ns, params, m);
  const bool ms_clock = fast && arith == 0 && ksa_sim::ms_clock_ok(horizon_ns, latency, params, m);
  if (fast_used) *fast_used = (fast ? 1 : 0) | (ms_clock ? 2 : 0);
  // the trace in the chosen arithmetic's element type
  std::vector<uint32_t> t32, r32;
  const size_t elem = fast ? sizeof(uint32_t) : sizeof(int64_t);
  const void* h_t = t_ms;
  const void* h_r = rate_milli;
  if (fast) {
    t32.resize(n);
    r32.resize(n);
    ksa_sim::narrow_trace(t_ms, rate_milli, n, t32.data(), r32.data());
    h_t = t32.data();
    h_r = r32.data();
  }
  ksa_gpu::DeviceArena* ar = ksa_gpu::device_arena(dev, &g_queue_error);
  if (!ar) return -1;
  std::lock_guard<std::mutex> lock(ar->mu);
  if (!ok(hipSetDevice(dev), "hipSetDevice")) return -1;
  void *d_t = nullptr, *d_r = nullptr, *d_p = nullptr, *d_o64 = nullptr, *d_o32 = nullptr;
  if (!ok(ar->get(0, n * elem, &d_t), "hipMalloc") || !ok(ar->get(1, n * elem, &d_r), "hipMalloc") ||
      !ok(ar->get(2, kNumParams * m * sizeof(int64_t), &d_p), "hipMalloc") ||
      !ok(ar->get(3, kNumOut64 * lanes * sizeof(int64_t), &d_o64), "hipMalloc") ||
      !ok(ar->get(4, kNumOut32 * lanes * sizeof(int32_t), &d_o32), "hipMalloc"))
    return -1;
  hipStream_t st = ar->stream;
  const ksa_gpu::StreamDrain drain{st};
  if (!ok(hipMemcpyAsync(d_t, h_t, n * elem, hipMemcpyHostToDevice, st), "hipMemcpyAsync") ||
      !ok(hipMemcpyAsync(d_r, h_r, n * elem, hipMemcpyHostToDevice, st), "hipMemcpyAsync") ||
      !ok(hipMemcpyAsync(d_p, params, kNumParams * m * sizeof(int64_t), hipMemcpyHostToDevice, st), "hipMemcpyAsync"))
    return -1;
  const ksa_sim::Latency lat{latency[0], latency[1], latency[2]};
  const int64_t* p = static_cast<const int64_t*>(d_p);
  int64_t* o64 = static_cast<int64_t*>(d_o64);
  int32_t* o32 = static_cast<int32_t*>(d_o32);
  if (!ok(hipEventRecord(ar->e0, st), "hipEventRecord")) return -1;
  const bool launched =
      ms_clock ? launch<ksa_sim::FastArith, uint32_t, true>(*ar, p, m, seeds, seed0, lat, qm,
                                                            static_cast<const uint32_t*>(d_t),
                                                            static_cast<const uint32_t*>(d_r), n, init_replicas,
                                                            horizon_ns, o64, o32)
      : fast ? launch<ksa_sim::FastArith>(*ar, p, m, seeds, seed0, lat, qm, static_cast<const uint32_t*>(d_t),
                                          static_cast<const uint32_t*>(d_r), n, init_replicas, horizon_ns, o64, o32)
           : launch<ksa_sim::SatArith>(*ar, p, m, seeds, seed0, lat, qm, static_cast<const int64_t*>(d_t),
                                       static_cast<const int64_t*>(d_r), n, init_replicas, horizon_ns, o64, o32);
  if (!launched) return -1;
  if (!ok(hipEventRecord(ar->e1, st), "hipEventRecord")) return -1;
  if (!ok(hipMemcpyAsync(out64, o64, kNumOut64 * lanes * sizeof(int64_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync") ||
      !ok(hipMemcpyAsync(out32, o32, kNumOut32 * lanes * sizeof(int32_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync"))
    return -1;
  // (`drain` also synchronizes on the error paths: the host trace copies t32 / r32 die with
  // this frame)
  if (!ok(hipStreamSynchronize(st), "hipStreamSynchronize")) return -1;
  float ms = 0;
  if (!ok(hipEventElapsedTime(&ms, ar->e0, ar->e1), "hipEventElapsedTime")) return -1;
  if (kernel_ms) *kernel_ms = ms;
  return 0;
}

}  // extern "C"
