// What-if policy sweep, CPU path (see csrc/sim/policy_sim.h for the model and the metrics).
#pragma once

#include <atomic>
#include <cstdint>

#include "../sim/policy_sim.h"
#include "../sim/queue_sim.h"

namespace ksa {

// Layouts as in ksa_sweep_gpu (csrc/hip/policy_sweep.hip): params [9][m], out64 [3][m],
// out32 [7][m], latency {sqs, get, update} ns. arith bits 0-1: 0 runs ksa_sim::simulate_ms when
// ms_path_ok holds, 1 forces simulate (nanosecond clock); bits 2-3: the steady-stretch skip, 0 when
// ksa_sim::skip_pays, 1 always, 2 never (same results). Returns bit 0: the ms clock ran, bit 1:
// the skip ran.
int sweep_cpu(const int64_t* trace_t, const int64_t* trace_d, int32_t n, int32_t init_replicas, int64_t horizon_ns,
              const int64_t* latency, const int64_t* params, int64_t m, int64_t* out64, int32_t* out32, int threads,
              int arith = 0);

// Closed-loop sweep (csrc/sim/queue_sim.h), CPU path; layouts as ksa_queue_sweep_gpu
// (csrc/hip/queue_sweep.hip): params [9][m], model {service_milli, startup_ns, slo_backlog,
// init_backlog}, out64 [7][m*seeds], out32 [5][m*seeds], lane = config * seeds + seed. arith: 0
// picks ksa_sim::FastArith when fast_path_ok holds (with the millisecond decision clock,
// simulate_queue_ms, when ms_clock_ok holds too), 1 forces SatArith, 2 allows FastArith without
// the ms clock. Returns bit 0: FastArith ran, bit 1: the ms clock ran.
int queue_sweep_cpu(const int64_t* t_ms, const int64_t* rate_milli, int32_t n, int32_t init_replicas,
                     int64_t horizon_ns, const int64_t* latency, const int64_t* model, const int64_t* params, int64_t m,
                     int32_t seeds, uint64_t seed0, int64_t* out64, int32_t* out32, int threads, int arith = 0);

}  // namespace ksa
