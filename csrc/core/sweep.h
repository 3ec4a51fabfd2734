// What-if policy sweep, CPU path (see csrc/sim/policy_sim.h for the model and the metrics).
#pragma once

#include <atomic>
#include <cstdint>

#include "../sim/policy_sim.h"

namespace ksa {

// Layouts as in ksa_sweep_gpu (csrc/hip/policy_sweep.hip): params [9][m], out64 [3][m],
// out32 [7][m], latency {sqs, get, update} ns.
void sweep_cpu(const int64_t* trace_t, const int64_t* trace_d, int32_t n, int32_t init_replicas, int64_t horizon_ns,
               const int64_t* latency, const int64_t* params, int64_t m, int64_t* out64, int32_t* out32, int threads);

}  // namespace ksa
