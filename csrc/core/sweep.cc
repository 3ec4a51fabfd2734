// CPU path of the what-if policy sweep: the same ksa_sim::simulate the gfx950 kernel runs
// (csrc/sim/policy_sim.h), over configurations split across std::threads. Used on hosts without
// a GPU and as the exactness/speed baseline of the kernel.
#include "sweep.h"

#include <algorithm>
#include <thread>
#include <vector>

namespace ksa {

int sweep_cpu(const int64_t* trace_t, const int64_t* trace_d, int32_t n, int32_t init_replicas, int64_t horizon_ns,
              const int64_t* latency, const int64_t* params, int64_t m, int64_t* out64, int32_t* out32, int threads,
              int arith) {
  if (m <= 0 || n < 1) return 0;
  for (int k = 0; k < 3; ++k)
    if (latency[k] < 0 || latency[k] > ksa_sim::kMaxLatencyNs) return 0;  // sweep.py validates first
  const ksa_sim::Latency lat{latency[0], latency[1], latency[2]};
  const bool ms = (arith & 3) == 0 && ksa_sim::ms_path_ok(trace_t, trace_d, n, horizon_ns, latency, params, m);
  const int skip_mode = (arith >> 2) & 3;
  const bool skip = skip_mode == 1 || (skip_mode == 0 && ksa_sim::skip_pays(trace_t, n, horizon_ns, latency, params, m, ms ? 4 : 5));
  const int used = (ms ? 1 : 0) | (skip ? 2 : 0);
  std::vector<int32_t> t32(ms ? n : 0), d32(ms ? n : 0);
  if (ms) ksa_sim::narrow_policy_trace(trace_t, trace_d, n, t32.data(), d32.data());
  const ksa_sim::MsLatency lat_ms = ksa_sim::ms_latency(lat);
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      ksa_sim::Params p;
      p.poll_ns = params[0 * m + i];
      p.up_cool_ns = params[1 * m + i];
      p.down_cool_ns = params[2 * m + i];
      p.up_msgs = params[3 * m + i];
      p.down_msgs = params[4 * m + i];
      p.up_pods = params[5 * m + i];
      p.down_pods = params[6 * m + i];
      p.max_pods = params[7 * m + i];
      p.min_pods = params[8 * m + i];
      const ksa_sim::Result r =
          ms ? (skip ? ksa_sim::simulate_ms<true>(p, lat_ms, t32.data(), d32.data(), n, init_replicas, horizon_ns)
                     : ksa_sim::simulate_ms<false>(p, lat_ms, t32.data(), d32.data(), n, init_replicas, horizon_ns))
             : (skip ? ksa_sim::simulate<true>(p, lat, trace_t, trace_d, n, init_replicas, horizon_ns)
                     : ksa_sim::simulate<false>(p, lat, trace_t, trace_d, n, init_replicas, horizon_ns));
      out64[0 * m + i] = r.pod_ms;
      out64[1 * m + i] = r.backlog;
      out64[2 * m + i] = r.first_up_ns;
      out32[0 * m + i] = r.ups;
      out32[1 * m + i] = r.downs;
      out32[2 * m + i] = r.noop_ups;
      out32[3 * m + i] = r.noop_downs;
      out32[4 * m + i] = r.final_replicas;
      out32[5 * m + i] = r.max_replicas;
      out32[6 * m + i] = r.polls;
    }
  };
  int t = std::max(1, threads);
  if (t > m) t = static_cast<int>(m);
  if (t == 1) {
    work(0, m);
    return used;
  }
  // Interleaved chunks balance the (period-dependent) cost across threads.
  std::vector<std::thread> pool;
  const int64_t chunk = 256;
  std::atomic<int64_t> next{0};
  for (int k = 0; k < t; ++k)
    pool.emplace_back([&] {
      for (;;) {
        const int64_t lo = next.fetch_add(chunk);
        if (lo >= m) return;
        work(lo, std::min(m, lo + chunk));
      }
    });
  for (auto& th : pool) th.join();
  return used;
}

int queue_sweep_cpu(const int64_t* t_ms, const int64_t* rate_milli, int32_t n, int32_t init_replicas,
                     int64_t horizon_ns, const int64_t* latency, const int64_t* model, const int64_t* params, int64_t m,
                     int32_t seeds, uint64_t seed0, int64_t* out64, int32_t* out32, int threads, int arith) {
  const int64_t lanes = m * seeds;
  if (lanes <= 0 || n < 1) return 0;
  for (int k = 0; k < 3; ++k)
    if (latency[k] < 0 || latency[k] > ksa_sim::kMaxLatencyNs) return 0;  // closedloop.py validates first
  const ksa_sim::Latency lat{latency[0], latency[1], latency[2]};
  const ksa_sim::QueueModel qm{model[0], model[1], model[2], model[3]};
  const bool fast = arith != 1 && ksa_sim::fast_path_ok(t_ms, rate_milli, n, qm, init_replicas, horizon_ns, params, m);
  const bool ms_clock = fast && arith == 0 && ksa_sim::ms_clock_ok(horizon_ns, latency, params, m);
  std::vector<uint32_t> t32(fast ? n : 0), r32(fast ? n : 0);
  if (fast) ksa_sim::narrow_trace(t_ms, rate_milli, n, t32.data(), r32.data());
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t l = lo; l < hi; ++l) {
      const int64_t i = l / seeds;
      const int32_t s = static_cast<int32_t>(l - i * seeds);
      ksa_sim::Params p;
      p.poll_ns = params[0 * m + i];
      p.up_cool_ns = params[1 * m + i];
      p.down_cool_ns = params[2 * m + i];
      p.up_msgs = params[3 * m + i];
      p.down_msgs = params[4 * m + i];
      p.up_pods = params[5 * m + i];
      p.down_pods = params[6 * m + i];
      p.max_pods = params[7 * m + i];
      p.min_pods = params[8 * m + i];
      const uint64_t seed = seed0 + static_cast<uint64_t>(s);
      const ksa_sim::QueueResult r =
          ms_clock ? ksa_sim::simulate_queue_ms(p, lat, qm, t32.data(), r32.data(), n, init_replicas, horizon_ns, seed)
          : fast   ? ksa_sim::simulate_queue<ksa_sim::FastArith>(p, lat, qm, t32.data(), r32.data(), n, init_replicas,
                                                               horizon_ns, seed)
               : ksa_sim::simulate_queue<ksa_sim::SatArith>(p, lat, qm, t_ms, rate_milli, n, init_replicas, horizon_ns,
                                                            seed);
      const int64_t o64[7] = {r.pod_ms, r.backlog_msg_ms, r.violation_ms, r.peak_backlog, r.arrived, r.served,
                              r.final_backlog};
      const int32_t o32[5] = {r.ups, r.downs, r.final_replicas, r.max_replicas, r.polls};
      for (int f = 0; f < 7; ++f) out64[f * lanes + l] = o64[f];
      for (int f = 0; f < 5; ++f) out32[f * lanes + l] = o32[f];
    }
  };
  int t = std::max(1, threads);
  if (t > lanes) t = static_cast<int>(lanes);
  const int used = (fast ? 1 : 0) | (ms_clock ? 2 : 0);
  if (t == 1) {
    work(0, lanes);
    return used;
  }
  std::vector<std::thread> pool;
  const int64_t chunk = 256;
  std::atomic<int64_t> next{0};
  for (int k = 0; k < t; ++k)
    pool.emplace_back([&] {
      for (;;) {
        const int64_t lo = next.fetch_add(chunk);
        if (lo >= lanes) return;
        work(lo, std::min(lanes, lo + chunk));
      }
    });
  for (auto& th : pool) th.join();
  return used;
}

}  // namespace ksa
