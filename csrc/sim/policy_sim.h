// Reference-semantics policy simulation for what-if sweeps (extension: tuning tool).
//
// One call simulates one candidate configuration of the reference's loop
// (/root/reference/main.go:35-78, /root/reference/scale/scale.go:54-107 -- the rules of
// SURVEY.md §3.3, identical to kube_sqs_autoscaler_amd/models/oracle.py) over a recorded or
// synthetic queue-depth trace, on a virtual clock with a constant per-call latency model, up to a
// time horizon. It is written once and compiled twice: into the gfx950 sweep kernel
// (csrc/hip/policy_sweep.hip, one configuration per lane) and into the multithreaded CPU path
// (csrc/core/sweep.cc). All arithmetic is integer, so both paths and the Python oracle agree
// exactly.
//
// Metrics, accumulated as a left Riemann sum between successive polls (and from t=0 to the first
// poll, and from the last poll to the horizon):
//   pod_ms   = sum(replicas * dt_ms)                          -- cost (pod-milliseconds)
//   backlog  = sum over runs of constant replicas r of
//              floor(sum(depth * dt_ms) / max(r, 1))          -- queue pressure per pod (msg-ms/pod)
// where depth/replicas are the values observed/set at the left poll (the trace's depth at t=0 and
// the initial replicas before the first poll). Dividing once per run instead of once per poll
// keeps a 64-bit integer division (a long expansion on the GPU) out of the per-poll path.
#pragma once

#include <cstdint>
#include <climits>

#if defined(__HIPCC__)
#define KSA_HD __host__ __device__ __forceinline__
#else
#define KSA_HD inline
#endif

// Keeps the compiler from folding select(c, x / k, y / k) back into select(c, x, y) / k,
// which would put the 64-bit division by 10^6 straight back into the per-poll loop.
#if defined(__HIP_DEVICE_COMPILE__)
#define KSA_OPAQUE(x) __asm__ volatile("" : "+v"(x))
#else
#define KSA_OPAQUE(x) __asm__ volatile("" : "+r"(x))
#endif

namespace ksa_sim {

// Hard per-configuration bound on simulated polls, so every GPU lane reaches its exit even for
// a degenerate request (the host also refuses sweeps whose estimated work exceeds a budget).
constexpr int32_t kMaxPolls = 1 << 26;
// Per-call latency bound of the model (hosts reject larger values): keeps the per-poll interval
// offsets below in 32 bits.
constexpr int64_t kMaxLatencyNs = 3600LL * 1000000000LL;

struct Params {
  int64_t poll_ns, up_cool_ns, down_cool_ns;
  int64_t up_msgs, down_msgs;
  int64_t up_pods, down_pods, max_pods, min_pods;  // as given on the command line (Go int)
};

struct Latency {
  int64_t sqs_ns, get_ns, update_ns;
};

struct Result {
  int64_t pod_ms = 0;
  int64_t backlog = 0;
  int32_t ups = 0, downs = 0, noop_ups = 0, noop_downs = 0;
  int32_t final_replicas = 0, max_replicas = 0;
  int64_t first_up_ns = -1;
  int32_t polls = 0;
};

KSA_HD int32_t go_i32(int64_t v) { return static_cast<int32_t>(static_cast<uint32_t>(static_cast<uint64_t>(v))); }
KSA_HD int32_t add_i32(int32_t a, int32_t b) { return static_cast<int32_t>(static_cast<uint32_t>(a) + static_cast<uint32_t>(b)); }
KSA_HD int32_t sub_i32(int32_t a, int32_t b) { return static_cast<int32_t>(static_cast<uint32_t>(a) - static_cast<uint32_t>(b)); }

// Trace: n segments, segment i covers [t_ns[i], t_ns[i+1]) with depth[i]; t_ns[0] must be 0.
// Forward-only cursor with the next boundary and depth held in registers: advancing issues the
// loads for the segment after next right away, so on the GPU their latency overlaps the rest of
// the poll instead of stalling the next lookup (lookups are one per poll and times only grow).
struct Cursor {
  int32_t c;
  int64_t cur_d, next_t, next_d;
};

constexpr int64_t kNever = INT64_MAX;

KSA_HD Cursor cursor_init(const int64_t* t_ns, const int64_t* depth, int32_t n) {
  Cursor k;
  k.c = 0;
  k.cur_d = depth[0];
  k.next_t = n > 1 ? t_ns[1] : kNever;
  k.next_d = n > 1 ? depth[1] : 0;
  return k;
}

KSA_HD int64_t depth_at(const int64_t* t_ns, const int64_t* depth, int32_t n, Cursor* k, int64_t t) {
  while (t >= k->next_t) {
    k->c++;
    k->cur_d = k->next_d;
    if (k->c + 1 < n) {
      k->next_t = t_ns[k->c + 1];
      k->next_d = depth[k->c + 1];
    } else {
      k->next_t = kNever;
    }
  }
  return k->cur_d;
}

struct Accum {
  int64_t run = 0;      // sum(depth * dt_ms) over the current run of constant replicas
  int32_t run_r = 0;    // replicas of the current run
};

KSA_HD void flush(Result* r, Accum* a) {
  const int64_t div = a->run_r > 0 ? a->run_r : 1;
  r->backlog += a->run / div;
  a->run = 0;
}

KSA_HD void accumulate_ms(Result* r, Accum* a, int64_t dt_ms, int32_t replicas, int64_t depth) {
  r->pod_ms += static_cast<int64_t>(replicas) * dt_ms;
  if (replicas != a->run_r) {
    flush(r, a);
    a->run_r = replicas;
  }
  a->run += depth * dt_ms;
}

constexpr int64_t kTimeBound = int64_t(1) << 61;

KSA_HD int64_t clamp_cool(int64_t c) { return c > kTimeBound ? kTimeBound : (c < -kTimeBound ? -kTimeBound : c); }

// Per-configuration constants of the decision rules (Go int -> int32 conversions done once).
struct Rules {
  int64_t up_msgs, down_msgs, up_cool, down_cool, period;
  int32_t max32, min32, up32, down32;
};

KSA_HD Rules make_rules(const Params& p) {
  Rules k;
  k.up_msgs = p.up_msgs;
  k.down_msgs = p.down_msgs;
  // Timers stay below 2^61 (the host bounds horizon and latencies), so clamping the cool-downs
  // to +-2^61 keeps `last + cool` from overflowing without changing any comparison with `now`.
  k.up_cool = clamp_cool(p.up_cool_ns);
  k.down_cool = clamp_cool(p.down_cool_ns);
  k.period = p.poll_ns > 0 ? (p.poll_ns < kTimeBound ? p.poll_ns : kTimeBound) : 0;
  k.max32 = go_i32(p.max_pods);
  k.min32 = go_i32(p.min_pods);
  k.up32 = go_i32(p.up_pods);
  k.down32 = go_i32(p.down_pods);
  return k;
}

// One poll's decision, main.go:51-77 with scale.go:54-107, on the virtual clock, as a statement
// macro shared by the open-loop (below) and closed-loop (queue_sim.h) simulators. `now` is the
// time the SQS call returned; each GET / write advances it by its latency, so later comparisons
// see the later time, as the reference re-reads time.Now() at every comparison. `gets`/`writes`
// count the API calls (they pick the next poll interval). ON_UP / ON_NOOP_UP / ON_DOWN /
// ON_NOOP_DOWN are statements run inside each action's branch.
// A macro, not a function: as a force-inlined function taking the state by pointer (or by
// reference, or returning it) the open-loop kernel's poll loop compiled 8 instructions longer
// and ran 6 % slower on gfx950 (29.96 vs 28.2 ms for 1M configurations, same box).
#define KSA_DECIDE(k, lat, d, now, last_up, last_down, replicas, gets, writes, ON_UP, ON_NOOP_UP, ON_DOWN,    \
                   ON_NOOP_DOWN)                                                                               \
  do {                                                                                                         \
    bool ksa_cont_ = false;                                                                                    \
    if ((d) >= (k).up_msgs) { /* main.go:51 */                                                                 \
      if ((last_up) + (k).up_cool > (now)) { /* main.go:52 (strict After) */                                   \
        ksa_cont_ = true;                                                                                      \
      } else {                                                                                                 \
        (now) += (lat).get_ns;                                                                                 \
        (gets)++;                                                                                              \
        if ((replicas) >= (k).max32) { /* scale.go:62 */                                                       \
          ON_NOOP_UP;                                                                                          \
        } else {                                                                                               \
          int32_t ksa_next_ = add_i32((replicas), (k).up32);                                                   \
          if (ksa_next_ > (k).max32) ksa_next_ = (k).max32;                                                    \
          (now) += (lat).update_ns;                                                                            \
          (writes)++;                                                                                          \
          (replicas) = ksa_next_;                                                                              \
          ON_UP;                                                                                               \
        }                                                                                                      \
        (last_up) = (now); /* main.go:62 (also after a no-op) */                                               \
      }                                                                                                        \
    }                                                                                                          \
    if (!ksa_cont_ && (d) <= (k).down_msgs) { /* main.go:65 */                                                 \
      if (!((last_down) + (k).down_cool > (now))) {                                                            \
        (now) += (lat).get_ns;                                                                                 \
        (gets)++;                                                                                              \
        if ((replicas) <= (k).min32) { /* scale.go:89 */                                                       \
          ON_NOOP_DOWN;                                                                                        \
        } else {                                                                                               \
          int32_t ksa_next_ = sub_i32((replicas), (k).down32);                                                 \
          if (ksa_next_ < (k).min32) ksa_next_ = (k).min32;                                                    \
          (now) += (lat).update_ns;                                                                            \
          (writes)++;                                                                                          \
          (replicas) = ksa_next_;                                                                              \
          ON_DOWN;                                                                                             \
        }                                                                                                      \
        (last_down) = (now); /* main.go:76 */                                                                  \
      }                                                                                                        \
    }                                                                                                          \
  } while (0)

// The time between two polls is the period plus the earlier poll's API latency: sqs plus 0-2
// GETs and at most as many writes, so one of six values. Their millisecond floors are taken once
// per configuration; the per-poll metric update then selects one instead of dividing a 64-bit
// interval (a long multiply-high expansion on the GPU). Exact: same operands, same division.
// The other five differ from the first by at most the latencies (bounded by the host: <= 1 h
// each), so they are kept as 32-bit offsets -- fewer registers, more resident waves.
struct Intervals {
  int64_t g0;
  int32_t g1u0, g1u1, g2u0, g2u1, g2u2;
};

KSA_HD Intervals make_intervals(int64_t period, const Latency& lat) {
  const int64_t base = period + lat.sqs_ns;
  Intervals t;
  t.g0 = base / 1000000;
  int32_t g1u0 = static_cast<int32_t>((base + lat.get_ns) / 1000000 - t.g0);
  int32_t g1u1 = static_cast<int32_t>((base + lat.get_ns + lat.update_ns) / 1000000 - t.g0);
  int32_t g2u0 = static_cast<int32_t>((base + 2 * lat.get_ns) / 1000000 - t.g0);
  int32_t g2u1 = static_cast<int32_t>((base + 2 * lat.get_ns + lat.update_ns) / 1000000 - t.g0);
  int32_t g2u2 = static_cast<int32_t>((base + 2 * lat.get_ns + 2 * lat.update_ns) / 1000000 - t.g0);
  KSA_OPAQUE(g1u0);
  KSA_OPAQUE(g1u1);
  KSA_OPAQUE(g2u0);
  KSA_OPAQUE(g2u1);
  KSA_OPAQUE(g2u2);
  t.g1u0 = g1u0;
  t.g1u1 = g1u1;
  t.g2u0 = g2u0;
  t.g2u1 = g2u1;
  t.g2u2 = g2u2;
  return t;
}

// By value on purpose: with a reference, the selects between fields became a select between
// field addresses, which kept the struct in scratch memory (a dynamically indexed private load
// per poll on the GPU).
KSA_HD int64_t interval_ms(Intervals t, int32_t gets, int32_t writes) {
  const int32_t g2 = writes == 0 ? t.g2u0 : (writes == 1 ? t.g2u1 : t.g2u2);
  return t.g0 + (gets == 0 ? 0 : (gets == 1 ? (writes == 0 ? t.g1u0 : t.g1u1) : g2));
}

// Steady stretches. A poll that called nothing leaves the timers and replicas as they were, so
// the polls after it call nothing either for as long as they see the same depth (until the
// trace's next boundary) and (a) that depth is strictly between the thresholds, or (b) it is at
// or past a threshold whose cool-down has not run out: blocked at `now` = t + sqs, it stays
// blocked while t + sqs < last + cool (the up check, blocked, also skips the down check, as the
// reference's `continue` does). Each such poll only adds a left sum of the same dt, so the
// simulators add a whole stretch at once, and a lane's loop runs once per decision or trace
// boundary instead of once per poll. Returns the exclusive bound on the start time of a poll in
// the stretch, capped at horizon + 1 (a poll starts at t <= horizon). T: int32 on the
// millisecond clock, int64 on the nanosecond one; the hosts' bounds keep every sum in range.
template <class K, class T>
KSA_HD T steady_limit(const K& k, T d, T last_up, T last_down, T sqs, T next_t, T horizon) {
  T lim = next_t < horizon + 1 ? next_t : horizon + 1;
  if (d >= k.up_msgs) {
    const T b = last_up + k.up_cool - sqs;
    if (b < lim) lim = b;
  } else if (d <= k.down_msgs) {
    const T b = last_down + k.down_cool - sqs;
    if (b < lim) lim = b;
  }
  return lim;
}

// floor(x / s) capped at `cap`, for 0 <= x < 2^60, 1 <= s <= 2^62 and cap <= 2^26 (the skip's
// poll count on the nanosecond clock): a double-precision estimate, then one exact integer step
// either way, instead of the GPU's long 64-bit division sequence. Below the cap the quotient is
// under 2^27, where the estimate's relative error (a few 2^-53) is far below one, so it is off by
// at most one only when x / s is within that error of an integer; the products stay below 2^63.
KSA_HD int64_t capped_quotient(int64_t x, int64_t s, int64_t cap) {
  const double e = static_cast<double>(x) / static_cast<double>(s);
  if (e >= static_cast<double>(cap) + 2.0) return cap;
  int64_t q = static_cast<int64_t>(e);
  if (q * s > x)
    --q;
  else if ((q + 1) * s <= x)
    ++q;
  return q < cap ? q : cap;
}

template <bool kSkip = true>
KSA_HD Result simulate(const Params& p, const Latency& lat, const int64_t* t_ns, const int64_t* depth, int32_t n,
                       int32_t init_replicas, int64_t horizon_ns) {
  Result res;
  Accum acc;
  acc.run_r = init_replicas;
  Cursor cursor = cursor_init(t_ns, depth, n);
  const Rules k = make_rules(p);
  int64_t now = 0;
  int64_t last_up = 0, last_down = 0;  // main.go:37-38
  int32_t replicas = init_replicas;
  int64_t prev_t = 0;
  int64_t prev_d = depth_at(t_ns, depth, n, &cursor, 0);
  res.max_replicas = replicas;
  const Intervals iv = make_intervals(k.period, lat);
  int64_t dt_ms = k.period / 1000000;  // t=0 -> first poll: no latency before it
  // Guard: a zero period with zero latency would never advance time.
  const bool advances = k.period > 0 || lat.sqs_ns > 0;
  while (advances && res.polls < kMaxPolls) {
    const int64_t t_poll = now + k.period;  // main.go:41 sleep, then poll
    if (t_poll > horizon_ns) break;
    now = t_poll;
    accumulate_ms(&res, &acc, dt_ms, replicas, prev_d);  // replicas as set by the previous poll
    prev_t = now;
    res.polls++;
    const int64_t d = depth_at(t_ns, depth, n, &cursor, now);  // sampled at call start
    now += lat.sqs_ns;
    int32_t gets = 0, writes = 0;
    KSA_DECIDE(k, lat, d, now, last_up, last_down, replicas, gets, writes,
               { res.ups++; if (res.first_up_ns < 0) res.first_up_ns = t_poll; }, res.noop_ups++, res.downs++,
               res.noop_downs++);
    if (replicas > res.max_replicas) res.max_replicas = replicas;
    prev_d = d;
    dt_ms = interval_ms(iv, gets, writes);
    if (kSkip && gets == 0) {  // a poll that called nothing: skip the stretch of polls just like it
      const int64_t lim = steady_limit(k, d, last_up, last_down, lat.sqs_ns, cursor.next_t, horizon_ns);
      const int64_t s = k.period + lat.sqs_ns;
      const int64_t t1 = now + k.period;
      if (t1 < lim) {
        const int64_t j = capped_quotient(lim - 1 - t1, s, kMaxPolls - res.polls - 1) + 1;
        res.pod_ms += static_cast<int64_t>(replicas) * dt_ms * j;  // j left sums of dt_ms, one run
        acc.run += d * dt_ms * j;
        res.polls += static_cast<int32_t>(j);
        prev_t += j * s;
        now = prev_t + lat.sqs_ns;
      }
    }
  }
  if (horizon_ns > prev_t) accumulate_ms(&res, &acc, (horizon_ns - prev_t) / 1000000, replicas, prev_d);
  flush(&res, &acc);
  res.final_replicas = replicas;
  return res;
}

// ---- Millisecond clock (the usual sweep: periods and latencies in whole milliseconds) --------
//
// When every poll period that can fire and every call latency is a whole number of
// milliseconds, every time the simulation produces is one too (sums of periods and latencies),
// so it can run on 32-bit millisecond clocks with the same decisions and metrics:
//   * a cool-down c enters as ceil(c / 1 ms): for whole-ms `last` and `now`,
//     last + c > now  <=>  c > (now - last)  <=>  ceil(c / 1 ms) > (now - last) / 1 ms;
//   * a trace boundary T as ceil(T / 1 ms): a whole-ms poll time t reaches it iff t >= that;
//   * the horizon H as floor(H / 1 ms): a whole-ms poll time t <= H iff t <= that, and the last
//     interval's floor((H - t) / 1 ms) is floor(H / 1 ms) - t;
//   * every time a lane holds stays within B = H + sqs + 2 (get + update) (ms); cool-downs and
//     periods beyond +-(B + 1) compare and end the loop as the clamped values do, and the host
//     (ms_path_ok) requires 2B + 1 < 2^31, so no 32-bit sum can wrap;
//   * depths are in [0, 2^31 - 2] (checked by the host), so thresholds clamp to 32 bits.
// On gfx950 this drops the per-poll 64-bit compares, adds and 64 x 64 products (each several
// VALU instructions) and halves the trace's LDS footprint. The CPU path runs the same function
// for the same sweeps, and tests pin it equal to simulate() on randomised inputs.
constexpr int32_t kMsNever = INT32_MAX;

// Th: the thresholds' type -- int32 for a replayed trace (depths bounded by the host), int64 for
// the closed-loop queue (queue_sim.h), whose backlog has no such bound.
template <class Th>
struct MsRulesT {
  Th up_msgs, down_msgs;
  int32_t up_cool, down_cool, period;
  int32_t max32, min32, up32, down32;
};
using MsRules = MsRulesT<int32_t>;

// Latencies in milliseconds (the field names are KSA_DECIDE's).
struct MsLatency {
  int32_t sqs_ns, get_ns, update_ns;
};

KSA_HD int64_t ceil_div_1e6(int64_t v) {
  const int64_t q = v / 1000000;  // truncates toward zero: already the ceiling for v < 0
  return q * 1000000 < v ? q + 1 : q;
}

KSA_HD int32_t clamp_i32(int64_t v, int64_t lo, int64_t hi) {
  return static_cast<int32_t>(v < lo ? lo : (v > hi ? hi : v));
}

KSA_HD MsLatency ms_latency(const Latency& lat) {
  return MsLatency{static_cast<int32_t>(lat.sqs_ns / 1000000), static_cast<int32_t>(lat.get_ns / 1000000),
                   static_cast<int32_t>(lat.update_ns / 1000000)};
}

// B: the bound on every time value of a lane (see above).
KSA_HD int32_t ms_bound(int32_t horizon_ms, const MsLatency& lat) {
  return horizon_ms + lat.sqs_ns + 2 * (lat.get_ns + lat.update_ns);
}

template <class Th = int32_t>
KSA_HD MsRulesT<Th> make_ms_rules(const Params& p, int64_t horizon_ns, int32_t bound) {
  MsRulesT<Th> k;
  const int64_t b1 = static_cast<int64_t>(bound) + 1;
  if constexpr (sizeof(Th) == 4) {
    k.up_msgs = clamp_i32(p.up_msgs, 0, INT32_MAX);       // d >= up_msgs, d in [0, 2^31 - 2]
    k.down_msgs = clamp_i32(p.down_msgs, -1, INT32_MAX);  // d <= down_msgs
  } else {
    k.up_msgs = p.up_msgs;
    k.down_msgs = p.down_msgs;
  }
  k.up_cool = clamp_i32(ceil_div_1e6(p.up_cool_ns), -b1, b1);
  k.down_cool = clamp_i32(ceil_div_1e6(p.down_cool_ns), -b1, b1);
  // a period past the horizon never fires (its first poll is past it); others are whole ms
  k.period = p.poll_ns <= 0 ? 0 : (p.poll_ns > horizon_ns ? static_cast<int32_t>(b1) : clamp_i32(p.poll_ns / 1000000, 0, b1));
  k.max32 = go_i32(p.max_pods);
  k.min32 = go_i32(p.min_pods);
  k.up32 = go_i32(p.up_pods);
  k.down32 = go_i32(p.down_pods);
  return k;
}

struct MsCursor {
  int32_t c;
  int32_t cur_d, next_t, next_d;
};

KSA_HD MsCursor ms_cursor_init(const int32_t* t_ms, const int32_t* depth, int32_t n) {
  MsCursor k;
  k.c = 0;
  k.cur_d = depth[0];
  k.next_t = n > 1 ? t_ms[1] : kMsNever;
  k.next_d = n > 1 ? depth[1] : 0;
  return k;
}

KSA_HD int32_t ms_depth_at(const int32_t* t_ms, const int32_t* depth, int32_t n, MsCursor* k, int32_t t) {
  while (t >= k->next_t) {
    k->c++;
    k->cur_d = k->next_d;
    if (k->c + 1 < n) {
      k->next_t = t_ms[k->c + 1];
      k->next_d = depth[k->c + 1];
    } else {
      k->next_t = kMsNever;
    }
  }
  return k->cur_d;
}

KSA_HD void accumulate_ms32(Result* r, Accum* a, int32_t dt_ms, int32_t replicas, int32_t depth) {
  r->pod_ms += static_cast<int64_t>(replicas) * dt_ms;
  if (replicas != a->run_r) {
    flush(r, a);
    a->run_r = replicas;
  }
  a->run += static_cast<int64_t>(depth) * dt_ms;
}

// simulate() on the millisecond clock: t_ms / depth as narrow_policy_trace makes them.
template <bool kSkip = true>
KSA_HD Result simulate_ms(const Params& p, const MsLatency& lat, const int32_t* t_ms, const int32_t* depth, int32_t n,
                          int32_t init_replicas, int64_t horizon_ns) {
  Result res;
  Accum acc;
  acc.run_r = init_replicas;
  MsCursor cursor = ms_cursor_init(t_ms, depth, n);
  const int32_t horizon_ms = static_cast<int32_t>(horizon_ns / 1000000);
  const MsRules k = make_ms_rules(p, horizon_ns, ms_bound(horizon_ms, lat));
  int32_t now = 0;
  int32_t last_up = 0, last_down = 0;  // main.go:37-38
  int32_t replicas = init_replicas;
  int32_t prev_t = 0;
  int32_t prev_d = ms_depth_at(t_ms, depth, n, &cursor, 0);
  int32_t first_up_ms = -1;
  res.max_replicas = replicas;
  const bool advances = k.period > 0 || lat.sqs_ns > 0;
  while (advances && res.polls < kMaxPolls) {
    const int32_t t_poll = now + k.period;  // main.go:41 sleep, then poll
    if (t_poll > horizon_ms) break;
    now = t_poll;
    accumulate_ms32(&res, &acc, t_poll - prev_t, replicas, prev_d);  // replicas as set by the previous poll
    prev_t = now;
    res.polls++;
    const int32_t d = ms_depth_at(t_ms, depth, n, &cursor, now);  // sampled at call start
    now += lat.sqs_ns;
    int32_t gets = 0, writes = 0;
    KSA_DECIDE(k, lat, d, now, last_up, last_down, replicas, gets, writes,
               { res.ups++; if (first_up_ms < 0) first_up_ms = t_poll; }, res.noop_ups++, res.downs++,
               res.noop_downs++);
    (void)gets;
    (void)writes;
    if (replicas > res.max_replicas) res.max_replicas = replicas;
    prev_d = d;
    if (kSkip && gets == 0) {  // a poll that called nothing: skip the stretch of polls just like it
      const int32_t lim = steady_limit(k, d, last_up, last_down, lat.sqs_ns, cursor.next_t, horizon_ms);
      const int32_t s = k.period + lat.sqs_ns;
      const int32_t t1 = now + k.period;
      if (t1 < lim) {
        int32_t j = (lim - 1 - t1) / s + 1;
        if (j > kMaxPolls - res.polls) j = kMaxPolls - res.polls;
        const int64_t span = static_cast<int64_t>(j) * s;
        res.pod_ms += static_cast<int64_t>(replicas) * span;  // j left sums of dt = s, one run
        acc.run += static_cast<int64_t>(d) * span;
        res.polls += j;
        prev_t = static_cast<int32_t>(prev_t + span);
        now = prev_t + lat.sqs_ns;
      }
    }
  }
  if (horizon_ms > prev_t) accumulate_ms32(&res, &acc, horizon_ms - prev_t, replicas, prev_d);
  flush(&res, &acc);
  res.first_up_ns = first_up_ms < 0 ? -1 : static_cast<int64_t>(first_up_ms) * 1000000;
  res.final_replicas = replicas;
  return res;
}

// Host check for simulate_ms (see above): whole-ms latencies, whole-ms periods wherever a
// period can fire (0 < poll <= horizon), depths in [0, 2^31 - 2], and 2B + 1 < 2^31.
// The clock part of it, shared with the closed-loop simulator (queue_sim.h).
inline bool ms_clock_ok(int64_t horizon_ns, const int64_t* latency, const int64_t* params, int64_t configs) {
  if (horizon_ns < 0) return false;
  int64_t lat_ms = 0;
  for (int k = 0; k < 3; ++k) {
    if (latency[k] < 0 || latency[k] > kMaxLatencyNs || latency[k] % 1000000 != 0) return false;
    lat_ms += (k == 0 ? 1 : 2) * (latency[k] / 1000000);
  }
  const int64_t bound = horizon_ns / 1000000 + lat_ms;
  if (2 * bound + 1 >= (int64_t(1) << 31)) return false;
  for (int64_t i = 0; i < configs; ++i) {
    const int64_t poll = params[i];  // params [9][m]: poll first
    if (poll > 0 && poll <= horizon_ns && poll % 1000000 != 0) return false;
  }
  return true;
}

inline bool ms_path_ok(const int64_t* t_ns, const int64_t* depth, int32_t n, int64_t horizon_ns, const int64_t* latency,
                       const int64_t* params, int64_t configs) {
  if (n < 1 || t_ns[0] != 0) return false;
  for (int32_t i = 0; i < n; ++i)
    if (depth[i] < 0 || depth[i] > INT32_MAX - 1) return false;
  return ms_clock_ok(horizon_ns, latency, params, configs);
}

// Whether the steady-stretch skip (simulate<true>) pays for a sweep: only when a trace segment
// spans `polls` polls or more -- a coarse trace (a sample a minute) under a poll of a few seconds.
// On a trace sampled at every poll (--trace-file spans, or 5 s samples under a 5 s poll) no
// stretch forms, and the check alone made the gfx950 kernel 19 % slower (profiles/r04v). Measured
// on gfx950 (profiles/r04aa): the millisecond clock gains from 3-4 polls a segment (3: 1.07x, 6:
// 1.65x, 12: 2.21x); the nanosecond clock, whose skip count takes a capped_quotient, from 5-6
// (3: 0.79x, 6: 1.19x, 12: 1.71x).
// The results do not depend on the choice: a skipped stretch adds exactly what its polls would.
inline bool skip_pays(const int64_t* t_ns, int32_t n, int64_t horizon_ns, const int64_t* latency, const int64_t* params,
                      int64_t configs, int64_t polls) {
  int64_t within = 0;  // segments starting inside the horizon
  while (within < n && t_ns[within] <= horizon_ns) ++within;
  if (within < 1) within = 1;
  const int64_t seg = horizon_ns / within;
  int64_t step = INT64_MAX;  // the shortest poll-to-poll interval of the grid
  for (int64_t i = 0; i < configs; ++i) {
    const int64_t poll = params[i] > 0 ? params[i] : 0;
    const int64_t st = poll < kMaxLatencyNs ? poll + latency[0] : kMaxLatencyNs;
    if (st > 0 && st < step) step = st;
  }
  return step != INT64_MAX && step <= seg / polls;
}

// The trace as simulate_ms reads it: boundaries ceil(t / 1 ms) (kMsNever past 2^31 ms), depths.
inline void narrow_policy_trace(const int64_t* t_ns, const int64_t* depth, int32_t n, int32_t* t32, int32_t* d32) {
  for (int32_t i = 0; i < n; ++i) {
    const int64_t t = ceil_div_1e6(t_ns[i]);
    t32[i] = t < kMsNever ? static_cast<int32_t>(t) : kMsNever;
    d32[i] = static_cast<int32_t>(depth[i]);
  }
}

}  // namespace ksa_sim
