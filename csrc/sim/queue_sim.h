// Closed-loop what-if simulation (extension: tuning tool).
//
// policy_sim.h replays a recorded depth trace, so the autoscaler's decisions cannot change the
// depth it sees. Here the depth is state that the replicas drain:
//   * messages arrive at a piecewise-constant rate (a trace of msgs/s);
//   * each ready pod drains `service` msgs/s (fluid service);
//   * a scale-up's pods start draining only `startup` after the write returned (GPU workers pull
//     an image and load a model first); a scale-down removes pending pods before ready ones;
//   * the decisions are the reference's rules -- KSA_DECIDE, the same code policy_sim.h
//     runs -- on the same virtual clock with the same API latency model.
// Arrivals per poll interval are random: a normal approximation of Poisson, its standard normal
// the Irwin-Hall sum of four uniform 16-bit draws (one 64-bit hash) scaled to unit variance,
// integer-only, so the gfx950 kernel and the CPU path agree bit for bit.
// The stream is counter-based on (seed, interval index) and the same seeds are used for every
// configuration (common random numbers), so configurations are compared on the same arrival
// sequences. The backlog is kept in micro-messages: a rate in milli-msgs/s times an interval in ms
// is exactly that unit, so integrating rates needs no division.
//
// One call simulates one (configuration, seed); the host reduces over seeds.
#pragma once

#include "policy_sim.h"

namespace ksa_sim {

struct QueueModel {
  int64_t service_milli;  // msgs/s drained per ready pod, x1000
  int64_t startup_ns;     // delay from a scale-up write to its pods taking work
  int64_t slo_backlog;    // backlog (msgs) above which time counts as an SLO violation
  int64_t init_backlog;   // msgs queued at t=0
};

struct QueueResult {
  int64_t pod_ms = 0;          // sum(spec replicas x dt): cost (starting pods are billed too)
  int64_t backlog_msg_ms = 0;  // sum(backlog x dt): mean backlog = / horizon_ms
  int64_t violation_ms = 0;    // time with backlog > slo_backlog
  int64_t peak_backlog = 0;    // msgs
  int64_t arrived = 0, served = 0, final_backlog = 0;  // msgs
  int32_t ups = 0, downs = 0, final_replicas = 0, max_replicas = 0, polls = 0;
};

// splitmix64 finaliser: the counter-based random stream.
KSA_HD uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// floor(sqrt(x)), exact on CPU and GPU: a floating-point estimate (within a few units whatever
// the rounding of the conversion and the sqrt) corrected with integer arithmetic. (An integer
// Newton iteration is exact too, but each step is a 64-bit division -- a long software sequence on
// the GPU.) Below 2^48 -- every mean arrival count but absurd ones -- the estimate is single
// precision: the two 32-bit halves converted and fused (|relative error| < 2^-23), one
// v_sqrt_f32 (1 ulp) on gfx950, so r < 2^24 is off by at most 3 before the correction; the
// double-precision sqrt it replaces is an rsq-and-Newton sequence of ~20 half-rate instructions
// plus 64-bit conversions each way.
KSA_HD uint64_t isqrt64(uint64_t x) {
  constexpr uint64_t kMax = 0xFFFFFFFFULL;  // floor(sqrt(2^64 - 1))
  uint64_t r;
  if (x < (uint64_t(1) << 48)) {
    const float xf = __builtin_fmaf(static_cast<float>(static_cast<uint32_t>(x >> 32)), 4294967296.0f,
                                    static_cast<float>(static_cast<uint32_t>(x)));
#if defined(__HIP_DEVICE_COMPILE__)
    r = static_cast<uint32_t>(__builtin_amdgcn_sqrtf(xf));
#else
    r = static_cast<uint32_t>(__builtin_sqrtf(xf));
#endif
  } else {
    r = static_cast<uint64_t>(__builtin_sqrt(static_cast<double>(x)));
    if (r > kMax) r = kMax;
  }
  while (r * r > x) --r;
  while (r < kMax && (r + 1) * (r + 1) <= x) ++r;
  return r;
}

constexpr int64_t kSat = int64_t(1) << 62;

// Saturating helpers for non-negative quantities: absurd inputs (a queue that never drains over
// months) clamp instead of overflowing.
// min(a*b, kSat) for a, b > 0 (0 otherwise). Operands below 2^31 -- nearly all of them -- cannot
// reach kSat; the rest use the overflow builtin. No division (a variable 64-bit divide is a long
// software sequence on the GPU).
KSA_HD int64_t sat_mul(int64_t a, int64_t b) {
  if (a <= 0 || b <= 0) return 0;
  if (((a | b) >> 31) == 0) return a * b;
  int64_t r;
  return __builtin_mul_overflow(a, b, &r) || r > kSat ? kSat : r;
}
// x / 10^6 for x >= 0 (backlogs, virtual times): as an unsigned division by a constant it drops
// the signed form's rounding correction (21 fewer VALU instructions in the gfx950 kernel).
KSA_HD int64_t udiv_1e6(int64_t x) { return static_cast<int64_t>(static_cast<uint64_t>(x) / 1000000u); }
// min(a + b, kSat) for 0 <= a, b < 2^63: the unsigned sum cannot wrap, so the add comes first
// and one compare clamps it (the form `a > kSat - b` needs a subtraction and an add on the GPU).
KSA_HD int64_t sat_add(int64_t a, int64_t b) {
  const uint64_t s = static_cast<uint64_t>(a) + static_cast<uint64_t>(b);
  return s > static_cast<uint64_t>(kSat) ? kSat : static_cast<int64_t>(s);
}

// Random arrivals (micro-messages) with mean `mean`: mean + sqrt(mean) * Z. Z is the sum of the
// four 16-bit fields of one splitmix64 draw (Irwin-Hall, n = 4: mean 131070, standard deviation
// 65536/sqrt(3)), centred and scaled by sqrt(3) to a standard deviation of 2^16 in fixed point;
// |Z| < 3.47. Round 2 drew twelve fields from three hashes (the CLT of 12): on gfx950 the three
// 64-bit hashes and their field sums were a third of the VALU work of a simulated poll, and four
// fields already give a normal approximation far finer than the Poisson noise it stands for.
// sqrt(mean) is kept for the last mean (*memo_mean, *memo_sd): polls of one interval length inside
// one rate segment -- most of them -- ask for the same mean, and the isqrt is the longest sequence
// of the poll on the GPU. `key` is seed * kSeedMul + the draw's index: QueueState::key, one
// 64-bit counter per lane (a separate base and index held two).
constexpr int64_t kSqrt3Q16 = 113512;  // round(sqrt(3) * 2^16)
constexpr uint64_t kSeedMul = 0xD1B54A32D192ED03ULL;
KSA_HD int64_t sample_arrivals(int64_t mean, uint64_t key, int64_t* memo_mean, int64_t* memo_sd) {
  if (mean <= 0) return 0;
  const uint64_t w = mix64(key);
  // the four 16-bit fields, summed in two 32-bit lanes (2 x 65535 fits), then folded
  constexpr uint64_t kM = 0x0000FFFF0000FFFFULL;
  const uint64_t lanes = (w & kM) + ((w >> 16) & kM);
  const int32_t u = static_cast<int32_t>((lanes & 0xFFFFFFFFULL) + (lanes >> 32)) - 131070;  // 2 x centred
  const int64_t z = (static_cast<int64_t>(u) * kSqrt3Q16) >> 16;  // arithmetic shift: floor, as Python's >>
  // sd in micro-messages = sqrt(mean / 1e6) * 1e6 = 1000 sqrt(mean), to a milli-message
  if (mean != *memo_mean) {
    *memo_mean = mean;
    *memo_sd = static_cast<int64_t>(isqrt64(static_cast<uint64_t>(mean))) * 1000;
  }
  // |sd * z| < 2^41 * 2^18: no overflow; the shift floors (a division would truncate toward zero
  // and cost a sign fix-up)
  const int64_t a = mean + ((*memo_sd * z) >> 16);
  return a > 0 ? a : 0;
}

// The arithmetic of one simulation, chosen per sweep by the host:
// * SatArith: every accumulator and product saturates at kSat and times are int64 milliseconds,
//   so any input the hosts accept (30-day horizons, 10^6 msgs/s rates, 2^31 replicas) is safe;
// * FastArith: plain integer adds and products and 32-bit millisecond times (every time a lane
//   compares is below the 30-day horizon, < 2^32 ms), for sweeps whose bounds (fast_path_ok) show
//   that no quantity of any lane can reach kSat nor a replica count wrap -- both then compute the
//   same values. On gfx950 the saturation checks, 64-bit time compares and 64 x 64 products were
//   about a fifth of a simulated poll's VALU instructions.
struct SatArith {
  using Ms = int64_t;
  static constexpr Ms kNeverMs = kNever;
  static constexpr bool kExact = false;  // products may saturate: no reassociation
  KSA_HD static int64_t add(int64_t a, int64_t b) { return sat_add(a, b); }
  KSA_HD static int64_t mul(int64_t a, int64_t b) { return sat_mul(a, b); }
  KSA_HD static int64_t count_ms(int32_t c, Ms dt) { return sat_mul(c, dt); }
  // pods x (a per-pod rate in milli-msgs/s x dt): micro-messages
  KSA_HD static int64_t pods_rate_ms(int32_t pods, int64_t rate_milli, Ms dt) {
    return sat_mul(pods, sat_mul(rate_milli, dt));
  }
};

struct FastArith {
  using Ms = uint32_t;
  static constexpr Ms kNeverMs = 0xFFFFFFFFu;
  static constexpr bool kExact = true;  // no product reaches 2^63 (fast_path_ok): sums reassociate
  KSA_HD static int64_t add(int64_t a, int64_t b) { return a + b; }
  KSA_HD static int64_t mul(int64_t a, int64_t b) { return a * b; }
  // counts (replicas, pods) are in [0, 2^31) under fast_path_ok: one 32 x 32 -> 64 multiply
  KSA_HD static int64_t count_ms(int32_t c, Ms dt) {
    return static_cast<int64_t>(static_cast<uint64_t>(static_cast<uint32_t>(c)) * dt);
  }
  KSA_HD static int64_t pods_rate_ms(int32_t pods, int64_t rate_milli, Ms dt) {
    const uint64_t per_pod = static_cast<uint64_t>(static_cast<uint32_t>(rate_milli)) * dt;
    return static_cast<int64_t>(static_cast<uint64_t>(static_cast<uint32_t>(pods)) * per_pod);
  }
  // rate x (ready x dt + pending x late) == pods_rate_ms(ready, rate, dt) +
  // pods_rate_ms(pending, rate, late): ready + pending <= the replica bound R of fast_path_ok and
  // late <= dt, so every partial sum and product is below rate x R x H < 2^61
  KSA_HD static int64_t capacity(int32_t ready, Ms dt, int32_t pending, Ms late, int64_t rate_milli) {
    const uint64_t pod_ms = static_cast<uint64_t>(static_cast<uint32_t>(ready)) * dt +
                            static_cast<uint64_t>(static_cast<uint32_t>(pending)) * late;
    return static_cast<int64_t>(pod_ms * static_cast<uint64_t>(static_cast<uint32_t>(rate_milli)));
  }
};

// Forward-only cursor over the arrival-rate trace, as policy_sim.h's Cursor: the current rate
// and the next boundary and rate live in registers, and advancing issues the loads for the
// segment after that at once. An interval inside one segment (a 5 s poll in a 60 s segment)
// then makes no memory access; before, every poll made 3-4 dependent trace loads. T is the
// trace's element type: int64 (SatArith) or uint32 (FastArith; times clamped to kNeverMs).
template <class A, class T>
struct RateCursor {
  int32_t c;
  typename A::Ms next_t;  // t_ms[c+1] (kNeverMs past the last)
  T rate, next_rate;      // rate_milli[c]; rate_milli[c+1]
};

template <class A, class T>
KSA_HD RateCursor<A, T> rate_cursor_init(const T* t_ms, const T* rate_milli, int32_t n) {
  RateCursor<A, T> k;
  k.c = 0;
  k.rate = rate_milli[0];
  k.next_t = n > 1 ? static_cast<typename A::Ms>(t_ms[1]) : A::kNeverMs;
  k.next_rate = n > 1 ? rate_milli[1] : 0;
  return k;
}

template <class A, class T>
KSA_HD void rate_cursor_advance(const T* t_ms, const T* rate_milli, int32_t n, RateCursor<A, T>* k) {
  k->c++;
  k->rate = k->next_rate;
  if (k->c + 1 < n) {
    k->next_t = static_cast<typename A::Ms>(t_ms[k->c + 1]);
    k->next_rate = rate_milli[k->c + 1];
  } else {
    k->next_t = A::kNeverMs;
  }
}

// Expected arrivals (micro-messages) over [t0_ms, t1_ms): the rate integrated segment by
// segment. Segment i covers [t_ms[i], t_ms[i+1]); the last one extends to infinity. Times only
// grow (each call starts where the last ended), so the cursor never moves back and is left on
// the segment holding t1_ms.
template <class A, class T>
KSA_HD int64_t expected_arrivals(const T* t_ms, const T* rate_milli, int32_t n, RateCursor<A, T>* k,
                                 typename A::Ms t0_ms, typename A::Ms t1_ms) {
  using Ms = typename A::Ms;
  while (t0_ms >= k->next_t) rate_cursor_advance(t_ms, rate_milli, n, k);
  int64_t sum = 0;
  Ms a = t0_ms;
  while (a < t1_ms) {
    const Ms b = k->next_t < t1_ms ? k->next_t : t1_ms;
    sum = A::add(sum, A::mul(k->rate, b - a));  // milli-msgs/s x ms = micro-messages
    a = b;
    if (a >= k->next_t) rate_cursor_advance(t_ms, rate_milli, n, k);
  }
  return sum;
}

template <class A>
struct QueueState {
  int64_t q_micro;       // backlog
  int64_t q_msgs;        // q_micro / 1e6, kept current (the depth SQS reports)
  int32_t ready, pending;
  typename A::Ms pending_at_ms;  // when the pending pods start draining
  uint64_t key;  // the next draw's counter: seed * kSeedMul + draws so far
  int64_t memo_mean, memo_sd;  // sample_arrivals' last mean and its sd (memo_mean -1: none yet)
};

// Advances the queue over [t0_ms, t1_ms): random arrivals, then fluid service by the ready pods
// (and by pending pods from the moment they become ready), accumulating the metrics with the
// backlog and replicas at the start of the interval (left Riemann sum, as policy_sim.h).
template <class A, class T>
KSA_HD void advance(QueueState<A>* s, QueueResult* r, const QueueModel& m, const T* t_ms, const T* rate_milli,
                    int32_t n, RateCursor<A, T>* cur, typename A::Ms t0_ms, typename A::Ms t1_ms,
                    int32_t replicas) {
  using Ms = typename A::Ms;
  if (t1_ms <= t0_ms) return;
  const Ms dt = t1_ms - t0_ms;
  const int64_t q0 = s->q_msgs;
  r->pod_ms = A::add(r->pod_ms, A::count_ms(replicas, dt));
  r->backlog_msg_ms = A::add(r->backlog_msg_ms, A::mul(q0, dt));
  if (q0 > m.slo_backlog) r->violation_ms += dt;
  const int64_t mean = expected_arrivals(t_ms, rate_milli, n, cur, t0_ms, t1_ms);
  const int64_t a = sample_arrivals(mean, s->key++, &s->memo_mean, &s->memo_sd);
  s->q_micro = A::add(s->q_micro, a);
  r->arrived = A::add(r->arrived, a);
  // capacity: ready pods for the whole interval, pending ones from their ready time
  int64_t cap;
  if constexpr (A::kExact) {
    // one pod-milliseconds sum times the rate, the pending pods' time chosen by selects: the
    // branch form made the gfx950 compiler copy the service step (its division by 10^6
    // included) into both arms, and a wave whose lanes disagree on `pending` ran both
    const Ms from = s->pending_at_ms > t0_ms ? s->pending_at_ms : t0_ms;
    const Ms late = s->pending > 0 && s->pending_at_ms < t1_ms ? t1_ms - from : 0;
    cap = A::capacity(s->ready, dt, s->pending, late, m.service_milli);
  } else {
    cap = A::pods_rate_ms(s->ready, m.service_milli, dt);
    if (s->pending > 0 && s->pending_at_ms < t1_ms) {
      const Ms from = s->pending_at_ms > t0_ms ? s->pending_at_ms : t0_ms;
      cap = A::add(cap, A::pods_rate_ms(s->pending, m.service_milli, t1_ms - from));
    }
  }
  const int64_t served = s->q_micro < cap ? s->q_micro : cap;
  s->q_micro -= served;
  s->q_msgs = udiv_1e6(s->q_micro);
  r->served = A::add(r->served, served);
  if (s->pending > 0 && s->pending_at_ms <= t1_ms) {
    s->ready += s->pending;
    s->pending = 0;
  }
}

template <class A, class T>
KSA_HD QueueResult simulate_queue(const Params& p, const Latency& lat, const QueueModel& m, const T* t_ms,
                                  const T* rate_milli, int32_t n, int32_t init_replicas, int64_t horizon_ns,
                                  uint64_t seed) {
  using Ms = typename A::Ms;
  QueueResult res;
  const Rules k = make_rules(p);
  QueueState<A> s;
  // backlog and virtual time never go negative (arrivals and latencies are >= 0; a negative
  // initial backlog is clamped), so the per-poll divisions by 10^6 can be unsigned
  const int64_t init_backlog = m.init_backlog > 0 ? m.init_backlog : 0;
  s.q_micro = init_backlog * 1000000;
  s.q_msgs = init_backlog;
  s.ready = init_replicas;
  s.pending = 0;
  s.pending_at_ms = 0;
  s.key = seed * kSeedMul;
  s.memo_mean = -1;
  s.memo_sd = 0;
  RateCursor<A, T> cur = rate_cursor_init<A>(t_ms, rate_milli, n);
  int64_t now = 0, last_up = 0, last_down = 0;  // main.go:37-38
  int32_t replicas = init_replicas;
  res.max_replicas = replicas;
  Ms prev_ms = 0;
  const Ms horizon_ms = static_cast<Ms>(horizon_ns / 1000000);
  const bool advances = k.period > 0 || lat.sqs_ns > 0;
  // `now` is also kept as whole milliseconds + the nanoseconds past them, advanced by the same
  // increments (the period, the SQS call, each GET and write), each split once here: the poll's
  // millisecond then needs no 64-bit division per poll. Exact: now == now_ms * 10^6 + now_sub.
  // (A period longer than the horizon is never added: the loop ends first. Under FastArith the
  // truncation of such a period's milliseconds to 32 bits is therefore harmless.)
  const Ms period_ms = static_cast<Ms>(udiv_1e6(k.period)), sqs_ms = static_cast<Ms>(udiv_1e6(lat.sqs_ns));
  const Ms get_ms = static_cast<Ms>(udiv_1e6(lat.get_ns)), upd_ms = static_cast<Ms>(udiv_1e6(lat.update_ns));
  const uint32_t period_sub = static_cast<uint32_t>(k.period - static_cast<int64_t>(udiv_1e6(k.period)) * 1000000);
  const uint32_t sqs_sub = static_cast<uint32_t>(lat.sqs_ns - static_cast<int64_t>(sqs_ms) * 1000000);
  const uint32_t get_sub = static_cast<uint32_t>(lat.get_ns - static_cast<int64_t>(get_ms) * 1000000);
  const uint32_t upd_sub = static_cast<uint32_t>(lat.update_ns - static_cast<int64_t>(upd_ms) * 1000000);
  Ms now_ms = 0;
  uint32_t now_sub = 0;
  // adds (ms, sub) with sub < 6 * 10^6 (now_sub, the SQS call's and up to four more latencies'
  // remainders): the sum stays far below 2^32
  auto carry = [&](Ms add_ms, uint32_t add_sub) {
    const uint32_t t = now_sub + add_sub;
    const uint32_t c = t / 1000000u;  // 32-bit division by a constant: a multiply-high
    now_sub = t - c * 1000000u;
    now_ms += add_ms + c;
  };
  while (advances && res.polls < kMaxPolls) {
    const int64_t t_poll = now + k.period;  // main.go:41 sleep, then poll
    if (t_poll > horizon_ns) break;
    carry(period_ms, period_sub);
    const Ms t_poll_ms = now_ms;
    advance(&s, &res, m, t_ms, rate_milli, n, &cur, prev_ms, t_poll_ms, replicas);
    prev_ms = t_poll_ms;
    now = t_poll;
    res.polls++;
    // depth the SQS call reports: every message not yet deleted (queued + in flight)
    const int64_t d = s.q_msgs;
    now += lat.sqs_ns;
    const int32_t before = replicas;
    int32_t gets = 0, writes = 0;
    KSA_DECIDE(k, lat, d, now, last_up, last_down, replicas, gets, writes, res.ups++, (void)0, res.downs++, (void)0);
    carry(sqs_ms + static_cast<Ms>(gets) * get_ms + static_cast<Ms>(writes) * upd_ms,
          sqs_sub + static_cast<uint32_t>(gets) * get_sub + static_cast<uint32_t>(writes) * upd_sub);
    const int32_t delta = sub_i32(replicas, before);
    if (delta > 0) {  // new pods: billed now, draining after the start-up delay
      s.pending += delta;
      const int64_t at = (now + m.startup_ns) / 1000000;
      // under FastArith a ready time past 2^32 ms is past the horizon: clamping changes nothing
      s.pending_at_ms = at < static_cast<int64_t>(A::kNeverMs) ? static_cast<Ms>(at) : A::kNeverMs;
    } else if (delta < 0) {  // the Deployment controller removes not-yet-ready pods first
      int32_t drop = -delta;
      const int32_t from_pending = drop < s.pending ? drop : s.pending;
      s.pending -= from_pending;
      drop -= from_pending;
      s.ready = s.ready > drop ? s.ready - drop : 0;
    }
    if (replicas > res.max_replicas) res.max_replicas = replicas;
    if (s.q_msgs > res.peak_backlog) res.peak_backlog = s.q_msgs;
  }
  if (horizon_ms > prev_ms) advance(&s, &res, m, t_ms, rate_milli, n, &cur, prev_ms, horizon_ms, replicas);
  res.final_replicas = replicas;
  res.final_backlog = s.q_msgs;
  res.arrived /= 1000000;
  res.served /= 1000000;
  return res;
}

// simulate_queue<FastArith> with the decisions on policy_sim.h's 32-bit millisecond clock: for
// sweeps whose periods and latencies are whole milliseconds (ms_clock_ok) every decision time is
// one, so `now`, the cool-down timers and the poll times are int32 milliseconds -- no 64-bit time
// compares and adds, and no carry of the poll's millisecond out of a nanosecond clock. The
// thresholds stay 64-bit (the backlog they compare with is not bounded by 2^31); a new pod's
// ready time is now + floor(startup / 1 ms), which is (now + startup) / 1 ms for a whole-ms now.
// Same values as simulate_queue (tests pin the two equal).
template <class T>
KSA_HD QueueResult simulate_queue_ms(const Params& p, const Latency& lat_ns, const QueueModel& m, const T* t_ms,
                                     const T* rate_milli, int32_t n, int32_t init_replicas, int64_t horizon_ns,
                                     uint64_t seed) {
  using A = FastArith;
  using Ms = A::Ms;
  QueueResult res;
  const MsLatency lat = ms_latency(lat_ns);
  const int32_t horizon_ms = static_cast<int32_t>(horizon_ns / 1000000);
  const MsRulesT<int64_t> k = make_ms_rules<int64_t>(p, horizon_ns, ms_bound(horizon_ms, lat));
  QueueState<A> s;
  const int64_t init_backlog = m.init_backlog > 0 ? m.init_backlog : 0;
  s.q_micro = init_backlog * 1000000;
  s.q_msgs = init_backlog;
  s.ready = init_replicas;
  s.pending = 0;
  s.pending_at_ms = 0;
  s.key = seed * kSeedMul;
  s.memo_mean = -1;
  s.memo_sd = 0;
  RateCursor<A, T> cur = rate_cursor_init<A>(t_ms, rate_milli, n);
  const int64_t startup_ms = udiv_1e6(m.startup_ns);  // >= 0 under fast_path_ok
  int32_t now = 0, last_up = 0, last_down = 0;  // main.go:37-38
  int32_t replicas = init_replicas;
  res.max_replicas = replicas;
  int32_t prev = 0;
  const bool advances = k.period > 0 || lat.sqs_ns > 0;
  while (advances && res.polls < kMaxPolls) {
    const int32_t t_poll = now + k.period;  // main.go:41 sleep, then poll
    if (t_poll > horizon_ms) break;
    advance(&s, &res, m, t_ms, rate_milli, n, &cur, static_cast<Ms>(prev), static_cast<Ms>(t_poll), replicas);
    prev = t_poll;
    now = t_poll;
    res.polls++;
    const int64_t d = s.q_msgs;  // depth the SQS call reports
    now += lat.sqs_ns;
    const int32_t before = replicas;
    int32_t gets = 0, writes = 0;
    KSA_DECIDE(k, lat, d, now, last_up, last_down, replicas, gets, writes, res.ups++, (void)0, res.downs++, (void)0);
    (void)gets;
    (void)writes;
    const int32_t delta = sub_i32(replicas, before);
    if (delta > 0) {  // new pods: billed now, draining after the start-up delay
      s.pending += delta;
      const int64_t at = static_cast<int64_t>(now) + startup_ms;
      s.pending_at_ms = at < static_cast<int64_t>(A::kNeverMs) ? static_cast<Ms>(at) : A::kNeverMs;
    } else if (delta < 0) {  // the Deployment controller removes not-yet-ready pods first
      int32_t drop = -delta;
      const int32_t from_pending = drop < s.pending ? drop : s.pending;
      s.pending -= from_pending;
      drop -= from_pending;
      s.ready = s.ready > drop ? s.ready - drop : 0;
    }
    if (replicas > res.max_replicas) res.max_replicas = replicas;
    if (s.q_msgs > res.peak_backlog) res.peak_backlog = s.q_msgs;
  }
  if (horizon_ms > prev)
    advance(&s, &res, m, t_ms, rate_milli, n, &cur, static_cast<Ms>(prev), static_cast<Ms>(horizon_ms), replicas);
  res.final_replicas = replicas;
  res.final_backlog = s.q_msgs;
  res.arrived /= 1000000;
  res.served /= 1000000;
  return res;
}

// Host check for FastArith: true when, for every configuration and seed, no accumulator,
// backlog or product can reach kSat and no replica count can wrap, so FastArith and SatArith
// compute the same values. Conservative bounds, in double with a factor-2 margin (2^61):
// * replicas stay in [0, R] with R = max(init, max_pods) when init, min/max/up/down pods are
//   non-negative 32-bit values and max + up < 2^31 (no add_i32 wrap);
// * arrivals: each draw is at most mean + 3465 sqrt(mean) (z < 3.4641 x 2^16, sd = 1000 isqrt),
//   so over N <= kMaxPolls + 2 intervals the total is at most E + 3470 sqrt(N E) (Cauchy-Schwarz)
//   with E = max rate x horizon; with the initial backlog this bounds backlog, arrived, served;
// * pod_ms <= R x H, backlog_msg_ms <= backlog_msgs x H, capacity <= R x service x H;
// * every time a lane compares is below the horizon: H < 2^32 - 1 ms.
// Negative or oversized inputs (the hosts' own range checks aside) fall back to SatArith.
inline bool fast_path_ok(const int64_t* t_ms, const int64_t* rate_milli, int32_t n, const QueueModel& m,
                         int32_t init_replicas, int64_t horizon_ns, const int64_t* params, int64_t configs) {
  constexpr double kLimit = 2305843009213693952.0;  // 2^61
  if (n < 1 || init_replicas < 0 || horizon_ns < 0) return false;
  const double H = static_cast<double>(horizon_ns / 1000000);
  if (horizon_ns / 1000000 >= 0xFFFFFFFFLL) return false;
  int64_t rate_max = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (t_ms[i] < 0 || rate_milli[i] < 0 || rate_milli[i] > 0xFFFFFFFFLL) return false;
    if (rate_milli[i] > rate_max) rate_max = rate_milli[i];
  }
  if (m.service_milli < 0 || m.service_milli > 0xFFFFFFFFLL || m.startup_ns < 0) return false;
  int64_t r_max = init_replicas;
  for (int64_t i = 0; i < configs; ++i) {
    // params [9][m]: poll, up_cool, down_cool, up_msgs, down_msgs, up_pods, down_pods, max, min
    const int64_t up = go_i32(params[5 * configs + i]), down = go_i32(params[6 * configs + i]);
    const int64_t mx = go_i32(params[7 * configs + i]), mn = go_i32(params[8 * configs + i]);
    if (up < 0 || down < 0 || mx < 0 || mn < 0 || mx + up >= (int64_t(1) << 31)) return false;
    if (mx > r_max) r_max = mx;
  }
  const double R = static_cast<double>(r_max);
  const double E = static_cast<double>(rate_max) * H;
  const double N = static_cast<double>(kMaxPolls) + 2.0;
  const double init_micro = static_cast<double>(m.init_backlog > 0 ? m.init_backlog : 0) * 1e6;
  const double backlog = init_micro + E + 3470.0 * __builtin_sqrt(N * E);
  if (backlog >= kLimit) return false;
  if ((backlog / 1e6 + 1.0) * H >= kLimit) return false;
  if (R * H >= kLimit) return false;
  if (static_cast<double>(m.service_milli) * H * (R > 1.0 ? R : 1.0) >= kLimit) return false;
  return true;
}

// The trace as FastArith reads it: 32-bit times (clamped to kNeverMs) and rates.
inline void narrow_trace(const int64_t* t_ms, const int64_t* rate_milli, int32_t n, uint32_t* t32, uint32_t* r32) {
  for (int32_t i = 0; i < n; ++i) {
    t32[i] = t_ms[i] < static_cast<int64_t>(FastArith::kNeverMs) ? static_cast<uint32_t>(t_ms[i]) : FastArith::kNeverMs;
    r32[i] = static_cast<uint32_t>(rate_milli[i]);
  }
}

}  // namespace ksa_sim
