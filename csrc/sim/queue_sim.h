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

// floor(sqrt(x)), exact on CPU and GPU: a double-precision estimate (within a unit or two
// whatever the rounding of the conversion and the sqrt) corrected with integer arithmetic. (An
// integer Newton iteration is exact too, but each step is a 64-bit division -- a long software
// sequence on the GPU.)
KSA_HD uint64_t isqrt64(uint64_t x) {
  constexpr uint64_t kMax = 0xFFFFFFFFULL;  // floor(sqrt(2^64 - 1))
  uint64_t r = static_cast<uint64_t>(__builtin_sqrt(static_cast<double>(x)));
  if (r > kMax) r = kMax;
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
// Messages (micro-messages) a rate of x_milli milli-msgs/s delivers in dt_ms: the product,
// saturating.
KSA_HD int64_t per_ms(int64_t x_milli, int64_t dt_ms) { return sat_mul(x_milli, dt_ms); }

// Random arrivals (micro-messages) with mean `mean`: mean + sqrt(mean) * Z. Z is the sum of the
// four 16-bit fields of one splitmix64 draw (Irwin-Hall, n = 4: mean 131070, standard deviation
// 65536/sqrt(3)), centred and scaled by sqrt(3) to a standard deviation of 2^16 in fixed point;
// |Z| < 3.47. Round 2 drew twelve fields from three hashes (the CLT of 12): on gfx950 the three
// 64-bit hashes and their field sums were a third of the VALU work of a simulated poll, and four
// fields already give a normal approximation far finer than the Poisson noise it stands for.
// sqrt(mean) is kept for the last mean (*memo_mean, *memo_sd): polls of one interval length inside
// one rate segment -- most of them -- ask for the same mean, and the isqrt is the longest sequence
// of the poll on the GPU.
constexpr int64_t kSqrt3Q16 = 113512;  // round(sqrt(3) * 2^16)
KSA_HD int64_t sample_arrivals(int64_t mean, uint64_t seed, uint64_t k, int64_t* memo_mean, int64_t* memo_sd) {
  if (mean <= 0) return 0;
  const uint64_t w = mix64(seed * 0xD1B54A32D192ED03ULL + k);
  // the four 16-bit fields, summed in two 32-bit lanes (2 x 65535 fits), then folded
  constexpr uint64_t kM = 0x0000FFFF0000FFFFULL;
  const uint64_t lanes = (w & kM) + ((w >> 16) & kM);
  const int64_t u = static_cast<int64_t>((lanes & 0xFFFFFFFFULL) + (lanes >> 32)) - 131070;  // 2 x centred
  const int64_t z = (u * kSqrt3Q16) >> 16;  // arithmetic shift: floor, as Python's >>
  // sd in micro-messages = sqrt(mean / 1e6) * 1e6 = 1000 sqrt(mean), to a milli-message
  if (mean != *memo_mean) {
    *memo_mean = mean;
    *memo_sd = static_cast<int64_t>(isqrt64(static_cast<uint64_t>(mean))) * 1000;
  }
  const int64_t sd = *memo_sd;
  const int64_t a = mean + sd * z / 65536;
  return a > 0 ? a : 0;
}

// Forward-only cursor over the arrival-rate trace, as policy_sim.h's Cursor: the current rate
// and the next boundary and rate live in registers, and advancing issues the loads for the
// segment after that at once. An interval inside one segment (a 5 s poll in a 60 s segment)
// then makes no memory access; before, every poll made 3-4 dependent trace loads.
struct RateCursor {
  int32_t c;
  int64_t rate, next_t, next_rate;  // rate_milli[c]; t_ms[c+1] (kNever past the last); rate_milli[c+1]
};

KSA_HD RateCursor rate_cursor_init(const int64_t* t_ms, const int64_t* rate_milli, int32_t n) {
  RateCursor k;
  k.c = 0;
  k.rate = rate_milli[0];
  k.next_t = n > 1 ? t_ms[1] : kNever;
  k.next_rate = n > 1 ? rate_milli[1] : 0;
  return k;
}

KSA_HD void rate_cursor_advance(const int64_t* t_ms, const int64_t* rate_milli, int32_t n, RateCursor* k) {
  k->c++;
  k->rate = k->next_rate;
  if (k->c + 1 < n) {
    k->next_t = t_ms[k->c + 1];
    k->next_rate = rate_milli[k->c + 1];
  } else {
    k->next_t = kNever;
  }
}

// Expected arrivals (micro-messages) over [t0_ms, t1_ms): the rate integrated segment by
// segment. Segment i covers [t_ms[i], t_ms[i+1]); the last one extends to infinity. Times only
// grow (each call starts where the last ended), so the cursor never moves back and is left on
// the segment holding t1_ms.
KSA_HD int64_t expected_arrivals(const int64_t* t_ms, const int64_t* rate_milli, int32_t n, RateCursor* k,
                                       int64_t t0_ms, int64_t t1_ms) {
  while (t0_ms >= k->next_t) rate_cursor_advance(t_ms, rate_milli, n, k);
  int64_t sum = 0, a = t0_ms;
  while (a < t1_ms) {
    const int64_t b = k->next_t < t1_ms ? k->next_t : t1_ms;
    sum = sat_add(sum, per_ms(k->rate, b - a));
    a = b;
    if (a >= k->next_t) rate_cursor_advance(t_ms, rate_milli, n, k);
  }
  return sum;
}

struct QueueState {
  int64_t q_micro;       // backlog
  int64_t q_msgs;        // q_micro / 1e6, kept current (the depth SQS reports)
  int32_t ready, pending;
  int64_t pending_at_ms;  // when the pending pods start draining
  uint64_t draws;
  int64_t memo_mean, memo_sd;  // sample_arrivals' last mean and its sd (memo_mean -1: none yet)
};

// Advances the queue over [t0_ms, t1_ms): random arrivals, then fluid service by the ready pods
// (and by pending pods from the moment they become ready), accumulating the metrics with the
// backlog and replicas at the start of the interval (left Riemann sum, as policy_sim.h).
KSA_HD void advance(QueueState* s, QueueResult* r, const QueueModel& m, const int64_t* t_ms,
                    const int64_t* rate_milli, int32_t n, RateCursor* cur, uint64_t seed, int64_t t0_ms, int64_t t1_ms,
                    int32_t replicas) {
  if (t1_ms <= t0_ms) return;
  const int64_t dt = t1_ms - t0_ms;
  const int64_t q0 = s->q_msgs;
  r->pod_ms = sat_add(r->pod_ms, sat_mul(replicas, dt));
  r->backlog_msg_ms = sat_add(r->backlog_msg_ms, sat_mul(q0, dt));
  if (q0 > m.slo_backlog) r->violation_ms += dt;
  const int64_t mean = expected_arrivals(t_ms, rate_milli, n, cur, t0_ms, t1_ms);
  const int64_t a = sample_arrivals(mean, seed, s->draws++, &s->memo_mean, &s->memo_sd);
  s->q_micro = sat_add(s->q_micro, a);
  r->arrived = sat_add(r->arrived, a);
  // capacity: ready pods for the whole interval, pending ones from their ready time
  int64_t cap = sat_mul(s->ready, per_ms(m.service_milli, dt));
  if (s->pending > 0 && s->pending_at_ms < t1_ms) {
    const int64_t from = s->pending_at_ms > t0_ms ? s->pending_at_ms : t0_ms;
    cap = sat_add(cap, sat_mul(s->pending, per_ms(m.service_milli, t1_ms - from)));
  }
  const int64_t served = s->q_micro < cap ? s->q_micro : cap;
  s->q_micro -= served;
  s->q_msgs = udiv_1e6(s->q_micro);
  r->served = sat_add(r->served, served);
  if (s->pending > 0 && s->pending_at_ms <= t1_ms) {
    s->ready += s->pending;
    s->pending = 0;
  }
}

KSA_HD QueueResult simulate_queue(const Params& p, const Latency& lat, const QueueModel& m, const int64_t* t_ms,
                                  const int64_t* rate_milli, int32_t n, int32_t init_replicas, int64_t horizon_ns,
                                  uint64_t seed) {
  QueueResult res;
  const Rules k = make_rules(p);
  QueueState s;
  // backlog and virtual time never go negative (arrivals and latencies are >= 0; a negative
  // initial backlog is clamped), so the per-poll divisions by 10^6 can be unsigned
  const int64_t init_backlog = m.init_backlog > 0 ? m.init_backlog : 0;
  s.q_micro = init_backlog * 1000000;
  s.q_msgs = init_backlog;
  s.ready = init_replicas;
  s.pending = 0;
  s.pending_at_ms = 0;
  s.draws = 0;
  s.memo_mean = -1;
  s.memo_sd = 0;
  RateCursor cur = rate_cursor_init(t_ms, rate_milli, n);
  int64_t now = 0, last_up = 0, last_down = 0;  // main.go:37-38
  int32_t replicas = init_replicas;
  res.max_replicas = replicas;
  int64_t prev_ms = 0;
  const int64_t horizon_ms = horizon_ns / 1000000;
  const bool advances = k.period > 0 || lat.sqs_ns > 0;
  // `now` is also kept as whole milliseconds + the nanoseconds past them, advanced by the same
  // increments (the period, the SQS call, each GET and write), each split once here: the poll's
  // millisecond then needs no 64-bit division per poll. Exact: now == now_ms * 10^6 + now_sub.
  const int64_t period_ms = udiv_1e6(k.period), sqs_ms = udiv_1e6(lat.sqs_ns);
  const int64_t get_ms = udiv_1e6(lat.get_ns), upd_ms = udiv_1e6(lat.update_ns);
  const uint32_t period_sub = static_cast<uint32_t>(k.period - period_ms * 1000000);
  const uint32_t sqs_sub = static_cast<uint32_t>(lat.sqs_ns - sqs_ms * 1000000);
  const uint32_t get_sub = static_cast<uint32_t>(lat.get_ns - get_ms * 1000000);
  const uint32_t upd_sub = static_cast<uint32_t>(lat.update_ns - upd_ms * 1000000);
  int64_t now_ms = 0;
  uint32_t now_sub = 0;
  // adds (ms, sub) with sub < 6 * 10^6 (now_sub, the SQS call's and up to four more latencies'
  // remainders): the sum stays far below 2^32
  auto carry = [&](int64_t add_ms, uint32_t add_sub) {
    const uint32_t t = now_sub + add_sub;
    const uint32_t c = t / 1000000u;  // 32-bit division by a constant: a multiply-high
    now_sub = t - c * 1000000u;
    now_ms += add_ms + c;
  };
  while (advances && res.polls < kMaxPolls) {
    const int64_t t_poll = now + k.period;  // main.go:41 sleep, then poll
    if (t_poll > horizon_ns) break;
    carry(period_ms, period_sub);
    const int64_t t_poll_ms = now_ms;
    advance(&s, &res, m, t_ms, rate_milli, n, &cur, seed, prev_ms, t_poll_ms, replicas);
    prev_ms = t_poll_ms;
    now = t_poll;
    res.polls++;
    // depth the SQS call reports: every message not yet deleted (queued + in flight)
    const int64_t d = s.q_msgs;
    now += lat.sqs_ns;
    const int32_t before = replicas;
    int32_t gets = 0, writes = 0;
    KSA_DECIDE(k, lat, d, now, last_up, last_down, replicas, gets, writes, res.ups++, (void)0, res.downs++, (void)0);
    carry(sqs_ms + gets * get_ms + writes * upd_ms,
          sqs_sub + static_cast<uint32_t>(gets) * get_sub + static_cast<uint32_t>(writes) * upd_sub);
    const int32_t delta = sub_i32(replicas, before);
    if (delta > 0) {  // new pods: billed now, draining after the start-up delay
      s.pending += delta;
      s.pending_at_ms = (now + m.startup_ns) / 1000000;
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
  if (horizon_ms > prev_ms) advance(&s, &res, m, t_ms, rate_milli, n, &cur, seed, prev_ms, horizon_ms, replicas);
  res.final_replicas = replicas;
  res.final_backlog = s.q_msgs;
  res.arrived /= 1000000;
  res.served /= 1000000;
  return res;
}

}  // namespace ksa_sim
