#include "runner.h"

#include <pthread.h>
#include <sched.h>
#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <cmath>
#include <limits>
#include <new>

#include "json.h"

namespace ksa {

const char* action_name(Action a) {
  switch (a) {
    case Action::None: return "none";
    case Action::CoolDown: return "cooldown";
    case Action::Scaled: return "scaled";
    case Action::NoopAtBound: return "noop";
    case Action::Failed: return "failed";
  }
  return "?";
}

namespace {

// last + cool with saturation (Go's Time.Add drops the monotonic reading on overflow; a
// saturated sum preserves the comparison outcome).
Nanos sat_add(Nanos a, Nanos b) {
  if (b > 0 && a > std::numeric_limits<Nanos>::max() - b) return std::numeric_limits<Nanos>::max();
  if (b < 0 && a < std::numeric_limits<Nanos>::min() - b) return std::numeric_limits<Nanos>::min();
  return a + b;
}

}  // namespace

Runner::Runner(LoopConfig cfg, std::shared_ptr<SqsClient> sqs, std::shared_ptr<PodAutoScaler> scaler,
               std::shared_ptr<Clock> clock, std::shared_ptr<Logger> log)
    : cfg_(cfg),
      sqs_(std::move(sqs)),
      scaler_(std::move(scaler)),
      clock_(std::move(clock)),
      log_(std::move(log)) {
  lat_ring_.reserve(1024);
  progress_ns_.store(clock_->now(), std::memory_order_release);
}

void Runner::arm() {
  last_up_ = clock_->now();
  last_down_ = clock_->now();
  progress_ns_.store(clock_->now(), std::memory_order_release);
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.last_good_ns = clock_->now();  // a failing streak is timed from Run() entry at the earliest
  }
  if (shared_) shared_->last_good_ns.store(clock_->now(), std::memory_order_relaxed);
}

// Would this poll call ScaleUp/ScaleDown if the queue depth were still the last one read?
// Evaluated at t0 + the last SQS round trip, which is when the gates of main.go:51-77 will run.
// An exact replay of those gates on the previous depth: a depth at or above the up threshold
// either passes the up cool-down (-> a GET) or `continue`s past the down check (main.go:54);
// a depth in the dead band reads nothing. Before the first depth read either open cool-down
// counts. A wrong guess costs nothing in decisions: an unsent prefetch means the reference's
// own synchronous GET after the SQS response, an unused one is drained.
bool Runner::action_likely(Nanos t0) const {
  const Nanos at = t0 + last_depth_rtt_;
  const bool up_open = sat_add(last_up_, cfg_.scale_up_cool_down) <= at;
  const bool down_open = sat_add(last_down_, cfg_.scale_down_cool_down) <= at;
  if (!have_depth_) return up_open || down_open;
  if (last_depth_ >= cfg_.scale_up_messages) return up_open;
  if (last_depth_ <= cfg_.scale_down_messages) return down_open;
  return false;
}

IterationRecord Runner::step(StopFlag* stop) {
  cpu_from_ = thread_cpu_ns();
  // main.go:41 -- sleep BEFORE the poll.
  const Nanos period = cfg_.poll_period, w = cfg_.prewarm;
  bool slept;
  if (w > 0 && period > 2 * w) {
    const Nanos due = clock_->now() + period;
    slept = clock_->sleep(period - w, stop);
    if (slept) {
      warm(due, true);
      // Then sleep out the lead -- or spin its end, within the warm-up's share of the poll's spin
      // budget (0 unless --busy-poll-budget), for a near SQS endpoint (an answer within
      // HttpClient::kMaxSpinThrough, or none measured yet), whose poll is short enough for an
      // awake core with warm caches to show. Against a remote endpoint (milliseconds) that saving
      // is noise while the spin would be most of the poll's CPU.
      const Nanos ewma = sqs_->api()->response_ewma();
      const Nanos rest = due - clock_->now();
      Nanos spin = cfg_.prewarm_spin && ewma <= HttpClient::kMaxSpinThrough ? rest : 0;
      if (prewarm_spin_budget_ >= 0) spin = std::min(spin, prewarm_spin_budget_);
      slept = clock_->sleep(rest - spin, stop) && clock_->spin_until(due, stop);
    }
  } else {
    slept = clock_->sleep(period, stop);
    // a period too short to wake early in: the same preparation, at the due time (cheap on
    // connections used within the last few milliseconds, which at such a period they were)
    if (slept && w > 0) warm(clock_->now());
  }
  if (!slept) {
    cpu_from_ = -1;  // no poll to charge it to
    IterationRecord rec;
    rec.stopped = true;
    return rec;
  }
  return poll_once();
}

void Runner::warm(Nanos due, bool presend) {
  sqs_->warm(clock_->unix_nanos() + (due - clock_->now()), presend && cfg_.presend && cfg_.prewarm <= kMaxPresendLead);
  // the Deployment read and write only follow on polls the gates may let through (or every
  // poll, with a GET sent on every poll)
  if ((cfg_.prefetch && cfg_.prefetch_always) || action_likely(due)) scaler_->warm();
  log_flush_pending();  // nothing held back past the due time
}

IterationRecord Runner::poll_once() {
  if (cpu_from_ < 0) cpu_from_ = thread_cpu_ns();  // pooled: the poll alone
  LogBatch batch;  // the poll's log lines go out together once it is done (log.h)
  return poll_body();
}

IterationRecord Runner::poll_body() {
  if (shared_) {  // the supervising process' GPU-capacity cap
    const int64_t cap = shared_->max_override.load(std::memory_order_relaxed);
    if (cap > 0 && cap != scaler_->max()) scaler_->set_max(cap);
  }
  IterationRecord rec;
  rec.index = ++index_;
  const Nanos t0 = clock_->now();
  rec.t_poll = t0;
  // Pipelined read: the Deployment GET overlaps the SQS call -- only when this poll is likely to
  // reach the apiserver at all (the reference reads the Deployment only past the threshold and
  // cool-down gates, main.go:51-77). Over HTTP the GET is sent as soon as the SQS request is on the wire (set_on_wire): sending
  // it first would put its write (the loopback/TCP send path, ~2 µs) ahead of the SQS request on
  // the critical path, while the GET's own round trip is shorter than the SQS call it overlaps.
  // If the SQS write fails before that point, the GET goes out after the call (when it
  // succeeded on a retry). In-memory clients (tests, the parity harness) get it first, as
  // the virtual-time model of the overlap expects.
  // From the on-wire hook the GET must not dial: that would run on the SQS call's deadline, so
  // an unreachable apiserver would fail the SQS read. Without a ready connection the poll does
  // the reference's synchronous GET after the SQS answer instead.
  struct Prefetch {
    Runner* self;
    IterationRecord* rec;
    bool may_dial;
    static void send(void* p) {
      auto* f = static_cast<Prefetch*>(p);
      f->rec->prefetched = f->self->scaler_->prefetch(f->may_dial);
      if (f->rec->prefetched) f->rec->gets++;
    }
  } pf{this, &rec, false};
  bool on_wire = false;
  if (cfg_.prefetch) {
    if (cfg_.prefetch_always || action_likely(t0)) {
      if (sqs_->api()->runs_on_wire_work()) {
        on_wire = true;
        set_on_wire(&Prefetch::send, &pf);
      } else {
        pf.may_dial = true;
        Prefetch::send(&pf);
      }
    } else {
      rec.prefetch_gated = true;
    }
  }

  // main.go:43-47
  auto depth = sqs_->num_messages();
  Nanos t1 = clock_->now();
  if (on_wire && on_wire_pending()) {
    clear_on_wire();
    pf.may_dial = true;  // outside the SQS call now
    if (depth.ok()) Prefetch::send(&pf);  // the SQS request never reached the wire first
  }
  rec.depth_ns = t1 - t0;
  last_depth_rtt_ = rec.depth_ns;
  if (!depth.ok()) {
    rec.error = depth.status.message();
    log_->error("Failed to get SQS messages: " + depth.status.message());
    scaler_->discard_prefetch();
    rec.total_ns = clock_->now() - t0;
    record(rec);
    return rec;
  }
  const int64_t n = depth.value;
  rec.depth_ok = true;
  rec.depth = n;
  have_depth_ = true;
  last_depth_ = n;
  log_->info("Found " + std::to_string(n) + " messages in the queue");  // main.go:49

  auto finish = [&]() -> IterationRecord& {
    scaler_->discard_prefetch();  // unused (no action this poll): drain it
    rec.total_ns = clock_->now() - t0;
    if (kHttpTiming && trace_fd_ >= 0) {  // per-call breakdowns of timed clients (bench attribution rows)
      const std::string sq = sqs_->api()->timing_json();
      const std::string wr = rec.patch_latency_ns >= 0 ? scaler_->api()->timing_json() : std::string();
      if (!sq.empty() || !wr.empty())
        rec.detail = "{\"sqs\":" + (sq.empty() ? std::string("null") : sq) +
                     ",\"write\":" + (wr.empty() ? std::string("null") : wr) + "}";
    }
    record(rec);
    return rec;
  };

  // main.go:51-63
  if (n >= cfg_.scale_up_messages) {
    if (sat_add(last_up_, cfg_.scale_up_cool_down) > clock_->now()) {
      log_->info("Waiting for cool down, skipping scale up ");  // trailing space: main.go:53
      rec.up = Action::CoolDown;
      return finish();
    }
    ScaleSpan span;
    Status s = scaler_->scale_up(&span);
    rec.get_ns += span.get_ns;
    rec.update_ns += span.update_ns;
    rec.prefetch_used |= span.used_prefetch;
    rec.gets += span.gets;
    if (span.read) {
      rec.replicas_before = span.before;
      rec.replicas_after = span.after;
    }
    if (!s.ok()) {
      rec.error = s.message();
      log_->error("Failed scaling up: " + s.message());
      rec.up = Action::Failed;
      return finish();
    }
    last_up_ = clock_->now();  // main.go:62 -- also after a no-op at max
    rec.up = span.wrote ? Action::Scaled : Action::NoopAtBound;
    if (span.wrote) rec.patch_latency_ns = clock_->now() - t0;
  }

  // main.go:65-77
  if (n <= cfg_.scale_down_messages) {
    if (sat_add(last_down_, cfg_.scale_down_cool_down) > clock_->now()) {
      log_->info("Waiting for cool down, skipping scale down");
      rec.down = Action::CoolDown;
      return finish();
    }
    ScaleSpan span;
    Status s = scaler_->scale_down(&span);
    rec.get_ns += span.get_ns;
    rec.update_ns += span.update_ns;
    rec.prefetch_used |= span.used_prefetch;
    rec.gets += span.gets;
    if (span.read) {
      if (rec.replicas_before < 0) rec.replicas_before = span.before;
      rec.replicas_after = span.after;
    }
    if (!s.ok()) {
      rec.error = s.message();
      log_->error("Failed scaling down: " + s.message());
      rec.down = Action::Failed;
      return finish();
    }
    last_down_ = clock_->now();  // main.go:76
    rec.down = span.wrote ? Action::Scaled : Action::NoopAtBound;
    if (span.wrote) rec.patch_latency_ns = clock_->now() - t0;
  }
  return finish();
}

void Runner::record(IterationRecord& r) {
  if (cpu_from_ >= 0) {
    r.cpu_ns = thread_cpu_ns() - cpu_from_;
    cpu_from_ = -1;
  }
  const Nanos now = clock_->now();
  progress_ns_.store(now, std::memory_order_release);
  const bool good = r.depth_ok && r.up != Action::Failed && r.down != Action::Failed;
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.polls++;
    if (r.cpu_ns > 0) stats_.poll_cpu_ns += r.cpu_ns;
    if (good) {
      stats_.consecutive_failed_polls = 0;
      stats_.last_good_ns = now;
    } else {
      stats_.consecutive_failed_polls++;
      last_error_ = r.error;
    }
    if (r.prefetched) stats_.speculative_reads++;
    if (r.prefetch_used) stats_.speculative_reads_used++;
    if (r.prefetch_gated) stats_.speculative_reads_gated++;
    stats_.apiserver_reads += static_cast<uint64_t>(r.gets);
    if (!r.depth_ok) stats_.depth_errors++;
    else stats_.last_depth = r.depth;
    switch (r.up) {
      case Action::Scaled: stats_.scale_ups++; break;
      case Action::NoopAtBound: stats_.noop_ups++; break;
      case Action::CoolDown: stats_.cooldown_skips_up++; break;
      case Action::Failed: stats_.failed_ups++; break;
      default: break;
    }
    switch (r.down) {
      case Action::Scaled: stats_.scale_downs++; break;
      case Action::NoopAtBound: stats_.noop_downs++; break;
      case Action::CoolDown: stats_.cooldown_skips_down++; break;
      case Action::Failed: stats_.failed_downs++; break;
      default: break;
    }
    if (r.replicas_after >= 0) stats_.last_replicas = r.replicas_after;
    if (r.patch_latency_ns >= 0) {
      stats_.latency_samples++;
      stats_.latency_sum_ns += r.patch_latency_ns;
      stats_.latency_buckets[latency_bucket(r.patch_latency_ns)]++;
      if (lat_ring_.size() < kLatRing) {
        lat_ring_.push_back(r.patch_latency_ns);
      } else {
        lat_ring_[lat_pos_] = r.patch_latency_ns;
        lat_pos_ = (lat_pos_ + 1) % kLatRing;
      }
    }
  }
  if (shared_) mirror(r);
  if (trace_fd_ >= 0) write_trace(r);
  if (observer_) observer_(r);
}

SharedWorkerState* init_shared_worker_state(void* at) {
  auto* s = new (at) SharedWorkerState;
  for (auto& c : s->counters) c.store(0, std::memory_order_relaxed);
  s->progress_ns.store(0, std::memory_order_relaxed);
  s->last_good_ns.store(0, std::memory_order_relaxed);
  s->last_depth.store(0, std::memory_order_relaxed);
  s->last_replicas.store(-1, std::memory_order_relaxed);
  s->lat_sum_ns.store(0, std::memory_order_relaxed);
  s->status.store(SharedWorkerState::kStarting, std::memory_order_relaxed);
  s->max_override.store(0, std::memory_order_relaxed);
  s->iterations.store(-1, std::memory_order_relaxed);
  s->control.store(SharedWorkerState::kWait, std::memory_order_relaxed);
  for (auto& v : s->lat_hist) v.store(0, std::memory_order_relaxed);
  for (auto& v : s->lat_ring) v.store(0, std::memory_order_relaxed);
  s->error_seq.store(0, std::memory_order_relaxed);
  s->error_len.store(0, std::memory_order_relaxed);
  for (auto& v : s->error_words) v.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  return s;
}

void write_shared_error(SharedWorkerState* s, const std::string& text) {
  size_t n = std::min(text.size(), SharedWorkerState::kErrorBytes - 1);
  if (n < text.size())  // cut at a UTF-8 character boundary
    while (n > 0 && (static_cast<unsigned char>(text[n]) & 0xC0) == 0x80) --n;
  const uint64_t seq = s->error_seq.load(std::memory_order_relaxed);
  s->error_seq.store(seq + 1, std::memory_order_relaxed);  // odd: being written
  std::atomic_thread_fence(std::memory_order_release);
  for (size_t w = 0; w * 8 < n; ++w) {
    uint64_t word = 0;
    std::memcpy(&word, text.data() + w * 8, std::min<size_t>(8, n - w * 8));
    s->error_words[w].store(word, std::memory_order_relaxed);
  }
  s->error_len.store(static_cast<uint32_t>(n), std::memory_order_relaxed);
  s->error_seq.store(seq + 2, std::memory_order_release);
}

std::string read_shared_error(const SharedWorkerState* s) {
  for (int attempt = 0; attempt < 64; ++attempt) {
    const uint64_t before = s->error_seq.load(std::memory_order_acquire);
    if (before & 1) continue;  // the worker is mid-write
    const size_t n = std::min<size_t>(s->error_len.load(std::memory_order_relaxed), SharedWorkerState::kErrorBytes - 1);
    std::string out(n, '\0');
    for (size_t w = 0; w * 8 < n; ++w) {
      const uint64_t word = s->error_words[w].load(std::memory_order_relaxed);
      std::memcpy(&out[w * 8], &word, std::min<size_t>(8, n - w * 8));
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (s->error_seq.load(std::memory_order_relaxed) == before) return out;
  }
  return "";
}

void Runner::mirror(const IterationRecord& r) {
  RunnerStats st;
  {
    std::lock_guard<std::mutex> lk(mu_);
    st = stats_;
  }
  const bool good = r.depth_ok && r.up != Action::Failed && r.down != Action::Failed;
  if (!good) write_shared_error(shared_, r.error);  // before the failure counters /readyz reads
  using W = SharedWorkerState;
  auto put = [&](int i, uint64_t v) { shared_->counters[i].store(v, std::memory_order_relaxed); };
  put(W::kPolls, st.polls);
  put(W::kDepthErrors, st.depth_errors);
  put(W::kScaleUps, st.scale_ups);
  put(W::kScaleDowns, st.scale_downs);
  put(W::kNoopUps, st.noop_ups);
  put(W::kNoopDowns, st.noop_downs);
  put(W::kCooldownSkipsUp, st.cooldown_skips_up);
  put(W::kCooldownSkipsDown, st.cooldown_skips_down);
  put(W::kFailedUps, st.failed_ups);
  put(W::kFailedDowns, st.failed_downs);
  put(W::kSpeculativeReads, st.speculative_reads);
  put(W::kSpeculativeReadsUsed, st.speculative_reads_used);
  put(W::kSpeculativeReadsGated, st.speculative_reads_gated);
  put(W::kApiserverReads, st.apiserver_reads);
  put(W::kConsecutiveFailedPolls, st.consecutive_failed_polls);
  put(W::kPollCpuNs, static_cast<uint64_t>(st.poll_cpu_ns));
  shared_->last_good_ns.store(st.last_good_ns, std::memory_order_relaxed);
  shared_->last_depth.store(st.last_depth, std::memory_order_relaxed);
  shared_->last_replicas.store(st.last_replicas, std::memory_order_relaxed);
  if (r.patch_latency_ns >= 0) {
    const uint64_t n = st.latency_samples;  // this sample is number n (1-based)
    shared_->lat_ring[(n - 1) % SharedWorkerState::kRing].store(r.patch_latency_ns, std::memory_order_relaxed);
    shared_->lat_sum_ns.store(st.latency_sum_ns, std::memory_order_relaxed);
    const int b = latency_bucket(r.patch_latency_ns);
    shared_->lat_hist[b].store(st.latency_buckets[b], std::memory_order_relaxed);
  }
  // the count last, with release: a reader that sees it sees the ring entries before it
  shared_->counters[W::kLatencySamples].store(st.latency_samples, std::memory_order_release);
}

std::string iteration_json(const IterationRecord& r, int64_t unix_ns, const std::string& queue,
                           const std::string& deployment) {
  std::string j = "{\"ts\":" + std::to_string(unix_ns) + ",\"queue\":" + json_quote(queue) +
                  ",\"deployment\":" + json_quote(deployment) + ",\"poll\":" + std::to_string(r.index) +
                  ",\"depth\":" + (r.depth_ok ? std::to_string(r.depth) : std::string("null")) +
                  ",\"up\":\"" + action_name(r.up) + "\",\"down\":\"" + action_name(r.down) +
                  "\",\"replicas_before\":" + std::to_string(r.replicas_before) +
                  ",\"replicas_after\":" + std::to_string(r.replicas_after) +
                  ",\"prefetched\":" + (r.prefetched ? "true" : "false") +
                  ",\"prefetch_used\":" + (r.prefetch_used ? "true" : "false") +
                  ",\"gets\":" + std::to_string(r.gets) +
                  ",\"depth_ns\":" + std::to_string(r.depth_ns) + ",\"get_ns\":" + std::to_string(r.get_ns) +
                  ",\"update_ns\":" + std::to_string(r.update_ns) + ",\"total_ns\":" + std::to_string(r.total_ns) +
                  ",\"patch_latency_ns\":" + std::to_string(r.patch_latency_ns) +
                  ",\"cpu_ns\":" + std::to_string(r.cpu_ns);
  if (!r.error.empty()) j += ",\"error\":" + json_quote(r.error);
  if (!r.detail.empty()) j += ",\"detail\":" + r.detail;
  j += "}";
  return j;
}

void Runner::write_trace(const IterationRecord& r) {
  std::string line = iteration_json(r, clock_->unix_nanos(), sqs_->queue_url(),
                                    scaler_->namespace_() + "/" + scaler_->deployment());
  line.push_back('\n');
  ssize_t n = ::write(trace_fd_, line.data(), line.size());
  (void)n;
}

Nanos Runner::spin_budget_for(const LoopConfig& cfg, const CpuQuota& quota) {
  const int64_t ppm = std::clamp<int64_t>(cfg.spin_budget_ppm, 0, 1000000);
  Nanos b = std::max<Nanos>(cfg.poll_period, 0) / 1000000 * ppm;
  // Under a CFS limit a poll spins at most a tenth of the quota of one CFS period (this queue's
  // share of it, as a 1 % budget split over the queues): 1 ms per poll under a 100m limit.
  if (quota.limited()) b = std::min<Nanos>(b, quota.quota_ns / 10 * std::min<int64_t>(ppm, 10000) / 10000);
  return b;
}

void Runner::run(StopFlag* stop, int64_t max_iterations, Nanos start_delay) {
  // This thread is the worker's own: it may spin before the due time and through a near
  // endpoint's answer within a share of the poll period (LoopConfig::spin_budget_ppm; a
  // back-to-back loop keeps the window), capped by the process's CPU limit.
  static const CpuQuota quota = read_cpu_quota();  // once per process
  set_spin_budget(spin_budget_for(cfg_, quota));
  if (start_delay > 0 && !clock_->sleep(start_delay, stop)) return;
  if (cfg_.connect_at_start) {
    sqs_->warm(clock_->unix_nanos());
    if (cfg_.prefetch) scaler_->warm();
  }
  arm();
  int64_t done = 0;
  while (!(stop && stop->stopped())) {
    if (max_iterations > 0 && done >= max_iterations) break;
    IterationRecord r = step(stop);
    if (r.stopped) break;
    ++done;
  }
}

Nanos Runner::idle_ns() const {
  const Nanos now = clock_->now();
  Nanos last = progress_ns_.load(std::memory_order_acquire);
  const Nanos waits = std::max(sqs_->api()->waiting_until(), scaler_->api()->waiting_until());
  last = std::max(last, std::min(waits, now));
  return now - last;
}

Nanos Runner::failing_ns() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (stats_.consecutive_failed_polls == 0) return 0;
  return std::max<Nanos>(clock_->now() - stats_.last_good_ns, 0);
}

std::string Runner::last_error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return last_error_;
}

RunnerStats Runner::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

std::vector<Nanos> Runner::latencies() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (lat_ring_.size() < kLatRing) return lat_ring_;
  std::vector<Nanos> out;
  out.reserve(kLatRing);
  out.insert(out.end(), lat_ring_.begin() + static_cast<long>(lat_pos_), lat_ring_.end());
  out.insert(out.end(), lat_ring_.begin(), lat_ring_.begin() + static_cast<long>(lat_pos_));
  return out;
}

void Runner::clear_latencies() {
  std::lock_guard<std::mutex> lk(mu_);
  lat_ring_.clear();
  lat_pos_ = 0;
}

// ---------------------------------------------------------------------------------------

bool read_thread_sched(ThreadSched* out) {
  *out = ThreadSched();
  FILE* f = std::fopen("/proc/thread-self/schedstat", "r");
  if (!f) return false;
  long long cpu = 0, wait = 0, slices = 0;
  const int n = std::fscanf(f, "%lld %lld %lld", &cpu, &wait, &slices);
  std::fclose(f);
  if (n != 3) return false;
  out->threads = 1;
  struct rusage ru;
  if (getrusage(RUSAGE_THREAD, &ru) == 0) {
    out->utime_ns = static_cast<int64_t>(ru.ru_utime.tv_sec) * 1000000000LL + ru.ru_utime.tv_usec * 1000LL;
    out->stime_ns = static_cast<int64_t>(ru.ru_stime.tv_sec) * 1000000000LL + ru.ru_stime.tv_usec * 1000LL;
    out->minflt = ru.ru_minflt;
  }
  out->cpu_ns = cpu;
  out->runq_wait_ns = wait;
  out->slices = slices;
  f = std::fopen("/proc/thread-self/status", "r");
  if (f) {
    char line[256];
    while (std::fgets(line, sizeof line, f)) {
      long long v = 0;
      if (std::sscanf(line, "voluntary_ctxt_switches: %lld", &v) == 1) out->vol_cs = v;
      else if (std::sscanf(line, "nonvoluntary_ctxt_switches: %lld", &v) == 1) out->invol_cs = v;
    }
    std::fclose(f);
  }
  return true;
}

Supervisor::Supervisor() = default;

HomeThread::HomeThread() {
  thread_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "ksa-worker");  // top -H / /proc/<pid>/task/*/comm
    cpu_set_t set;
    if (pthread_getaffinity_np(pthread_self(), sizeof set, &set) == 0) {
      std::lock_guard<std::mutex> lk(mu_);
      for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &set)) start_mask_.push_back(c);
    }
    loop();
  });
}

void HomeThread::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return quit_ || task_ != nullptr; });
    if (!task_) return;  // quit with nothing left to run
    std::function<void()> task = std::move(task_);
    task_ = nullptr;
    lk.unlock();
    task();
    task = nullptr;  // the task's captures go before the thread reports idle
    lk.lock();
    busy_ = false;
    cv_.notify_all();
  }
}

void HomeThread::post(std::function<void()> task) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return !busy_; });
  task_ = std::move(task);
  busy_ = true;
  cv_.notify_all();
}

void HomeThread::wait_idle() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return !busy_; });
}

void HomeThread::unpin() {
  CpuList mask;
  {
    std::lock_guard<std::mutex> lk(mu_);
    mask = start_mask_;
  }
  pin_current_thread(mask);
}

HomeThread::~HomeThread() {
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !busy_; });
    quit_ = true;
  }
  cv_.notify_all();
  if (thread_.get_id() == std::this_thread::get_id()) thread_.detach();  // never from its own task
  else if (thread_.joinable()) thread_.join();
}

HomeThread* Runner::home_thread() {
  if (!home_) home_ = std::make_unique<HomeThread>();
  return home_.get();
}

void Supervisor::start(int64_t max_iterations) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    running_ += runners_.size();
  }
  const size_t n = runners_.size();
  // Posting waits for a task a runner's thread still runs, and that task's last step takes
  // mu_: so no lock is held from here on.
  for (size_t i = 0; i < n; ++i) {
    Runner* rp = runners_[i].get();  // runners_ keeps it alive until join()
    HomeThread* h = rp->home_thread();
    const Nanos period = std::max<Nanos>(rp->config().poll_period, 0);
    const Nanos delay = stagger_ && n > 1 ? static_cast<Nanos>(static_cast<double>(period) * i / n) : 0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      started_.push_back(h);
    }
    h->post([this, rp, h, max_iterations, delay] {
      if (rp->cpus().empty()) h->unpin();
      else pin_current_thread(rp->cpus());
      ThreadSched before, after;
      const bool have = read_thread_sched(&before);
      rp->run(&stop_, max_iterations, delay);
      const bool have_after = have && read_thread_sched(&after);
      std::lock_guard<std::mutex> g(mu_);
      if (have_after) sched_.add(after.since(before));
      --running_;
      cv_.notify_all();
    });
  }
}

bool Supervisor::wait(Nanos timeout) {
  std::unique_lock<std::mutex> lk(mu_);
  if (timeout <= 0) {
    cv_.wait(lk, [&] { return running_ == 0; });
    return true;
  }
  return cv_wait_for(cv_, lk, timeout, [&] { return running_ == 0; });
}

void Supervisor::join() {
  std::vector<HomeThread*> started;
  {
    std::lock_guard<std::mutex> lk(mu_);
    started.swap(started_);
  }
  for (HomeThread* h : started) h->wait_idle();
}

Supervisor::~Supervisor() {
  stop_.request_stop();  // no cancel(): the clients may outlive this supervisor and be reused
  join();
}

// ---------------------------------------------------------------------------------------

Scheduler::Scheduler(size_t threads, std::shared_ptr<Clock> clock, bool stagger)
    : nthreads_(threads < 1 ? 1 : threads), clock_(std::move(clock)), stagger_(stagger) {}

Scheduler::~Scheduler() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_.store(true);  // no cancel(): the clients may outlive this scheduler and be reused
  }
  cv_.notify_all();
  join();
}

void Scheduler::start(int64_t max_iterations) {
  std::lock_guard<std::mutex> lk(mu_);
  max_iter_ = max_iterations;
  done_.assign(runners_.size(), 0);
  heap_.clear();
  const Nanos t0 = clock_->now();
  const size_t n = runners_.size();
  for (size_t i = 0; i < n; ++i) {
    const Nanos period = std::max<Nanos>(runners_[i]->config().poll_period, 0);
    runners_[i]->set_spin_budget(0);  // shared threads: a spin would hold up the other queues
    if (stagger_ && n > 1 && period > 0) {
      heap_.push_back(Item{t0 + static_cast<Nanos>(static_cast<double>(period) * i / n), i, true});
    } else {
      runners_[i]->arm();
      push_poll(i, t0, false);  // heapified below
    }
  }
  std::make_heap(heap_.begin(), heap_.end(), std::greater<Item>());
  finished_ = 0;
  running_ = nthreads_;
  for (size_t t = 0; t < nthreads_; ++t)
    threads_.emplace_back([this] {
      pthread_setname_np(pthread_self(), "ksa-sched");
      worker();
    });
}

void Scheduler::push_poll(size_t idx, Nanos from, bool heapify) {
  const LoopConfig& c = runners_[idx]->config();
  const Nanos period = std::max<Nanos>(c.poll_period, 0), w = c.prewarm;
  const Nanos due = from + period;  // sleep-then-poll (main.go:41)
  if (w > 0 && period > 2 * w)
    heap_.push_back(Item{due - w, idx, false, due});
  else
    heap_.push_back(Item{due, idx, false});
  if (heapify) std::push_heap(heap_.begin(), heap_.end(), std::greater<Item>());
}

void Scheduler::worker() {
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_.load() && finished_ < runners_.size()) {
    if (heap_.empty()) {  // every runner is being polled by another worker
      cv_.wait(lk, [&] { return stop_.load() || !heap_.empty() || finished_ >= runners_.size(); });
      continue;
    }
    const Nanos now = clock_->now();
    const Item top = heap_.front();
    if (top.due > now) {
      cv_wait_for(cv_, lk, top.due - now, [&] {
        return stop_.load() || heap_.empty() || heap_.front().due != top.due || heap_.front().idx != top.idx ||
               clock_->now() >= top.due;
      });
      continue;
    }
    std::pop_heap(heap_.begin(), heap_.end(), std::greater<Item>());
    heap_.pop_back();
    if (top.arm) {  // staggered start: Run() entry for this queue
      runners_[top.idx]->arm();
      push_poll(top.idx, clock_->now());
      cv_.notify_all();
      continue;
    }
    if (top.poll_at > 0) {  // --poll-prewarm: prepare now, poll at its due time (no spinning here:
                            // the thread serves other queues meanwhile)
      lk.unlock();
      runners_[top.idx]->prepare(top.poll_at);
      lk.lock();
      heap_.push_back(Item{top.poll_at, top.idx, false});
      std::push_heap(heap_.begin(), heap_.end(), std::greater<Item>());
      cv_.notify_all();
      continue;
    }
    if (now - top.due > kMillisecond) {
      late_++;
      max_late_ = std::max(max_late_, now - top.due);
    }
    lk.unlock();
    runners_[top.idx]->poll_once();
    lk.lock();
    if (max_iter_ > 0 && ++done_[top.idx] >= max_iter_) {
      ++finished_;
    } else {
      push_poll(top.idx, clock_->now());
    }
    cv_.notify_all();
  }
  --running_;
  cv_.notify_all();
}

void Scheduler::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_.store(true);
  }
  cv_.notify_all();
  for (auto& r : runners_) r->cancel();  // in-flight polls end now instead of at their timeout
}

bool Scheduler::wait(Nanos timeout) {
  std::unique_lock<std::mutex> lk(mu_);
  if (timeout <= 0) {
    cv_.wait(lk, [&] { return running_ == 0; });
    return true;
  }
  return cv_wait_for(cv_, lk, timeout, [&] { return running_ == 0; });
}

void Scheduler::join() {
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

uint64_t Scheduler::late_polls() const {
  std::lock_guard<std::mutex> lk(mu_);
  return late_;
}

Nanos Scheduler::max_lateness() const {
  std::lock_guard<std::mutex> lk(mu_);
  return max_late_;
}

void Scheduler::reset_lateness() {
  std::lock_guard<std::mutex> lk(mu_);
  late_ = 0;
  max_late_ = 0;
}

Nanos percentile(std::vector<Nanos> v, double p) {
  if (v.empty()) return -1;
  std::sort(v.begin(), v.end());
  double rank = std::ceil(p / 100.0 * static_cast<double>(v.size()));
  size_t idx = rank < 1 ? 0 : static_cast<size_t>(rank) - 1;
  if (idx >= v.size()) idx = v.size() - 1;
  return v[idx];
}

}  // namespace ksa
