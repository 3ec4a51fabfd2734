// The control loop and its multi-queue supervisor.
//
// Runner::step() is one iteration of the reference's `Run` loop (/root/reference/main.go:40-78):
//   sleep(poll) -> depth := NumMessages() -> scale-up gate -> scale-down gate
// with the exact decision semantics catalogued in SURVEY.md §3.3:
//   * timers armed at Run() entry (main.go:37-38) -- Runner::arm();
//   * inclusive thresholds (main.go:51,65);
//   * proceed iff now >= last + cool-down (`After` is strict, main.go:52,66), `now` re-read at
//     every comparison and again when the timer is refreshed (main.go:62,76);
//   * a cool-down skip or a failed scale-up `continue`s, so the scale-down check is skipped in
//     that iteration (main.go:54,59);
//   * the timer is refreshed after a successful call even when it was a no-op at a bound,
//     and NOT refreshed after a failure (main.go:57-62,71-76).
// Each step returns an IterationRecord, which is what the decision-parity harness compares
// against the reference-semantics oracle, and carries the poll->patch latency span (the
// BASELINE.json metric), measured from the end of the sleep to the end of the last write.
//
// Supervisor runs one Runner per tracked queue on its own thread (the reference tracks a
// single queue per process); runners share nothing, so there is no cross-queue locking.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "affinity.h"
#include "clock.h"
#include "kube.h"
#include "log.h"
#include "sqs.h"

namespace ksa {

// --poll-presend stages only when the warm-up lead is this short: far inside the kernel's 200 ms
// TCP_CORK limit.
inline constexpr Nanos kMaxPresendLead = 50 * kMillisecond;

struct LoopConfig {
  Nanos poll_period = 5 * kSecond;            // --poll-period           main.go:83
  Nanos scale_down_cool_down = 30 * kSecond;  // --scale-down-cool-down  main.go:84
  Nanos scale_up_cool_down = 10 * kSecond;    // --scale-up-cool-down    main.go:85
  int64_t scale_up_messages = 100;            // --scale-up-messages     main.go:86
  int64_t scale_down_messages = 10;           // --scale-down-messages   main.go:87
  // Overlap the Deployment GET with the SQS poll (PodAutoScaler::prefetch). Decisions are the
  // reference's; only the read is issued earlier and validated by the write's resourceVersion.
  bool prefetch = false;                      // --pipeline-reads
  // By default the speculative GET is only sent when a scale call is likely to follow the SQS
  // response (Runner::action_likely), so an idle queue costs the apiserver what the reference
  // costs it: nothing between cool-down expiries. true: send it with every poll.
  bool prefetch_always = false;
  // Pre-poll warm-up (--poll-prewarm): wake this long before a poll is due, do what the poll
  // would do first without sending anything -- credentials, the signed SQS request for that
  // second, the bearer token, both connections checked (or dialled) -- then, for a near SQS
  // endpoint (response EWMA within HttpClient::kMaxSpinThrough), spin until the due time, so the
  // poll starts on time on an awake core with its code and data in cache; against a remote one
  // sleep out the rest of the lead (the spin would cost more CPU than the poll and save noise).
  // The spin is the last part of the lead, at most the warm-up's quarter of the poll's spin
  // budget (Runner::set_spin_budget); the part before it is slept. The poll itself, and so every
  // decision, is unchanged (sleep-then-poll, main.go:41).
  // 0 disables. With a poll period under 2x `prewarm` the preparation runs at the due time
  // instead, without the early wake-up.
  Nanos prewarm = 0;
  // After the warm-up, spin to the due time when the SQS endpoint is near (above); false: always
  // sleep out the rest of the lead (the A/B knob of scripts/spin_arms.py).
  bool prewarm_spin = true;
  // With the early wake-up, also pre-send the SQS request (HttpClient::stage; --poll-presend,
  // off by default): all but its last bytes are handed to the kernel corked, so the kernel's send
  // path has run before the due time and the poll's own write runs warm; nothing reaches the wire
  // before the due time, and the request is byte for byte the one the poll sends (when it is not
  // -- its signing second rolled over -- the staged connection is dropped and the poll dials a
  // fresh one). Linux releases a cork after 200 ms, so only a lead under kMaxPresendLead stages
  // (a poll that starts over 200 ms late lets the peer see a partial request until the rest
  // comes). Off by default: paired A/Bs showed no end-to-end win beyond noise (p50 0.96x,
  // profiles/r04r_presend_ab.jsonl) for a staging path and a redial on a discard.
  bool presend = false;
  // Dial both clients at Run() entry, on the worker's own thread, before the timers are armed
  // (decisions unchanged). A harness that would otherwise connect them from its main thread
  // (the bench) gets each connection's TLS state and buffers from the worker's allocator arena
  // instead of one shared arena. The CLI needs none: its first poll, or its first warm-up, dials
  // on the worker thread.
  bool connect_at_start = false;
  // On a worker's own thread, the share of the poll period (parts per million) a poll may spend
  // spinning beyond the --busy-poll window: to the due time after the warm-up, and through an
  // answer slower than the window while twice the response-time EWMA fits (Runner::set_spin_budget
  // splits it over the warm-up, the SQS call, the GET and the write, so it bounds the poll's
  // spinning as a whole). The CLI's --busy-poll-budget gives a process's queues that percent in
  // total (10000 ppm per percent, divided by the queue count), so their spinning stays within it
  // whatever the queue count; under a cgroup CPU limit, within a tenth of the quota
  // (Runner::spin_budget_for). Only answers within HttpClient::kMaxSpinThrough are ever spun
  // through: a remote endpoint costs no spinning. 0 (the CLI's default since round 5: paired runs
  // showed no latency gain beyond noise for about 1.5x the CPU per poll, profiles/r05c, r05d):
  // the window only. Pooled threads never spin beyond the window.
  int64_t spin_budget_ppm = 0;
};

enum class Action : int { None = 0, CoolDown = 1, Scaled = 2, NoopAtBound = 3, Failed = 4 };
const char* action_name(Action a);

struct IterationRecord {
  uint64_t index = 0;     // 1-based poll number
  bool stopped = false;   // the sleep was interrupted by a stop request
  Nanos t_poll = 0;       // clock time at the end of the sleep
  bool depth_ok = false;
  int64_t depth = 0;
  Action up = Action::None;
  Action down = Action::None;
  int32_t replicas_before = -1;  // as read by the last GET of the iteration (-1: not read)
  int32_t replicas_after = -1;
  bool prefetched = false;     // a pipelined GET was issued with the poll
  bool prefetch_gated = false; // --pipeline-reads, but the gate predicted no action: none sent
  bool prefetch_used = false;  // ... and a scale decision consumed it
  int gets = 0;                // Deployment GETs this poll (speculative + synchronous)
  Nanos depth_ns = 0;          // SQS GetQueueAttributes round trip
  Nanos get_ns = 0;            // Deployment GET(s)
  Nanos update_ns = 0;         // Deployment PUT/PATCH(es)
  Nanos total_ns = 0;          // end of sleep -> end of iteration
  Nanos patch_latency_ns = -1; // end of sleep -> end of last successful write (-1: no write)
  // CPU time of the worker thread for this poll: from the start of the iteration (its sleep, then
  // the warm-up and its spin, then the poll) to the end of the poll -- everything but a sleep
  // costs CPU here, spinning included. Pooled threads (Scheduler) count the poll alone. -1: none.
  Nanos cpu_ns = -1;
  std::string error;
  std::string detail;  // traced polls with timed clients: {"sqs":{...},"write":{...}} (HttpTiming)
};

// Poll->patch latency histogram: bucket i counts samples <= kLatBucketLeNs[i] (and above the
// previous bound); the last bucket is everything above 10 s. Prometheus-style bounds from 10 µs
// (a localhost poll) to 10 s (a throttled apiserver).
constexpr int kLatBuckets = 20;
constexpr int64_t kLatBucketLeNs[kLatBuckets - 1] = {
    10000,     25000,     50000,      100000,     250000,     500000,     1000000,
    2500000,   5000000,   10000000,   25000000,   50000000,   100000000,  250000000,
    500000000, 1000000000, 2500000000, 5000000000, 10000000000};
inline int latency_bucket(int64_t ns) {
  int i = 0;
  while (i < kLatBuckets - 1 && ns > kLatBucketLeNs[i]) ++i;
  return i;
}

struct RunnerStats {
  uint64_t polls = 0;
  uint64_t depth_errors = 0;
  uint64_t scale_ups = 0;
  uint64_t scale_downs = 0;
  uint64_t noop_ups = 0;
  uint64_t noop_downs = 0;
  uint64_t cooldown_skips_up = 0;
  uint64_t cooldown_skips_down = 0;
  uint64_t failed_ups = 0;
  uint64_t failed_downs = 0;
  uint64_t speculative_reads = 0;       // pipelined GETs issued (one per poll with --pipeline-reads)
  uint64_t speculative_reads_used = 0;  // ... consumed by a scale decision (the rest are extra API load)
  uint64_t speculative_reads_gated = 0; // polls where the gate predicted no action and sent none
  uint64_t apiserver_reads = 0;         // Deployment GETs of any kind (speculative + synchronous)
  int64_t last_depth = 0;
  int32_t last_replicas = -1;
  uint64_t latency_samples = 0;
  int64_t latency_sum_ns = 0;                 // over every sample (the ring keeps the latest)
  int64_t poll_cpu_ns = 0;                    // sum of IterationRecord::cpu_ns over every poll
  // Readiness: polls in a row that failed to read the depth or to write the Deployment, and
  // when the last poll that did neither ended (clock time; Run() entry before any poll).
  uint64_t consecutive_failed_polls = 0;
  Nanos last_good_ns = 0;
  uint64_t latency_buckets[kLatBuckets] = {};  // per bucket, not cumulative
};

// A worker's state mirrored into memory shared with a supervising process (the process-per-queue
// fleet, kube_sqs_autoscaler_amd/parallel/procfleet.py): its counters, liveness and recent
// poll->patch latencies for /metrics, /healthz and the benchmark, plus two words the parent
// writes (a start/stop control and a max-pods override from the GPU-capacity cap). Lock-free
// atomics only -- address-free on x86-64, so they work across processes -- and each word has one
// writer: the worker for its state, the parent for the control words.
struct SharedWorkerState {
  enum Counter : int {
    kPolls, kDepthErrors, kScaleUps, kScaleDowns, kNoopUps, kNoopDowns, kCooldownSkipsUp,
    kCooldownSkipsDown, kFailedUps, kFailedDowns, kSpeculativeReads, kSpeculativeReadsUsed,
    kSpeculativeReadsGated, kApiserverReads, kLatencySamples, kConsecutiveFailedPolls, kPollCpuNs, kNumCounters
  };
  enum Control : int32_t { kWait = 0, kGo = 1, kStop = 2 };
  enum Status : int32_t { kStarting = 0, kReady = 1, kRunning = 2, kExited = 3, kFailed = 4 };
  static constexpr uint32_t kRing = 1 << 14;  // latency samples kept (the most recent)
  alignas(64) std::atomic<uint64_t> counters[kNumCounters];
  std::atomic<int64_t> progress_ns;  // CLOCK_MONOTONIC of the last progress (the worker process' heartbeat)
  std::atomic<int64_t> last_good_ns;  // CLOCK_MONOTONIC of the last poll that did not fail
  std::atomic<int64_t> last_depth;
  std::atomic<int64_t> last_replicas;
  std::atomic<int64_t> lat_sum_ns;
  std::atomic<int32_t> status;
  alignas(64) std::atomic<int64_t> max_override;  // parent -> worker: > 0 caps max-pods
  std::atomic<int64_t> iterations;                // parent -> worker: polls to run (<= 0: until stopped)
  std::atomic<int32_t> control;                   // parent -> worker
  alignas(64) std::atomic<uint64_t> lat_hist[kLatBuckets];  // per bucket (RunnerStats::latency_buckets)
  alignas(64) std::atomic<int64_t> lat_ring[kRing];
  // The worker's last poll error (Runner::last_error), truncated to kErrorBytes - 1 bytes, for
  // the parent's /readyz reason. A seqlock: error_seq is odd while the worker rewrites the text;
  // the text is stored as relaxed atomic words, so a racing read is torn, never undefined, and is
  // retried when the sequence moved (write_shared_error / read_shared_error).
  static constexpr size_t kErrorBytes = 512;
  alignas(64) std::atomic<uint64_t> error_seq;
  std::atomic<uint32_t> error_len;
  std::atomic<uint64_t> error_words[kErrorBytes / 8];
};
static_assert(std::atomic<int64_t>::is_always_lock_free, "shared-memory atomics must be lock-free");
// Zero-initialises a SharedWorkerState in place (memory from a fresh shared mapping).
SharedWorkerState* init_shared_worker_state(void* at);
// The error slot of a SharedWorkerState: the worker (single writer) stores its last poll error,
// the supervising process reads it. read_shared_error returns "" when it could not get a
// consistent copy within a few retries (the worker rewriting it continuously).
void write_shared_error(SharedWorkerState* s, const std::string& text);
std::string read_shared_error(const SharedWorkerState* s);

// The OS thread a Runner's loop runs on, kept for the Runner's lifetime across Supervisor runs
// (named ksa-worker). glibc gives every thread a malloc arena of its own and hands the arena of
// an exited thread to the next thread created. When a fleet's threads are replaced -- a
// warm-up run, any restart of a Supervisor -- queue i's new thread inherits the arena in which
// queue j's old thread allocated j's lazily-built buffers, and i's per-poll temporaries land on
// the cache lines of buffers j's thread writes every poll. Measured on the 8-queue thread fleet
// (docs/HISTORY.md, r02l): the same instructions per poll, +70 % user cycles and ~80 more
// cache misses per poll, +30 % p50; with the threads kept, the fleet polls like one queue.
class HomeThread {
 public:
  HomeThread();
  ~HomeThread();  // lets the task in progress finish, then ends the thread
  HomeThread(const HomeThread&) = delete;
  HomeThread& operator=(const HomeThread&) = delete;
  // Runs `task` on the thread (after the previous task, if one is still running).
  void post(std::function<void()> task);
  void wait_idle();
  // Restores the CPU mask the thread started with (a run without explicit CPUs after a pinned one).
  void unpin();

 private:
  void loop();
  std::mutex mu_;
  std::condition_variable cv_;
  std::function<void()> task_;
  bool busy_ = false;
  bool quit_ = false;
  CpuList start_mask_;
  std::thread thread_;
};

class alignas(kCacheLine) Runner {
 public:
  Runner(LoopConfig cfg, std::shared_ptr<SqsClient> sqs, std::shared_ptr<PodAutoScaler> scaler,
         std::shared_ptr<Clock> clock, std::shared_ptr<Logger> log);

  // main.go:37-38: lastScaleUpTime = lastScaleDownTime = time.Now().
  void arm();
  // One loop iteration; `stop` may interrupt the sleep.
  IterationRecord step(StopFlag* stop = nullptr);
  // The iteration without the leading sleep (main.go:43-77); used by Scheduler, which owns
  // the waiting between polls.
  IterationRecord poll_once();
  // The pre-poll warm-up (LoopConfig::prewarm) for a poll due at `due`, without waiting: the
  // Scheduler runs it as its own event `prewarm` before the poll's.
  void prepare(Nanos due) { warm(due, true); }
  // Shutdown: aborts this worker's API call in progress and its back-off/throttle waits.
  void cancel() {
    sqs_->cancel();
    scaler_->cancel();
  }
  // Splits one poll's spin budget over what a poll spins for: a quarter to the warm-up's spin
  // to the due time, half to the SQS call's read, an eighth to each of the apiserver's GET and
  // write (HttpClient::set_spin_budget applies per request), so a scaling poll spins at most
  // `ns` in total. The SQS answer is the one slow enough to need a read budget (at a cadence its
  // EWMA is past 4x the busy-poll window); the apiserver's answers mostly come within the window,
  // which needs none. (An SDK retry of the SQS call spins within its own share again; retries
  // are the error path.)
  void set_spin_budget(Nanos ns) {
    prewarm_spin_budget_ = ns / 4;
    sqs_->api()->set_spin_budget(ns / 2);
    scaler_->api()->set_spin_budget(ns / 8);
  }
  // The warm-up's share: the spin before the due time is at most this (the rest of the lead is
  // slept). -1 (before set_spin_budget, e.g. a harness calling step() itself): the whole lead.
  Nanos prewarm_spin_budget() const { return prewarm_spin_budget_; }
  // The spin budget run() gives a poll: LoopConfig::spin_budget_ppm of the poll period, and
  // under a cgroup CPU limit at most a tenth of one CFS period's quota (times this queue's share).
  static Nanos spin_budget_for(const LoopConfig& cfg, const CpuQuota& quota);
  // Closes the clients' keep-alive connections (on the calling thread's file table).
  void release_connections() {
    sqs_->api()->close_connections();
    scaler_->api()->close_connections();
  }
  // The reference's Run(): arm(), then step() until stopped (or max_iterations > 0 reached).
  // start_delay > 0: wait that long first (interruptible by `stop`), then arm -- a staggered
  // start, as if this queue's reference process had been launched that much later.
  void run(StopFlag* stop, int64_t max_iterations = -1, Nanos start_delay = 0);

  RunnerStats stats() const;
  // Time since the loop last made progress (armed, or finished a poll) -- the liveness signal:
  // a worker wedged inside a call, or whose thread died, stops resetting it.
  // A deliberate wait of its clients (Retry-After, back-off, throttle) counts as progress up
  // to its end: a worker correctly waiting out a server's Retry-After is not wedged.
  Nanos idle_ns() const;
  // How long every poll has been failing (0 while the last poll succeeded): the time since the
  // last poll that read the depth and wrote what it decided, or since Run() entry. The
  // reference retries such a poll forever (main.go:44-47,57-60,71-74), so this is a readiness
  // signal (/readyz), not a liveness one.
  Nanos failing_ns() const;
  std::string last_error() const;
  // Recent poll->patch latencies (ns), oldest first; bounded ring.
  std::vector<Nanos> latencies() const;
  void clear_latencies();
  // Optional per-iteration observer (metrics export, tests). Called on the runner thread.
  void set_observer(std::function<void(const IterationRecord&)> f) { observer_ = std::move(f); }
  // Span tracing: one JSON object per iteration, written with a single write(2) to `fd`
  // (an O_APPEND file shared by all workers stays line-atomic). -1 disables.
  void set_trace_fd(int fd) { trace_fd_ = fd; }
  const LoopConfig& config() const { return cfg_; }
  std::shared_ptr<SqsClient> sqs() const { return sqs_; }
  std::shared_ptr<PodAutoScaler> scaler() const { return scaler_; }
  Nanos last_scale_up() const { return last_up_; }
  Nanos last_scale_down() const { return last_down_; }
  // CPUs the thread running this worker is pinned to (Supervisor; empty: no pinning).
  void set_cpus(CpuList cpus) { cpus_ = std::move(cpus); }
  // Mirror the stats into `s` after every poll and follow its max-pods override (may be null).
  void set_shared_state(SharedWorkerState* s) { shared_ = s; }
  const CpuList& cpus() const { return cpus_; }
  // This runner's HomeThread (created on first use, kept for the runner's lifetime).
  HomeThread* home_thread();

 private:
  IterationRecord poll_body();
  void warm(Nanos due, bool presend = false);
  void record(IterationRecord& r);
  int64_t cpu_from_ = -1;  // thread CPU time at the start of the iteration in progress
  Nanos prewarm_spin_budget_ = -1;
  void mirror(const IterationRecord& r);
  CpuList cpus_;
  SharedWorkerState* shared_ = nullptr;

  LoopConfig cfg_;
  std::shared_ptr<SqsClient> sqs_;
  std::shared_ptr<PodAutoScaler> scaler_;
  std::shared_ptr<Clock> clock_;
  std::shared_ptr<Logger> log_;
  Nanos last_up_ = 0, last_down_ = 0;
  uint64_t index_ = 0;
  // Prefetch gate inputs: the last depth read (if any) and the last SQS round trip.
  bool have_depth_ = false;
  int64_t last_depth_ = 0;
  Nanos last_depth_rtt_ = 0;
  bool action_likely(Nanos t0) const;
  std::function<void(const IterationRecord&)> observer_;
  int trace_fd_ = -1;
  void write_trace(const IterationRecord& r);

  mutable std::mutex mu_;
  std::atomic<Nanos> progress_ns_{0};
  RunnerStats stats_;
  std::string last_error_;
  std::vector<Nanos> lat_ring_;
  size_t lat_pos_ = 0;
  static constexpr size_t kLatRing = 1 << 16;
  std::unique_ptr<HomeThread> home_;  // last: ends (after its task) before the state it runs on
};

// Scheduler accounting of one thread (/proc/thread-self/schedstat and status): time on CPU, time
// runnable but waiting for a CPU, timeslices, voluntary / involuntary context switches.
struct ThreadSched {
  int64_t threads = 0;
  int64_t cpu_ns = 0;
  int64_t runq_wait_ns = 0;
  int64_t slices = 0;
  int64_t vol_cs = 0;
  int64_t invol_cs = 0;
  int64_t utime_ns = 0;  // getrusage(RUSAGE_THREAD): user / system CPU, minor page faults
  int64_t stime_ns = 0;
  int64_t minflt = 0;
  void add(const ThreadSched& o) {
    utime_ns += o.utime_ns;
    stime_ns += o.stime_ns;
    minflt += o.minflt;
    threads += o.threads;
    cpu_ns += o.cpu_ns;
    runq_wait_ns += o.runq_wait_ns;
    slices += o.slices;
    vol_cs += o.vol_cs;
    invol_cs += o.invol_cs;
  }
  // What the same thread accumulated since `o` was read (a HomeThread serves many runs).
  ThreadSched since(const ThreadSched& o) const {
    ThreadSched d = *this;
    d.utime_ns -= o.utime_ns;
    d.stime_ns -= o.stime_ns;
    d.minflt -= o.minflt;
    d.cpu_ns -= o.cpu_ns;
    d.runq_wait_ns -= o.runq_wait_ns;
    d.slices -= o.slices;
    d.vol_cs -= o.vol_cs;
    d.invol_cs -= o.invol_cs;
    return d;
  }
};
// The calling thread's counters (false when /proc is unavailable).
bool read_thread_sched(ThreadSched* out);

class Supervisor {
 public:
  Supervisor();
  void add(std::shared_ptr<Runner> r) { runners_.push_back(std::move(r)); }
  // Staggered start (the Scheduler's default too): runner i of N arms its timers and starts its
  // sleep-then-poll loop i/N of its poll period after start(), so N queues with one poll period
  // do not poll in one burst every period -- as N reference processes launched a little apart
  // would not. Per-queue decisions are unchanged: each queue's timers start at its own Run()
  // entry (main.go:37-38), exactly as the reference's.
  void set_stagger(bool on) { stagger_ = on; }
  bool stagger() const { return stagger_; }
  // Runs every runner on its HomeThread (one thread per runner, kept across runs); each arms
  // its timers then loops.
  void start(int64_t max_iterations = -1);
  // Stop request: interrupts poll sleeps and cancels every worker's in-flight API call, so a
  // SIGTERM does not wait for a slow or hung endpoint (the call's own timeout can be 30 s).
  void stop() {
    stop_.request_stop();
    for (auto& r : runners_) r->cancel();
  }
  bool stopped() const { return stop_.stopped(); }
  // Waits up to `timeout` (<= 0: forever); true when every runner thread has exited.
  bool wait(Nanos timeout);
  void join();
  size_t size() const { return runners_.size(); }
  std::shared_ptr<Runner> runner(size_t i) const { return runners_.at(i); }
  StopFlag* stop_flag() { return &stop_; }
  // Totals over the worker threads that have exited (each adds its counters on the way out):
  // where a worker's wall time went besides its own work -- e.g. run-queue waits when more
  // threads are runnable than the process's CPU share.
  ThreadSched thread_sched() const {
    std::lock_guard<std::mutex> lk(mu_);
    return sched_;
  }
  ~Supervisor();

 private:
  std::vector<std::shared_ptr<Runner>> runners_;
  std::vector<HomeThread*> started_;  // the runners' threads this supervisor posted to
  StopFlag stop_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  size_t running_ = 0;
  ThreadSched sched_;
  bool stagger_ = false;
};

// JSON line of an iteration record (span trace format).
std::string iteration_json(const IterationRecord& r, int64_t unix_ns, const std::string& queue,
                           const std::string& deployment);

// N runners on K worker threads (K << N for processes tracking many queues). Each runner keeps
// the reference's cadence: its next poll is due one poll period after its previous poll
// finished (sleep-then-work, main.go:41), and a runner never has two polls in flight, so its
// decisions are exactly those of a dedicated thread. If more polls are due than there are
// workers, a poll starts late -- what an oversleeping time.Sleep would do; the cool-down
// comparisons read the clock at decision time either way.
class Scheduler {
 public:
  // stagger: runner i starts (arms its timers, main.go:37-38) at i/N of its poll period instead
  // of all at once -- as if N reference processes had been launched a little apart -- so the
  // first polls do not arrive as one burst. Per-queue semantics are unchanged.
  explicit Scheduler(size_t threads, std::shared_ptr<Clock> clock = std::make_shared<RealClock>(),
                     bool stagger = true);
  ~Scheduler();
  void add(std::shared_ptr<Runner> r) { runners_.push_back(std::move(r)); }
  // Arms every runner (timers start now, main.go:37-38) and starts the workers; each runner
  // stops after max_iterations polls (<= 0: until stop()).
  void start(int64_t max_iterations = -1);
  void stop();
  bool stopped() const { return stop_.load(); }
  bool wait(Nanos timeout);  // true when all workers exited
  void join();
  size_t size() const { return runners_.size(); }
  size_t threads() const { return nthreads_; }
  std::shared_ptr<Runner> runner(size_t i) const { return runners_.at(i); }
  // Polls that started later than due (scheduler saturation), and the worst lateness.
  uint64_t late_polls() const;
  Nanos max_lateness() const;
  void reset_lateness();

 private:
  struct Item {
    Nanos due;
    size_t idx;
    bool arm = false;  // start event: arm the runner, first poll one period later
    Nanos poll_at = 0;  // > 0: a warm-up event (Runner::prepare) for the poll due then
    bool operator>(const Item& o) const { return due != o.due ? due > o.due : idx > o.idx; }
  };
  // Queues runner idx's next poll one period after `from`: preceded by a warm-up event when its
  // LoopConfig::prewarm fits the period (the same rule as Runner::step).
  void push_poll(size_t idx, Nanos from, bool heapify = true);
  void worker();

  size_t nthreads_;
  std::shared_ptr<Clock> clock_;
  std::vector<std::shared_ptr<Runner>> runners_;
  std::vector<std::thread> threads_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Item> heap_;  // min-heap on due
  std::vector<int64_t> done_;
  int64_t max_iter_ = -1;
  size_t finished_ = 0;  // runners that reached max_iter_
  size_t running_ = 0;   // live worker threads
  std::atomic<bool> stop_{false};
  uint64_t late_ = 0;
  Nanos max_late_ = 0;
  bool stagger_ = true;
};

// Percentile (nearest-rank on a sorted copy), p in [0, 100].
Nanos percentile(std::vector<Nanos> v, double p);

}  // namespace ksa
