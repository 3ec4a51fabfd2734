// Injectable time source for the control loop.
//
// The reference reads wall-clock time directly (`time.Sleep`, `time.Now`,
// /root/reference/main.go:37-38,41,52,62,66,76), which is why its loop tests take ~56 s of
// real sleeping (/root/reference/main_test.go:51,88,124,160,198,236). Every native component
// here takes a Clock instead: RealClock in production, VirtualClock in tests and in the
// decision-parity harness, where a whole hour of polling runs in microseconds.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <ctime>

#include "log.h"

namespace ksa {

using Nanos = int64_t;

// Timed condition wait. libstdc++ implements wait_for() with pthread_cond_clockwait
// (CLOCK_MONOTONIC), which GCC 11's ThreadSanitizer does not intercept -- it then misses the
// unlock inside the wait and reports a false "double lock". Under TSan only, wait on the
// system clock (pthread_cond_timedwait, intercepted); production keeps the monotonic clock so
// poll sleeps are immune to wall-clock steps.
template <class Lock, class Pred>
bool cv_wait_for(std::condition_variable& cv, Lock& lk, int64_t ns, Pred pred) {
#if defined(__SANITIZE_THREAD__)
  return cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::nanoseconds(ns), pred);
#else
  return cv.wait_for(lk, std::chrono::nanoseconds(ns), pred);
#endif
}
// CLOCK_MONOTONIC nanoseconds (what RealClock::now() reads): deadlines and diagnostics.
inline int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// CPU time of the calling thread (CLOCK_THREAD_CPUTIME_ID), nanoseconds.
inline int64_t thread_cpu_ns() {
  struct timespec ts;
  if (clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts) != 0) return 0;
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

constexpr Nanos kMicrosecond = 1000;
constexpr Nanos kMillisecond = 1000 * kMicrosecond;
constexpr Nanos kSecond = 1000 * kMillisecond;

// Cooperative cancellation shared between a supervisor and its workers. Sleeping on a
// StopFlag returns early when stop is requested (graceful SIGTERM shutdown, which the
// reference lacks: it never cancels its context, /root/reference/main.go:36).
class StopFlag {
 public:
  void request_stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stopped_.store(true, std::memory_order_release);
    }
    cv_.notify_all();
  }
  bool stopped() const { return stopped_.load(std::memory_order_acquire); }
  // Waits up to `d`; returns true when the full duration elapsed, false if stopped.
  bool wait_for(Nanos d) {
    // Every worker of a Supervisor shares one StopFlag, and a zero poll period calls this on
    // every poll: no lock unless there is something to wait for, or the workers serialise on
    // this mutex (a futex round trip per poll once they collide).
    if (d <= 0) return !stopped();
    std::unique_lock<std::mutex> lk(mu_);
    return !cv_wait_for(cv_, lk, d, [&] { return stopped(); });
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<bool> stopped_{false};
};

class Clock {
 public:
  virtual ~Clock() = default;
  // Monotonic nanoseconds; the origin is arbitrary.
  virtual Nanos now() = 0;
  // Sleeps for `d` (no-op when d <= 0, like time.Sleep). Returns false if `stop` fired.
  virtual bool sleep(Nanos d, StopFlag* stop) = 0;
  // Unix wall-clock nanoseconds (for log timestamps and SigV4 dates).
  virtual int64_t unix_nanos() = 0;
  // Waits until now() >= deadline, busy-waiting on a real clock (for a short final stretch
  // that must end on time with the core awake). Returns false if `stop` fired.
  virtual bool spin_until(Nanos deadline, StopFlag* stop) { return sleep(deadline - now(), stop); }
};

class RealClock final : public Clock {
 public:
  Nanos now() override {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  bool sleep(Nanos d, StopFlag* stop) override {
    if (d > 0) log_flush_pending();  // nothing held back by a wait (log.h)
    if (stop) return stop->wait_for(d);
    if (d > 0) {
      struct timespec ts;
      ts.tv_sec = d / kSecond;
      ts.tv_nsec = d % kSecond;
      while (nanosleep(&ts, &ts) != 0) {
      }
    }
    return true;
  }
  int64_t unix_nanos() override {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
  }
  bool spin_until(Nanos deadline, StopFlag* stop) override {
    for (unsigned i = 0;; ++i) {
      if (now() >= deadline) return true;
      if ((i & 63) == 63 && stop && stop->stopped()) return false;
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
  }
};

// Deterministic clock: sleep() advances time instantly. Fakes advance it to model API
// latency (advance()), which is how the parity harness reproduces the reference's
// "now is read fresh at every comparison" semantics.
class VirtualClock final : public Clock {
 public:
  explicit VirtualClock(Nanos start = 0, int64_t unix_epoch_ns = 1700000000LL * kSecond)
      : t_(start), start_(start), epoch_(unix_epoch_ns) {}
  Nanos now() override { return t_.load(std::memory_order_acquire); }
  bool sleep(Nanos d, StopFlag* stop) override {
    if (stop && stop->stopped()) return false;
    if (d > 0) t_.fetch_add(d, std::memory_order_acq_rel);
    return true;
  }
  int64_t unix_nanos() override { return epoch_ + (now() - start_); }
  void advance(Nanos d) {
    if (d > 0) t_.fetch_add(d, std::memory_order_acq_rel);
  }
  void set(Nanos t) { t_.store(t, std::memory_order_release); }

 private:
  std::atomic<Nanos> t_;
  Nanos start_;
  int64_t epoch_;
};

}  // namespace ksa
