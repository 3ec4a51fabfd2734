// Replica actuator: Kubernetes Deployment scaling.
//
// Reference: /root/reference/scale/scale.go. PodAutoScaler reads the Deployment, computes the
// clamped next replica count and writes it back (full-object GET + PUT through client-go,
// scale.go:54-107). Here:
//   * DeploymentApi       -- the injectable seam (the reference's typedappv1.DeploymentInterface,
//                            scale.go:22); `get` returns the replica count plus the opaque object
//                            that `update` writes back (optimistic concurrency via
//                            metadata.resourceVersion, exactly like client-go's Update).
//   * KubeRestDeployments -- REST client: ScaleMode::Deployment reproduces the reference's
//                            GET/PUT of the whole apps/v1 Deployment; ScaleMode::Scale (the
//                            default, per BASELINE.json) uses the autoscaling/v1 /scale
//                            subresource (smaller payloads, narrower RBAC); ScaleMode::Patch
//                            sends a JSON merge patch with a resourceVersion precondition.
//                            When RBAC refuses /scale (a Role written for the reference) the
//                            client falls back to ScaleMode::Deployment once and for all.
//   (FakeDeployments, the in-memory object tracker the reference tests use via client-go's fake
//   clientset, scale_test.go:85-115, is in csrc/fakes/mem_fakes.h: test builds only.)
//   * PodAutoScaler       -- ScaleUp/ScaleDown with the reference's int32 clamp arithmetic and
//                            log messages; a no-op at a bound returns OK (scale.go:62-65,89-92).
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "clock.h"
#include "http.h"
#include "log.h"
#include "status.h"

namespace ksa {

struct ScaleObject {
  bool has_replicas = false;
  int32_t replicas = 0;
  std::string resource_version;
  std::string raw;  // object as fetched (JSON); empty for in-memory fakes
};

class DeploymentApi {
 public:
  virtual ~DeploymentApi() = default;
  virtual Result<ScaleObject> get(const std::string& name) = 0;
  // Writes `fetched` back with spec.replicas = replicas.
  virtual Status update(const std::string& name, const ScaleObject& fetched, int32_t replicas) = 0;
  // Pipelined read: begin_get() starts a GET and returns without waiting (false: not
  // supported, nothing started); finish_get() returns its result. Implementations that
  // cannot overlap I/O keep the defaults and the control loop reads synchronously.
  // may_dial false: start it only on a connection that needs no dial (the caller is inside
  // another request's deadline); otherwise return false and let the synchronous GET run.
  virtual bool begin_get(const std::string& name, bool may_dial = true) {
    (void)name;
    (void)may_dial;
    return false;
  }
  virtual Result<ScaleObject> finish_get() {
    return Result<ScaleObject>::Err(Status::Err("no pipelined GET in flight"));
  }
  // Shutdown: abort the request in progress and any throttle wait (sticky). Default: nothing.
  virtual void cancel() {}
  // Closes the keep-alive connection (and drops a pipelined GET in flight); see SqsApi.
  virtual void close_connections() {}
  // Clock time at which the latest deliberate wait (client-side throttle, Retry-After) ends or
  // ended; 0: none yet. The liveness check counts such a wait as progress.
  virtual Nanos waiting_until() const { return 0; }
  // Pre-poll warm-up (Runner prewarm): the bearer token and the connection check or dial, done
  // before the poll is due. Sends nothing. Default: nothing.
  virtual void warm() {}
  // The last request's time breakdown as a JSON object ("" when not timed).
  virtual std::string timing_json() const { return ""; }
  // HttpClient::set_spin_budget of the client's connection. Default: nothing.
  virtual void set_spin_budget(Nanos ns) { (void)ns; }
};

class TokenProvider {
 public:
  virtual ~TokenProvider() = default;
  virtual Result<std::string> token() = 0;
  // The apiserver answered 401 to a request carrying `used`: drop it if it is still the cached
  // token, so the next token() fetches a fresh one (client-go's exec authenticator and token
  // file source both refresh on 401).
  virtual void invalidate(const std::string& used) { (void)used; }
  // A client of this source stops (its API's cancel()): a fetch in flight is abandoned and its
  // waiters get "request canceled". Later calls fetch as usual. Default: nothing to interrupt.
  virtual void cancel() {}
};

class StaticTokenProvider final : public TokenProvider {
 public:
  explicit StaticTokenProvider(std::string t) : t_(std::move(t)) {}
  Result<std::string> token() override { return Result<std::string>::Ok(t_); }

 private:
  std::string t_;
};

// Bound service-account tokens rotate (~1 h lifetime); client-go re-reads the projected
// token file periodically. Re-read every `refresh` (default 60 s) using `clock`.
class FileTokenProvider final : public TokenProvider {
 public:
  FileTokenProvider(std::string path, std::shared_ptr<Clock> clock, Nanos refresh = 60 * kSecond);
  Result<std::string> token() override;
  void invalidate(const std::string& used) override;

 private:
  std::string path_;
  std::shared_ptr<Clock> clock_;
  Nanos refresh_;
  std::mutex mu_;
  bool have_ = false;
  Nanos read_at_ = 0;
  std::string cached_;
};

// Client-side request throttle: client-go's rest.Config default (QPS 5, burst 10) through
// flowcontrol.NewTokenBucketRateLimiter, whose Accept() reserves a token from a
// golang.org/x/time/rate limiter and sleeps until it is due. The bucket starts full; a reservation
// takes its token at once (the count may go negative), so waiters are served in order.
class alignas(kCacheLine) TokenBucket {
 public:
  TokenBucket(double qps, int burst, std::shared_ptr<Clock> clock);
  // Reserves one token; returns how long the caller must wait before using it.
  Nanos reserve();
  // reserve() + sleep on the clock (interrupted by `stop`). Returns the time waited.
  Nanos take(StopFlag* stop = nullptr);
  // Takes a token only if one is available right now (never waits, never goes into debt).
  bool try_take();

 private:
  void refill_locked();
  std::mutex mu_;
  double qps_, burst_, tokens_;
  Nanos last_ = 0;
  bool started_ = false;
  std::shared_ptr<Clock> clock_;
};

enum class ScaleMode { Deployment, Scale, Patch };

struct KubeOptions {
  std::string server;  // https://host:port
  std::string namespace_ = "default";
  ScaleMode mode = ScaleMode::Scale;
  TlsOptions tls;
  std::shared_ptr<TokenProvider> token;  // bearer token (may be null)
  std::string basic_user, basic_password;  // legacy kubeconfig basic auth
  Nanos timeout = 30 * kSecond;
  Nanos busy_poll = 0;  // HttpClient::set_busy_poll
  std::string proxy;    // HttpClient::set_proxy ("" = direct)
  // Per-client throttle (client-go: QPS 5, burst 10 per clientset). qps <= 0: unthrottled.
  double qps = 0;
  int burst = 0;
  std::shared_ptr<Clock> clock;  // for the throttle's waits (null: RealClock)
  // Scale/Patch modes: when the apiserver refuses the /scale subresource (403: a Role written
  // for the reference grants only get/update on `deployments`, /root/reference/scale/scale.go:55,72;
  // 404: no such subresource) but the Deployment itself can be read, switch this client to
  // Mode::Deployment for good -- the reference's full-object GET+PUT -- and log one warning.
  bool rbac_fallback = true;
  std::shared_ptr<Logger> log;  // for that warning (null: none)
};

struct KubeStats {
  uint64_t gets = 0;
  uint64_t updates = 0;
  uint64_t errors = 0;
  uint64_t conflicts = 0;
  uint64_t throttled = 0;     // requests that waited for the client-side throttle
  int64_t throttle_ns = 0;    // total time spent waiting
  uint64_t speculative_skipped = 0;  // pipelined GETs not sent: no throttle token free
  uint64_t retry_after = 0;          // client-go style retries (Retry-After, or a reset GET)
  uint64_t scale_fallbacks = 0;      // switches from /scale to the whole Deployment (0 or 1)
  HttpClientStats http;
};

class alignas(kCacheLine) KubeRestDeployments final : public DeploymentApi {
 public:
  explicit KubeRestDeployments(KubeOptions opts);
  Result<ScaleObject> get(const std::string& name) override;
  Status update(const std::string& name, const ScaleObject& fetched, int32_t replicas) override;
  bool begin_get(const std::string& name, bool may_dial = true) override;
  Result<ScaleObject> finish_get() override;
  void warm() override;
  void set_timing(bool on) {
    if (http_) http_->set_timing(on);
  }
  void set_spin_budget(Nanos ns) override {
    if (http_) http_->set_spin_budget(ns);
  }
  std::string timing_json() const override {
    return http_ && http_->timing() ? http_timing_json(http_->last_timing()) : "";
  }
  KubeStats stats() const;
  void cancel() override;
  void close_connections() override {
    if (http_) http_->close();
  }
  std::string path_for(const std::string& name) const;
  ScaleMode mode() const { return static_cast<ScaleMode>(mode_.load(std::memory_order_acquire)); }
  Nanos waiting_until() const override { return wait_until_.load(std::memory_order_acquire); }

 private:
  std::atomic<Nanos> wait_until_{0};
  std::shared_ptr<Clock> wait_clock_;  // opts_.clock or a RealClock
  std::string path_in(ScaleMode m, const std::string& name) const;
  Result<ScaleObject> get_in(ScaleMode m, const std::string& name);
  // A /scale request failed with `s`: read the Deployment; when that works, switch to
  // Mode::Deployment (once, with a warning) and return it, else return nothing.
  bool try_fallback(const Status& s, const std::string& name, Result<ScaleObject>* deployment);
  std::atomic<int> mode_;
  // Seconds client-go would wait before retrying this outcome (rest.Request.request, checkWait):
  // the integer Retry-After of a 429 / 5xx response, or 1 for a GET whose connection was reset
  // or hit EOF; -1 = do not retry.
  int64_t retry_wait_s(const HttpRequest& req, const HttpResponse& resp, const Status& transport) const;
  bool sleep_retry(int64_t seconds);
  Status do_request(const std::string& verb_desc, HttpRequest* req, HttpResponse* resp,
                    const std::string& name);
  Status add_auth(HttpRequest* req);
  Status check_response(const std::string& verb_desc, const HttpRequest& req, const HttpResponse& resp,
                        const std::string& name, const Status& transport);
  Result<ScaleObject> parse_get(ScaleMode m, const Status& s, const HttpResponse& resp);
  std::string pending_name_;
  ScaleMode pending_mode_ = ScaleMode::Scale;
  HttpRequest pending_req_;
  Status pending_status_;

  KubeOptions opts_;
  Status init_status_;
  Url url_;
  std::unique_ptr<HttpClient> http_;
  std::unique_ptr<TokenBucket> limiter_;
  StopFlag cancel_;
  void throttle();
  mutable std::mutex mu_;
  KubeStats stats_;
};

// Parses a Deployment or Scale object (JSON) into a ScaleObject. `absent_is_zero` is true for
// autoscaling/v1 Scale, whose spec.replicas is omitempty (absent means 0).
Result<ScaleObject> parse_scale_object(const std::string& json, bool absent_is_zero);
// Returns `raw` with spec.replicas set to `replicas` (inserted when absent).
Result<std::string> set_spec_replicas(const std::string& raw, int32_t replicas);
// The same two through the JSON DOM (json_parse): what the fast single-scan paths above fall
// back to outside the plain case, and the reference the differential tests hold them to.
Result<ScaleObject> parse_scale_object_dom(const std::string& json, bool absent_is_zero);
Result<std::string> set_spec_replicas_dom(const std::string& raw, int32_t replicas);

// Per-call timing of one ScaleUp/ScaleDown (for poll->patch latency spans).
struct ScaleSpan {
  Nanos get_ns = 0;
  Nanos update_ns = 0;
  bool read = false;   // the GET succeeded and carried a replica count
  bool wrote = false;
  int32_t before = 0;
  int32_t after = 0;
  bool used_prefetch = false;  // the decision used the pipelined GET
  bool refetched = false;      // the pipelined object was stale (409) and was re-read
  int gets = 0;                // synchronous GETs this call sent (the pipelined one not counted)
};

class alignas(kCacheLine) PodAutoScaler {
 public:
  PodAutoScaler(std::shared_ptr<DeploymentApi> api, std::string deployment, std::string ns,
                int64_t max, int64_t min, int64_t scale_up_pods, int64_t scale_down_pods,
                std::shared_ptr<Logger> log, std::shared_ptr<Clock> clock);
  Status scale_up(ScaleSpan* span = nullptr);    // scale.go:54-79
  Status scale_down(ScaleSpan* span = nullptr);  // scale.go:81-107

  // Pipelined read (optimisation, decisions unchanged): prefetch() starts the Deployment GET
  // before the SQS poll so the two round trips overlap; the next scale_up/scale_down consumes
  // it instead of issuing its own GET. If the write then fails with 409 (the object changed
  // after the prefetch) the call re-reads and retries once -- exactly the GET-then-write the
  // reference would have done at that point. discard_prefetch() drains an unused prefetch.
  // may_dial: see DeploymentApi::begin_get.
  bool prefetch(bool may_dial = true);
  void discard_prefetch();
  void warm() { api_->warm(); }
  bool prefetch_pending() const { return prefetch_pending_; }

  std::shared_ptr<DeploymentApi> api() const { return api_; }
  void cancel() { api_->cancel(); }
  const std::string& deployment() const { return deployment_; }
  const std::string& namespace_() const { return ns_; }
  int64_t max() const { return max_.load(std::memory_order_relaxed); }
  int64_t min() const { return min_; }
  int64_t scale_up_pods() const { return up_; }
  int64_t scale_down_pods() const { return down_; }
  // Shadow mode (--dry-run): decide and log "Dry run: would scale ...", never write.
  void set_dry_run(bool on) { dry_run_ = on; }
  bool dry_run() const { return dry_run_; }
  // Safe to call from another thread while the loop runs (GPU-capacity refresh).
  void set_max(int64_t m) { max_.store(m, std::memory_order_relaxed); }

 private:
  std::shared_ptr<DeploymentApi> api_;
  std::string deployment_, ns_;
  std::atomic<int64_t> max_;
  int64_t min_, up_, down_;
  std::shared_ptr<Logger> log_;
  std::shared_ptr<Clock> clock_;
  bool prefetch_pending_ = false;
  bool dry_run_ = false;

  Result<ScaleObject> read(ScaleSpan* span, bool* from_prefetch);
  Status scale(bool up, ScaleSpan* span);
};

}  // namespace ksa
