// Queue-depth source: SQS GetQueueAttributes + attribute summing.
//
// Mirrors the reference's two-level design (/root/reference/sqs/sqs.go):
//   * SqsApi       -- the injectable service seam (the reference's `SQS` interface,
//                     sqs.go:14-18); HttpSqsApi is the real client (Query or JSON protocol,
//                     SigV4-signed, SDK-style retries); the fakes MockSqsApi/TraceSqsApi
//                     live in csrc/fakes/mem_fakes.h (test builds only).
//   * SqsClient    -- NumMessages(): request the configured attribute names and sum their
//                     strconv.Atoi values (sqs.go:45-67), with the reference's error texts.
// Deliberate deviation: a requested attribute that is absent from the
// response is an error, not a nil-pointer panic (sqs.go:58).
#pragma once

#include <functional>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "clock.h"
#include "http.h"
#include "sigv4.h"
#include "status.h"

namespace ksa {

using AttrMap = std::map<std::string, std::string>;

// sqs.go:26-33
const std::vector<std::string>& default_attribute_names();

// DNS suffix of the AWS partition `region` belongs to (aws-sdk-go v1 endpoints model):
// amazonaws.com, amazonaws.com.cn, c2s.ic.gov or sc2s.sgov.gov.
std::string aws_dns_suffix(const std::string& region);

class SqsApi {
 public:
  virtual ~SqsApi() = default;
  virtual Result<AttrMap> get_queue_attributes(const std::string& queue_url,
                                               const std::vector<std::string>& names) = 0;
  // Shutdown: abort the call in progress and any retry back-off (sticky). Default: nothing.
  virtual void cancel() {}
  // Closes the keep-alive connection(s); the next call dials again. Called by the thread that
  // owns the client (Supervisor: before and after a worker runs on a private file table).
  virtual void close_connections() {}
  // Clock time at which the latest deliberate wait (retry back-off, Retry-After) ends or ended;
  // 0: none yet. The liveness check counts such a wait as progress.
  virtual Nanos waiting_until() const { return 0; }
  // True when a call writes an HTTP request through HttpClient, so work handed to set_on_wire
  // (http.h) runs while the call is in flight.
  virtual bool runs_on_wire_work() const { return false; }
  // The last call's time breakdown as a JSON object ("" when not timed): set_timing below.
  virtual std::string timing_json() const { return ""; }
  // HttpClient::set_spin_budget of the client's connection. Default: nothing.
  virtual void set_spin_budget(Nanos ns) { (void)ns; }
  // The endpoint's response-time EWMA (HttpClient::rtt_ewma); -1: unknown (no sample, or not HTTP).
  virtual Nanos response_ewma() const { return -1; }
  // Pre-poll warm-up (Runner prewarm), just before a call due at unix time `at_unix_ns`: do
  // now what the call would otherwise do first -- credentials, the request and its signature
  // for that second, the connection check or dial -- and, with `presend`, hand all but the
  // request's last bytes to the kernel corked (HttpClient::stage): nothing reaches the wire
  // before the call. Default: nothing.
  virtual void warm(const std::string& queue_url, const std::vector<std::string>& names, int64_t at_unix_ns,
                    bool presend = false) {
    (void)queue_url;
    (void)names;
    (void)at_unix_ns;
    (void)presend;
  }
};

enum class SqsProtocol { Query, Json };

struct SqsHttpOptions {
  std::string region;
  std::string endpoint;  // override (e.g. http://127.0.0.1:9324); empty = regional endpoint
  SqsProtocol protocol = SqsProtocol::Query;
  Nanos timeout = 30 * kSecond;
  Nanos busy_poll = 0;  // HttpClient::set_busy_poll
  int max_retries = 3;  // aws-sdk-go v1 DefaultRetryer.NumMaxRetries
  Nanos min_retry_delay = 30 * kMillisecond;
  Nanos min_throttle_delay = 500 * kMillisecond;
  Nanos max_retry_delay = 300 * kSecond;
  TlsOptions tls;
  std::string proxy;    // HttpClient::set_proxy ("" = direct)
};

struct SqsApiStats {
  uint64_t calls = 0;
  uint64_t retries = 0;
  uint64_t throttle_retries = 0;  // retries with the throttle back-off (429/502/503/504, throttle codes)
  uint64_t errors = 0;
  HttpClientStats http;
};

class alignas(kCacheLine) HttpSqsApi final : public SqsApi {
 public:
  HttpSqsApi(SqsHttpOptions opts, std::shared_ptr<CredentialsProvider> creds,
             std::shared_ptr<Clock> clock);
  Result<AttrMap> get_queue_attributes(const std::string& queue_url,
                                       const std::vector<std::string>& names) override;
  SqsApiStats stats() const;
  void cancel() override;
  void close_connections() override {
    if (http_) http_->close();
  }
  // Regional endpoint aws-sdk-go would resolve for `region` ("" if region is empty).
  static std::string endpoint_for_region(const std::string& region);
  static std::string signing_region(const std::string& region);
  std::string endpoint() const { return endpoint_; }
  Nanos waiting_until() const override { return wait_until_.load(std::memory_order_acquire); }
  bool runs_on_wire_work() const override { return true; }
  void warm(const std::string& queue_url, const std::vector<std::string>& names, int64_t at_unix_ns,
            bool presend = false) override;
  void set_spin_budget(Nanos ns) override {
    if (http_) http_->set_spin_budget(ns);
  }
  Nanos response_ewma() const override { return http_ ? http_->rtt_ewma() : -1; }
  // Diagnostics: time each call -- credentials + signing, the HTTP phases (HttpTiming), the
  // response parse -- for timing_json().
  void set_timing(bool on) {
    if (http_) http_->set_timing(on);
  }
  std::string timing_json() const override;

 private:
  std::atomic<int64_t> sign_ns_{0}, parse_ns_{0};
  std::atomic<Nanos> wait_until_{0};
  // The prepared request for (queue_url, names), signed for the second of `unix_ns` with `c`
  // (cached per second); leaves the signed headers in signed_headers_. Needs prep_mu_.
  void sign_locked(const std::string& queue_url, const std::vector<std::string>& names, const Credentials& c,
                   int64_t unix_ns);
  // *retry_after: the extra initial delay of a throttle answered 429/503 with an integer
  // Retry-After (DefaultRetryer.RetryRules, getRetryAfterDelay); 0 otherwise.
  Result<AttrMap> call_once(const std::string& queue_url, const std::vector<std::string>& names,
                            bool* retryable, bool* throttle, bool* expired, Nanos* retry_after);
  Nanos retry_delay(int retry_count, bool throttle);

  SqsHttpOptions opts_;
  std::shared_ptr<Clock> clock_;
  CachedCredentials creds_;
  SigV4Signer signer_;
  std::string endpoint_;
  Status endpoint_status_;
  Url url_;
  std::unique_ptr<HttpClient> http_;
  // Prepared request for the last (queue, attribute names): the body and every fixed signing
  // input are built once per queue instead of once per poll.
  std::mutex prep_mu_;  // guards the prepared request (an HttpSqsApi may be shared by workers)
  bool prepared_valid_ = false;
  std::string prepared_url_;
  std::vector<std::string> prepared_names_;
  SigV4Prepared prepared_;
  std::string prepared_body_;
  // Signed headers of the prepared request, kept for the second they were signed in: X-Amz-Date
  // has one-second resolution, so within that second (and for the same credentials) the
  // signature is the same bytes and is not recomputed.
  int64_t signed_sec_ = 0;
  bool signed_valid_ = false;
  Credentials signed_creds_;
  Headers signed_headers_;
  mutable std::mutex mu_;
  SqsApiStats stats_;
  uint64_t rng_ = 0x9E3779B97F4A7C15ULL;
  StopFlag cancel_;  // cancel(): interrupts retry back-off sleeps
};

class alignas(kCacheLine) SqsClient {
 public:
  SqsClient(std::shared_ptr<SqsApi> api, std::string queue_url,
            std::vector<std::string> attribute_names);
  // sqs.go:45-67
  Result<int64_t> num_messages();
  const std::string& queue_url() const { return queue_url_; }
  const std::vector<std::string>& attribute_names() const { return names_; }
  std::shared_ptr<SqsApi> api() const { return api_; }
  void cancel() { api_->cancel(); }
  void warm(int64_t at_unix_ns, bool presend = false) { api_->warm(queue_url_, names_, at_unix_ns, presend); }

 private:
  std::shared_ptr<SqsApi> api_;
  std::string queue_url_;
  std::vector<std::string> names_;
};

// Formats an aws-sdk-go awserr.RequestFailure message.
std::string aws_request_failure(const std::string& code, const std::string& message, int status,
                                const std::string& request_id);

}  // namespace ksa
