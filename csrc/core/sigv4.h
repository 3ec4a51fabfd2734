// AWS Signature Version 4 and credential caching.
//
// The reference delegates request signing and the credential chain to aws-sdk-go v1.35.35
// (session.NewSession + sqs.New, /root/reference/sqs/sqs.go:36; go.mod:6). Without the SDK
// this module implements the published SigV4 algorithm directly:
//   canonical request -> string to sign -> HMAC-SHA256 chain -> Authorization header.
// The derived signing key only changes once per UTC day (and per secret), so it is cached;
// steady-state signing costs two SHA-256 digests and one HMAC.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "status.h"

namespace ksa {

using Headers = std::vector<std::pair<std::string, std::string>>;

std::string sha256_hex(const std::string& data);
std::string hmac_sha256(const std::string& key, const std::string& data);  // raw bytes
std::string hex_encode(const std::string& raw);

// HMAC-SHA256 with the key schedule precomputed: the SHA-256 states after absorbing
// key^ipad and key^opad are kept, so each MAC costs only the message blocks plus one
// outer block (~0.3 us for a SigV4 string-to-sign) instead of OpenSSL 3's one-shot HMAC()
// (~2.5 us of provider dispatch per call). The SigV4 signing key changes once a day, so the
// signer keeps one of these per (secret, date).
class HmacSha256Key {
 public:
  HmacSha256Key();
  explicit HmacSha256Key(const std::string& key);
  HmacSha256Key(const HmacSha256Key&);
  HmacSha256Key& operator=(const HmacSha256Key&);
  ~HmacSha256Key();
  std::string mac(const std::string& data) const;  // raw 32 bytes
  // The MAC of the concatenation of `parts`, without building it.
  void mac_parts(std::initializer_list<std::string_view> parts, unsigned char out[32]) const;

 private:
  struct State;
  std::unique_ptr<State> st_;
};

// RFC 3986 percent-encoding of everything outside [A-Za-z0-9-_.~]; '/' kept when
// `keep_slash` (canonical URI) -- this equals Go's url.QueryEscape with '+' -> "%20".
std::string aws_uri_encode(const std::string& s, bool keep_slash);
std::string url_decode(const std::string& s, bool plus_is_space);
// Form/query parsing of "a=1&b=2" into decoded pairs (order preserved).
std::vector<std::pair<std::string, std::string>> parse_query(const std::string& q);

struct Credentials {
  std::string access_key_id;
  std::string secret_access_key;
  std::string session_token;
  int64_t expires_unix_ns = 0;  // 0 = does not expire
  std::string provider_name;
  // Set by a provider that handed out a set inside its refresh window because the refresh
  // failed (cred_slot.h): a request signed with it is reported through signed_with_kept().
  bool kept_after_failed_refresh = false;
  bool valid() const { return !access_key_id.empty() && !secret_access_key.empty(); }
};

// A set whose refresh failed is still signed with until this long before its Expiration
// (cred_slot.h, SharedCredentialsProvider): a deliberate deviation from aws-sdk-go, which fails
// the call once its 5-minute window is reached and the refresh fails (README.md).
constexpr int64_t kStaleSkew = 60LL * 1000 * 1000 * 1000;
// While such a set is kept, the refresh is tried again at most this often.
constexpr int64_t kKeptRetry = 10LL * 1000 * 1000 * 1000;

// Credential source (env, shared file, web identity, ECS, IMDS ... live in Python; see
// kube_sqs_autoscaler_amd/sqs/credentials.py). Native code only needs retrieve().
class CredentialsProvider {
 public:
  virtual ~CredentialsProvider() = default;
  virtual Result<Credentials> retrieve() = 0;
  // A client found `c` rejected (ExpiredToken): a provider that caches drops it. Default: none.
  virtual void stale(const Credentials& c) { (void)c; }
  // A request was signed with `c`, a set handed out with kept_after_failed_refresh: a provider
  // that counts those does so here. Default: nothing.
  virtual void signed_with_kept(const Credentials& c) { (void)c; }
  // The client that owns this source stops for good (its API's cancel(), on Runner::stop): a
  // provider that waits for credentials stops waiting. Lock-free: the wait may hold the caller's
  // lock. Default: nothing to interrupt.
  virtual void cancel() {}
};

class StaticCredentialsProvider final : public CredentialsProvider {
 public:
  explicit StaticCredentialsProvider(Credentials c) : c_(std::move(c)) {}
  Result<Credentials> retrieve() override { return Result<Credentials>::Ok(c_); }

 private:
  Credentials c_;
};

// aws.Credentials-style cache: retrieve() again only when the cached value is within
// `expiry_window_ns` of its expiry (or was invalidated after a 403).
class alignas(kCacheLine) CachedCredentials {
 public:
  CachedCredentials(std::shared_ptr<CredentialsProvider> p, int64_t expiry_window_ns)
      : provider_(std::move(p)), window_(expiry_window_ns) {}
  Result<Credentials> get(int64_t unix_now_ns);
  void invalidate();
  void cancel() { provider_->cancel(); }  // lock-free: get() may be waiting in retrieve()
  // The client signed a request with `c` (from get()): counted by the provider when it was kept.
  void signed_with(const Credentials& c) {
    if (c.kept_after_failed_refresh) provider_->signed_with_kept(c);
  }

 private:
  std::shared_ptr<CredentialsProvider> provider_;
  int64_t window_;
  std::mutex mu_;
  bool have_ = false;
  Credentials cached_;
};

// One credential source for every SQS client of a process with the same chain configuration
// (region). Each client's CachedCredentials asks it when its own copy nears expiry; it calls
// `inner` only when its copy does too (or a client reported it stale), so N tracked queues make
// one STS / ECS / IMDS fetch per expiry instead of N -- the reference builds one session per
// process (/root/reference/sqs/sqs.go:36). Callers that arrive while a fetch is in flight wait
// for that fetch and take its outcome, its error included: against a hung or failing endpoint
// the N queues share one timeout rather than queueing N of them behind each other. `unix_now`
// is the clock (wall time). cancel() (one client's Runner::stop) releases the callers waiting
// for a fetch at that moment with "request canceled"; it does not stop the fetch, which the
// other clients still wait for, and later calls wait as before -- the provider is shared.
// A refresh that fails while the cached set has more than kStaleSkew left keeps that set: it is
// handed out (kept_after_failed_refresh) and the refresh retried every kKeptRetry, as the CLI's
// broker does (cred_slot.h).
class SharedCredentialsProvider final : public CredentialsProvider {
 public:
  SharedCredentialsProvider(std::shared_ptr<CredentialsProvider> inner, std::function<int64_t()> unix_now,
                            int64_t expiry_window_ns)
      : inner_(std::move(inner)), now_(std::move(unix_now)), window_(expiry_window_ns) {}
  Result<Credentials> retrieve() override;
  void stale(const Credentials& c) override;
  void cancel() override;
  void signed_with_kept(const Credentials& c) override {
    (void)c;
    stale_signs_.fetch_add(1, std::memory_order_relaxed);
  }
  uint64_t fetches() const {
    std::lock_guard<std::mutex> lk(mu_);
    return fetches_;
  }
  // Requests signed with a set kept after its refresh failed.
  uint64_t stale_signs() const { return stale_signs_.load(std::memory_order_relaxed); }

 private:
  std::shared_ptr<CredentialsProvider> inner_;
  std::function<int64_t()> now_;
  int64_t window_;
  mutable std::mutex mu_;
  std::condition_variable done_;  // a fetch finished (fetched_ moved on)
  bool have_ = false;
  Credentials cached_;
  bool fetching_ = false;
  uint64_t fetched_ = 0;      // fetches finished
  uint64_t cancels_ = 0;      // cancel() calls: a waiter that saw another count returns
  Result<Credentials> last_;  // the outcome of the last one
  uint64_t fetches_ = 0;
  bool kept_ = false;         // cached_ is a set whose refresh failed
  int64_t retry_at_ = 0;      // (unix ns) while kept_: no fetch before this
  std::atomic<uint64_t> stale_signs_{0};
};

struct SignDebug {
  std::string canonical_request;
  std::string string_to_sign;
  std::string signed_headers;
  std::string signature;
  std::string scope;
};

// Signing state precomputed for a request that is re-sent unchanged except for its date (the
// per-queue SQS poll): body hash, canonical URI/query and the canonical form of every fixed
// header are built once, so a poll only hashes the small canonical request and MACs it.
struct SigV4Prepared {
  std::string method, path, raw_query;
  Headers headers;            // fixed headers as sent (Host, Content-Type, ...)
  std::string payload_hash;   // hex SHA-256 of the body
  std::vector<std::pair<std::string, std::string>> canon;  // lower-case name, trimmed value; sorted
  std::string canonical_uri, canonical_query;
  // Credentials without a session token (the common case): the canonical request is
  // creq_prefix + X-Amz-Date + creq_suffix, so a signature hashes those three pieces in place.
  std::string creq_prefix, creq_suffix, signed_headers;
};

class SigV4Signer {
 public:
  SigV4Signer(std::string region, std::string service)
      : region_(std::move(region)), service_(std::move(service)) {}

  // Signs in place: appends X-Amz-Date, X-Amz-Security-Token (session credentials) and
  // Authorization to `headers`. `headers` must already contain Host. `raw_query` is the
  // query string as sent (percent-encoded), `path` the path as sent.
  void sign(const Credentials& creds, int64_t unix_ns, const std::string& method,
            const std::string& path, const std::string& raw_query, Headers* headers,
            const std::string& body, SignDebug* debug = nullptr);

  SigV4Prepared prepare(const std::string& method, const std::string& path, const std::string& raw_query,
                        const Headers& headers, const std::string& body) const;
  // Same result as sign() on (prepared headers, body), without re-deriving the fixed parts.
  void sign_prepared(const SigV4Prepared& p, const Credentials& creds, int64_t unix_ns, Headers* out,
                     SignDebug* debug = nullptr);

  // Derived key for (secret, yyyymmdd); cached per day.
  std::string signing_key(const std::string& secret, const std::string& date);
  // HMAC schedule of that key (what sign() uses).
  HmacSha256Key signing_mac(const std::string& secret, const std::string& date);
  // MAC with that key of the concatenation of `parts` (no key or schedule copied).
  void mac_with_signing_key(const std::string& secret, const std::string& date,
                            std::initializer_list<std::string_view> parts, unsigned char out[32]);

  const std::string& region() const { return region_; }
  const std::string& service() const { return service_; }

 private:
  std::string region_, service_;
  std::mutex mu_;
  std::string key_secret_, key_date_, key_;
  HmacSha256Key key_mac_;
};

// Builds the canonical request pieces; shared with the fake server's verifier.
struct CanonicalParts {
  std::string canonical_request;
  std::string signed_headers;
};
CanonicalParts sigv4_canonical(const std::string& method, const std::string& path,
                               const std::string& raw_query, const Headers& headers,
                               const std::vector<std::string>* only_headers,
                               const std::string& payload_hash);

// Server-side verification of an incoming request's Authorization header.
Status sigv4_verify(const std::string& method, const std::string& path,
                    const std::string& raw_query, const Headers& headers,
                    const std::string& body, const std::string& expected_access_key,
                    const std::string& secret, const std::string& region,
                    const std::string& service);

}  // namespace ksa
