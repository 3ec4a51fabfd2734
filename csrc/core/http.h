// HTTP/1.1 transport: keep-alive client (plain TCP or TLS). The fakes' server is in
// csrc/fakes/http_server.h (test and benchmark builds only).
//
// The reference's only "communication backend" is two HTTPS request/response APIs: SQS
// GetQueueAttributes (/root/reference/sqs/sqs.go:51) and the kube-apiserver Deployment GET/PUT
// (/root/reference/scale/scale.go:55,72,82,100), made through the AWS SDK's and client-go's
// pooled net/http transports. Poll->patch latency is three sequential round trips, so what
// matters is (a) never paying a TCP/TLS handshake on the hot path (persistent connection per
// endpoint, transparent reconnect when the peer closed an idle socket), (b) TCP_NODELAY so
// small request/response pairs are not held back by Nagle, and (c) no per-request
// allocation churn beyond the body strings. Per-call deadlines are enforced with poll(2);
// the reference has none.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "clock.h"
#include "sigv4.h"  // Headers
#include "status.h"

typedef struct ssl_ctx_st SSL_CTX;
typedef struct ssl_session_st SSL_SESSION;

namespace ksa {

struct Url {
  std::string scheme;  // "http" | "https"
  std::string host;    // without brackets for IPv6
  int port = 0;
  std::string path;    // path + query as it appears on the wire ("/" when empty)
  bool tls() const { return scheme == "https"; }
  std::string host_header() const;  // host[:port], port omitted when default
  std::string origin() const;       // scheme://host[:port]
};
Result<Url> parse_url(const std::string& s);

struct TlsOptions {
  bool insecure_skip_verify = false;
  std::string ca_file;
  std::string ca_pem;
  std::string cert_pem;  // client certificate (mutual TLS, kubeconfig client-certificate-data)
  std::string key_pem;
  std::string server_name;  // SNI / verification name override (kubeconfig tls-server-name)
};

struct HttpRequest {
  std::string method = "GET";
  std::string target = "/";  // origin-form request target (path + query)
  Headers headers;
  std::string body;
  std::string header(const std::string& name) const;  // case-insensitive, first match
};

struct HttpResponse {
  int status = 0;
  std::string reason;
  Headers headers;
  std::string body;
  std::string header(const std::string& name) const;
};

struct HttpClientStats {
  uint64_t requests = 0;
  uint64_t connects = 0;
  uint64_t tls_resumptions = 0;  // reconnects that resumed the previous TLS session
  uint64_t reconnect_retries = 0;
  uint64_t idle_closed = 0;  // reused connections found closed by the peer before a write
  uint64_t presends = 0;     // requests whose staged (pre-sent) prefix was completed
  uint64_t presend_discards = 0;  // staged requests that did not match the next request
  uint64_t bytes_out = 0;
  uint64_t bytes_in = 0;
  std::string tls_version;  // of the last TLS connection ("" before one), e.g. "TLSv1.3"
  std::string tls_cipher;   // its cipher suite, e.g. "TLS_AES_128_GCM_SHA256"
};

// Per-request timing (HttpClient::set_timing: HttpTiming, SO_TIMESTAMPNS receive stamps) is a
// diagnostic for the benchmark's attribution rows. The image build compiles it out
// (-DKSA_HTTP_TIMING=0, `ops.build --image`): set_timing() is then a no-op and timing() false.
#ifndef KSA_HTTP_TIMING
#define KSA_HTTP_TIMING 1
#endif
inline constexpr bool kHttpTiming = KSA_HTTP_TIMING != 0;

// Where one request's time went (HttpClient::set_timing), CLOCK_MONOTONIC ns; 0 = not known.
// rx is the kernel's receive time of the response's first bytes (SO_TIMESTAMPNS; plain sockets
// only), so seen - rx is how long those bytes waited for this thread: its wake-up.
struct HttpTiming {
  int64_t start = 0;        // the request call began
  int64_t write_begin = 0;  // connection ready (peek / dial done), request serialised
  int64_t written = 0;      // request fully written
  int64_t rx = 0;           // kernel receive time of the first response bytes
  int64_t seen = 0;         // this thread read the first response bytes
  int64_t done = 0;         // response fully read
  bool spun = false;        // the first bytes came while busy-polling (no sleep)
};
// {"pre":..,"write":..,"wait":..,"wake":..,"read":..,"spun":..} in ns (empty when not timed).
std::string http_timing_json(const HttpTiming& t);

// One-shot work for the calling thread to run as soon as its next HTTP request is on the wire
// (HttpClient::attempt, after the write and before the wait for the response). The control loop
// sends its pipelined Deployment GET from here: the SQS request goes out first and the GET
// overlaps the SQS round trip, instead of its write delaying the SQS request. Setting replaces
// a pending one; taking it clears it, so a request made by `fn` itself does not run it again.
void set_on_wire(void (*fn)(void*), void* arg);
bool on_wire_pending();
void clear_on_wire();

// One persistent connection to one origin. Thread-safe (requests are serialised), but each
// control-loop worker owns its clients, so there is no contention in practice.
class alignas(kCacheLine) HttpClient {
 public:
  HttpClient(const Url& origin, TlsOptions tls, Nanos timeout);
  ~HttpClient();
  HttpClient(const HttpClient&) = delete;
  HttpClient& operator=(const HttpClient&) = delete;

  // Sends `req` (Host / Content-Length / User-Agent added when absent) and reads the full
  // response. Reuses the connection unless the peer closed it while idle (then dials anew).
  // If a reused connection dies before any response byte arrived, reconnects and retries once
  // -- as Go's transport does, only for a request that never reached the wire or is
  // replayable (GET/HEAD/OPTIONS/TRACE or an Idempotency-Key): a PUT/PATCH/POST that was
  // written is never sent twice.
  Status round_trip(const HttpRequest& req, HttpResponse* resp);
  // The same with this call's own time limit (< 0: the client's timeout; 0: fails at once).
  Status round_trip(const HttpRequest& req, HttpResponse* resp, Nanos timeout);
  // Pipelined use: send() writes the request and returns at once; receive() reads its
  // response. Between the two the caller is free to do other I/O -- the control loop sends the
  // Deployment GET, then makes the SQS call on another connection, so both round trips overlap.
  // One request may be in flight per client. A dead reused connection is replayed once, as in
  // round_trip().
  Status send(const HttpRequest& req);
  Status receive(HttpResponse* resp);
  bool in_flight() const;
  void close();
  // Pre-poll warm-up (Runner prewarm): checks the idle keep-alive connection now -- the
  // idle-close peek the next request would make -- and dials (with TLS) when there is none or
  // the peer closed it, so the request itself finds a live, freshly checked connection. Dial
  // errors are left for the request to report. Returns whether a connection is ready.
  // The dial runs under `dial_budget` -- or twice the last successful dial's time when that is
  // longer, capped by the client's timeout -- not the full request timeout: an endpoint that
  // drops packets must not hold up the poll it prepares (the SQS read comes after the
  // warm-up). After a warm-up dial fails, later warm-ups do not dial again until a request has
  // connected: while an endpoint is down the poll behaves like the reference's sleep-then-poll,
  // each request dialing under its own timeout.
  static constexpr Nanos kWarmDialBudget = 100 * kMillisecond;
  bool warm(Nanos dial_budget = kWarmDialBudget);
  // Pre-send (Runner prewarm, after warm()): hands all but the last few bytes of `req` -- the
  // request the next round_trip() will make -- to the kernel now, corked: nothing goes on the
  // wire until that round_trip() writes the rest (or the kernel's 200 ms cork limit passes --
  // far beyond the warm-up window), so the peer sees the request when it would have, but the
  // kernel's send path has run and the request's final write runs warm.
  // When the next request turns out different, or the connection was replaced meanwhile, the
  // staged connection is closed (its queued bytes cannot be taken back) and the request dials
  // a fresh one. Needs a live connection; returns whether the request was staged.
  bool stage(const HttpRequest& req);
  // Whether a request could go out now without dialing: a connection exists and is either
  // fresh (a response or a check within kFreshConnNs) or passes the idle-close peek. The
  // pipelined GET, sent from inside the SQS call, goes out only then (a dial there would run
  // on the SQS call's deadline).
  bool ready_without_dial();
  // The caller retries a failed request itself (the SQS client's SDK-style retryer): a request
  // that is not replayable may then skip the idle-close peek on a fresh connection. Without it
  // (the apiserver client) a PUT/PATCH is always preceded by the peek, so a connection the
  // peer half-closed is redialled instead of failing the write.
  void set_caller_retries(bool on) { caller_retries_ = on; }
  // Per-request timing breakdown (diagnostics: a benchmark's attribution rows); adds a
  // timestamp read per phase and a recvmsg for the first response bytes. Off by default.
  void set_timing(bool on) { timing_ = kHttpTiming && on; }
  bool timing() const { return kHttpTiming && timing_; }
  HttpTiming last_timing() const;
  // Aborts any request in progress ("request canceled") and every later one: graceful shutdown
  // must not wait for a slow or hung peer (the in-flight call's timeout can be 30 s). Sticky.
  void cancel();
  bool cancelled() const { return cancelled_.load(std::memory_order_acquire); }
  HttpClientStats stats() const;
  const Url& origin() const { return origin_; }
  void set_timeout(Nanos t) { timeout_ = t; }
  // Adaptive busy-poll: while the peer's response-time EWMA is within 4x `ns`, a read spins for
  // up to `ns` before blocking in poll(2) (saves the scheduler wake-up on fast local peers); for
  // slower peers it does not spin, and a peer slower than kMaxSpinThrough (real AWS / apiserver
  // RTTs of milliseconds) is never spun for, whatever the budget. 0 disables.
  void set_busy_poll(Nanos ns) { spin_ns_ = ns; }
  // With busy-poll on, a read may also spin through a near peer's expected response time (twice
  // the EWMA, at most kMaxSpinThrough) when that fits in `ns` per request -- the Runner sets its
  // share of the poll period on a worker's own thread (LoopConfig::spin_budget_ppm, capped by the
  // cgroup CPU quota), so a cadenced poll of a near endpoint is not woken from an idle sleep on
  // its answer. 0 (default): never beyond the window.
  void set_spin_budget(Nanos ns) { spin_budget_ns_ = ns; }
  Nanos rtt_ewma() const;
  // The absolute ceiling of one read's spin. A peer whose EWMA is above it is a network round
  // trip away: spinning would burn CPU for the whole RTT (under a 100m CPU limit -- the
  // reference's manifest, README.md:60-66 -- 10 ms per 100 ms CFS period, a few such spins
  // exhaust the quota and the throttled thread then answers late).
  static constexpr Nanos kMaxSpinThrough = 200 * kMicrosecond;
  // The read spin of the next response: `busy_poll` (the window) while the EWMA is unknown or
  // within 4x the window, else 0; raised to twice the EWMA when the EWMA is within
  // kMaxSpinThrough and that spin (capped at kMaxSpinThrough) fits in `budget`.
  static Nanos spin_window_for(Nanos busy_poll, Nanos ewma, Nanos budget);
  // Forward proxy (Go's http.ProxyFromEnvironment; the proxy is chosen by the caller), the
  // three kinds Go's transport speaks:
  //   "http://[user:pass@]host:port"   an https origin is reached through a CONNECT tunnel (TLS
  //                                    runs end to end inside it); an http origin gets
  //                                    absolute-form requests. Credentials become
  //                                    Proxy-Authorization: Basic.
  //   "https://[user:pass@]host:port"  the same, over TLS to the proxy (verified against the
  //                                    client's trust settings and the proxy's host name, as
  //                                    Go's transport does); an https origin then runs TLS
  //                                    inside that TLS.
  //   "socks5://[user:pass@]host:port" a SOCKS5 CONNECT (RFC 1928; user/password auth per
  //                                    RFC 1929) with the origin's host name resolved by the
  //                                    proxy; requests then go out as on a direct connection.
  // Empty = connect directly. Call before the first request.
  Status set_proxy(const std::string& proxy_url);
  bool proxied() const {
    std::lock_guard<std::mutex> lk(mu_);
    return has_proxy_;
  }

 private:
  struct Conn;
  Status connect_locked(int64_t deadline_ns);
  Status dial(const Url& to, int64_t deadline_ns, int* fd_out);
  Status attempt(const HttpRequest& req, HttpResponse* resp, int64_t deadline_ns,
                 bool* retryable);
  Status write_request(const HttpRequest& req, int64_t deadline_ns, bool* retryable);
  Status read_response(const HttpRequest& req, HttpResponse* resp, int64_t deadline_ns,
                       bool* retryable);

  Url origin_;
  TlsOptions tls_;
  Nanos timeout_;
  SSL_CTX* ctx_ = nullptr;
  Status ctx_status_;
  mutable std::mutex mu_;
  std::unique_ptr<Conn> conn_;
  HttpClientStats stats_;
  SSL_SESSION* session_ = nullptr;  // last resumable TLS session
  Nanos spin_ns_ = 0;
  std::atomic<Nanos> spin_budget_ns_{0};
  Nanos ewma_ns_ = -1;   // response-time EWMA (-1: no sample yet)
  int64_t sent_at_ = 0;  // mono time the current request finished writing
  Nanos spin_window() const;
  Status init_tls_ctx();
  bool forward_proxy() const { return has_proxy_ && proxy_kind_ != ProxyKind::Socks5; }
  enum class ProxyKind { Http, Https, Socks5 };
  bool has_proxy_ = false;
  ProxyKind proxy_kind_ = ProxyKind::Http;
  Url proxy_;
  std::string proxy_user_, proxy_pass_;  // socks5 credentials
  std::string proxy_auth_;  // "Basic ..." or empty
  bool in_flight_ = false;
  bool caller_retries_ = false;
  bool warm_dial_failed_ = false;  // warm(): the last warm-up dial failed, none since connected
  uint64_t conn_gen_ = 0;          // connections made so far (identifies conn_ across resets)
  std::string staged_;             // stage(): the staged request's wire bytes ("" = none)
  size_t staged_sent_ = 0;         // how many of them are queued in the kernel, corked
  uint64_t staged_gen_ = 0;        // the connection they are queued on
  void serialize_locked(const HttpRequest& req, std::string* wire) const;
  Nanos last_dial_ns_ = 0;          // how long the last successful dial (TCP + proxy + TLS) took
  bool timing_ = false;
  HttpTiming timing_cur_, timing_last_;
  bool fresh_locked() const;
  int cancel_fd_ = -1;  // eventfd signalled by cancel(); polled next to the socket
  std::atomic<bool> cancelled_{false};
  HttpRequest pending_;
  int64_t pending_deadline_ = 0;
  std::string wire_;  // request serialisation buffer (write_request)
  std::string head_;  // response head buffer (read_response)
};

const char* http_reason(int status);

}  // namespace ksa
