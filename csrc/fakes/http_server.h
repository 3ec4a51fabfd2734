// HTTP/1.1 server for the localhost fake endpoints (csrc/fakes): tests and the latency benchmark
// only. Built into the _ksa_fakes module and the native test binaries, never into _ksa_native.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../core/http.h"

namespace ksa {

// Threaded HTTP/1.1 server (accept thread + one thread per connection). Used by the fake
// SQS / kube-apiserver endpoints in tests and benchmarks; blocking reads give the lowest
// wake-up latency for a handful of persistent connections.
class HttpServer {
 public:
  using Handler = std::function<void(const HttpRequest&, HttpResponse*)>;
  explicit HttpServer(Handler h);
  ~HttpServer();
  // TLS: PEM certificate chain + key; call before listen().
  Status enable_tls(const std::string& cert_pem, const std::string& key_pem);
  Status listen(const std::string& host, int port);
  int port() const { return port_; }
  void stop();
  uint64_t requests_served() const { return served_.load(); }
  uint64_t connections_accepted() const { return accepted_.load(); }
  // Connection threads not yet joined (running, or finished and reaped on the next accept).
  size_t connection_threads() const {
    std::lock_guard<std::mutex> lk(mu_);
    return workers_.size();
  }
  // Close every open client connection after its in-flight response (idle-close test).
  void drop_connections();
  // CPUs for the acceptor and connection threads (call before listen(); empty: unpinned).
  void set_cpus(std::vector<int> cpus) { cpus_ = std::move(cpus); }
  // Per request served (the latest 64K) while set_timing(true): the wake-up delay -- the
  // kernel's receive timestamp of the request's first segment (SO_TIMESTAMPNS) to the
  // connection thread running -- and the service time, from then to the response written. A
  // benchmark subtracts the first from a client's round trip: it is what a fake endpoint idle
  // between polls adds by sleeping, which a production endpoint does not. Off by default: the
  // receive timestamp costs a poll(2) and a peeking recvmsg(2) per request on the endpoint's
  // side of every round trip (any time; applies from each connection's next request).
  void set_timing(bool on) { timing_.store(on, std::memory_order_relaxed); }
  struct ServeTiming {
    int64_t wake_ns;
    int64_t service_ns;
  };
  std::vector<ServeTiming> timings() const;
  void clear_timings();
  // Hot mode (call before listen()): one thread serves every connection from a busy-polled
  // epoll set and never sleeps -- a model of a loaded production endpoint (AWS, a busy
  // apiserver), which is awake when a request arrives. The default thread-per-connection
  // server sleeps between requests, so a client polling every second pays the endpoint's
  // wake-up from a deep idle state on top of its own round trip. Costs one CPU per server.
  void set_hot(bool on) { hot_ = on; }

 private:
  void accept_loop();
  void serve(int fd);
  void hot_loop();
  bool hot_ = false;

  Handler handler_;
  SSL_CTX* ctx_ = nullptr;
  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> stopping_{false};
  std::thread acceptor_;
  mutable std::mutex mu_;
  std::vector<int> open_fds_;
  // Connection threads; finished ones are joined on the next accept, so a long-lived fake
  // serving many short connections does not accumulate dead threads (and their stacks).
  struct Worker {
    std::thread thread;
    std::shared_ptr<std::atomic<bool>> done;
  };
  std::vector<Worker> workers_;
  std::atomic<uint64_t> served_{0};
  std::atomic<uint64_t> accepted_{0};
  std::vector<int> cpus_;
  std::atomic<bool> timing_{false};
  mutable std::mutex timing_mu_;
  std::vector<ServeTiming> timings_;
  size_t timing_pos_ = 0;
  void record_timing(ServeTiming t);
};

// Self-signed certificate for `host` (DNS name or IP literal) -- fakes only.
Status generate_self_signed(const std::string& host, std::string* cert_pem,
                            std::string* key_pem);

}  // namespace ksa
