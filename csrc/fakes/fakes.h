// Localhost fake endpoints for end-to-end tests and the latency benchmark.
//
// The reference's tests never leave the process (MockSQS, client-go's fake clientset;
// /root/reference/main_test.go:241-304). To exercise the real wire path -- SigV4, the Query
// and JSON protocols, keep-alive, TLS, resourceVersion conflicts, 5xx handling -- these
// servers speak the actual HTTP APIs:
//   * FakeSqsServer  -- POST / GetQueueAttributes (Query form or AWS JSON 1.0), verifies the
//                       SigV4 signature by recomputation when credentials are configured.
//   * FakeKubeServer -- apps/v1 Deployment GET/PUT and the autoscaling/v1 /scale subresource
//                       GET/PUT/PATCH, bearer-token auth, resourceVersion optimistic
//                       concurrency, realistic (~3 KB) Deployment bodies.
// Both support injected failures and per-request latency.
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "http_server.h"
#include "../core/sqs.h"

namespace ksa {

struct InjectedFault {
  int status = 500;
  std::string body;
  std::string content_type = "text/plain";
  bool drop_connection = false;  // close the socket without responding
  std::string retry_after;       // Retry-After header value ("" = none)
  std::string method;            // only requests with this method ("" = any)
};

class FakeSqsServer {
 public:
  FakeSqsServer();
  ~FakeSqsServer();
  // Requires valid SigV4 signatures for (access_key, secret, region).
  void require_signature(std::string access_key, std::string secret, std::string region);
  // CPUs for the server's threads (call before start(); the benchmark keeps a queue's fake
  // endpoints in its worker's L3 domain).
  void set_cpus(std::vector<int> cpus) { cpus_ = std::move(cpus); }
  // HttpServer::set_hot: one busy-polling thread serves every connection (call before start()).
  void set_hot(bool on) { hot_ = on; }
  // HttpServer::set_timing: record timings() (off by default; any time).
  void set_timing(bool on) {
    timing_ = on;
    if (server_) server_->set_timing(on);
  }
  Status start(const std::string& host = "127.0.0.1", int port = 0, bool tls = false);
  void stop();
  int port() const;
  std::string url() const;
  std::string cert_pem() const { return cert_pem_; }

  void set_attributes(const std::string& queue_url, AttrMap attrs);
  void set_default_attributes(AttrMap attrs);  // for queues not set explicitly
  // Successive GetQueueAttributes calls for `queue_url` return cycle[0], cycle[1], ... and wrap
  // around (a step trace driven by call count; the latency benchmark's 200 <-> 0 trace).
  void set_attribute_cycle(const std::string& queue_url, std::vector<AttrMap> cycle);
  void inject(int count, InjectedFault fault);
  void set_latency(Nanos per_request);
  void drop_connections();

  uint64_t requests() const { return requests_.load(); }
  uint64_t signature_failures() const { return sig_failures_.load(); }
  uint64_t connections() const;
  size_t connection_threads() const { return server_ ? server_->connection_threads() : 0; }
  // HttpServer::timings(): per request, the server's wake-up delay and service time.
  std::vector<HttpServer::ServeTiming> timings() const { return server_ ? server_->timings() : std::vector<HttpServer::ServeTiming>{}; }
  void clear_timings() { if (server_) server_->clear_timings(); }
  std::string last_body() const;
  Headers last_headers() const;

 private:
  void handle(const HttpRequest& req, HttpResponse* resp);

  std::unique_ptr<HttpServer> server_;
  std::vector<int> cpus_;
  bool hot_ = false;
  bool timing_ = false;
  StopFlag shutdown_;  // stop() cuts injected-latency sleeps short
  bool tls_ = false;
  std::string cert_pem_, key_pem_;
  mutable std::mutex mu_;
  // Attribute maps are immutable once stored, so a request takes a reference under the lock
  // and reads the map after releasing it.
  using AttrsPtr = std::shared_ptr<const AttrMap>;
  std::map<std::string, AttrsPtr> queues_;
  struct Cycle {
    std::vector<AttrsPtr> maps;
    size_t next = 0;
  };
  std::map<std::string, Cycle> cycles_;
  AttrsPtr default_attrs_;
  bool verify_ = false;
  std::string akid_, secret_, region_;
  std::vector<InjectedFault> faults_;
  Nanos latency_ = 0;
  std::string last_body_;
  Headers last_headers_;
  std::atomic<uint64_t> requests_{0};
  std::atomic<uint64_t> sig_failures_{0};
};

class FakeKubeServer {
 public:
  FakeKubeServer();
  ~FakeKubeServer();
  void require_token(std::string token);
  void set_cpus(std::vector<int> cpus) { cpus_ = std::move(cpus); }
  void set_hot(bool on) { hot_ = on; }
  // HttpServer::set_timing: record timings() (off by default; any time).
  void set_timing(bool on) {
    timing_ = on;
    if (server_) server_->set_timing(on);
  }
  Status start(const std::string& host = "127.0.0.1", int port = 0, bool tls = false);
  void stop();
  int port() const;
  std::string url() const;
  std::string cert_pem() const { return cert_pem_; }

  void add_deployment(const std::string& ns, const std::string& name, int32_t replicas);
  int32_t replicas(const std::string& ns, const std::string& name) const;  // -1 if absent
  void set_replicas(const std::string& ns, const std::string& name, int32_t replicas);
  std::string deployment_json(const std::string& ns, const std::string& name) const;
  void inject(int count, InjectedFault fault);
  // The next n GETs are followed by a concurrent write (resourceVersion bump) -> next PUT 409s.
  void conflict_next(int n);
  void set_latency(Nanos per_request);
  void drop_connections();
  // RBAC of the caller on Deployments: "resource:verb" rules, e.g. {"deployments:get",
  // "deployments:update"} (a Role written for the reference) or "deployments/scale:patch";
  // "*" allows everything (the default). A request outside them gets the apiserver's 403.
  void set_rbac(std::vector<std::string> rules);
  uint64_t forbidden() const { return forbidden_.load(); }

  // coordination.k8s.io/v1 Leases (leader election): raw JSON objects with resourceVersion
  // optimistic concurrency; POST creates (409 AlreadyExists), PUT replaces (409 Conflict).
  std::string lease_json(const std::string& ns, const std::string& name) const;  // "" if absent
  // core/v1 Nodes for GPU-capacity discovery: GET /api/v1/nodes[?labelSelector=k=v,k2=v2]
  // (equality selectors) returns a NodeList with status.allocatable[resource] = gpus.
  void add_node(const std::string& name, const std::map<std::string, std::string>& labels,
                const std::string& resource, int64_t gpus, bool unschedulable = false);

  uint64_t requests() const { return requests_.load(); }
  uint64_t gets() const { return gets_.load(); }
  uint64_t writes() const { return writes_.load(); }
  uint64_t conflicts() const { return conflicts_.load(); }
  uint64_t auth_failures() const { return auth_failures_.load(); }
  uint64_t connections() const;
  std::vector<HttpServer::ServeTiming> timings() const { return server_ ? server_->timings() : std::vector<HttpServer::ServeTiming>{}; }
  void clear_timings() { if (server_) server_->clear_timings(); }
  std::string last_method() const;
  std::string last_body() const;
  std::string last_path() const;

 private:
  struct Obj {
    int32_t replicas = 1;
    uint64_t rv = 1;
    int64_t generation = 1;
  };
  void handle(const HttpRequest& req, HttpResponse* resp);
  std::string render_deployment(const std::string& ns, const std::string& name, const Obj& o) const;
  std::string render_scale(const std::string& ns, const std::string& name, const Obj& o) const;
  static std::string status_json(int code, const std::string& reason, const std::string& message);

  std::unique_ptr<HttpServer> server_;
  std::vector<int> cpus_;
  bool hot_ = false;
  bool timing_ = false;
  StopFlag shutdown_;  // stop() cuts injected-latency sleeps short
  bool tls_ = false;
  std::string cert_pem_, key_pem_;
  mutable std::mutex mu_;
  std::map<std::string, Obj> objs_;  // key: ns + "/" + name
  struct Lease {
    std::string json;
    uint64_t rv = 0;
  };
  std::map<std::string, Lease> leases_;  // key: ns + "/" + name
  struct Node {
    std::map<std::string, std::string> labels;
    std::string resource;
    int64_t gpus = 0;
    bool unschedulable = false;
  };
  std::map<std::string, Node> nodes_;
  void handle_nodes(const std::string& query, HttpResponse* resp);
  void handle_lease(const HttpRequest& req, const std::vector<std::string>& parts, HttpResponse* resp);
  std::string token_;
  std::vector<std::string> rbac_{"*"};
  std::vector<InjectedFault> faults_;
  int conflict_ = 0;
  Nanos latency_ = 0;
  uint64_t rv_counter_ = 5000;
  std::string last_method_, last_body_, last_path_;
  std::atomic<uint64_t> requests_{0}, gets_{0}, writes_{0}, conflicts_{0}, auth_failures_{0}, forbidden_{0};
};

}  // namespace ksa
