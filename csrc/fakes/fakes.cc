#include "fakes.h"

#include <algorithm>
#include <thread>

#include "../core/json.h"
#include "../core/sigv4.h"
#include "../core/xml.h"

namespace ksa {

namespace {

// The first queued fault for a request with `method` (a fault may name one).
bool pop_fault(std::vector<InjectedFault>* faults, const std::string& method, InjectedFault* out) {
  for (auto it = faults->begin(); it != faults->end(); ++it) {
    if (!it->method.empty() && it->method != method) continue;
    *out = std::move(*it);
    faults->erase(it);
    return true;
  }
  return false;
}

void apply_fault(const InjectedFault& f, HttpResponse* resp) {
  if (f.drop_connection) {
    resp->status = -1;
    return;
  }
  resp->status = f.status;
  resp->body = f.body;
  resp->headers.emplace_back("Content-Type", f.content_type);
  if (!f.retry_after.empty()) resp->headers.emplace_back("Retry-After", f.retry_after);
}

std::string split_path_query(const std::string& target, std::string* query) {
  size_t q = target.find('?');
  if (q == std::string::npos) {
    query->clear();
    return target;
  }
  *query = target.substr(q + 1);
  return target.substr(0, q);
}

}  // namespace

// ---------------------------------------------------------------------------------------
// FakeSqsServer

FakeSqsServer::FakeSqsServer() = default;
FakeSqsServer::~FakeSqsServer() { stop(); }

void FakeSqsServer::require_signature(std::string access_key, std::string secret, std::string region) {
  std::lock_guard<std::mutex> lk(mu_);
  verify_ = true;
  akid_ = std::move(access_key);
  secret_ = std::move(secret);
  region_ = std::move(region);
}

Status FakeSqsServer::start(const std::string& host, int port, bool tls) {
  server_ = std::make_unique<HttpServer>([this](const HttpRequest& q, HttpResponse* r) { handle(q, r); });
  server_->set_cpus(cpus_);
  server_->set_hot(hot_);
  server_->set_timing(timing_);
  tls_ = tls;
  if (tls) {
    Status s = generate_self_signed(host, &cert_pem_, &key_pem_);
    if (!s.ok()) return s;
    s = server_->enable_tls(cert_pem_, key_pem_);
    if (!s.ok()) return s;
  }
  return server_->listen(host, port);
}

void FakeSqsServer::stop() {
  shutdown_.request_stop();
  if (server_) server_->stop();
}

int FakeSqsServer::port() const { return server_ ? server_->port() : 0; }
std::string FakeSqsServer::url() const {
  return std::string(tls_ ? "https" : "http") + "://127.0.0.1:" + std::to_string(port());
}
uint64_t FakeSqsServer::connections() const { return server_ ? server_->connections_accepted() : 0; }
void FakeSqsServer::drop_connections() {
  if (server_) server_->drop_connections();
}

void FakeSqsServer::set_attributes(const std::string& queue_url, AttrMap attrs) {
  auto p = std::make_shared<const AttrMap>(std::move(attrs));
  std::lock_guard<std::mutex> lk(mu_);
  queues_[queue_url] = std::move(p);
}

void FakeSqsServer::set_attribute_cycle(const std::string& queue_url, std::vector<AttrMap> cycle) {
  Cycle c;
  for (auto& m : cycle) c.maps.push_back(std::make_shared<const AttrMap>(std::move(m)));
  std::lock_guard<std::mutex> lk(mu_);
  if (c.maps.empty()) {
    cycles_.erase(queue_url);
    return;
  }
  cycles_[queue_url] = std::move(c);
}

void FakeSqsServer::set_default_attributes(AttrMap attrs) {
  auto p = attrs.empty() ? nullptr : std::make_shared<const AttrMap>(std::move(attrs));
  std::lock_guard<std::mutex> lk(mu_);
  default_attrs_ = std::move(p);
}

void FakeSqsServer::inject(int count, InjectedFault fault) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int i = 0; i < count; ++i) faults_.push_back(fault);
}

void FakeSqsServer::set_latency(Nanos per_request) {
  std::lock_guard<std::mutex> lk(mu_);
  latency_ = per_request;
}

std::string FakeSqsServer::last_body() const {
  std::lock_guard<std::mutex> lk(mu_);
  return last_body_;
}

Headers FakeSqsServer::last_headers() const {
  std::lock_guard<std::mutex> lk(mu_);
  return last_headers_;
}

void FakeSqsServer::handle(const HttpRequest& req, HttpResponse* resp) {
  requests_++;
  std::string query;
  const std::string path = split_path_query(req.target, &query);
  const bool json = !req.header("X-Amz-Target").empty();
  Nanos latency;
  InjectedFault fault;
  bool faulted;
  bool verify;
  std::string akid, secret, region;
  // Copy outside the lock and swap inside it (the old values are freed after unlocking), so
  // concurrent connections hold the shared mutex only for pointer swaps.
  std::string body_copy = req.body;
  auto headers_copy = req.headers;
  {
    std::lock_guard<std::mutex> lk(mu_);
    last_body_.swap(body_copy);
    last_headers_.swap(headers_copy);
    latency = latency_;
    faulted = pop_fault(&faults_, req.method, &fault);
    verify = verify_;
    akid = akid_;
    secret = secret_;
    region = region_;
  }
  if (latency > 0) shutdown_.wait_for(latency);
  if (faulted) {
    apply_fault(fault, resp);
    return;
  }
  auto error = [&](int status, const std::string& code, const std::string& message) {
    resp->status = status;
    resp->headers.emplace_back("x-amzn-RequestId", "fake-request-id");
    if (json) {
      resp->headers.emplace_back("Content-Type", "application/x-amz-json-1.0");
      resp->headers.emplace_back("x-amzn-query-error", code + ";Sender");
      resp->body = "{\"__type\":\"com.amazonaws.sqs#" + code + "\",\"message\":" + json_quote(message) + "}";
    } else {
      resp->headers.emplace_back("Content-Type", "text/xml");
      resp->body = "<?xml version=\"1.0\"?><ErrorResponse xmlns=\"http://queue.amazonaws.com/doc/2012-11-05/\">"
                   "<Error><Type>Sender</Type><Code>" + xml_escape(code) + "</Code><Message>" +
                   xml_escape(message) + "</Message><Detail/></Error><RequestId>fake-request-id</RequestId></ErrorResponse>";
    }
  };
  if (req.method != "POST" && req.method != "GET") {
    error(405, "UnsupportedOperation", "method not allowed");
    return;
  }
  if (verify) {
    Status s = sigv4_verify(req.method, path, query, req.headers, req.body, akid, secret, region, "sqs");
    if (!s.ok()) {
      sig_failures_++;
      std::string code = s.message().substr(0, s.message().find(':'));
      error(403, code, "The request signature we calculated does not match the signature you provided. (" + s.message() + ")");
      return;
    }
  }
  std::string queue_url;
  std::vector<std::string> names;
  if (json) {
    if (req.header("X-Amz-Target") != "AmazonSQS.GetQueueAttributes") {
      error(400, "InvalidAction", "unsupported target " + req.header("X-Amz-Target"));
      return;
    }
    auto j = json_parse(req.body);
    if (!j.ok()) {
      error(400, "MalformedQueryString", "bad JSON body");
      return;
    }
    const JsonValue* q = j.value.get("QueueUrl");
    queue_url = q ? q->string_or("") : "";
    const JsonValue* an = j.value.get("AttributeNames");
    if (an && an->type == JsonValue::Type::Array)
      for (auto& v : an->arr) names.push_back(v.string_or(""));
  } else {
    auto params = parse_query(req.method == "GET" ? query : req.body);
    std::string action;
    std::map<int, std::string> ordered;
    for (auto& [k, v] : params) {
      if (k == "Action") action = v;
      else if (k == "QueueUrl") queue_url = v;
      else if (k.rfind("AttributeName.", 0) == 0) ordered[std::atoi(k.c_str() + 14)] = v;
    }
    if (action != "GetQueueAttributes") {
      error(400, "InvalidAction", "The action " + action + " is not valid for this endpoint.");
      return;
    }
    for (auto& kv : ordered) names.push_back(kv.second);
  }
  AttrsPtr attrs;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto cy = cycles_.find(queue_url);
    auto it = queues_.find(queue_url);
    if (cy != cycles_.end()) {
      attrs = cy->second.maps[cy->second.next];
      cy->second.next = (cy->second.next + 1) % cy->second.maps.size();
    } else if (it != queues_.end()) attrs = it->second;
    else attrs = default_attrs_;
  }
  if (!attrs) {
    error(400, "AWS.SimpleQueueService.NonExistentQueue", "The specified queue does not exist for this wsdl version.");
    return;
  }
  AttrMap out;
  bool all = std::find(names.begin(), names.end(), "All") != names.end();
  for (auto& [k, v] : *attrs)
    if (all || std::find(names.begin(), names.end(), k) != names.end()) out[k] = v;
  resp->status = 200;
  resp->headers.emplace_back("x-amzn-RequestId", "fake-request-id");
  if (json) {
    resp->headers.emplace_back("Content-Type", "application/x-amz-json-1.0");
    JsonValue a = JsonValue::make_object();
    for (auto& [k, v] : out) a.set(k, JsonValue::make_string(v));
    JsonValue root = JsonValue::make_object();
    root.set("Attributes", std::move(a));
    resp->body = json_serialize(root);
  } else {
    resp->headers.emplace_back("Content-Type", "text/xml");
    std::string b = "<?xml version=\"1.0\"?><GetQueueAttributesResponse xmlns=\"http://queue.amazonaws.com/doc/2012-11-05/\"><GetQueueAttributesResult>";
    for (auto& [k, v] : out)
      b += "<Attribute><Name>" + xml_escape(k) + "</Name><Value>" + xml_escape(v) + "</Value></Attribute>";
    b += "</GetQueueAttributesResult><ResponseMetadata><RequestId>fake-request-id</RequestId></ResponseMetadata></GetQueueAttributesResponse>";
    resp->body = std::move(b);
  }
}

// ---------------------------------------------------------------------------------------
// FakeKubeServer

FakeKubeServer::FakeKubeServer() = default;
FakeKubeServer::~FakeKubeServer() { stop(); }

void FakeKubeServer::require_token(std::string token) {
  std::lock_guard<std::mutex> lk(mu_);
  token_ = std::move(token);
}

Status FakeKubeServer::start(const std::string& host, int port, bool tls) {
  server_ = std::make_unique<HttpServer>([this](const HttpRequest& q, HttpResponse* r) { handle(q, r); });
  server_->set_cpus(cpus_);
  server_->set_hot(hot_);
  server_->set_timing(timing_);
  tls_ = tls;
  if (tls) {
    Status s = generate_self_signed(host, &cert_pem_, &key_pem_);
    if (!s.ok()) return s;
    s = server_->enable_tls(cert_pem_, key_pem_);
    if (!s.ok()) return s;
  }
  return server_->listen(host, port);
}

void FakeKubeServer::stop() {
  shutdown_.request_stop();
  if (server_) server_->stop();
}

int FakeKubeServer::port() const { return server_ ? server_->port() : 0; }
std::string FakeKubeServer::url() const {
  return std::string(tls_ ? "https" : "http") + "://127.0.0.1:" + std::to_string(port());
}
uint64_t FakeKubeServer::connections() const { return server_ ? server_->connections_accepted() : 0; }
void FakeKubeServer::drop_connections() {
  if (server_) server_->drop_connections();
}

void FakeKubeServer::add_deployment(const std::string& ns, const std::string& name, int32_t replicas) {
  std::lock_guard<std::mutex> lk(mu_);
  Obj o;
  o.replicas = replicas;
  o.rv = ++rv_counter_;
  objs_[ns + "/" + name] = o;
}

int32_t FakeKubeServer::replicas(const std::string& ns, const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = objs_.find(ns + "/" + name);
  return it == objs_.end() ? -1 : it->second.replicas;
}

void FakeKubeServer::set_replicas(const std::string& ns, const std::string& name, int32_t replicas) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& o = objs_[ns + "/" + name];
  o.replicas = replicas;
  o.rv = ++rv_counter_;
  o.generation++;
}

void FakeKubeServer::add_node(const std::string& name, const std::map<std::string, std::string>& labels,
                              const std::string& resource, int64_t gpus, bool unschedulable) {
  std::lock_guard<std::mutex> lk(mu_);
  nodes_[name] = Node{labels, resource, gpus, unschedulable};
}

void FakeKubeServer::handle_nodes(const std::string& query, HttpResponse* resp) {
  std::vector<std::pair<std::string, std::string>> want;
  for (auto& [k, v] : parse_query(query)) {
    if (k != "labelSelector" || v.empty()) continue;
    size_t i = 0;
    while (i <= v.size()) {
      size_t c = v.find(',', i);
      if (c == std::string::npos) c = v.size();
      std::string term = v.substr(i, c - i);
      size_t eq = term.find('=');
      if (eq != std::string::npos) {
        std::string key = term.substr(0, eq), val = term.substr(eq + 1);
        if (!val.empty() && val[0] == '=') val.erase(0, 1);  // "=="
        want.emplace_back(key, val);
      }
      i = c + 1;
    }
  }
  std::lock_guard<std::mutex> lk(mu_);
  std::string items;
  for (auto& [name, n] : nodes_) {
    bool match = true;
    for (auto& [k, v] : want) {
      auto it = n.labels.find(k);
      if (it == n.labels.end() || it->second != v) match = false;
    }
    if (!match) continue;
    std::string labels;
    for (auto& [k, v] : n.labels) labels += (labels.empty() ? "" : ",") + json_quote(k) + ":" + json_quote(v);
    if (!items.empty()) items += ",";
    items += "{\"metadata\":{\"name\":" + json_quote(name) + ",\"labels\":{" + labels + "}},\"spec\":{" +
             (n.unschedulable ? "\"unschedulable\":true" : "") + "},\"status\":{\"allocatable\":{\"cpu\":\"192\"," +
             json_quote(n.resource) + ":\"" + std::to_string(n.gpus) + "\"}}}";
  }
  resp->status = 200;
  resp->body = "{\"kind\":\"NodeList\",\"apiVersion\":\"v1\",\"metadata\":{\"resourceVersion\":\"" +
               std::to_string(rv_counter_) + "\"},\"items\":[" + items + "]}";
}

std::string FakeKubeServer::lease_json(const std::string& ns, const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = leases_.find(ns + "/" + name);
  return it == leases_.end() ? "" : it->second.json;
}

void FakeKubeServer::handle_lease(const HttpRequest& req, const std::vector<std::string>& parts,
                                  HttpResponse* resp) {
  auto fail = [&](int code, const std::string& reason, const std::string& msg) {
    resp->status = code;
    resp->body = status_json(code, reason, msg);
  };
  // parts: {ns, "leases"} (collection) or {ns, "leases", name}
  if (parts.size() < 2 || parts.size() > 3 || parts[1] != "leases") {
    fail(404, "NotFound", "the server could not find the requested resource");
    return;
  }
  const std::string& ns = parts[0];
  std::lock_guard<std::mutex> lk(mu_);
  auto store = [&](const std::string& key, const JsonValue& body, uint64_t rv) {
    JsonValue obj = body;
    JsonValue* md = obj.get("metadata");
    if (!md || !md->is_object()) {
      obj.set("metadata", JsonValue::make_object());
      md = obj.get("metadata");
    }
    md->set("resourceVersion", JsonValue::make_string(std::to_string(rv)));
    md->set("namespace", JsonValue::make_string(ns));
    leases_[key] = Lease{json_serialize(obj), rv};
    resp->status = 200;
    resp->body = leases_[key].json;
  };
  if (parts.size() == 2) {
    if (req.method != "POST") {
      fail(405, "MethodNotAllowed", "the server does not allow this method on the requested resource");
      return;
    }
    auto body = json_parse(req.body);
    const JsonValue* nm = body.ok() ? body.value.path({"metadata", "name"}) : nullptr;
    if (!nm || !nm->is_string() || nm->str.empty()) {
      fail(422, "Invalid", "metadata.name: Required value: name or generateName is required");
      return;
    }
    const std::string key = ns + "/" + nm->str;
    if (leases_.count(key)) {
      fail(409, "AlreadyExists", "leases.coordination.k8s.io \"" + nm->str + "\" already exists");
      return;
    }
    writes_++;
    store(key, body.value, ++rv_counter_);
    resp->status = 201;
    return;
  }
  const std::string& name = parts[2];
  const std::string key = ns + "/" + name;
  auto it = leases_.find(key);
  if (req.method == "GET") {
    if (it == leases_.end()) {
      fail(404, "NotFound", "leases.coordination.k8s.io \"" + name + "\" not found");
      return;
    }
    resp->status = 200;
    resp->body = it->second.json;
    return;
  }
  if (req.method != "PUT") {
    fail(405, "MethodNotAllowed", "the server does not allow this method on the requested resource");
    return;
  }
  if (it == leases_.end()) {
    fail(404, "NotFound", "leases.coordination.k8s.io \"" + name + "\" not found");
    return;
  }
  auto body = json_parse(req.body);
  if (!body.ok() || !body.value.is_object()) {
    fail(400, "BadRequest", "the body of the request was in an unknown format");
    return;
  }
  const JsonValue* rv = body.value.path({"metadata", "resourceVersion"});
  if (!rv || rv->string_or("") != std::to_string(it->second.rv)) {
    conflicts_++;
    fail(409, "Conflict",
         "Operation cannot be fulfilled on leases.coordination.k8s.io \"" + name +
             "\": the object has been modified; please apply your changes to the latest version and try again");
    return;
  }
  writes_++;
  store(key, body.value, ++rv_counter_);
}

std::string FakeKubeServer::deployment_json(const std::string& ns, const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = objs_.find(ns + "/" + name);
  return it == objs_.end() ? "" : render_deployment(ns, name, it->second);
}

void FakeKubeServer::inject(int count, InjectedFault fault) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int i = 0; i < count; ++i) faults_.push_back(fault);
}

void FakeKubeServer::set_rbac(std::vector<std::string> rules) {
  std::lock_guard<std::mutex> lk(mu_);
  rbac_ = std::move(rules);
}

void FakeKubeServer::conflict_next(int n) {
  std::lock_guard<std::mutex> lk(mu_);
  conflict_ = n;
}

void FakeKubeServer::set_latency(Nanos per_request) {
  std::lock_guard<std::mutex> lk(mu_);
  latency_ = per_request;
}

std::string FakeKubeServer::last_method() const {
  std::lock_guard<std::mutex> lk(mu_);
  return last_method_;
}
std::string FakeKubeServer::last_body() const {
  std::lock_guard<std::mutex> lk(mu_);
  return last_body_;
}
std::string FakeKubeServer::last_path() const {
  std::lock_guard<std::mutex> lk(mu_);
  return last_path_;
}

std::string FakeKubeServer::status_json(int code, const std::string& reason, const std::string& message) {
  return "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"metadata\":{},\"status\":\"Failure\",\"message\":" +
         json_quote(message) + ",\"reason\":\"" + reason + "\",\"details\":{\"group\":\"apps\",\"kind\":\"deployments\"},\"code\":" +
         std::to_string(code) + "}";
}

// A Deployment as kube-apiserver serves it for a GPU-worker workload (one MI355X per pod).
std::string FakeKubeServer::render_deployment(const std::string& ns, const std::string& name, const Obj& o) const {
  const std::string r = std::to_string(o.replicas);
  const std::string rv = std::to_string(o.rv);
  const std::string gen = std::to_string(o.generation);
  return "{\"kind\":\"Deployment\",\"apiVersion\":\"apps/v1\",\"metadata\":{\"name\":" + json_quote(name) +
         ",\"namespace\":" + json_quote(ns) +
         ",\"uid\":\"4f7c2a9e-1b3d-4c8e-9a51-6d2e0f8b7c13\",\"resourceVersion\":\"" + rv +
         "\",\"generation\":" + gen +
         ",\"creationTimestamp\":\"2025-01-01T00:00:00Z\",\"labels\":{\"app\":" + json_quote(name) +
         ",\"accelerator\":\"amd-mi355x\"},\"annotations\":{\"deployment.kubernetes.io/revision\":\"1\"},"
         "\"managedFields\":[{\"manager\":\"kubectl-client-side-apply\",\"operation\":\"Update\",\"apiVersion\":\"apps/v1\","
         "\"time\":\"2025-01-01T00:00:00Z\",\"fieldsType\":\"FieldsV1\",\"fieldsV1\":{\"f:metadata\":{\"f:labels\":{\".\":{},"
         "\"f:app\":{},\"f:accelerator\":{}}},\"f:spec\":{\"f:progressDeadlineSeconds\":{},\"f:replicas\":{},"
         "\"f:revisionHistoryLimit\":{},\"f:selector\":{},\"f:strategy\":{\"f:rollingUpdate\":{\".\":{},\"f:maxSurge\":{},"
         "\"f:maxUnavailable\":{}},\"f:type\":{}},\"f:template\":{\"f:metadata\":{\"f:labels\":{\".\":{},\"f:app\":{}}},"
         "\"f:spec\":{\"f:containers\":{\"k:{\\\"name\\\":\\\"worker\\\"}\":{\".\":{},\"f:image\":{},\"f:name\":{},"
         "\"f:resources\":{\".\":{},\"f:limits\":{\".\":{},\"f:amd.com/gpu\":{}}}}}}}}}},"
         "{\"manager\":\"kube-controller-manager\",\"operation\":\"Update\",\"apiVersion\":\"apps/v1\",\"time\":\"2025-01-01T00:00:05Z\","
         "\"fieldsType\":\"FieldsV1\",\"fieldsV1\":{\"f:status\":{\"f:availableReplicas\":{},\"f:conditions\":{},"
         "\"f:observedGeneration\":{},\"f:readyReplicas\":{},\"f:replicas\":{},\"f:updatedReplicas\":{}}},\"subresource\":\"status\"}]},"
         "\"spec\":{\"replicas\":" + r +
         ",\"selector\":{\"matchLabels\":{\"app\":" + json_quote(name) +
         "}},\"template\":{\"metadata\":{\"creationTimestamp\":null,\"labels\":{\"app\":" + json_quote(name) +
         "}},\"spec\":{\"containers\":[{\"name\":\"worker\",\"image\":\"rocm/pytorch:rocm7.2_ubuntu22.04_py3.10_pytorch_2.10\","
         "\"command\":[\"python\",\"-m\",\"worker\",\"--queue-url=$(QUEUE_URL)\"],\"env\":[{\"name\":\"HIP_VISIBLE_DEVICES\",\"value\":\"0\"}],"
         "\"resources\":{\"limits\":{\"amd.com/gpu\":\"1\",\"memory\":\"256Gi\"},\"requests\":{\"amd.com/gpu\":\"1\",\"cpu\":\"16\",\"memory\":\"256Gi\"}},"
         "\"terminationMessagePath\":\"/dev/termination-log\",\"terminationMessagePolicy\":\"File\",\"imagePullPolicy\":\"IfNotPresent\"}],"
         "\"restartPolicy\":\"Always\",\"terminationGracePeriodSeconds\":30,\"dnsPolicy\":\"ClusterFirst\","
         "\"nodeSelector\":{\"amd.com/gpu.product-name\":\"AMD_Instinct_MI355X\"},\"securityContext\":{},\"schedulerName\":\"default-scheduler\"}},"
         "\"strategy\":{\"type\":\"RollingUpdate\",\"rollingUpdate\":{\"maxUnavailable\":\"25%\",\"maxSurge\":\"25%\"}},"
         "\"revisionHistoryLimit\":10,\"progressDeadlineSeconds\":600},"
         "\"status\":{\"observedGeneration\":" + gen + ",\"replicas\":" + r + ",\"updatedReplicas\":" + r +
         ",\"readyReplicas\":" + r + ",\"availableReplicas\":" + r +
         ",\"conditions\":[{\"type\":\"Available\",\"status\":\"True\",\"lastUpdateTime\":\"2025-01-01T00:00:05Z\","
         "\"lastTransitionTime\":\"2025-01-01T00:00:05Z\",\"reason\":\"MinimumReplicasAvailable\",\"message\":\"Deployment has minimum availability.\"},"
         "{\"type\":\"Progressing\",\"status\":\"True\",\"lastUpdateTime\":\"2025-01-01T00:00:05Z\",\"lastTransitionTime\":\"2025-01-01T00:00:00Z\","
         "\"reason\":\"NewReplicaSetAvailable\",\"message\":\"ReplicaSet \\\"" + name + "-7d9f8b6c5d\\\" has successfully progressed.\"}]}}";
}

std::string FakeKubeServer::render_scale(const std::string& ns, const std::string& name, const Obj& o) const {
  // autoscaling/v1 Scale; spec.replicas is omitempty.
  std::string spec = o.replicas != 0 ? "{\"replicas\":" + std::to_string(o.replicas) + "}" : "{}";
  return "{\"kind\":\"Scale\",\"apiVersion\":\"autoscaling/v1\",\"metadata\":{\"name\":" + json_quote(name) +
         ",\"namespace\":" + json_quote(ns) +
         ",\"uid\":\"4f7c2a9e-1b3d-4c8e-9a51-6d2e0f8b7c13\",\"resourceVersion\":\"" + std::to_string(o.rv) +
         "\",\"creationTimestamp\":\"2025-01-01T00:00:00Z\"},\"spec\":" + spec +
         ",\"status\":{\"replicas\":" + std::to_string(o.replicas) + ",\"selector\":\"app=" + name + "\"}}";
}

void FakeKubeServer::handle(const HttpRequest& req, HttpResponse* resp) {
  requests_++;
  std::string query;
  const std::string path = split_path_query(req.target, &query);
  Nanos latency;
  InjectedFault fault;
  bool faulted;
  std::string token;
  std::string method_copy = req.method, body_copy = req.body, path_copy = path;
  {
    std::lock_guard<std::mutex> lk(mu_);
    last_method_.swap(method_copy);
    last_body_.swap(body_copy);
    last_path_.swap(path_copy);
    latency = latency_;
    faulted = pop_fault(&faults_, req.method, &fault);
    token = token_;
  }
  if (latency > 0) shutdown_.wait_for(latency);
  if (faulted) {
    apply_fault(fault, resp);
    return;
  }
  resp->headers.emplace_back("Content-Type", "application/json");
  auto fail = [&](int code, const std::string& reason, const std::string& msg) {
    resp->status = code;
    resp->body = status_json(code, reason, msg);
  };
  if (!token.empty() && req.header("Authorization") != "Bearer " + token) {
    auth_failures_++;
    fail(401, "Unauthorized", "Unauthorized");
    return;
  }
  if (path == "/api/v1/nodes") {
    if (req.method != "GET") {
      fail(405, "MethodNotAllowed", "the server does not allow this method on the requested resource");
      return;
    }
    handle_nodes(query, resp);
    return;
  }
  static const std::string lease_prefix = "/apis/coordination.k8s.io/v1/namespaces/";
  if (path.compare(0, lease_prefix.size(), lease_prefix) == 0) {
    std::vector<std::string> lp;
    size_t j = lease_prefix.size();
    while (j <= path.size()) {
      size_t e = path.find('/', j);
      if (e == std::string::npos) e = path.size();
      lp.push_back(url_decode(path.substr(j, e - j), false));
      j = e + 1;
    }
    handle_lease(req, lp, resp);
    return;
  }
  // /apis/apps/v1/namespaces/{ns}/deployments/{name}[/scale]
  static const std::string prefix = "/apis/apps/v1/namespaces/";
  if (path.compare(0, prefix.size(), prefix) != 0) {
    fail(404, "NotFound", "the server could not find the requested resource");
    return;
  }
  std::vector<std::string> parts;
  size_t i = prefix.size();
  while (i <= path.size()) {
    size_t s = path.find('/', i);
    if (s == std::string::npos) s = path.size();
    parts.push_back(url_decode(path.substr(i, s - i), false));
    i = s + 1;
  }
  if (parts.size() < 3 || parts[1] != "deployments" || parts.size() > 4 ||
      (parts.size() == 4 && parts[3] != "scale")) {
    fail(404, "NotFound", "the server could not find the requested resource");
    return;
  }
  const std::string& ns = parts[0];
  const std::string& name = parts[2];
  const bool scale = parts.size() == 4;
  {
    // authorization runs before the handler: a forbidden request is 403 whether or not the
    // object exists
    const std::string verb = req.method == "GET" ? "get" : req.method == "PUT" ? "update" : req.method == "PATCH" ? "patch" : "";
    const std::string resource = scale ? "deployments/scale" : "deployments";
    bool allowed;
    {
      std::lock_guard<std::mutex> lk(mu_);
      allowed = std::find(rbac_.begin(), rbac_.end(), "*") != rbac_.end() ||
                std::find(rbac_.begin(), rbac_.end(), resource + ":" + verb) != rbac_.end();
    }
    if (!verb.empty() && !allowed) {
      forbidden_++;
      fail(403, "Forbidden",
           "deployments.apps \"" + name + "\" is forbidden: User \"system:serviceaccount:" + ns +
               ":kube-sqs-autoscaler\" cannot " + verb + " resource \"" + resource +
               "\" in API group \"apps\" in the namespace \"" + ns + "\"");
      return;
    }
  }
  // Critical sections cover only the object state; rendering happens outside the lock so
  // concurrent workers are not serialised by the fake (a real apiserver serves them in parallel).
  Obj snapshot;
  const std::string key = ns + "/" + name;
  if (req.method == "GET") {
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = objs_.find(key);
      if (it == objs_.end()) {
        fail(404, "NotFound", "deployments.apps \"" + name + "\" not found");
        return;
      }
      gets_++;
      snapshot = it->second;
      if (conflict_ > 0) {
        conflict_--;
        it->second.rv = ++rv_counter_;  // concurrent status update by the deployment controller
      }
    }
    resp->status = 200;
    resp->body = scale ? render_scale(ns, name, snapshot) : render_deployment(ns, name, snapshot);
    return;
  }
  if (req.method != "PUT" && req.method != "PATCH") {
    fail(405, "MethodNotAllowed", "the server does not allow this method on the requested resource");
    return;
  }
  auto body = json_parse(req.body);
  if (!body.ok() || !body.value.is_object()) {
    fail(400, "BadRequest", "the body of the request was in an unknown format");
    return;
  }
  const JsonValue* rv = body.value.path({"metadata", "resourceVersion"});
  std::string rvs = rv ? rv->string_or("") : "";
  if (req.method == "PUT" && rvs.empty()) {
    fail(422, "Invalid", "metadata.resourceVersion: Invalid value: 0x0: must be specified for an update");
    return;
  }
  const JsonValue* r = body.value.path({"spec", "replicas"});
  int64_t nr = 0;
  if (r && !r->as_int64(&nr)) {
    fail(400, "BadRequest", "spec.replicas must be an integer");
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = objs_.find(key);
    if (it == objs_.end()) {
      fail(404, "NotFound", "deployments.apps \"" + name + "\" not found");
      return;
    }
    Obj& o = it->second;
    if (!rvs.empty() && rvs != std::to_string(o.rv)) {
      conflicts_++;
      fail(409, "Conflict",
           "Operation cannot be fulfilled on deployments.apps \"" + name +
               "\": the object has been modified; please apply your changes to the latest version and try again");
      return;
    }
    if (!r) {
      if (req.method == "PATCH") nr = o.replicas;  // merge patch without replicas: unchanged
      else nr = scale ? 0 : 1;                     // Scale omitempty / Deployment defaulting
    }
    if (nr < 0) {
      fail(422, "Invalid", "spec.replicas: Invalid value: " + std::to_string(nr) +
                               ": must be greater than or equal to 0");
      return;
    }
    writes_++;
    if (o.replicas != static_cast<int32_t>(nr)) o.generation++;
    o.replicas = static_cast<int32_t>(nr);
    o.rv = ++rv_counter_;
    snapshot = o;
  }
  resp->status = 200;
  resp->body = scale ? render_scale(ns, name, snapshot) : render_deployment(ns, name, snapshot);
}

}  // namespace ksa
