#include "kube.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <fstream>
#include <sstream>

#include "goutil.h"
#include "json.h"
#include "sigv4.h"  // aws_uri_encode for path segments

namespace ksa {

// ---------------------------------------------------------------------------------------
// Token providers

FileTokenProvider::FileTokenProvider(std::string path, std::shared_ptr<Clock> clock, Nanos refresh)
    : path_(std::move(path)), clock_(std::move(clock)), refresh_(refresh) {}

Result<std::string> FileTokenProvider::token() {
  std::lock_guard<std::mutex> lk(mu_);
  Nanos now = clock_->now();
  if (have_ && now - read_at_ < refresh_) return Result<std::string>::Ok(cached_);
  std::ifstream f(path_);
  if (!f) {
    if (have_) return Result<std::string>::Ok(cached_);  // keep the last good token
    return Result<std::string>::Err(Status::Err("open " + path_ + ": no such file or directory"));
  }
  std::stringstream ss;
  ss << f.rdbuf();
  std::string t = ss.str();
  while (!t.empty() && (t.back() == '\n' || t.back() == '\r' || t.back() == ' ')) t.pop_back();
  cached_ = t;
  have_ = true;
  read_at_ = now;
  return Result<std::string>::Ok(cached_);
}

void FileTokenProvider::invalidate(const std::string& used) {
  std::lock_guard<std::mutex> lk(mu_);
  if (have_ && cached_ == used) read_at_ = clock_->now() - refresh_;  // re-read on next use
}

// ---------------------------------------------------------------------------------------
// Client-side throttle

TokenBucket::TokenBucket(double qps, int burst, std::shared_ptr<Clock> clock)
    : qps_(qps), burst_(burst < 1 ? 1 : burst), tokens_(0), clock_(std::move(clock)) {}

void TokenBucket::refill_locked() {
  const Nanos now = clock_->now();
  if (!started_) {
    started_ = true;
    tokens_ = burst_;
    last_ = now;
  } else if (now > last_) {
    tokens_ = std::min(burst_, tokens_ + static_cast<double>(now - last_) * qps_ / 1e9);
    last_ = now;
  }
}

bool TokenBucket::try_take() {
  std::lock_guard<std::mutex> lk(mu_);
  refill_locked();
  if (tokens_ < 1) return false;
  tokens_ -= 1;
  return true;
}

Nanos TokenBucket::reserve() {
  std::lock_guard<std::mutex> lk(mu_);
  refill_locked();
  tokens_ -= 1;
  if (tokens_ >= 0) return 0;
  return static_cast<Nanos>(std::ceil(-tokens_ * 1e9 / qps_));
}

Nanos TokenBucket::take(StopFlag* stop) {
  const Nanos wait = reserve();
  if (wait > 0) clock_->sleep(wait, stop);
  return wait;
}

// ---------------------------------------------------------------------------------------
// Object helpers

namespace {

// JsonValue::as_int64 on a number literal in place.
bool int_literal(const std::string& s, size_t b, size_t e, int64_t* out) {
  if (b >= e) return false;
  bool neg = false;
  if (s[b] == '-') {
    neg = true;
    ++b;
  }
  uint64_t acc = 0;
  for (size_t i = b; i < e; ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') return false;  // fraction/exponent: not an integer literal
    const uint64_t d = static_cast<uint64_t>(c - '0');
    if (acc > (~uint64_t(0) - d) / 10) return false;
    acc = acc * 10 + d;
  }
  const uint64_t cutoff = uint64_t(1) << 63;
  if ((!neg && acc >= cutoff) || (neg && acc > cutoff)) return false;
  *out = neg ? static_cast<int64_t>(0 - acc) : static_cast<int64_t>(acc);
  return true;
}

}  // namespace

Result<ScaleObject> parse_scale_object(const std::string& json, bool absent_is_zero) {
  // Fast path: one scan, no DOM (every poll parses a Scale or a whole Deployment).
  const ScaleFields f = json_scan_scale(json);
  if (f.ok && !f.rv_escaped && (!f.has_replicas || f.replicas_null || f.replicas_number)) {
    ScaleObject o;
    o.raw = json;
    if (f.has_rv) o.resource_version.assign(json, f.rv_begin, f.rv_end - f.rv_begin);
    if (f.has_replicas && !f.replicas_null) {
      int64_t v;
      if (!int_literal(json, f.replicas_begin, f.replicas_end, &v))
        return Result<ScaleObject>::Err(Status::Err("spec.replicas is not an integer"));
      o.has_replicas = true;
      o.replicas = go_int32(v);
    } else if (absent_is_zero) {
      o.has_replicas = true;
      o.replicas = 0;
    }
    return Result<ScaleObject>::Ok(std::move(o));
  }
  return parse_scale_object_dom(json, absent_is_zero);
}

Result<ScaleObject> parse_scale_object_dom(const std::string& json, bool absent_is_zero) {
  auto j = json_parse(json);
  if (!j.ok()) return Result<ScaleObject>::Err(j.status);
  ScaleObject o;
  o.raw = json;
  const JsonValue* rv = j.value.path({"metadata", "resourceVersion"});
  if (rv && rv->is_string()) o.resource_version = rv->str;
  const JsonValue* r = j.value.path({"spec", "replicas"});
  if (r && r->type != JsonValue::Type::Null) {
    int64_t v;
    if (!r->as_int64(&v)) return Result<ScaleObject>::Err(Status::Err("spec.replicas is not an integer"));
    o.has_replicas = true;
    o.replicas = go_int32(v);
  } else if (absent_is_zero) {
    o.has_replicas = true;
    o.replicas = 0;
  }
  return Result<ScaleObject>::Ok(std::move(o));
}

Result<std::string> set_spec_replicas(const std::string& raw, int32_t replicas) {
  const std::string num = std::to_string(replicas);
  const ScaleFields f = json_scan_scale(raw);
  if (f.ok) {
    std::string out;
    out.reserve(raw.size() + 32);
    if (f.has_spec && f.spec_is_object) {
      if (f.has_replicas) {  // splice the value in place
        out.append(raw, 0, f.replicas_begin);
        out += num;
        out.append(raw, f.replicas_end, std::string::npos);
      } else {  // insert as the first member of spec
        out.append(raw, 0, f.spec_begin + 1);
        out += "\"replicas\":";
        out += num;
        if (!f.spec_empty) out.push_back(',');
        out.append(raw, f.spec_begin + 1, std::string::npos);
      }
    } else {
      out.append(raw, 0, f.root_begin + 1);
      out += "\"spec\":{\"replicas\":";
      out += num;
      out.push_back('}');
      if (!f.root_empty) out.push_back(',');
      out.append(raw, f.root_begin + 1, std::string::npos);
    }
    return Result<std::string>::Ok(std::move(out));
  }
  return set_spec_replicas_dom(raw, replicas);
}

Result<std::string> set_spec_replicas_dom(const std::string& raw, int32_t replicas) {
  const std::string num = std::to_string(replicas);
  auto j = json_parse(raw);
  if (!j.ok()) return Result<std::string>::Err(j.status);
  if (!j.value.is_object()) return Result<std::string>::Err(Status::Err("object is not a JSON object"));
  const JsonValue* spec = j.value.get("spec");
  if (spec && spec->is_object()) {
    const JsonValue* r = spec->get("replicas");
    if (r) return Result<std::string>::Ok(json_splice(raw, *r, num));
    // insert as the first member of spec
    std::string out = raw.substr(0, spec->begin + 1) + "\"replicas\":" + num +
                      (spec->obj.empty() ? "" : ",") + raw.substr(spec->begin + 1);
    return Result<std::string>::Ok(out);
  }
  std::string ins = "\"spec\":{\"replicas\":" + num + "}";
  const JsonValue& root = j.value;
  std::string out = raw.substr(0, root.begin + 1) + ins + (root.obj.empty() ? "" : ",") +
                    raw.substr(root.begin + 1);
  return Result<std::string>::Ok(out);
}

// ---------------------------------------------------------------------------------------
// REST client

KubeRestDeployments::KubeRestDeployments(KubeOptions opts)
    : mode_(static_cast<int>(opts.mode)), opts_(std::move(opts)) {
  auto u = parse_url(opts_.server);
  if (!u.ok()) {
    init_status_ = u.status;
    return;
  }
  url_ = u.value;
  http_ = std::make_unique<HttpClient>(url_, opts_.tls, opts_.timeout);
  http_->set_busy_poll(opts_.busy_poll);
  Status ps = http_->set_proxy(opts_.proxy);
  if (!ps.ok()) init_status_ = ps;
  wait_clock_ = opts_.clock ? opts_.clock : std::make_shared<RealClock>();
  if (opts_.qps > 0) limiter_ = std::make_unique<TokenBucket>(opts_.qps, opts_.burst, wait_clock_);
}

void KubeRestDeployments::cancel() {
  cancel_.request_stop();
  if (opts_.token) opts_.token->cancel();  // an exec plugin run this client waits for
  if (http_) http_->cancel();
}

void KubeRestDeployments::throttle() {
  if (!limiter_) return;
  const Nanos waited = limiter_->reserve();
  if (waited > 0) {
    wait_until_.store(wait_clock_->now() + waited, std::memory_order_release);
    wait_clock_->sleep(waited, &cancel_);
    std::lock_guard<std::mutex> lk(mu_);
    stats_.throttled++;
    stats_.throttle_ns += waited;
  }
}

KubeStats KubeRestDeployments::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  KubeStats s = stats_;
  if (http_) s.http = http_->stats();
  return s;
}

std::string KubeRestDeployments::path_for(const std::string& name) const { return path_in(mode(), name); }

std::string KubeRestDeployments::path_in(ScaleMode m, const std::string& name) const {
  std::string base = url_.path;
  while (!base.empty() && base.back() == '/') base.pop_back();
  std::string p = base + "/apis/apps/v1/namespaces/" + aws_uri_encode(opts_.namespace_, false) +
                  "/deployments/" + aws_uri_encode(name, false);
  if (m != ScaleMode::Deployment) p += "/scale";
  return p;
}

namespace {

// client-go's error text for a non-2xx response.
std::string kube_error_message(const HttpResponse& resp, const std::string& verb,
                               const std::string& name, const std::string& resource) {
  auto j = json_parse(resp.body);
  if (j.ok() && j.value.is_object()) {
    const JsonValue* kind = j.value.get("kind");
    const JsonValue* msg = j.value.get("message");
    if (kind && kind->string_or("") == "Status" && msg && msg->is_string() && !msg->str.empty())
      return msg->str;
  }
  std::string what = "(" + verb + " " + resource + " " + name + ")";
  switch (resp.status) {
    case 401: return "Unauthorized";
    case 403: return "forbidden: User cannot " + verb + " resource " + what;
    case 404: return "the server could not find the requested resource " + what;
    case 409: return "the server reported a conflict " + what;
    case 429: return "the server has received too many requests and has asked us to try again later " + what;
    default: break;
  }
  if (resp.status >= 500) {
    std::string body = resp.body.size() > 200 ? resp.body.substr(0, 200) : resp.body;
    return "an error on the server (" + go_quote(body) +
           ") has prevented the request from succeeding " + what;
  }
  return "the server responded with the status code " + std::to_string(resp.status) +
         " but did not return more information " + what;
}

std::string base64(const std::string& in) {
  static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  size_t i = 0;
  while (i + 2 < in.size()) {
    uint32_t v = (uint8_t(in[i]) << 16) | (uint8_t(in[i + 1]) << 8) | uint8_t(in[i + 2]);
    out.push_back(tbl[v >> 18]);
    out.push_back(tbl[(v >> 12) & 63]);
    out.push_back(tbl[(v >> 6) & 63]);
    out.push_back(tbl[v & 63]);
    i += 3;
  }
  if (i + 1 == in.size()) {
    uint32_t v = uint8_t(in[i]) << 16;
    out.push_back(tbl[v >> 18]);
    out.push_back(tbl[(v >> 12) & 63]);
    out += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = (uint8_t(in[i]) << 16) | (uint8_t(in[i + 1]) << 8);
    out.push_back(tbl[v >> 18]);
    out.push_back(tbl[(v >> 12) & 63]);
    out.push_back(tbl[(v >> 6) & 63]);
    out.push_back('=');
  }
  return out;
}

}  // namespace

Status KubeRestDeployments::add_auth(HttpRequest* req) {
  req->headers.emplace_back("Accept", "application/json, */*");
  if (opts_.token) {
    auto t = opts_.token->token();
    if (!t.ok()) return t.status;
    if (!t.value.empty()) req->headers.emplace_back("Authorization", "Bearer " + t.value);
  } else if (!opts_.basic_user.empty()) {
    req->headers.emplace_back("Authorization",
                              "Basic " + base64(opts_.basic_user + ":" + opts_.basic_password));
  }
  return Status::OK();
}

Status KubeRestDeployments::check_response(const std::string& verb_desc, const HttpRequest& req,
                                           const HttpResponse& resp, const std::string& name,
                                           const Status& transport) {
  if (!transport.ok()) {
    std::string m = req.method;
    std::string verb = m.substr(0, 1) + std::string(m.begin() + 1, m.end());
    for (size_t i = 1; i < verb.size(); ++i) verb[i] = static_cast<char>(std::tolower(verb[i]));
    return Status::Err(verb + " \"" + url_.origin() + req.target + "\": " + transport.message());
  }
  if (resp.status == 401 && opts_.token) {
    const std::string auth = req.header("Authorization");
    if (auth.compare(0, 7, "Bearer ") == 0) opts_.token->invalidate(auth.substr(7));
  }
  if (resp.status < 200 || resp.status >= 300) {
    const std::string resource = "deployments.apps";
    std::lock_guard<std::mutex> lk(mu_);
    if (resp.status == 409) stats_.conflicts++;
    return Status::Err(kube_error_message(resp, verb_desc, name, resource), resp.status);
  }
  return Status::OK();
}

// client-go rest.Request.request retries at most this many times (maxRetries).
constexpr int kMaxRetryAfter = 10;

int64_t KubeRestDeployments::retry_wait_s(const HttpRequest& req, const HttpResponse& resp,
                                          const Status& transport) const {
  if (!transport.ok()) {
    // net.IsConnectionReset / net.IsProbableEOF: only GETs are replayed (writes are not idempotent)
    if (req.method != "GET") return -1;
    const std::string& m = transport.message();
    const bool eof = m == "EOF" || m == "unexpected EOF" || (m.size() > 4 && m.compare(m.size() - 4, 4, ": EOF") == 0);
    if (eof || m.find("connection reset by peer") != std::string::npos ||
        m.find("use of closed network connection") != std::string::npos)
      return 1;
    return -1;
  }
  if (resp.status != 429 && resp.status < 500) return -1;
  const std::string h = resp.header("Retry-After");
  if (h.empty()) return -1;
  auto v = go_atoi(h);  // strconv.Atoi: an HTTP-date is not retried
  if (!v.ok()) return -1;
  return v.value;
}

bool KubeRestDeployments::sleep_retry(int64_t seconds) {
  // Go sleeps the (possibly negative: no wait) Duration; cap one wait at an hour so a bogus
  // header cannot park the loop (stop still interrupts it).
  const int64_t s = seconds < 0 ? 0 : (seconds > 3600 ? 3600 : seconds);
  if (s > 0) {
    wait_until_.store(wait_clock_->now() + s * kSecond, std::memory_order_release);
    if (!wait_clock_->sleep(s * kSecond, &cancel_)) return false;
  }
  return !cancel_.stopped();
}

Status KubeRestDeployments::do_request(const std::string& verb_desc, HttpRequest* req,
                                       HttpResponse* resp, const std::string& name) {
  Status a = add_auth(req);
  if (!a.ok()) return a;
  throttle();
  for (int retries = 1;; ++retries) {
    Status t = http_->round_trip(*req, resp);
    const int64_t wait = retry_wait_s(*req, *resp, t);
    if (wait < 0 || retries > kMaxRetryAfter || !sleep_retry(wait))
      return check_response(verb_desc, *req, *resp, name, t);
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.retry_after++;
    }
    throttle();  // every retry also goes through the client-side rate limiter
    *resp = HttpResponse();
  }
}

Result<ScaleObject> KubeRestDeployments::parse_get(ScaleMode m, const Status& s, const HttpResponse& resp) {
  if (!s.ok()) {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.errors++;
    return Result<ScaleObject>::Err(s);
  }
  return parse_scale_object(resp.body, m != ScaleMode::Deployment);
}

bool KubeRestDeployments::try_fallback(const Status& s, const std::string& name,
                                       Result<ScaleObject>* deployment) {
  if (!opts_.rbac_fallback || mode() == ScaleMode::Deployment) return false;
  // 403 only when RBAC refuses the subresource itself: its message names it ("User ... cannot
  // get resource \"deployments/scale\" in API group \"apps\" ..."). An admission webhook
  // (Gatekeeper, Kyverno) or a quota also answers 403, but it judged this write: sending the
  // same write to the whole Deployment would step around a policy that only matches
  // deployments/scale. 404 only when it names no object -- the route is missing ("the server
  // could not find the requested resource"), not the Deployment.
  const std::string& m = s.message();
  const bool rbac_refusal = s.code() == 403 && m.find(" cannot ") != std::string::npos &&
                            m.find("resource \"deployments/scale\"") != std::string::npos &&
                            m.find("admission webhook") == std::string::npos;
  const bool missing_route =
      s.code() == 404 && m.rfind("the server could not find the requested resource", 0) == 0;
  if (!rbac_refusal && !missing_route) return false;
  // Can the Deployment itself be read? If not, the /scale error stands and the mode is kept.
  auto d = get_in(ScaleMode::Deployment, name);
  if (!d.ok()) return false;
  int expected = mode_.load(std::memory_order_acquire);
  if (expected != static_cast<int>(ScaleMode::Deployment) &&
      mode_.compare_exchange_strong(expected, static_cast<int>(ScaleMode::Deployment))) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.scale_fallbacks++;
    }
    if (opts_.log)
      opts_.log->warn("The deployments/scale subresource is not usable (" + s.message() +
                      "); scaling " + opts_.namespace_ + "/" + name +
                      " with GET+PUT of the whole Deployment, as the reference does");
  }
  *deployment = std::move(d);
  return true;
}

void KubeRestDeployments::warm() {
  if (!init_status_.ok() || cancel_.stopped()) return;
  if (opts_.token) (void)opts_.token->token();  // a token file due for a re-read is read now
  http_->warm();
}

bool KubeRestDeployments::begin_get(const std::string& name, bool may_dial) {
  if (!init_status_.ok() || name.empty() || http_->in_flight()) return false;
  if (!may_dial && !http_->ready_without_dial()) return false;
  HttpRequest req;
  req.method = "GET";
  const ScaleMode m = mode();
  req.target = path_in(m, name);
  if (!add_auth(&req).ok()) return false;
  // A speculative read never waits for the throttle: without a free token it is skipped and
  // the decision (if any) does the reference's own throttled GET. So the extra reads of
  // --pipeline-reads cannot slow polls down at a fast --poll-period.
  if (limiter_ && !limiter_->try_take()) {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.speculative_skipped++;
    return false;
  }
  if (!http_->send(req).ok()) return false;  // the synchronous GET will report the error
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.gets++;
  }
  pending_name_ = name;
  pending_mode_ = m;
  pending_req_ = std::move(req);
  return true;
}

Result<ScaleObject> KubeRestDeployments::finish_get() {
  if (!http_->in_flight()) return Result<ScaleObject>::Err(Status::Err("no pipelined GET in flight"));
  HttpResponse resp;
  Status t = http_->receive(&resp);
  // A pipelined read that client-go would retry (Retry-After, reset connection) continues as
  // the reference's own synchronous GET after the wait.
  const int64_t wait = retry_wait_s(pending_req_, resp, t);
  if (wait >= 0 && sleep_retry(wait)) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.retry_after++;
    }
    return get(pending_name_);
  }
  auto r = parse_get(pending_mode_, check_response("get", pending_req_, resp, pending_name_, t), resp);
  Result<ScaleObject> d;
  if (!r.ok() && try_fallback(r.status, pending_name_, &d)) return d;
  return r;
}

Result<ScaleObject> KubeRestDeployments::get_in(ScaleMode m, const std::string& name) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.gets++;
  }
  HttpRequest req;
  req.method = "GET";
  req.target = path_in(m, name);
  HttpResponse resp;
  return parse_get(m, do_request("get", &req, &resp, name), resp);
}

Result<ScaleObject> KubeRestDeployments::get(const std::string& name) {
  if (!init_status_.ok()) return Result<ScaleObject>::Err(init_status_);
  if (name.empty()) return Result<ScaleObject>::Err(Status::Err("resource name may not be empty"));
  auto r = get_in(mode(), name);
  Result<ScaleObject> d;
  if (!r.ok() && try_fallback(r.status, name, &d)) return d;
  return r;
}

Status KubeRestDeployments::update(const std::string& name, const ScaleObject& fetched,
                                   int32_t replicas) {
  if (!init_status_.ok()) return init_status_;
  if (name.empty()) return Status::Err("resource name may not be empty");
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.updates++;
  }
  const ScaleMode m = mode();
  HttpRequest req;
  req.target = path_in(m, name);
  if (m == ScaleMode::Patch) {
    req.method = "PATCH";
    req.headers.emplace_back("Content-Type", "application/merge-patch+json");
    req.body = "{\"metadata\":{\"resourceVersion\":" + json_quote(fetched.resource_version) +
               "},\"spec\":{\"replicas\":" + std::to_string(replicas) + "}}";
  } else {
    req.method = "PUT";
    req.headers.emplace_back("Content-Type", "application/json");
    auto body = set_spec_replicas(fetched.raw, replicas);
    if (!body.ok()) return body.status;
    req.body = std::move(body.value);
  }
  HttpResponse resp;
  Status s = do_request("update", &req, &resp, name);
  if (!s.ok()) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.errors++;
    }
    // The Role may grant get on deployments/scale but not update: write through the Deployment
    // instead, provided it is still the object that was read (the Scale carries the
    // Deployment's resourceVersion), else report the conflict the write would have had.
    Result<ScaleObject> d;
    if (m != ScaleMode::Deployment && try_fallback(s, name, &d)) {
      if (d.value.resource_version != fetched.resource_version) {
        std::lock_guard<std::mutex> lk(mu_);
        stats_.conflicts++;
        return Status::Err("Operation cannot be fulfilled on deployments.apps \"" + name +
                               "\": the object has been modified; please apply your changes to the latest "
                               "version and try again",
                           409);
      }
      return update(name, d.value, replicas);
    }
  }
  return s;
}

// ---------------------------------------------------------------------------------------
// PodAutoScaler

PodAutoScaler::PodAutoScaler(std::shared_ptr<DeploymentApi> api, std::string deployment,
                             std::string ns, int64_t max, int64_t min, int64_t scale_up_pods,
                             int64_t scale_down_pods, std::shared_ptr<Logger> log,
                             std::shared_ptr<Clock> clock)
    : api_(std::move(api)),
      deployment_(std::move(deployment)),
      ns_(std::move(ns)),
      max_(max),
      min_(min),
      up_(scale_up_pods),
      down_(scale_down_pods),
      log_(std::move(log)),
      clock_(std::move(clock)) {}

bool PodAutoScaler::prefetch(bool may_dial) {
  if (prefetch_pending_) return true;
  prefetch_pending_ = api_->begin_get(deployment_, may_dial);
  return prefetch_pending_;
}

void PodAutoScaler::discard_prefetch() {
  if (!prefetch_pending_) return;
  prefetch_pending_ = false;
  (void)api_->finish_get();  // drain the response so the connection stays in sync
}

Result<ScaleObject> PodAutoScaler::read(ScaleSpan* span, bool* from_prefetch) {
  *from_prefetch = false;
  if (prefetch_pending_) {
    prefetch_pending_ = false;
    auto r = api_->finish_get();
    if (r.ok()) {
      *from_prefetch = true;
      return r;
    }
    // A failed speculative read is not reported: fall through to the reference's own GET.
  }
  span->gets++;
  return api_->get(deployment_);
}

Status PodAutoScaler::scale(bool up, ScaleSpan* span) {
  ScaleSpan local;
  if (!span) span = &local;
  const std::string dir = up ? "up" : "down";
  const std::string get_ctx = "Failed to get deployment from kube server, no scale " + dir + " occurred";
  Nanos t0 = clock_->now();
  bool from_prefetch = false;
  auto d = read(span, &from_prefetch);
  span->get_ns = clock_->now() - t0;
  span->used_prefetch = from_prefetch;
  for (int attempt = 0;; ++attempt) {
    if (!d.ok()) return d.status.wrap(get_ctx);
    if (!d.value.has_replicas)  // the reference dereferences a nil pointer here (scale.go:60,87)
      return Status::Err("deployment has no spec.replicas").wrap(get_ctx);
    const int32_t cur = d.value.replicas;
    span->read = true;
    span->before = span->after = cur;
    int32_t next;
    if (up) {
      const int32_t max32 = go_int32(max_.load(std::memory_order_relaxed));  // scale.go:62-69
      if (cur >= max32) {
        log_->info("More than max pods running. No scale up. Replicas: " + std::to_string(cur));
        return Status::OK();
      }
      next = wrap_add32(cur, go_int32(up_));
      if (next > max32) next = max32;
    } else {
      const int32_t min32 = go_int32(min_);  // scale.go:89-97
      if (cur <= min32) {
        log_->info("Less than min pods running. No scale down. Replicas: " + std::to_string(cur));
        return Status::OK();
      }
      next = wrap_sub32(cur, go_int32(down_));
      if (next < min32) next = min32;
    }
    if (dry_run_) {
      // Shadow mode: the decision is made and logged exactly as for a write, nothing is sent.
      span->after = next;
      log_->info("Dry run: would scale " + dir + ". Replicas: " + std::to_string(cur) + " -> " +
                 std::to_string(next));
      return Status::OK();
    }
    Nanos tw = clock_->now();
    Status s = api_->update(deployment_, d.value, next);
    span->update_ns += clock_->now() - tw;
    if (!s.ok() && s.code() == 409 && from_prefetch && attempt == 0) {
      // The object changed after the pipelined read: re-read and decide again, which is the
      // reference's GET-after-poll. Only a conflict on this fresh read is reported.
      Nanos tg = clock_->now();
      span->gets++;
      d = api_->get(deployment_);
      span->get_ns += clock_->now() - tg;
      span->refetched = true;
      from_prefetch = false;
      continue;
    }
    span->wrote = s.ok();
    if (!s.ok()) return s.wrap("Failed to scale " + dir);
    span->after = next;
    log_->info("Scale " + dir + " successful. Replicas: " + std::to_string(next));
    return Status::OK();
  }
}

Status PodAutoScaler::scale_up(ScaleSpan* span) { return scale(true, span); }      // scale.go:54-79
Status PodAutoScaler::scale_down(ScaleSpan* span) { return scale(false, span); }  // scale.go:81-107

}  // namespace ksa
