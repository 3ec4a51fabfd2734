#include "sqs.h"

#include <algorithm>

#include "goutil.h"
#include "json.h"
#include "xml.h"

namespace ksa {

const std::vector<std::string>& default_attribute_names() {
  static const std::vector<std::string> names = {
      "ApproximateNumberOfMessages",
      "ApproximateNumberOfMessagesDelayed",
      "ApproximateNumberOfMessagesNotVisible",
  };
  return names;
}

std::string aws_request_failure(const std::string& code, const std::string& message, int status,
                                const std::string& request_id) {
  return code + ": " + message + "\n\tstatus code: " + std::to_string(status) +
         ", request id: " + request_id;
}

// ---------------------------------------------------------------------------------------
// HttpSqsApi

// aws-sdk-go v1.35 endpoints model: the partition is chosen by region pattern (aws-cn, aws-iso,
// aws-iso-b, otherwise the commercial/GovCloud suffix) and "sqs" uses the default hostname
// template "{service}.{region}.{dnsSuffix}". The "fips-<region>" pseudo-regions map to
// "sqs-fips.<region>" and sign for <region> (their credentialScope).
std::string aws_dns_suffix(const std::string& region) {
  if (region.rfind("cn-", 0) == 0) return "amazonaws.com.cn";
  if (region.rfind("us-isob-", 0) == 0) return "sc2s.sgov.gov";
  if (region.rfind("us-iso-", 0) == 0) return "c2s.ic.gov";
  return "amazonaws.com";
}

namespace {

bool fips_region(const std::string& region, std::string* base) {
  if (region.rfind("fips-", 0) == 0 && region.size() > 5) {
    *base = region.substr(5);
    return true;
  }
  return false;
}

}  // namespace

std::string HttpSqsApi::endpoint_for_region(const std::string& region) {
  if (region.empty()) return "";
  std::string base;
  if (fips_region(region, &base)) return "https://sqs-fips." + base + "." + aws_dns_suffix(base);
  return "https://sqs." + region + "." + aws_dns_suffix(region);
}

std::string HttpSqsApi::signing_region(const std::string& region) {
  std::string base;
  return fips_region(region, &base) ? base : region;
}

HttpSqsApi::HttpSqsApi(SqsHttpOptions opts, std::shared_ptr<CredentialsProvider> creds,
                       std::shared_ptr<Clock> clock)
    : opts_(std::move(opts)),
      clock_(std::move(clock)),
      creds_(std::move(creds), 5LL * 60 * kSecond),
      signer_(signing_region(opts_.region), "sqs") {
  endpoint_ = opts_.endpoint.empty() ? endpoint_for_region(opts_.region) : opts_.endpoint;
  if (opts_.region.empty()) {
    // aws-sdk-go v1 validates the region before sending (request.ValidateEndpointHandler).
    endpoint_status_ = Status::Err("MissingRegion: could not find region configuration");
    return;
  }
  auto u = parse_url(endpoint_);
  if (!u.ok()) {
    endpoint_status_ = u.status;
    return;
  }
  url_ = u.value;
  http_ = std::make_unique<HttpClient>(url_, opts_.tls, opts_.timeout);
  http_->set_busy_poll(opts_.busy_poll);
  http_->set_caller_retries(true);  // DefaultRetryer: a failed send is retried above the client
  Status ps = http_->set_proxy(opts_.proxy);
  if (!ps.ok()) endpoint_status_ = ps;
}

void HttpSqsApi::cancel() {
  cancel_.request_stop();
  creds_.cancel();  // a worker process waiting for its supervisor's next credential set
  if (http_) http_->cancel();
}

SqsApiStats HttpSqsApi::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  SqsApiStats s = stats_;
  if (http_) s.http = http_->stats();
  return s;
}

Nanos HttpSqsApi::retry_delay(int retry_count, bool throttle) {
  // DefaultRetryer.RetryRules: 2^retryCount * jitter(minDelay), jitter(d) in [d, 2d),
  // capped at jitter(maxDelay/2).
  Nanos min_delay = throttle ? opts_.min_throttle_delay : opts_.min_retry_delay;
  Nanos max_delay = opts_.max_retry_delay;
  std::lock_guard<std::mutex> lk(mu_);  // rng_ (an HttpSqsApi may be shared by workers)
  auto jitter = [&](Nanos d) -> Nanos {
    if (d <= 0) return 0;
    rng_ ^= rng_ << 13;
    rng_ ^= rng_ >> 7;
    rng_ ^= rng_ << 17;
    return d + static_cast<Nanos>(rng_ % static_cast<uint64_t>(d));
  };
  if (retry_count >= 62) return jitter(max_delay / 2);
  Nanos base = jitter(min_delay);
  if (base > (max_delay >> retry_count)) return jitter(max_delay / 2);
  Nanos d = base << retry_count;
  return d > max_delay ? jitter(max_delay / 2) : d;
}

void HttpSqsApi::sign_locked(const std::string& queue_url, const std::vector<std::string>& names,
                             const Credentials& c, int64_t unix_ns) {
  if (!prepared_valid_ || queue_url != prepared_url_ || names != prepared_names_) {
    HttpRequest proto;
    proto.method = "POST";
    proto.target = url_.path.empty() ? "/" : url_.path;
    proto.headers.emplace_back("Host", url_.host_header());
    if (opts_.protocol == SqsProtocol::Query) {
      // url.Values.Encode(): keys sorted, QueryEscape'd.
      std::vector<std::pair<std::string, std::string>> params;
      params.emplace_back("Action", "GetQueueAttributes");
      for (size_t i = 0; i < names.size(); ++i)
        params.emplace_back("AttributeName." + std::to_string(i + 1), names[i]);
      params.emplace_back("QueueUrl", queue_url);
      params.emplace_back("Version", "2012-11-05");
      std::stable_sort(params.begin(), params.end(),
                       [](const auto& a, const auto& b) { return a.first < b.first; });
      for (size_t i = 0; i < params.size(); ++i) {
        if (i) proto.body.push_back('&');
        proto.body += aws_uri_encode(params[i].first, false) + "=" + aws_uri_encode(params[i].second, false);
      }
      proto.headers.emplace_back("Content-Type", "application/x-www-form-urlencoded; charset=utf-8");
    } else {
      JsonValue body = JsonValue::make_object();
      JsonValue arr;
      arr.type = JsonValue::Type::Array;
      for (auto& n : names) arr.arr.push_back(JsonValue::make_string(n));
      body.set("AttributeNames", std::move(arr));
      body.set("QueueUrl", JsonValue::make_string(queue_url));
      proto.body = json_serialize(body);
      proto.headers.emplace_back("Content-Type", "application/x-amz-json-1.0");
      proto.headers.emplace_back("X-Amz-Target", "AmazonSQS.GetQueueAttributes");
    }
    std::string path = proto.target, query;
    size_t q = path.find('?');
    if (q != std::string::npos) {
      query = path.substr(q + 1);
      path = path.substr(0, q);
    }
    prepared_ = signer_.prepare("POST", path, query, proto.headers, proto.body);
    prepared_body_ = std::move(proto.body);
    prepared_url_ = queue_url;
    prepared_names_ = names;
    prepared_valid_ = true;
    signed_valid_ = false;
  }
  const int64_t now_ns = unix_ns;
  const int64_t sec = now_ns / 1000000000 - (now_ns % 1000000000 < 0 ? 1 : 0);  // floor: amz_date's second
  if (!signed_valid_ || sec != signed_sec_ || c.access_key_id != signed_creds_.access_key_id ||
      c.secret_access_key != signed_creds_.secret_access_key || c.session_token != signed_creds_.session_token) {
    signer_.sign_prepared(prepared_, c, now_ns, &signed_headers_);
    signed_sec_ = sec;
    signed_creds_ = c;
    signed_valid_ = true;
  }
}

void HttpSqsApi::warm(const std::string& queue_url, const std::vector<std::string>& names, int64_t at_unix_ns,
                      bool presend) {
  if (!endpoint_status_.ok() || cancel_.stopped()) return;
  // Credentials first: a refresh (IMDS, STS, a credential process) happens here, not inside
  // the poll. Then the request signed for the second the poll is due in, and the connection.
  auto cr = creds_.get(at_unix_ns);
  if (!cr.ok()) {
    http_->warm();
    return;
  }
  HttpRequest req;
  {
    std::lock_guard<std::mutex> lk(prep_mu_);
    sign_locked(queue_url, names, cr.value, at_unix_ns);
    if (presend) {  // the request call_once() will make, byte for byte, when the second holds
      req.method = "POST";
      req.target = url_.path.empty() ? "/" : url_.path;
      req.body = prepared_body_;
      req.headers = signed_headers_;
    }
  }
  if (http_->warm() && presend) http_->stage(req);
}

Result<AttrMap> HttpSqsApi::call_once(const std::string& queue_url,
                                      const std::vector<std::string>& names, bool* retryable,
                                      bool* throttle, bool* expired, Nanos* retry_after) {
  *retryable = *throttle = *expired = false;
  *retry_after = 0;
  const bool timed = http_->timing();
  const int64_t t_sign = timed ? mono_ns() : 0;
  auto cr = creds_.get(clock_->unix_nanos());
  if (!cr.ok()) return Result<AttrMap>::Err(cr.status);

  std::unique_lock<std::mutex> prep_lock(prep_mu_);
  sign_locked(queue_url, names, cr.value, clock_->unix_nanos());
  if (timed) sign_ns_.store(mono_ns() - t_sign, std::memory_order_relaxed);
  creds_.signed_with(cr.value);  // a set kept after a failed refresh: the provider counts the request
  HttpRequest req;
  req.method = "POST";
  req.target = url_.path.empty() ? "/" : url_.path;
  req.body = prepared_body_;
  req.headers = signed_headers_;
  prep_lock.unlock();

  HttpResponse resp;
  Status s = http_->round_trip(req, &resp);
  if (!s.ok()) {
    *retryable = true;
    return Result<AttrMap>::Err(Status::Err("RequestError: send request failed\ncaused by: Post \"" +
                                            endpoint_ + req.target + "\": " + s.message()));
  }
  const std::string request_id = !resp.header("x-amzn-RequestId").empty()
                                     ? resp.header("x-amzn-RequestId")
                                     : resp.header("x-amz-request-id");
  if (resp.status >= 300) {
    std::string code, message, rid = request_id;
    if (opts_.protocol == SqsProtocol::Query) {
      bool found = false;
      code = xml_first_text(resp.body, "Code", &found);
      message = xml_first_text(resp.body, "Message", &found);
      if (rid.empty()) rid = xml_first_text(resp.body, "RequestId", &found);
    } else {
      auto j = json_parse(resp.body);
      if (j.ok()) {
        const JsonValue* t = j.value.get("__type");
        if (!t) t = j.value.get("code");
        code = t ? t->string_or("") : "";
        size_t hash = code.rfind('#');
        if (hash != std::string::npos) code = code.substr(hash + 1);
        const JsonValue* m = j.value.get("message");
        if (!m) m = j.value.get("Message");
        message = m ? m->string_or("") : "";
      }
      // Query-compatible error code, when the service provides one.
      std::string qe = resp.header("x-amzn-query-error");
      if (!qe.empty()) code = qe.substr(0, qe.find(';'));
    }
    if (code.empty()) code = resp.status >= 500 ? "InternalFailure" : "SerializationError";
    static const char* throttle_codes[] = {
        "Throttling", "ThrottlingException", "ThrottledException", "RequestThrottledException",
        "TooManyRequestsException", "ProvisionedThroughputExceededException",
        "TransactionInProgressException", "RequestLimitExceeded", "BandwidthLimitExceeded",
        "LimitExceededException", "RequestThrottled", "SlowDown", "PriorRequestNotComplete",
        "EC2ThrottledException", "AWS.SimpleQueueService.RequestThrottled"};
    for (const char* tc : throttle_codes)
      if (code == tc) *throttle = true;
    // Request.IsErrorThrottle: these statuses are throttles whatever the error code says.
    const int st = resp.status;
    if (st == 429 || st == 502 || st == 503 || st == 504) *throttle = true;
    if (code == "ExpiredToken" || code == "ExpiredTokenException" || code == "RequestExpired")
      *expired = true;
    // Request.IsErrorRetryable: the retryable codes, expired credentials, and HTTP 500. A 501
    // (Not Implemented) or any other status without such a code is final.
    static const char* retry_codes[] = {"RequestError", "RequestTimeout", "ResponseTimeout",
                                        "RequestTimeoutException"};
    bool retry_code = false;
    for (const char* rc : retry_codes)
      if (code == rc) retry_code = true;
    *retryable = *throttle || *expired || retry_code || st == 500;
    if (*throttle && (st == 429 || st == 503)) {  // canUseRetryAfterHeader
      auto secs = go_atoi(resp.header("Retry-After"));
      if (secs.ok()) {
        const int64_t c = secs.value > 3600 ? 3600 : (secs.value < -3600 ? -3600 : secs.value);
        *retry_after = c * kSecond;
      }
    }
    return Result<AttrMap>::Err(
        Status::Err(aws_request_failure(code, message, resp.status, rid), resp.status));
  }

  AttrMap out;
  struct ParseTimer {
    bool on;
    std::atomic<int64_t>* out;
    int64_t t0;
    ~ParseTimer() {
      if (on) out->store(mono_ns() - t0, std::memory_order_relaxed);
    }
  } parse_timer{timed, &parse_ns_, timed ? mono_ns() : 0};
  if (opts_.protocol == SqsProtocol::Query) {
    for (auto& [k, v] : xml_sqs_attributes(resp.body)) out[std::move(k)] = std::move(v);
  } else {
    auto j = json_parse(resp.body);
    if (!j.ok())
      return Result<AttrMap>::Err(Status::Err("SerializationError: failed decoding JSON RPC response\ncaused by: " +
                                              j.status.message()));
    const JsonValue* attrs = j.value.get("Attributes");
    if (attrs && attrs->is_object())
      for (auto& [k, v] : attrs->obj) out[k] = v.is_string() ? v.str : json_serialize(v);
  }
  return Result<AttrMap>::Ok(std::move(out));
}

std::string HttpSqsApi::timing_json() const {
  if (!http_ || !http_->timing()) return "";
  std::string h = http_timing_json(http_->last_timing());
  if (h.empty()) return "";
  return "{\"sign\":" + std::to_string(sign_ns_.load(std::memory_order_relaxed)) + "," + h.substr(1, h.size() - 2) +
         ",\"parse\":" + std::to_string(parse_ns_.load(std::memory_order_relaxed)) + "}";
}

Result<AttrMap> HttpSqsApi::get_queue_attributes(const std::string& queue_url,
                                                 const std::vector<std::string>& names) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.calls++;
  }
  if (!endpoint_status_.ok()) {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.errors++;
    return Result<AttrMap>::Err(endpoint_status_);
  }
  Result<AttrMap> r;
  for (int attempt = 0;; ++attempt) {
    bool retryable, throttle, expired;
    Nanos retry_after = 0;
    r = call_once(queue_url, names, &retryable, &throttle, &expired, &retry_after);
    if (r.ok() || !retryable || attempt >= opts_.max_retries || cancel_.stopped()) break;
    if (expired) creds_.invalidate();
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.retries++;
      if (throttle) stats_.throttle_retries++;
    }
    const Nanos delay = retry_delay(attempt, throttle) + retry_after;  // a negative header shortens it
    wait_until_.store(clock_->now() + (delay > 0 ? delay : 0), std::memory_order_release);
    if (!clock_->sleep(delay > 0 ? delay : 0, &cancel_)) break;  // cancelled mid back-off
  }
  if (!r.ok()) {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.errors++;
  }
  return r;
}

// ---------------------------------------------------------------------------------------
// SqsClient

SqsClient::SqsClient(std::shared_ptr<SqsApi> api, std::string queue_url,
                     std::vector<std::string> attribute_names)
    : api_(std::move(api)), queue_url_(std::move(queue_url)), names_(std::move(attribute_names)) {}

Result<int64_t> SqsClient::num_messages() {
  auto out = api_->get_queue_attributes(queue_url_, names_);
  if (!out.ok()) return Result<int64_t>::Err(out.status.wrap("Failed to get messages in SQS"));
  int64_t messages = 0;
  for (const auto& attr : names_) {
    auto it = out.value.find(attr);
    if (it == out.value.end()) {
      return Result<int64_t>::Err(
          Status::Err("attribute not present in GetQueueAttributes response")
              .wrap("Failed to get '" + attr + "' number of messages in queue"));
    }
    auto n = go_atoi(it->second);
    if (!n.ok())
      return Result<int64_t>::Err(n.status.wrap("Failed to get '" + attr + "' number of messages in queue"));
    messages = wrap_add64(messages, n.value);
  }
  return Result<int64_t>::Ok(messages);
}

}  // namespace ksa
