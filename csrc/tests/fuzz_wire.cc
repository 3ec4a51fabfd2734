// libFuzzer harness for everything that parses bytes from the network or from a plugin.
//
// The reference trusts aws-sdk-go and client-go with this (/root/reference/sqs/sqs.go:51,
// /root/reference/scale/scale.go:55,72); here the parsers are our own C++, so they are fuzzed
// under ASan + UBSan. The first input byte picks the target, the rest is the payload:
//   0  JSON DOM: parse, serialise, re-parse, spec.replicas splice, Scale/Deployment decode
//   1  XML scanner: SQS <Attribute> list, first-text lookups, entity decoding
//   2  scalar parsers: URLs, strconv.Atoi, RFC3339, strconv.Quote
//   3  HTTP response -> HttpSqsApi (Query protocol: status line, headers, chunking, XML, errors)
//   4  HTTP response -> HttpSqsApi (JSON 1.0 protocol)
//   5  HTTP response -> KubeRestDeployments GET + write (JSON objects, Status errors, 401/409)
//   6  HTTP request  -> HttpServer (request line, headers, Content-Length / chunked bodies)
// Targets 3-6 run the real socket code against a loopback peer that replays the payload.
//
// Build + run: python -m kube_sqs_autoscaler_amd.ops.build --fuzz && build/fuzz_wire -runs=N
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "../core/goutil.h"
#include "../core/http.h"
#include "../fakes/http_server.h"
#include "../core/json.h"
#include "../core/kube.h"
#include "../core/sigv4.h"
#include "../core/sqs.h"
#include "../core/xml.h"

using namespace ksa;

namespace {

// Loopback peer: accepts a connection, reads the request head (and nothing else), writes the
// current payload, closes. One connection per fuzz input.
class ReplayServer {
 public:
  ReplayServer() {
    fd_ = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    bind(fd_, reinterpret_cast<sockaddr*>(&a), sizeof a);
    listen(fd_, 64);
    socklen_t len = sizeof a;
    getsockname(fd_, reinterpret_cast<sockaddr*>(&a), &len);
    port_ = ntohs(a.sin_port);
    thread_ = std::thread([this] { loop(); });
    thread_.detach();
  }
  int port() const { return port_; }
  void set_payload(std::string p) {
    std::lock_guard<std::mutex> lk(mu_);
    payload_ = std::move(p);
  }

 private:
  void loop() {
    for (;;) {
      int c = accept4(fd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (c < 0) continue;
      std::string head;
      char buf[4096];
      while (head.find("\r\n\r\n") == std::string::npos) {
        pollfd p{c, POLLIN, 0};
        if (poll(&p, 1, 200) <= 0) break;
        ssize_t n = read(c, buf, sizeof buf);
        if (n <= 0) break;
        head.append(buf, static_cast<size_t>(n));
      }
      std::string out;
      {
        std::lock_guard<std::mutex> lk(mu_);
        out = payload_;
      }
      size_t off = 0;
      while (off < out.size()) {
        ssize_t n = send(c, out.data() + off, out.size() - off, MSG_NOSIGNAL);
        if (n <= 0) break;
        off += static_cast<size_t>(n);
      }
      shutdown(c, SHUT_WR);
      // drain whatever the client still sends (a write after a 409, a retried request head)
      while (true) {
        pollfd p{c, POLLIN, 0};
        if (poll(&p, 1, 50) <= 0) break;
        if (read(c, buf, sizeof buf) <= 0) break;
      }
      close(c);
    }
  }
  int fd_ = -1;
  int port_ = 0;
  std::mutex mu_;
  std::string payload_;
  std::thread thread_;
};

ReplayServer& replay() {
  static ReplayServer* s = new ReplayServer();  // lives for the process
  return *s;
}

std::string origin() { return "http://127.0.0.1:" + std::to_string(replay().port()); }

void fuzz_json(const std::string& in) {
  auto j = json_parse(in);
  if (j.ok()) {
    std::string s = json_serialize(j.value);
    auto again = json_parse(s);
    if (!again.ok() || json_serialize(again.value) != s) __builtin_trap();  // round trip is stable
    (void)j.value.path({"spec", "replicas"});
    int64_t v;
    if (const JsonValue* r = j.value.path({"spec", "replicas"})) (void)r->as_int64(&v);
  }
  // the single-scan fast paths give exactly what the DOM gives, errors included
  auto a = set_spec_replicas(in, 7), b = set_spec_replicas_dom(in, 7);
  if (a.ok() != b.ok() || (a.ok() ? a.value != b.value : a.status.message() != b.status.message())) __builtin_trap();
  for (bool zero : {true, false}) {
    auto p = parse_scale_object(in, zero), q = parse_scale_object_dom(in, zero);
    if (p.ok() != q.ok()) __builtin_trap();
    if (!p.ok() && p.status.message() != q.status.message()) __builtin_trap();
    if (p.ok() && (p.value.has_replicas != q.value.has_replicas || p.value.replicas != q.value.replicas ||
                   p.value.resource_version != q.value.resource_version || p.value.raw != q.value.raw))
      __builtin_trap();
  }
}

void fuzz_xml(const std::string& in) {
  (void)xml_sqs_attributes(in);
  bool found;
  (void)xml_first_text(in, "Code", &found);
  (void)xml_first_text(in, "Message", &found, in.size() / 3, in.size() / 2 + 1);
  (void)xml_unescape(in);
  const std::string e = xml_escape(in);
  if (xml_unescape(e) != in) __builtin_trap();  // escape/unescape round trip
}

void fuzz_scalars(const std::string& in) {
  (void)parse_url(in);
  (void)go_atoi(in);
  int64_t ns;
  if (parse_rfc3339(in, &ns) && ns > -(int64_t(1) << 62) && ns < (int64_t(1) << 62)) {
    // formatting and re-parsing the whole seconds lands on the same instant
    const int64_t secs = ns / 1000000000LL - (ns < 0 && ns % 1000000000LL ? 1 : 0);
    int64_t back;
    if (secs > -62135596800LL && secs < 253402300799LL &&
        (!parse_rfc3339(rfc3339_utc(secs * 1000000000LL), &back) || back != secs * 1000000000LL))
      __builtin_trap();
  }
  (void)go_quote(in);
}

void fuzz_sqs(const std::string& in, SqsProtocol proto) {
  replay().set_payload(in);
  SqsHttpOptions o;
  o.region = "us-east-1";
  o.endpoint = origin();
  o.protocol = proto;
  o.timeout = 300 * kMillisecond;
  o.max_retries = 0;
  Credentials c;
  c.access_key_id = "AKID";
  c.secret_access_key = "SECRET";
  HttpSqsApi api(o, std::make_shared<StaticCredentialsProvider>(c), std::make_shared<RealClock>());
  (void)api.get_queue_attributes(origin() + "/1/q", default_attribute_names());
}

void fuzz_kube(const std::string& in, ScaleMode mode) {
  replay().set_payload(in);
  KubeOptions o;
  o.server = origin();
  o.namespace_ = "ml";
  o.mode = mode;
  o.timeout = 300 * kMillisecond;
  o.token = std::make_shared<StaticTokenProvider>("tok");
  o.clock = std::make_shared<VirtualClock>();  // Retry-After / reset-GET retry waits: instant
  KubeRestDeployments api(o);
  auto g = api.get("workers");
  if (g.ok()) (void)api.update("workers", g.value, g.value.replicas + 1);
}

void fuzz_server(const std::string& in) {
  static HttpServer* server = [] {
    auto* s = new HttpServer([](const HttpRequest& req, HttpResponse* resp) {
      resp->status = 200;
      resp->body = req.method + " " + req.target + " " + std::to_string(req.body.size());
    });
    if (!s->listen("127.0.0.1", 0).ok()) __builtin_trap();
    return s;
  }();
  int c = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons(static_cast<uint16_t>(server->port()));
  if (connect(c, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
    close(c);
    return;
  }
  size_t off = 0;
  while (off < in.size()) {
    ssize_t n = send(c, in.data() + off, in.size() - off, MSG_NOSIGNAL);
    if (n <= 0) break;
    off += static_cast<size_t>(n);
  }
  shutdown(c, SHUT_WR);
  char buf[4096];
  while (true) {
    pollfd p{c, POLLIN, 0};
    if (poll(&p, 1, 300) <= 0) break;
    if (read(c, buf, sizeof buf) <= 0) break;
  }
  close(c);
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size == 0) return 0;
  const std::string in(reinterpret_cast<const char*>(data) + 1, size - 1);
  switch (data[0] % 7) {
    case 0: fuzz_json(in); break;
    case 1: fuzz_xml(in); break;
    case 2: fuzz_scalars(in); break;
    case 3: fuzz_sqs(in, SqsProtocol::Query); break;
    case 4: fuzz_sqs(in, SqsProtocol::Json); break;
    case 5: fuzz_kube(in, data[0] & 0x80 ? ScaleMode::Deployment : ScaleMode::Scale); break;
    case 6: fuzz_server(in); break;
  }
  return 0;
}
