// Host-only unit tests of the native runtime, built plain, with ASan+UBSan and with TSan
// (kube_sqs_autoscaler_amd/ops/build.py build_native_tests; `make sanitize`).
//
// The reference never ran its tests under the race detector (Makefile:7) and
// its loop tests leak goroutines that race on package globals. Here the multi-queue supervisor,
// the threaded fake servers and the keep-alive clients are exercised concurrently so TSan can
// see every cross-thread access of the runtime.
#include <arpa/inet.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/ioctl.h>
#include <unistd.h>

#include <atomic>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../core/affinity.h"
#include "../core/clock.h"
#include "../core/cred_slot.h"
#include "../core/exec_auth.h"
#include "../fakes/fakes.h"
#include "../fakes/http_server.h"
#include "../fakes/mem_fakes.h"
#include "../core/goutil.h"
#include "../core/http.h"
#include "../core/json.h"
#include "../core/kube.h"
#include "../core/log.h"
#include "../core/runner.h"
#include "../core/sigv4.h"
#include "../core/sqs.h"
#include "../core/xml.h"
#include "../sim/policy_sim.h"

using namespace ksa;

namespace {

int g_failed = 0;
int g_checks = 0;

#define CHECK(cond)                                                                 \
  do {                                                                              \
    ++g_checks;                                                                     \
    if (!(cond)) {                                                                  \
      std::fprintf(stderr, "  CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failed;                                                                   \
    }                                                                               \
  } while (0)

#define CHECK_EQ(a, b)                                                                        \
  do {                                                                                        \
    ++g_checks;                                                                               \
    auto va = (a);                                                                            \
    auto vb = (b);                                                                            \
    if (!(va == vb)) {                                                                        \
      std::fprintf(stderr, "  CHECK_EQ failed %s:%d: %s != %s\n", __FILE__, __LINE__, #a, #b); \
      ++g_failed;                                                                             \
    }                                                                                         \
  } while (0)

struct Test {
  const char* name;
  std::function<void()> fn;
};
std::vector<Test>& registry() {
  static std::vector<Test> t;
  return t;
}
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
#define TEST(name)                       \
  void name();                           \
  Reg reg_##name(#name, name);           \
  void name()

std::shared_ptr<Logger> quiet_logger() {
  auto l = std::make_shared<Logger>();
  l->set_level(Level::Panic);
  return l;
}

AttrMap attrs(int64_t visible, int64_t delayed = 0, int64_t not_visible = 0) {
  return {{"ApproximateNumberOfMessages", std::to_string(visible)},
          {"ApproximateNumberOfMessagesDelayed", std::to_string(delayed)},
          {"ApproximateNumberOfMessagesNotVisible", std::to_string(not_visible)}};
}

// ---------------------------------------------------------------------------------------

TEST(go_atoi_semantics) {
  CHECK_EQ(go_atoi("42").value, 42);
  CHECK_EQ(go_atoi("-7").value, -7);
  CHECK_EQ(go_atoi("+7").value, 7);
  CHECK_EQ(go_atoi("9223372036854775807").value, INT64_MAX);
  CHECK(!go_atoi("").ok());
  CHECK(!go_atoi("1_0").ok());
  CHECK(!go_atoi(" 1").ok());
  auto r = go_atoi("9223372036854775808");
  CHECK(!r.ok());
  CHECK_EQ(r.status.message(), std::string("strconv.Atoi: parsing \"9223372036854775808\": value out of range"));
}

TEST(int32_wrap) {
  CHECK_EQ(go_int32(INT64_C(4294967299)), 3);
  CHECK_EQ(wrap_add32(INT32_MAX, 1), INT32_MIN);
  CHECK_EQ(wrap_sub32(INT32_MIN, 1), INT32_MAX);
}

TEST(json_splice_replicas) {
  std::string raw = R"({"kind":"Deployment","metadata":{"resourceVersion":"12"},"spec":{"replicas":3,"x":1}})";
  auto s = set_spec_replicas(raw, 5);
  CHECK(s.ok());
  auto o = parse_scale_object(s.value, false);
  CHECK(o.ok() && o.value.replicas == 5 && o.value.resource_version == "12");
  auto s2 = set_spec_replicas(R"({"spec":{}})", 2);
  CHECK(s2.ok() && parse_scale_object(s2.value, false).value.replicas == 2);
  auto scale = parse_scale_object(R"({"kind":"Scale","spec":{}})", true);
  CHECK(scale.ok() && scale.value.has_replicas && scale.value.replicas == 0);
  CHECK(!json_parse("{\"a\":").ok());
}

// The single-scan parse_scale_object / set_spec_replicas against the JSON-DOM versions on
// hand-picked edge cases and ~30k random mutations of real objects: same results, same errors.
TEST(json_fast_paths_equal_dom) {
  std::vector<std::string> seeds = {
      R"({"kind":"Deployment","metadata":{"name":"w","resourceVersion":"12"},"spec":{"replicas":3,"x":1}})",
      R"({"kind":"Scale","apiVersion":"autoscaling/v1","metadata":{"resourceVersion":"5001"},"spec":{},"status":{"replicas":1}})",
      R"({"spec":{"replicas":null}})", R"({"spec":{"replicas":"3"}})", R"({"spec":{"replicas":3.0}})",
      R"({"spec":{"replicas":1e2}})", R"({"spec":{"replicas":-2147483649}})", R"({"spec":{"replicas":9223372036854775808}})",
      R"({"spec":{"replicas":1},"spec":{"replicas":2}})", R"({"spec":{"replicas":1,"replicas":2}})",
      R"({"spec":[1,2]})", R"({"spec":7})", R"({})", R"([])", R"("x")", R"({"metadata":{"resourceVersion":"a\"b"}})",
      R"({"metadata":{"resourceVersion":7},"spec":{}})", R"({"metadata":[],"spec":{"replicas":4}})",
      R"({"spec":{"replicas":4}})", R"({"metadata":{"resourceVersion":"1"},"metadata":{"resourceVersion":"2"}})",
      R"({"a":{"spec":{"replicas":9}},"spec":{"b":{"replicas":8}}})", R"(  {"spec" : { "replicas" : 6 } }  )",
      R"({"spec":{"replicas":0}} x)", R"({"spec":{"replicas":01}})", R"({"s":"\ud800A"})", R"({"s":"\ud800\uzzzz"})",
      "{\"s\":\"tab\tin\"}", R"({"spec":{"replicas":true}})", R"({"spec":{}, "x":[{"spec":{"replicas":1}}]})"};
  std::string deep = "{\"spec\":";
  for (int i = 0; i < 300; ++i) deep += "[";
  for (int i = 0; i < 300; ++i) deep += "]";
  seeds.push_back(deep + "}");
  auto same = [](const std::string& in) {
    auto a = set_spec_replicas(in, 7), b = set_spec_replicas_dom(in, 7);
    if (a.ok() != b.ok()) return false;
    if (a.ok() ? a.value != b.value : a.status.message() != b.status.message()) return false;
    for (bool zero : {true, false}) {
      auto p = parse_scale_object(in, zero), q = parse_scale_object_dom(in, zero);
      if (p.ok() != q.ok()) return false;
      if (!p.ok()) {
        if (p.status.message() != q.status.message()) return false;
        continue;
      }
      if (p.value.has_replicas != q.value.has_replicas || p.value.replicas != q.value.replicas ||
          p.value.resource_version != q.value.resource_version || p.value.raw != q.value.raw)
        return false;
    }
    return true;
  };
  for (auto& sd : seeds) CHECK(same(sd));
  uint64_t rng = 0x243F6A8885A308D3ULL;
  auto next = [&] {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  const std::string alphabet = "{}[]\":,\\ 0123456789-.eEnulltrfasreplicaspecmetadataresourceVersion\t\n\x01u";
  int bad = 0;
  for (int it = 0; it < 30000; ++it) {
    std::string s = seeds[next() % seeds.size()];
    const int edits = 1 + static_cast<int>(next() % 4);
    for (int e = 0; e < edits && !s.empty(); ++e) {
      const size_t pos = next() % (s.size() + 1);
      const char c = alphabet[next() % alphabet.size()];
      switch (next() % 3) {
        case 0: s.insert(pos, 1, c); break;
        case 1: if (pos < s.size()) s.erase(pos, 1); break;
        default: if (pos < s.size()) s[pos] = c; break;
      }
    }
    if (!same(s) && ++bad < 5) std::fprintf(stderr, "fast != dom for: %s\n", s.c_str());
  }
  CHECK_EQ(bad, 0);
}

TEST(xml_attributes) {
  auto a = xml_sqs_attributes(
      "<GetQueueAttributesResult><Attribute><Name>A</Name><Value>1</Value></Attribute>"
      "<Attribute><Name>B&amp;C</Name><Value>&lt;2&gt;</Value></Attribute></GetQueueAttributesResult>");
  CHECK_EQ(a.size(), size_t(2));
  CHECK(a[1].first == "B&C" && a[1].second == "<2>");
}

TEST(sigv4_published_vector) {
  SigV4Signer s("us-east-1", "service");
  Credentials c;
  c.access_key_id = "AKIDEXAMPLE";
  c.secret_access_key = "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY";
  Headers h{{"Host", "example.amazonaws.com"}};
  SignDebug d;
  s.sign(c, INT64_C(1440938160) * kSecond, "GET", "/", "", &h, "", &d);
  CHECK_EQ(d.signature, std::string("5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31"));
  CHECK(sigv4_verify("GET", "/", "", h, "", "AKIDEXAMPLE", c.secret_access_key, "us-east-1", "service").ok());
}

TEST(logger_text_format) {
  Logger l;
  CHECK_EQ(l.format(Level::Info, "Found 3 messages in the queue", {}, INT64_C(1700000000) * kSecond),
           std::string("time=\"2023-11-14T22:13:20Z\" level=info msg=\"Found 3 messages in the queue\""));
}

// Appendix C, config C2: UP at 60..120 s, DOWN at 180..360 s every 30 s.
TEST(runner_c2_golden_virtual_clock) {
  auto clock = std::make_shared<VirtualClock>(0);
  auto api = std::make_shared<TraceSqsApi>(
      clock, std::vector<std::pair<Nanos, AttrMap>>{{0, attrs(0)}, {60 * kSecond, attrs(200)}, {180 * kSecond, attrs(0)}},
      kMillisecond);
  auto fake = std::make_shared<FakeDeployments>("default");
  fake->add("w", 1);
  fake->set_latency(clock, kMillisecond);
  auto log = quiet_logger();
  auto sqs = std::make_shared<SqsClient>(api, "q", default_attribute_names());
  auto scaler = std::make_shared<PodAutoScaler>(fake, "w", "default", 8, 1, 1, 1, log, clock);
  Runner r(LoopConfig{}, sqs, scaler, clock, log);
  r.arm();
  std::vector<std::pair<int64_t, int>> ups, downs;
  for (int i = 0; i < 100; ++i) {
    auto rec = r.step();
    if (rec.up == Action::Scaled) ups.emplace_back(rec.t_poll / kSecond, rec.replicas_after);
    if (rec.down == Action::Scaled) downs.emplace_back(rec.t_poll / kSecond, rec.replicas_after);
  }
  CHECK_EQ(ups.size(), size_t(7));
  CHECK_EQ(downs.size(), size_t(7));
  for (size_t i = 0; i < ups.size() && i < 7; ++i) {
    CHECK_EQ(ups[i].first, int64_t(60 + 10 * i));
    CHECK_EQ(ups[i].second, int(2 + i));
  }
  for (size_t i = 0; i < downs.size() && i < 7; ++i) {
    CHECK_EQ(downs[i].first, int64_t(180 + 30 * i));
    CHECK_EQ(downs[i].second, int(7 - i));
  }
  CHECK_EQ(fake->replicas("w"), 1);
}

TEST(http_keepalive_roundtrips) {
  std::atomic<int> served{0};
  HttpServer srv([&](const HttpRequest& req, HttpResponse* resp) {
    served++;
    resp->status = 200;
    resp->body = req.method + " " + req.target + " " + req.body;
  });
  CHECK(srv.listen("127.0.0.1", 0).ok());
  auto u = parse_url("http://127.0.0.1:" + std::to_string(srv.port()));
  HttpClient c(u.value, TlsOptions{}, 5 * kSecond);
  for (int i = 0; i < 50; ++i) {
    HttpRequest req;
    req.method = "POST";
    req.target = "/x?i=" + std::to_string(i);
    req.body = std::string(1000 + i, 'b');
    HttpResponse resp;
    CHECK(c.round_trip(req, &resp).ok());
    CHECK_EQ(resp.status, 200);
    CHECK_EQ(resp.body.size(), std::string("POST /x?i=" + std::to_string(i) + " ").size() + 1000 + i);
  }
  CHECK_EQ(c.stats().connects, uint64_t(1));
  srv.drop_connections();
  HttpRequest req;
  HttpResponse resp;
  CHECK(c.round_trip(req, &resp).ok());  // transparent reconnect
  CHECK_EQ(c.stats().connects, uint64_t(2));
  srv.stop();
}

// set_on_wire: the work runs once, after the request is written (the server may already hold
// it) and before the response is read; a request the work makes itself does not run it again;
// a request that never reaches the wire leaves it pending; clear_on_wire drops it.
TEST(http_on_wire_hook) {
  HttpServer srv([](const HttpRequest& req, HttpResponse* resp) {
    resp->status = 200;
    resp->body = req.target;
  });
  CHECK(srv.listen("127.0.0.1", 0).ok());
  auto u = parse_url("http://127.0.0.1:" + std::to_string(srv.port()));
  HttpClient a(u.value, TlsOptions{}, 5 * kSecond), b(u.value, TlsOptions{}, 5 * kSecond);
  struct Ctx {
    HttpClient* other;
    int runs = 0;
    bool inner_ok = false;
  } ctx{&b};
  auto work = [](void* p) {
    auto* c = static_cast<Ctx*>(p);
    c->runs++;
    HttpRequest r;
    r.target = "/inner";
    c->inner_ok = c->other->send(r).ok();  // an HTTP request from inside the hook
  };
  set_on_wire(work, &ctx);
  CHECK(on_wire_pending());
  HttpRequest req;
  req.target = "/outer";
  HttpResponse resp;
  CHECK(a.round_trip(req, &resp).ok());
  CHECK_EQ(resp.body, std::string("/outer"));
  CHECK_EQ(ctx.runs, 1);
  CHECK(ctx.inner_ok);
  CHECK(!on_wire_pending());
  HttpResponse inner;
  CHECK(b.receive(&inner).ok());
  CHECK_EQ(inner.body, std::string("/inner"));
  CHECK(a.round_trip(req, &resp).ok());  // one-shot
  CHECK_EQ(ctx.runs, 1);
  // nothing listens there: the request never reaches the wire, the work stays pending
  auto dead = parse_url("http://127.0.0.1:1");
  HttpClient c(dead.value, TlsOptions{}, 200 * kMillisecond);
  set_on_wire(work, &ctx);
  CHECK(!c.round_trip(req, &resp).ok());
  CHECK_EQ(ctx.runs, 1);
  CHECK(on_wire_pending());
  clear_on_wire();
  CHECK(!on_wire_pending());
  srv.stop();
}

TEST(http_tls_roundtrip) {
  std::string cert, key;
  CHECK(generate_self_signed("127.0.0.1", &cert, &key).ok());
  HttpServer srv([](const HttpRequest&, HttpResponse* resp) {
    resp->status = 200;
    resp->body = "tls-ok";
  });
  CHECK(srv.enable_tls(cert, key).ok());
  CHECK(srv.listen("127.0.0.1", 0).ok());
  auto u = parse_url("https://127.0.0.1:" + std::to_string(srv.port()));
  TlsOptions tls;
  tls.ca_pem = cert;
  HttpClient c(u.value, tls, 5 * kSecond);
  for (int i = 0; i < 5; ++i) {
    HttpRequest req;
    HttpResponse resp;
    CHECK(c.round_trip(req, &resp).ok());
    CHECK_EQ(resp.body, std::string("tls-ok"));
  }
  srv.drop_connections();  // reconnect must resume the TLS session
  {
    HttpRequest req;
    HttpResponse resp;
    CHECK(c.round_trip(req, &resp).ok());
    CHECK_EQ(c.stats().tls_resumptions, uint64_t(1));
  }
  HttpClient bad(u.value, TlsOptions{}, 5 * kSecond);  // no CA: must fail verification
  HttpRequest req;
  HttpResponse resp;
  CHECK(!bad.round_trip(req, &resp).ok());
  srv.stop();
}

// Minimal CONNECT relay (one tunnel): records the request head, dials the target, relays bytes.
class ConnectRelay {
 public:
  // With a certificate, the relay is an https:// proxy: clients reach it over TLS.
  explicit ConnectRelay(const std::string& cert_pem = "", const std::string& key_pem = "") {
    if (!cert_pem.empty()) {
      ctx_ = SSL_CTX_new(TLS_server_method());
      BIO* cb = BIO_new_mem_buf(cert_pem.data(), static_cast<int>(cert_pem.size()));
      X509* x = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr);
      BIO* kb = BIO_new_mem_buf(key_pem.data(), static_cast<int>(key_pem.size()));
      EVP_PKEY* k = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
      SSL_CTX_use_certificate(ctx_, x);
      SSL_CTX_use_PrivateKey(ctx_, k);
      X509_free(x);
      EVP_PKEY_free(k);
      BIO_free(cb);
      BIO_free(kb);
    }
    lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    ::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof a);
    ::listen(lfd_, 4);
    socklen_t len = sizeof a;
    getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &len);
    port_ = ntohs(a.sin_port);
    th_ = std::thread([this] { run(); });
  }
  ~ConnectRelay() {
    ::shutdown(lfd_, SHUT_RDWR);
    th_.join();
    ::close(lfd_);
    if (ctx_) SSL_CTX_free(ctx_);
  }
  int port() const { return port_; }
  std::string head() {
    std::lock_guard<std::mutex> lk(mu_);
    return head_;
  }

 private:
  // Client side of the relay: plain socket or (https proxy) a blocking TLS session on it.
  ssize_t crecv(int c, char* b, size_t n) { return ssl_ ? SSL_read(ssl_, b, static_cast<int>(n)) : ::recv(c, b, n, 0); }
  ssize_t csend(int c, const char* b, size_t n) {
    return ssl_ ? SSL_write(ssl_, b, static_cast<int>(n)) : ::send(c, b, n, MSG_NOSIGNAL);
  }

  void run() {
    int c = ::accept(lfd_, nullptr, nullptr);
    if (c < 0) return;
    if (ctx_) {
      ssl_ = SSL_new(ctx_);
      SSL_set_fd(ssl_, c);
      if (SSL_accept(ssl_) != 1) {
        SSL_free(ssl_);
        ssl_ = nullptr;
        ::close(c);
        return;
      }
    }
    std::string buf;
    char tmp[4096];
    while (buf.find("\r\n\r\n") == std::string::npos) {
      ssize_t n = crecv(c, tmp, sizeof tmp);
      if (n <= 0) {
        if (ssl_) SSL_free(ssl_);
        ssl_ = nullptr;
        ::close(c);
        return;
      }
      buf.append(tmp, static_cast<size_t>(n));
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      head_ = buf.substr(0, buf.find("\r\n\r\n"));
    }
    // "CONNECT 127.0.0.1:PORT HTTP/1.1"
    const size_t colon = buf.find(':'), sp = buf.find(' ', colon);
    const int up_port = std::atoi(buf.substr(colon + 1, sp - colon - 1).c_str());
    int u = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons(static_cast<uint16_t>(up_port));
    if (::connect(u, reinterpret_cast<sockaddr*>(&a), sizeof a) == 0) {
      const char ok[] = "HTTP/1.1 200 Connection established\r\n\r\n";
      csend(c, ok, sizeof ok - 1);
      pollfd p[2] = {{c, POLLIN, 0}, {u, POLLIN, 0}};
      while ((ssl_ && SSL_pending(ssl_) > 0) || ::poll(p, 2, 5000) > 0) {
        bool done = false;
        if ((ssl_ && SSL_pending(ssl_) > 0) || (p[0].revents & (POLLIN | POLLHUP | POLLERR))) {
          ssize_t n = crecv(c, tmp, sizeof tmp);
          if (n <= 0 || ::send(u, tmp, static_cast<size_t>(n), MSG_NOSIGNAL) != n) done = true;
        }
        if (p[1].revents & (POLLIN | POLLHUP | POLLERR)) {
          ssize_t n = ::recv(u, tmp, sizeof tmp, 0);
          if (n <= 0 || csend(c, tmp, static_cast<size_t>(n)) != n) done = true;
        }
        p[0].revents = p[1].revents = 0;
        if (done) break;
      }
    }
    ::close(u);
    if (ssl_) SSL_free(ssl_);
    ssl_ = nullptr;
    ::close(c);
  }

  int lfd_ = -1, port_ = 0;
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
  std::thread th_;
  std::mutex mu_;
  std::string head_;
};

TEST(http_tls_through_connect_proxy) {
  std::string cert, key;
  CHECK(generate_self_signed("127.0.0.1", &cert, &key).ok());
  HttpServer srv([](const HttpRequest& req, HttpResponse* resp) {
    resp->status = 200;
    resp->body = "via-proxy " + req.target;
  });
  CHECK(srv.enable_tls(cert, key).ok());
  CHECK(srv.listen("127.0.0.1", 0).ok());
  ConnectRelay relay;
  TlsOptions tls;
  tls.ca_pem = cert;
  HttpClient c(parse_url("https://127.0.0.1:" + std::to_string(srv.port())).value, tls, 5 * kSecond);
  CHECK(c.set_proxy("http://user:p%40ss@127.0.0.1:" + std::to_string(relay.port())).ok());
  for (int i = 0; i < 3; ++i) {
    HttpRequest req;
    req.target = "/x";
    HttpResponse resp;
    CHECK(c.round_trip(req, &resp).ok());
    CHECK_EQ(resp.body, std::string("via-proxy /x"));
  }
  CHECK_EQ(c.stats().connects, uint64_t(1));
  const std::string head = relay.head();
  CHECK(head.rfind("CONNECT 127.0.0.1:" + std::to_string(srv.port()) + " HTTP/1.1\r\n", 0) == 0);
  CHECK(head.find("Proxy-Authorization: Basic dXNlcjpwQHNz") != std::string::npos);  // user:p@ss
  CHECK(!c.set_proxy("ftp://127.0.0.1:1").ok());
  c.close();
  srv.stop();
}

// https:// proxy: TLS to the proxy, then the origin's TLS inside it (the tunnel BIO), under
// the sanitizer builds too.
TEST(http_tls_inside_tls_proxy) {
  std::string cert, key, pcert, pkey;
  CHECK(generate_self_signed("127.0.0.1", &cert, &key).ok());
  CHECK(generate_self_signed("127.0.0.1", &pcert, &pkey).ok());
  HttpServer srv([](const HttpRequest& req, HttpResponse* resp) {
    resp->status = 200;
    resp->body = std::string(70000, 'z') + req.target;  // several TLS records each way
  });
  CHECK(srv.enable_tls(cert, key).ok());
  CHECK(srv.listen("127.0.0.1", 0).ok());
  ConnectRelay relay(pcert, pkey);
  TlsOptions tls;
  tls.ca_pem = cert + pcert;
  HttpClient c(parse_url("https://127.0.0.1:" + std::to_string(srv.port())).value, tls, 5 * kSecond);
  CHECK(c.set_proxy("https://127.0.0.1:" + std::to_string(relay.port())).ok());
  for (int i = 0; i < 3; ++i) {
    HttpRequest req;
    req.method = "POST";
    req.target = "/y" + std::to_string(i);
    req.body = std::string(50000, 'q');
    HttpResponse resp;
    CHECK(c.round_trip(req, &resp).ok());
    CHECK_EQ(resp.body.size(), size_t(70003));
    CHECK_EQ(resp.body.substr(70000), "/y" + std::to_string(i));
  }
  CHECK_EQ(c.stats().connects, uint64_t(1));
  CHECK(relay.head().rfind("CONNECT 127.0.0.1:" + std::to_string(srv.port()) + " HTTP/1.1\r\n", 0) == 0);
  c.close();
  srv.stop();
}

TEST(http_timeout) {
  HttpServer srv([](const HttpRequest&, HttpResponse* resp) {
    std::this_thread::sleep_for(std::chrono::milliseconds(300));
    resp->status = 200;
  });
  CHECK(srv.listen("127.0.0.1", 0).ok());
  auto u = parse_url("http://127.0.0.1:" + std::to_string(srv.port()));
  HttpClient c(u.value, TlsOptions{}, 50 * kMillisecond);
  HttpRequest req;
  HttpResponse resp;
  CHECK(!c.round_trip(req, &resp).ok());
  srv.stop();
}

// Eight queues on eight native worker threads against shared threaded fake servers: the
// concurrency the reference never ran under a race detector.
TEST(supervisor_multi_queue_over_wire) {
  FakeSqsServer sqs;
  sqs.require_signature("AKID", "SECRET", "us-east-1");
  CHECK(sqs.start().ok());
  FakeKubeServer kube;
  kube.require_token("tok");
  CHECK(kube.start().ok());
  auto clock = std::make_shared<RealClock>();
  auto log = quiet_logger();
  Credentials cr;
  cr.access_key_id = "AKID";
  cr.secret_access_key = "SECRET";
  auto creds = std::make_shared<StaticCredentialsProvider>(cr);
  Supervisor sup;
  const int kQueues = 8, kIters = 40;
  for (int q = 0; q < kQueues; ++q) {
    std::string url = sqs.url() + "/1/q" + std::to_string(q);
    sqs.set_attribute_cycle(url, {attrs(150), attrs(0)});
    kube.add_deployment("ns", "w" + std::to_string(q), 1);
    SqsHttpOptions so;
    so.region = "us-east-1";
    so.endpoint = sqs.url();
    so.protocol = (q % 2) ? SqsProtocol::Json : SqsProtocol::Query;
    auto api = std::make_shared<HttpSqsApi>(so, creds, clock);
    KubeOptions ko;
    ko.server = kube.url();
    ko.namespace_ = "ns";
    ko.mode = static_cast<ScaleMode>(q % 3);
    ko.token = std::make_shared<StaticTokenProvider>("tok");
    auto dep = std::make_shared<KubeRestDeployments>(ko);
    auto scaler = std::make_shared<PodAutoScaler>(dep, "w" + std::to_string(q), "ns", 8, 1, 1, 1, log, clock);
    LoopConfig lc;
    lc.poll_period = 0;
    lc.scale_up_cool_down = 0;
    lc.scale_down_cool_down = 0;
    sup.add(std::make_shared<Runner>(lc, std::make_shared<SqsClient>(api, url, default_attribute_names()), scaler,
                                     clock, log));
  }
  sup.start(kIters);
  CHECK(sup.wait(60 * kSecond));
  sup.join();
  for (int q = 0; q < kQueues; ++q) {
    auto st = sup.runner(q)->stats();
    CHECK_EQ(st.polls, uint64_t(kIters));
    CHECK_EQ(st.scale_ups, uint64_t(kIters / 2));
    CHECK_EQ(st.scale_downs, uint64_t(kIters / 2));
    CHECK_EQ(kube.replicas("ns", "w" + std::to_string(q)), 1);
    CHECK_EQ(sup.runner(q)->latencies().size(), size_t(kIters));
  }
  CHECK_EQ(sqs.signature_failures(), uint64_t(0));
  sqs.stop();
  kube.stop();
}

TEST(supervisor_stop_interrupts_sleep) {
  auto clock = std::make_shared<RealClock>();
  auto log = quiet_logger();
  auto api = std::make_shared<MockSqsApi>(attrs(0));
  auto fake = std::make_shared<FakeDeployments>("ns");
  fake->add("w", 1);
  Supervisor sup;
  LoopConfig lc;
  lc.poll_period = 3600 * kSecond;
  for (int i = 0; i < 4; ++i)
    sup.add(std::make_shared<Runner>(lc, std::make_shared<SqsClient>(api, "q", default_attribute_names()),
                                     std::make_shared<PodAutoScaler>(fake, "w", "ns", 8, 1, 1, 1, log, clock), clock,
                                     log));
  sup.start();
  CHECK(!sup.wait(50 * kMillisecond));
  sup.stop();
  CHECK(sup.wait(5 * kSecond));
  sup.join();
  CHECK_EQ(api->calls(), uint64_t(0));
}

// Runners outlive their supervisors and keep their HomeThread: three supervisors in a row over
// the same runners (the last one stopped mid-run), a second start() on a busy runner waiting for
// the first run, then the runners dropped -- the threads end with them (TSan target).
TEST(supervisor_runs_reuse_home_threads) {
  auto clock = std::make_shared<RealClock>();
  auto log = quiet_logger();
  auto fake = std::make_shared<FakeDeployments>("ns");
  std::vector<std::shared_ptr<Runner>> runners;
  LoopConfig lc;
  lc.poll_period = 0;
  lc.scale_up_cool_down = 0;
  lc.scale_down_cool_down = 0;
  for (int i = 0; i < 4; ++i) {
    fake->add("w" + std::to_string(i), 1);
    auto api = std::make_shared<MockSqsApi>(attrs(150));
    runners.push_back(std::make_shared<Runner>(
        lc, std::make_shared<SqsClient>(api, "q", default_attribute_names()),
        std::make_shared<PodAutoScaler>(fake, "w" + std::to_string(i), "ns", 8, 1, 1, 1, log, clock), clock, log));
  }
  for (int round = 0; round < 2; ++round) {
    Supervisor sup;
    for (auto& r : runners) sup.add(r);
    sup.start(25);
    CHECK(sup.wait(10 * kSecond));
    sup.join();
    CHECK_EQ(sup.thread_sched().threads, int64_t(4));
  }
  for (auto& r : runners) CHECK_EQ(r->stats().polls, uint64_t(50));
  {
    Supervisor sup;
    for (auto& r : runners) sup.add(r);
    sup.start(100);
    sup.start(10);  // waits for each runner's first run, then runs again
    CHECK(sup.wait(10 * kSecond));
    sup.join();
  }
  for (auto& r : runners) CHECK_EQ(r->stats().polls, uint64_t(160));
  {
    Supervisor sup;
    for (auto& r : runners) sup.add(r);
    sup.start();  // until stopped
    sup.stop();
    CHECK(sup.wait(5 * kSecond));
  }  // ~Supervisor joins
  runners.clear();  // ~Runner ends each HomeThread
}

// 32 queues on 3 workers against the threaded fakes (TSan target for the scheduler heap).
TEST(scheduler_many_queues_few_threads) {
  FakeSqsServer sqs;
  CHECK(sqs.start().ok());
  FakeKubeServer kube;
  CHECK(kube.start().ok());
  auto clock = std::make_shared<RealClock>();
  auto log = quiet_logger();
  Credentials cr;
  cr.access_key_id = "AKID";
  cr.secret_access_key = "SECRET";
  auto creds = std::make_shared<StaticCredentialsProvider>(cr);
  Scheduler sched(3, clock);
  const int kQueues = 32, kIters = 10;
  for (int q = 0; q < kQueues; ++q) {
    std::string url = sqs.url() + "/1/s" + std::to_string(q);
    sqs.set_attribute_cycle(url, {attrs(150), attrs(0)});
    kube.add_deployment("ns", "s" + std::to_string(q), 1);
    SqsHttpOptions so;
    so.region = "us-east-1";
    so.endpoint = sqs.url();
    auto api = std::make_shared<HttpSqsApi>(so, creds, clock);
    KubeOptions ko;
    ko.server = kube.url();
    ko.namespace_ = "ns";
    auto dep = std::make_shared<KubeRestDeployments>(ko);
    auto scaler = std::make_shared<PodAutoScaler>(dep, "s" + std::to_string(q), "ns", 8, 1, 1, 1, log, clock);
    LoopConfig lc;
    lc.poll_period = kMillisecond;
    lc.scale_up_cool_down = 0;
    lc.scale_down_cool_down = 0;
    lc.prefetch = (q % 2) == 0;
    sched.add(std::make_shared<Runner>(lc, std::make_shared<SqsClient>(api, url, default_attribute_names()), scaler,
                                       clock, log));
  }
  sched.start(kIters);
  CHECK(sched.wait(60 * kSecond));
  sched.join();
  for (int q = 0; q < kQueues; ++q) {
    auto st = sched.runner(q)->stats();
    CHECK_EQ(st.polls, uint64_t(kIters));
    CHECK_EQ(st.scale_ups + st.scale_downs, uint64_t(kIters));
  }
  sqs.stop();
  kube.stop();
}

// --poll-prewarm over the wire (TSan target): dedicated threads wake early, sign, check both
// connections and spin to the due time; pooled threads run the warm-up as an event of its own
// before each poll. Decisions and poll counts are those without it; a period under 2x the
// warm-up takes the at-due-time branch.
TEST(prewarm_over_wire_dedicated_and_pooled) {
  FakeSqsServer sqs;
  sqs.require_signature("AKID", "SECRET", "us-east-1");
  CHECK(sqs.start().ok());
  FakeKubeServer kube;
  kube.require_token("tok");
  CHECK(kube.start().ok());
  auto clock = std::make_shared<RealClock>();
  auto log = quiet_logger();
  Credentials cr;
  cr.access_key_id = "AKID";
  cr.secret_access_key = "SECRET";
  auto creds = std::make_shared<StaticCredentialsProvider>(cr);
  const int kQueues = 6, kIters = 12;
  auto make = [&](const std::string& tag, int q) {
    std::string url = sqs.url() + "/1/" + tag + std::to_string(q);
    sqs.set_attribute_cycle(url, {attrs(150), attrs(0)});
    kube.add_deployment("ns", tag + std::to_string(q), 1);
    SqsHttpOptions so;
    so.region = "us-east-1";
    so.endpoint = sqs.url();
    auto api = std::make_shared<HttpSqsApi>(so, creds, clock);
    KubeOptions ko;
    ko.server = kube.url();
    ko.namespace_ = "ns";
    ko.token = std::make_shared<StaticTokenProvider>("tok");
    auto dep = std::make_shared<KubeRestDeployments>(ko);
    auto scaler = std::make_shared<PodAutoScaler>(dep, tag + std::to_string(q), "ns", 8, 1, 1, 1, log, clock);
    LoopConfig lc;
    lc.poll_period = (q % 3 == 2) ? 300 * kMicrosecond : 2 * kMillisecond;  // the last: under 2x prewarm
    lc.prewarm = 250 * kMicrosecond;
    lc.scale_up_cool_down = 0;
    lc.scale_down_cool_down = 0;
    lc.prefetch = (q % 2) == 0;
    return std::make_shared<Runner>(lc, std::make_shared<SqsClient>(api, url, default_attribute_names()), scaler,
                                    clock, log);
  };
  Supervisor sup;
  sup.set_stagger(true);
  Scheduler sched(2, clock);
  for (int q = 0; q < kQueues; ++q) {
    sup.add(make("d", q));
    sched.add(make("p", q));
  }
  sup.start(kIters);
  sched.start(kIters);
  CHECK(sup.wait(60 * kSecond));
  CHECK(sched.wait(60 * kSecond));
  sup.join();
  sched.join();
  for (int q = 0; q < kQueues; ++q) {
    for (const auto& r : {sup.runner(q), sched.runner(q)}) {
      auto st = r->stats();
      CHECK_EQ(st.polls, uint64_t(kIters));
      CHECK_EQ(st.scale_ups, uint64_t(kIters / 2));
      CHECK_EQ(st.scale_downs, uint64_t(kIters / 2));
      CHECK_EQ(st.depth_errors, uint64_t(0));
    }
    CHECK_EQ(kube.replicas("ns", "d" + std::to_string(q)), 1);
    CHECK_EQ(kube.replicas("ns", "p" + std::to_string(q)), 1);
  }
  CHECK_EQ(sqs.signature_failures(), uint64_t(0));
  sqs.stop();
  kube.stop();
}

TEST(scheduler_stop) {
  auto clock = std::make_shared<RealClock>();
  auto log = quiet_logger();
  auto api = std::make_shared<MockSqsApi>(attrs(0));
  auto fake = std::make_shared<FakeDeployments>("ns");
  fake->add("w", 1);
  Scheduler sched(2, clock);
  LoopConfig lc;
  lc.poll_period = 3600 * kSecond;
  for (int i = 0; i < 5; ++i)
    sched.add(std::make_shared<Runner>(lc, std::make_shared<SqsClient>(api, "q", default_attribute_names()),
                                       std::make_shared<PodAutoScaler>(fake, "w", "ns", 8, 1, 1, 1, log, clock), clock,
                                       log));
  sched.start();
  CHECK(!sched.wait(50 * kMillisecond));
  sched.stop();
  CHECK(sched.wait(5 * kSecond));
  sched.join();
  CHECK_EQ(api->calls(), uint64_t(0));
}

TEST(concurrent_logger_lines_are_whole) {
  auto lines = std::make_shared<std::vector<std::string>>();
  auto mu = std::make_shared<std::mutex>();
  auto log = std::make_shared<Logger>();
  log->set_sink([lines, mu](const std::string& l) {
    std::lock_guard<std::mutex> g(*mu);
    lines->push_back(l);
  });
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([log, t] {
      auto child = log->with_fields({{"queue", "q" + std::to_string(t)}});
      for (int i = 0; i < 200; ++i) child->info("Found " + std::to_string(i) + " messages in the queue");
    });
  for (auto& t : ts) t.join();
  CHECK_EQ(lines->size(), size_t(1600));
  for (auto& l : *lines) CHECK(l.rfind("time=\"", 0) == 0 && l.find(" queue=q") != std::string::npos);
}

TEST(concurrent_fd_sink_lines_are_whole) {
  // The fd sink writes without the logger's mutex (one write(2) per line). 8 threads into one
  // pipe: every line must arrive whole, including one longer than PIPE_BUF (locked path).
  int p[2];
  CHECK_EQ(::pipe(p), 0);
  auto log = std::make_shared<Logger>();
  log->set_sink_fd(p[1]);
  std::string data;
  std::thread reader([&] {
    char buf[65536];
    ssize_t r;
    while ((r = ::read(p[0], buf, sizeof buf)) > 0) data.append(buf, static_cast<size_t>(r));
  });
  const std::string big(PIPE_BUF + 100, 'x');
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([log, t, &big] {
      auto child = log->with_fields({{"queue", "q" + std::to_string(t)}});
      for (int i = 0; i < 500; ++i) child->info("Found " + std::to_string(i) + " messages in the queue");
      if (t == 0) child->error(big);
    });
  for (auto& t : ts) t.join();
  ::close(p[1]);
  reader.join();
  ::close(p[0]);
  size_t n = 0, bigs = 0, start = 0;
  for (size_t nl; (nl = data.find('\n', start)) != std::string::npos; start = nl + 1, ++n) {
    std::string l = data.substr(start, nl - start);
    CHECK(l.rfind("time=\"", 0) == 0);
    if (l.find(big) != std::string::npos) {
      ++bigs;
      continue;
    }
    CHECK(l.find(" level=info msg=\"Found ") != std::string::npos);
    CHECK(l.size() > 8 && l.compare(l.size() - 8, 7, "queue=q") == 0);
  }
  CHECK_EQ(start, data.size());
  CHECK_EQ(n, size_t(4001));
  CHECK_EQ(bigs, size_t(1));
}

TEST(log_batch_holds_lines_until_end) {
  // Lines logged inside a LogBatch reach the fd only when the outermost batch ends, in order,
  // with their own timestamps; a fatal line flushes what is held first; batches of several
  // threads into one pipe (some over PIPE_BUF) arrive whole.
  int p[2];
  CHECK_EQ(::pipe(p), 0);
  auto log = std::make_shared<Logger>();
  log->set_sink_fd(p[1]);
  auto pending = [&] {
    int n = 0;
    CHECK_EQ(::ioctl(p[0], FIONREAD, &n), 0);
    return n;
  };
  {
    LogBatch outer;
    CHECK(LogBatch::active());
    log->info("Found 200 messages in the queue");
    {
      LogBatch inner;
      log->info("Scale up successful");
    }
    CHECK_EQ(pending(), 0);
    RealClock().sleep(0, nullptr);  // no wait: nothing flushed
    CHECK_EQ(pending(), 0);
  }
  CHECK(!LogBatch::active());
  std::string got(static_cast<size_t>(pending()), '\0');
  CHECK_EQ(::read(p[0], got.data(), got.size()), static_cast<ssize_t>(got.size()));
  const size_t a = got.find("msg=\"Found 200 messages in the queue\"\n");
  const size_t b = got.find("msg=\"Scale up successful\"\n");
  CHECK(a != std::string::npos && b != std::string::npos && a < b);
  CHECK(got.rfind("time=\"", 0) == 0 && got.back() == '\n');
  {
    LogBatch batch;
    log->info("first");
    log->log(Level::Fatal, "second");
    CHECK(pending() > 0);
    std::string now(static_cast<size_t>(pending()), '\0');
    CHECK_EQ(::read(p[0], now.data(), now.size()), static_cast<ssize_t>(now.size()));
    CHECK(now.find("msg=first") < now.find("msg=second"));
    log->info("third");
    CHECK_EQ(pending(), 0);
    RealClock().sleep(1000, nullptr);  // a deliberate wait writes out what is held
    CHECK(pending() > 0);
    std::string third(static_cast<size_t>(pending()), '\0');
    CHECK_EQ(::read(p[0], third.data(), third.size()), static_cast<ssize_t>(third.size()));
    CHECK(third.find("msg=third\n") != std::string::npos);
  }
  std::string data;
  std::thread reader([&] {
    char buf[65536];
    ssize_t r;
    while ((r = ::read(p[0], buf, sizeof buf)) > 0) data.append(buf, static_cast<size_t>(r));
  });
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([log, t] {
      auto child = log->with_fields({{"queue", "q" + std::to_string(t)}});
      for (int i = 0; i < 200; ++i) {
        LogBatch batch;  // 2 lines per batch; every 50th batch over PIPE_BUF
        child->info("Found " + std::to_string(i) + " messages in the queue");
        child->info(i % 50 == 0 ? std::string(PIPE_BUF, 'y') : std::string("Scale up successful"));
      }
    });
  for (auto& t : ts) t.join();
  ::close(p[1]);
  reader.join();
  ::close(p[0]);
  size_t n = 0, start = 0;
  for (size_t nl; (nl = data.find('\n', start)) != std::string::npos; start = nl + 1, ++n) {
    std::string l = data.substr(start, nl - start);
    CHECK(l.rfind("time=\"", 0) == 0);
    CHECK(l.size() > 8 && l.compare(l.size() - 8, 7, "queue=q") == 0);
  }
  CHECK_EQ(start, data.size());
  CHECK_EQ(n, size_t(3200));
}

TEST(token_bucket_concurrent_reservations) {
  // 8 threads x 50 reservations on one bucket: the wait each caller is handed is the queue
  // position beyond the burst, so the sum over all callers is fixed whatever the interleaving.
  auto clock = std::make_shared<VirtualClock>(0);
  TokenBucket b(1000.0, 100, clock);
  std::atomic<int64_t> total{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&] {
      for (int i = 0; i < 50; ++i) total += b.reserve();
    });
  for (auto& t : ts) t.join();
  // 400 reservations, 100 free, the k-th beyond waits k ms: sum_{k=1..300} k ms
  CHECK_EQ(total.load(), int64_t(300) * 301 / 2 * kMillisecond);
}

TEST(exec_provider_shared_across_threads) {
  // One authenticator shared by 8 workers: the plugin runs once, every thread gets its token.
  char dir[] = "/tmp/ksa_exec_XXXXXX";
  if (!mkdtemp(dir)) {
    CHECK(false);
    return;
  }
  const std::string script = std::string(dir) + "/plugin.sh";
  {
    std::FILE* f = std::fopen(script.c_str(), "w");
    std::fputs("#!/bin/sh\necho x >> \"$(dirname \"$0\")/runs\"\n"
               "echo '{\"kind\":\"ExecCredential\",\"apiVersion\":\"client.authentication.k8s.io/v1beta1\","
               "\"status\":{\"token\":\"tok-'$KSA_SUFFIX'\"}}'\n",
               f);
    std::fclose(f);
  }
  chmod(script.c_str(), 0755);
  ExecConfig cfg;
  cfg.command = script;
  cfg.api_version = "client.authentication.k8s.io/v1beta1";
  cfg.env = {{"KSA_SUFFIX", "42"}};
  cfg.timeout = 10 * kSecond;
  auto p = std::make_shared<ExecTokenProvider>(cfg, std::make_shared<RealClock>());
  std::atomic<int> good{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&] {
      for (int i = 0; i < 20; ++i) {
        auto r = p->token();
        if (r.ok() && r.value == "tok-42") ++good;
      }
    });
  for (auto& t : ts) t.join();
  CHECK_EQ(good.load(), 160);
  CHECK_EQ(p->runs(), uint64_t(1));
  p->invalidate("tok-42");
  CHECK(p->token().ok());
  CHECK_EQ(p->runs(), uint64_t(2));
  // A plugin that fails slowly: the 8 threads asking at once share one run's error instead of
  // running it one after another (8 x 300 ms).
  const std::string failing = std::string(dir) + "/failing.sh";
  {
    std::FILE* f = std::fopen(failing.c_str(), "w");
    std::fputs("#!/bin/sh\nsleep 0.3\necho 'no credentials' >&2\nexit 3\n", f);
    std::fclose(f);
  }
  chmod(failing.c_str(), 0755);
  cfg.command = failing;
  auto q = std::make_shared<ExecTokenProvider>(cfg, std::make_shared<RealClock>());
  std::atomic<int> failed{0};
  std::atomic<bool> go{false};
  ts.clear();
  const int64_t t0 = mono_ns();
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&] {
      while (!go) std::this_thread::yield();
      if (!q->token().ok()) ++failed;
    });
  go = true;
  for (auto& t : ts) t.join();
  CHECK_EQ(failed.load(), 8);
  CHECK(q->runs() <= uint64_t(2));
  CHECK(mono_ns() - t0 < 1500 * kMillisecond);
  // A hanging plugin: a stopping client's cancel() kills the run, which ends with "request
  // canceled" for it and its waiters, long before the plugin timeout.
  const std::string hanging = std::string(dir) + "/hanging.sh";
  {
    std::FILE* f = std::fopen(hanging.c_str(), "w");
    std::fputs("#!/bin/sh\nexec sleep 30\n", f);
    std::fclose(f);
  }
  chmod(hanging.c_str(), 0755);
  cfg.command = hanging;
  cfg.timeout = 20 * kSecond;
  auto h = std::make_shared<ExecTokenProvider>(cfg, std::make_shared<RealClock>());
  std::atomic<int> canceled{0};
  ts.clear();
  const int64_t t1 = mono_ns();
  for (int t = 0; t < 3; ++t)
    ts.emplace_back([&] {
      auto r = h->token();
      if (!r.ok() && r.status.message() == "request canceled") ++canceled;
    });
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  h->cancel();
  for (auto& t : ts) t.join();
  CHECK_EQ(canceled.load(), 3);
  CHECK(mono_ns() - t1 < 3 * kSecond);
  CHECK_EQ(h->runs(), uint64_t(1));
  std::remove(hanging.c_str());
  std::remove(failing.c_str());
  std::remove((std::string(dir) + "/runs").c_str());
  std::remove(script.c_str());
  rmdir(dir);
}

// One credential source shared by 16 clients' caches on 16 threads (the CLI's 16 tracked
// queues): the inner provider runs once per expiry, whatever the concurrency, and a stale report
// about an older set is ignored (TSan target: the caches and the shared copy under their locks).
TEST(shared_credentials_one_fetch_per_expiry) {
  struct Counting final : CredentialsProvider {
    std::atomic<int> calls{0};
    std::atomic<int64_t>* now;
    Result<Credentials> retrieve() override {
      const int n = ++calls;
      Credentials c;
      c.access_key_id = "AKID";
      c.secret_access_key = "secret";
      c.session_token = "tok-" + std::to_string(n);
      c.expires_unix_ns = now->load() + 600 * kSecond;
      return Result<Credentials>::Ok(c);
    }
  };
  std::atomic<int64_t> now{1700000000LL * kSecond};
  auto inner = std::make_shared<Counting>();
  inner->now = &now;
  auto shared = std::make_shared<SharedCredentialsProvider>(inner, [&now] { return now.load(); }, 300 * kSecond);
  std::vector<std::unique_ptr<CachedCredentials>> caches;
  for (int i = 0; i < 16; ++i) caches.push_back(std::make_unique<CachedCredentials>(shared, 300 * kSecond));
  auto round = [&](const std::string& want) {
    std::atomic<int> good{0};
    std::vector<std::thread> ts;
    for (int i = 0; i < 16; ++i)
      ts.emplace_back([&, i] {
        for (int k = 0; k < 50; ++k) {
          auto r = caches[i]->get(now.load());
          if (r.ok() && r.value.session_token == want) ++good;
        }
      });
    for (auto& t : ts) t.join();
    CHECK_EQ(good.load(), 16 * 50);
  };
  round("tok-1");
  CHECK_EQ(inner->calls.load(), 1);
  now += 301 * kSecond;  // 299 s left: every cache is in its refresh window
  round("tok-2");
  CHECK_EQ(inner->calls.load(), 2);
  caches[3]->invalidate();  // ExpiredToken on one client: one re-fetch for all
  auto r = caches[3]->get(now.load());
  CHECK(r.ok() && r.value.session_token == "tok-3");
  CHECK_EQ(inner->calls.load(), 3);
  caches[5]->invalidate();  // a late report about tok-2 (already replaced): no fetch
  r = caches[5]->get(now.load());
  CHECK(r.ok() && r.value.session_token == "tok-3");
  CHECK_EQ(inner->calls.load(), 3);
  CHECK_EQ(shared->fetches(), uint64_t(3));
}

// Against a credential endpoint that fails slowly (a hung ECS / IMDS answering with a timeout),
// the clients asking at once share the one fetch's error instead of queueing a fetch each: one
// inner call, every caller's answer within about one fetch's time.
TEST(shared_credentials_share_a_failing_fetch) {
  struct SlowFailing final : CredentialsProvider {
    std::atomic<int> calls{0};
    Result<Credentials> retrieve() override {
      calls++;
      std::this_thread::sleep_for(std::chrono::milliseconds(150));
      return Result<Credentials>::Err(Status::Err("EC2RoleRequestError: timed out"));
    }
  };
  auto inner = std::make_shared<SlowFailing>();
  auto shared = std::make_shared<SharedCredentialsProvider>(inner, [] { return int64_t(0); }, 0);
  std::atomic<int> failed{0};
  const int64_t t0 = mono_ns();
  std::vector<std::thread> clients;
  std::atomic<bool> go{false};
  for (int i = 0; i < 8; ++i)
    clients.emplace_back([&] {
      while (!go) std::this_thread::yield();
      auto r = shared->retrieve();
      if (!r.ok() && r.status.message() == "EC2RoleRequestError: timed out") ++failed;
    });
  go = true;
  for (auto& t : clients) t.join();
  const int64_t took = mono_ns() - t0;
  CHECK_EQ(failed.load(), 8);
  CHECK(inner->calls.load() <= 2);  // one, or two for a caller that arrived after the first ended
  CHECK(took < 600 * kMillisecond);  // not 8 x 150 ms
  // the next poll's ask is a fresh fetch (nothing cached from an error)
  (void)shared->retrieve();
  CHECK(inner->calls.load() <= 3 && shared->fetches() == static_cast<uint64_t>(inner->calls.load()));
}

// The process fleet's credential slot (cred_slot.h): a supervisor thread publishing sets of
// varying sizes while worker threads read them never yields a torn set (every field of a read
// comes from one publication), and a waiting worker gets the next generation (TSan target: all
// shared words are atomics, as across processes).
TEST(credential_slot_seqlock) {
  auto mem = std::make_unique<SharedCredentialSlot>();
  SharedCredentialSlot* slot = init_credential_slot(mem.get());
  Credentials c0;
  std::string e0;
  uint64_t g0 = 0;
  CHECK(!read_credential_slot(slot, &c0, &e0, &g0));  // nothing published yet
  std::atomic<bool> done{false};
  std::atomic<int> torn{0}, reads{0};
  std::thread writer([&] {
    for (int i = 1; i <= 3000; ++i) {
      Credentials c;
      c.access_key_id = "AKID" + std::to_string(i);
      c.secret_access_key = "secret-" + std::to_string(i);
      c.session_token = std::string(static_cast<size_t>(i % 700), 't') + std::to_string(i);
      c.expires_unix_ns = i;
      publish_credentials(slot, c);
      while (i == 1 && reads.load() == 0) std::this_thread::yield();  // the readers overlap the rest
    }
    done = true;
  });
  std::vector<std::thread> readers;
  for (int r = 0; r < 4; ++r)
    readers.emplace_back([&] {
      int mine = 0;
      while (!done || mine == 0) {
        Credentials c;
        std::string e;
        uint64_t g = 0;
        if (!read_credential_slot(slot, &c, &e, &g)) continue;
        ++reads;
        ++mine;
        const std::string n = std::to_string(c.expires_unix_ns);
        if (c.access_key_id != "AKID" + n || c.secret_access_key != "secret-" + n ||
            c.session_token.size() < n.size() || c.session_token.substr(c.session_token.size() - n.size()) != n)
          ++torn;
      }
    });
  writer.join();
  for (auto& t : readers) t.join();
  CHECK_EQ(torn.load(), 0);
  CHECK(reads.load() > 0);
  Credentials last;
  std::string err;
  uint64_t gen = 0;
  CHECK(read_credential_slot(slot, &last, &err, &gen) && gen == 3000 && last.expires_unix_ns == 3000);
  // a worker whose set is within its window asks, and waits for the supervisor's next one
  SlotCredentialsProvider worker(slot, [] { return int64_t(2990); }, 100, 5 * kSecond);
  CHECK(!credential_slot_needs_fetch(slot, 0, 0));
  std::thread supervisor([&] {
    while (!credential_slot_needs_fetch(slot, 0, 0)) std::this_thread::yield();
    Credentials next;
    next.access_key_id = "AKIDnext";
    next.secret_access_key = "s";
    next.expires_unix_ns = 1 << 30;
    publish_credentials(slot, next);
  });
  auto r = worker.retrieve();
  supervisor.join();
  CHECK(r.ok() && r.value.access_key_id == "AKIDnext");
  publish_credential_error(slot, "STS said no");
  CHECK(read_credential_slot(slot, &last, &err, &gen) && err == "STS said no" && gen == 3002);
}

// HttpClient::spin_window_for: no answer slower than kMaxSpinThrough is ever spun for, and no
// spin exceeds it, whatever the budget.
// A worker waiting for its supervisor's first set (an empty slot) stops waiting when its API is
// cancelled (Runner::stop -> HttpSqsApi::cancel -> CachedCredentials -> the provider), instead of
// holding the worker's shutdown for the whole wait limit.
TEST(credential_slot_wait_cancels) {
  auto mem = std::make_unique<SharedCredentialSlot>();
  SharedCredentialSlot* slot = init_credential_slot(mem.get());
  auto provider = std::make_shared<SlotCredentialsProvider>(slot, [] { return int64_t(0); }, 0, 30 * kSecond);
  CachedCredentials cache(provider, 0);
  const int64_t t0 = mono_ns();
  std::thread stopper([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    cache.cancel();  // while get() waits in retrieve() under the cache's lock
  });
  auto r = cache.get(0);
  stopper.join();
  const int64_t waited = mono_ns() - t0;
  CHECK(!r.ok() && r.status.message() == "request canceled");
  CHECK(waited < 5 * kSecond);
  CHECK(credential_slot_needs_fetch(slot, 0, 0));  // the request stays asked for
}

// After the service rejects a set (stale()), no worker of the slot signs with it again -- not
// even before the supervisor has looked at the slot -- and the next retrieve() waits for the
// replacement (the SDK expires its cache before retrying).
TEST(credential_slot_rejected_set_not_resigned) {
  auto mem = std::make_unique<SharedCredentialSlot>();
  SharedCredentialSlot* slot = init_credential_slot(mem.get());
  Credentials first;
  first.access_key_id = "AKIDold";
  first.secret_access_key = "s";
  first.expires_unix_ns = 3600 * kSecond;
  publish_credentials(slot, first);
  SlotCredentialsProvider a(slot, [] { return int64_t(0); }, 300 * kSecond, 5 * kSecond);
  SlotCredentialsProvider b(slot, [] { return int64_t(0); }, 300 * kSecond, 200 * kMillisecond);
  auto r = a.retrieve();
  CHECK(r.ok() && r.value.access_key_id == "AKIDold");
  a.stale(r.value);
  CHECK(slot->rejected.load() == 1 && credential_slot_needs_fetch(slot, 0, 0));
  CHECK(!credential_slot_still_signs(slot, 0, kStaleSkew));
  auto rb = b.retrieve();  // nobody answers: an error, not the rejected set
  CHECK(!rb.ok() && rb.status.message().find("NoCredentialProviders") == 0);
  std::thread supervisor([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    Credentials next = first;
    next.access_key_id = "AKIDnew";
    publish_credentials(slot, next);
  });
  auto ra = a.retrieve();
  supervisor.join();
  CHECK(ra.ok() && ra.value.access_key_id == "AKIDnew");
}

// A refresh that failed while the set still signs: the supervisor republishes the set with the
// error and the workers, inside their window, sign with it at once (counted) until the set is
// within the skew of its expiry; then they ask, and the chain's error reaches them.
TEST(credential_slot_rides_out_a_failed_refresh) {
  auto mem = std::make_unique<SharedCredentialSlot>();
  SharedCredentialSlot* slot = init_credential_slot(mem.get());
  Credentials c;
  c.access_key_id = "AKID";
  c.secret_access_key = "s";
  c.expires_unix_ns = 420 * kSecond;
  publish_credentials(slot, c);
  std::atomic<int64_t> now{130 * kSecond};  // inside the 5-minute window
  SlotCredentialsProvider w(slot, [&] { return now.load(); }, 300 * kSecond, 2 * kSecond);
  CHECK(credential_slot_still_signs(slot, now, kStaleSkew));
  publish_credentials(slot, c, "EcsCredentialsError: 500");
  const int64_t t0 = mono_ns();
  CachedCredentials cache(std::shared_ptr<CredentialsProvider>(&w, [](CredentialsProvider*) {}), 300 * kSecond);
  for (int i = 0; i < 100; ++i) {
    auto r = cache.get(now);
    CHECK(r.ok() && r.value.kept_after_failed_refresh);
    if (i % 2 == 0) cache.signed_with(r.value);  // half the gets sign a request (warm-ups do not)
  }
  CHECK(mono_ns() - t0 < kSecond);  // no waits
  CHECK_EQ(slot->stale_signs.load(), uint64_t(50));
  CHECK(!credential_slot_needs_fetch(slot, now, 0));  // nobody had to ask
  now = 361 * kSecond;  // 59 s left: inside the skew
  CHECK(!credential_slot_still_signs(slot, now, kStaleSkew));
  std::thread supervisor([&] {
    while (!credential_slot_needs_fetch(slot, now, 0)) std::this_thread::yield();
    publish_credential_error(slot, "EcsCredentialsError: 500");
  });
  auto r = w.retrieve();
  supervisor.join();
  CHECK(!r.ok() && r.status.message() == "EcsCredentialsError: 500");
  CHECK_EQ(slot->stale_signs.load(), uint64_t(50));
}

// Nobody polls the slot: the supervisor's serving thread sleeps on `asks` and a worker's ask
// wakes it at once; a waiting worker sleeps on `published` and a publication wakes it at once.
TEST(credential_slot_futex_wakeups) {
  auto mem = std::make_unique<SharedCredentialSlot>();
  SharedCredentialSlot* slot = init_credential_slot(mem.get());
  const uint32_t seen = credential_slot_asks(slot);
  std::atomic<int64_t> woke_after{-1};
  std::thread supervisor([&] {
    const int64_t t0 = mono_ns();
    const uint32_t now_asks = credential_slot_wait_ask(slot, seen, 10 * kSecond);
    woke_after = mono_ns() - t0;
    CHECK(now_asks != seen);
    Credentials c;
    c.access_key_id = "AKID";
    c.secret_access_key = "s";
    publish_credentials(slot, c);
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  SlotCredentialsProvider w(slot, [] { return int64_t(0); }, 0, 10 * kSecond);
  const int64_t t0 = mono_ns();
  auto r = w.retrieve();  // asks (waking the supervisor), then sleeps until the publication
  const int64_t took = mono_ns() - t0;
  supervisor.join();
  CHECK(r.ok() && r.value.access_key_id == "AKID");
  CHECK(woke_after.load() >= 0 && woke_after.load() < 5 * kSecond);
  CHECK(took < kSecond);
  // a poke (the supervisor's stop) ends the wait without an ask
  std::thread stopper([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    credential_slot_poke(slot);
  });
  const int64_t t1 = mono_ns();
  credential_slot_wait_ask(slot, credential_slot_asks(slot), 10 * kSecond);
  stopper.join();
  CHECK(mono_ns() - t1 < 5 * kSecond);
}

// A library user's SharedCredentialsProvider rides out a failing refresh like the broker: inside
// the window the cached set is handed out (marked kept) while it has more than kStaleSkew left,
// the refresh retried every kKeptRetry, and the inner error surfaces only past the skew; a set the
// service rejected is never kept.
TEST(shared_provider_rides_out_a_failed_refresh) {
  struct Chain final : CredentialsProvider {
    std::atomic<int> calls{0};
    std::atomic<bool> fail{false};
    std::atomic<int64_t>* now;
    Result<Credentials> retrieve() override {
      ++calls;
      if (fail) return Result<Credentials>::Err(Status::Err("EcsCredentialsError: 500"));
      Credentials c;
      c.access_key_id = "AKID";
      c.secret_access_key = "s";
      c.session_token = "t" + std::to_string(calls.load());
      c.expires_unix_ns = now->load() + 420 * kSecond;
      return Result<Credentials>::Ok(c);
    }
  };
  std::atomic<int64_t> now{0};
  auto chain = std::make_shared<Chain>();
  chain->now = &now;
  SharedCredentialsProvider shared(chain, [&] { return now.load(); }, 300 * kSecond);
  CHECK(shared.retrieve().value.session_token == "t1");
  chain->fail = true;
  now = 130 * kSecond;  // inside the window, refresh failing
  auto r = shared.retrieve();
  CHECK(r.ok() && r.value.session_token == "t1" && r.value.kept_after_failed_refresh);
  CHECK_EQ(chain->calls.load(), 2);
  for (int i = 0; i < 50; ++i) CHECK(shared.retrieve().ok());  // within kKeptRetry: no fetch
  CHECK_EQ(chain->calls.load(), 2);
  shared.signed_with_kept(r.value);
  CHECK_EQ(shared.stale_signs(), uint64_t(1));
  now = 141 * kSecond;  // kKeptRetry later: one more (failing) fetch, the set still kept
  CHECK(shared.retrieve().value.kept_after_failed_refresh);
  CHECK_EQ(chain->calls.load(), 3);
  now = 361 * kSecond;  // within the skew of Expiration: the chain's error
  auto e = shared.retrieve();
  CHECK(!e.ok() && e.status.message() == "EcsCredentialsError: 500");
  // recovery, then a rejection during an outage: the rejected set is not kept
  chain->fail = false;
  CHECK(shared.retrieve().ok());
  const Credentials fresh = shared.retrieve().value;
  chain->fail = true;
  shared.stale(fresh);
  CHECK(!shared.retrieve().ok());
}

// SharedCredentialsProvider::cancel releases the callers waiting for another client's fetch
// (a stop no longer waits out the whole fetch timeout); the fetch itself, and the
// callers that come later, are unaffected.
TEST(shared_provider_cancel_releases_waiters) {
  struct Slow final : CredentialsProvider {
    std::atomic<bool> go{false};
    std::atomic<bool> in{false};
    Result<Credentials> retrieve() override {
      in = true;
      while (!go) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      Credentials c;
      c.access_key_id = "AKID";
      c.secret_access_key = "s";
      return Result<Credentials>::Ok(c);
    }
  };
  auto inner = std::make_shared<Slow>();
  SharedCredentialsProvider shared(inner, [] { return int64_t(0); }, 0);
  Result<Credentials> fetched, waited;
  std::thread fetcher([&] { fetched = shared.retrieve(); });
  while (!inner->in) std::this_thread::yield();
  std::atomic<bool> returned{false};
  std::thread waiter([&] {
    waited = shared.retrieve();
    returned = true;
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  CHECK(!returned.load());
  shared.cancel();
  waiter.join();
  CHECK(!waited.ok() && waited.status.message() == "request canceled");
  inner->go = true;
  fetcher.join();
  CHECK(fetched.ok() && fetched.value.access_key_id == "AKID");
  CHECK(shared.retrieve().ok() && shared.fetches() == 1);
}

TEST(spin_window_ceiling) {
  const Nanos us = kMicrosecond;
  CHECK_EQ(HttpClient::spin_window_for(25 * us, 15000 * us, 37500 * us), Nanos(0));
  CHECK_EQ(HttpClient::spin_window_for(25 * us, 201 * us, kSecond), Nanos(0));
  CHECK_EQ(HttpClient::spin_window_for(25 * us, 150 * us, kSecond), HttpClient::kMaxSpinThrough);
  CHECK_EQ(HttpClient::spin_window_for(25 * us, 40 * us, 80 * us), 80 * us);
  CHECK_EQ(HttpClient::spin_window_for(25 * us, 40 * us, 79 * us), 25 * us);
  for (Nanos bp : {Nanos(0), 25 * us, 300 * us})
    for (Nanos ewma = -1; ewma < 20 * kMillisecond; ewma += 7 * us)
      CHECK(HttpClient::spin_window_for(bp, ewma, kSecond) <= std::max(bp, HttpClient::kMaxSpinThrough));
}

TEST(cgroup_cpu_quota_parsers) {
  CHECK(!parse_cpu_max("max 100000").limited());
  CpuQuota q = parse_cpu_max("10000 100000\n");
  CHECK(q.limited() && q.quota_ns == 10 * kMillisecond && q.period_ns == 100 * kMillisecond);
  CHECK(!parse_cpu_max("").limited() && !parse_cpu_max("x y").limited() && !parse_cpu_max("0 100000").limited());
  CHECK(!parse_cfs_quota("-1\n", "100000\n").limited());
  CHECK(parse_cfs_quota("50000\n", "100000\n").quota_ns == 50 * kMillisecond);
  LoopConfig lc;
  CHECK_EQ(lc.spin_budget_ppm, int64_t(0));  // the CLI's default: the --busy-poll window only
  lc.poll_period = 5 * kSecond;
  CHECK_EQ(Runner::spin_budget_for(lc, CpuQuota()), Nanos(0));
  lc.spin_budget_ppm = 10000;  // --busy-poll-budget=1
  CHECK_EQ(Runner::spin_budget_for(lc, CpuQuota()), 50 * kMillisecond);
  CHECK_EQ(Runner::spin_budget_for(lc, q), kMillisecond);
}

}  // namespace

// The worker-process error slot (SharedWorkerState, seqlock over relaxed atomic words): a reader
// racing the writer gets one of the texts written, whole, or "" -- never a mix (TSan-clean: every
// shared access is atomic).
// policy_sim.h capped_quotient (the nanosecond clock's skip count): equal to exact integer
// division capped at `cap` over its whole domain (0 <= x < 2^60, 1 <= s <= 2^62, cap <= 2^26),
// at quotients exactly on, one below and one above an integer, and under UBSan for overflow.
TEST(capped_quotient_exact) {
  auto want = [](int64_t x, int64_t s, int64_t cap) { return std::min(x / s, cap); };
  const int64_t caps[] = {-1, 0, 1, 7, (1 << 26) - 1, 1 << 26};
  const int64_t ss[] = {1, 2, 3, 999'999, 1'000'000, 5'002'000'000LL, (1LL << 40) + 1, 1LL << 61, 1LL << 62};
  uint64_t r = 0x9e3779b97f4a7c15ULL;
  int checked = 0;
  for (int64_t cap : caps)
    for (int64_t s : ss) {
      for (int64_t q : {int64_t(0), int64_t(1), cap - 1, cap, cap + 1, int64_t(1) << 25, (int64_t(1) << 26) + 5}) {
        if (q < 0) continue;
        for (int64_t d : {int64_t(-1), int64_t(0), int64_t(1), s - 1}) {  // x around q * s
          if (q > 0 && s > ((int64_t(1) << 60) - 1) / q) continue;
          const int64_t x = q * s + d;
          if (x < 0 || x >= (int64_t(1) << 60)) continue;
          CHECK(ksa_sim::capped_quotient(x, s, cap) == want(x, s, cap));
          ++checked;
        }
      }
      for (int k = 0; k < 2000; ++k) {  // random x over the domain
        r = r * 6364136223846793005ULL + 1442695040888963407ULL;
        const int64_t x = static_cast<int64_t>(r >> 4) >> (r % 40);
        CHECK(ksa_sim::capped_quotient(x, s, cap) == want(x, s, cap));
        ++checked;
      }
    }
  CHECK(checked > 100000);
}

TEST(shared_error_slot_seqlock) {
  alignas(64) static unsigned char mem[sizeof(SharedWorkerState)];
  SharedWorkerState* s = init_shared_worker_state(mem);
  CHECK(read_shared_error(s).empty());
  const std::string a(300, 'a'), b = "short b error", c(600, 'c');
  std::atomic<bool> done{false}, reading{false};
  std::thread writer([&] {
    while (!reading.load()) std::this_thread::yield();  // the reads overlap the writes
    for (int i = 0; i < 20000; ++i) write_shared_error(s, i % 3 == 0 ? a : i % 3 == 1 ? b : c);
    done = true;
  });
  const std::string c_cut(SharedWorkerState::kErrorBytes - 1, 'c');
  long reads = 0, bad = 0;
  reading = true;
  do {
    const std::string t = read_shared_error(s);
    ++reads;
    if (!(t.empty() || t == a || t == b || t == c_cut)) ++bad;
  } while (!done.load());
  writer.join();
  CHECK(bad == 0);
  CHECK(reads > 0);
  CHECK(read_shared_error(s) == b || read_shared_error(s) == a || read_shared_error(s) == c_cut);
}

int main() {
  for (auto& t : registry()) {
    int before = g_failed;
    t.fn();
    std::fprintf(stderr, "[%s] %s\n", g_failed == before ? " ok " : "FAIL", t.name);
  }
  std::fprintf(stderr, "%d checks, %d failed\n", g_checks, g_failed);
  return g_failed ? 1 : 0;
}
