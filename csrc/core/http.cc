#include "http_wire.h"

#include "affinity.h"
#include "goutil.h"
#include "log.h"

#include <csignal>
#include <map>
#include <mutex>

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rand.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstring>

namespace ksa {

using namespace wire;

namespace {

// BIO carrying one TLS session's records inside another (the https-proxy tunnel). Non-blocking
// like the socket under it: when the outer session needs socket readiness the BIO reports a
// retry, the inner SSL call returns WANT_READ / WANT_WRITE, and Stream::ssl_op waits on the fd.
int tunnel_result(BIO* b, SSL* outer, int r) {
  if (r > 0) return r;
  switch (SSL_get_error(outer, r)) {
    case SSL_ERROR_WANT_READ: BIO_set_retry_read(b); return -1;
    case SSL_ERROR_WANT_WRITE: BIO_set_retry_write(b); return -1;
    case SSL_ERROR_ZERO_RETURN: return 0;
    default: return -1;
  }
}

int tunnel_write(BIO* b, const char* buf, int len) {
  BIO_clear_retry_flags(b);
  SSL* outer = static_cast<SSL*>(BIO_get_data(b));
  return tunnel_result(b, outer, SSL_write(outer, buf, len));
}

int tunnel_read(BIO* b, char* buf, int len) {
  BIO_clear_retry_flags(b);
  SSL* outer = static_cast<SSL*>(BIO_get_data(b));
  return tunnel_result(b, outer, SSL_read(outer, buf, len));
}

long tunnel_ctrl(BIO* b, int cmd, long, void*) {
  switch (cmd) {
    case BIO_CTRL_FLUSH: return 1;
    case BIO_CTRL_PENDING: return SSL_pending(static_cast<SSL*>(BIO_get_data(b)));
    default: return 0;
  }
}

BIO* tunnel_bio(SSL* outer) {
  static BIO_METHOD* method = [] {
    BIO_METHOD* m = BIO_meth_new(BIO_get_new_index() | BIO_TYPE_SOURCE_SINK, "tls-in-tls");
    BIO_meth_set_write(m, tunnel_write);
    BIO_meth_set_read(m, tunnel_read);
    BIO_meth_set_ctrl(m, tunnel_ctrl);
    BIO_meth_set_create(m, [](BIO* b) {
      BIO_set_init(b, 1);
      return 1;
    });
    return m;
  }();
  BIO* b = BIO_new(method);
  if (b) BIO_set_data(b, outer);
  return b;
}

std::string percent_decode(const std::string& in) {
  std::string out;
  for (size_t i = 0; i < in.size(); ++i) {
    if (in[i] == '%' && i + 2 < in.size() && std::isxdigit(static_cast<unsigned char>(in[i + 1])) &&
        std::isxdigit(static_cast<unsigned char>(in[i + 2]))) {
      out.push_back(static_cast<char>(std::stoi(in.substr(i + 1, 2), nullptr, 16)));
      i += 2;
    } else {
      out.push_back(in[i]);
    }
  }
  return out;
}

std::string base64(const std::string& in) {
  std::string out(4 * ((in.size() + 2) / 3) + 1, '\0');
  int n = EVP_EncodeBlock(reinterpret_cast<unsigned char*>(&out[0]),
                          reinterpret_cast<const unsigned char*>(in.data()), static_cast<int>(in.size()));
  out.resize(n > 0 ? static_cast<size_t>(n) : 0);
  return out;
}


// getaddrinfo(3) has no timeout, so a stuck resolver would hold a worker far past
// --api-timeout (Go's dialer bounds the lookup by the request's context). Names are resolved on
// a helper thread and the caller stops waiting at the deadline, or when `cancelled` is set (a
// stop: checked every 10 ms); a late answer is freed by the helper. IP literals (and calls
// without a deadline) resolve inline.
Status resolve(const std::string& host, const std::string& port, int64_t deadline_ns, struct addrinfo** out,
               const std::atomic<bool>* cancelled) {
  struct addrinfo hints;
  std::memset(&hints, 0, sizeof hints);
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  const bool literal = is_ip_literal(host);
  if (literal || deadline_ns == 0) {
    if (literal) hints.ai_flags = AI_NUMERICHOST;
    int gai = getaddrinfo(host.c_str(), port.c_str(), &hints, out);
    if (gai != 0) return Status::Err("dial tcp: lookup " + host + ": " + gai_strerror(gai));
    return Status::OK();
  }
  struct Lookup {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    int rc = 0;
    struct addrinfo* res = nullptr;
  };
  auto st = std::make_shared<Lookup>();
  std::thread([st, host, port, hints] {
    struct addrinfo* r = nullptr;
    const int rc = getaddrinfo(host.c_str(), port.c_str(), &hints, &r);
    std::lock_guard<std::mutex> lk(st->mu);
    if (st->abandoned) {
      if (r) freeaddrinfo(r);
      return;
    }
    st->rc = rc;
    st->res = r;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->mu);
  while (!st->done) {
    const int64_t left = deadline_ns - mono_ns();
    if (left <= 0) {
      st->abandoned = true;
      return Status::Err("dial tcp: lookup " + host + ": i/o timeout");
    }
    if (cancelled && cancelled->load(std::memory_order_acquire)) {
      st->abandoned = true;
      return Status::Err("request canceled");
    }
    cv_wait_for(st->cv, lk, std::min<int64_t>(left, 10 * kMillisecond), [&] { return st->done; });
  }
  if (st->rc != 0) return Status::Err("dial tcp: lookup " + host + ": " + gai_strerror(st->rc));
  *out = st->res;
  return Status::OK();
}

}  // namespace

// ---------------------------------------------------------------------------------------
// URL

std::string Url::host_header() const {
  std::string h = host.find(':') != std::string::npos ? "[" + host + "]" : host;
  bool dflt = (tls() && port == 443) || (!tls() && port == 80);
  return dflt ? h : h + ":" + std::to_string(port);
}

std::string Url::origin() const { return scheme + "://" + host_header(); }

Result<Url> parse_url(const std::string& s) {
  Url u;
  size_t p = s.find("://");
  if (p == std::string::npos) return Result<Url>::Err(Status::Err("invalid URL " + s + ": missing scheme"));
  u.scheme = lower(s.substr(0, p));
  if (u.scheme != "http" && u.scheme != "https")
    return Result<Url>::Err(Status::Err("unsupported protocol scheme \"" + u.scheme + "\""));
  size_t host_start = p + 3;
  size_t path_start = s.find_first_of("/?#", host_start);
  std::string authority = s.substr(host_start, path_start == std::string::npos ? std::string::npos : path_start - host_start);
  size_t at = authority.rfind('@');
  if (at != std::string::npos) authority = authority.substr(at + 1);
  std::string port_str;
  if (!authority.empty() && authority[0] == '[') {
    size_t rb = authority.find(']');
    if (rb == std::string::npos) return Result<Url>::Err(Status::Err("invalid URL " + s + ": bad IPv6 host"));
    u.host = authority.substr(1, rb - 1);
    if (rb + 1 < authority.size() && authority[rb + 1] == ':') port_str = authority.substr(rb + 2);
  } else {
    size_t colon = authority.rfind(':');
    if (colon != std::string::npos) {
      u.host = authority.substr(0, colon);
      port_str = authority.substr(colon + 1);
    } else {
      u.host = authority;
    }
  }
  if (u.host.empty()) return Result<Url>::Err(Status::Err("invalid URL " + s + ": empty host"));
  if (!port_str.empty()) {
    for (char c : port_str)
      if (c < '0' || c > '9') return Result<Url>::Err(Status::Err("invalid URL " + s + ": bad port"));
    u.port = std::atoi(port_str.c_str());
    if (u.port <= 0 || u.port > 65535) return Result<Url>::Err(Status::Err("invalid URL " + s + ": bad port"));
  } else {
    u.port = u.tls() ? 443 : 80;
  }
  if (path_start == std::string::npos) {
    u.path = "/";
  } else {
    u.path = s.substr(path_start);
    size_t hash = u.path.find('#');
    if (hash != std::string::npos) u.path = u.path.substr(0, hash);
    if (u.path.empty() || u.path[0] != '/') u.path = "/" + u.path;
  }
  return Result<Url>::Ok(u);
}

std::string HttpRequest::header(const std::string& name) const { return header_of(headers, name); }
std::string HttpResponse::header(const std::string& name) const { return header_of(headers, name); }

const char* http_reason(int status) {
  switch (status) {
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
  }
  return "Status";
}

// ---------------------------------------------------------------------------------------
// Client

namespace {

const char* socks5_reply_text(int code) {
  switch (code) {
    case 1: return "general SOCKS server failure";
    case 2: return "connection not allowed by ruleset";
    case 3: return "network unreachable";
    case 4: return "host unreachable";
    case 5: return "connection refused";
    case 6: return "TTL expired";
    case 7: return "command not supported";
    case 8: return "address type not supported";
    default: return "unknown code";
  }
}

// SOCKS5 CONNECT to `origin` (RFC 1928), with username/password authentication (RFC 1929)
// when the proxy URL carried credentials. Host names go to the proxy unresolved, as Go's
// socks dialer sends them. Error texts follow Go's "socks connect tcp proxy->dst: reason".
Status socks5_connect(Stream* stream, std::string* rbuf, const Url& proxy, const Url& origin, const std::string& user,
                      const std::string& pass, int64_t deadline_ns) {
  auto bracket = [](const std::string& h) { return h.find(':') != std::string::npos ? "[" + h + "]" : h; };
  const std::string where = "socks connect tcp " + bracket(proxy.host) + ":" + std::to_string(proxy.port) + "->" +
                            bracket(origin.host) + ":" + std::to_string(origin.port) + ": ";
  const bool auth = !user.empty() || !pass.empty();
  Reader rd(stream, rbuf);
  std::string greet = auth ? std::string("\x05\x02\x00\x02", 4) : std::string("\x05\x01\x00", 3);
  Status s = stream->write_all(greet, deadline_ns);
  if (!s.ok()) return Status::Err(where + s.message());
  std::string r;
  s = rd.read_exact(2, &r, deadline_ns);
  if (!s.ok()) return Status::Err(where + s.message());
  if (r[0] != 0x05) return Status::Err(where + "unexpected protocol version " + std::to_string(static_cast<uint8_t>(r[0])));
  const uint8_t method = static_cast<uint8_t>(r[1]);
  if (method == 0x02 && auth) {
    std::string up;
    up.push_back(0x01);
    up.push_back(static_cast<char>(user.size()));
    up += user;
    up.push_back(static_cast<char>(pass.size()));
    up += pass;
    s = stream->write_all(up, deadline_ns);
    if (!s.ok()) return Status::Err(where + s.message());
    r.clear();
    s = rd.read_exact(2, &r, deadline_ns);
    if (!s.ok()) return Status::Err(where + s.message());
    if (r[1] != 0x00) return Status::Err(where + "username/password authentication failed");
  } else if (method != 0x00) {
    return Status::Err(where + "no acceptable authentication methods");
  }
  std::string req("\x05\x01\x00", 3);
  unsigned char addr[16];
  if (inet_pton(AF_INET, origin.host.c_str(), addr) == 1) {
    req.push_back(0x01);
    req.append(reinterpret_cast<char*>(addr), 4);
  } else if (inet_pton(AF_INET6, origin.host.c_str(), addr) == 1) {
    req.push_back(0x04);
    req.append(reinterpret_cast<char*>(addr), 16);
  } else {
    if (origin.host.size() > 255) return Status::Err(where + "FQDN too long");
    req.push_back(0x03);
    req.push_back(static_cast<char>(origin.host.size()));
    req += origin.host;
  }
  req.push_back(static_cast<char>((origin.port >> 8) & 0xFF));
  req.push_back(static_cast<char>(origin.port & 0xFF));
  s = stream->write_all(req, deadline_ns);
  if (!s.ok()) return Status::Err(where + s.message());
  r.clear();
  s = rd.read_exact(4, &r, deadline_ns);
  if (!s.ok()) return Status::Err(where + s.message());
  if (r[0] != 0x05) return Status::Err(where + "unexpected protocol version " + std::to_string(static_cast<uint8_t>(r[0])));
  if (r[1] != 0x00) return Status::Err(where + socks5_reply_text(static_cast<uint8_t>(r[1])));
  size_t skip = 2;  // bound port
  switch (static_cast<uint8_t>(r[3])) {
    case 0x01: skip += 4; break;
    case 0x04: skip += 16; break;
    case 0x03: {
      std::string n;
      s = rd.read_exact(1, &n, deadline_ns);
      if (!s.ok()) return Status::Err(where + s.message());
      skip += static_cast<uint8_t>(n[0]);
      break;
    }
    default: return Status::Err(where + "unknown address type " + std::to_string(static_cast<uint8_t>(r[3])));
  }
  std::string bound;
  s = rd.read_exact(skip, &bound, deadline_ns);
  if (!s.ok()) return Status::Err(where + s.message());
  if (!rbuf->empty()) return Status::Err(where + "unexpected data after the reply");
  return Status::OK();
}

}  // namespace

// Cache-line aligned: a connection's per-request fields (uses, last_response_ns, the read
// buffer's pointers) are written on every request by the worker that owns it; connections of
// several workers dialled from one thread would otherwise sit next to each other in that
// thread's allocator arena and share cache lines.
struct alignas(kCacheLine) HttpClient::Conn {
  std::unique_ptr<Stream> stream;
  std::string rbuf;
  uint64_t uses = 0;
  bool session_saved = false;
  int64_t last_response_ns = 0;  // mono time a response was last read in full (0: none yet)
  int64_t last_checked_ns = 0;   // mono time the idle-close peek last passed (HttpClient::warm)
};

namespace {
// A connection that delivered a complete keep-alive response this recently is reused without
// the idle-close peek (one system call per request). Go's transport makes the same call
// without any system call: its per-connection read loop flags a connection the peer closed, and
// the flag is checked at reuse. A peer closes an idle keep-alive connection after seconds
// (AWS, the apiserver), not milliseconds. At production poll periods the peek therefore still
// runs for a poll's first request on each connection, and is skipped for the replica write
// that follows the Deployment GET.
constexpr int64_t kFreshConnNs = 20 * 1000 * 1000;
}  // namespace

HttpClient::HttpClient(const Url& origin, TlsOptions tls, Nanos timeout)
    : origin_(origin), tls_(std::move(tls)), timeout_(timeout) {
  cancel_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (origin_.tls()) ctx_status_ = init_tls_ctx();
}

// The client's TLS configuration: used for an https origin and for an https proxy (Go's
// transport also dials an https proxy with its TLSClientConfig).
Status HttpClient::init_tls_ctx() {
  if (ctx_) return Status::OK();
  ensure_ssl();
  ignore_sigpipe_once();
  ctx_ = SSL_CTX_new(TLS_client_method());
  if (!ctx_) return Status::Err("SSL_CTX_new: " + ssl_error_string());
  Status st;
  SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
  // TLS 1.3 suites in crypto/tls's client order on AES-capable CPUs (AES-128-GCM first; OpenSSL's
  // own default leads with AES-256-GCM): the reference's clients offer this order.
  SSL_CTX_set_ciphersuites(ctx_, "TLS_AES_128_GCM_SHA256:TLS_CHACHA20_POLY1305_SHA256:TLS_AES_256_GCM_SHA384");
  if (tls_.insecure_skip_verify) {
    SSL_CTX_set_verify(ctx_, SSL_VERIFY_NONE, nullptr);
  } else {
    SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
    if (!tls_.ca_pem.empty()) {
      st = load_ca_pem(ctx_, tls_.ca_pem);
    } else if (!tls_.ca_file.empty()) {
      if (SSL_CTX_load_verify_locations(ctx_, tls_.ca_file.c_str(), nullptr) != 1)
        st = Status::Err("unable to load CA file " + tls_.ca_file + ": " + ssl_error_string());
    } else {
      SSL_CTX_set_default_verify_paths(ctx_);
    }
  }
  if (st.ok() && !tls_.cert_pem.empty()) st = use_cert_key(ctx_, tls_.cert_pem, tls_.key_pem);
  // Session resumption makes reconnects after an idle close cheap.
  SSL_CTX_set_session_cache_mode(ctx_, SSL_SESS_CACHE_CLIENT);
  // Read-ahead: pull whatever the socket holds in one read(2) instead of a 5-byte record
  // header and then the body -- one syscall less per response record on the hot path.
  SSL_CTX_set_read_ahead(ctx_, 1);
  // Peers (AWS endpoints included) often close idle keep-alive connections without
  // close_notify; treat that as a plain EOF instead of a protocol error.
#ifdef SSL_OP_IGNORE_UNEXPECTED_EOF
  SSL_CTX_set_options(ctx_, SSL_OP_IGNORE_UNEXPECTED_EOF);
#endif
  return st;
}

HttpClient::~HttpClient() {
  conn_.reset();
  if (cancel_fd_ >= 0) ::close(cancel_fd_);
  if (session_) SSL_SESSION_free(session_);
  if (ctx_) SSL_CTX_free(ctx_);
}

void HttpClient::close() {
  std::lock_guard<std::mutex> lk(mu_);
  conn_.reset();
  in_flight_ = false;  // a pipelined response that was never read goes with the connection
}

void HttpClient::cancel() {
  // Lock-free on purpose: the request being cancelled holds mu_ while it waits.
  cancelled_.store(true, std::memory_order_release);
  if (cancel_fd_ >= 0) {
    const uint64_t one = 1;
    ssize_t r = ::write(cancel_fd_, &one, sizeof one);
    (void)r;
  }
}

HttpTiming HttpClient::last_timing() const {
  std::lock_guard<std::mutex> lk(mu_);
  return timing_last_;
}

std::string http_timing_json(const HttpTiming& t) {
  if (t.done == 0) return "";
  auto d = [](int64_t a, int64_t b) { return std::to_string(a > 0 && b > 0 ? b - a : -1); };
  // the wait ends when the kernel received the first response bytes (seen, without a stamp)
  const int64_t arrival = t.rx > 0 ? t.rx : t.seen;
  return "{\"pre\":" + d(t.start, t.write_begin) + ",\"write\":" + d(t.write_begin, t.written) +
         ",\"wait\":" + d(t.written, arrival) + ",\"wake\":" + (t.rx > 0 ? d(t.rx, t.seen) : std::string("-1")) +
         ",\"read\":" + d(t.seen, t.done) + ",\"spun\":" + (t.spun ? "true" : "false") + "}";
}

HttpClientStats HttpClient::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

Status HttpClient::set_proxy(const std::string& proxy_url) {
  std::lock_guard<std::mutex> lk(mu_);
  if (in_flight_) return Status::Err("http: a pipelined request is still in flight");
  conn_.reset();
  has_proxy_ = false;
  proxy_auth_.clear();
  proxy_user_.clear();
  proxy_pass_.clear();
  if (proxy_url.empty()) return Status::OK();
  const size_t sep = proxy_url.find("://");
  const std::string scheme = sep == std::string::npos ? "" : lower(proxy_url.substr(0, sep));
  ProxyKind kind = ProxyKind::Http;
  std::string as_http = proxy_url;  // parse_url knows http(s) only; socks5 shares the syntax
  if (scheme == "https") {
    kind = ProxyKind::Https;
  } else if (scheme == "socks5" || scheme == "socks5h") {
    kind = ProxyKind::Socks5;
    as_http = "http" + proxy_url.substr(sep);
  } else if (scheme != "http") {
    return Status::Err("proxy: unknown scheme \"" + scheme + "\" (http, https or socks5)");
  }
  auto u = parse_url(as_http);
  if (!u.status.ok()) return Status::Err("proxy: " + u.status.message());
  if (kind == ProxyKind::Socks5) {  // no explicit port: 1080, not http's 80
    std::string host_port = proxy_url.substr(sep + 3);
    host_port = host_port.substr(0, host_port.find_first_of("/?#"));
    host_port = host_port.substr(host_port.rfind('@') == std::string::npos ? 0 : host_port.rfind('@') + 1);
    const size_t rb = host_port.rfind(']');
    if (host_port.find(':', rb == std::string::npos ? 0 : rb) == std::string::npos) u.value.port = 1080;
  }
  if (kind == ProxyKind::Https) {
    if (!ctx_) ctx_status_ = init_tls_ctx();
    if (!ctx_status_.ok()) return Status::Err("proxy: " + ctx_status_.message());
  }
  // userinfo (parse_url drops it): scheme://user[:pass]@host
  const size_t a = proxy_url.find("://") + 3;
  const size_t end = proxy_url.find_first_of("/?#", a);
  const std::string authority = proxy_url.substr(a, end == std::string::npos ? std::string::npos : end - a);
  const size_t at = authority.rfind('@');
  if (at != std::string::npos) {
    std::string info = authority.substr(0, at);
    const size_t colon = info.find(':');
    std::string user = percent_decode(info.substr(0, colon));
    std::string pass = colon == std::string::npos ? "" : percent_decode(info.substr(colon + 1));
    if (kind == ProxyKind::Socks5) {
      if (user.size() > 255 || pass.size() > 255) return Status::Err("proxy: socks5 user or password longer than 255 bytes");
      proxy_user_ = user;
      proxy_pass_ = pass;
    } else {
      proxy_auth_ = "Basic " + base64(user + ":" + pass);
    }
  }
  proxy_ = u.value;
  proxy_kind_ = kind;
  has_proxy_ = true;
  return Status::OK();
}

Status HttpClient::dial(const Url& to, int64_t deadline_ns, int* fd_out) {
  struct addrinfo* res = nullptr;
  Status rs = resolve(to.host, std::to_string(to.port), deadline_ns, &res, &cancelled_);
  if (!rs.ok()) return rs;
  Status last = Status::Err("dial tcp " + to.host_header() + ": no addresses");
  int fd = -1;
  for (auto* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, ai->ai_protocol);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    int r = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (r != 0 && errno == EINPROGRESS) {
      Status w = wait_fd(fd, POLLOUT, deadline_ns, cancel_fd_);
      int err = 0;
      socklen_t len = sizeof err;
      getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
      if (w.ok() && err == 0) r = 0;
      else {
        last = Status::Err("dial tcp " + to.host_header() + ": " +
                           (w.ok() ? std::strerror(err) : w.message()));
      }
    } else if (r != 0) {
      last = Status::Err("dial tcp " + to.host_header() + ": " + std::strerror(errno));
    }
    if (r == 0) break;
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) return last;
  *fd_out = fd;
  return Status::OK();
}

Status HttpClient::connect_locked(int64_t deadline_ns) {
  if (!ctx_status_.ok()) return ctx_status_;
  const int64_t t_dial = mono_ns();
  int fd = -1;
  Status d = dial(has_proxy_ ? proxy_ : origin_, deadline_ns, &fd);
  if (!d.ok()) return has_proxy_ ? Status::Err("proxyconnect tcp: " + d.message()) : d;
  auto stream = std::make_unique<Stream>(fd, nullptr);
  stream->set_cancel_fd(cancel_fd_);
  std::string rbuf;
  if (has_proxy_ && proxy_kind_ == ProxyKind::Https) {
    // TLS to the proxy itself, verified like the origin would be but against the proxy's name.
    SSL* outer = SSL_new(ctx_);
    stream->attach_ssl(outer);
    SSL_set_fd(outer, fd);
    if (!is_ip_literal(proxy_.host)) SSL_set_tlsext_host_name(outer, proxy_.host.c_str());
    if (!tls_.insecure_skip_verify) {
      X509_VERIFY_PARAM* param = SSL_get0_param(outer);
      if (is_ip_literal(proxy_.host)) X509_VERIFY_PARAM_set1_ip_asc(param, proxy_.host.c_str());
      else X509_VERIFY_PARAM_set1_host(param, proxy_.host.c_str(), 0);
    }
    Status h = stream->handshake(false, deadline_ns);
    if (!h.ok()) {
      long vr = SSL_get_verify_result(outer);
      if (vr != X509_V_OK)
        return Status::Err("proxyconnect tcp: x509: certificate verification failed: " +
                           std::string(X509_verify_cert_error_string(vr)));
      return Status::Err("proxyconnect tcp: " + h.message());
    }
  }
  if (has_proxy_ && proxy_kind_ == ProxyKind::Socks5) {
    Status sc = socks5_connect(stream.get(), &rbuf, proxy_, origin_, proxy_user_, proxy_pass_, deadline_ns);
    if (!sc.ok()) return sc;
  } else if (has_proxy_ && origin_.tls()) {
    // CONNECT tunnel: the proxy relays bytes; TLS (and its verification) is end to end.
    std::string authority = origin_.host.find(':') != std::string::npos ? "[" + origin_.host + "]" : origin_.host;
    authority += ":" + std::to_string(origin_.port);
    std::string wire = "CONNECT " + authority + " HTTP/1.1\r\nHost: " + authority + "\r\n";
    if (!proxy_auth_.empty()) wire += "Proxy-Authorization: " + proxy_auth_ + "\r\n";
    wire += "\r\n";
    Status w = stream->write_all(wire, deadline_ns);
    if (!w.ok()) return Status::Err("proxyconnect tcp: " + w.message());
    Reader rd(stream.get(), &rbuf);
    std::string head;
    bool got_any = false;
    Status r = rd.read_head(&head, deadline_ns, &got_any);
    if (!r.ok()) return Status::Err("proxyconnect tcp: " + r.message());
    const std::string status_line = head.substr(0, head.find("\r\n"));
    const size_t sp = status_line.find(' ');
    const int code = sp == std::string::npos ? 0 : std::atoi(status_line.c_str() + sp + 1);
    if (status_line.compare(0, 5, "HTTP/") != 0 || code < 200 || code > 299)
      return Status::Err("proxy CONNECT " + authority + ": " +
                         (sp == std::string::npos ? status_line : status_line.substr(sp + 1)));
    // The server speaks only after our ClientHello, so nothing may follow the proxy's reply.
    if (!rbuf.empty()) return Status::Err("proxy CONNECT " + authority + ": unexpected data after the reply");
    stats_.bytes_out += wire.size();
  }

  SSL* ssl = nullptr;
  if (origin_.tls()) {
    ssl = SSL_new(ctx_);
    if (stream->ssl()) {  // https proxy: the origin's TLS runs inside the proxy's
      BIO* b = tunnel_bio(stream->ssl());
      if (!b) {
        SSL_free(ssl);
        return Status::Err("tls: cannot create the tunnel BIO");
      }
      SSL_set_bio(ssl, b, b);
      stream->push_ssl(ssl);
    } else {
      stream->attach_ssl(ssl);
      SSL_set_fd(ssl, fd);
    }
    const std::string& name = tls_.server_name.empty() ? origin_.host : tls_.server_name;
    if (!is_ip_literal(name)) SSL_set_tlsext_host_name(ssl, name.c_str());
    if (!tls_.insecure_skip_verify) {
      X509_VERIFY_PARAM* param = SSL_get0_param(ssl);
      if (is_ip_literal(name)) X509_VERIFY_PARAM_set1_ip_asc(param, name.c_str());
      else X509_VERIFY_PARAM_set1_host(param, name.c_str(), 0);
    }
    // Resume the previous session (abbreviated handshake) when the peer closed an idle
    // keep-alive connection -- AWS endpoints do after about a minute.
    if (session_) SSL_set_session(ssl, session_);
  }
  if (ssl) {
    Status h = stream->handshake(false, deadline_ns);
    if (!h.ok()) {
      long vr = SSL_get_verify_result(ssl);
      if (vr != X509_V_OK)
        return Status::Err("x509: certificate verification failed: " +
                           std::string(X509_verify_cert_error_string(vr)));
      return h;
    }
    if (SSL_session_reused(ssl)) stats_.tls_resumptions++;
    stats_.tls_version = SSL_get_version(ssl);
    stats_.tls_cipher = SSL_get_cipher_name(ssl);
  }
  conn_ = std::make_unique<Conn>();
  conn_->stream = std::move(stream);
  conn_->rbuf = std::move(rbuf);
  if (timing()) conn_->stream->enable_rx_timestamps();
  stats_.connects++;
  conn_gen_++;
  warm_dial_failed_ = false;  // reachable again: warm-ups may dial
  last_dial_ns_ = mono_ns() - t_dial;
  return Status::OK();
}

namespace {

// Go's Request.isReplayable: a request the transport may send again after it was written
// (net/http transport.go). Writes (PUT/PATCH/POST) are not: the first copy may have been
// applied, and a second resourceVersion-checked PUT would then fail with 409.
bool replayable(const HttpRequest& req) {
  if (req.method == "GET" || req.method == "HEAD" || req.method == "OPTIONS" || req.method == "TRACE")
    return true;
  return has_header(req.headers, "Idempotency-Key") || has_header(req.headers, "X-Idempotency-Key");
}

}  // namespace

bool HttpClient::fresh_locked() const {
  const int64_t now = mono_ns();
  return conn_ && ((conn_->last_response_ns > 0 && now - conn_->last_response_ns < kFreshConnNs) ||
                   (conn_->last_checked_ns > 0 && now - conn_->last_checked_ns < kFreshConnNs));
}

bool HttpClient::warm(Nanos dial_budget) {
  std::lock_guard<std::mutex> lk(mu_);
  if (in_flight_ || cancelled()) return false;
  if (fresh_locked()) return true;
  if (conn_ && conn_->uses > 0 && conn_->stream->peer_closed()) {
    stats_.idle_closed++;
    conn_.reset();
  }
  if (!conn_) {
    if (warm_dial_failed_) return false;  // the endpoint is down: the request dials
    // an endpoint whose dials are known to take longer (a distant apiserver, a proxy) gets
    // twice its last dial time, so a slow but healthy endpoint is still warmed
    const Nanos want = std::max(dial_budget, 2 * last_dial_ns_);
    const Nanos budget = timeout_ > 0 ? std::min(timeout_, want) : want;
    if (!connect_locked(mono_ns() + std::max<Nanos>(budget, 0)).ok()) {
      warm_dial_failed_ = true;
      return false;
    }
  }
  conn_->last_checked_ns = mono_ns();
  return true;
}

bool HttpClient::ready_without_dial() {
  std::lock_guard<std::mutex> lk(mu_);
  if (in_flight_ || !conn_) return false;
  if (fresh_locked() || conn_->uses == 0) return true;
  if (conn_->stream->peer_closed()) {
    stats_.idle_closed++;
    conn_.reset();
    return false;
  }
  conn_->last_checked_ns = mono_ns();
  return true;
}

void HttpClient::serialize_locked(const HttpRequest& req, std::string* out) const {
  std::string& wire = *out;
  if (wire.capacity() > 64 * 1024) std::string().swap(wire);
  wire.clear();
  wire.reserve(256 + req.body.size());
  wire += req.method;
  wire.push_back(' ');
  // A plain-HTTP origin behind a proxy gets the absolute-form target (RFC 9112 §3.2.2).
  if (forward_proxy() && !origin_.tls()) wire += origin_.origin();
  wire += req.target.empty() ? "/" : req.target;
  wire += " HTTP/1.1\r\n";
  auto line = [&wire](const std::string& k, const std::string& v) {
    wire += k;
    wire += ": ";
    wire += v;
    wire += "\r\n";
  };
  if (!has_header(req.headers, "Host")) line("Host", origin_.host_header());
  if (forward_proxy() && !origin_.tls() && !proxy_auth_.empty()) line("Proxy-Authorization", proxy_auth_);
  if (!has_header(req.headers, "User-Agent")) wire += "User-Agent: kube-sqs-autoscaler-amd/1.0\r\n";
  for (auto& [k, v] : req.headers) line(k, v);
  if (!req.body.empty() || req.method == "POST" || req.method == "PUT" || req.method == "PATCH") {
    if (!has_header(req.headers, "Content-Length")) {
      wire += "Content-Length: ";
      wire += std::to_string(req.body.size());
      wire += "\r\n";
    }
  }
  wire += "\r\n";
  wire += req.body;

}

bool HttpClient::stage(const HttpRequest& req) {
  std::lock_guard<std::mutex> lk(mu_);
  if (in_flight_ || cancelled() || !conn_ || !staged_.empty()) return false;
  serialize_locked(req, &staged_);
  constexpr size_t kHoldBack = 64;  // written at the due time: releases the rest
  if (staged_.size() <= 2 * kHoldBack) {
    staged_.clear();
    return false;
  }
  staged_sent_ = staged_.size() - kHoldBack;
  staged_gen_ = conn_gen_;
  if (!conn_->stream->write_corked(staged_.data(), staged_sent_)) {
    staged_.clear();
    conn_.reset();  // part of it may be queued: the connection cannot carry another request
    return false;
  }
  return true;
}

Status HttpClient::write_request(const HttpRequest& req, int64_t deadline_ns, bool* retryable) {
  *retryable = false;
  // The idle-close peek may be skipped on a connection used or checked this recently -- unless
  // the request must not be replayed and nobody above retries it (a Deployment write).
  if (conn_ && conn_->uses > 0 && !(fresh_locked() && (caller_retries_ || replayable(req))) &&
      conn_->stream->peer_closed()) {
    stats_.idle_closed++;
    conn_.reset();  // closed while idle: dial a fresh one (the request was never sent)
  }
  if (!conn_) {
    Status s = connect_locked(deadline_ns);
    if (!s.ok()) return s;
  }
  bool reused = conn_->uses > 0;
  conn_->uses++;
  if (timing()) timing_cur_.write_begin = mono_ns();

  std::string& wire = wire_;  // kept across requests: no allocation per request
  serialize_locked(req, &wire);
  // A staged prefix of this request (stage()) is queued, corked, on this connection: write the
  // rest, which releases it. One staged for a different request, or on a connection since
  // replaced, is dropped with its connection.
  size_t skip = 0;
  if (!staged_.empty()) {
    if (staged_gen_ == conn_gen_ && wire == staged_) {
      skip = staged_sent_;
      stats_.presends++;
    } else if (staged_gen_ == conn_gen_) {
      stats_.presend_discards++;
      staged_.clear();
      conn_.reset();
      Status c = connect_locked(deadline_ns);
      if (!c.ok()) return c;
      conn_->uses++;
      reused = false;  // a failed write on the fresh connection is not a stale-connection retry
    } else {
      stats_.presend_discards++;
    }
    staged_.clear();
  }
  size_t written = 0;
  Status s = conn_->stream->write_all(wire, deadline_ns, &written, skip);
  if (skip) conn_->stream->uncork();
  if (!s.ok()) {
    // Go's transport retries a request that never reached the wire (nothingWrittenError), and
    // a partly written one only if it is replayable.
    *retryable = reused && s.message() != "i/o timeout" && (written == 0 || replayable(req));
    conn_.reset();
    return s;
  }
  stats_.bytes_out += wire.size();
  sent_at_ = mono_ns();
  if (timing()) timing_cur_.written = sent_at_;
  return Status::OK();
}

Nanos HttpClient::spin_window_for(Nanos busy_poll, Nanos ewma, Nanos budget) {
  if (busy_poll <= 0) return 0;
  if (ewma < 0) return busy_poll;  // no sample yet: try
  const Nanos window = ewma <= 4 * busy_poll ? busy_poll : 0;
  // A peer answering within the absolute ceiling may be spun through (twice its EWMA, at most
  // the ceiling) when the budget allows; a slower one -- any remote endpoint -- never beyond
  // the window, whatever the budget: its answer is a network round trip away.
  if (ewma > kMaxSpinThrough) return window;
  const Nanos through = std::min(2 * ewma, kMaxSpinThrough);
  return through > window && through <= budget ? through : window;
}

Nanos HttpClient::spin_window() const {
  return spin_window_for(spin_ns_, ewma_ns_, spin_budget_ns_.load(std::memory_order_relaxed));
}

Nanos HttpClient::rtt_ewma() const {
  std::lock_guard<std::mutex> lk(mu_);
  return ewma_ns_;
}

Status HttpClient::read_response(const HttpRequest& req, HttpResponse* resp, int64_t deadline_ns,
                                 bool* retryable) {
  *retryable = false;
  if (!conn_) return Status::Err("connection closed before the response");
  const bool reused = conn_->uses > 1;
  Status s;
  conn_->stream->set_spin_ns(spin_window());
  if (timing()) conn_->stream->arm_first_bytes();
  Reader rd(conn_->stream.get(), &conn_->rbuf);
  std::string& head = head_;  // kept across responses: no allocation per response
  if (head.capacity() > 64 * 1024) std::string().swap(head);
  head.clear();
  bool got_any = false;
  while (true) {
    s = rd.read_head(&head, deadline_ns, &got_any);
    if (!s.ok()) {
      // The whole request was written: only a replayable one may be sent again.
      *retryable = reused && !got_any && s.message() != "i/o timeout" && replayable(req);
      conn_.reset();
      return s;
    }
    // Status line
    size_t eol = head.find("\r\n");
    std::string status_line = head.substr(0, eol);
    if (status_line.compare(0, 5, "HTTP/") != 0) {
      conn_.reset();
      return Status::Err("malformed HTTP response " + status_line);
    }
    size_t sp1 = status_line.find(' ');
    if (sp1 == std::string::npos) {
      conn_.reset();
      return Status::Err("malformed HTTP status line");
    }
    resp->status = std::atoi(status_line.c_str() + sp1 + 1);
    size_t sp2 = status_line.find(' ', sp1 + 1);
    resp->reason = sp2 == std::string::npos ? "" : status_line.substr(sp2 + 1);
    resp->headers.clear();
    std::string bad;
    if (eol != std::string::npos && !parse_header_lines(head, eol + 2, &resp->headers, &bad)) {
      conn_.reset();
      return Status::Err("net/http: malformed MIME header line: " + bad);
    }
    if (resp->status >= 100 && resp->status < 200 && resp->status != 101) continue;  // interim
    break;
  }
  const bool http10 = head.compare(0, 8, "HTTP/1.0") == 0;
  bool close_after = wants_close(resp->headers, http10);
  resp->body.clear();
  if (req.method == "HEAD" || resp->status == 204 || resp->status == 304) {
    // no body
  } else if (is_chunked(resp->headers)) {
    s = rd.read_chunked(&resp->body, deadline_ns);
  } else if (!resp->header("Content-Length").empty()) {
    long long n = std::atoll(resp->header("Content-Length").c_str());
    if (n < 0 || static_cast<unsigned long long>(n) > kMaxBody) s = Status::Err("bad Content-Length");
    else s = rd.read_exact(static_cast<size_t>(n), &resp->body, deadline_ns);
  } else {
    s = rd.read_to_eof(&resp->body, deadline_ns);
    close_after = true;
  }
  if (!s.ok()) {
    conn_.reset();
    return s;
  }
  stats_.bytes_in += head.size() + resp->body.size();
  {
    const int64_t now = mono_ns();
    const Nanos rtt = now - sent_at_;
    ewma_ns_ = ewma_ns_ < 0 ? rtt : (ewma_ns_ * 7 + rtt) / 8;
    conn_->last_response_ns = now;
    if (timing()) {
      const auto& fb = conn_->stream->first_bytes();
      timing_cur_.seen = fb.seen;
      timing_cur_.spun = fb.spun;
      timing_cur_.rx = 0;
      if (fb.rx_real > 0) {  // CLOCK_REALTIME -> CLOCK_MONOTONIC
        struct timespec rt;
        clock_gettime(CLOCK_REALTIME, &rt);
        const int64_t real_now = static_cast<int64_t>(rt.tv_sec) * 1000000000LL + rt.tv_nsec;
        timing_cur_.rx = fb.rx_real - (real_now - mono_ns());
      }
      timing_cur_.done = now;
      timing_last_ = timing_cur_;
    }
  }
  // TLS 1.3 tickets arrive after the handshake (with the first response): keep the session of
  // each new connection once, for resumption on the next reconnect.
  if (!conn_->session_saved && conn_->stream->ssl()) {
    conn_->session_saved = true;
    // A private copy: OpenSSL flags the live session non-resumable if this connection later
    // dies without close_notify, which must not cost us the ticket.
    SSL_SESSION* live = SSL_get0_session(conn_->stream->ssl());
    if (live && SSL_SESSION_is_resumable(live)) {
      SSL_SESSION* copy = SSL_SESSION_dup(live);
      if (copy) {
        if (session_) SSL_SESSION_free(session_);
        session_ = copy;
      }
    }
  }
  if (close_after) conn_.reset();
  return Status::OK();
}

namespace {
struct OnWire {
  void (*fn)(void*) = nullptr;
  void* arg = nullptr;
};
thread_local OnWire t_on_wire;
void run_on_wire() {
  OnWire w = t_on_wire;
  if (!w.fn) return;
  t_on_wire = OnWire{};  // one-shot, and not re-entered by a request `fn` makes
  w.fn(w.arg);
}
}  // namespace

void set_on_wire(void (*fn)(void*), void* arg) { t_on_wire = OnWire{fn, arg}; }
bool on_wire_pending() { return t_on_wire.fn != nullptr; }
void clear_on_wire() { t_on_wire = OnWire{}; }

Status HttpClient::attempt(const HttpRequest& req, HttpResponse* resp, int64_t deadline_ns,
                           bool* retryable) {
  Status s = write_request(req, deadline_ns, retryable);
  if (!s.ok()) return s;
  // Work that waits for this request to be on the wire (set_on_wire): the pipelined GET.
  run_on_wire();
  // The request is on the wire: the poll's held log lines go out while the server works on it.
  // (Not in receive(): a pipelined response has usually arrived already, and the write would
  // sit between it and the next request.)
  log_flush_pending();
  return read_response(req, resp, deadline_ns, retryable);
}

Status HttpClient::round_trip(const HttpRequest& req, HttpResponse* resp) { return round_trip(req, resp, -1); }

Status HttpClient::round_trip(const HttpRequest& req, HttpResponse* resp, Nanos timeout) {
  std::lock_guard<std::mutex> lk(mu_);
  if (in_flight_) return Status::Err("http: a pipelined request is still in flight");
  if (cancelled()) return Status::Err("request canceled");
  const Nanos t = timeout >= 0 ? timeout : timeout_;
  if (timeout == 0) return Status::Err("i/o timeout");  // no time left at all
  const int64_t deadline = t > 0 ? mono_ns() + t : 0;
  stats_.requests++;
  if (timing()) timing_cur_ = HttpTiming{mono_ns()};
  bool retryable = false;
  Status s = attempt(req, resp, deadline, &retryable);
  if (!s.ok() && retryable && !cancelled()) {
    stats_.reconnect_retries++;
    s = attempt(req, resp, deadline, &retryable);
  }
  return s;
}

Status HttpClient::send(const HttpRequest& req) {
  std::lock_guard<std::mutex> lk(mu_);
  if (in_flight_) return Status::Err("http: a pipelined request is still in flight");
  if (cancelled()) return Status::Err("request canceled");
  const int64_t deadline = timeout_ > 0 ? mono_ns() + timeout_ : 0;
  stats_.requests++;
  if (timing()) timing_cur_ = HttpTiming{mono_ns()};
  bool retryable = false;
  Status s = write_request(req, deadline, &retryable);
  if (!s.ok() && retryable && !cancelled()) {
    stats_.reconnect_retries++;
    s = write_request(req, deadline, &retryable);
  }
  if (!s.ok()) return s;
  pending_ = req;
  pending_deadline_ = deadline;
  in_flight_ = true;
  return Status::OK();
}

Status HttpClient::receive(HttpResponse* resp) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!in_flight_) return Status::Err("http: no request in flight");
  in_flight_ = false;
  bool retryable = false;
  Status s = read_response(pending_, resp, pending_deadline_, &retryable);
  if (!s.ok() && retryable && !cancelled()) {  // the reused connection was dead: replay on a fresh one
    stats_.reconnect_retries++;
    s = attempt(pending_, resp, pending_deadline_, &retryable);
  }
  return s;
}

bool HttpClient::in_flight() const {
  std::lock_guard<std::mutex> lk(mu_);
  return in_flight_;
}
}  // namespace ksa
