// HTTP/1.1 server of the localhost fakes: thread-per-connection or one busy-polled epoll thread
// (hot mode), optional TLS and per-request wake-up / service timing. Test and benchmark code only:
// it is linked into _ksa_fakes, never into the production _ksa_native.
#include "http_server.h"

#include "../core/affinity.h"
#include "../core/http_wire.h"

#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/rand.h>
#include <openssl/x509v3.h>
#include <pthread.h>
#include <sys/epoll.h>

#include <algorithm>
#include <map>

namespace ksa {

using namespace wire;

HttpServer::HttpServer(Handler h) : handler_(std::move(h)) {}

HttpServer::~HttpServer() {
  stop();
  if (ctx_) SSL_CTX_free(ctx_);
}

Status HttpServer::enable_tls(const std::string& cert_pem, const std::string& key_pem) {
  ensure_ssl();
  ignore_sigpipe_once();
  ctx_ = SSL_CTX_new(TLS_server_method());
  if (!ctx_) return Status::Err("SSL_CTX_new: " + ssl_error_string());
  return use_cert_key(ctx_, cert_pem, key_pem);
}

Status HttpServer::listen(const std::string& host, int port) {
  struct addrinfo hints;
  std::memset(&hints, 0, sizeof hints);
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  struct addrinfo* res = nullptr;
  std::string p = std::to_string(port);
  if (getaddrinfo(host.c_str(), p.c_str(), &hints, &res) != 0) return Status::Err("bad listen address " + host);
  int fd = ::socket(res->ai_family, res->ai_socktype | SOCK_CLOEXEC, res->ai_protocol);
  if (fd < 0) {
    freeaddrinfo(res);
    return Status::Err(std::string("socket: ") + std::strerror(errno));
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  // with timing on from the start, accepted sockets inherit receive stamps from the listener:
  // a client's first request can arrive before its connection thread runs
  if (timing_.load(std::memory_order_relaxed)) setsockopt(fd, SOL_SOCKET, SO_TIMESTAMPNS, &one, sizeof one);
  if (::bind(fd, res->ai_addr, res->ai_addrlen) != 0 || ::listen(fd, 128) != 0) {
    std::string e = std::strerror(errno);
    ::close(fd);
    freeaddrinfo(res);
    return Status::Err("listen " + host + ":" + p + ": " + e);
  }
  freeaddrinfo(res);
  struct sockaddr_storage ss;
  socklen_t len = sizeof ss;
  getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &len);
  port_ = ss.ss_family == AF_INET6 ? ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port)
                                   : ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
  listen_fd_ = fd;
  acceptor_ = std::thread([this] {
    pthread_setname_np(pthread_self(), hot_ ? "ksa-serve-hot" : "ksa-accept");
    pin_current_thread(cpus_);
    if (hot_) hot_loop();
    else accept_loop();
  });
  return Status::OK();
}

void HttpServer::accept_loop() {
  while (!stopping_.load()) {
    int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      break;  // listener shut down
    }
    if (stopping_.load()) {
      ::close(fd);
      break;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    accepted_++;
    std::vector<std::thread> finished;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = workers_.begin(); it != workers_.end();) {
        if (it->done->load(std::memory_order_acquire)) {
          finished.push_back(std::move(it->thread));
          it = workers_.erase(it);
        } else {
          ++it;
        }
      }
      open_fds_.push_back(fd);
      auto done = std::make_shared<std::atomic<bool>>(false);
      workers_.push_back(Worker{std::thread([this, fd, done] {
                                  pthread_setname_np(pthread_self(), "ksa-serve");
                                  pin_current_thread(cpus_);
                                  serve(fd);
                                  done->store(true, std::memory_order_release);
                                }),
                                done});
    }
    for (auto& t : finished) t.join();  // already returned (or about to): no blocking
  }
}

namespace {
int64_t realtime_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// The kernel receive time (CLOCK_REALTIME ns) of the first queued byte of `fd`, 0 when there is
// none (closed, nothing queued, or timestamps unavailable). `block`: wait until `fd` is readable
// first (a connection thread, which has nothing else to do); the hot loop peeks without waiting
// -- an epoll event can carry no request (a TLS handshake record) and the single thread must
// not stall on it.
int64_t wait_rx_timestamp(int fd, bool block) {
  if (block) {
    struct pollfd p = {fd, POLLIN, 0};
    while (::poll(&p, 1, -1) < 0 && errno == EINTR) {
    }
  }
  char c;
  struct iovec iov = {&c, 1};
  alignas(struct cmsghdr) char ctrl[CMSG_SPACE(sizeof(struct timespec))];
  struct msghdr msg = {};
  msg.msg_iov = &iov;
  msg.msg_iovlen = 1;
  msg.msg_control = ctrl;
  msg.msg_controllen = sizeof ctrl;
  if (::recvmsg(fd, &msg, MSG_PEEK | MSG_DONTWAIT) <= 0) return 0;
  for (struct cmsghdr* cm = CMSG_FIRSTHDR(&msg); cm; cm = CMSG_NXTHDR(&msg, cm)) {
    if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_TIMESTAMPNS) {
      struct timespec ts;
      std::memcpy(&ts, CMSG_DATA(cm), sizeof ts);
      return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
    }
  }
  return 0;
}
}  // namespace

void HttpServer::record_timing(ServeTiming t) {
  std::lock_guard<std::mutex> lk(timing_mu_);
  constexpr size_t kKeep = 1 << 16;
  if (timings_.size() < kKeep) {
    timings_.push_back(t);
  } else {
    timings_[timing_pos_] = t;
    timing_pos_ = (timing_pos_ + 1) % kKeep;
  }
}

std::vector<HttpServer::ServeTiming> HttpServer::timings() const {
  std::lock_guard<std::mutex> lk(timing_mu_);
  return timings_;
}

void HttpServer::clear_timings() {
  std::lock_guard<std::mutex> lk(timing_mu_);
  timings_.clear();
  timing_pos_ = 0;
}

void HttpServer::serve(int fd) {
  SSL* ssl = nullptr;
  if (ctx_) {
    ssl = SSL_new(ctx_);
    SSL_set_fd(ssl, fd);
  }
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  {
    Stream stream(fd, ssl);
    bool ok = true;
    if (ssl) ok = stream.handshake(true, mono_ns() + 10 * kSecond).ok();
    std::string rbuf;
    Reader rd(&stream, &rbuf);
    // receive stamps from the first request on when timing is already on (a socket stamps only
    // the segments queued after the option is set); else from the first request after it is
    bool stamps = false, stamps_tried = false;
    auto arm_stamps = [&] {
      int on = 1;
      stamps = setsockopt(fd, SOL_SOCKET, SO_TIMESTAMPNS, &on, sizeof on) == 0;
      stamps_tried = true;
    };
    if (timing_.load(std::memory_order_relaxed)) arm_stamps();
    while (ok && !stopping_.load()) {
      // With timing on: the next request's arrival, its kernel receive time and when this
      // thread got to it.
      int64_t rx = 0, t_read = 0;
      if (timing_.load(std::memory_order_relaxed)) {
        if (!stamps_tried) arm_stamps();
        if (stamps && rbuf.empty() && !(ssl && SSL_pending(ssl) > 0)) rx = wait_rx_timestamp(fd, true);
        t_read = realtime_ns();
      }
      std::string head;
      bool got_any = false;
      if (!rd.read_head(&head, 0, &got_any).ok()) break;
      HttpRequest req;
      size_t eol = head.find("\r\n");
      std::string line = head.substr(0, eol);
      size_t a = line.find(' '), b = line.rfind(' ');
      if (a == std::string::npos || b == a) break;
      req.method = line.substr(0, a);
      req.target = line.substr(a + 1, b - a - 1);
      // absolute-form (what clients send to a proxy; servers must accept it): keep path+query
      if (req.target.compare(0, 7, "http://") == 0 || req.target.compare(0, 8, "https://") == 0) {
        const size_t slash = req.target.find_first_of("/?", req.target.find("://") + 3);
        req.target = slash == std::string::npos ? "/" : req.target.substr(slash);
        if (req.target[0] == '?') req.target = "/" + req.target;
      }
      const bool http10 = line.compare(b + 1, 8, "HTTP/1.0") == 0;
      std::string bad;
      if (eol != std::string::npos && !parse_header_lines(head, eol + 2, &req.headers, &bad)) {
        // net/http's server answers a malformed header with 400 and closes the connection
        const std::string msg = "400 Bad Request: malformed MIME header line: " + bad;
        stream.write_all("HTTP/1.1 400 Bad Request\r\nContent-Type: text/plain; charset=utf-8\r\n"
                         "Connection: close\r\nContent-Length: " + std::to_string(msg.size()) + "\r\n\r\n" + msg,
                         mono_ns() + kSecond);
        break;
      }
      Status s;
      if (is_chunked(req.headers)) {
        s = rd.read_chunked(&req.body, 0);
      } else if (!req.header("Content-Length").empty()) {
        long long n = std::atoll(req.header("Content-Length").c_str());
        if (n < 0 || n > (64LL << 20)) break;
        s = rd.read_exact(static_cast<size_t>(n), &req.body, 0);
      }
      if (!s.ok()) break;
      HttpResponse resp;
      resp.status = 200;
      handler_(req, &resp);
      bool close_after = wants_close(req.headers, http10) || resp.status < 0;
      if (resp.status < 0) break;  // handler asked to drop the connection without replying
      std::string wire = "HTTP/1.1 " + std::to_string(resp.status) + " " +
                         (resp.reason.empty() ? http_reason(resp.status) : resp.reason) + "\r\n";
      for (auto& [k, v] : resp.headers) wire += k + ": " + v + "\r\n";
      if (!has_header(resp.headers, "Content-Length")) {
        wire += "Content-Length: ";
        wire += std::to_string(resp.body.size());
        wire += "\r\n";
      }
      if (close_after) wire += "Connection: close\r\n";
      wire += "\r\n";
      wire += resp.body;
      if (!stream.write_all(wire, mono_ns() + 10 * kSecond).ok()) break;
      served_++;
      if (rx > 0) record_timing(ServeTiming{std::max<int64_t>(t_read - rx, 0), realtime_ns() - t_read});
      if (close_after) break;
    }
    std::lock_guard<std::mutex> lk(mu_);
    open_fds_.erase(std::remove(open_fds_.begin(), open_fds_.end(), fd), open_fds_.end());
  }  // Stream dtor closes fd (after removal from open_fds_, so no fd-reuse race)
}

namespace {

// One complete request at the front of `buf`: parses it into *req and returns the bytes it
// took; 0 while incomplete; -1 for a request this server cannot take (malformed, chunked).
long take_request(const std::string& buf, HttpRequest* req, bool* http10) {
  const size_t end = buf.find("\r\n\r\n");
  if (end == std::string::npos) return buf.size() > (64u << 10) ? -1 : 0;
  const size_t eol = buf.find("\r\n");
  const std::string line = buf.substr(0, eol);
  const size_t a = line.find(' '), b = line.rfind(' ');
  if (a == std::string::npos || b == a) return -1;
  req->method = line.substr(0, a);
  req->target = line.substr(a + 1, b - a - 1);
  *http10 = line.compare(b + 1, 8, "HTTP/1.0") == 0;
  req->headers.clear();
  std::string bad;
  const std::string head = buf.substr(0, end + 4);
  if (!parse_header_lines(head, eol + 2, &req->headers, &bad)) return -1;
  if (is_chunked(req->headers)) return -1;
  size_t n = 0;
  if (!req->header("Content-Length").empty()) {
    const long long cl = std::atoll(req->header("Content-Length").c_str());
    if (cl < 0 || cl > (64LL << 20)) return -1;
    n = static_cast<size_t>(cl);
  }
  if (buf.size() < end + 4 + n) return 0;
  req->body.assign(buf, end + 4, n);
  return static_cast<long>(end + 4 + n);
}

std::string response_wire(const HttpResponse& resp, bool close_after) {
  std::string wire = "HTTP/1.1 " + std::to_string(resp.status) + " " +
                     (resp.reason.empty() ? http_reason(resp.status) : resp.reason) + "\r\n";
  for (auto& [k, v] : resp.headers) wire += k + ": " + v + "\r\n";
  if (!has_header(resp.headers, "Content-Length")) {
    wire += "Content-Length: ";
    wire += std::to_string(resp.body.size());
    wire += "\r\n";
  }
  if (close_after) wire += "Connection: close\r\n";
  wire += "\r\n";
  wire += resp.body;
  return wire;
}

}  // namespace

void HttpServer::hot_loop() {
  struct Conn {
    int fd = -1;
    SSL* ssl = nullptr;
    bool handshaken = false;
    bool stamps = false, stamps_tried = false;
    std::string rbuf;
  };
  const int ep = epoll_create1(EPOLL_CLOEXEC);
  if (ep < 0) return;
  fcntl(listen_fd_, F_SETFL, fcntl(listen_fd_, F_GETFL, 0) | O_NONBLOCK);
  struct epoll_event lev = {};
  lev.events = EPOLLIN;
  lev.data.fd = listen_fd_;
  epoll_ctl(ep, EPOLL_CTL_ADD, listen_fd_, &lev);
  std::map<int, Conn> conns;
  auto drop = [&](int fd) {
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
    if (it->second.ssl) SSL_free(it->second.ssl);
    {
      std::lock_guard<std::mutex> lk(mu_);
      open_fds_.erase(std::remove(open_fds_.begin(), open_fds_.end(), fd), open_fds_.end());
    }
    ::close(fd);
    conns.erase(it);
  };
  struct epoll_event evs[64];
  while (!stopping_.load(std::memory_order_relaxed)) {
    const int n = epoll_wait(ep, evs, 64, 0);  // busy-polled: this thread never sleeps
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == listen_fd_) {
        for (;;) {
          const int c = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK);
          if (c < 0) break;
          int one = 1;
          setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          accepted_++;
          Conn cn;
          cn.fd = c;
          if (timing_.load(std::memory_order_relaxed)) {
            cn.stamps = setsockopt(c, SOL_SOCKET, SO_TIMESTAMPNS, &one, sizeof one) == 0;
            cn.stamps_tried = true;
          }
          if (ctx_) {
            cn.ssl = SSL_new(ctx_);
            SSL_set_fd(cn.ssl, c);
          } else {
            cn.handshaken = true;
          }
          conns[c] = std::move(cn);
          {
            std::lock_guard<std::mutex> lk(mu_);
            open_fds_.push_back(c);
          }
          struct epoll_event ev = {};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.fd = c;
          epoll_ctl(ep, EPOLL_CTL_ADD, c, &ev);
        }
        continue;
      }
      auto it = conns.find(fd);
      if (it == conns.end()) continue;
      Conn& cn = it->second;
      if (!cn.handshaken) {
        const int r = SSL_accept(cn.ssl);
        if (r == 1) {
          cn.handshaken = true;
        } else {
          const int e = SSL_get_error(cn.ssl, r);
          if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) drop(fd);
          continue;
        }
      }
      // with timing on: the kernel's receive time of the oldest unread byte, when nothing is
      // buffered yet
      int64_t rx = 0, t_read = 0;
      if (timing_.load(std::memory_order_relaxed)) {
        if (!cn.stamps_tried) {
          int on = 1;
          cn.stamps = setsockopt(fd, SOL_SOCKET, SO_TIMESTAMPNS, &on, sizeof on) == 0;
          cn.stamps_tried = true;
        }
        if (cn.stamps && cn.rbuf.empty() && !(cn.ssl && SSL_pending(cn.ssl) > 0)) rx = wait_rx_timestamp(fd, false);
        t_read = realtime_ns();
      }
      bool closed = false;
      char tmp[16384];
      for (;;) {
        int got;
        if (cn.ssl) {
          got = SSL_read(cn.ssl, tmp, sizeof tmp);
          if (got <= 0) {
            const int e = SSL_get_error(cn.ssl, got);
            if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) closed = true;
            break;
          }
        } else {
          got = static_cast<int>(::recv(fd, tmp, sizeof tmp, 0));
          if (got == 0) closed = true;
          if (got <= 0) break;
        }
        cn.rbuf.append(tmp, static_cast<size_t>(got));
      }
      bool close_after = false;
      for (;;) {
        HttpRequest req;
        bool http10 = false;
        const long used = take_request(cn.rbuf, &req, &http10);
        if (used == 0) break;
        if (used < 0) {
          close_after = true;
          break;
        }
        cn.rbuf.erase(0, static_cast<size_t>(used));
        HttpResponse resp;
        resp.status = 200;
        handler_(req, &resp);
        if (resp.status < 0) {
          close_after = true;
          break;
        }
        close_after = wants_close(req.headers, http10);
        const std::string wire = response_wire(resp, close_after);
        size_t off = 0;
        while (off < wire.size()) {  // small responses: spin until written
          int w;
          if (cn.ssl) {
            w = SSL_write(cn.ssl, wire.data() + off, static_cast<int>(wire.size() - off));
            if (w <= 0) {
              const int e = SSL_get_error(cn.ssl, w);
              if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) continue;
              close_after = true;
              break;
            }
          } else {
            w = static_cast<int>(::send(fd, wire.data() + off, wire.size() - off, MSG_NOSIGNAL));
            if (w < 0) {
              if (errno == EAGAIN || errno == EINTR) continue;
              close_after = true;
              break;
            }
          }
          off += static_cast<size_t>(w);
        }
        served_++;
        if (rx > 0) record_timing(ServeTiming{std::max<int64_t>(t_read - rx, 0), realtime_ns() - t_read});
        rx = 0;
        if (close_after) break;
      }
      if (closed || close_after) drop(fd);
    }
  }
  while (!conns.empty()) drop(conns.begin()->first);
  ::close(ep);
}

void HttpServer::drop_connections() {
  std::lock_guard<std::mutex> lk(mu_);
  for (int fd : open_fds_) ::shutdown(fd, SHUT_RDWR);
}

void HttpServer::stop() {
  if (stopping_.exchange(true)) return;
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
  }
  {
    // before joining the acceptor: in hot mode it is the thread serving the connections, and
    // a connection thread may be waiting on an idle client; shutting the sockets down wakes both
    std::lock_guard<std::mutex> lk(mu_);
    for (int fd : open_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  if (acceptor_.joinable()) acceptor_.join();
  if (listen_fd_ >= 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
  }
  std::vector<Worker> ws;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int fd : open_fds_) ::shutdown(fd, SHUT_RDWR);
    ws.swap(workers_);
  }
  for (auto& w : ws)
    if (w.thread.joinable()) w.thread.join();
}

// ---------------------------------------------------------------------------------------
// Self-signed certificates for TLS fakes

Status generate_self_signed(const std::string& host, std::string* cert_pem, std::string* key_pem) {
  ensure_ssl();
  EVP_PKEY* pkey = EVP_EC_gen("P-256");
  if (!pkey) return Status::Err("EVP_EC_gen: " + ssl_error_string());
  X509* x = X509_new();
  X509_set_version(x, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(x), 1);
  X509_gmtime_adj(X509_getm_notBefore(x), -3600);
  X509_gmtime_adj(X509_getm_notAfter(x), 3600L * 24 * 365);
  X509_set_pubkey(x, pkey);
  X509_NAME* name = X509_get_subject_name(x);
  X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC,
                             reinterpret_cast<const unsigned char*>(host.c_str()), -1, -1, 0);
  // A distinct subject per certificate: two self-signed certificates for the same host (a proxy
  // and an apiserver, both trusted in one CA bundle) must not shadow each other in the store's
  // lookup by subject name.
  unsigned char rnd[8];
  RAND_bytes(rnd, sizeof rnd);
  char org[32];
  std::snprintf(org, sizeof org, "ksa-%02x%02x%02x%02x%02x%02x%02x%02x", rnd[0], rnd[1], rnd[2], rnd[3], rnd[4],
                rnd[5], rnd[6], rnd[7]);
  X509_NAME_add_entry_by_txt(name, "O", MBSTRING_ASC, reinterpret_cast<const unsigned char*>(org), -1, -1, 0);
  X509_set_issuer_name(x, name);
  std::string san = (is_ip_literal(host) ? "IP:" : "DNS:") + host;
  X509V3_CTX v3;
  X509V3_set_ctx_nodb(&v3);
  X509V3_set_ctx(&v3, x, x, nullptr, nullptr, 0);
  X509_EXTENSION* ext = X509V3_EXT_conf_nid(nullptr, &v3, NID_subject_alt_name, san.c_str());
  if (ext) {
    X509_add_ext(x, ext, -1);
    X509_EXTENSION_free(ext);
  }
  X509_EXTENSION* bc = X509V3_EXT_conf_nid(nullptr, &v3, NID_basic_constraints, "critical,CA:TRUE");
  if (bc) {
    X509_add_ext(x, bc, -1);
    X509_EXTENSION_free(bc);
  }
  if (!X509_sign(x, pkey, EVP_sha256())) {
    X509_free(x);
    EVP_PKEY_free(pkey);
    return Status::Err("X509_sign: " + ssl_error_string());
  }
  BIO* cb = BIO_new(BIO_s_mem());
  PEM_write_bio_X509(cb, x);
  BIO* kb = BIO_new(BIO_s_mem());
  PEM_write_bio_PrivateKey(kb, pkey, nullptr, nullptr, 0, nullptr, nullptr);
  char* data = nullptr;
  long n = BIO_get_mem_data(cb, &data);
  cert_pem->assign(data, static_cast<size_t>(n));
  n = BIO_get_mem_data(kb, &data);
  key_pem->assign(data, static_cast<size_t>(n));
  BIO_free(cb);
  BIO_free(kb);
  X509_free(x);
  EVP_PKEY_free(pkey);
  return Status::OK();
}

}  // namespace ksa
