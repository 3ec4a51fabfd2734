// Wire-level pieces shared by the HTTP client (http.cc) and the fakes' server
// (csrc/fakes/http_server.cc): the deadline-bounded plain/TLS Stream, HTTP/1.1 message framing
// (Reader), Go textproto header parsing and the OpenSSL set-up helpers. Internal to the
// native build; not part of the public transport API in http.h.
#pragma once

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>

#include <arpa/inet.h>
#include <errno.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <poll.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>
#include <csignal>

#include "clock.h"
#include "goutil.h"
#include "http.h"
#include "status.h"

namespace ksa {
namespace wire {

// OpenSSL writes through a socket BIO (plain write(2)), so a peer that closes mid-stream would
// raise SIGPIPE and kill a process that has not ignored it (Python does; a C++ embedder may not).
// Like Go's runtime, ignore SIGPIPE process-wide -- only if nobody installed a handler -- and
// let the write fail with EPIPE instead. Plain sockets additionally use MSG_NOSIGNAL.
inline void ignore_sigpipe_once() {
  static std::once_flag once;
  std::call_once(once, [] {
    struct sigaction cur;
    if (sigaction(SIGPIPE, nullptr, &cur) == 0 && cur.sa_handler == SIG_DFL) signal(SIGPIPE, SIG_IGN);
  });
}

inline std::string lower(std::string s) {
  for (auto& c : s) c = ascii_lower(c);
  return s;
}

inline bool iequals(const std::string& a, const std::string& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (ascii_lower(a[i]) != ascii_lower(b[i])) return false;
  return true;
}

inline std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && (s[b] == ' ' || s[b] == '\t')) ++b;
  while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r')) --e;
  return s.substr(b, e - b);
}

inline std::string header_of(const Headers& hs, const std::string& name) {
  for (auto& [k, v] : hs)
    if (iequals(k, name)) return v;
  return "";
}

inline bool has_header(const Headers& hs, const std::string& name) {
  for (auto& kv : hs)
    if (iequals(kv.first, name)) return true;
  return false;
}

// Case-insensitive "does `hay` contain `needle`" (needle given in lower case), no copies.
inline bool icontains(const std::string& hay, const char* needle) {
  const size_t n = std::strlen(needle);
  if (n > hay.size()) return false;
  for (size_t i = 0; i + n <= hay.size(); ++i) {
    size_t k = 0;
    while (k < n && ascii_lower(hay[i + k]) == needle[k]) ++k;
    if (k == n) return true;
  }
  return false;
}

inline const std::string* header_ptr(const Headers& hs, const char* name, size_t len) {
  for (auto& [k, v] : hs) {
    if (k.size() != len) continue;
    size_t i = 0;
    while (i < len && ascii_lower(k[i]) == ascii_lower(name[i])) ++i;
    if (i == len) return &v;
  }
  return nullptr;
}

inline std::string ssl_error_string() {
  unsigned long e = ERR_get_error();
  if (!e) return "unknown TLS error";
  char buf[256];
  ERR_error_string_n(e, buf, sizeof buf);
  ERR_clear_error();
  return buf;
}

// Waits for `events` on fd until the absolute deadline (0 = forever). A readable `cancel_fd`
// (HttpClient::cancel) ends the wait with "request canceled".
inline Status wait_fd(int fd, short events, int64_t deadline_ns, int cancel_fd = -1) {
  while (true) {
    int timeout_ms = -1;
    if (deadline_ns) {
      int64_t left = deadline_ns - mono_ns();
      if (left <= 0) return Status::Err("i/o timeout");
      timeout_ms = static_cast<int>((left + 999999) / 1000000);
    }
    struct pollfd p[2] = {{fd, events, 0}, {cancel_fd, POLLIN, 0}};
    int r = ::poll(p, cancel_fd >= 0 ? 2 : 1, timeout_ms);
    if (r > 0 && cancel_fd >= 0 && (p[1].revents & POLLIN)) return Status::Err("request canceled");
    if (r > 0) return Status::OK();
    if (r == 0) {
      if (deadline_ns && mono_ns() >= deadline_ns) return Status::Err("i/o timeout");
      continue;
    }
    if (errno == EINTR) continue;
    return Status::Err(std::string("poll: ") + std::strerror(errno));
  }
}

// A non-blocking socket, optionally wrapped in TLS, with deadline-bounded I/O. Cache-line
// aligned, as Conn: the streams of different workers' clients never share a line, whichever
// thread dialled them.
class alignas(kCacheLine) Stream {
 public:
  Stream(int fd, SSL* ssl) : fd_(fd), ssl_(ssl) {}
  ~Stream() {
    if (ssl_) {
      SSL_shutdown(ssl_);
      SSL_free(ssl_);
    }
    if (outer_) {
      SSL_shutdown(outer_);
      SSL_free(outer_);
    }
    if (fd_ >= 0) ::close(fd_);
  }
  int fd() const { return fd_; }

  // Drives an SSL_* call that may want read/write readiness.
  template <class F>
  Status ssl_op(F op, int64_t deadline_ns, int* out, const char* what) {
    int64_t spin_end = 0;
    bool spin_over = false;
    // SSL_get_error reads the thread's error queue, so it must start empty. A WANT_READ /
    // WANT_WRITE result queues nothing: the busy-poll retries skip the clear (OpenSSL 3 resets
    // all 16 queue slots per call, the largest cost of a TLS spin iteration in the r02q
    // profile) unless something is queued after all.
    ERR_clear_error();
    for (int i = 0;; ++i) {
      if (i > 0 && ERR_peek_error() != 0) ERR_clear_error();
      int r = op();
      if (r > 0) {
        *out = r;
        return Status::OK();
      }
      int e = SSL_get_error(ssl_, r);
      if (e == SSL_ERROR_WANT_READ) {
        // Busy-poll applies to TLS too: retry the operation itself (a non-blocking read of the
        // socket underneath) for up to spin_ns_, so the call that sees the record's bytes also
        // decrypts them; then sleep in poll(2).
        if (spin_ns_ > 0 && !spin_over) {
          if (spin_end == 0) spin_end = mono_ns() + spin_ns_;
          if ((i & 7) != 7 || mono_ns() < spin_end) {
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
            continue;
          }
          spin_over = true;
        }
        Status s = wait_fd(fd_, POLLIN, deadline_ns, cancel_fd_);
        if (!s.ok()) return s;
      } else if (e == SSL_ERROR_WANT_WRITE) {
        Status s = wait_fd(fd_, POLLOUT, deadline_ns, cancel_fd_);
        if (!s.ok()) return s;
      } else if (e == SSL_ERROR_ZERO_RETURN) {
        *out = 0;
        return Status::OK();
      } else if (e == SSL_ERROR_SYSCALL && ERR_peek_error() == 0) {
        *out = 0;  // unexpected EOF: treat as connection closed
        return Status::OK();
      } else {
        return Status::Err(std::string(what) + ": " + ssl_error_string());
      }
    }
  }

  Status handshake(bool server, int64_t deadline_ns) {
    int out = 0;
    if (server) return ssl_op([&] { return SSL_accept(ssl_); }, deadline_ns, &out, "tls accept");
    Status s = ssl_op([&] { return SSL_connect(ssl_); }, deadline_ns, &out, "tls handshake");
    if (s.ok() && out == 0) return Status::Err("tls handshake: connection closed");
    return s;
  }

  // Appends what is available (at least one byte) to buf. *eof on orderly close.
  Status read_some(std::string* buf, int64_t deadline_ns, bool* eof) {
    char tmp[16384];
    *eof = false;
    if (ssl_) {
      int n = 0;
      Status s = ssl_op([&] { return SSL_read(ssl_, tmp, sizeof tmp); }, deadline_ns, &n, "tls read");
      if (!s.ok()) return s;
      if (n == 0) *eof = true;
      else buf->append(tmp, static_cast<size_t>(n));
      if (n > 0 && first_.armed) {
        first_.armed = false;
        first_.seen = mono_ns();
      }
      return Status::OK();
    }
    while (true) {
      ssize_t n = recv_some(tmp, sizeof tmp);
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK) && spin_ns_ > 0) {
        n = spin_recv(tmp, sizeof tmp);
        if (n > 0 && first_.armed) first_.spun = true;
      }
      if (n > 0) {
        if (first_.armed) {
          first_.armed = false;
          first_.seen = mono_ns();
          first_.rx_real = pending_rx_real_;
        }
        buf->append(tmp, static_cast<size_t>(n));
        return Status::OK();
      }
      if (n == 0) {
        *eof = true;
        return Status::OK();
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        Status s = wait_fd(fd_, POLLIN, deadline_ns, cancel_fd_);
        if (!s.ok()) return s;
        continue;
      }
      if (errno == ECONNRESET) {
        *eof = true;
        return Status::Err("connection reset by peer");
      }
      return Status::Err(std::string("read: ") + std::strerror(errno));
    }
  }

  // Writes data[from..]; *written: the bytes of data written in all (from included).
  Status write_all(const std::string& data, int64_t deadline_ns, size_t* written = nullptr, size_t from = 0) {
    size_t off = from;
    struct Report {
      size_t* w;
      size_t& off;
      ~Report() {
        if (w) *w = off;
      }
    } report{written, off};
    while (off < data.size()) {
      if (ssl_) {
        int n = 0;
        Status s = ssl_op(
            [&] { return SSL_write(ssl_, data.data() + off, static_cast<int>(data.size() - off)); },
            deadline_ns, &n, "tls write");
        if (!s.ok()) return s;
        if (n == 0) return Status::Err("write: connection closed");
        off += static_cast<size_t>(n);
        continue;
      }
      ssize_t n = ::send(fd_, data.data() + off, data.size() - off, MSG_NOSIGNAL);
      if (n > 0) {
        off += static_cast<size_t>(n);
        continue;
      }
      if (n < 0 && errno == EINTR) continue;
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        Status s = wait_fd(fd_, POLLOUT, deadline_ns, cancel_fd_);
        if (!s.ok()) return s;
        continue;
      }
      return Status::Err(std::string("write: ") + std::strerror(errno));
    }
    return Status::OK();
  }

  // An idle keep-alive connection about to be reused: has the peer closed it (FIN, RST, a TLS
  // close_notify) or sent something unsolicited? Go's transport learns this from the idle
  // connection's read loop and dials a new one instead of writing into a dead socket; here the
  // socket is peeked without blocking. TLS records that carry no application data (session
  // tickets) are consumed by the peek and leave the connection usable.
  bool peer_closed() {
    if (ssl_) {
      char c;
      ERR_clear_error();
      const int n = SSL_peek(ssl_, &c, 1);
      if (n > 0) return true;  // unsolicited response bytes: the connection is out of sync
      const int e = SSL_get_error(ssl_, n);
      return !(e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE);
    }
    char c;
    while (true) {
      const ssize_t n = ::recv(fd_, &c, 1, MSG_PEEK | MSG_DONTWAIT);
      if (n >= 0) return true;  // 0: orderly close; > 0: unsolicited bytes
      if (errno == EINTR) continue;
      return !(errno == EAGAIN || errno == EWOULDBLOCK);
    }
  }

  // Corked write (HttpClient::stage): `len` bytes handed to the kernel now but held back from
  // the wire until the next uncorked write -- a plain socket with MSG_MORE, TLS under TCP_CORK
  // (uncork() after the final record). The kernel's send path runs for them here, so the final
  // write later runs warm. Never blocks: a socket that cannot take the bytes at once fails it.
  bool write_corked(const char* data, size_t len) {
    if (ssl_) {
      int on = 1;
      if (setsockopt(fd_, IPPROTO_TCP, TCP_CORK, &on, sizeof on) != 0) return false;
      corked_ = true;
      ERR_clear_error();
      const int n = SSL_write(ssl_, data, static_cast<int>(len));
      return n == static_cast<int>(len);
    }
    size_t off = 0;
    while (off < len) {
      const ssize_t n = ::send(fd_, data + off, len - off, MSG_NOSIGNAL | MSG_MORE | MSG_DONTWAIT);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) return false;
      off += static_cast<size_t>(n);
    }
    return true;
  }
  // Releases TCP_CORK (TLS after write_corked): what is queued goes on the wire now.
  void uncork() {
    if (!corked_) return;
    int off = 0;
    setsockopt(fd_, IPPROTO_TCP, TCP_CORK, &off, sizeof off);
    corked_ = false;
  }

  void set_spin_ns(int64_t ns) { spin_ns_ = ns; }
  void set_cancel_fd(int fd) { cancel_fd_ = fd; }
  // First-bytes timing of the next response (HttpClient::set_timing): arm before reading it;
  // the first read that gets data stamps when this thread saw it and, on a plain socket with
  // receive timestamps on, the kernel's receive time (CLOCK_REALTIME) of those bytes.
  struct FirstBytes {
    bool armed = false;
    bool spun = false;
    int64_t seen = 0;
    int64_t rx_real = 0;
  };
  void enable_rx_timestamps() {
    int on = 1;
    ts_ = setsockopt(fd_, SOL_SOCKET, SO_TIMESTAMPNS, &on, sizeof on) == 0;
  }
  void arm_first_bytes() { first_ = FirstBytes{true, false, 0, 0}; }
  const FirstBytes& first_bytes() const { return first_; }
  SSL* ssl() const { return ssl_; }
  void attach_ssl(SSL* ssl) { ssl_ = ssl; }  // TLS inside an established CONNECT tunnel
  // TLS inside TLS (an https origin behind an https proxy): `inner` becomes the session the
  // stream reads and writes; its BIO (tunnel_bio) carries its records through the current one.
  void push_ssl(SSL* inner) {
    outer_ = ssl_;
    ssl_ = inner;
  }

 private:
  // Busy-poll on a plain socket: keep reading (non-blocking) for up to spin_ns_ before sleeping
  // in poll(2). A response that lands within the window is picked up without a scheduler
  // wake-up (several microseconds on every round trip), and by the same system call that sees
  // it; past the window the thread blocks as usual, so idle waits cost no CPU.
  // Returns recv's result; -1 with errno EAGAIN when the window passed without data.
  ssize_t spin_recv(char* out, size_t cap) {
    const int64_t end = mono_ns() + spin_ns_;
    for (int i = 0;; ++i) {
      const ssize_t n = recv_some(out, cap);
      if (n >= 0) return n;
      if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) return n;
      if ((i & 15) == 15 && mono_ns() >= end) {
        errno = EAGAIN;
        return -1;
      }
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
  }

  // recv(2), or recvmsg(2) with the receive timestamp while first-bytes timing is armed.
  ssize_t recv_some(char* out, size_t cap) {
    if (!(kHttpTiming && ts_ && first_.armed)) return ::recv(fd_, out, cap, 0);
    struct iovec iov = {out, cap};
    alignas(struct cmsghdr) char ctrl[CMSG_SPACE(sizeof(struct timespec))];
    struct msghdr msg = {};
    msg.msg_iov = &iov;
    msg.msg_iovlen = 1;
    msg.msg_control = ctrl;
    msg.msg_controllen = sizeof ctrl;
    const ssize_t n = ::recvmsg(fd_, &msg, 0);
    if (n > 0) {
      pending_rx_real_ = 0;
      for (struct cmsghdr* cm = CMSG_FIRSTHDR(&msg); cm; cm = CMSG_NXTHDR(&msg, cm)) {
        if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_TIMESTAMPNS) {
          struct timespec ts;
          std::memcpy(&ts, CMSG_DATA(cm), sizeof ts);
          pending_rx_real_ = static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
        }
      }
    }
    return n;
  }

  int fd_;
  SSL* ssl_;
  SSL* outer_ = nullptr;  // the proxy's TLS session when ssl_ runs inside it
  int64_t spin_ns_ = 0;
  int cancel_fd_ = -1;
  bool corked_ = false;
  bool ts_ = false;
  FirstBytes first_;
  int64_t pending_rx_real_ = 0;
};

// Largest message body either side accepts. Scale objects and Deployments are a few KiB and a
// NodeList of a large cluster a few tens of MiB; a peer announcing more (or a chunked /
// read-to-EOF body that keeps growing) is cut off instead of exhausting the 200 MiB pod.
constexpr size_t kMaxBody = 128u << 20;

// Incremental HTTP/1.1 message framing over a Stream with a carry-over buffer.
class Reader {
 public:
  Reader(Stream* s, std::string* buf) : s_(s), buf_(buf) {}

  // Reads through the blank line; returns the head (without the terminator).
  Status read_head(std::string* head, int64_t deadline_ns, bool* got_any) {
    *got_any = !buf_->empty();
    while (true) {
      size_t p = buf_->find("\r\n\r\n");
      if (p != std::string::npos) {
        head->assign(*buf_, 0, p);
        buf_->erase(0, p + 4);
        return Status::OK();
      }
      if (buf_->size() > 1 << 20) return Status::Err("header too large");
      bool eof = false;
      Status s = s_->read_some(buf_, deadline_ns, &eof);
      if (!s.ok()) return s;
      if (eof) return Status::Err(buf_->empty() ? "EOF" : "unexpected EOF");
      *got_any = true;
    }
  }

  Status read_exact(size_t n, std::string* out, int64_t deadline_ns) {
    if (n > kMaxBody || out->size() + n > kMaxBody) return Status::Err("message body too large");
    while (buf_->size() < n) {
      bool eof = false;
      Status s = s_->read_some(buf_, deadline_ns, &eof);
      if (!s.ok()) return s;
      if (eof) return Status::Err("unexpected EOF");
    }
    out->append(*buf_, 0, n);
    buf_->erase(0, n);
    return Status::OK();
  }

  Status read_line(std::string* line, int64_t deadline_ns) {
    while (true) {
      size_t p = buf_->find("\r\n");
      if (p != std::string::npos) {
        line->assign(*buf_, 0, p);
        buf_->erase(0, p + 2);
        return Status::OK();
      }
      if (buf_->size() > 1 << 20) return Status::Err("line too long");
      bool eof = false;
      Status s = s_->read_some(buf_, deadline_ns, &eof);
      if (!s.ok()) return s;
      if (eof) return Status::Err("unexpected EOF");
    }
  }

  Status read_chunked(std::string* out, int64_t deadline_ns) {
    while (true) {
      std::string line;
      Status s = read_line(&line, deadline_ns);
      if (!s.ok()) return s;
      size_t semi = line.find(';');
      std::string hex = trim(semi == std::string::npos ? line : line.substr(0, semi));
      if (hex.empty()) return Status::Err("malformed chunk size");
      char* end = nullptr;
      errno = 0;
      unsigned long long n = std::strtoull(hex.c_str(), &end, 16);
      if (*end != '\0' || errno == ERANGE) return Status::Err("malformed chunk size");
      if (n > kMaxBody || out->size() + n > kMaxBody) return Status::Err("message body too large");
      if (n == 0) {
        // trailers until blank line
        while (true) {
          std::string t;
          s = read_line(&t, deadline_ns);
          if (!s.ok()) return s;
          if (t.empty()) return Status::OK();
        }
      }
      s = read_exact(static_cast<size_t>(n), out, deadline_ns);
      if (!s.ok()) return s;
      std::string crlf;
      s = read_line(&crlf, deadline_ns);
      if (!s.ok()) return s;
    }
  }

  Status read_to_eof(std::string* out, int64_t deadline_ns) {
    out->append(*buf_);
    buf_->clear();
    while (true) {
      bool eof = false;
      std::string tmp;
      Status s = s_->read_some(&tmp, deadline_ns, &eof);
      if (!s.ok()) return s;
      if (eof) return Status::OK();
      if (out->size() + tmp.size() > kMaxBody) return Status::Err("message body too large");
      out->append(tmp);
    }
  }

 private:
  Stream* s_;
  std::string* buf_;
};

// Header lines as Go's textproto.Reader.ReadMIMEHeader reads them (net/http, client and server):
// "Name: value", a line starting with a space or tab continues the previous value (obs-fold),
// and a line without a colon -- or a continuation with nothing to continue -- is a protocol error
// ("malformed MIME header line"); *bad gets the line. Spans are trimmed in place: one string per
// name and per value, nothing else allocated.
inline bool parse_header_lines(const std::string& head, size_t from, Headers* out, std::string* bad) {
  auto trimmed = [&](size_t b, size_t e) {
    while (b < e && (head[b] == ' ' || head[b] == '\t')) ++b;
    while (e > b && (head[e - 1] == ' ' || head[e - 1] == '\t' || head[e - 1] == '\r')) --e;
    return std::string(head, b, e - b);
  };
  size_t pos = from;
  const size_t first = out->size();
  while (pos < head.size()) {
    size_t e = head.find("\r\n", pos);
    if (e == std::string::npos) e = head.size();
    if (e > pos && (head[pos] == ' ' || head[pos] == '\t')) {
      if (out->size() == first) {  // "malformed MIME header initial line"
        *bad = head.substr(pos, e - pos);
        return false;
      }
      std::string more = trimmed(pos, e);
      if (!more.empty()) {
        std::string& v = out->back().second;
        if (!v.empty()) v.push_back(' ');
        v += more;
      }
    } else if (e > pos) {
      const char* colon = static_cast<const char*>(std::memchr(head.data() + pos, ':', e - pos));
      if (!colon) {
        *bad = head.substr(pos, e - pos);
        return false;
      }
      const size_t c = static_cast<size_t>(colon - head.data());
      out->emplace_back(trimmed(pos, c), trimmed(c + 1, e));
    }
    pos = e + 2;
  }
  return true;
}

inline bool wants_close(const Headers& hs, bool http10) {
  const std::string* c = header_ptr(hs, "Connection", 10);
  if (c && icontains(*c, "close")) return true;
  if (http10 && !(c && icontains(*c, "keep-alive"))) return true;
  return false;
}

inline bool is_chunked(const Headers& hs) {
  const std::string* t = header_ptr(hs, "Transfer-Encoding", 17);
  return t && icontains(*t, "chunked");
}

struct SslInit {
  SslInit() { OPENSSL_init_ssl(0, nullptr); }
};
inline void ensure_ssl() { static SslInit once; }

inline Status load_ca_pem(SSL_CTX* ctx, const std::string& pem) {
  BIO* bio = BIO_new_mem_buf(pem.data(), static_cast<int>(pem.size()));
  X509_STORE* store = SSL_CTX_get_cert_store(ctx);
  int added = 0;
  while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
    X509_STORE_add_cert(store, x);
    X509_free(x);
    ++added;
  }
  ERR_clear_error();
  BIO_free(bio);
  if (!added) return Status::Err("no certificates found in CA data");
  return Status::OK();
}

inline Status use_cert_key(SSL_CTX* ctx, const std::string& cert_pem, const std::string& key_pem) {
  BIO* cb = BIO_new_mem_buf(cert_pem.data(), static_cast<int>(cert_pem.size()));
  X509* cert = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr);
  if (!cert) {
    BIO_free(cb);
    return Status::Err("invalid certificate PEM: " + ssl_error_string());
  }
  int ok = SSL_CTX_use_certificate(ctx, cert);
  X509_free(cert);
  // Remaining certificates form the chain.
  while (X509* extra = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr)) {
    SSL_CTX_add_extra_chain_cert(ctx, extra);  // takes ownership
  }
  ERR_clear_error();
  BIO_free(cb);
  if (ok != 1) return Status::Err("SSL_CTX_use_certificate: " + ssl_error_string());
  BIO* kb = BIO_new_mem_buf(key_pem.data(), static_cast<int>(key_pem.size()));
  EVP_PKEY* key = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
  BIO_free(kb);
  if (!key) return Status::Err("invalid private key PEM: " + ssl_error_string());
  ok = SSL_CTX_use_PrivateKey(ctx, key);
  EVP_PKEY_free(key);
  if (ok != 1) return Status::Err("SSL_CTX_use_PrivateKey: " + ssl_error_string());
  return Status::OK();
}

inline bool is_ip_literal(const std::string& h) {
  unsigned char buf[16];
  return inet_pton(AF_INET, h.c_str(), buf) == 1 || inet_pton(AF_INET6, h.c_str(), buf) == 1;
}

}  // namespace wire
}  // namespace ksa
