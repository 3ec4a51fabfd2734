#include "log.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <climits>
#include <cstdio>
#include <unistd.h>

#include "goutil.h"
#include "json.h"

namespace ksa {

const char* level_name(Level l) {
  switch (l) {
    case Level::Panic: return "panic";
    case Level::Fatal: return "fatal";
    case Level::Error: return "error";
    case Level::Warn: return "warning";
    case Level::Info: return "info";
    case Level::Debug: return "debug";
    case Level::Trace: return "trace";
  }
  return "unknown";
}

bool parse_level(const std::string& s, Level* out) {
  std::string l = s;
  std::transform(l.begin(), l.end(), l.begin(), ::tolower);
  static const std::pair<const char*, Level> table[] = {
      {"panic", Level::Panic}, {"fatal", Level::Fatal}, {"error", Level::Error},
      {"warn", Level::Warn},   {"warning", Level::Warn}, {"info", Level::Info},
      {"debug", Level::Debug}, {"trace", Level::Trace}};
  for (auto& [name, lvl] : table) {
    if (l == name) {
      *out = lvl;
      return true;
    }
  }
  return false;
}

bool logrus_needs_quoting(const std::string& s) {
  for (unsigned char ch : s) {
    bool ok = (ch >= 'a' && ch <= 'z') || (ch >= 'A' && ch <= 'Z') || (ch >= '0' && ch <= '9') ||
              ch == '-' || ch == '.' || ch == '_' || ch == '/' || ch == '@' || ch == '^' ||
              ch == '+';
    if (!ok) return true;
  }
  return false;
}

namespace {

int64_t wall_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

// One write(2) for the whole line; loops only on EINTR / a short write.
void write_line(int fd, const std::string& l) {
  size_t off = 0;
  while (off < l.size()) {
    ssize_t r = ::write(fd, l.data() + off, l.size() - off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return;
    off += static_cast<size_t>(r);
  }
}

Logger::Sink fd_sink(int fd) {
  return [fd](const std::string& line) {
    std::string l = line;
    l.push_back('\n');
    write_line(fd, l);
  };
}

// The calling thread's open batch (LogBatch): lines for one fd, through one gate.
struct ThreadBatch {
  int depth = 0;
  int fd = -1;
  LineGate* gate = nullptr;
  std::shared_ptr<void> keep;  // keeps the gate's owner alive until the flush
  std::string buf;

  void flush() {
    if (!buf.empty() && gate) {
      if (buf.size() <= PIPE_BUF) gate->shared([&] { write_line(fd, buf); });
      else gate->exclusive([&] { write_line(fd, buf); });
    }
    buf.clear();
    if (buf.capacity() > 16 * PIPE_BUF) buf.shrink_to_fit();
  }
};

ThreadBatch& thread_batch() {
  thread_local ThreadBatch b;
  return b;
}

}  // namespace

LogBatch::LogBatch() { ++thread_batch().depth; }

LogBatch::~LogBatch() {
  ThreadBatch& b = thread_batch();
  if (--b.depth == 0) {
    b.flush();
    b.keep.reset();
    b.gate = nullptr;
    b.fd = -1;
  }
}

bool LogBatch::active() { return thread_batch().depth > 0; }

void log_flush_pending() {
  ThreadBatch& b = thread_batch();
  if (b.depth > 0 && !b.buf.empty()) b.flush();
}

size_t LineGate::slot_index() {
  static std::atomic<size_t> next{0};
  thread_local const size_t idx = next.fetch_add(1, std::memory_order_relaxed) % kSlots;
  return idx;
}

Logger::Logger() : base_unix_ns_(wall_now_ns()), shared_(std::make_shared<Shared>()) {
  shared_->sink = fd_sink(2);
  shared_->time = wall_now_ns;
}

std::shared_ptr<Logger> Logger::default_logger() {
  static std::shared_ptr<Logger> l = std::make_shared<Logger>();
  return l;
}

void Logger::set_sink(Sink s) {
  std::lock_guard<std::mutex> lk(shared_->mu);
  shared_->fd.store(-1, std::memory_order_release);
  shared_->sink = std::move(s);
}

void Logger::set_sink_fd(int fd) {
  std::lock_guard<std::mutex> lk(shared_->mu);
  shared_->sink = fd_sink(fd);
  shared_->fd.store(fd, std::memory_order_release);
}

void Logger::set_time_source(TimeSource t) {
  std::lock_guard<std::mutex> lk(shared_->mu);
  shared_->custom_time.store(true, std::memory_order_release);
  shared_->time = std::move(t);
}

std::shared_ptr<Logger> Logger::with_fields(const Fields& extra) const {
  auto l = std::make_shared<Logger>(*this);  // shares sink/time (shared_ptr copy)
  for (auto& kv : extra) l->base_.push_back(kv);
  l->sort_base();
  return l;
}

void Logger::sort_base() {
  base_sorted_ = base_;
  std::stable_sort(base_sorted_.begin(), base_sorted_.end(),
                   [](const auto& a, const auto& b) { return a.first < b.first; });
}

std::string Logger::format(Level l, const std::string& msg, const Fields& fields,
                           int64_t unix_ns) const {
  Fields merged;
  if (!fields.empty()) {
    merged = base_;
    merged.insert(merged.end(), fields.begin(), fields.end());
    std::stable_sort(merged.begin(), merged.end(),
                     [](const auto& a, const auto& b) { return a.first < b.first; });
  }
  const Fields& data = fields.empty() ? base_sorted_ : merged;
  std::string out;
  if (format_ == LogFormat::Json) {
    // encoding/json marshals the map with sorted keys; time/level/msg sort among them.
    Fields all = data;
    all.emplace_back("level", level_name(l));
    all.emplace_back("msg", msg);
    all.emplace_back("time", rfc3339_utc(unix_ns));
    std::stable_sort(all.begin(), all.end(),
                     [](const auto& a, const auto& b) { return a.first < b.first; });
    out.push_back('{');
    bool first = true;
    for (auto& kv : all) {
      if (!first) out.push_back(',');
      first = false;
      out += json_quote(kv.first);
      out.push_back(':');
      out += json_quote(kv.second);
    }
    out.push_back('}');
    return out;
  }
  if (format_ == LogFormat::TextColor) {
    // logrus TextFormatter.printColored (non-FullTimestamp): colour by level, upper-case
    // level truncated to 4 letters, [seconds since baseTimestamp], message %-44s.
    int color = 36;  // info (and unknown): blue
    if (l == Level::Debug || l == Level::Trace) color = 37;
    else if (l == Level::Warn) color = 33;
    else if (l == Level::Error || l == Level::Fatal || l == Level::Panic) color = 31;
    std::string lvl = level_name(l);
    for (auto& c : lvl) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
    lvl = lvl.substr(0, 4);
    std::string m = msg;
    if (!m.empty() && m.back() == '\n') m.pop_back();
    char head[64];
    std::snprintf(head, sizeof head, "\x1b[%dm%s\x1b[0m[%04lld] ", color, lvl.c_str(),
                  static_cast<long long>((unix_ns - base_unix_ns_) / 1000000000LL));
    out = head;
    out += m;
    if (m.size() < 44) out.append(44 - m.size(), ' ');
    out.push_back(' ');
    for (auto& kv : data) {
      char key[32];
      std::snprintf(key, sizeof key, " \x1b[%dm", color);
      out += key;
      out += kv.first;
      out += "\x1b[0m=";
      out += logrus_needs_quoting(kv.second) ? go_quote(kv.second) : kv.second;
    }
    return out;
  }
  out.reserve(64 + msg.size() + 32 * data.size());
  auto value = [&](const std::string& v) {
    if (logrus_needs_quoting(v)) out += go_quote(v);
    else out += v;
  };
  // time= is an RFC 3339 UTC stamp: always quoted (':'), never escaped.
  out += "time=\"";
  out += rfc3339_utc(unix_ns);
  out += "\" level=";
  out += level_name(l);  // [a-z] only: never quoted
  out += " msg=";
  value(msg);
  for (auto& kv : data) {
    out.push_back(' ');
    out += kv.first;
    out.push_back('=');
    value(kv.second);
  }
  return out;
}

void Logger::log(Level l, const std::string& msg, const Fields& fields) {
  if (!enabled(l)) return;
  const int fd = shared_->fd.load(std::memory_order_acquire);
  if (fd >= 0 && !shared_->custom_time.load(std::memory_order_acquire)) {
    std::string line = format(l, msg, fields, wall_now_ns());
    line.push_back('\n');
    ThreadBatch& b = thread_batch();
    if (b.depth > 0 && l > Level::Fatal) {
      if (b.fd != fd || b.gate != &shared_->gate) {
        b.flush();
        b.fd = fd;
        b.gate = &shared_->gate;
        b.keep = shared_;
      }
      b.buf += line;
      return;
    }
    if (b.depth > 0) b.flush();  // keep the order ahead of a fatal line
    if (line.size() <= PIPE_BUF) {  // one atomic write(2), on pipes too
      shared_->gate.shared([&] { write_line(fd, line); });
      return;
    }
    shared_->gate.exclusive([&] { write_line(fd, line); });
    return;
  }
  Sink sink;
  int64_t ts;
  {
    std::lock_guard<std::mutex> lk(shared_->mu);
    ts = shared_->time();
    sink = shared_->sink;
  }
  std::string line = format(l, msg, fields, ts);
  std::lock_guard<std::mutex> lk(shared_->mu);  // one line at a time across threads
  sink(line);
}

}  // namespace ksa
