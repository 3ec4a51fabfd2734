// logrus-compatible structured logger.
//
// The reference logs through the logrus package-level logger with default settings
// (text formatter, stderr, Info level; /root/reference/main.go:13, scale/scale.go:9). Off a
// TTY each line is
//   time="2024-01-01T00:00:00Z" level=info msg="Found 3 messages in the queue"
// This formatter reproduces that layout (fixed keys time/level/msg, then the remaining
// fields sorted by key, values quoted with Go %q only when they contain characters outside
// [A-Za-z0-9-._/@^+]) so log-based parity diffs against the reference work. On a TTY logrus
// switches to its coloured layout, e.g.
//   \x1b[36mINFO\x1b[0m[0005] Found 3 messages in the queue
// (4-letter level, seconds since process start, message padded to 44 columns, fields as
// " \x1b[36mkey\x1b[0m=value"); LogFormat::TextColor is that layout and the CLI picks it when
// stderr is a terminal, as logrus does. A JSON formatter (logrus.JSONFormatter layout) is
// offered as an extension.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace ksa {

// Lets lines of at most PIPE_BUF bytes (one atomic write(2) each) go out concurrently while a
// longer line -- possibly several writes -- goes out alone. A reader/writer lock would do, but
// its lock word is written by every line of every worker: one cache line bouncing between the
// cores (and sockets) of all tracked queues on every poll. Here each thread announces itself in
// a slot of its own cache line; the rare long-line writer raises a flag and waits for the slots
// to drain (Dekker-style: both sides store, then load, sequentially consistent).
class LineGate {
 public:
  template <class F>
  void shared(F&& write) {
    Slot& s = slots_[slot_index()];
    s.n.fetch_add(1, std::memory_order_seq_cst);
    if (long_.load(std::memory_order_seq_cst) == 0) {
      write();
      s.n.fetch_sub(1, std::memory_order_release);
      return;
    }
    s.n.fetch_sub(1, std::memory_order_release);
    std::lock_guard<std::mutex> lk(mu_);  // behind the long line
    write();
  }
  template <class F>
  void exclusive(F&& write) {
    std::lock_guard<std::mutex> lk(mu_);
    long_.store(1, std::memory_order_seq_cst);
    for (auto& s : slots_)
      while (s.n.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    write();
    long_.store(0, std::memory_order_release);
  }

 private:
  static constexpr size_t kSlots = 64;
  struct alignas(64) Slot {
    std::atomic<int> n{0};
  };
  static size_t slot_index();
  Slot slots_[kSlots];
  alignas(64) std::atomic<int> long_{0};
  std::mutex mu_;
};

// Holds back the fd-sink lines the calling thread logs while it lives and writes them with one
// write(2) when it ends (nested batches join the outermost). The control loop opens one per
// poll, so the poll's lines -- "Found N messages", the scale result -- cost one system call,
// made after the replica write instead of between the SQS response and the PUT. Each line keeps
// the timestamp of the moment it was logged and the order is unchanged; only the write moves
// (by at most one round trip: see log_flush_pending). A batch of at most PIPE_BUF bytes is one atomic write, like a
// single line; a longer one goes out alone (LineGate::exclusive). Fatal and panic lines, custom
// sinks and custom time sources are never held back.
class LogBatch {
 public:
  LogBatch();
  ~LogBatch();
  LogBatch(const LogBatch&) = delete;
  LogBatch& operator=(const LogBatch&) = delete;
  static bool active();  // is the calling thread inside a batch?
};

// Writes out what the calling thread's batch holds so far (the batch stays open). Called where
// the thread is about to wait anyway -- a request is on the wire (HttpClient), or a deliberate
// sleep (RealClock: back-off, Retry-After, throttle) -- so a line is never held back by a wait
// longer than a round trip and its write overlaps the wait. No-op outside a batch.
void log_flush_pending();

enum class Level : int { Panic = 0, Fatal = 1, Error = 2, Warn = 3, Info = 4, Debug = 5, Trace = 6 };

const char* level_name(Level l);  // "panic", ..., "warning", "info", ...
bool parse_level(const std::string& s, Level* out);

using Fields = std::vector<std::pair<std::string, std::string>>;

enum class LogFormat { Text, Json, TextColor };

class Logger {
 public:
  using Sink = std::function<void(const std::string& line)>;
  using TimeSource = std::function<int64_t()>;  // unix nanos

  Logger();
  static std::shared_ptr<Logger> default_logger();

  void set_level(Level l) { level_ = l; }
  Level level() const { return level_; }
  void set_format(LogFormat f) { format_ = f; }
  void set_base_time(int64_t unix_ns) { base_unix_ns_ = unix_ns; }
  // Replaces the output (default: stderr). The sink receives the line without '\n'. Calls are
  // serialised by the logger's mutex, so the sink need not be thread-safe.
  void set_sink(Sink s);
  // Output to a file descriptor (the default is fd 2). Each line is one write(2), which the
  // kernel keeps whole for pipes (up to PIPE_BUF), regular files and terminals, so a line on the
  // wall clock is formatted and written without taking the logger's mutex, and without
  // writing any memory the workers of other queues write (LineGate); a line longer than
  // PIPE_BUF (possibly several writes) goes out alone so nothing interleaves with its pieces.
  void set_sink_fd(int fd);
  void set_time_source(TimeSource t);
  // Fields appended to every entry of this logger (e.g. queue=... in multi-queue mode).
  void set_base_fields(Fields f) {
    base_ = std::move(f);
    sort_base();
  }
  std::shared_ptr<Logger> with_fields(const Fields& extra) const;

  bool enabled(Level l) const { return static_cast<int>(l) <= static_cast<int>(level_); }
  void log(Level l, const std::string& msg, const Fields& fields = {});
  void info(const std::string& msg) { log(Level::Info, msg); }
  void error(const std::string& msg) { log(Level::Error, msg); }
  void warn(const std::string& msg) { log(Level::Warn, msg); }
  void debug(const std::string& msg) { log(Level::Debug, msg); }

  // Exposed for tests.
  std::string format(Level l, const std::string& msg, const Fields& fields, int64_t unix_ns) const;

 private:
  int64_t base_unix_ns_;  // logrus' baseTimestamp (package init) for the TTY layout
  struct Shared {
    std::mutex mu;
    // fd sink: a line of at most PIPE_BUF bytes is one atomic write(2), so those writers go
    // concurrently; a longer line may take several writes and goes alone, so no short line can
    // land between its pieces.
    LineGate gate;
    Sink sink;
    TimeSource time;
    alignas(64) std::atomic<int> fd{2};    // >= 0: `sink` writes to this fd (lock-free path)
    std::atomic<bool> custom_time{false};  // set_time_source was called
  };
  Level level_ = Level::Info;
  LogFormat format_ = LogFormat::Text;
  void sort_base();
  Fields base_;
  Fields base_sorted_;  // base_ stable-sorted by key: the layout of a line without extra fields
  std::shared_ptr<Shared> shared_;
  friend class LogBatch;
};

// logrus TextFormatter.needsQuoting
bool logrus_needs_quoting(const std::string& s);

}  // namespace ksa
