// Error plumbing for the native runtime.
//
// The reference wraps every failure with github.com/pkg/errors
// (`errors.Wrap(err, msg)` -> "<msg>: <cause>", /root/reference/sqs/sqs.go:53,60,
// /root/reference/scale/scale.go:57,74,84,102). Status::wrap reproduces that text so the
// log lines ("Failed scaling up: Failed to scale up: <cause>") match byte for byte.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>

namespace ksa {

// Cache-line size for the objects each worker writes on every poll (Runner, its clients and
// their connections). They are built one queue after another on one thread, so without the
// alignment the end of one queue's object and the start of the next share a line, and two
// workers on different cores write it every poll.
constexpr std::size_t kCacheLine = 64;

class Status {
 public:
  Status() = default;
  static Status OK() { return Status(); }
  static Status Err(std::string msg, int code = 0) {
    Status s;
    s.ok_ = false;
    s.msg_ = std::move(msg);
    s.code_ = code;
    return s;
  }

  bool ok() const { return ok_; }
  const std::string& message() const { return msg_; }
  // Optional machine-readable code: HTTP status for transport/service failures, 0 otherwise.
  int code() const { return code_; }

  // pkg/errors.Wrap: "<context>: <cause>"; wrapping OK stays OK (Wrap(nil, ..) == nil).
  Status wrap(const std::string& context) const {
    if (ok_) return *this;
    return Err(context + ": " + msg_, code_);
  }

 private:
  bool ok_ = true;
  std::string msg_;
  int code_ = 0;
};

template <class T>
struct Result {
  T value{};
  Status status;

  static Result Ok(T v) {
    Result r;
    r.value = std::move(v);
    return r;
  }
  static Result Err(Status s) {
    Result r;
    r.status = std::move(s);
    return r;
  }
  bool ok() const { return status.ok(); }
};

}  // namespace ksa
