// Go standard-library behaviours the reference relies on implicitly.
//
// * strconv.Atoi -- the per-attribute count parser (/root/reference/sqs/sqs.go:58), including
//   its exact error strings, which surface in the "Failed to get SQS messages" log line.
// * strconv.Quote -- logrus' text formatter quotes field values with %q.
// * time.RFC3339 -- logrus' default timestamp format.
#pragma once

#include <cstdint>
#include <string>

#include "status.h"

namespace ksa {

// strconv.Atoi on a 64-bit platform. Errors are formatted like *strconv.NumError:
//   strconv.Atoi: parsing "abc": invalid syntax
//   strconv.Atoi: parsing "9999999999999999999": value out of range
Result<int64_t> go_atoi(const std::string& s);

// strconv.Quote (UTF-8 aware; invalid bytes become \xNN).
std::string go_quote(const std::string& s);

// RFC3339 ("2006-01-02T15:04:05Z07:00") in UTC for the given unix time.
std::string rfc3339_utc(int64_t unix_nanos);
// time.Parse(time.RFC3339, s): "2006-01-02T15:04:05[.frac](Z|+07:00)". false on bad input.
bool parse_rfc3339(const std::string& s, int64_t* unix_nanos);
// ISO-8601 basic format used by SigV4: "20150830T123600Z" and its date part "20150830".
std::string amz_date(int64_t unix_nanos);

// Wrapping int32 arithmetic, matching Go's defined overflow for int32(x) conversions and
// `*currentReplicas + int32(p.ScaleUpPods)` (/root/reference/scale/scale.go:62-69).
// ASCII-only lower case, as Go's textproto/strings.ToLower for header names and SigV4 (C's
// tolower follows the process locale, which Python sets from the environment, and is a call).
inline char ascii_lower(char c) { return (c >= 'A' && c <= 'Z') ? static_cast<char>(c + ('a' - 'A')) : c; }
inline int32_t go_int32(int64_t v) { return static_cast<int32_t>(static_cast<uint32_t>(static_cast<uint64_t>(v))); }
inline int32_t wrap_add32(int32_t a, int32_t b) {
  return static_cast<int32_t>(static_cast<uint32_t>(a) + static_cast<uint32_t>(b));
}
inline int32_t wrap_sub32(int32_t a, int32_t b) {
  return static_cast<int32_t>(static_cast<uint32_t>(a) - static_cast<uint32_t>(b));
}
inline int64_t wrap_add64(int64_t a, int64_t b) {
  return static_cast<int64_t>(static_cast<uint64_t>(a) + static_cast<uint64_t>(b));
}

}  // namespace ksa
