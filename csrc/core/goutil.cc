#include "goutil.h"

#include <cstdio>
#include <ctime>

namespace ksa {

Result<int64_t> go_atoi(const std::string& s) {
  auto syntax = [&] {
    return Result<int64_t>::Err(
        Status::Err("strconv.Atoi: parsing " + go_quote(s) + ": invalid syntax"));
  };
  auto range = [&] {
    return Result<int64_t>::Err(
        Status::Err("strconv.Atoi: parsing " + go_quote(s) + ": value out of range"));
  };
  if (s.empty()) return syntax();
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return syntax();
  }
  // Base 10, no underscores (Atoi passes base 10 to ParseInt, which forbids them).
  // Like strconv.ParseUint, a uint64 overflow is reported immediately (the rest of the
  // string is not scanned); the int64 bound is checked after a complete scan.
  uint64_t acc = 0;
  const uint64_t kMaxU64 = ~uint64_t(0);
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (c < '0' || c > '9') return syntax();
    uint64_t d = static_cast<uint64_t>(c - '0');
    if (acc > (kMaxU64 - d) / 10) return range();
    acc = acc * 10 + d;
  }
  const uint64_t cutoff = uint64_t(1) << 63;
  if ((!neg && acc >= cutoff) || (neg && acc > cutoff)) return range();
  int64_t v = neg ? static_cast<int64_t>(0 - acc) : static_cast<int64_t>(acc);
  return Result<int64_t>::Ok(v);
}

namespace {

// Decodes one UTF-8 rune at s[i]; returns the rune and its width, or -1/width 1 on error.
int32_t decode_rune(const std::string& s, size_t i, size_t* width) {
  const unsigned char c0 = static_cast<unsigned char>(s[i]);
  *width = 1;
  if (c0 < 0x80) return c0;
  auto cont = [&](size_t k) -> int {
    if (i + k >= s.size()) return -1;
    unsigned char c = static_cast<unsigned char>(s[i + k]);
    if ((c & 0xC0) != 0x80) return -1;
    return c & 0x3F;
  };
  if (c0 >= 0xC2 && c0 <= 0xDF) {
    int c1 = cont(1);
    if (c1 < 0) return -1;
    *width = 2;
    return ((c0 & 0x1F) << 6) | c1;
  }
  if (c0 >= 0xE0 && c0 <= 0xEF) {
    int c1 = cont(1), c2 = cont(2);
    if (c1 < 0 || c2 < 0) return -1;
    int32_t r = ((c0 & 0x0F) << 12) | (c1 << 6) | c2;
    if (r < 0x800 || (r >= 0xD800 && r <= 0xDFFF)) return -1;
    *width = 3;
    return r;
  }
  if (c0 >= 0xF0 && c0 <= 0xF4) {
    int c1 = cont(1), c2 = cont(2), c3 = cont(3);
    if (c1 < 0 || c2 < 0 || c3 < 0) return -1;
    int32_t r = ((c0 & 0x07) << 18) | (c1 << 12) | (c2 << 6) | c3;
    if (r < 0x10000 || r > 0x10FFFF) return -1;
    *width = 4;
    return r;
  }
  return -1;
}

// Approximation of unicode.IsPrint for non-ASCII runes: Latin-1 controls, the soft hyphen,
// line/paragraph separators, BOM and the surrogate/noncharacter ranges are not printable.
bool is_print_rune(int32_t r) {
  if (r < 0x20 || r == 0x7F) return false;
  if (r < 0x7F) return true;
  if (r >= 0x80 && r < 0xA0) return false;
  if (r == 0xAD) return false;
  if (r == 0x2028 || r == 0x2029 || r == 0xFEFF) return false;
  if ((r & 0xFFFE) == 0xFFFE) return false;
  if (r >= 0xE000 && r <= 0xF8FF) return false;  // private use
  return true;
}

}  // namespace

std::string go_quote(const std::string& s) {
  static const char* hex = "0123456789abcdef";
  std::string out;
  out.reserve(s.size() + 2);
  out.push_back('"');
  size_t i = 0;
  while (i < s.size()) {
    size_t w = 1;
    int32_t r = decode_rune(s, i, &w);
    if (r < 0) {
      unsigned char b = static_cast<unsigned char>(s[i]);
      out += "\\x";
      out.push_back(hex[b >> 4]);
      out.push_back(hex[b & 0xF]);
      i += 1;
      continue;
    }
    if (r == '"' || r == '\\') {
      out.push_back('\\');
      out.push_back(static_cast<char>(r));
    } else if (is_print_rune(r)) {
      out.append(s, i, w);
    } else {
      switch (r) {
        case '\a': out += "\\a"; break;
        case '\b': out += "\\b"; break;
        case '\f': out += "\\f"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        case '\v': out += "\\v"; break;
        default: {
          char buf[16];
          if (r < ' ' || r == 0x7F) {
            std::snprintf(buf, sizeof buf, "\\x%02x", r);
          } else if (r < 0x10000) {
            std::snprintf(buf, sizeof buf, "\\u%04x", r);
          } else {
            std::snprintf(buf, sizeof buf, "\\U%08x", r);
          }
          out += buf;
        }
      }
    }
    i += w;
  }
  out.push_back('"');
  return out;
}

std::string rfc3339_utc(int64_t unix_nanos) {
  time_t secs = static_cast<time_t>(unix_nanos / 1000000000LL);
  if (unix_nanos < 0 && unix_nanos % 1000000000LL) secs -= 1;
  struct tm tm;
  gmtime_r(&secs, &tm);
  char buf[32];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

std::string amz_date(int64_t unix_nanos) {
  time_t secs = static_cast<time_t>(unix_nanos / 1000000000LL);
  struct tm tm;
  gmtime_r(&secs, &tm);
  char buf[32];
  std::strftime(buf, sizeof buf, "%Y%m%dT%H%M%SZ", &tm);
  return buf;
}

}  // namespace ksa
