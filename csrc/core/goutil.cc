#include "goutil.h"

#include <cstdint>
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
    // Runs of printable ASCII other than '"' and '\\' are copied as they are, in one append.
    size_t j = i;
    while (j < s.size() && s[j] >= 0x20 && s[j] < 0x7F && s[j] != '"' && s[j] != '\\') ++j;
    if (j > i) {
      out.append(s, i, j - i);
      i = j;
      continue;
    }
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

namespace {

// UTC calendar fields of a Unix time, by arithmetic (H. Hinnant's civil_from_days). Not
// gmtime_r + strftime: glibc takes its process-wide tzset lock in both, and strftime also
// re-runs tzset() -- with TZ unset that is a getenv, a free + strdup and a stat() of
// /etc/localtime under the lock, on every call. Every SigV4 signature (X-Amz-Date) and every
// log line formats a time, so workers tracking different queues serialised on that lock; one
// process per queue never did.
struct UtcFields {
  int64_t year;
  unsigned month, day, hour, minute, second;
};

UtcFields utc_fields(int64_t unix_nanos) {
  int64_t secs = unix_nanos / 1000000000LL;
  if (unix_nanos < 0 && unix_nanos % 1000000000LL) secs -= 1;  // floor
  int64_t days = secs / 86400;
  int64_t rem = secs % 86400;
  if (rem < 0) {
    rem += 86400;
    days -= 1;
  }
  const int64_t z = days + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = static_cast<unsigned>(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  UtcFields f;
  f.day = doy - (153 * mp + 2) / 5 + 1;
  f.month = mp < 10 ? mp + 3 : mp - 9;
  f.year = static_cast<int64_t>(yoe) + era * 400 + (f.month <= 2);
  f.hour = static_cast<unsigned>(rem / 3600);
  f.minute = static_cast<unsigned>(rem % 3600 / 60);
  f.second = static_cast<unsigned>(rem % 60);
  return f;
}

// Appends v as exactly `width` decimal digits (v < 10^width).
char* put_digits(char* p, uint64_t v, int width) {
  for (int i = width - 1; i >= 0; --i) {
    p[i] = static_cast<char>('0' + v % 10);
    v /= 10;
  }
  return p + width;
}

// "%Y" of strftime: the year in decimal, at least 4 digits here (int64 nanoseconds only span
// the years 1677..2262, so this is always four).
char* put_year(char* p, int64_t y) {
  if (y >= 0 && y <= 9999) return put_digits(p, static_cast<uint64_t>(y), 4);
  const std::string s = std::to_string(y);
  for (char c : s) *p++ = c;
  return p;
}

}  // namespace

std::string rfc3339_utc(int64_t unix_nanos) {
  const UtcFields f = utc_fields(unix_nanos);
  char buf[48];
  char* p = put_year(buf, f.year);
  *p++ = '-';
  p = put_digits(p, f.month, 2);
  *p++ = '-';
  p = put_digits(p, f.day, 2);
  *p++ = 'T';
  p = put_digits(p, f.hour, 2);
  *p++ = ':';
  p = put_digits(p, f.minute, 2);
  *p++ = ':';
  p = put_digits(p, f.second, 2);
  *p++ = 'Z';
  return std::string(buf, static_cast<size_t>(p - buf));
}

namespace {

// Days since 1970-01-01 of a proleptic Gregorian date (H. Hinnant's days_from_civil).
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = static_cast<unsigned>(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + static_cast<int64_t>(doe) - 719468;
}

bool fixed_digits(const std::string& s, size_t pos, size_t n, int* out) {
  if (pos + n > s.size()) return false;
  int v = 0;
  for (size_t i = pos; i < pos + n; ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
  }
  *out = v;
  return true;
}

}  // namespace

bool parse_rfc3339(const std::string& s, int64_t* unix_nanos) {
  int Y, M, D, h, m, sec;
  if (!fixed_digits(s, 0, 4, &Y) || s.size() < 20 || s[4] != '-' || !fixed_digits(s, 5, 2, &M) || s[7] != '-' ||
      !fixed_digits(s, 8, 2, &D) || (s[10] != 'T' && s[10] != 't') || !fixed_digits(s, 11, 2, &h) ||
      s[13] != ':' || !fixed_digits(s, 14, 2, &m) || s[16] != ':' || !fixed_digits(s, 17, 2, &sec))
    return false;
  static const int kDays[] = {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  if (M < 1 || M > 12 || D < 1 || D > kDays[M - 1] || (M == 2 && D == 29 && !leap) || h > 23 || m > 59 || sec > 59)
    return false;
  size_t i = 19;
  int64_t frac = 0;
  if (i < s.size() && s[i] == '.') {
    size_t j = i + 1;
    int64_t scale = 100000000;
    while (j < s.size() && s[j] >= '0' && s[j] <= '9') {
      frac += (s[j] - '0') * scale;
      scale /= 10;
      ++j;
    }
    if (j == i + 1) return false;
    i = j;
  }
  int64_t offset = 0;
  if (i < s.size() && (s[i] == 'Z' || s[i] == 'z')) {
    ++i;
  } else if (i < s.size() && (s[i] == '+' || s[i] == '-')) {
    int oh, om;
    if (!fixed_digits(s, i + 1, 2, &oh) || i + 3 >= s.size() || s[i + 3] != ':' || !fixed_digits(s, i + 4, 2, &om) ||
        oh > 23 || om > 59)
      return false;
    offset = (oh * 3600 + om * 60) * (s[i] == '-' ? -1 : 1);
    i += 6;
  } else {
    return false;
  }
  if (i != s.size()) return false;
  const int64_t secs = days_from_civil(Y, static_cast<unsigned>(M), static_cast<unsigned>(D)) * 86400 +
                       h * 3600 + m * 60 + sec - offset;
  // int64 nanoseconds span 1677..2262; Go's time.Time reaches further. Saturate, which keeps
  // every comparison with a representable instant (an expiry in 3000 simply never passes).
  constexpr int64_t kMaxSecs = INT64_MAX / 1000000000LL - 1;
  if (secs > kMaxSecs) {
    *unix_nanos = INT64_MAX;
  } else if (secs < -kMaxSecs) {
    *unix_nanos = INT64_MIN;
  } else {
    *unix_nanos = secs * 1000000000LL + frac;
  }
  return true;
}

std::string amz_date(int64_t unix_nanos) {
  const UtcFields f = utc_fields(unix_nanos);
  char buf[48];
  char* p = put_year(buf, f.year);
  p = put_digits(p, f.month, 2);
  p = put_digits(p, f.day, 2);
  *p++ = 'T';
  p = put_digits(p, f.hour, 2);
  p = put_digits(p, f.minute, 2);
  p = put_digits(p, f.second, 2);
  *p++ = 'Z';
  return std::string(buf, static_cast<size_t>(p - buf));
}

}  // namespace ksa
