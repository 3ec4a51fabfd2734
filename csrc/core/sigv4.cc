#include "sigv4.h"

// The low-level SHA256_* API is deprecated in OpenSSL 3 but it is the fast path: EVP one-shots
// pay a provider fetch per call, which dominated signing time (see HmacSha256Key).
#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/sha.h>

#include <cstring>

#include <algorithm>
#include <cctype>

#include "goutil.h"

namespace ksa {

std::string hex_encode(const std::string& raw) {
  static const char* hex = "0123456789abcdef";
  std::string out;
  out.reserve(raw.size() * 2);
  for (unsigned char c : raw) {
    out.push_back(hex[c >> 4]);
    out.push_back(hex[c & 0xF]);
  }
  return out;
}

namespace {

void sha256_raw(const void* data, size_t n, unsigned char out[32]) {
  SHA256_CTX c;
  SHA256_Init(&c);
  SHA256_Update(&c, data, n);
  SHA256_Final(out, &c);
}

std::string hex32(const unsigned char* md) {
  static const char* hex = "0123456789abcdef";
  std::string out(64, '0');
  for (int i = 0; i < 32; ++i) {
    out[2 * i] = hex[md[i] >> 4];
    out[2 * i + 1] = hex[md[i] & 0xF];
  }
  return out;
}

}  // namespace

std::string sha256_hex(const std::string& data) {
  unsigned char md[32];
  sha256_raw(data.data(), data.size(), md);
  return hex32(md);
}

struct HmacSha256Key::State {
  SHA256_CTX inner, outer;
};

HmacSha256Key::HmacSha256Key() : HmacSha256Key(std::string()) {}

HmacSha256Key::HmacSha256Key(const std::string& key) : st_(std::make_unique<State>()) {
  unsigned char k[64] = {0};
  if (key.size() > 64) sha256_raw(key.data(), key.size(), k);
  else std::memcpy(k, key.data(), key.size());
  unsigned char pad[64];
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x36;
  SHA256_Init(&st_->inner);
  SHA256_Update(&st_->inner, pad, 64);
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x5c;
  SHA256_Init(&st_->outer);
  SHA256_Update(&st_->outer, pad, 64);
}

HmacSha256Key::HmacSha256Key(const HmacSha256Key& o) : st_(std::make_unique<State>(*o.st_)) {}
HmacSha256Key& HmacSha256Key::operator=(const HmacSha256Key& o) {
  if (this != &o) *st_ = *o.st_;
  return *this;
}
HmacSha256Key::~HmacSha256Key() = default;

std::string HmacSha256Key::mac(const std::string& data) const {
  SHA256_CTX c = st_->inner;
  unsigned char in[32], out[32];
  SHA256_Update(&c, data.data(), data.size());
  SHA256_Final(in, &c);
  c = st_->outer;
  SHA256_Update(&c, in, 32);
  SHA256_Final(out, &c);
  return std::string(reinterpret_cast<char*>(out), 32);
}

void HmacSha256Key::mac_parts(std::initializer_list<std::string_view> parts, unsigned char out[32]) const {
  SHA256_CTX c = st_->inner;
  unsigned char in[32];
  for (auto p : parts) SHA256_Update(&c, p.data(), p.size());
  SHA256_Final(in, &c);
  c = st_->outer;
  SHA256_Update(&c, in, 32);
  SHA256_Final(out, &c);
}

std::string hmac_sha256(const std::string& key, const std::string& data) {
  return HmacSha256Key(key).mac(data);
}

std::string aws_uri_encode(const std::string& s, bool keep_slash) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  out.reserve(s.size() * 3 / 2);
  for (unsigned char c : s) {
    if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' ||
        c == '_' || c == '.' || c == '~' || (keep_slash && c == '/')) {
      out.push_back(static_cast<char>(c));
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 0xF]);
    }
  }
  return out;
}

std::string url_decode(const std::string& s, bool plus_is_space) {
  auto hv = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '%') {
      int a = (i + 1 < s.size()) ? hv(s[i + 1]) : -1;
      int b = (i + 2 < s.size()) ? hv(s[i + 2]) : -1;
      if (a >= 0 && b >= 0) {
        out.push_back(static_cast<char>((a << 4) | b));
        i += 2;
        continue;
      }
      out.push_back(c);
    } else if (c == '+' && plus_is_space) {
      out.push_back(' ');
    } else {
      out.push_back(c);
    }
  }
  return out;
}

std::vector<std::pair<std::string, std::string>> parse_query(const std::string& q) {
  std::vector<std::pair<std::string, std::string>> out;
  size_t i = 0;
  while (i <= q.size()) {
    size_t amp = q.find('&', i);
    if (amp == std::string::npos) amp = q.size();
    std::string part = q.substr(i, amp - i);
    if (!part.empty()) {
      size_t eq = part.find('=');
      if (eq == std::string::npos) {
        out.emplace_back(url_decode(part, true), "");
      } else {
        out.emplace_back(url_decode(part.substr(0, eq), true),
                         url_decode(part.substr(eq + 1), true));
      }
    }
    i = amp + 1;
  }
  return out;
}

Result<Credentials> CachedCredentials::get(int64_t unix_now_ns) {
  std::lock_guard<std::mutex> lk(mu_);
  bool fresh = have_ && (cached_.expires_unix_ns == 0 ||
                         unix_now_ns + window_ < cached_.expires_unix_ns);
  if (fresh) return Result<Credentials>::Ok(cached_);
  auto r = provider_->retrieve();
  if (!r.ok()) {
    have_ = false;
    return r;
  }
  if (!r.value.valid()) {
    have_ = false;
    return Result<Credentials>::Err(Status::Err(
        "NoCredentialProviders: no valid providers in chain"));
  }
  cached_ = r.value;
  have_ = true;
  return r;
}

void CachedCredentials::invalidate() {
  std::lock_guard<std::mutex> lk(mu_);
  if (have_) provider_->stale(cached_);
  have_ = false;
}

Result<Credentials> SharedCredentialsProvider::retrieve() {
  std::unique_lock<std::mutex> lk(mu_);
  const int64_t now = now_();
  if (have_ && (cached_.expires_unix_ns == 0 || now + window_ < cached_.expires_unix_ns))
    return Result<Credentials>::Ok(cached_);
  if (have_ && kept_ && now < retry_at_ && now + kStaleSkew < cached_.expires_unix_ns) {
    Credentials k = cached_;  // its refresh failed a moment ago: sign with it, retry later
    k.kept_after_failed_refresh = true;
    return Result<Credentials>::Ok(k);
  }
  if (fetching_) {  // another client is fetching: its outcome is this caller's too
    const uint64_t ticket = fetched_, cancels = cancels_;
    done_.wait(lk, [&] { return fetched_ != ticket || cancels_ != cancels; });
    if (fetched_ == ticket) return Result<Credentials>::Err(Status::Err("request canceled"));
    return last_;
  }
  fetching_ = true;
  fetches_++;
  lk.unlock();
  Result<Credentials> r;  // outside the lock: stale() and fetches() stay quick meanwhile
  try {
    r = inner_->retrieve();
  } catch (const std::exception& e) {  // the waiters must be released whatever happens
    r = Result<Credentials>::Err(Status::Err(e.what()));
  }
  lk.lock();
  fetching_ = false;
  const int64_t after = now_();
  if (r.ok() && r.value.valid()) {
    have_ = true;
    kept_ = false;
    cached_ = r.value;
  } else if (!r.ok() && have_ && cached_.expires_unix_ns != 0 && after + kStaleSkew < cached_.expires_unix_ns) {
    kept_ = true;  // the set still signs: keep it rather than fail the call (README.md)
    retry_at_ = after + kKeptRetry;
    Credentials k = cached_;
    k.kept_after_failed_refresh = true;
    r = Result<Credentials>::Ok(k);
  } else {
    have_ = kept_ = false;
  }
  last_ = r;
  fetched_++;
  done_.notify_all();
  return r;
}

void SharedCredentialsProvider::cancel() {
  std::lock_guard<std::mutex> lk(mu_);  // never held across a fetch: quick
  cancels_++;
  done_.notify_all();
}

void SharedCredentialsProvider::stale(const Credentials& c) {
  std::lock_guard<std::mutex> lk(mu_);
  // the first client to see this set rejected drops it; the others then get its replacement
  if (have_ && c.access_key_id == cached_.access_key_id && c.session_token == cached_.session_token &&
      c.expires_unix_ns == cached_.expires_unix_ns)
    have_ = kept_ = false;
}

namespace {

std::string lower(std::string s) {
  for (auto& c : s) c = ascii_lower(c);
  return s;
}

// Trim and collapse runs of spaces (SigV4 "Trimall").
std::string trimall(const std::string& v) {
  std::string out;
  bool space = false;
  for (char c : v) {
    if (c == ' ' || c == '\t') {
      space = true;
      continue;
    }
    if (space && !out.empty()) out.push_back(' ');
    space = false;
    out.push_back(c);
  }
  return out;
}

bool ignored_header(const std::string& lname) {
  return lname == "authorization" || lname == "user-agent" || lname == "x-amzn-trace-id" ||
         lname == "content-length" || lname == "connection" || lname == "expect";
}

}  // namespace

CanonicalParts sigv4_canonical(const std::string& method, const std::string& path,
                               const std::string& raw_query, const Headers& headers,
                               const std::vector<std::string>* only_headers,
                               const std::string& payload_hash) {
  // Canonical URI: the on-the-wire path, encoded once more (non-S3 services).
  std::string uri = path.empty() ? "/" : aws_uri_encode(path, true);

  // Canonical query: decode, sort by key then value, re-encode strictly.
  auto params = parse_query(raw_query);
  std::sort(params.begin(), params.end());
  std::string cq;
  for (size_t i = 0; i < params.size(); ++i) {
    if (i) cq.push_back('&');
    cq += aws_uri_encode(params[i].first, false);
    cq.push_back('=');
    cq += aws_uri_encode(params[i].second, false);
  }

  // Canonical headers: lowercase names; repeated headers joined with ','.
  std::vector<std::pair<std::string, std::string>> hs;
  for (auto& [k, v] : headers) {
    std::string lk = lower(k);
    if (only_headers) {
      if (std::find(only_headers->begin(), only_headers->end(), lk) == only_headers->end())
        continue;
    } else if (ignored_header(lk)) {
      continue;
    }
    bool merged = false;
    for (auto& h : hs) {
      if (h.first == lk) {
        h.second += "," + trimall(v);
        merged = true;
        break;
      }
    }
    if (!merged) hs.emplace_back(lk, trimall(v));
  }
  std::sort(hs.begin(), hs.end(),
            [](const auto& a, const auto& b) { return a.first < b.first; });
  std::string ch, sh;
  for (size_t i = 0; i < hs.size(); ++i) {
    ch += hs[i].first + ":" + hs[i].second + "\n";
    if (i) sh.push_back(';');
    sh += hs[i].first;
  }
  CanonicalParts parts;
  parts.signed_headers = sh;
  parts.canonical_request =
      method + "\n" + uri + "\n" + cq + "\n" + ch + "\n" + sh + "\n" + payload_hash;
  return parts;
}

namespace {
std::string derive_key(const std::string& secret, const std::string& date, const std::string& region,
                       const std::string& service) {
  std::string k = hmac_sha256("AWS4" + secret, date);
  k = hmac_sha256(k, region);
  k = hmac_sha256(k, service);
  return hmac_sha256(k, "aws4_request");
}
}  // namespace

std::string SigV4Signer::signing_key(const std::string& secret, const std::string& date) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!key_.empty() && key_secret_ == secret && key_date_ == date) return key_;
  key_ = derive_key(secret, date, region_, service_);
  key_secret_ = secret;
  key_date_ = date;
  key_mac_ = HmacSha256Key(key_);
  return key_;
}

void SigV4Signer::mac_with_signing_key(const std::string& secret, const std::string& date,
                                       std::initializer_list<std::string_view> parts, unsigned char out[32]) {
  std::lock_guard<std::mutex> lk(mu_);
  if (key_.empty() || key_secret_ != secret || key_date_ != date) {
    key_ = derive_key(secret, date, region_, service_);
    key_secret_ = secret;
    key_date_ = date;
    key_mac_ = HmacSha256Key(key_);
  }
  key_mac_.mac_parts(parts, out);
}

HmacSha256Key SigV4Signer::signing_mac(const std::string& secret, const std::string& date) {
  signing_key(secret, date);
  std::lock_guard<std::mutex> lk(mu_);
  return key_mac_;
}

void SigV4Signer::sign(const Credentials& creds, int64_t unix_ns, const std::string& method,
                       const std::string& path, const std::string& raw_query, Headers* headers,
                       const std::string& body, SignDebug* debug) {
  const std::string amzdate = amz_date(unix_ns);
  const std::string date = amzdate.substr(0, 8);
  headers->emplace_back("X-Amz-Date", amzdate);
  if (!creds.session_token.empty()) headers->emplace_back("X-Amz-Security-Token", creds.session_token);

  CanonicalParts parts =
      sigv4_canonical(method, path, raw_query, *headers, nullptr, sha256_hex(body));
  const std::string scope = date + "/" + region_ + "/" + service_ + "/aws4_request";
  const std::string sts =
      "AWS4-HMAC-SHA256\n" + amzdate + "\n" + scope + "\n" + sha256_hex(parts.canonical_request);
  const std::string sig = hex_encode(signing_mac(creds.secret_access_key, date).mac(sts));
  headers->emplace_back("Authorization", "AWS4-HMAC-SHA256 Credential=" + creds.access_key_id +
                                             "/" + scope + ", SignedHeaders=" +
                                             parts.signed_headers + ", Signature=" + sig);
  if (debug) {
    debug->canonical_request = parts.canonical_request;
    debug->string_to_sign = sts;
    debug->signed_headers = parts.signed_headers;
    debug->signature = sig;
    debug->scope = scope;
  }
}

SigV4Prepared SigV4Signer::prepare(const std::string& method, const std::string& path,
                                   const std::string& raw_query, const Headers& headers,
                                   const std::string& body) const {
  SigV4Prepared p;
  p.method = method;
  p.path = path;
  p.raw_query = raw_query;
  p.headers = headers;
  p.payload_hash = sha256_hex(body);
  // Reuse the generic canonicaliser for the fixed parts so both paths agree by construction.
  Headers fixed;
  for (auto& [k, v] : headers) {
    std::string lk = lower(k);
    if (lk == "x-amz-date" || lk == "x-amz-security-token" || ignored_header(lk)) continue;
    fixed.emplace_back(k, v);
  }
  std::vector<std::pair<std::string, std::string>> hs;
  for (auto& [k, v] : fixed) {
    std::string lk = lower(k);
    bool merged = false;
    for (auto& h : hs)
      if (h.first == lk) {
        h.second += "," + trimall(v);
        merged = true;
      }
    if (!merged) hs.emplace_back(lk, trimall(v));
  }
  std::sort(hs.begin(), hs.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  p.canon = std::move(hs);
  p.canonical_uri = path.empty() ? "/" : aws_uri_encode(path, true);
  auto params = parse_query(raw_query);
  std::sort(params.begin(), params.end());
  for (size_t i = 0; i < params.size(); ++i) {
    if (i) p.canonical_query.push_back('&');
    p.canonical_query += aws_uri_encode(params[i].first, false) + "=" + aws_uri_encode(params[i].second, false);
  }
  // the canonical request around the date, for the no-session-token fast path
  p.creq_prefix = p.method + "\n" + p.canonical_uri + "\n" + p.canonical_query + "\n";
  std::string after;
  bool date_done = false;
  for (auto& [k, v] : p.canon) {
    if (!date_done && std::string("x-amz-date") < k) {
      date_done = true;
      if (!p.signed_headers.empty()) p.signed_headers.push_back(';');
      p.signed_headers += "x-amz-date";
    }
    std::string& dst = date_done ? after : p.creq_prefix;
    dst += k;
    dst.push_back(':');
    dst += v;
    dst.push_back('\n');
    if (!p.signed_headers.empty()) p.signed_headers.push_back(';');
    p.signed_headers += k;
  }
  if (!date_done) {
    if (!p.signed_headers.empty()) p.signed_headers.push_back(';');
    p.signed_headers += "x-amz-date";
  }
  p.creq_prefix += "x-amz-date:";
  p.creq_suffix = "\n" + after + "\n" + p.signed_headers + "\n" + p.payload_hash;
  return p;
}

void SigV4Signer::sign_prepared(const SigV4Prepared& p, const Credentials& creds, int64_t unix_ns, Headers* out,
                                SignDebug* debug) {
  const std::string amzdate = amz_date(unix_ns);
  const std::string date = amzdate.substr(0, 8);
  if (creds.session_token.empty() && !debug && !p.creq_prefix.empty()) {
    // hash the canonical request and MAC the string to sign in place: no request, string to
    // sign or key copies (this runs on every SQS poll)
    unsigned char md[32], mac[32];
    SHA256_CTX c;
    SHA256_Init(&c);
    SHA256_Update(&c, p.creq_prefix.data(), p.creq_prefix.size());
    SHA256_Update(&c, amzdate.data(), amzdate.size());
    SHA256_Update(&c, p.creq_suffix.data(), p.creq_suffix.size());
    SHA256_Final(md, &c);
    const std::string creq_hash = hex32(md);
    std::string scope;
    scope.reserve(date.size() + region_.size() + service_.size() + 16);
    scope += date;
    scope.push_back('/');
    scope += region_;
    scope.push_back('/');
    scope += service_;
    scope += "/aws4_request";
    mac_with_signing_key(creds.secret_access_key, date,
                         {"AWS4-HMAC-SHA256\n", amzdate, "\n", scope, "\n", creq_hash}, mac);
    out->clear();
    out->reserve(p.headers.size() + 2);
    *out = p.headers;
    out->emplace_back("X-Amz-Date", amzdate);
    std::string auth;
    auth.reserve(64 + creds.access_key_id.size() + scope.size() + p.signed_headers.size() + 64);
    auth += "AWS4-HMAC-SHA256 Credential=";
    auth += creds.access_key_id;
    auth.push_back('/');
    auth += scope;
    auth += ", SignedHeaders=";
    auth += p.signed_headers;
    auth += ", Signature=";
    auth += hex32(mac);
    out->emplace_back("Authorization", std::move(auth));
    return;
  }
  *out = p.headers;
  out->emplace_back("X-Amz-Date", amzdate);
  if (!creds.session_token.empty()) out->emplace_back("X-Amz-Security-Token", creds.session_token);
  // merge the two per-request headers into the sorted fixed ones
  std::pair<std::string, std::string> extra[2] = {{"x-amz-date", amzdate},
                                                  {"x-amz-security-token", trimall(creds.session_token)}};
  const int n_extra = creds.session_token.empty() ? 1 : 2;
  std::string ch, sh;
  ch.reserve(256);
  size_t i = 0;
  int e = 0;
  auto emit = [&](const std::string& k, const std::string& v) {
    ch += k;
    ch.push_back(':');
    ch += v;
    ch.push_back('\n');
    if (!sh.empty()) sh.push_back(';');
    sh += k;
  };
  while (i < p.canon.size() || e < n_extra) {
    if (e < n_extra && (i >= p.canon.size() || extra[e].first < p.canon[i].first)) {
      emit(extra[e].first, extra[e].second);
      ++e;
    } else {
      emit(p.canon[i].first, p.canon[i].second);
      ++i;
    }
  }
  std::string creq;
  creq.reserve(p.method.size() + p.canonical_uri.size() + p.canonical_query.size() + ch.size() + sh.size() + 80);
  creq += p.method;
  creq.push_back('\n');
  creq += p.canonical_uri;
  creq.push_back('\n');
  creq += p.canonical_query;
  creq.push_back('\n');
  creq += ch;
  creq.push_back('\n');
  creq += sh;
  creq.push_back('\n');
  creq += p.payload_hash;
  const std::string scope = date + "/" + region_ + "/" + service_ + "/aws4_request";
  const std::string sts = "AWS4-HMAC-SHA256\n" + amzdate + "\n" + scope + "\n" + sha256_hex(creq);
  const std::string sig = hex_encode(signing_mac(creds.secret_access_key, date).mac(sts));
  out->emplace_back("Authorization", "AWS4-HMAC-SHA256 Credential=" + creds.access_key_id + "/" + scope +
                                         ", SignedHeaders=" + sh + ", Signature=" + sig);
  if (debug) {
    debug->canonical_request = creq;
    debug->string_to_sign = sts;
    debug->signed_headers = sh;
    debug->signature = sig;
    debug->scope = scope;
  }
}

Status sigv4_verify(const std::string& method, const std::string& path,
                    const std::string& raw_query, const Headers& headers,
                    const std::string& body, const std::string& expected_access_key,
                    const std::string& secret, const std::string& region,
                    const std::string& service) {
  std::string auth, amzdate;
  for (auto& [k, v] : headers) {
    std::string lk = lower(k);
    if (lk == "authorization") auth = v;
    if (lk == "x-amz-date") amzdate = v;
  }
  if (auth.empty()) return Status::Err("MissingAuthenticationToken", 403);
  const std::string prefix = "AWS4-HMAC-SHA256 ";
  if (auth.compare(0, prefix.size(), prefix) != 0)
    return Status::Err("IncompleteSignature: unsupported algorithm", 403);
  auto field = [&](const std::string& name) -> std::string {
    size_t p = auth.find(name + "=");
    if (p == std::string::npos) return "";
    p += name.size() + 1;
    size_t e = auth.find(',', p);
    std::string v = auth.substr(p, e == std::string::npos ? std::string::npos : e - p);
    while (!v.empty() && v.back() == ' ') v.pop_back();
    return v;
  };
  std::string cred = field("Credential"), sh = field("SignedHeaders"), sig = field("Signature");
  if (cred.empty() || sh.empty() || sig.empty() || amzdate.size() != 16)
    return Status::Err("IncompleteSignature", 403);
  size_t slash = cred.find('/');
  std::string akid = cred.substr(0, slash);
  std::string scope = slash == std::string::npos ? "" : cred.substr(slash + 1);
  if (akid != expected_access_key) return Status::Err("InvalidClientTokenId", 403);
  const std::string date = amzdate.substr(0, 8);
  const std::string want_scope = date + "/" + region + "/" + service + "/aws4_request";
  if (scope != want_scope)
    return Status::Err("SignatureDoesNotMatch: credential scope " + scope + " != " + want_scope,
                       403);
  std::vector<std::string> only;
  size_t i = 0;
  while (i <= sh.size()) {
    size_t semi = sh.find(';', i);
    if (semi == std::string::npos) semi = sh.size();
    only.push_back(sh.substr(i, semi - i));
    i = semi + 1;
  }
  if (std::find(only.begin(), only.end(), "host") == only.end())
    return Status::Err("SignatureDoesNotMatch: host not signed", 403);
  CanonicalParts parts = sigv4_canonical(method, path, raw_query, headers, &only, sha256_hex(body));
  // Derived keys change once a day per secret: cache the last one per thread (server workers).
  thread_local std::string c_secret, c_date, c_region, c_service;
  thread_local HmacSha256Key c_mac;
  if (c_secret != secret || c_date != date || c_region != region || c_service != service) {
    c_mac = HmacSha256Key(derive_key(secret, date, region, service));
    c_secret = secret;
    c_date = date;
    c_region = region;
    c_service = service;
  }
  const std::string sts = "AWS4-HMAC-SHA256\n" + amzdate + "\n" + want_scope + "\n" +
                          sha256_hex(parts.canonical_request);
  const std::string want = hex_encode(c_mac.mac(sts));
  if (want != sig) return Status::Err("SignatureDoesNotMatch", 403);
  return Status::OK();
}

}  // namespace ksa
