#include "json.h"

#include <cstdio>
#include <cstdlib>

namespace ksa {

namespace {

class Parser {
 public:
  explicit Parser(const std::string& t) : t_(t) {}

  Status parse(JsonValue* out) {
    skip_ws();
    Status s = value(out, 0);
    if (!s.ok()) return s;
    skip_ws();
    if (i_ != t_.size()) return err("trailing data");
    return Status::OK();
  }

 private:
  Status err(const std::string& what) {
    return Status::Err("invalid JSON at offset " + std::to_string(i_) + ": " + what);
  }
  void skip_ws() {
    while (i_ < t_.size() && (t_[i_] == ' ' || t_[i_] == '\n' || t_[i_] == '\r' || t_[i_] == '\t'))
      ++i_;
  }
  bool lit(const char* s) {
    size_t n = 0;
    while (s[n]) ++n;
    if (t_.compare(i_, n, s) == 0) {
      i_ += n;
      return true;
    }
    return false;
  }

  Status value(JsonValue* v, int depth) {
    if (depth > 256) return err("nesting too deep");
    if (i_ >= t_.size()) return err("unexpected end");
    v->begin = i_;
    char c = t_[i_];
    Status s;
    if (c == '{') {
      s = object(v, depth);
    } else if (c == '[') {
      s = array(v, depth);
    } else if (c == '"') {
      v->type = JsonValue::Type::String;
      s = string(&v->str);
    } else if (c == 't') {
      if (!lit("true")) return err("bad literal");
      v->type = JsonValue::Type::Bool;
      v->b = true;
    } else if (c == 'f') {
      if (!lit("false")) return err("bad literal");
      v->type = JsonValue::Type::Bool;
      v->b = false;
    } else if (c == 'n') {
      if (!lit("null")) return err("bad literal");
      v->type = JsonValue::Type::Null;
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      s = number(v);
    } else {
      return err(std::string("unexpected character '") + c + "'");
    }
    if (!s.ok()) return s;
    v->end = i_;
    return Status::OK();
  }

  Status object(JsonValue* v, int depth) {
    v->type = JsonValue::Type::Object;
    ++i_;
    skip_ws();
    if (i_ < t_.size() && t_[i_] == '}') {
      ++i_;
      return Status::OK();
    }
    while (true) {
      skip_ws();
      if (i_ >= t_.size() || t_[i_] != '"') return err("expected object key");
      std::string key;
      Status s = string(&key);
      if (!s.ok()) return s;
      skip_ws();
      if (i_ >= t_.size() || t_[i_] != ':') return err("expected ':'");
      ++i_;
      skip_ws();
      JsonValue child;
      s = value(&child, depth + 1);
      if (!s.ok()) return s;
      v->obj.emplace_back(std::move(key), std::move(child));
      skip_ws();
      if (i_ < t_.size() && t_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < t_.size() && t_[i_] == '}') {
        ++i_;
        return Status::OK();
      }
      return err("expected ',' or '}'");
    }
  }

  Status array(JsonValue* v, int depth) {
    v->type = JsonValue::Type::Array;
    ++i_;
    skip_ws();
    if (i_ < t_.size() && t_[i_] == ']') {
      ++i_;
      return Status::OK();
    }
    while (true) {
      skip_ws();
      JsonValue child;
      Status s = value(&child, depth + 1);
      if (!s.ok()) return s;
      v->arr.push_back(std::move(child));
      skip_ws();
      if (i_ < t_.size() && t_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < t_.size() && t_[i_] == ']') {
        ++i_;
        return Status::OK();
      }
      return err("expected ',' or ']'");
    }
  }

  Status number(JsonValue* v) {
    size_t start = i_;
    if (t_[i_] == '-') ++i_;
    if (i_ >= t_.size()) return err("bad number");
    if (t_[i_] == '0') {
      ++i_;
    } else if (t_[i_] >= '1' && t_[i_] <= '9') {
      while (i_ < t_.size() && t_[i_] >= '0' && t_[i_] <= '9') ++i_;
    } else {
      return err("bad number");
    }
    if (i_ < t_.size() && t_[i_] == '.') {
      ++i_;
      size_t d = i_;
      while (i_ < t_.size() && t_[i_] >= '0' && t_[i_] <= '9') ++i_;
      if (d == i_) return err("bad fraction");
    }
    if (i_ < t_.size() && (t_[i_] == 'e' || t_[i_] == 'E')) {
      ++i_;
      if (i_ < t_.size() && (t_[i_] == '+' || t_[i_] == '-')) ++i_;
      size_t d = i_;
      while (i_ < t_.size() && t_[i_] >= '0' && t_[i_] <= '9') ++i_;
      if (d == i_) return err("bad exponent");
    }
    v->type = JsonValue::Type::Number;
    v->str.assign(t_, start, i_ - start);
    return Status::OK();
  }

  static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  bool hex4(uint32_t* out) {
    if (i_ + 4 > t_.size()) return false;
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      int h = hexval(t_[i_ + k]);
      if (h < 0) return false;
      v = (v << 4) | static_cast<uint32_t>(h);
    }
    i_ += 4;
    *out = v;
    return true;
  }

  static void put_utf8(std::string* s, uint32_t cp) {
    if (cp < 0x80) {
      s->push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      s->push_back(static_cast<char>(0xC0 | (cp >> 6)));
      s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      s->push_back(static_cast<char>(0xE0 | (cp >> 12)));
      s->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      s->push_back(static_cast<char>(0xF0 | (cp >> 18)));
      s->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      s->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }

  Status string(std::string* out) {
    ++i_;  // opening quote
    out->clear();
    while (i_ < t_.size()) {
      char c = t_[i_];
      if (c == '"') {
        ++i_;
        return Status::OK();
      }
      if (static_cast<unsigned char>(c) < 0x20) return err("control character in string");
      if (c != '\\') {
        out->push_back(c);
        ++i_;
        continue;
      }
      ++i_;
      if (i_ >= t_.size()) break;
      char e = t_[i_++];
      switch (e) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return err("bad \\u escape");
          if (cp >= 0xD800 && cp <= 0xDBFF && i_ + 1 < t_.size() && t_[i_] == '\\' &&
              t_[i_ + 1] == 'u') {
            size_t save = i_;
            i_ += 2;
            uint32_t lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo <= 0xDFFF) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              i_ = save;
              cp = 0xFFFD;
            }
          } else if (cp >= 0xD800 && cp <= 0xDFFF) {
            cp = 0xFFFD;
          }
          put_utf8(out, cp);
          break;
        }
        default:
          return err("bad escape");
      }
    }
    return err("unterminated string");
  }

  const std::string& t_;
  size_t i_ = 0;
};

}  // namespace

namespace {

// Validating single-pass scanner for json_scan_scale. Accepts exactly the grammar Parser does
// (RFC 8259, same depth limit); records only the spans it is asked about.
class Scanner {
 public:
  explicit Scanner(const std::string& t) : t_(t.data()), n_(t.size()) {}

  bool run(ScaleFields* f) {
    f_ = f;
    ws();
    if (i_ >= n_ || t_[i_] != '{') return false;  // the actuator only handles objects
    f->root_begin = i_;
    if (!object(0, kRoot)) return false;
    ws();
    return i_ == n_;
  }

 private:
  enum Ctx { kOther, kRoot, kMetadata, kSpec };

  void ws() {
    while (i_ < n_ && (t_[i_] == ' ' || t_[i_] == '\n' || t_[i_] == '\r' || t_[i_] == '\t')) ++i_;
  }
  static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  // String at t_[i_] == '"'; sets [*b, *e) to the contents and *esc if escapes occur.
  bool string(size_t* b, size_t* e, bool* esc) {
    ++i_;
    *b = i_;
    *esc = false;
    while (i_ < n_) {
      const char c = t_[i_];
      if (c == '"') {
        *e = i_++;
        return true;
      }
      if (static_cast<unsigned char>(c) < 0x20) return false;
      if (c != '\\') {
        ++i_;
        continue;
      }
      *esc = true;
      if (++i_ >= n_) return false;
      const char x = t_[i_++];
      if (x == 'u') {
        if (i_ + 4 > n_) return false;
        for (int k = 0; k < 4; ++k)
          if (hexval(t_[i_ + k]) < 0) return false;
        i_ += 4;
      } else if (x != '"' && x != '\\' && x != '/' && x != 'b' && x != 'f' && x != 'n' && x != 'r' && x != 't') {
        return false;
      }
    }
    return false;
  }
  bool number() {
    if (t_[i_] == '-') ++i_;
    if (i_ >= n_) return false;
    if (t_[i_] == '0') {
      ++i_;
    } else if (t_[i_] >= '1' && t_[i_] <= '9') {
      while (i_ < n_ && t_[i_] >= '0' && t_[i_] <= '9') ++i_;
    } else {
      return false;
    }
    if (i_ < n_ && t_[i_] == '.') {
      const size_t d = ++i_;
      while (i_ < n_ && t_[i_] >= '0' && t_[i_] <= '9') ++i_;
      if (d == i_) return false;
    }
    if (i_ < n_ && (t_[i_] == 'e' || t_[i_] == 'E')) {
      ++i_;
      if (i_ < n_ && (t_[i_] == '+' || t_[i_] == '-')) ++i_;
      const size_t d = i_;
      while (i_ < n_ && t_[i_] >= '0' && t_[i_] <= '9') ++i_;
      if (d == i_) return false;
    }
    return true;
  }
  bool lit(const char* s, size_t len) {
    if (i_ + len > n_ || std::char_traits<char>::compare(t_ + i_, s, len) != 0) return false;
    i_ += len;
    return true;
  }
  bool value(int depth, Ctx ctx) {
    if (depth > 256 || i_ >= n_) return false;
    const char c = t_[i_];
    if (c == '{') return object(depth, ctx);
    if (c == '[') return array(depth);
    if (c == '"') {
      size_t b, e;
      bool esc;
      return string(&b, &e, &esc);
    }
    if (c == 't') return lit("true", 4);
    if (c == 'f') return lit("false", 5);
    if (c == 'n') return lit("null", 4);
    if (c == '-' || (c >= '0' && c <= '9')) return number();
    return false;
  }
  bool key_is(size_t b, size_t e, const char* k, size_t len) const {
    return e - b == len && std::char_traits<char>::compare(t_ + b, k, len) == 0;
  }
  bool object(int depth, Ctx ctx) {
    const size_t open = i_++;
    ws();
    bool empty = i_ < n_ && t_[i_] == '}';
    if (ctx == kRoot) f_->root_empty = empty;
    if (ctx == kSpec) {
      f_->spec_begin = open;
      f_->spec_empty = empty;
    }
    if (empty) {
      ++i_;
      return true;
    }
    while (true) {
      ws();
      if (i_ >= n_ || t_[i_] != '"') return false;
      size_t kb, ke;
      bool kesc;
      if (!string(&kb, &ke, &kesc)) return false;
      ws();
      if (i_ >= n_ || t_[i_] != ':') return false;
      ++i_;
      ws();
      if (i_ >= n_) return false;
      Ctx child = kOther;
      if (ctx == kRoot || ctx == kMetadata || ctx == kSpec) {
        if (kesc) return false;  // a key of interest could hide behind an escape: no fast path
        if (ctx == kRoot && key_is(kb, ke, "metadata", 8)) {
          if (seen_metadata_++) return false;
          child = kMetadata;
        } else if (ctx == kRoot && key_is(kb, ke, "spec", 4)) {
          if (f_->has_spec) return false;
          f_->has_spec = true;
          f_->spec_is_object = t_[i_] == '{';
          child = kSpec;
        } else if (ctx == kMetadata && key_is(kb, ke, "resourceVersion", 15)) {
          if (seen_rv_++) return false;
          if (t_[i_] == '"') {
            f_->has_rv = true;
            if (!string(&f_->rv_begin, &f_->rv_end, &f_->rv_escaped)) return false;
            goto next;
          }
        } else if (ctx == kSpec && key_is(kb, ke, "replicas", 8)) {
          if (f_->has_replicas) return false;
          f_->has_replicas = true;
          f_->replicas_begin = i_;
          f_->replicas_null = t_[i_] == 'n';
          f_->replicas_number = t_[i_] == '-' || (t_[i_] >= '0' && t_[i_] <= '9');
          if (!value(depth + 1, kOther)) return false;
          f_->replicas_end = i_;
          goto next;
        }
      }
      if (!value(depth + 1, child)) return false;
    next:
      ws();
      if (i_ < n_ && t_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < n_ && t_[i_] == '}') {
        ++i_;
        return true;
      }
      return false;
    }
  }
  bool array(int depth) {
    ++i_;
    ws();
    if (i_ < n_ && t_[i_] == ']') {
      ++i_;
      return true;
    }
    while (true) {
      ws();
      if (!value(depth + 1, kOther)) return false;
      ws();
      if (i_ < n_ && t_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < n_ && t_[i_] == ']') {
        ++i_;
        return true;
      }
      return false;
    }
  }

  const char* t_;
  size_t n_;
  size_t i_ = 0;
  ScaleFields* f_ = nullptr;
  int seen_metadata_ = 0, seen_rv_ = 0;
};

}  // namespace

ScaleFields json_scan_scale(const std::string& text) {
  ScaleFields f;
  Scanner s(text);
  f.ok = s.run(&f);
  return f;
}

const JsonValue* JsonValue::get(const std::string& key) const {
  if (type != Type::Object) return nullptr;
  // Last duplicate wins, like encoding/json.
  for (auto it = obj.rbegin(); it != obj.rend(); ++it)
    if (it->first == key) return &it->second;
  return nullptr;
}

JsonValue* JsonValue::get(const std::string& key) {
  return const_cast<JsonValue*>(static_cast<const JsonValue*>(this)->get(key));
}

const JsonValue* JsonValue::path(std::initializer_list<const char*> keys) const {
  const JsonValue* cur = this;
  for (const char* k : keys) {
    cur = cur->get(k);
    if (!cur) return nullptr;
  }
  return cur;
}

bool JsonValue::as_int64(int64_t* out) const {
  if (type != Type::Number || str.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (str[0] == '-') {
    neg = true;
    i = 1;
  }
  uint64_t acc = 0;
  for (; i < str.size(); ++i) {
    char c = str[i];
    if (c < '0' || c > '9') return false;  // fraction/exponent: not an integer literal
    uint64_t d = static_cast<uint64_t>(c - '0');
    if (acc > (~uint64_t(0) - d) / 10) return false;
    acc = acc * 10 + d;
  }
  const uint64_t cutoff = uint64_t(1) << 63;
  if ((!neg && acc >= cutoff) || (neg && acc > cutoff)) return false;
  *out = neg ? static_cast<int64_t>(0 - acc) : static_cast<int64_t>(acc);
  return true;
}

JsonValue JsonValue::make_string(std::string s) {
  JsonValue v;
  v.type = Type::String;
  v.str = std::move(s);
  return v;
}

JsonValue JsonValue::make_number(int64_t n) {
  JsonValue v;
  v.type = Type::Number;
  v.str = std::to_string(n);
  return v;
}

JsonValue JsonValue::make_object() {
  JsonValue v;
  v.type = Type::Object;
  return v;
}

void JsonValue::set(const std::string& key, JsonValue v) {
  type = Type::Object;
  for (auto& kv : obj) {
    if (kv.first == key) {
      kv.second = std::move(v);
      return;
    }
  }
  obj.emplace_back(key, std::move(v));
}

Result<JsonValue> json_parse(const std::string& text) {
  JsonValue v;
  Parser p(text);
  Status s = p.parse(&v);
  if (!s.ok()) return Result<JsonValue>::Err(s);
  return Result<JsonValue>::Ok(std::move(v));
}

std::string json_quote(const std::string& s) {
  static const char* hex = "0123456789abcdef";
  std::string out;
  out.reserve(s.size() + 2);
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          out += "\\u00";
          out.push_back(hex[c >> 4]);
          out.push_back(hex[c & 0xF]);
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
  return out;
}

static void serialize_into(const JsonValue& v, std::string* out) {
  switch (v.type) {
    case JsonValue::Type::Null: *out += "null"; break;
    case JsonValue::Type::Bool: *out += v.b ? "true" : "false"; break;
    case JsonValue::Type::Number: *out += v.str; break;
    case JsonValue::Type::String: *out += json_quote(v.str); break;
    case JsonValue::Type::Array: {
      out->push_back('[');
      for (size_t i = 0; i < v.arr.size(); ++i) {
        if (i) out->push_back(',');
        serialize_into(v.arr[i], out);
      }
      out->push_back(']');
      break;
    }
    case JsonValue::Type::Object: {
      out->push_back('{');
      for (size_t i = 0; i < v.obj.size(); ++i) {
        if (i) out->push_back(',');
        *out += json_quote(v.obj[i].first);
        out->push_back(':');
        serialize_into(v.obj[i].second, out);
      }
      out->push_back('}');
      break;
    }
  }
}

std::string json_serialize(const JsonValue& v) {
  std::string out;
  serialize_into(v, &out);
  return out;
}

std::string json_splice(const std::string& text, const JsonValue& node,
                        const std::string& replacement) {
  std::string out;
  out.reserve(text.size() + replacement.size());
  out.append(text, 0, node.begin);
  out += replacement;
  out.append(text, node.end, std::string::npos);
  return out;
}

}  // namespace ksa
