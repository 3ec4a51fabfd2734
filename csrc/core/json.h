// Minimal JSON DOM with source spans.
//
// Used for Kubernetes objects (Deployment / autoscaling/v1 Scale / Status), the AWS JSON 1.0
// SQS protocol and the fakes. Every node remembers the byte range it was parsed from, so the
// replica actuator can rewrite `spec.replicas` in the fetched Deployment without
// re-serialising (and possibly dropping) fields it does not model -- the reference gets the
// same effect from client-go's typed round trip (/root/reference/scale/scale.go:55-72).
#pragma once

#include <cstdint>
#include <initializer_list>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "status.h"

namespace ksa {

struct JsonValue {
  enum class Type { Null, Bool, Number, String, Array, Object };
  Type type = Type::Null;
  bool b = false;
  std::string str;  // decoded string, or the raw number literal
  std::vector<JsonValue> arr;
  std::vector<std::pair<std::string, JsonValue>> obj;  // insertion order preserved
  size_t begin = 0, end = 0;                           // [begin, end) in the source text

  bool is_object() const { return type == Type::Object; }
  bool is_string() const { return type == Type::String; }
  bool is_number() const { return type == Type::Number; }
  const JsonValue* get(const std::string& key) const;
  JsonValue* get(const std::string& key);
  const JsonValue* path(std::initializer_list<const char*> keys) const;
  // Integer value of a Number node (fails on fractions/overflow).
  bool as_int64(int64_t* out) const;
  std::string string_or(const std::string& dflt) const { return is_string() ? str : dflt; }

  static JsonValue make_string(std::string s);
  static JsonValue make_number(int64_t v);
  static JsonValue make_object();
  void set(const std::string& key, JsonValue v);  // replaces or appends
};

Result<JsonValue> json_parse(const std::string& text);
std::string json_serialize(const JsonValue& v);
std::string json_quote(const std::string& s);

// The fields the replica actuator needs from a Deployment or autoscaling/v1 Scale, located by
// one validating pass over the text with no DOM and no allocation (json_parse builds a tree of
// strings and vectors for every field of a ~3 KB Deployment on every poll). Offsets are into
// the scanned text. `ok` is false -- and the caller must fall back to json_parse -- whenever
// the text is not valid JSON or is anything but the plain case: keys of interest written with
// escapes, duplicated `metadata` / `spec` / `resourceVersion` / `replicas` keys, nesting deeper
// than json_parse allows. In the plain case the answer is exactly what json_parse + path()
// would give.
struct ScaleFields {
  bool ok = false;
  size_t root_begin = 0;         // offset of the root object's '{'
  bool root_empty = false;
  bool has_rv = false;           // metadata.resourceVersion is a string ...
  bool rv_escaped = false;       // ... containing escapes (decode with json_parse)
  size_t rv_begin = 0, rv_end = 0;  // its contents, without the quotes
  bool has_spec = false;         // root key "spec" present
  bool spec_is_object = false;
  size_t spec_begin = 0;         // offset of spec's '{'
  bool spec_empty = false;
  bool has_replicas = false;     // spec.replicas present (any type)
  bool replicas_null = false;
  bool replicas_number = false;
  size_t replicas_begin = 0, replicas_end = 0;
};
ScaleFields json_scan_scale(const std::string& text);

// Replaces the bytes of `node` (located in `text`) with `replacement`.
std::string json_splice(const std::string& text, const JsonValue& node,
                        const std::string& replacement);

}  // namespace ksa
