// Minimal JSON DOM for the node-side native tools (OCI runtime shim, CDI specs).
//
// Just enough for OCI bundle config.json and CDI specs: objects keep their key order (so a
// rewritten config.json diffs cleanly), numbers keep their original text (uid/gid, device
// major/minor and 64-bit values survive a round trip bit-exactly), strings are UTF-8 with
// \uXXXX escapes decoded (including surrogate pairs) and re-escaped minimally on output.
#pragma once

#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace minijson {

struct Value;
using Object = std::vector<std::pair<std::string, Value>>;
using Array = std::vector<Value>;

struct Value {
  enum Kind { Null, Bool, Number, String, Arr, Obj } kind = Null;
  bool b = false;
  std::string s;   // string contents, or number text
  Array a;
  Object o;

  Value() = default;
  static Value null() { return Value(); }
  static Value boolean(bool v) { Value x; x.kind = Bool; x.b = v; return x; }
  static Value number(long long v) { Value x; x.kind = Number; x.s = std::to_string(v); return x; }
  static Value number_text(std::string t) { Value x; x.kind = Number; x.s = std::move(t); return x; }
  static Value string(std::string v) { Value x; x.kind = String; x.s = std::move(v); return x; }
  static Value array() { Value x; x.kind = Arr; return x; }
  static Value object() { Value x; x.kind = Obj; return x; }

  bool is_null() const { return kind == Null; }
  bool is_object() const { return kind == Obj; }
  bool is_array() const { return kind == Arr; }
  bool is_string() const { return kind == String; }

  // object access
  const Value* find(const std::string& k) const {
    if (kind != Obj) return nullptr;
    for (auto& kv : o) if (kv.first == k) return &kv.second;
    return nullptr;
  }
  Value* find(const std::string& k) {
    if (kind != Obj) return nullptr;
    for (auto& kv : o) if (kv.first == k) return &kv.second;
    return nullptr;
  }
  // get-or-create a member (turns null into an object)
  Value& operator[](const std::string& k) {
    if (kind == Null) kind = Obj;
    if (kind != Obj) throw std::runtime_error("json: member access on non-object");
    for (auto& kv : o) if (kv.first == k) return kv.second;
    o.emplace_back(k, Value());
    return o.back().second;
  }
  bool erase(const std::string& k) {
    for (auto it = o.begin(); it != o.end(); ++it)
      if (it->first == k) { o.erase(it); return true; }
    return false;
  }
  void push(Value v) {
    if (kind == Null) kind = Arr;
    a.push_back(std::move(v));
  }
  std::string str(const std::string& dflt = "") const { return kind == String ? s : dflt; }
  long long integer(long long dflt = 0) const {
    if (kind != Number) return dflt;
    try { return std::stoll(s); } catch (...) { return dflt; }
  }
};

class Parser {
 public:
  explicit Parser(const std::string& text) : t_(text) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t p_ = 0;
  int depth_ = 0;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(p_));
  }
  void ws() { while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\r' || t_[p_] == '\t')) ++p_; }
  bool lit(const char* w) {
    size_t n = 0;
    while (w[n]) ++n;
    if (t_.compare(p_, n, w) == 0) { p_ += n; return true; }
    return false;
  }
  Value value() {
    ws();
    if (p_ >= t_.size()) fail("unexpected end");
    char c = t_[p_];
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') return Value::string(string());
    if (lit("true")) return Value::boolean(true);
    if (lit("false")) return Value::boolean(false);
    if (lit("null")) return Value::null();
    return number();
  }
  Value object() {
    if (++depth_ > 256) fail("nesting too deep");
    ++p_;
    Value v = Value::object();
    ws();
    if (p_ < t_.size() && t_[p_] == '}') { ++p_; --depth_; return v; }
    for (;;) {
      ws();
      if (p_ >= t_.size() || t_[p_] != '"') fail("expected key");
      std::string k = string();
      ws();
      if (p_ >= t_.size() || t_[p_] != ':') fail("expected ':'");
      ++p_;
      v.o.emplace_back(std::move(k), value());
      ws();
      if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
      if (p_ < t_.size() && t_[p_] == '}') { ++p_; break; }
      fail("expected ',' or '}'");
    }
    --depth_;
    return v;
  }
  Value array() {
    if (++depth_ > 256) fail("nesting too deep");
    ++p_;
    Value v = Value::array();
    ws();
    if (p_ < t_.size() && t_[p_] == ']') { ++p_; --depth_; return v; }
    for (;;) {
      v.a.push_back(value());
      ws();
      if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
      if (p_ < t_.size() && t_[p_] == ']') { ++p_; break; }
      fail("expected ',' or ']'");
    }
    --depth_;
    return v;
  }
  // RFC 8259 number: -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)? -- its text is kept and written back
  // verbatim, so anything looser ("1.", "--1", ".5", "1e") would make a rewritten config.json invalid
  // (tests/native/fuzz_minijson.cpp found the loose form accepting "[.]").
  Value number() {
    const size_t s = p_;
    auto digit = [&] { return p_ < t_.size() && t_[p_] >= '0' && t_[p_] <= '9'; };
    auto digits = [&] {
      const size_t b = p_;
      while (digit()) ++p_;
      return p_ > b;
    };
    if (p_ < t_.size() && t_[p_] == '-') ++p_;
    if (p_ < t_.size() && t_[p_] == '0') ++p_;
    else if (!digits()) fail("invalid value");
    if (p_ < t_.size() && t_[p_] == '.') {
      ++p_;
      if (!digits()) fail("invalid number");
    }
    if (p_ < t_.size() && (t_[p_] == 'e' || t_[p_] == 'E')) {
      ++p_;
      if (p_ < t_.size() && (t_[p_] == '+' || t_[p_] == '-')) ++p_;
      if (!digits()) fail("invalid number");
    }
    return Value::number_text(t_.substr(s, p_ - s));
  }
  unsigned hex4() {
    if (p_ + 4 > t_.size()) fail("bad \\u escape");
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = t_[p_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) out += char(cp);
    else if (cp < 0x800) { out += char(0xC0 | (cp >> 6)); out += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += char(0xE0 | (cp >> 12)); out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F));
    } else {
      out += char(0xF0 | (cp >> 18)); out += char(0x80 | ((cp >> 12) & 0x3F));
      out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F));
    }
  }
  std::string string() {
    ++p_;  // opening quote
    std::string out;
    while (p_ < t_.size()) {
      char c = t_[p_++];
      if (c == '"') return out;
      if (c != '\\') { out += c; continue; }
      if (p_ >= t_.size()) break;
      char e = t_[p_++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00) {      // a high surrogate must be followed by a low one
            if (!(p_ + 1 < t_.size() && t_[p_] == '\\' && t_[p_ + 1] == 'u')) fail("lone surrogate");
            p_ += 2;
            const unsigned lo = hex4();
            if (lo < 0xDC00 || lo > 0xDFFF) fail("bad surrogate pair");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            fail("lone surrogate");
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    fail("unterminated string");
  }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

inline void escape(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += char(c);
        }
    }
  }
  out += '"';
}

inline void dump(std::string& out, const Value& v, int indent = -1, int level = 0) {
  auto nl = [&](int l) {
    if (indent < 0) return;
    out += '\n';
    out.append(size_t(indent * l), ' ');
  };
  switch (v.kind) {
    case Value::Null: out += "null"; break;
    case Value::Bool: out += v.b ? "true" : "false"; break;
    case Value::Number: out += v.s; break;
    case Value::String: escape(out, v.s); break;
    case Value::Arr:
      out += '[';
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) out += ',';
        nl(level + 1);
        dump(out, v.a[i], indent, level + 1);
      }
      if (!v.a.empty()) nl(level);
      out += ']';
      break;
    case Value::Obj:
      out += '{';
      for (size_t i = 0; i < v.o.size(); ++i) {
        if (i) out += ',';
        nl(level + 1);
        escape(out, v.o[i].first);
        out += indent < 0 ? ":" : ": ";
        dump(out, v.o[i].second, indent, level + 1);
      }
      if (!v.o.empty()) nl(level);
      out += '}';
      break;
  }
}

inline std::string dump(const Value& v, int indent = -1) {
  std::string out;
  dump(out, v, indent);
  return out;
}

}  // namespace minijson
