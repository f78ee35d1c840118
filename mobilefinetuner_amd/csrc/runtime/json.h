// Minimal, fast JSON reader/writer for the host runtime (safetensors headers, HF config.json,
// vocab.json, tokenizer.json, pretokenized meta.json, trainer_state.json).
// Replaces the reference's regex-based field extraction (graph/safetensors_loader.cpp:58-109,
// graph/gpt2_model.cpp:41-71, core/tokenizer_gemma.cpp:203-271) with a real parser.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mft {
namespace json {

struct Value;
using Object = std::vector<std::pair<std::string, Value>>;  // keeps file order
using Array = std::vector<Value>;

struct Value {
  enum Type { Null, Bool, Number, String, Arr, Obj } type = Null;
  bool b = false;
  double num = 0.0;
  bool is_int = false;
  int64_t i = 0;
  std::string str;
  std::shared_ptr<Array> arr;
  std::shared_ptr<Object> obj;

  bool is_null() const { return type == Null; }
  bool is_object() const { return type == Obj; }
  bool is_array() const { return type == Arr; }
  bool is_string() const { return type == String; }
  bool is_number() const { return type == Number; }
  const Value* get(const std::string& k) const {
    if (type != Obj) return nullptr;
    for (auto& kv : *obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Value& operator[](const std::string& k) const {
    const Value* v = get(k);
    if (!v) throw std::runtime_error("json: missing key '" + k + "'");
    return *v;
  }
  int64_t as_int() const {
    if (type != Number) throw std::runtime_error("json: not a number");
    return is_int ? i : (int64_t)num;
  }
  double as_double() const {
    if (type != Number) throw std::runtime_error("json: not a number");
    return is_int ? (double)i : num;
  }
  const std::string& as_string() const {
    if (type != String) throw std::runtime_error("json: not a string");
    return str;
  }
  const Array& as_array() const {
    if (type != Arr) throw std::runtime_error("json: not an array");
    return *arr;
  }
  const Object& as_object() const {
    if (type != Obj) throw std::runtime_error("json: not an object");
    return *obj;
  }
};

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), end_(p + n) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != end_) fail("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* end_;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json parse error: ") + m); }
  void ws() {
    while (p_ < end_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) s += (char)cp;
    else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
    } else {
      s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 0x3F));
      s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (end_ - p_ < 4) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string() {
    if (*p_ != '"') fail("expected string");
    ++p_;
    std::string s;
    const char* run = p_;
    while (true) {
      if (p_ >= end_) fail("unterminated string");
      char c = *p_;
      if (c == '"') { s.append(run, p_); ++p_; return s; }
      if (c == '\\') {
        s.append(run, p_);
        ++p_;
        if (p_ >= end_) fail("bad escape");
        char e = *p_++;
        switch (e) {
          case '"': s += '"'; break;
          case '\\': s += '\\'; break;
          case '/': s += '/'; break;
          case 'b': s += '\b'; break;
          case 'f': s += '\f'; break;
          case 'n': s += '\n'; break;
          case 'r': s += '\r'; break;
          case 't': s += '\t'; break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && end_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
              p_ += 2;
              uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(s, cp);
            break;
          }
          default: fail("bad escape char");
        }
        run = p_;
      } else {
        ++p_;
      }
    }
  }
  Value value() {
    ws();
    if (p_ >= end_) fail("unexpected end");
    Value v;
    char c = *p_;
    if (c == '{') {
      ++p_;
      v.type = Value::Obj;
      v.obj = std::make_shared<Object>();
      ws();
      if (*p_ == '}') { ++p_; return v; }
      while (true) {
        ws();
        std::string k = string();
        ws();
        if (*p_ != ':') fail("expected ':'");
        ++p_;
        v.obj->emplace_back(std::move(k), value());
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == '}') { ++p_; return v; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p_;
      v.type = Value::Arr;
      v.arr = std::make_shared<Array>();
      ws();
      if (*p_ == ']') { ++p_; return v; }
      while (true) {
        v.arr->push_back(value());
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == ']') { ++p_; return v; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v.type = Value::String;
      v.str = string();
      return v;
    }
    if (c == 't' && end_ - p_ >= 4 && std::string(p_, 4) == "true") { p_ += 4; v.type = Value::Bool; v.b = true; return v; }
    if (c == 'f' && end_ - p_ >= 5 && std::string(p_, 5) == "false") { p_ += 5; v.type = Value::Bool; return v; }
    if (c == 'n' && end_ - p_ >= 4 && std::string(p_, 4) == "null") { p_ += 4; return v; }
    // number
    const char* s = p_;
    bool isint = true;
    if (*p_ == '-' || *p_ == '+') ++p_;
    while (p_ < end_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '-' || *p_ == '+')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') isint = false;
      ++p_;
    }
    if (p_ == s) fail("unexpected character");
    std::string t(s, p_);
    v.type = Value::Number;
    v.is_int = isint;
    if (isint) v.i = std::strtoll(t.c_str(), nullptr, 10);
    v.num = std::strtod(t.c_str(), nullptr);
    return v;
  }
};

inline Value parse(const std::string& s) { return Parser(s.data(), s.size()).parse(); }
inline Value parse(const char* p, size_t n) { return Parser(p, n).parse(); }

inline std::string escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  o += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof(buf), "\\u%04x", c);
          o += buf;
        } else {
          o += (char)c;
        }
    }
  }
  o += '"';
  return o;
}

}  // namespace json
}  // namespace mft
