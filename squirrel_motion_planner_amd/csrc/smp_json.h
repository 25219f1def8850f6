// Minimal JSON reader for the robot-model / sphere fixtures (numbers via strtod: exact round trip of the
// repr() doubles the generator writes).
#pragma once
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace smp {
namespace json {

struct Value {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Value> arr;
  std::map<std::string, Value> obj;

  const Value& operator[](const std::string& k) const {
    auto it = obj.find(k);
    if (kind != Obj || it == obj.end()) throw std::runtime_error("json: missing key " + k);
    return it->second;
  }
  const Value& operator[](size_t i) const {
    if (kind != Arr || i >= arr.size()) throw std::runtime_error("json: bad index");
    return arr[i];
  }
  bool has(const std::string& k) const { return kind == Obj && obj.count(k); }
  size_t size() const { return kind == Arr ? arr.size() : obj.size(); }
  double d() const {
    if (kind != Num) throw std::runtime_error("json: not a number");
    return num;
  }
  int i() const { return (int)d(); }
  const std::string& s() const {
    if (kind != Str) throw std::runtime_error("json: not a string");
    return str;
  }
};

class Parser {
 public:
  explicit Parser(const char* t) : p_(t) {}
  Value parse() {
    Value v = value();
    ws();
    if (*p_) throw std::runtime_error("json: trailing data");
    return v;
  }

 private:
  const char* p_;
  void ws() { while (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t') ++p_; }
  Value value() {
    ws();
    Value v;
    if (*p_ == '{') {
      v.kind = Value::Obj;
      ++p_;
      ws();
      if (*p_ == '}') { ++p_; return v; }
      for (;;) {
        ws();
        std::string k = string();
        ws();
        if (*p_++ != ':') throw std::runtime_error("json: expected ':'");
        v.obj[k] = value();
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == '}') { ++p_; return v; }
        throw std::runtime_error("json: expected ',' or '}'");
      }
    }
    if (*p_ == '[') {
      v.kind = Value::Arr;
      ++p_;
      ws();
      if (*p_ == ']') { ++p_; return v; }
      for (;;) {
        v.arr.push_back(value());
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == ']') { ++p_; return v; }
        throw std::runtime_error("json: expected ',' or ']'");
      }
    }
    if (*p_ == '"') { v.kind = Value::Str; v.str = string(); return v; }
    if (!strncmp(p_, "true", 4)) { p_ += 4; v.kind = Value::Bool; v.b = true; return v; }
    if (!strncmp(p_, "false", 5)) { p_ += 5; v.kind = Value::Bool; v.b = false; return v; }
    if (!strncmp(p_, "null", 4)) { p_ += 4; return v; }
    char* end = nullptr;
    v.num = strtod(p_, &end);
    if (end == p_) throw std::runtime_error("json: bad token");
    v.kind = Value::Num;
    p_ = end;
    return v;
  }
  std::string string() {
    if (*p_ != '"') throw std::runtime_error("json: expected string");
    ++p_;
    std::string s;
    while (*p_ && *p_ != '"') {
      if (*p_ == '\\') {
        ++p_;
        char c = *p_++;
        switch (c) {
          case 'n': s += '\n'; break;
          case 't': s += '\t'; break;
          case 'u': s += '?'; p_ += 4; break;
          default: s += c;
        }
      } else {
        s += *p_++;
      }
    }
    if (*p_ != '"') throw std::runtime_error("json: unterminated string");
    ++p_;
    return s;
  }
};

inline Value parse(const char* text) { return Parser(text).parse(); }

}  // namespace json
}  // namespace smp
