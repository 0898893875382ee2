// Minimal JSON reader for the JSON-lines metrics format
// (file-metricscollector.go:130-170) and the store journal. Numbers keep their
// source text so that "timestamp" floats can be re-formatted the way Go's
// strconv.FormatFloat(f, 'f', -1, 64) does.
#pragma once
#include <cctype>
#include <cstdlib>
#include <string>
#include <utility>
#include <vector>

namespace katib {
namespace json {

struct Value {
  enum Type { Null, Bool, Number, String, Array, Object } type = Null;
  bool b = false;
  double num = 0;
  std::string str;  // string value, or the literal text of a number
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  const Value* get(const std::string& k) const {
    // Go's json.Unmarshal into a map keeps the LAST duplicate key
    const Value* r = nullptr;
    for (const auto& kv : obj)
      if (kv.first == k) r = &kv.second;
    return r;
  }
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}
  bool parse(Value& v) {
    ws();
    if (!value(v, 0)) return false;
    ws();
    return p_ == s_.size();
  }

 private:
  const std::string& s_;
  size_t p_ = 0;
  void ws() {
    while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\t' || s_[p_] == '\n' || s_[p_] == '\r')) ++p_;
  }
  bool lit(const char* w) {
    size_t n = 0;
    while (w[n]) ++n;
    if (s_.compare(p_, n, w) != 0) return false;
    p_ += n;
    return true;
  }
  static void put_utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) {
      o += static_cast<char>(cp);
    } else if (cp < 0x800) {
      o += static_cast<char>(0xC0 | (cp >> 6));
      o += static_cast<char>(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += static_cast<char>(0xE0 | (cp >> 12));
      o += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      o += static_cast<char>(0x80 | (cp & 0x3F));
    } else {
      o += static_cast<char>(0xF0 | (cp >> 18));
      o += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
      o += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      o += static_cast<char>(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(unsigned& cp) {
    if (p_ + 4 > s_.size()) return false;
    cp = 0;
    for (int i = 0; i < 4; ++i) {
      char c = s_[p_++];
      cp <<= 4;
      if (c >= '0' && c <= '9') cp |= c - '0';
      else if (c >= 'a' && c <= 'f') cp |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') cp |= c - 'A' + 10;
      else return false;
    }
    return true;
  }
  bool string(std::string& o) {
    if (p_ >= s_.size() || s_[p_] != '"') return false;
    ++p_;
    while (p_ < s_.size()) {
      char c = s_[p_++];
      if (c == '"') return true;
      if (static_cast<unsigned char>(c) < 0x20) return false;
      if (c != '\\') {
        o += c;
        continue;
      }
      if (p_ >= s_.size()) return false;
      char e = s_[p_++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          unsigned cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00 && p_ + 6 <= s_.size() && s_[p_] == '\\' && s_[p_ + 1] == 'u') {
            p_ += 2;
            unsigned lo;
            if (!hex4(lo)) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: return false;
      }
    }
    return false;
  }
  bool number(Value& v) {
    size_t st = p_;
    if (p_ < s_.size() && s_[p_] == '-') ++p_;
    if (p_ >= s_.size()) return false;
    if (s_[p_] == '0') {
      ++p_;
    } else if (s_[p_] >= '1' && s_[p_] <= '9') {
      while (p_ < s_.size() && isdigit(static_cast<unsigned char>(s_[p_]))) ++p_;
    } else {
      return false;
    }
    if (p_ < s_.size() && s_[p_] == '.') {
      ++p_;
      size_t d = p_;
      while (p_ < s_.size() && isdigit(static_cast<unsigned char>(s_[p_]))) ++p_;
      if (p_ == d) return false;
    }
    if (p_ < s_.size() && (s_[p_] == 'e' || s_[p_] == 'E')) {
      ++p_;
      if (p_ < s_.size() && (s_[p_] == '+' || s_[p_] == '-')) ++p_;
      size_t d = p_;
      while (p_ < s_.size() && isdigit(static_cast<unsigned char>(s_[p_]))) ++p_;
      if (p_ == d) return false;
    }
    v.type = Value::Number;
    v.str = s_.substr(st, p_ - st);
    v.num = strtod(v.str.c_str(), nullptr);
    return true;
  }
  bool value(Value& v, int depth) {
    if (depth > 256 || p_ >= s_.size()) return false;
    char c = s_[p_];
    if (c == '{') {
      ++p_;
      v.type = Value::Object;
      ws();
      if (p_ < s_.size() && s_[p_] == '}') { ++p_; return true; }
      while (true) {
        ws();
        std::string k;
        if (!string(k)) return false;
        ws();
        if (p_ >= s_.size() || s_[p_] != ':') return false;
        ++p_;
        ws();
        Value child;
        if (!value(child, depth + 1)) return false;
        v.obj.emplace_back(std::move(k), std::move(child));
        ws();
        if (p_ < s_.size() && s_[p_] == ',') { ++p_; continue; }
        if (p_ < s_.size() && s_[p_] == '}') { ++p_; return true; }
        return false;
      }
    }
    if (c == '[') {
      ++p_;
      v.type = Value::Array;
      ws();
      if (p_ < s_.size() && s_[p_] == ']') { ++p_; return true; }
      while (true) {
        ws();
        Value child;
        if (!value(child, depth + 1)) return false;
        v.arr.push_back(std::move(child));
        ws();
        if (p_ < s_.size() && s_[p_] == ',') { ++p_; continue; }
        if (p_ < s_.size() && s_[p_] == ']') { ++p_; return true; }
        return false;
      }
    }
    if (c == '"') {
      v.type = Value::String;
      return string(v.str);
    }
    if (c == 't') { v.type = Value::Bool; v.b = true; return lit("true"); }
    if (c == 'f') { v.type = Value::Bool; v.b = false; return lit("false"); }
    if (c == 'n') { v.type = Value::Null; return lit("null"); }
    return number(v);
  }
};

inline bool parse(const std::string& s, Value& v) {
  Parser p(s);
  return p.parse(v);
}

}  // namespace json
}  // namespace katib
