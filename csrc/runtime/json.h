// Minimal JSON value + parser + serializer for the arena runtime tools (no third-party deps).
// Supports objects, arrays, strings (with \uXXXX escapes), numbers, booleans and null.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace arena {

class Json {
 public:
  enum Type { Null, Bool, Number, String, Array, Object };

  Json() : type_(Null) {}
  Json(bool b) : type_(Bool), b_(b) {}                       // NOLINT
  Json(double d) : type_(Number), d_(d) {}                   // NOLINT
  Json(int i) : type_(Number), d_(i) {}                      // NOLINT
  Json(long long i) : type_(Number), d_((double)i) {}        // NOLINT
  Json(const char* s) : type_(String), s_(s) {}              // NOLINT
  Json(std::string s) : type_(String), s_(std::move(s)) {}   // NOLINT

  static Json array() { Json j; j.type_ = Array; return j; }
  static Json object() { Json j; j.type_ = Object; return j; }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Null; }
  bool is_object() const { return type_ == Object; }
  bool is_array() const { return type_ == Array; }

  bool as_bool(bool dflt = false) const { return type_ == Bool ? b_ : dflt; }
  double as_num(double dflt = 0) const { return type_ == Number ? d_ : dflt; }
  long long as_int(long long dflt = 0) const { return type_ == Number ? (long long)d_ : dflt; }
  const std::string& as_str() const {
    static const std::string empty;
    return type_ == String ? s_ : empty;
  }

  // object access
  bool has(const std::string& k) const { return type_ == Object && o_.count(k); }
  const Json& operator[](const std::string& k) const {
    static const Json null;
    if (type_ != Object) return null;
    auto it = o_.find(k);
    return it == o_.end() ? null : it->second;
  }
  Json& set(const std::string& k, Json v) {
    if (type_ != Object) { type_ = Object; o_.clear(); }
    o_[k] = std::move(v);
    return o_[k];
  }
  const std::map<std::string, Json>& items() const { return o_; }

  // array access
  size_t size() const { return type_ == Array ? a_.size() : (type_ == Object ? o_.size() : 0); }
  const Json& at(size_t i) const { return a_.at(i); }
  void push(Json v) {
    if (type_ != Array) { type_ = Array; a_.clear(); }
    a_.push_back(std::move(v));
  }
  const std::vector<Json>& elems() const { return a_; }

  std::string dump() const {
    std::string out;
    dump_to(out);
    return out;
  }

  static Json parse(const std::string& text) {
    size_t i = 0;
    Json v = parse_value(text, i);
    skip_ws(text, i);
    if (i != text.size()) throw std::runtime_error("json: trailing characters");
    return v;
  }

 private:
  Type type_;
  bool b_ = false;
  double d_ = 0;
  std::string s_;
  std::vector<Json> a_;
  std::map<std::string, Json> o_;

  static void escape(const std::string& s, std::string& out) {
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
            out += (char)c;
          }
      }
    }
    out += '"';
  }

  void dump_to(std::string& out) const {
    switch (type_) {
      case Null: out += "null"; break;
      case Bool: out += b_ ? "true" : "false"; break;
      case Number: {
        if (std::isfinite(d_) && d_ == std::floor(d_) && std::fabs(d_) < 9.0e15) {
          out += std::to_string((long long)d_);
        } else if (std::isfinite(d_)) {
          char buf[40];
          std::snprintf(buf, sizeof buf, "%.17g", d_);
          out += buf;
        } else {
          out += "null";
        }
        break;
      }
      case String: escape(s_, out); break;
      case Array: {
        out += '[';
        for (size_t i = 0; i < a_.size(); ++i) {
          if (i) out += ',';
          a_[i].dump_to(out);
        }
        out += ']';
        break;
      }
      case Object: {
        out += '{';
        bool first = true;
        for (const auto& kv : o_) {
          if (!first) out += ',';
          first = false;
          escape(kv.first, out);
          out += ':';
          kv.second.dump_to(out);
        }
        out += '}';
        break;
      }
    }
  }

  static void skip_ws(const std::string& t, size_t& i) {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\r' || t[i] == '\t')) ++i;
  }

  static void append_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }

  static std::string parse_string(const std::string& t, size_t& i) {
    if (t[i] != '"') throw std::runtime_error("json: expected string");
    ++i;
    std::string out;
    while (i < t.size() && t[i] != '"') {
      char c = t[i++];
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i >= t.size()) break;
      char e = t[i++];
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
          if (i + 4 > t.size()) throw std::runtime_error("json: bad \\u escape");
          uint32_t cp = (uint32_t)std::stoul(t.substr(i, 4), nullptr, 16);
          i += 4;
          if (cp >= 0xD800 && cp <= 0xDBFF && i + 6 <= t.size() && t[i] == '\\' && t[i + 1] == 'u') {
            uint32_t lo = (uint32_t)std::stoul(t.substr(i + 2, 4), nullptr, 16);
            if (lo >= 0xDC00 && lo <= 0xDFFF) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              i += 6;
            }
          }
          append_utf8(out, cp);
          break;
        }
        default: throw std::runtime_error("json: bad escape");
      }
    }
    if (i >= t.size()) throw std::runtime_error("json: unterminated string");
    ++i;
    return out;
  }

  static Json parse_value(const std::string& t, size_t& i) {
    skip_ws(t, i);
    if (i >= t.size()) throw std::runtime_error("json: unexpected end");
    char c = t[i];
    if (c == '{') {
      ++i;
      Json o = object();
      skip_ws(t, i);
      if (i < t.size() && t[i] == '}') { ++i; return o; }
      while (true) {
        skip_ws(t, i);
        std::string k = parse_string(t, i);
        skip_ws(t, i);
        if (i >= t.size() || t[i] != ':') throw std::runtime_error("json: expected ':'");
        ++i;
        o.set(k, parse_value(t, i));
        skip_ws(t, i);
        if (i < t.size() && t[i] == ',') { ++i; continue; }
        if (i < t.size() && t[i] == '}') { ++i; return o; }
        throw std::runtime_error("json: expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++i;
      Json a = array();
      skip_ws(t, i);
      if (i < t.size() && t[i] == ']') { ++i; return a; }
      while (true) {
        a.push(parse_value(t, i));
        skip_ws(t, i);
        if (i < t.size() && t[i] == ',') { ++i; continue; }
        if (i < t.size() && t[i] == ']') { ++i; return a; }
        throw std::runtime_error("json: expected ',' or ']'");
      }
    }
    if (c == '"') return Json(parse_string(t, i));
    if (t.compare(i, 4, "true") == 0) { i += 4; return Json(true); }
    if (t.compare(i, 5, "false") == 0) { i += 5; return Json(false); }
    if (t.compare(i, 4, "null") == 0) { i += 4; return Json(); }
    size_t j = i;
    while (j < t.size() && (std::isdigit((unsigned char)t[j]) || t[j] == '-' || t[j] == '+' ||
                            t[j] == '.' || t[j] == 'e' || t[j] == 'E'))
      ++j;
    if (j == i) throw std::runtime_error("json: unexpected character");
    double d = std::stod(t.substr(i, j - i));
    i = j;
    return Json(d);
  }
};

}  // namespace arena
