/*
 * json.hpp -- strict RFC 8259 JSON reader/writer for the control socket.
 *
 * The reference decodes control datagrams with serde_json
 * (/root/reference/src/main.rs:1008-1009 `serde_json::from_str`) and encodes
 * the QueryUsedPorts answer with `serde_json::to_string` (:572).  This reader
 * accepts exactly JSON text (no comments, no trailing commas, no leading
 * zeros, no raw control characters in strings, nothing after the value but
 * whitespace), keeps object members in order (serde rejects duplicate struct
 * fields, so duplicates must stay visible) and keeps integer literals exact.
 */
#ifndef USND_JSON_HPP
#define USND_JSON_HPP

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace usnd {

struct Json {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  /* Number: the literal, and whether it is a non-negative integer without
   * fraction/exponent that fits u64 (what serde's unsigned visitors accept) */
  std::string num;
  bool is_uint = false;
  uint64_t u = 0;
  std::string s;                                     // String
  std::vector<Json> a;                               // Array
  std::vector<std::pair<std::string, Json>> o;       // Object, in order

  const Json *get(const std::string &key) const {    // first member named key
    for (const auto &kv : o)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
};

class JsonReader {
 public:
  explicit JsonReader(const std::string &text) : t_(text) {}
  /* false on any syntax error or trailing garbage */
  bool parse(Json &out) {
    pos_ = 0;
    depth_ = 0;
    ws();
    if (!value(out)) return false;
    ws();
    return pos_ == t_.size();
  }

 private:
  const std::string &t_;
  size_t pos_ = 0;
  int depth_ = 0;

  bool eof() const { return pos_ >= t_.size(); }
  char peek() const { return eof() ? '\0' : t_[pos_]; }
  void ws() {
    while (!eof() && (t_[pos_] == ' ' || t_[pos_] == '\t' || t_[pos_] == '\n' || t_[pos_] == '\r'))
      ++pos_;
  }
  bool lit(const char *w) {
    size_t n = 0;
    while (w[n]) ++n;
    if (t_.compare(pos_, n, w) != 0) return false;
    pos_ += n;
    return true;
  }
  bool value(Json &v) {
    if (++depth_ > 128) return false;   // serde_json's recursion limit
    bool ok = false;
    switch (peek()) {
      case 'n': ok = lit("null"); v.kind = Json::Null; break;
      case 't': ok = lit("true"); v.kind = Json::Bool; v.b = true; break;
      case 'f': ok = lit("false"); v.kind = Json::Bool; v.b = false; break;
      case '"': v.kind = Json::String; ok = str(v.s); break;
      case '[': ok = arr(v); break;
      case '{': ok = obj(v); break;
      default: ok = number(v); break;
    }
    --depth_;
    return ok;
  }
  static void utf8(std::string &out, uint32_t cp) {
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
  bool hex4(uint32_t &v) {
    if (pos_ + 4 > t_.size()) return false;
    v = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = t_[pos_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    return true;
  }
  bool str(std::string &out) {
    ++pos_;   // opening quote
    out.clear();
    while (!eof()) {
      const unsigned char c = (unsigned char)t_[pos_++];
      if (c == '"') return true;
      if (c < 0x20) return false;
      if (c != '\\') { out += (char)c; continue; }
      if (eof()) return false;
      const char e = t_[pos_++];
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
          uint32_t cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {            // high surrogate: needs a low one
            uint32_t lo;
            if (!(lit("\\u") && hex4(lo) && lo >= 0xDC00 && lo < 0xE000)) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp < 0xE000) {
            return false;                                 // lone low surrogate
          }
          utf8(out, cp);
          break;
        }
        default: return false;
      }
    }
    return false;
  }
  bool number(Json &v) {
    const size_t start = pos_;
    bool neg = false, frac = false;
    if (peek() == '-') { neg = true; ++pos_; }
    if (peek() == '0') {
      ++pos_;
    } else if (peek() >= '1' && peek() <= '9') {
      while (peek() >= '0' && peek() <= '9') ++pos_;
    } else {
      return false;
    }
    if (peek() == '.') {
      frac = true;
      ++pos_;
      if (!(peek() >= '0' && peek() <= '9')) return false;
      while (peek() >= '0' && peek() <= '9') ++pos_;
    }
    if (peek() == 'e' || peek() == 'E') {
      frac = true;
      ++pos_;
      if (peek() == '+' || peek() == '-') ++pos_;
      if (!(peek() >= '0' && peek() <= '9')) return false;
      while (peek() >= '0' && peek() <= '9') ++pos_;
    }
    v.kind = Json::Number;
    v.num = t_.substr(start, pos_ - start);
    v.is_uint = false;
    if (!neg && !frac) {
      uint64_t u = 0;
      bool fits = true;
      for (char c : v.num) {
        const uint64_t d = (uint64_t)(c - '0');
        if (u > (UINT64_MAX - d) / 10) { fits = false; break; }
        u = u * 10 + d;
      }
      v.is_uint = fits;
      v.u = u;
    }
    return true;
  }
  bool arr(Json &v) {
    v.kind = Json::Array;
    ++pos_;
    ws();
    if (peek() == ']') { ++pos_; return true; }
    for (;;) {
      v.a.emplace_back();
      ws();
      if (!value(v.a.back())) return false;
      ws();
      if (peek() == ',') { ++pos_; continue; }
      if (peek() == ']') { ++pos_; return true; }
      return false;
    }
  }
  bool obj(Json &v) {
    v.kind = Json::Object;
    ++pos_;
    ws();
    if (peek() == '}') { ++pos_; return true; }
    for (;;) {
      ws();
      if (peek() != '"') return false;
      std::string key;
      if (!str(key)) return false;
      ws();
      if (peek() != ':') return false;
      ++pos_;
      ws();
      v.o.emplace_back(std::move(key), Json());
      if (!value(v.o.back().second)) return false;
      ws();
      if (peek() == ',') { ++pos_; continue; }
      if (peek() == '}') { ++pos_; return true; }
      return false;
    }
  }
};

/* serde_json::to_string string escaping */
inline void json_quote(std::string &out, const std::string &s) {
  static const char *hex = "0123456789abcdef";
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
          out += "\\u00";
          out += hex[c >> 4];
          out += hex[c & 15];
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

}  // namespace usnd

#endif
