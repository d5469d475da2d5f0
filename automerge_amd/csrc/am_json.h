// am_json.h -- JSON reader for the request objects that cross the C ABI as text (host code).
//
// The frontend's change requests (applyLocalChange / encodeChange, columnar.js:710-739) and sync
// message objects (encodeSyncMessage, sync.js:153-170) are JS objects. The Node and Python hosts
// hand them over as JSON with two conventions for what JSON cannot carry:
//   {"__bytes": "<hex>"}          a Uint8Array (or any ArrayBuffer view: its whole buffer)
//   {"__f64": "NaN"|"Infinity"|"-Infinity"}   a non-finite number
// Absent keys are JS `undefined`. Object key order is kept (error messages print objects).
// The reference's type rules (Number.isInteger, truthiness, template-string conversion) are
// restated here so the encoders can raise the reference's errors.
#pragma once
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace amjson {

enum Kind { UNDEF, NUL, BOOL, NUM, STR, ARR, OBJ, BYTES };

struct JV {
  Kind k = UNDEF;
  bool b = false;
  double n = 0;
  std::string s;  // STR: UTF-8 text; BYTES: raw bytes
  std::vector<JV> a;
  std::vector<std::pair<std::string, JV>> o;

  const JV* get(const char* key) const {
    if (k != OBJ) return nullptr;
    for (auto& kv : o)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
  // property access as in JS: a missing key reads `undefined`
  const JV& operator[](const char* key) const {
    static const JV undef;
    const JV* v = get(key);
    return v ? *v : undef;
  }
  bool truthy() const {
    switch (k) {
      case UNDEF: case NUL: return false;
      case BOOL: return b;
      case NUM: return n != 0 && !std::isnan(n);
      case STR: return !s.empty();
      default: return true;
    }
  }
  bool is_int() const { return k == NUM && std::isfinite(n) && std::floor(n) == n; }  // Number.isInteger
};

// JS Number.prototype.toString() (ECMA-262 Number::toString, radix 10)
inline std::string js_num(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
  if (v == 0) return "0";
  std::string sign = v < 0 ? "-" : "";
  const double av = std::fabs(v);
  char buf[64];
  int p = 1;
  for (; p <= 17; p++) {
    std::snprintf(buf, sizeof buf, "%.*e", p - 1, av);
    if (std::strtod(buf, nullptr) == av) break;
  }
  // buf = d[.ddd]e±XX
  std::string digits;
  const char* q = buf;
  for (; *q && *q != 'e'; q++)
    if (*q >= '0' && *q <= '9') digits += *q;
  const int e10 = std::atoi(q + 1);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int k = (int)digits.size(), n = e10 + 1;
  std::string r;
  if (k <= n && n <= 21) {
    r = digits + std::string(n - k, '0');
  } else if (0 < n && n <= 21) {
    r = digits.substr(0, n) + "." + digits.substr(n);
  } else if (-6 < n && n <= 0) {
    r = "0." + std::string(-n, '0') + digits;
  } else {
    r = digits.substr(0, 1);
    if (k > 1) r += "." + digits.substr(1);
    r += "e";
    r += (n - 1 >= 0) ? "+" : "-";
    r += std::to_string(std::abs(n - 1));
  }
  return sign + r;
}

// String(v) / `${v}`
inline std::string js_str(const JV& v) {
  switch (v.k) {
    case UNDEF: return "undefined";
    case NUL: return "null";
    case BOOL: return v.b ? "true" : "false";
    case NUM: return js_num(v.n);
    case STR: return v.s;
    case ARR: {
      std::string r;
      for (size_t i = 0; i < v.a.size(); i++) {
        if (i) r += ",";
        if (v.a[i].k != UNDEF && v.a[i].k != NUL) r += js_str(v.a[i]);
      }
      return r;
    }
    case BYTES: {  // Uint8Array.prototype.toString
      std::string r;
      for (size_t i = 0; i < v.s.size(); i++) {
        if (i) r += ",";
        r += std::to_string((uint8_t)v.s[i]);
      }
      return r;
    }
    default: return "[object Object]";
  }
}

// JSON.stringify (for the values error messages print)
inline void js_quote(const std::string& s, std::string& r) {
  r += '"';
  for (unsigned char c : s) {
    if (c == '"') r += "\\\"";
    else if (c == '\\') r += "\\\\";
    else if (c == '\n') r += "\\n";
    else if (c == '\r') r += "\\r";
    else if (c == '\t') r += "\\t";
    else if (c == '\b') r += "\\b";
    else if (c == '\f') r += "\\f";
    else if (c < 0x20) { char b[8]; std::snprintf(b, sizeof b, "\\u%04x", c); r += b; }
    else r += (char)c;
  }
  r += '"';
}
inline void js_stringify(const JV& v, std::string& r) {
  switch (v.k) {
    case UNDEF: case NUL: r += "null"; return;
    case BOOL: r += v.b ? "true" : "false"; return;
    case NUM: r += std::isfinite(v.n) ? js_num(v.n) : "null"; return;
    case STR: js_quote(v.s, r); return;
    case ARR:
      r += '[';
      for (size_t i = 0; i < v.a.size(); i++) { if (i) r += ','; js_stringify(v.a[i], r); }
      r += ']';
      return;
    case BYTES: {  // a Uint8Array stringifies as {"0":b0,"1":b1,...}
      r += '{';
      for (size_t i = 0; i < v.s.size(); i++) {
        if (i) r += ',';
        r += "\"" + std::to_string(i) + "\":" + std::to_string((uint8_t)v.s[i]);
      }
      r += '}';
      return;
    }
    case OBJ: {
      r += '{';
      bool first = true;
      for (auto& kv : v.o) {
        if (kv.second.k == UNDEF) continue;
        if (!first) r += ',';
        first = false;
        js_quote(kv.first, r);
        r += ':';
        js_stringify(kv.second, r);
      }
      r += '}';
      return;
    }
  }
}
inline std::string js_stringify(const JV& v) {
  std::string r;
  js_stringify(v, r);
  return r;
}

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), n_(n) {}
  bool parse(JV& out) {
    ws();
    if (!value(out, 0)) return false;
    ws();
    return i_ == n_;
  }

 private:
  const char* p_;
  size_t n_, i_ = 0;
  void ws() { while (i_ < n_ && (p_[i_] == ' ' || p_[i_] == '\t' || p_[i_] == '\n' || p_[i_] == '\r')) i_++; }
  bool lit(const char* w) {
    const size_t l = std::strlen(w);
    if (n_ - i_ < l || std::memcmp(p_ + i_, w, l)) return false;
    i_ += l;
    return true;
  }
  static void utf8(uint32_t cp, std::string& s) {
    if (cp < 0x80) s += (char)cp;
    else if (cp < 0x800) { s += (char)(0xc0 | cp >> 6); s += (char)(0x80 | (cp & 0x3f)); }
    else if (cp < 0x10000) { s += (char)(0xe0 | cp >> 12); s += (char)(0x80 | (cp >> 6 & 0x3f)); s += (char)(0x80 | (cp & 0x3f)); }
    else { s += (char)(0xf0 | cp >> 18); s += (char)(0x80 | (cp >> 12 & 0x3f)); s += (char)(0x80 | (cp >> 6 & 0x3f)); s += (char)(0x80 | (cp & 0x3f)); }
  }
  bool hex4(uint32_t& v) {
    if (n_ - i_ < 4) return false;
    v = 0;
    for (int k = 0; k < 4; k++) {
      const char c = p_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else return false;
    }
    return true;
  }
  // strings become UTF-8 as TextEncoder writes them: a lone surrogate is U+FFFD
  bool str(std::string& s) {
    if (i_ >= n_ || p_[i_] != '"') return false;
    i_++;
    while (i_ < n_) {
      const char c = p_[i_++];
      if (c == '"') return true;
      if (c != '\\') { s += c; continue; }
      if (i_ >= n_) return false;
      const char e = p_[i_++];
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
          uint32_t u;
          if (!hex4(u)) return false;
          if (u >= 0xd800 && u < 0xdc00) {
            uint32_t lo;
            const size_t save = i_;
            if (n_ - i_ >= 6 && p_[i_] == '\\' && p_[i_ + 1] == 'u' && (i_ += 2, hex4(lo)) && lo >= 0xdc00 && lo < 0xe000) {
              utf8(0x10000 + ((u - 0xd800) << 10) + (lo - 0xdc00), s);
            } else {
              i_ = save;
              utf8(0xfffd, s);
            }
          } else if (u >= 0xdc00 && u < 0xe000) {
            utf8(0xfffd, s);
          } else {
            utf8(u, s);
          }
          break;
        }
        default: return false;
      }
    }
    return false;
  }
  static bool unhex(const std::string& h, std::string& out) {
    if (h.size() % 2) return false;
    out.clear();
    for (size_t i = 0; i < h.size(); i += 2) {
      int v = 0;
      for (int k = 0; k < 2; k++) {
        const char c = h[i + k];
        v <<= 4;
        if (c >= '0' && c <= '9') v |= c - '0';
        else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
        else return false;
      }
      out += (char)v;
    }
    return true;
  }
  bool value(JV& v, int depth) {
    if (depth > 200 || i_ >= n_) return false;
    const char c = p_[i_];
    if (c == 'n') { v.k = NUL; return lit("null"); }
    if (c == 't') { v.k = BOOL; v.b = true; return lit("true"); }
    if (c == 'f') { v.k = BOOL; v.b = false; return lit("false"); }
    if (c == '"') { v.k = STR; return str(v.s); }
    if (c == '[') {
      i_++;
      v.k = ARR;
      ws();
      if (i_ < n_ && p_[i_] == ']') { i_++; return true; }
      for (;;) {
        JV e;
        ws();
        if (!value(e, depth + 1)) return false;
        v.a.push_back(std::move(e));
        ws();
        if (i_ < n_ && p_[i_] == ',') { i_++; continue; }
        if (i_ < n_ && p_[i_] == ']') { i_++; return true; }
        return false;
      }
    }
    if (c == '{') {
      i_++;
      v.k = OBJ;
      ws();
      if (i_ < n_ && p_[i_] == '}') { i_++; return true; }
      for (;;) {
        std::string key;
        JV e;
        ws();
        if (!str(key)) return false;
        ws();
        if (i_ >= n_ || p_[i_++] != ':') return false;
        ws();
        if (!value(e, depth + 1)) return false;
        bool dup = false;
        for (auto& kv : v.o)
          if (kv.first == key) { kv.second = std::move(e); dup = true; break; }
        if (!dup) v.o.emplace_back(std::move(key), std::move(e));
        ws();
        if (i_ < n_ && p_[i_] == ',') { i_++; continue; }
        if (i_ < n_ && p_[i_] == '}') { i_++; break; }
        return false;
      }
      // the two transport conventions
      if (v.o.size() == 1 && v.o[0].first == "__bytes" && v.o[0].second.k == STR) {
        std::string raw;
        if (!unhex(v.o[0].second.s, raw)) return false;
        v.k = BYTES;
        v.s = std::move(raw);
        v.o.clear();
      } else if (v.o.size() == 1 && v.o[0].first == "__f64" && v.o[0].second.k == STR) {
        const std::string t = v.o[0].second.s;
        v.k = NUM;
        v.n = t == "NaN" ? NAN : t == "Infinity" ? INFINITY : t == "-Infinity" ? -INFINITY : 0;
        v.o.clear();
      }
      return true;
    }
    // number
    const size_t b = i_;
    if (p_[i_] == '-') i_++;
    while (i_ < n_ && ((p_[i_] >= '0' && p_[i_] <= '9') || p_[i_] == '.' || p_[i_] == 'e' || p_[i_] == 'E' || p_[i_] == '+' ||
                       p_[i_] == '-'))
      i_++;
    if (i_ == b) return false;
    const std::string t(p_ + b, i_ - b);
    char* end = nullptr;
    v.k = NUM;
    v.n = std::strtod(t.c_str(), &end);
    return end && *end == 0;
  }
};

inline bool parse(const char* p, size_t n, JV& out) { return Parser(p, n).parse(out); }

}  // namespace amjson
