// Dynamic values for the native servers: a JSON parser (server configs), a
// canonical JSON dump (semantic config comparison on load, the reference's
// config check in server_base.cpp load_file), a msgpack decoder (model
// files, RPC arguments) and a msgpack writer (responses, model files).
//
// Strings written into RPC responses use the old msgpack spec (RAW only),
// like the Python transport (common/mprpc.py packb use_bin_type=False) and
// the reference's msgpack 0.5.x clients; model payloads carry bin types.
#pragma once
#include <errno.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace jb {
namespace val {

struct Value {
  enum Kind { NIL, BOOL, INT, UINT, DBL, STR, BIN, ARR, MAP } kind = NIL;
  bool b = false;
  int64_t i = 0;
  uint64_t u = 0;
  double d = 0;
  std::string s;                                  // STR / BIN bytes
  std::vector<Value> a;                           // ARR
  std::vector<std::pair<std::string, Value>> o;   // MAP (keys as byte strings)

  bool is_num() const { return kind == INT || kind == UINT || kind == DBL; }
  double num() const { return kind == INT ? (double)i : kind == UINT ? (double)u : d; }
  bool is_str() const { return kind == STR || kind == BIN; }
  const Value* get(const std::string& k) const {
    if (kind != MAP) return nullptr;
    for (const auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  std::string str_or(const std::string& k, const std::string& dflt) const {
    const Value* v = get(k);
    return v && v->is_str() ? v->s : dflt;
  }
};

// ------------------------------------------------------------------- JSON
class JsonParser {
 public:
  JsonParser(const char* p, size_t n) : p_(p), e_(p + n) {}
  Value parse() {
    Value v = value(0);
    ws();
    if (p_ != e_) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const char* what) { throw std::runtime_error(std::string("JSON: ") + what); }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if ((size_t)(e_ - p_) >= n && memcmp(p_, w, n) == 0) { p_ += n; return true; }
    return false;
  }
  static void utf8(std::string& out, uint32_t c) {
    if (c < 0x80) { out.push_back((char)c); }
    else if (c < 0x800) { out.push_back((char)(0xc0 | (c >> 6))); out.push_back((char)(0x80 | (c & 0x3f))); }
    else if (c < 0x10000) {
      out.push_back((char)(0xe0 | (c >> 12)));
      out.push_back((char)(0x80 | ((c >> 6) & 0x3f)));
      out.push_back((char)(0x80 | (c & 0x3f)));
    } else {
      out.push_back((char)(0xf0 | (c >> 18)));
      out.push_back((char)(0x80 | ((c >> 12) & 0x3f)));
      out.push_back((char)(0x80 | ((c >> 6) & 0x3f)));
      out.push_back((char)(0x80 | (c & 0x3f)));
    }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) fail("bad \\u escape");
    uint32_t c = 0;
    for (int k = 0; k < 4; ++k) {
      char h = *p_++;
      c <<= 4;
      if (h >= '0' && h <= '9') c |= (uint32_t)(h - '0');
      else if (h >= 'a' && h <= 'f') c |= (uint32_t)(h - 'a' + 10);
      else if (h >= 'A' && h <= 'F') c |= (uint32_t)(h - 'A' + 10);
      else fail("bad \\u escape");
    }
    return c;
  }
  std::string string() {
    ++p_;  // opening quote
    std::string out;
    while (true) {
      if (p_ >= e_) fail("unterminated string");
      char c = *p_++;
      if (c == '"') return out;
      if (c != '\\') { out.push_back(c); continue; }
      if (p_ >= e_) fail("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xd800 && cp < 0xdc00 && lit("\\u")) {
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xd800) << 10) + (lo - 0xdc00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
  }
  Value value(int depth) {
    if (depth > 128) fail("nesting too deep");
    ws();
    if (p_ >= e_) fail("unexpected end");
    Value v;
    char c = *p_;
    if (c == '{') {
      ++p_;
      v.kind = Value::MAP;
      ws();
      if (p_ < e_ && *p_ == '}') { ++p_; return v; }
      while (true) {
        ws();
        if (p_ >= e_ || *p_ != '"') fail("expected key");
        std::string k = string();
        ws();
        if (p_ >= e_ || *p_ != ':') fail("expected ':'");
        ++p_;
        Value x = value(depth + 1);
        bool dup = false;
        for (auto& kv : v.o)   // last duplicate wins, like Python's json
          if (kv.first == k) { kv.second = std::move(x); dup = true; break; }
        if (!dup) v.o.emplace_back(std::move(k), std::move(x));
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; return v; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p_;
      v.kind = Value::ARR;
      ws();
      if (p_ < e_ && *p_ == ']') { ++p_; return v; }
      while (true) {
        v.a.push_back(value(depth + 1));
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; return v; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') { v.kind = Value::STR; v.s = string(); return v; }
    if (lit("true")) { v.kind = Value::BOOL; v.b = true; return v; }
    if (lit("false")) { v.kind = Value::BOOL; v.b = false; return v; }
    if (lit("null")) return v;
    const char* s = p_;
    bool flt = false;
    if (p_ < e_ && *p_ == '-') ++p_;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                       *p_ == '+' || *p_ == '-')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') flt = true;
      ++p_;
    }
    if (p_ == s) fail("unexpected character");
    std::string num(s, p_);
    char* end = nullptr;
    if (!flt) {
      errno = 0;
      long long x = strtoll(num.c_str(), &end, 10);
      if (*end == 0 && errno == 0) { v.kind = Value::INT; v.i = x; return v; }
    }
    double d = strtod(num.c_str(), &end);
    if (*end != 0) fail("bad number");
    v.kind = Value::DBL;
    v.d = d;
    return v;
  }
  const char* p_;
  const char* e_;
};

inline Value parse_json(const std::string& text) { return JsonParser(text.data(), text.size()).parse(); }

inline void dump_json_str(std::string& out, const std::string& s) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); out += b; }
        else out.push_back((char)c);
    }
  }
  out.push_back('"');
}

// canonical form: sorted keys, no spaces (two configs are the same
// configuration iff their canonical forms are equal)
inline void dump_canonical(std::string& out, const Value& v) {
  switch (v.kind) {
    case Value::NIL: out += "null"; return;
    case Value::BOOL: out += v.b ? "true" : "false"; return;
    case Value::INT: out += std::to_string(v.i); return;
    case Value::UINT: out += std::to_string(v.u); return;
    case Value::DBL: { char b[32]; snprintf(b, sizeof b, "%.17g", v.d); out += b; out += "f"; return; }
    case Value::STR: case Value::BIN: dump_json_str(out, v.s); return;
    case Value::ARR:
      out.push_back('[');
      for (size_t k = 0; k < v.a.size(); ++k) { if (k) out.push_back(','); dump_canonical(out, v.a[k]); }
      out.push_back(']');
      return;
    case Value::MAP: {
      std::vector<const std::pair<std::string, Value>*> kv;
      for (const auto& x : v.o) kv.push_back(&x);
      std::sort(kv.begin(), kv.end(), [](auto* a, auto* b) { return a->first < b->first; });
      out.push_back('{');
      for (size_t k = 0; k < kv.size(); ++k) {
        if (k) out.push_back(',');
        dump_json_str(out, kv[k]->first);
        out.push_back(':');
        dump_canonical(out, kv[k]->second);
      }
      out.push_back('}');
      return;
    }
  }
}

inline bool same_config(const std::string& a, const std::string& b) {
  try {
    std::string x, y;
    dump_canonical(x, parse_json(a));
    dump_canonical(y, parse_json(b));
    return x == y;
  } catch (const std::exception&) {
    return a == b;
  }
}

// ---------------------------------------------------------------- msgpack
class MsgpackReader {
 public:
  MsgpackReader(const uint8_t* p, size_t n) : p_(p), e_(p + n) {}
  Value read(int depth = 0) {
    if (depth > 128) fail();
    need(1);
    const uint8_t t = *p_++;
    Value v;
    if (t <= 0x7f) { v.kind = Value::INT; v.i = t; return v; }
    if (t >= 0xe0) { v.kind = Value::INT; v.i = (int8_t)t; return v; }
    if ((t & 0xf0) == 0x80) return map(t & 0x0f, depth);
    if ((t & 0xf0) == 0x90) return arr(t & 0x0f, depth);
    if ((t & 0xe0) == 0xa0) return bytes(t & 0x1f, Value::STR);
    switch (t) {
      case 0xc0: return v;
      case 0xc2: v.kind = Value::BOOL; v.b = false; return v;
      case 0xc3: v.kind = Value::BOOL; v.b = true; return v;
      case 0xc4: return bytes(be(1), Value::BIN);
      case 0xc5: return bytes(be(2), Value::BIN);
      case 0xc6: return bytes(be(4), Value::BIN);
      case 0xca: { uint32_t x = (uint32_t)be(4); float f; memcpy(&f, &x, 4); v.kind = Value::DBL; v.d = f; return v; }
      case 0xcb: { uint64_t x = be(8); double f; memcpy(&f, &x, 8); v.kind = Value::DBL; v.d = f; return v; }
      case 0xcc: v.kind = Value::UINT; v.u = be(1); return norm(v);
      case 0xcd: v.kind = Value::UINT; v.u = be(2); return norm(v);
      case 0xce: v.kind = Value::UINT; v.u = be(4); return norm(v);
      case 0xcf: v.kind = Value::UINT; v.u = be(8); return norm(v);
      case 0xd0: v.kind = Value::INT; v.i = (int8_t)be(1); return v;
      case 0xd1: v.kind = Value::INT; v.i = (int16_t)be(2); return v;
      case 0xd2: v.kind = Value::INT; v.i = (int32_t)be(4); return v;
      case 0xd3: v.kind = Value::INT; v.i = (int64_t)be(8); return v;
      case 0xd9: return bytes(be(1), Value::STR);
      case 0xda: return bytes(be(2), Value::STR);
      case 0xdb: return bytes(be(4), Value::STR);
      case 0xdc: return arr(be(2), depth);
      case 0xdd: return arr(be(4), depth);
      case 0xde: return map(be(2), depth);
      case 0xdf: return map(be(4), depth);
    }
    fail();
  }
  bool done() const { return p_ == e_; }

 private:
  [[noreturn]] static void fail() { throw std::runtime_error("malformed msgpack"); }
  void need(uint64_t n) const { if ((uint64_t)(e_ - p_) < n) fail(); }
  uint64_t be(int n) {
    need((uint64_t)n);
    uint64_t x = 0;
    for (int k = 0; k < n; ++k) x = (x << 8) | *p_++;
    return x;
  }
  static Value norm(Value v) {   // small unsigned values read as INT
    if (v.u <= (uint64_t)INT64_MAX) { v.kind = Value::INT; v.i = (int64_t)v.u; }
    return v;
  }
  Value bytes(uint64_t n, Value::Kind k) {
    need(n);
    Value v;
    v.kind = k;
    v.s.assign((const char*)p_, (size_t)n);
    p_ += n;
    return v;
  }
  Value arr(uint64_t n, int depth) {
    Value v;
    v.kind = Value::ARR;
    if (n > (uint64_t)(e_ - p_)) fail();
    v.a.reserve((size_t)n);
    for (uint64_t k = 0; k < n; ++k) v.a.push_back(read(depth + 1));
    return v;
  }
  Value map(uint64_t n, int depth) {
    Value v;
    v.kind = Value::MAP;
    if (n > (uint64_t)(e_ - p_)) fail();
    for (uint64_t k = 0; k < n; ++k) {
      Value key = read(depth + 1);
      std::string ks = key.is_str() ? key.s : key.kind == Value::INT ? std::to_string(key.i) : "";
      v.o.emplace_back(std::move(ks), read(depth + 1));
    }
    return v;
  }
  const uint8_t* p_;
  const uint8_t* e_;
};

class MsgpackWriter {
 public:
  std::string out;
  void byte(uint8_t b) { out.push_back((char)b); }
  void be(uint64_t x, int n) { for (int k = n - 1; k >= 0; --k) byte((uint8_t)(x >> (8 * k))); }
  void nil() { byte(0xc0); }
  void boolean(bool b) { byte(b ? 0xc3 : 0xc2); }
  void uint(uint64_t x) {
    if (x < 128) byte((uint8_t)x);
    else if (x < 256) { byte(0xcc); be(x, 1); }
    else if (x < 65536) { byte(0xcd); be(x, 2); }
    else if (x < (1ull << 32)) { byte(0xce); be(x, 4); }
    else { byte(0xcf); be(x, 8); }
  }
  void sint(int64_t x) {
    if (x >= 0) { uint((uint64_t)x); return; }
    if (x >= -32) byte((uint8_t)(int8_t)x);
    else if (x >= -128) { byte(0xd0); be((uint64_t)x, 1); }
    else if (x >= -32768) { byte(0xd1); be((uint64_t)x, 2); }
    else if (x >= INT32_MIN) { byte(0xd2); be((uint64_t)x, 4); }
    else { byte(0xd3); be((uint64_t)x, 8); }
  }
  void dbl(double d) { uint64_t x; memcpy(&x, &d, 8); byte(0xcb); be(x, 8); }
  // old-spec raw (fixraw / raw16 / raw32): what the Python transport sends
  void raw(const char* s, size_t n) {
    if (n < 32) byte((uint8_t)(0xa0 | n));
    else if (n < 65536) { byte(0xda); be(n, 2); }
    else { byte(0xdb); be(n, 4); }
    out.append(s, n);
  }
  void raw(const std::string& s) { raw(s.data(), s.size()); }
  // new-spec str / bin (model payloads, msgpack-python use_bin_type=True)
  void str(const std::string& s) {
    const size_t n = s.size();
    if (n < 32) byte((uint8_t)(0xa0 | n));
    else if (n < 256) { byte(0xd9); be(n, 1); }
    else if (n < 65536) { byte(0xda); be(n, 2); }
    else { byte(0xdb); be(n, 4); }
    out += s;
  }
  void bin(const void* p, size_t n) {
    if (n < 256) { byte(0xc4); be(n, 1); }
    else if (n < 65536) { byte(0xc5); be(n, 2); }
    else { byte(0xc6); be(n, 4); }
    out.append((const char*)p, n);
  }
  void arr(size_t n) {
    if (n < 16) byte((uint8_t)(0x90 | n));
    else if (n < 65536) { byte(0xdc); be(n, 2); }
    else { byte(0xdd); be(n, 4); }
  }
  void map(size_t n) {
    if (n < 16) byte((uint8_t)(0x80 | n));
    else if (n < 65536) { byte(0xde); be(n, 2); }
    else { byte(0xdf); be(n, 4); }
  }
};

// [1, msgid, error, result] with error nil and the result already encoded
inline std::string response_ok(uint32_t msgid, const std::string& result) {
  MsgpackWriter w;
  w.arr(4);
  w.uint(1);
  w.uint(msgid);
  w.nil();
  w.out += result;
  return std::move(w.out);
}

// error: an integer code (1 no method, 2 argument error) or a message
inline std::string response_code(uint32_t msgid, int code) {
  MsgpackWriter w;
  w.arr(4);
  w.uint(1);
  w.uint(msgid);
  w.uint((uint64_t)code);
  w.nil();
  return std::move(w.out);
}

inline std::string response_msg(uint32_t msgid, const std::string& msg) {
  MsgpackWriter w;
  w.arr(4);
  w.uint(1);
  w.uint(msgid);
  w.raw(msg);
  w.nil();
  return std::move(w.out);
}

}  // namespace val
}  // namespace jb
