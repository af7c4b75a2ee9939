// Header-only msgpack-RPC client for Jubatus servers (C++17, no dependencies).
//
// Reference: the C++ client library jubatus/client/common/{client,datum}.hpp
// (client::common::client get_config / save / load / get_status / do_mix /
// get_proxy_status, name handling) over jubatus-msgpack-rpc. This library
// carries its own msgpack codec: strings are written as old-spec RAW (the
// wire format every Jubatus server and proxy speaks), str8 / bin are
// accepted on read. Per-engine clients are generated from the IDL by
// `python -m jubatus_amd.idl.jenerator -l cpp`.
#ifndef JUBATUS_AMD_MSGPACK_RPC_HPP_
#define JUBATUS_AMD_MSGPACK_RPC_HPP_

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace jubatus_amd {
namespace mp {

// ------------------------------------------------------------------ value
struct Value {
  enum Type { NIL, BOOL, INT, UINT, FLOAT, STR, ARRAY, MAP };
  Type type = NIL;
  bool b = false;
  int64_t i = 0;
  uint64_t u = 0;
  double f = 0.0;
  std::string s;
  std::vector<Value> a;
  std::vector<std::pair<Value, Value>> m;

  Value() = default;
  static Value nil() { return Value(); }
  static Value boolean(bool v) { Value x; x.type = BOOL; x.b = v; return x; }
  static Value integer(int64_t v) {
    Value x;
    if (v >= 0) { x.type = UINT; x.u = (uint64_t)v; } else { x.type = INT; x.i = v; }
    return x;
  }
  static Value uinteger(uint64_t v) { Value x; x.type = UINT; x.u = v; return x; }
  static Value real(double v) { Value x; x.type = FLOAT; x.f = v; return x; }
  static Value str(std::string v) { Value x; x.type = STR; x.s = std::move(v); return x; }
  static Value array(std::vector<Value> v = {}) { Value x; x.type = ARRAY; x.a = std::move(v); return x; }
  static Value map(std::vector<std::pair<Value, Value>> v = {}) {
    Value x; x.type = MAP; x.m = std::move(v); return x;
  }

  int64_t as_int() const {
    if (type == INT) return i;
    if (type == UINT) return (int64_t)u;
    if (type == FLOAT) return (int64_t)f;
    throw std::runtime_error("msgpack: not an integer");
  }
  uint64_t as_uint() const { return (uint64_t)as_int(); }
  double as_double() const {
    if (type == FLOAT) return f;
    if (type == INT) return (double)i;
    if (type == UINT) return (double)u;
    throw std::runtime_error("msgpack: not a number");
  }
  bool as_bool() const {
    if (type != BOOL) throw std::runtime_error("msgpack: not a bool");
    return b;
  }
  const std::string& as_str() const {
    if (type != STR) throw std::runtime_error("msgpack: not a string");
    return s;
  }
  const std::vector<Value>& as_array() const {
    if (type != ARRAY) throw std::runtime_error("msgpack: not an array");
    return a;
  }
  const std::vector<std::pair<Value, Value>>& as_map() const {
    if (type != MAP) throw std::runtime_error("msgpack: not a map");
    return m;
  }
};

// ---------------------------------------------------------------- encoder
inline void put_be(std::string& o, uint64_t v, int n) {
  for (int k = n - 1; k >= 0; --k) o.push_back((char)((v >> (8 * k)) & 0xff));
}

inline void encode(const Value& v, std::string& o) {
  switch (v.type) {
    case Value::NIL: o.push_back((char)0xc0); break;
    case Value::BOOL: o.push_back((char)(v.b ? 0xc3 : 0xc2)); break;
    case Value::UINT:
      if (v.u < 128) o.push_back((char)v.u);
      else if (v.u <= 0xff) { o.push_back((char)0xcc); put_be(o, v.u, 1); }
      else if (v.u <= 0xffff) { o.push_back((char)0xcd); put_be(o, v.u, 2); }
      else if (v.u <= 0xffffffffULL) { o.push_back((char)0xce); put_be(o, v.u, 4); }
      else { o.push_back((char)0xcf); put_be(o, v.u, 8); }
      break;
    case Value::INT:
      if (v.i >= -32) o.push_back((char)(int8_t)v.i);
      else if (v.i >= -128) { o.push_back((char)0xd0); put_be(o, (uint64_t)v.i, 1); }
      else if (v.i >= -32768) { o.push_back((char)0xd1); put_be(o, (uint64_t)v.i, 2); }
      else if (v.i >= INT32_MIN) { o.push_back((char)0xd2); put_be(o, (uint64_t)v.i, 4); }
      else { o.push_back((char)0xd3); put_be(o, (uint64_t)v.i, 8); }
      break;
    case Value::FLOAT: {
      uint64_t bits;
      std::memcpy(&bits, &v.f, 8);
      o.push_back((char)0xcb);
      put_be(o, bits, 8);
      break;
    }
    case Value::STR: {  // old-spec RAW
      const size_t n = v.s.size();
      if (n < 32) o.push_back((char)(0xa0 | n));
      else if (n <= 0xffff) { o.push_back((char)0xda); put_be(o, n, 2); }
      else { o.push_back((char)0xdb); put_be(o, n, 4); }
      o += v.s;
      break;
    }
    case Value::ARRAY: {
      const size_t n = v.a.size();
      if (n < 16) o.push_back((char)(0x90 | n));
      else if (n <= 0xffff) { o.push_back((char)0xdc); put_be(o, n, 2); }
      else { o.push_back((char)0xdd); put_be(o, n, 4); }
      for (const auto& x : v.a) encode(x, o);
      break;
    }
    case Value::MAP: {
      const size_t n = v.m.size();
      if (n < 16) o.push_back((char)(0x80 | n));
      else if (n <= 0xffff) { o.push_back((char)0xde); put_be(o, n, 2); }
      else { o.push_back((char)0xdf); put_be(o, n, 4); }
      for (const auto& kv : v.m) { encode(kv.first, o); encode(kv.second, o); }
      break;
    }
  }
}

// ---------------------------------------------------------------- decoder
// returns false when the buffer holds an incomplete object
class Decoder {
 public:
  Decoder(const char* p, size_t n) : p_((const uint8_t*)p), n_(n) {}
  bool next(Value& out) {
    size_t save = pos_;
    if (!value(out, 0)) { pos_ = save; return false; }
    return true;
  }
  size_t consumed() const { return pos_; }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t pos_ = 0;

  bool need(size_t k) const { return pos_ + k <= n_; }
  uint64_t be(int k) {
    uint64_t v = 0;
    for (int j = 0; j < k; ++j) v = (v << 8) | p_[pos_++];
    return v;
  }
  bool raw(size_t len, Value& out) {
    if (!need(len)) return false;
    out.type = Value::STR;
    out.s.assign((const char*)p_ + pos_, len);
    pos_ += len;
    return true;
  }
  bool arr(size_t len, Value& out, int depth) {
    out.type = Value::ARRAY;
    out.a.resize(len);
    for (size_t k = 0; k < len; ++k)
      if (!value(out.a[k], depth + 1)) return false;
    return true;
  }
  bool map(size_t len, Value& out, int depth) {
    out.type = Value::MAP;
    out.m.resize(len);
    for (size_t k = 0; k < len; ++k)
      if (!value(out.m[k].first, depth + 1) || !value(out.m[k].second, depth + 1)) return false;
    return true;
  }
  bool value(Value& out, int depth) {
    if (depth > 64) throw std::runtime_error("msgpack: nesting too deep");
    if (!need(1)) return false;
    const uint8_t c = p_[pos_++];
    out = Value();
    if (c <= 0x7f) { out.type = Value::UINT; out.u = c; return true; }
    if (c >= 0xe0) { out.type = Value::INT; out.i = (int8_t)c; return true; }
    if ((c & 0xe0) == 0xa0) return raw(c & 0x1f, out);
    if ((c & 0xf0) == 0x90) return arr(c & 0x0f, out, depth);
    if ((c & 0xf0) == 0x80) return map(c & 0x0f, out, depth);
    switch (c) {
      case 0xc0: return true;
      case 0xc2: out.type = Value::BOOL; out.b = false; return true;
      case 0xc3: out.type = Value::BOOL; out.b = true; return true;
      case 0xcc: if (!need(1)) return false; out.type = Value::UINT; out.u = be(1); return true;
      case 0xcd: if (!need(2)) return false; out.type = Value::UINT; out.u = be(2); return true;
      case 0xce: if (!need(4)) return false; out.type = Value::UINT; out.u = be(4); return true;
      case 0xcf: if (!need(8)) return false; out.type = Value::UINT; out.u = be(8); return true;
      case 0xd0: if (!need(1)) return false; out.type = Value::INT; out.i = (int8_t)be(1); return true;
      case 0xd1: if (!need(2)) return false; out.type = Value::INT; out.i = (int16_t)be(2); return true;
      case 0xd2: if (!need(4)) return false; out.type = Value::INT; out.i = (int32_t)be(4); return true;
      case 0xd3: if (!need(8)) return false; out.type = Value::INT; out.i = (int64_t)be(8); return true;
      case 0xca: {
        if (!need(4)) return false;
        uint32_t bits = (uint32_t)be(4);
        float f;
        std::memcpy(&f, &bits, 4);
        out.type = Value::FLOAT;
        out.f = f;
        return true;
      }
      case 0xcb: {
        if (!need(8)) return false;
        uint64_t bits = be(8);
        std::memcpy(&out.f, &bits, 8);
        out.type = Value::FLOAT;
        return true;
      }
      case 0xd9: case 0xc4: if (!need(1)) return false; return raw(be(1), out);
      case 0xda: case 0xc5: if (!need(2)) return false; return raw(be(2), out);
      case 0xdb: case 0xc6: if (!need(4)) return false; return raw(be(4), out);
      case 0xdc: if (!need(2)) return false; return arr(be(2), out, depth);
      case 0xdd: if (!need(4)) return false; return arr(be(4), out, depth);
      case 0xde: if (!need(2)) return false; return map(be(2), out, depth);
      case 0xdf: if (!need(4)) return false; return map(be(4), out, depth);
      default: throw std::runtime_error("msgpack: unsupported type byte");
    }
  }
};

// --------------------------------------------------- C++ <-> Value mapping
inline Value to_value(const std::string& v) { return Value::str(v); }
inline Value to_value(const char* v) { return Value::str(v); }
inline Value to_value(bool v) { return Value::boolean(v); }
inline Value to_value(int32_t v) { return Value::integer(v); }
inline Value to_value(int64_t v) { return Value::integer(v); }
inline Value to_value(uint32_t v) { return Value::uinteger(v); }
inline Value to_value(uint64_t v) { return Value::uinteger(v); }
inline Value to_value(float v) { return Value::real(v); }
inline Value to_value(double v) { return Value::real(v); }
template <typename T> Value to_value(const std::vector<T>& v);
template <typename K, typename V> Value to_value(const std::map<K, V>& v);
template <typename A, typename B> Value to_value(const std::pair<A, B>& v);
template <typename T> auto to_value(const T& v) -> decltype(v.to_value()) { return v.to_value(); }
template <typename T> Value to_value(const std::vector<T>& v) {
  Value a = Value::array();
  for (const auto& x : v) a.a.push_back(to_value(x));
  return a;
}
template <typename K, typename V> Value to_value(const std::map<K, V>& v) {
  Value m = Value::map();
  for (const auto& kv : v) m.m.emplace_back(to_value(kv.first), to_value(kv.second));
  return m;
}
template <typename A, typename B> Value to_value(const std::pair<A, B>& v) {
  return Value::array({to_value(v.first), to_value(v.second)});
}

inline void from_value(const Value& v, std::string& o) { o = v.as_str(); }
inline void from_value(const Value& v, bool& o) { o = v.as_bool(); }
inline void from_value(const Value& v, int32_t& o) { o = (int32_t)v.as_int(); }
inline void from_value(const Value& v, int64_t& o) { o = v.as_int(); }
inline void from_value(const Value& v, uint32_t& o) { o = (uint32_t)v.as_uint(); }
inline void from_value(const Value& v, uint64_t& o) { o = v.as_uint(); }
inline void from_value(const Value& v, float& o) { o = (float)v.as_double(); }
inline void from_value(const Value& v, double& o) { o = v.as_double(); }
template <typename T> auto from_value(const Value& v, T& o) -> decltype(o.from_value(v)) {
  return o.from_value(v);
}
template <typename T> void from_value(const Value& v, std::vector<T>& o) {
  o.clear();
  for (const auto& x : v.as_array()) { T t; from_value(x, t); o.push_back(std::move(t)); }
}
template <typename K, typename V> void from_value(const Value& v, std::map<K, V>& o) {
  o.clear();
  for (const auto& kv : v.as_map()) {
    K k; V x;
    from_value(kv.first, k);
    from_value(kv.second, x);
    o.emplace(std::move(k), std::move(x));
  }
}
template <typename A, typename B> void from_value(const Value& v, std::pair<A, B>& o) {
  const auto& a = v.as_array();
  if (a.size() != 2) throw std::runtime_error("msgpack: pair expects 2 elements");
  from_value(a[0], o.first);
  from_value(a[1], o.second);
}

}  // namespace mp

// -------------------------------------------------------------- rpc errors
struct rpc_error : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct rpc_no_method : rpc_error {
  explicit rpc_no_method(const std::string& m) : rpc_error("no such method: " + m) {}
};
struct rpc_type_error : rpc_error {
  explicit rpc_type_error(const std::string& m) : rpc_error("argument error: " + m) {}
};
struct rpc_call_error : rpc_error {
  using rpc_error::rpc_error;
};
struct rpc_io_error : rpc_error {
  using rpc_error::rpc_error;
};
struct rpc_timeout_error : rpc_error {
  using rpc_error::rpc_error;
};

// ------------------------------------------------------------- rpc client
class RpcClient {
 public:
  RpcClient(const std::string& host, int port, double timeout_sec)
      : host_(host), port_(port), timeout_ms_((int)(timeout_sec * 1000)) {}
  ~RpcClient() { close(); }
  RpcClient(const RpcClient&) = delete;
  RpcClient& operator=(const RpcClient&) = delete;

  void close() {
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    buf_.clear();
  }

  template <typename... Args>
  mp::Value call(const std::string& method, const Args&... args) {
    std::vector<mp::Value> params{mp::to_value(args)...};
    return call_values(method, params);
  }

  mp::Value call_values(const std::string& method, const std::vector<mp::Value>& params) {
    connect_();
    const uint32_t id = ++msgid_;
    std::string out;
    mp::encode(mp::Value::array({mp::Value::uinteger(0), mp::Value::uinteger(id),
                                 mp::Value::str(method), mp::Value::array(params)}), out);
    send_all_(out);
    for (;;) {
      mp::Value resp;
      recv_one_(resp);
      const auto& a = resp.as_array();
      if (a.size() != 4 || a[0].as_int() != 1) throw rpc_io_error("malformed response");
      if (a[1].as_uint() != id) continue;  // stale reply of a timed-out call
      const mp::Value& err = a[2];
      if (err.type != mp::Value::NIL) {
        if (err.type == mp::Value::UINT || err.type == mp::Value::INT) {
          if (err.as_int() == 1) throw rpc_no_method(method);
          if (err.as_int() == 2) throw rpc_type_error(method);
          throw rpc_call_error("rpc error code " + std::to_string(err.as_int()));
        }
        if (err.type == mp::Value::STR) throw rpc_call_error(err.s);
        throw rpc_call_error("rpc error");
      }
      return a[3];
    }
  }

 private:
  std::string host_;
  int port_;
  int timeout_ms_;
  int fd_ = -1;
  uint32_t msgid_ = 0;
  std::string buf_;

  void connect_() {
    if (fd_ >= 0) return;
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host_.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res)
      throw rpc_io_error("cannot resolve " + host_);
    int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
    if (fd < 0) { freeaddrinfo(res); throw rpc_io_error("socket failed"); }
    if (::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
      freeaddrinfo(res);
      ::close(fd);
      throw rpc_io_error("cannot connect to " + host_ + ":" + std::to_string(port_));
    }
    freeaddrinfo(res);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    fd_ = fd;
  }

  void send_all_(const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
      ssize_t k = ::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (k <= 0) {
        if (k < 0 && errno == EINTR) continue;
        close();
        throw rpc_io_error("send failed");
      }
      off += (size_t)k;
    }
  }

  void recv_one_(mp::Value& out) {
    for (;;) {
      if (!buf_.empty()) {
        mp::Decoder d(buf_.data(), buf_.size());
        if (d.next(out)) {
          buf_.erase(0, d.consumed());
          return;
        }
      }
      pollfd p{fd_, POLLIN, 0};
      int r = ::poll(&p, 1, timeout_ms_);
      if (r == 0) { close(); throw rpc_timeout_error("request timed out"); }
      if (r < 0) { if (errno == EINTR) continue; close(); throw rpc_io_error("poll failed"); }
      char tmp[65536];
      ssize_t k = ::recv(fd_, tmp, sizeof(tmp), 0);
      if (k <= 0) {
        if (k < 0 && errno == EINTR) continue;
        close();
        throw rpc_io_error("connection closed");
      }
      buf_.append(tmp, (size_t)k);
    }
  }
};

// ------------------------------------------------------------------ datum
struct datum {
  std::vector<std::pair<std::string, std::string>> string_values;
  std::vector<std::pair<std::string, double>> num_values;
  std::vector<std::pair<std::string, std::string>> binary_values;

  datum& add_string(const std::string& k, const std::string& v) {
    string_values.emplace_back(k, v);
    return *this;
  }
  datum& add_number(const std::string& k, double v) {
    num_values.emplace_back(k, v);
    return *this;
  }
  datum& add_binary(const std::string& k, const std::string& v) {
    binary_values.emplace_back(k, v);
    return *this;
  }
  mp::Value to_value() const {
    return mp::Value::array({mp::to_value(string_values), mp::to_value(num_values),
                             mp::to_value(binary_values)});
  }
  void from_value(const mp::Value& v) {
    const auto& a = v.as_array();
    if (a.size() < 2) throw std::runtime_error("datum: expected [string_values, num_values, ...]");
    mp::from_value(a[0], string_values);
    mp::from_value(a[1], num_values);
    if (a.size() > 2) mp::from_value(a[2], binary_values);
  }
};

// ---------------------------------------------------- common client base
class client {
 public:
  client(const std::string& host, int port, const std::string& name, double timeout_sec)
      : c_(host, port, timeout_sec), name_(name) {}
  virtual ~client() = default;

  std::string get_config() { return get<std::string>("get_config"); }
  std::map<std::string, std::string> save(const std::string& id) {
    return get<std::map<std::string, std::string>>("save", id);
  }
  bool load(const std::string& id) { return get<bool>("load", id); }
  std::map<std::string, std::map<std::string, std::string>> get_status() {
    return get<std::map<std::string, std::map<std::string, std::string>>>("get_status");
  }
  bool do_mix() { return get<bool>("do_mix"); }
  std::map<std::string, std::map<std::string, std::string>> get_proxy_status() {
    return get<std::map<std::string, std::map<std::string, std::string>>>("get_proxy_status");
  }
  const std::string& get_name() const { return name_; }
  void set_name(const std::string& n) { name_ = n; }
  RpcClient& get_client() { return c_; }

 protected:
  template <typename R, typename... Args>
  R get(const std::string& method, const Args&... args) {
    mp::Value v = c_.call(method, name_, args...);
    R r;
    mp::from_value(v, r);
    return r;
  }

 private:
  RpcClient c_;
  std::string name_;
};

}  // namespace jubatus_amd

#endif  // JUBATUS_AMD_MSGPACK_RPC_HPP_
