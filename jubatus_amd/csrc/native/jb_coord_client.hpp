// Native coordinator client shared by the native cluster executables
// (jubaproxy, jubavisor): a blocking msgpack-RPC connection plus a session
// with heartbeat and a stat-polled cache of list/read results.
//
// Reference: the cached ZooKeeper client the proxy and jubavisor use
// (common/cached_zk.cpp:40-186: list/read cached until a watch fires;
// common/zk.cpp:81-104 session; membership.cpp:257-259: losing the session
// shuts the process down). The server side is csrc/coord/jubacoordinator.cpp;
// the Python twin of this client is jubatus_amd/common/lock_service.py.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "jb_msgpack.hpp"
#include "jb_rpc.hpp"
#include "jubatus_amd/msgpack_rpc.hpp"
#include "jb_log.hpp"

namespace jb {
namespace cc {

using jubatus_amd::mp::Value;

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline void log_tagged(const char* tag, const char* level, const std::string& msg) {
  jb::jlog::write(level, tag, msg.c_str());
}

// ------------------------------------------------------------ msgpack bits
inline void put_u32(std::string& o, uint32_t v) {
  o.push_back((char)0xce);
  for (int k = 3; k >= 0; --k) o.push_back((char)((v >> (8 * k)) & 0xff));
}
inline void put_raw(std::string& o, const std::string& s) {
  const size_t n = s.size();
  if (n < 32) o.push_back((char)(0xa0 | n));
  else if (n <= 0xffff) { o.push_back((char)0xda); o.push_back((char)(n >> 8)); o.push_back((char)n); }
  else { o.push_back((char)0xdb); for (int k = 3; k >= 0; --k) o.push_back((char)((n >> (8 * k)) & 0xff)); }
  o += s;
}
// [1, msgid, err, result] from raw pieces
inline std::string response_raw(uint32_t msgid, const std::string& err, const std::string& res) {
  std::string o;
  o.push_back((char)0x94);
  o.push_back((char)0x01);
  put_u32(o, msgid);
  o += err.empty() ? std::string(1, (char)0xc0) : err;
  o += res.empty() ? std::string(1, (char)0xc0) : res;
  return o;
}
inline std::string enc(const Value& v) {
  std::string o;
  jubatus_amd::mp::encode(v, o);
  return o;
}
inline Value dec(const std::string& b) {
  Value v;
  jubatus_amd::mp::Decoder d(b.data(), b.size());
  if (!d.next(v)) throw std::runtime_error("truncated msgpack");
  return v;
}

// ------------------------------------------------------------ connection
struct CallResult {
  bool transport_ok = false;   // a response arrived
  std::string transport_error; // io / timeout message
  std::string err;             // raw msgpack error ("" = nil)
  std::string res;             // raw msgpack result
};

// one non-blocking TCP session; requests may be pipelined (send several,
// then collect each response by msgid against a deadline)
class Conn {
 public:
  Conn(const std::string& host, int port, double timeout) : host_(host), port_(port) {
    addrinfo hints{}, *ai = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &ai) != 0 || !ai)
      throw std::runtime_error("cannot resolve " + host);
    fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd_ < 0) { freeaddrinfo(ai); throw std::runtime_error("socket failed"); }
    fcntl(fd_, F_SETFL, fcntl(fd_, F_GETFL) | O_NONBLOCK);
    int rc = ::connect(fd_, ai->ai_addr, ai->ai_addrlen);
    freeaddrinfo(ai);
    if (rc != 0 && errno != EINPROGRESS) { ::close(fd_); throw std::runtime_error("connect refused"); }
    if (rc != 0) {
      pollfd p{fd_, POLLOUT, 0};
      if (::poll(&p, 1, (int)(timeout * 1000)) <= 0) { ::close(fd_); throw std::runtime_error("connect timeout"); }
      int err = 0;
      socklen_t len = sizeof err;
      getsockopt(fd_, SOL_SOCKET, SO_ERROR, &err, &len);
      if (err) { ::close(fd_); throw std::runtime_error(std::string("connect: ") + strerror(err)); }
    }
    int one = 1;
    setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    last_used = now_s();
  }
  ~Conn() { if (fd_ >= 0) ::close(fd_); }
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;

  uint32_t send_request(const std::string& method, const std::string& params_raw, double deadline) {
    const uint32_t id = next_id_++;
    std::string o;
    o.push_back((char)0x94);
    o.push_back((char)0x00);
    put_u32(o, id);
    put_raw(o, method);
    o += params_raw;
    size_t off = 0;
    while (off < o.size()) {
      ssize_t k = ::send(fd_, o.data() + off, o.size() - off, MSG_NOSIGNAL);
      if (k > 0) { off += (size_t)k; continue; }
      if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!wait(POLLOUT, deadline)) throw std::runtime_error("send timeout");
        continue;
      }
      if (k < 0 && errno == EINTR) continue;
      throw std::runtime_error("send failed");
    }
    return id;
  }

  // one response for msgid; fills err/res raw spans
  void recv_response(uint32_t msgid, double deadline, CallResult* out) {
    for (;;) {
      const int64_t f = rbuf_.empty() ? 0 : jb::msgpack_frame((const uint8_t*)rbuf_.data(), rbuf_.size());
      if (f < 0) throw std::runtime_error("malformed response");
      if (f > 0) {
        std::string msg = rbuf_.substr(0, (size_t)f);
        rbuf_.erase(0, (size_t)f);
        jb::Cursor c{(const uint8_t*)msg.data(), (const uint8_t*)msg.data() + msg.size()};
        uint32_t n;
        double type, id;
        if (!c.array(&n) || n != 4 || !c.number(&type) || !c.number(&id))
          throw std::runtime_error("malformed response");
        const uint8_t* e0 = c.p;
        if (!c.skip()) throw std::runtime_error("malformed response");
        const uint8_t* e1 = c.p;
        if (!c.skip()) throw std::runtime_error("malformed response");
        if ((uint32_t)id != msgid) continue;   // stale answer of a timed-out call
        out->transport_ok = true;
        out->err = (e1 - e0 == 1 && *e0 == 0xc0) ? std::string() : std::string((const char*)e0, e1 - e0);
        out->res.assign((const char*)e1, c.p - e1);
        return;
      }
      char buf[65536];
      ssize_t k = ::recv(fd_, buf, sizeof buf, 0);
      if (k > 0) { rbuf_.append(buf, (size_t)k); continue; }
      if (k == 0) throw std::runtime_error("connection closed by peer");
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        if (!wait(POLLIN, deadline)) throw std::runtime_error("timeout");
        continue;
      }
      throw std::runtime_error("recv failed");
    }
  }

  double last_used;
  const std::string host_;
  const int port_;

 private:
  bool wait(short ev, double deadline) {
    const double left = deadline - now_s();
    if (left <= 0) return false;
    pollfd p{fd_, ev, 0};
    return ::poll(&p, 1, (int)(left * 1000) + 1) > 0;
  }
  int fd_ = -1;
  uint32_t next_id_ = 1;
  std::string rbuf_;
};

// ------------------------------------------------------------ coordinator
// A session on the first reachable coordinator of "h1:p1,h2:p2". A heartbeat
// thread keeps it alive; when the coordinator reports it expired the process
// gets SIGTERM, so its sigwait loop runs the normal shutdown (for jubavisor
// that stops every child). list/read are cached and invalidated by a 100 ms
// stat_many poller.
class Coord {
 public:
  Coord(const std::string& hosts, double timeout, const char* tag = "coord")
      : timeout_(timeout), tag_(tag) {
    std::string err;
    const double deadline = now_s() + timeout;
    while (!conn_) {
      size_t s = 0;
      while (s <= hosts.size()) {
        size_t e = hosts.find(',', s);
        if (e == std::string::npos) e = hosts.size();
        std::string hp = hosts.substr(s, e - s);
        s = e + 1;
        const size_t colon = hp.rfind(':');
        if (colon == std::string::npos) continue;
        try {
          conn_.reset(new Conn(hp.substr(0, colon), atoi(hp.c_str() + colon + 1), timeout));
          connected_ = hp;
          sid_ = call_locked("open_session", {Value::real(timeout)}).as_int();
          jb::jlog::zk("INFO", tag_, "coordinator session " + std::to_string(sid_) + " opened on " + hp);
          break;
        } catch (const std::exception& ex) {
          conn_.reset();
          err = ex.what();
        }
      }
      if (!conn_) {
        if (now_s() > deadline) throw std::runtime_error("failed to connect to coordinator " + hosts + ": " + err);
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
      }
    }
    hb_ = std::thread([this] { heartbeat_loop(); });
    poll_ = std::thread([this] { poll_loop(); });
  }
  ~Coord() { close(); }

  void close() {
    if (stop_.exchange(true)) return;
    if (hb_.joinable()) hb_.join();
    if (poll_.joinable()) poll_.join();
    try { call("close_session", {Value::integer(sid_)}); } catch (...) {}
    jb::jlog::zk("INFO", tag_, "coordinator session " + std::to_string(sid_) + " closed");
  }

  Value call(const std::string& m, std::vector<Value> args) {
    std::lock_guard<std::mutex> g(mu_);
    return call_locked(m, std::move(args));
  }

  // true when created (or, for a persistent node, already there)
  bool create(const std::string& path, const std::string& data, bool eph) {
    const int64_t rc = call("create", {Value::integer(sid_), Value::str(path), Value::str(data),
                                       Value::boolean(eph)}).as_int();
    return rc == 0 || (rc == -110 && !eph);
  }
  bool exists(const std::string& path) { return call("exists", {Value::str(path)}).as_bool(); }

  // cached list / read (invalidated by the stat poller)
  std::vector<std::string> list(const std::string& path) {
    {
      std::lock_guard<std::mutex> g(cmu_);
      auto it = lcache_.find(path);
      if (it != lcache_.end()) return it->second;
    }
    Value r = call("list", {Value::str(path)});
    std::vector<std::string> out;
    if (r.as_array().at(0).as_int() == 0)
      for (const auto& x : r.as_array().at(1).as_array()) out.push_back(x.as_str());
    std::lock_guard<std::mutex> g(cmu_);
    lcache_[path] = out;
    watch(path);
    return out;
  }
  bool read(const std::string& path, std::string* data) {
    {
      std::lock_guard<std::mutex> g(cmu_);
      auto it = rcache_.find(path);
      if (it != rcache_.end()) { *data = it->second; return true; }
    }
    Value r = call("read", {Value::str(path)});
    if (r.as_array().at(0).as_int() != 0) return false;
    *data = r.as_array().at(1).as_str();
    std::lock_guard<std::mutex> g(cmu_);
    rcache_[path] = *data;
    watch(path);
    return true;
  }
  const std::string& connected() const { return connected_; }
  int64_t session() const { return sid_; }

 private:
  Value call_locked(const std::string& m, std::vector<Value> args) {
    const double dl = now_s() + timeout_;
    const uint32_t id = conn_->send_request(m, enc(Value::array(std::move(args))), dl);
    CallResult r;
    conn_->recv_response(id, dl, &r);
    if (!r.err.empty()) throw std::runtime_error("coordinator error in " + m);
    return dec(r.res);
  }
  void watch(const std::string& path) {   // cmu_ held
    if (!stat_.count(path)) stat_[path] = {-1, -1, -1};
  }
  void heartbeat_loop() {
    const double period = std::max(0.05, timeout_ / 3.0);
    while (!stop_.load()) {
      for (int i = 0; i < (int)(period * 20) && !stop_.load(); ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
      if (stop_.load()) break;
      try {
        if (!call("heartbeat", {Value::integer(sid_)}).as_bool()) {
          jb::jlog::zk("ERROR", tag_, "coordinator session expired: shutting down");
          log_tagged(tag_, "ERROR", "coordinator session expired: shutting down");
          kill(getpid(), SIGTERM);   // the reference's shutdown_server (membership.cpp:257-259)
          return;
        }
      } catch (...) {
        // unreachable: keep trying until the session TTL decides
      }
    }
  }
  void poll_loop() {
    while (!stop_.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      std::vector<std::string> paths;
      {
        std::lock_guard<std::mutex> g(cmu_);
        for (const auto& kv : stat_) paths.push_back(kv.first);
      }
      if (paths.empty()) continue;
      Value arr = Value::array();
      for (const auto& p : paths) arr.a.push_back(Value::str(p));
      Value r;
      try { r = call("stat_many", {arr}); } catch (...) { continue; }
      std::lock_guard<std::mutex> g(cmu_);
      for (size_t i = 0; i < paths.size() && i < r.a.size(); ++i) {
        const auto& st = r.a[i].as_array();
        std::array<int64_t, 3> now{st[0].as_bool() ? 1 : 0, st[1].as_int(), st[2].as_int()};
        auto& old = stat_[paths[i]];
        if (old[0] >= 0 && old != now) {   // changed: invalidate (CHILD / DATA / DELETED)
          lcache_.erase(paths[i]);
          rcache_.erase(paths[i]);
        }
        old = now;
      }
    }
  }

  double timeout_;
  const char* tag_;
  std::unique_ptr<Conn> conn_;
  std::string connected_;
  int64_t sid_ = 0;
  std::mutex mu_;
  std::mutex cmu_;
  std::map<std::string, std::vector<std::string>> lcache_;
  std::map<std::string, std::string> rcache_;
  std::map<std::string, std::array<int64_t, 3>> stat_;
  std::atomic<bool> stop_{false};
  std::thread hb_, poll_;
};

}  // namespace cc
}  // namespace jb
