// juba<engine>_proxy (native): the stateless request router.
//
// Reference C25: jubatus/server/framework/proxy.hpp (random_async_vproxy
// :230-247, broadcast :249-266, cht<N> :268-286, async_task fan-out with
// per-request timeout, transport-error preference and reducer fold
// :295-495, session pool :502-593), proxy.cpp:43-66 (default methods),
// proxy_common.cpp:77-186 (members from cached ZK `actives`, request /
// forward counters, get_proxy_status), aggregators.hpp:27-63.
// The Python twin is jubatus_amd/framework/proxy.py.
//
// Design:
//   * requests arrive on the native epoll transport (csrc/native/jb_rpc.cpp);
//     the params are forwarded *verbatim*: the proxy only reads the cluster
//     name (and, for cht methods, the id) out of the params bytes, and
//     relays single-target results byte for byte. Broadcast / cht results
//     are decoded and folded by the method's aggregator.
//   * fan-out is pipelined: the request goes out on every target's pooled
//     session first, then the responses are collected against one deadline
//     (interconnect_timeout), so N targets cost one round trip.
//   * per-worker-thread session pools (expire -E seconds idle, at most -S
//     sessions, 0 = unlimited); a broken session is evicted.
//   * members / CHT come from the coordinator through a cache invalidated by
//     a 100 ms stat poller (the cached_zk model, cached_zk.cpp:40-186).
//
// Usage: jubaproxy <engine> [proxy flags]   (bin/juba<engine>_proxy)
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <net/if.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pwd.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <functional>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "jb_hash.hpp"
#include "jb_msgpack.hpp"
#include "jb_proxy_tables.hpp"
#include "jb_rpc.hpp"
#include "jubatus_amd/msgpack_rpc.hpp"

namespace {

using jubatus_amd::mp::Value;
const char* kVersion = "1.0.0";

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void log_line(const char* level, const std::string& msg) {
  char ts[64];
  time_t t = time(nullptr);
  struct tm tmv;
  localtime_r(&t, &tmv);
  strftime(ts, sizeof ts, "%Y-%m-%d %H:%M:%S", &tmv);
  fprintf(stderr, "%s %d %-5s [jubaproxy] %s\n", ts, (int)getpid(), level, msg.c_str());
  fflush(stderr);
}

// ------------------------------------------------------------ msgpack bits
void put_u32(std::string& o, uint32_t v) {
  o.push_back((char)0xce);
  for (int k = 3; k >= 0; --k) o.push_back((char)((v >> (8 * k)) & 0xff));
}
void put_raw(std::string& o, const std::string& s) {
  const size_t n = s.size();
  if (n < 32) o.push_back((char)(0xa0 | n));
  else if (n <= 0xffff) { o.push_back((char)0xda); o.push_back((char)(n >> 8)); o.push_back((char)n); }
  else { o.push_back((char)0xdb); for (int k = 3; k >= 0; --k) o.push_back((char)((n >> (8 * k)) & 0xff)); }
  o += s;
}
// [1, msgid, err, result] from raw pieces
std::string response_raw(uint32_t msgid, const std::string& err, const std::string& res) {
  std::string o;
  o.push_back((char)0x94);
  o.push_back((char)0x01);
  put_u32(o, msgid);
  o += err.empty() ? std::string(1, (char)0xc0) : err;
  o += res.empty() ? std::string(1, (char)0xc0) : res;
  return o;
}
std::string enc(const Value& v) {
  std::string o;
  jubatus_amd::mp::encode(v, o);
  return o;
}
Value dec(const std::string& b) {
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
class Coord {
 public:
  Coord(const std::string& hosts, double timeout) : timeout_(timeout) {
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
  }

  Value call(const std::string& m, std::vector<Value> args) {
    std::lock_guard<std::mutex> g(mu_);
    return call_locked(m, std::move(args));
  }

  bool create(const std::string& path, const std::string& data, bool eph) {
    const int64_t rc = call("create", {Value::integer(sid_), Value::str(path), Value::str(data),
                                       Value::boolean(eph)}).as_int();
    return rc == 0 || (rc == -110 && !eph);
  }

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
          log_line("ERROR", "coordinator session expired: shutting down");
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

// ------------------------------------------------------------ aggregators
Value aggregate(const std::string& agg, const Value& a, const Value& b) {
  if (agg == "merge") {
    Value o = a;
    for (const auto& kv : b.as_map()) {
      bool found = false;
      for (auto& x : o.m)
        if (x.first.type == Value::STR && kv.first.type == Value::STR && x.first.s == kv.first.s) {
          x.second = kv.second;
          found = true;
          break;
        }
      if (!found) o.m.push_back(kv);
    }
    return o;
  }
  if (agg == "concat") {
    Value o = a;
    for (const auto& x : b.as_array()) o.a.push_back(x);
    return o;
  }
  if (agg == "add") {
    if (a.type == Value::FLOAT || b.type == Value::FLOAT) return Value::real(a.as_double() + b.as_double());
    return Value::integer(a.as_int() + b.as_int());
  }
  if (agg == "all_and") return Value::boolean(a.as_bool() && b.as_bool());
  if (agg == "all_or") return Value::boolean(a.as_bool() || b.as_bool());
  return a;   // pass / ignore
}

// ------------------------------------------------------------ flags / system
struct Args {
  std::string engine;
  int port = 9199;
  std::string bind_addr, bind_if;
  int threads = 4;
  int timeout = 10, zk_timeout = 10, ic_timeout = 10;
  std::string zk = "localhost:2181";
  int pool_expire = 60, pool_size = 0;
  std::string logdir, log_config;
  bool daemon = false;
  std::string eth;
  std::string prog;
};

std::string if_ipv4(const std::string& want_if, bool skip_loopback) {
  ifaddrs* ifs = nullptr;
  if (getifaddrs(&ifs) != 0) return "";
  std::string out;
  for (ifaddrs* i = ifs; i; i = i->ifa_next) {
    if (!i->ifa_addr || i->ifa_addr->sa_family != AF_INET) continue;
    if (!want_if.empty() && want_if != i->ifa_name) continue;
    if (skip_loopback && (i->ifa_flags & IFF_LOOPBACK)) continue;
    char buf[INET_ADDRSTRLEN];
    inet_ntop(AF_INET, &((sockaddr_in*)i->ifa_addr)->sin_addr, buf, sizeof buf);
    out = buf;
    break;
  }
  freeifaddrs(ifs);
  return out;
}

void usage(const std::string& prog) {
  fprintf(stderr,
          "usage: %s [options]\n"
          "  -p, --rpc-port PORT            port number (9199)\n"
          "  -b, --listen_addr ADDR         bind IP address\n"
          "  -B, --listen_if IF             bind network interface\n"
          "  -c, --thread N                 concurrency = thread number (4)\n"
          "  -t, --timeout SEC              time out (10)\n"
          "  -Z, --zookeeper_timeout SEC    coordinator time out (10)\n"
          "  -I, --interconnect_timeout SEC interconnect time out between servers (10)\n"
          "  -z, --zookeeper HOST:PORT      coordinator location (localhost:2181)\n"
          "  -E, --pool_expire SEC          session-pool expire time (60)\n"
          "  -S, --pool_size N              session-pool maximum size (0 = unlimited)\n"
          "  -l, --logdir DIR  -g, --log_config FILE  -D, --daemon  -v, --version\n",
          prog.c_str());
}

int parse_args(int argc, char** argv, Args* a) {
  if (argc < 2) { fprintf(stderr, "usage: jubaproxy <engine> [options]\n"); return 1; }
  a->engine = argv[1];
  a->prog = "juba" + a->engine + "_proxy";
  for (int i = 2; i < argc; ++i) {
    std::string s = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error(s + " needs a value");
      return argv[++i];
    };
    auto num = [&](int lo) -> int {
      std::string v = val();
      char* end = nullptr;
      long x = strtol(v.c_str(), &end, 10);
      if (!end || *end || x < lo) throw std::runtime_error("bad value for " + s + ": " + v);
      return (int)x;
    };
    if (s == "-p" || s == "--rpc-port") a->port = num(1);
    else if (s == "-b" || s == "--listen_addr") a->bind_addr = val();
    else if (s == "-B" || s == "--listen_if") a->bind_if = val();
    else if (s == "-c" || s == "--thread") a->threads = num(1);
    else if (s == "-t" || s == "--timeout") a->timeout = num(0);
    else if (s == "-Z" || s == "--zookeeper_timeout") a->zk_timeout = num(-1000000);
    else if (s == "-I" || s == "--interconnect_timeout") a->ic_timeout = num(-1000000);
    else if (s == "-z" || s == "--zookeeper") a->zk = val();
    else if (s == "-E" || s == "--pool_expire") a->pool_expire = num(0);
    else if (s == "-S" || s == "--pool_size") a->pool_size = num(0);
    else if (s == "-l" || s == "--logdir") a->logdir = val();
    else if (s == "-g" || s == "--log_config") a->log_config = val();
    else if (s == "-D" || s == "--daemon") a->daemon = true;
    else if (s == "-v" || s == "--version") { printf("jubatus-%s (mi355x, native proxy)\n", kVersion); return -1; }
    else if (s == "-h" || s == "--help") { usage(a->prog); return -1; }
    else { fprintf(stderr, "unknown option: %s\n", s.c_str()); usage(a->prog); return 1; }
  }
  if (a->zk_timeout < 1 || a->ic_timeout < 1) {
    fprintf(stderr, "can't start with a timeout less than 1\n");
    return 1;
  }
  if (!a->logdir.empty() && access(a->logdir.c_str(), W_OK) != 0) {
    fprintf(stderr, "can't create log file\n");
    return 1;
  }
  if (!a->bind_addr.empty()) a->eth = a->bind_addr;
  else if (!a->bind_if.empty()) a->eth = a->bind_addr = if_ipv4(a->bind_if, false);
  else { a->bind_addr = "0.0.0.0"; a->eth = if_ipv4("", true); if (a->eth.empty()) a->eth = "127.0.0.1"; }
  return 0;
}

std::map<std::string, std::string> machine_status() {
  std::map<std::string, std::string> m{{"VIRT", "0"}, {"RSS", "0"}, {"SHR", "0"}};
  FILE* f = fopen("/proc/self/statm", "r");
  if (f) {
    long size = 0, res = 0, shr = 0;
    if (fscanf(f, "%ld %ld %ld", &size, &res, &shr) == 3) {
      const long kb = sysconf(_SC_PAGESIZE) / 1024;
      m["VIRT"] = std::to_string(size * kb);
      m["RSS"] = std::to_string(res * kb);
      m["SHR"] = std::to_string(shr * kb);
    }
    fclose(f);
  }
  return m;
}

std::string user_name() {
  passwd* pw = getpwuid(getuid());
  return pw ? pw->pw_name : std::to_string(getuid());
}

// ------------------------------------------------------------ proxy
struct Route {
  std::string routing, agg;
  int cht_n = 0, arity = 0;
};

struct PoolEntry {
  std::unique_ptr<Conn> conn;
};

class Proxy {
 public:
  Proxy(const Args& a, Coord* coord) : a_(a), coord_(coord), start_(time(nullptr)) {
    for (const auto& e : jb::proxy::kEngines)
      if (a.engine == e.engine)
        for (int i = 0; i < e.n; ++i)
          routes_[e.methods[i].name] = Route{e.methods[i].routing, e.methods[i].agg,
                                             e.methods[i].cht_n, e.methods[i].arity};
    if (routes_.empty()) throw std::runtime_error("unknown engine: " + a.engine);
  }

  std::string handle(const jb::RpcRequest& r) {
    requests_.fetch_add(1, std::memory_order_relaxed);
    if (r.method == "get_proxy_status") return r.notify ? "" : response_raw(r.msgid, "", enc(status()));
    auto it = routes_.find(r.method);
    if (it == routes_.end()) return r.notify ? "" : response_raw(r.msgid, enc(Value::uinteger(1)), "");
    std::string err, res;
    try {
      route(it->first, it->second, r.params, &err, &res);
    } catch (const std::invalid_argument&) {
      err = enc(Value::uinteger(2));
      res.clear();
    } catch (const std::exception& e) {
      err = enc(Value::str(e.what()));
      res.clear();
    }
    return r.notify ? "" : response_raw(r.msgid, err, res);
  }

 private:
  std::vector<std::pair<std::string, int>> members(const std::string& name) {
    std::vector<std::pair<std::string, int>> out;
    for (const auto& loc : coord_->list(actor(name) + "/actives")) out.push_back(revert(loc));
    return out;
  }
  std::string actor(const std::string& name) const {
    return "/jubatus/actors/" + a_.engine + "/" + name;
  }
  static std::pair<std::string, int> revert(const std::string& loc) {
    const size_t u = loc.find('_');
    if (u == std::string::npos) return {loc, 0};
    return {loc.substr(0, u), atoi(loc.c_str() + u + 1)};
  }

  // CHT: n consecutive vnodes from lower_bound(md5(key)), with wrap-around (cht.cpp:107-143)
  std::vector<std::pair<std::string, int>> cht_find(const std::string& name, const std::string& key, int n) {
    const std::string path = actor(name) + "/cht";
    std::vector<std::string> h = coord_->list(path);
    if (h.empty()) throw std::runtime_error("failed to fetch list of CHT entry: " + key);
    std::sort(h.begin(), h.end());
    size_t idx = std::lower_bound(h.begin(), h.end(), jb::Md5::hex(key)) - h.begin();
    idx %= h.size();
    std::vector<std::pair<std::string, int>> out;
    for (int i = 0; i < n; ++i) {
      std::string loc;
      if (!coord_->read(path + "/" + h[idx], &loc)) throw std::runtime_error("failed to read CHT entry: " + path);
      out.push_back(revert(loc));
      idx = (idx + 1) % h.size();
    }
    return out;
  }

  void route(const std::string& method, const Route& rt, const std::string& params,
             std::string* err, std::string* res) {
    jb::Cursor c{(const uint8_t*)params.data(), (const uint8_t*)params.data() + params.size()};
    uint32_t n;
    if (!c.array(&n) || (int)n != rt.arity) throw std::invalid_argument("arity");
    const uint8_t* s;
    uint32_t sl;
    if (!c.raw(&s, &sl)) throw std::invalid_argument("cluster name must be a string");
    const std::string name((const char*)s, sl);
    std::vector<std::pair<std::string, int>> targets;
    if (rt.routing == "cht") {
      if (!c.raw(&s, &sl)) throw std::invalid_argument("cht key must be a string");
      targets = cht_find(name, std::string((const char*)s, sl), rt.cht_n);
    } else {
      targets = members(name);
      if (targets.empty())
        throw std::runtime_error("no server found in coordinator: " + a_.engine + "/" + name);
      if (rt.routing == "random") {
        thread_local std::mt19937_64 rng{std::random_device{}()};
        targets = {targets[rng() % targets.size()]};
      }
    }
    forwards_.fetch_add(targets.size(), std::memory_order_relaxed);
    fanout(method, params, targets, rt.agg, err, res);
  }

  // this worker thread's session pool
  static std::map<std::pair<std::string, int>, PoolEntry>& pool() {
    thread_local std::map<std::pair<std::string, int>, PoolEntry> p;
    return p;
  }

  Conn* session(const std::pair<std::string, int>& t, double now) {
    auto& pool = this->pool();
    auto it = pool.find(t);
    if (it != pool.end() && a_.pool_expire > 0 && now - it->second.conn->last_used > a_.pool_expire)
      { pool.erase(it); it = pool.end(); }
    if (it == pool.end()) {
      if (a_.pool_size > 0 && (int)pool.size() >= a_.pool_size) {
        auto oldest = pool.begin();
        for (auto j = pool.begin(); j != pool.end(); ++j)
          if (j->second.conn->last_used < oldest->second.conn->last_used) oldest = j;
        pool.erase(oldest);
      }
      PoolEntry e;
      e.conn.reset(new Conn(t.first, t.second, a_.ic_timeout));
      it = pool.emplace(t, std::move(e)).first;
    }
    it->second.conn->last_used = now;
    return it->second.conn.get();
  }

  void fanout(const std::string& method, const std::string& params,
              const std::vector<std::pair<std::string, int>>& targets, const std::string& agg,
              std::string* err, std::string* res) {
    const double t0 = now_s();
    const double deadline = t0 + a_.ic_timeout;
    std::vector<CallResult> out(targets.size());
    std::vector<Conn*> conns(targets.size(), nullptr);
    std::vector<uint32_t> ids(targets.size(), 0);
    for (size_t i = 0; i < targets.size(); ++i) {   // send everywhere first
      try {
        conns[i] = session(targets[i], t0);
        ids[i] = conns[i]->send_request(method, params, deadline);
      } catch (const std::exception& e) {
        out[i].transport_error = e.what();
        conns[i] = nullptr;
        drop(targets[i]);
      }
    }
    for (size_t i = 0; i < targets.size(); ++i) {   // then collect
      if (!conns[i]) continue;
      try {
        conns[i]->recv_response(ids[i], deadline, &out[i]);
      } catch (const std::exception& e) {
        out[i].transport_error = e.what();
        drop(targets[i]);
      }
    }
    std::vector<size_t> ok;
    for (size_t i = 0; i < out.size(); ++i)
      if (out[i].transport_ok && out[i].err.empty()) ok.push_back(i);
    if (ok.empty()) {
      // prefer a transport error in the reply (proxy.hpp:325-376)
      for (size_t i = 0; i < out.size(); ++i)
        if (!out[i].transport_ok) {
          *err = enc(Value::str(targets[i].first + ":" + std::to_string(targets[i].second) + ": " +
                                out[i].transport_error));
          return;
        }
      *err = out[0].err;   // the server's own error, verbatim
      return;
    }
    for (size_t i = 0; i < out.size(); ++i)
      if (std::find(ok.begin(), ok.end(), i) == ok.end())
        log_line("WARN", "partial failure from " + targets[i].first + ":" +
                             std::to_string(targets[i].second));
    if (ok.size() == 1 || agg == "pass" || agg == "ignore") {
      *res = out[ok[0]].res;   // relayed byte for byte
      return;
    }
    Value acc = dec(out[ok[0]].res);
    for (size_t j = 1; j < ok.size(); ++j) acc = aggregate(agg, acc, dec(out[ok[j]].res));
    *res = enc(acc);
  }

  // evict a broken session of this worker thread (reconnected on next use)
  void drop(const std::pair<std::string, int>& t) { pool().erase(t); }

  Value status() {
    const time_t now = time(nullptr);
    auto mt = machine_status();
    std::vector<std::pair<std::string, std::string>> kv = {
        {"clock_time", std::to_string((long)now)},
        {"start_time", std::to_string((long)start_)},
        {"uptime", std::to_string((long)(now - start_))},
        {"VIRT", mt["VIRT"]}, {"RSS", mt["RSS"]}, {"SHR", mt["SHR"]},
        {"VERSION", kVersion}, {"PROGNAME", a_.prog}, {"pid", std::to_string((int)getpid())},
        {"user", user_name()}, {"threadnum", std::to_string(a_.threads)},
        {"timeout", std::to_string(a_.timeout)}, {"logdir", a_.logdir},
        {"log_config", a_.log_config}, {"zookeeper", a_.zk},
        {"connected_zookeeper", coord_->connected()},
        {"zookeeper_timeout", std::to_string(a_.zk_timeout)},
        {"interconnect_timeout", std::to_string(a_.ic_timeout)},
        {"session_pool_expire", std::to_string(a_.pool_expire)},
        {"session_pool_size", std::to_string(a_.pool_size)},
        {"request_count", std::to_string(requests_.load())},
        {"forward_count", std::to_string(forwards_.load())},
        {"implementation", "native"},
    };
    Value inner = Value::map();
    for (auto& p : kv) inner.m.emplace_back(Value::str(p.first), Value::str(p.second));
    Value outer = Value::map();
    outer.m.emplace_back(Value::str(a_.eth + "_" + std::to_string(a_.port)), inner);
    return outer;
  }

  Args a_;
  Coord* coord_;
  time_t start_;
  std::map<std::string, Route> routes_;
  std::atomic<uint64_t> requests_{0}, forwards_{0};
};

}  // namespace

int main(int argc, char** argv) {
  Args a;
  int rc;
  try {
    rc = parse_args(argc, argv, &a);
  } catch (const std::exception& e) {
    fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  if (rc) return rc < 0 ? 0 : rc;

  sigset_t ss;
  sigemptyset(&ss);
  sigaddset(&ss, SIGTERM);
  sigaddset(&ss, SIGINT);
  sigaddset(&ss, SIGHUP);
  pthread_sigmask(SIG_BLOCK, &ss, nullptr);
  signal(SIGPIPE, SIG_IGN);

  std::unique_ptr<Coord> coord;
  try {
    coord.reset(new Coord(a.zk, a.zk_timeout));
  } catch (const std::exception& e) {
    log_line("FATAL", e.what());
    return 1;
  }
  std::unique_ptr<Proxy> proxy;
  try {
    proxy.reset(new Proxy(a, coord.get()));
  } catch (const std::exception& e) {
    log_line("FATAL", e.what());
    return 1;
  }
  Proxy* px = proxy.get();
  jb::RpcServer srv([px](const jb::RpcRequest& r) { return px->handle(r); }, a.threads, 0.0);
  srv.set_io_threads(a.threads >= 8 ? a.threads / 4 : 1);
  try {
    const int bound = srv.listen(a.bind_addr, a.port);
    a.port = bound;
  } catch (const std::exception& e) {
    log_line("FATAL", std::string("listen failed: ") + e.what());
    return 1;
  }
  srv.start();
  // register_proxy (membership.cpp:208-233)
  coord->create("/jubatus", "", false);
  coord->create("/jubatus/jubaproxies", "", false);
  coord->create("/jubatus/jubaproxies/" + a.engine, "", false);
  if (!coord->create("/jubatus/jubaproxies/" + a.engine + "/" + a.eth + "_" + std::to_string(a.port), "", true)) {
    log_line("FATAL", "Failed to register_proxy");
    srv.stop();
    return 1;
  }
  log_line("INFO", a.prog + " (native) listening at " + a.eth + ":" + std::to_string(a.port));
  printf("jubaproxy ready %d\n", a.port);
  fflush(stdout);
  for (;;) {
    int sig = 0;
    sigwait(&ss, &sig);
    if (sig == SIGHUP) continue;
    log_line("INFO", "stopping on signal " + std::to_string(sig));
    break;
  }
  srv.stop();
  coord->close();
  return 0;
}
