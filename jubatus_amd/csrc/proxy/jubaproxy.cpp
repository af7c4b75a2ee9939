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

#include "jb_coord_client.hpp"
#include "jb_hash.hpp"
#include "jb_msgpack.hpp"
#include "jb_proxy_tables.hpp"
#include "jb_rpc.hpp"
#include "jubatus_amd/msgpack_rpc.hpp"

namespace {

using jubatus_amd::mp::Value;
const char* kVersion = "1.0.0";

using jb::cc::Conn;
using jb::cc::CallResult;
using jb::cc::Coord;
using jb::cc::dec;
using jb::cc::enc;
using jb::cc::now_s;
using jb::cc::put_raw;
using jb::cc::put_u32;
using jb::cc::response_raw;

void log_line(const char* level, const std::string& msg) { jb::cc::log_tagged("jubaproxy", level, msg); }

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
    coord.reset(new Coord(a.zk, a.zk_timeout, "jubaproxy"));
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
