// jubacoordinator (native): the cluster coordination server.
//
// Replaces the ZooKeeper ensemble the reference runs against (lock_service
// C5-C11: zk.cpp, cached_zk.cpp, membership.cpp, cht.cpp, config.cpp,
// global_id_generator_zk.cpp all talk to it through the same RPCs the
// Python CoordinatorClient uses, jubatus_amd/common/lock_service.py).
//
// Process model: the native epoll msgpack-RPC transport (csrc/native/jb_rpc.cpp)
// with C++ handlers over a ZNodeStore (jb_znode.hpp); a sweeper thread
// expires sessions whose heartbeat is older than their timeout (their
// ephemeral nodes go with them: the liveness mechanism behind membership,
// CHT and the mixer master lock). SIGTERM/SIGINT stop it.
//
// RPCs (params as msgpack arrays, results as in the Python twin):
//   open_session(timeout) -> sid            heartbeat(sid) -> bool
//   close_session(sid) -> nil               create(sid, path, data, eph) -> rc
//   create_seq(sid, path) -> [rc, path]     set(path, data) -> [rc, version]
//   remove(path) -> rc                      exists(path) -> bool
//   list(path) -> [rc, [child]]             read(path) -> [rc, data, version]
//   stat_many([path]) -> [[exists, mzxid, pzxid]]     dump() -> {path: data}
// Errors: unknown method -> 1 (NO_METHOD_ERROR), bad arity / argument type
// -> 2 (ARGUMENT_ERROR), as the reference's rpc_server (rpc_server.cpp:31-54).
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "jb_rpc.hpp"
#include "jb_znode.hpp"
#include "jubatus_amd/msgpack_rpc.hpp"

namespace {

using jubatus_amd::mp::Value;
using jb::coord::ZNodeStore;

struct ArgError : std::runtime_error {
  ArgError() : std::runtime_error("argument error") {}
};

void log_line(const char* level, const std::string& msg) {
  char ts[64];
  time_t t = time(nullptr);
  struct tm tmv;
  localtime_r(&t, &tmv);
  strftime(ts, sizeof ts, "%Y-%m-%d %H:%M:%S", &tmv);
  fprintf(stderr, "%s %d %-5s [jubacoordinator] %s\n", ts, (int)getpid(), level, msg.c_str());
  fflush(stderr);
}

const Value& arg(const std::vector<Value>& a, size_t i) {
  if (i >= a.size()) throw ArgError();
  return a[i];
}
const std::string& s_arg(const std::vector<Value>& a, size_t i) {
  const Value& v = arg(a, i);
  if (v.type != Value::STR) throw ArgError();
  return v.s;
}
int64_t i_arg(const std::vector<Value>& a, size_t i) {
  const Value& v = arg(a, i);
  if (v.type != Value::INT && v.type != Value::UINT) throw ArgError();
  return v.as_int();
}
double d_arg(const std::vector<Value>& a, size_t i) {
  const Value& v = arg(a, i);
  if (v.type != Value::INT && v.type != Value::UINT && v.type != Value::FLOAT) throw ArgError();
  return v.as_double();
}
bool b_arg(const std::vector<Value>& a, size_t i) {
  const Value& v = arg(a, i);
  if (v.type == Value::BOOL) return v.b;
  if (v.type == Value::INT || v.type == Value::UINT) return v.as_int() != 0;
  throw ArgError();
}
void arity(const std::vector<Value>& a, size_t n) {
  if (a.size() != n) throw ArgError();
}

Value dispatch(ZNodeStore& st, const std::string& m, const std::vector<Value>& a) {
  using jubatus_amd::mp::to_value;
  if (m == "heartbeat") { arity(a, 1); return Value::boolean(st.heartbeat(i_arg(a, 0))); }
  if (m == "exists") { arity(a, 1); return Value::boolean(st.exists(s_arg(a, 0))); }
  if (m == "read") {
    arity(a, 1);
    auto r = st.read(s_arg(a, 0));
    return Value::array({Value::integer(std::get<0>(r)), Value::str(std::get<1>(r)),
                         Value::integer(std::get<2>(r))});
  }
  if (m == "list") {
    arity(a, 1);
    auto r = st.list(s_arg(a, 0));
    return Value::array({Value::integer(r.first), to_value(r.second)});
  }
  if (m == "stat_many") {
    arity(a, 1);
    const Value& ps = arg(a, 0);
    if (ps.type != Value::ARRAY) throw ArgError();
    std::vector<std::string> paths;
    for (const auto& p : ps.a) {
      if (p.type != Value::STR) throw ArgError();
      paths.push_back(p.s);
    }
    Value out = Value::array();
    for (const auto& t : st.stat_many(paths))
      out.a.push_back(Value::array({Value::boolean(std::get<0>(t)), Value::integer(std::get<1>(t)),
                                    Value::integer(std::get<2>(t))}));
    return out;
  }
  if (m == "create") {
    arity(a, 4);
    return Value::integer(st.create(i_arg(a, 0), s_arg(a, 1), s_arg(a, 2), b_arg(a, 3)));
  }
  if (m == "create_seq") {
    arity(a, 2);
    auto r = st.create_seq(i_arg(a, 0), s_arg(a, 1), "", true);
    return Value::array({Value::integer(r.first), Value::str(r.second)});
  }
  if (m == "set") {
    arity(a, 2);
    auto r = st.set(s_arg(a, 0), s_arg(a, 1));
    return Value::array({Value::integer(r.first), Value::integer(r.second)});
  }
  if (m == "remove") { arity(a, 1); return Value::integer(st.remove(s_arg(a, 0))); }
  if (m == "open_session") { arity(a, 1); return Value::integer(st.open_session(d_arg(a, 0))); }
  if (m == "close_session") { arity(a, 1); st.close_session(i_arg(a, 0)); return Value::nil(); }
  if (m == "dump") {
    arity(a, 0);
    Value out = Value::map();
    for (auto& kv : st.dump()) out.m.emplace_back(Value::str(kv.first), Value::str(kv.second));
    return out;
  }
  throw std::out_of_range(m);
}

std::string response(uint32_t msgid, const Value& err, const Value& result) {
  std::string o;
  jubatus_amd::mp::encode(Value::array({Value::uinteger(1), Value::uinteger(msgid), err, result}), o);
  return o;
}

std::string handle(ZNodeStore& st, const jb::RpcRequest& r) {
  Value err, result;
  try {
    Value params;
    jubatus_amd::mp::Decoder dec(r.params.data(), r.params.size());
    if (!dec.next(params) || params.type != Value::ARRAY) throw ArgError();
    result = dispatch(st, r.method, params.a);
  } catch (const ArgError&) {
    err = Value::uinteger(2);
  } catch (const std::out_of_range&) {
    err = Value::uinteger(1);
  } catch (const std::exception& e) {
    err = Value::str(e.what());
  }
  if (r.notify) return std::string();
  return response(r.msgid, err, result);
}

void usage(const char* prog) {
  fprintf(stderr,
          "usage: %s [-p port] [-b listen_addr] [-c threads]\n"
          "  -p, --port         listen port (default 2181)\n"
          "  -b, --listen_addr  bind address (default 0.0.0.0)\n"
          "  -c, --thread       RPC worker threads (default 4)\n",
          prog);
}

}  // namespace

int main(int argc, char** argv) {
  int port = 2181, threads = 4;
  std::string bind = "0.0.0.0";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* name) -> std::string {
      if (i + 1 >= argc) { fprintf(stderr, "%s needs a value\n", name); exit(1); }
      return argv[++i];
    };
    if (a == "-p" || a == "--port") port = atoi(val("--port").c_str());
    else if (a == "-b" || a == "--listen_addr") bind = val("--listen_addr");
    else if (a == "-c" || a == "--thread") threads = atoi(val("--thread").c_str());
    else if (a == "-h" || a == "--help") { usage(argv[0]); return 0; }
    else { fprintf(stderr, "unknown option: %s\n", a.c_str()); usage(argv[0]); return 1; }
  }
  if (threads < 1) threads = 1;

  // TERM/INT/HUP are handled by sigwait on the main thread (the reference's
  // signals.cpp:98-181 model); block them before any thread starts
  sigset_t ss;
  sigemptyset(&ss);
  sigaddset(&ss, SIGTERM);
  sigaddset(&ss, SIGINT);
  sigaddset(&ss, SIGHUP);
  pthread_sigmask(SIG_BLOCK, &ss, nullptr);
  signal(SIGPIPE, SIG_IGN);

  ZNodeStore store;
  jb::RpcServer srv([&store](const jb::RpcRequest& r) { return handle(store, r); }, threads, 0.0);
  int bound;
  try {
    bound = srv.listen(bind, port);
  } catch (const std::exception& e) {
    log_line("FATAL", std::string("listen failed: ") + e.what());
    return 1;
  }
  srv.start();
  log_line("INFO", "coordinator listening on " + bind + ":" + std::to_string(bound) +
                       " (native, " + std::to_string(threads) + " threads)");
  // stdout line for launchers waiting on readiness
  printf("jubacoordinator ready %d\n", bound);
  fflush(stdout);

  std::atomic<bool> stop{false};
  std::thread sweeper([&] {
    while (!stop.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      for (int64_t sid : store.expire_sessions())
        log_line("INFO", "session " + std::to_string(sid) + " expired");
    }
  });
  for (;;) {
    int sig = 0;
    sigwait(&ss, &sig);
    if (sig == SIGHUP) continue;   // nothing to reopen: logs go to stderr
    log_line("INFO", "stopping on signal " + std::to_string(sig));
    break;
  }
  stop.store(true);
  sweeper.join();
  srv.stop();
  return 0;
}
