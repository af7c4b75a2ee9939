// jubavisor (native): the per-host process supervisor.
//
// Reference C31: jubatus/server/jubavisor/jubavisor.cpp:55-265 (register
// /jubatus/supervisors/<ip>_<port>, start/stop, port pool, SIGCHLD reaping,
// coordinator loss stops every child), process.cpp:46-160 (child command
// line), main.cpp:76-143 (flags). The Python twin is
// jubatus_amd/cmd/jubavisor.py; jubactl (cmd/jubactl.py) drives either.
//
// Design:
//   * RPCs arrive on the native epoll transport (csrc/native/jb_rpc.cpp);
//     the coordinator session is the shared native client
//     (csrc/native/jb_coord_client.hpp).
//   * children are started with posix_spawn (no fork of this multi-threaded
//     process), each in its own process group, with the reference's flag set
//     -z -n -p -B -c -t -Z -I -d -l -g -s -i -x. The server program is
//     <repo>/bin/juba<engine> next to this binary's tree, or
//     $JUBAVISOR_SERVER_DIR/juba<engine> when set.
//   * a reaper thread collects exited children every 100 ms (waitpid
//     WNOHANG on each known pid) and returns their ports to the pool: the
//     SIGCHLD handler of jubavisor.cpp:113-156 without async-signal work.
//   * TERM/INT, including the SIGTERM the coordinator client raises when the
//     session expires, stop every child (SIGTERM, then SIGKILL after 10 s)
//     before the process exits.
//
// RPCs:  start(server_name "juba<engine>/<name>", N, server_argv) -> int
//        stop(server_name, N) -> int      (N is ignored, as in the
//                                          reference, jubavisor.hpp:80-82)
// server_argv on the wire (server_util.hpp:91-94): [port, bind_address,
// bind_if, timeout, zookeeper_timeout, interconnect_timeout, threadnum,
// program_name, type, z, name, datadir, logdir, log_config, eth,
// interval_sec, interval_count, mixer, daemon]; a map with those keys is
// accepted too.
#include <arpa/inet.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <limits.h>
#include <net/if.h>
#include <signal.h>
#include <spawn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "jb_coord_client.hpp"
#include "jb_rpc.hpp"
#include "jubatus_amd/msgpack_rpc.hpp"

extern char** environ;

namespace {

using jb::cc::Coord;
using jb::cc::Value;

const char* kVersion = "1.0.0";

void log_line(const char* level, const std::string& msg) { jb::cc::log_tagged("jubavisor", level, msg); }

const char* const kArgvFields[] = {"port", "bind_address", "bind_if", "timeout", "zookeeper_timeout",
                                   "interconnect_timeout", "threadnum", "program_name", "type", "z",
                                   "name", "datadir", "logdir", "log_config", "eth", "interval_sec",
                                   "interval_count", "mixer", "daemon"};
constexpr int kNumArgvFields = sizeof(kArgvFields) / sizeof(kArgvFields[0]);

struct ArgError : std::runtime_error {
  ArgError() : std::runtime_error("argument error") {}
};

std::string value_text(const Value& v) {
  switch (v.type) {
    case Value::STR: return v.s;
    case Value::INT:
    case Value::UINT: return std::to_string(v.as_int());
    case Value::FLOAT: {
      const double d = v.as_double();
      if (d == (double)(long long)d) return std::to_string((long long)d);
      char b[64];
      snprintf(b, sizeof b, "%g", d);
      return b;
    }
    default: return "";   // nil / bool / containers: not passed on
  }
}

// server_argv (array in MSGPACK_DEFINE order, or a map) -> field -> text
std::map<std::string, std::string> argv_fields(const Value& v) {
  std::map<std::string, std::string> out;
  if (v.type == Value::ARRAY) {
    for (int i = 0; i < kNumArgvFields && i < (int)v.a.size(); ++i) out[kArgvFields[i]] = value_text(v.a[i]);
  } else if (v.type == Value::MAP) {
    for (const auto& kv : v.m)
      if (kv.first.type == Value::STR) out[kv.first.s] = value_text(kv.second);
  } else {
    throw ArgError();
  }
  return out;
}

std::string exe_dir() {
  char buf[PATH_MAX];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p(buf);
  return p.substr(0, p.rfind('/'));
}

// <repo>/jubatus_amd/native_bin[/<sanitizer>]/jubavisor -> <repo>/bin
std::string default_server_dir() {
  const char* env = getenv("JUBAVISOR_SERVER_DIR");
  if (env && *env) return env;
  std::string d = exe_dir();
  for (int up = 0; up < 4; ++up) {
    struct stat st;
    const std::string cand = d + "/bin";
    if (stat((cand + "/jubaclassifier").c_str(), &st) == 0) return cand;
    const size_t s = d.rfind('/');
    if (s == std::string::npos || s == 0) break;
    d = d.substr(0, s);
  }
  return exe_dir();
}

struct Args {
  int gpus = -1;                 // GPUs handed out to children (-1: count the host's)
  int port = 9198;
  std::string zk = "localhost:2181";
  int max_children = 16;
  std::string logdir;
  int timeout = 10;
  std::string listen_addr;
  std::string eth;
  std::string server_dir;
};

struct Child {
  pid_t pid;
  int port;
  int gpu;                       // device index given with --gpu (-1: none)
  std::string server_name;
};

class Visor {
 public:
  explicit Visor(const Args& a) : a_(a), gpu_users_(a.gpus > 0 ? a.gpus : 0, 0) {
    for (int p = a.port + 1; p <= a.port + a.max_children; ++p) pool_.push_back(p);
    reaper_ = std::thread([this] { reap_loop(); });
  }
  ~Visor() {
    stop_.store(true);
    if (reaper_.joinable()) reaper_.join();
  }

  int start(const std::string& server_name, int64_t n, const Value& argv) {
    std::string server, name;
    if (!split(server_name, &server, &name)) {
      log_line("ERROR", "cannot parse " + server_name);
      return -1;
    }
    const auto f = argv_fields(argv);
    std::lock_guard<std::mutex> g(mu_);
    auto& procs = children_[name];
    if ((int64_t)procs.size() > n) {
      log_line("ERROR", std::to_string(procs.size()) + " " + name + " already running at this machine.");
      return -1;
    }
    const int64_t need = n - (int64_t)procs.size();
    if ((int64_t)pool_.size() < need) {
      log_line("ERROR", "cannot spawn more than " + std::to_string(a_.max_children) + " processes.");
      return -1;
    }
    for (int64_t i = 0; i < need; ++i) {
      const int port = pool_.front();
      pool_.pop_front();
      const int gpu = take_gpu();
      const pid_t pid = spawn(server, name, port, gpu, f);
      if (pid <= 0) {
        pool_.push_back(port);
        give_gpu(gpu);
        return -1;
      }
      log_line("INFO", "started " + server_name + " on port " + std::to_string(port) + " (pid " +
                           std::to_string(pid) + (gpu >= 0 ? ", gpu " + std::to_string(gpu) : "") +
                           ")");
      procs.push_back(Child{pid, port, gpu, server_name});
    }
    return 0;
  }

  int stop(const std::string& server_name) {
    std::string server, name;
    if (!split(server_name, &server, &name)) return -1;
    std::vector<Child> procs;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = children_.find(name);
      if (it == children_.end()) return 0;
      procs.swap(it->second);
      children_.erase(it);
    }
    terminate(procs);
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& c : procs) {
      pool_.push_back(c.port);
      give_gpu(c.gpu);
    }
    return 0;
  }

  void stop_all() {
    std::vector<Child> all;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : children_)
        for (auto& c : kv.second) all.push_back(c);
      children_.clear();
    }
    terminate(all);
  }

 private:
  static bool split(const std::string& s, std::string* server, std::string* name) {
    // "jubaclassifier/name" (process.cpp:61-69)
    if (s.find(' ') != std::string::npos) return false;
    const size_t k = s.find('/');
    if (k == std::string::npos) return false;
    *server = s.substr(0, k);
    *name = s.substr(k + 1);
    return server->size() > 4 && server->compare(0, 4, "juba") == 0 && !name->empty() &&
           server->find_first_of("./") == std::string::npos;
  }

  // One server process per GPU: each child gets the least
  // used device of this host (devices are reused round-robin once every one
  // has a server). -1 when the host has no GPU (children run on the host).
  int take_gpu() {
    if (gpu_users_.empty()) return -1;
    int best = 0;
    for (int i = 1; i < (int)gpu_users_.size(); ++i)
      if (gpu_users_[i] < gpu_users_[best]) best = i;
    ++gpu_users_[best];
    return best;
  }
  void give_gpu(int gpu) {
    if (gpu >= 0 && gpu < (int)gpu_users_.size() && gpu_users_[gpu] > 0) --gpu_users_[gpu];
  }

  pid_t spawn(const std::string& server, const std::string& name, int port, int gpu,
              const std::map<std::string, std::string>& f) {
    const std::string prog = a_.server_dir + "/" + server;
    std::vector<std::string> args{prog, "-z", a_.zk, "-n", name, "-p", std::to_string(port)};
    if (gpu >= 0) { args.push_back("--gpu"); args.push_back(std::to_string(gpu)); }
    if (!a_.listen_addr.empty()) { args.push_back("-b"); args.push_back(a_.listen_addr); }
    static const char* const opts[][2] = {
        {"-B", "bind_if"},      {"-c", "threadnum"}, {"-t", "timeout"},
        {"-Z", "zookeeper_timeout"}, {"-I", "interconnect_timeout"}, {"-d", "datadir"},
        {"-l", "logdir"},       {"-g", "log_config"}, {"-s", "interval_sec"},
        {"-i", "interval_count"}, {"-x", "mixer"}};
    for (const auto& o : opts) {
      auto it = f.find(o[1]);
      if (it != f.end() && !it->second.empty()) { args.push_back(o[0]); args.push_back(it->second); }
    }
    std::vector<char*> av;
    for (auto& s : args) av.push_back(const_cast<char*>(s.c_str()));
    av.push_back(nullptr);

    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
    if (!a_.logdir.empty()) {   // with -l the children's output goes to a file (process.cpp:99-100 discards it)
      const std::string out = a_.logdir + "/" + server + "." + name + "." + std::to_string(port) + ".log";
      posix_spawn_file_actions_addopen(&fa, 1, out.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
      posix_spawn_file_actions_adddup2(&fa, 1, 2);
    }
    posix_spawnattr_t at;
    posix_spawnattr_init(&at);
    sigset_t none, dfl;
    sigemptyset(&none);
    sigemptyset(&dfl);
    for (int sg : {SIGTERM, SIGINT, SIGHUP, SIGPIPE}) sigaddset(&dfl, sg);
    posix_spawnattr_setsigmask(&at, &none);      // this process blocks TERM/INT/HUP for sigwait
    posix_spawnattr_setsigdefault(&at, &dfl);    // and ignores SIGPIPE
    posix_spawnattr_setpgroup(&at, 0);
    posix_spawnattr_setflags(&at, POSIX_SPAWN_SETSIGMASK | POSIX_SPAWN_SETSIGDEF | POSIX_SPAWN_SETPGROUP);
    pid_t pid = -1;
    const int rc = posix_spawn(&pid, prog.c_str(), &fa, &at, av.data(), environ);
    posix_spawnattr_destroy(&at);
    posix_spawn_file_actions_destroy(&fa);
    if (rc != 0) {
      log_line("ERROR", "cannot start " + prog + ": " + strerror(rc));
      return -1;
    }
    return pid;
  }

  // SIGTERM each child's process group, wait up to 10 s, then SIGKILL
  // (process.cpp:140-156 waits without a bound)
  void terminate(const std::vector<Child>& procs) {
    for (const auto& c : procs) {
      if (!reaped(c.pid)) ::kill(-c.pid, SIGTERM);
    }
    const double deadline = jb::cc::now_s() + 10.0;
    for (const auto& c : procs) {
      while (!reaped(c.pid)) {
        if (jb::cc::now_s() > deadline) {
          log_line("WARN", "pid " + std::to_string(c.pid) + " ignored SIGTERM: killing");
          ::kill(-c.pid, SIGKILL);
          int st;
          waitpid(c.pid, &st, 0);
          break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
      log_line("INFO", "stopped " + c.server_name + " on port " + std::to_string(c.port));
    }
  }

  // true once the child is gone (reaped here or by the reaper thread)
  static bool reaped(pid_t pid) {
    int st;
    const pid_t r = waitpid(pid, &st, WNOHANG);
    return r == pid || (r < 0 && errno == ECHILD);
  }

  void reap_loop() {
    while (!stop_.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : children_) {
        auto& v = kv.second;
        for (size_t i = 0; i < v.size();) {
          int st;
          if (waitpid(v[i].pid, &st, WNOHANG) == v[i].pid) {
            log_line("INFO", v[i].server_name + " with port " + std::to_string(v[i].port) +
                                 " exited pid: " + std::to_string(v[i].pid));
            pool_.push_back(v[i].port);
            give_gpu(v[i].gpu);
            v.erase(v.begin() + i);
          } else {
            ++i;
          }
        }
      }
    }
  }

  Args a_;
  std::mutex mu_;
  std::map<std::string, std::vector<Child>> children_;
  std::deque<int> pool_;
  std::vector<int> gpu_users_;   // children per device
  std::atomic<bool> stop_{false};
  std::thread reaper_;
};

std::string response(uint32_t msgid, const Value& err, const Value& result) {
  std::string o;
  jubatus_amd::mp::encode(Value::array({Value::uinteger(1), Value::uinteger(msgid), err, result}), o);
  return o;
}

std::string handle(Visor& v, const jb::RpcRequest& r) {
  Value err, result;
  try {
    Value params;
    jubatus_amd::mp::Decoder dec(r.params.data(), r.params.size());
    if (!dec.next(params) || params.type != Value::ARRAY) throw ArgError();
    const auto& a = params.a;
    auto str0 = [&]() -> const std::string& {
      if (a.empty() || a[0].type != Value::STR) throw ArgError();
      return a[0].s;
    };
    auto int1 = [&]() -> int64_t {
      if (a.size() < 2 || (a[1].type != Value::INT && a[1].type != Value::UINT)) throw ArgError();
      return a[1].as_int();
    };
    if (r.method == "start") {
      if (a.size() != 3) throw ArgError();
      result = Value::integer(v.start(str0(), int1(), a[2]));
    } else if (r.method == "stop") {
      if (a.size() != 2) throw ArgError();
      int1();
      result = Value::integer(v.stop(str0()));
    } else {
      err = Value::uinteger(1);   // NO_METHOD_ERROR
    }
  } catch (const ArgError&) {
    err = Value::uinteger(2);     // ARGUMENT_ERROR
  } catch (const std::exception& e) {
    err = Value::str(e.what());
  }
  if (r.notify) return std::string();
  return response(r.msgid, err, result);
}

void usage() {
  fprintf(stderr,
          "usage: jubavisor [options]\n"
          "  -p, --rpc-port PORT       port number (9198); children use PORT+1 .. PORT+max\n"
          "  -z, --zookeeper HOSTS     coordinator location (localhost:2181)\n"
          "  -m, --max-children N      maximum number of children (16)\n"
          "  -l, --logdir DIR          directory for the children's output\n"
          "  -t, --timeout SEC         coordinator session timeout (10)\n"
          "  -b, --listen_addr ADDR    address to bind, register and give the children\n"
          "  -G, --gpus N              GPUs to hand out, one per child (--gpu i); default:\n"
          "                            the host's GPU count (0: children get no --gpu)\n"
          "  -v, --version\n");
}

int parse_args(int argc, char** argv, Args* a) {
  for (int i = 1; i < argc; ++i) {
    const std::string s = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error(s + " needs a value");
      return argv[++i];
    };
    auto num = [&](int lo) -> int {
      const std::string v = val();
      char* end = nullptr;
      const long x = strtol(v.c_str(), &end, 10);
      if (!end || *end || x < lo) throw std::runtime_error("bad value for " + s + ": " + v);
      return (int)x;
    };
    if (s == "-p" || s == "--rpc-port") a->port = num(1);
    else if (s == "-z" || s == "--zookeeper") a->zk = val();
    else if (s == "-m" || s == "--max-children") a->max_children = num(1);
    else if (s == "-l" || s == "--logdir") a->logdir = val();
    else if (s == "-t" || s == "--timeout") a->timeout = num(1);
    else if (s == "-b" || s == "--listen_addr") a->listen_addr = val();
    else if (s == "-G" || s == "--gpus") a->gpus = num(0);
    else if (s == "-v" || s == "--version") { printf("jubatus-%s (mi355x, native jubavisor)\n", kVersion); return -1; }
    else if (s == "-h" || s == "--help") { usage(); return -1; }
    else { fprintf(stderr, "unknown option: %s\n", s.c_str()); usage(); return 1; }
  }
  if (!a->logdir.empty() && access(a->logdir.c_str(), W_OK) != 0) {
    fprintf(stderr, "can't write to the log directory %s\n", a->logdir.c_str());
    return 1;
  }
  return 0;
}

// GPUs of this host: KFD topology nodes with SIMDs (no HIP runtime needed)
int count_gpus() {
  int n = 0;
  for (int i = 0; i < 256; ++i) {
    const std::string path = "/sys/class/kfd/kfd/topology/nodes/" + std::to_string(i) + "/properties";
    FILE* fp = fopen(path.c_str(), "r");
    if (!fp) break;
    char key[128];
    long long v;
    while (fscanf(fp, "%127s %lld", key, &v) == 2) {
      if (strcmp(key, "simd_count") == 0) {
        if (v > 0) ++n;
        break;
      }
    }
    fclose(fp);
  }
  return n;
}

std::string default_v4() {
  // first non-loopback IPv4 (network.cpp get_default_v4_address)
  ifaddrs* ifs = nullptr;
  std::string out = "127.0.0.1";
  if (getifaddrs(&ifs) != 0) return out;
  for (ifaddrs* i = ifs; i; i = i->ifa_next) {
    if (!i->ifa_addr || i->ifa_addr->sa_family != AF_INET || (i->ifa_flags & IFF_LOOPBACK)) continue;
    char buf[INET_ADDRSTRLEN];
    inet_ntop(AF_INET, &((sockaddr_in*)i->ifa_addr)->sin_addr, buf, sizeof buf);
    out = buf;
    break;
  }
  freeifaddrs(ifs);
  return out;
}

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
  a.server_dir = default_server_dir();
  if (a.gpus < 0) a.gpus = count_gpus();
  a.eth = a.listen_addr.empty() ? default_v4() : a.listen_addr;

  sigset_t ss;
  sigemptyset(&ss);
  sigaddset(&ss, SIGTERM);
  sigaddset(&ss, SIGINT);
  sigaddset(&ss, SIGHUP);
  pthread_sigmask(SIG_BLOCK, &ss, nullptr);
  signal(SIGPIPE, SIG_IGN);

  std::unique_ptr<Coord> coord;
  try {
    coord.reset(new Coord(a.zk, a.timeout, "jubavisor"));
  } catch (const std::exception& e) {
    log_line("FATAL", e.what());
    return 1;
  }
  Visor visor(a);
  jb::RpcServer srv([&visor](const jb::RpcRequest& r) { return handle(visor, r); }, 2, 0.0);
  int bound;
  try {
    bound = srv.listen(a.listen_addr.empty() ? "0.0.0.0" : a.listen_addr, a.port);
  } catch (const std::exception& e) {
    log_line("FATAL", std::string("listen failed: ") + e.what());
    return 1;
  }
  srv.start();
  // register_supervisor (jubavisor.cpp:70-76): base paths, then the
  // ephemeral /jubatus/supervisors/<ip>_<port>
  coord->create("/jubatus", "", false);
  coord->create("/jubatus/supervisors", "", false);
  coord->create("/jubatus/actors", "", false);
  if (!coord->create("/jubatus/supervisors/" + a.eth + "_" + std::to_string(bound), "", true)) {
    log_line("FATAL", "Failed to register_supervisor");
    srv.stop();
    return 1;
  }
  log_line("INFO", "jubavisor (native) listening at " + a.eth + ":" + std::to_string(bound) +
                       ", servers from " + a.server_dir);
  printf("jubavisor ready %d\n", bound);
  fflush(stdout);
  for (;;) {
    int sig = 0;
    sigwait(&ss, &sig);
    if (sig == SIGHUP) continue;
    log_line("INFO", "stopping on signal " + std::to_string(sig));
    break;
  }
  srv.stop();
  visor.stop_all();
  coord->close();
  return 0;
}
