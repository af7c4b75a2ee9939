// jubactl: cluster control, native (reference C32,
// jubatus/server/cmd/jubactl.cpp:56-315).
//
// -c start|stop: fan out to every jubavisor registered in the coordinator,
// N processes spread as N / |visors| (+1 on the first N % |visors|); N = 0
// means one per visor. start creates the actor node first and hands every
// supervisor the server argv (server_util.hpp:91-94 MSGPACK_DEFINE order).
// -c save|load: call every node of the cluster directly (id defaults to the
// cluster name). -c status: list the proxies, supervisors and nodes.
// The coordinator comes from -z or $ZK. Output lines match the Python twin
// (jubatus_amd/cmd/jubactl.py), which stays as the library the tests and
// scripts import.
#include <stdio.h>

#include <string>
#include <vector>

#include "jb_cmd.hpp"
#include "jubatus_amd/msgpack_rpc.hpp"

namespace {

using jb::cmd::Value;

constexpr double kVisorCallTimeout = 30.0;

std::vector<int> split_counts(int n, int nvisors) {
  if (n == 0) n = nvisors;
  std::vector<int> out;
  for (int i = 0; i < nvisors; ++i) out.push_back(n / nvisors + (i < n % nvisors ? 1 : 0));
  return out;
}

// [port, bind_address, bind_if, timeout, zookeeper_timeout,
//  interconnect_timeout, threadnum, program_name, type, z, name, datadir,
//  logdir, log_config, eth, interval_sec, interval_count, mixer, daemon]
Value server_argv(const jb::cmd::Flags& f, const std::string& zk, const std::string& full_name) {
  auto I = [&](const char* k) { return Value::integer(f.num(k)); };
  auto S = [&](const char* k) { return Value::str(f.get(k)); };
  return Value::array({Value::integer(0), Value::str(""), S("listen_if"), I("timeout"), I("zookeeper_timeout"),
                       I("interconnect_timeout"), I("thread"), S("type"), S("type"), Value::str(zk),
                       Value::str(full_name), S("datadir"), S("logdir"), S("log_config"), Value::str(""),
                       I("interval_sec"), I("interval_count"), S("mixer"), Value::boolean(false)});
}

int send2supervisor(jb::cmd::Zk& zk, const jb::cmd::Flags& f, const std::string& zkloc) {
  const std::string cmd = f.get("cmd");
  const std::string name = f.get("server") + "/" + f.get("name");
  Value argv;
  if (cmd == "start") {
    zk.create(jb::cmd::actor_path(f.get("type"), f.get("name")));
    zk.create(jb::cmd::actor_path(f.get("type"), f.get("name")) + "/nodes");
    argv = server_argv(f, zkloc, name);
  }
  const std::vector<std::string> visors = zk.list(jb::cmd::kVisorBase);
  if (visors.empty()) {
    printf("no server to %s %s\n", cmd.c_str(), name.c_str());
    return -1;
  }
  const std::vector<int> counts = split_counts(f.num("num"), (int)visors.size());
  int rc = 0;
  for (size_t i = 0; i < visors.size(); ++i) {
    std::string host;
    int port;
    printf("sending %s / %s to %s...", cmd.c_str(), name.c_str(), visors[i].c_str());
    fflush(stdout);
    if (!jb::cmd::revert(visors[i], &host, &port)) { printf("failed (bad location).\n"); rc = -1; continue; }
    int64_t r;
    try {
      // a supervisor's stop waits up to 10 s for each child before SIGKILL
      // (csrc/visor/jubavisor.cpp terminate): the call gets more than that
      jubatus_amd::RpcClient c(host, port, kVisorCallTimeout);
      std::vector<Value> params{Value::str(name), Value::integer(counts[i])};
      if (cmd == "start") params.push_back(argv);
      r = c.call_values(cmd, params).as_int();
    } catch (const std::exception& e) {
      printf("failed (%s).\n", e.what());
      rc = -1;
      continue;
    }
    printf(r == 0 ? "ok.\n" : "failed.\n");
    if (r != 0) rc = (int)r;
  }
  return rc;
}

int send2server(jb::cmd::Zk& zk, const jb::cmd::Flags& f) {
  const std::string cmd = f.get("cmd"), name = f.get("name");
  const std::string id = f.get("id").empty() ? name : f.get("id");
  const std::vector<std::string> nodes = zk.list(jb::cmd::actor_path(f.get("type"), name) + "/nodes");
  if (nodes.empty()) printf("no server to %s %s\n", cmd.c_str(), name.c_str());
  int rc = 0;
  for (const auto& loc : nodes) {
    std::string host;
    int port;
    printf("sending %s / %s to %s...", cmd.c_str(), name.c_str(), loc.c_str());
    fflush(stdout);
    try {
      if (!jb::cmd::revert(loc, &host, &port)) throw std::runtime_error("bad location");
      jubatus_amd::RpcClient c(host, port, 10.0);
      c.call_values(cmd, {Value::str(name), Value::str(id)});
      printf("ok.\n");
    } catch (const std::exception&) {
      printf("failed.\n");
      rc = -1;
    }
  }
  return rc;
}

void status(jb::cmd::Zk& zk, const jb::cmd::Flags& f) {
  const std::string type = f.get("type"), name = f.get("name");
  const std::pair<std::string, std::string> groups[] = {
      {std::string(jb::cmd::kProxyBase) + "/" + type, "jubaproxy"},
      {jb::cmd::kVisorBase, "jubavisor"},
      {jb::cmd::actor_path(type, name) + "/nodes", name}};
  for (const auto& g : groups) {
    printf("\033[34mactive %s members:\033[0m\n", g.second.c_str());
    for (const auto& m : zk.list(g.first)) printf("%s\n", m.c_str());
  }
}

}  // namespace

int main(int argc, char** argv) {
  jb::cmd::Flags f("jubactl");
  f.add('c', "cmd", "", "command: start|stop|save|load|status");
  f.add('s', "server", "", "server exec name (jubaclassifier, ...)");
  f.add('n', "name", "", "cluster name");
  f.add('t', "type", "", "engine type (classifier, ...)");
  f.add('N', "num", "0", "number of processes (0: one per supervisor)");
  f.add('z', "zookeeper", "", "coordinator hosts (host:port[,...]; default $ZK)");
  f.add('i', "id", "", "model id of save / load (default: the cluster name)");
  f.add('B', "listen_if", "", "network interface the servers listen on");
  f.add('C', "thread", "2", "server RPC threads");
  f.add('T', "timeout", "10", "server RPC timeout (sec)");
  f.add('D', "datadir", "/tmp", "server model directory");
  f.add('L', "logdir", "", "server log directory");
  f.add('G', "log_config", "", "server log configuration");
  f.add('X', "mixer", "linear_mixer", "mixer strategy");
  f.add('S', "interval_sec", "16", "mix interval by seconds");
  f.add('I', "interval_count", "512", "mix interval by update count");
  f.add('Z', "zookeeper_timeout", "10", "coordinator session timeout (sec)");
  f.add('R', "interconnect_timeout", "10", "server-to-server timeout (sec)");
  f.flag('d', "debug", "debug mode");
  int code = 0;
  if (!f.parse(argc, argv, &code)) return code;
  const std::string cmd = f.get("cmd");
  if (cmd != "start" && cmd != "stop" && cmd != "save" && cmd != "load" && cmd != "status") {
    fprintf(stderr, "-c must be one of start, stop, save, load, status\n");
    f.usage(stderr);
    return 1;
  }
  for (const char* k : {"server", "name", "type"})
    if (f.get(k).empty()) {
      fprintf(stderr, "--%s is required\n", k);
      f.usage(stderr);
      return 1;
    }
  const std::string zkloc = jb::cmd::zk_location(f.get("zookeeper"));
  if (zkloc.empty()) {
    printf("can't get ZK location: set 'ZK' environment or specify '-z <somezkaddrs>'\n");
    return 1;
  }
  try {
    jb::cmd::Zk zk(zkloc, 10.0);
    if (cmd == "status") {
      status(zk, f);
      return 0;
    }
    if (cmd == "start" || cmd == "stop") return send2supervisor(zk, f, zkloc) == 0 ? 0 : 1;
    return send2server(zk, f) == 0 ? 0 : 1;
  } catch (const std::exception& e) {
    fprintf(stderr, "jubactl: %s\n", e.what());
    return 1;
  }
}
