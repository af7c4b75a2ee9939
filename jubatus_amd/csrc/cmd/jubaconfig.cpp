// jubaconfig: engine configs in the coordinator, native (reference C33,
// jubatus/server/cmd/jubaconfig.cpp:63-226; common/config.cpp).
//
// -c write -f FILE -t TYPE -n NAME: the file must be valid JSON; takes the
// config_lock write lock (3 tries) and refuses while any server of the
// cluster is registered, then writes /jubatus/config/<type>/<name>.
// -c read / -c delete (delete: same lock and refusal). -c list: every
// /jubatus/config/<type>/<name> with its text. Coordinator from -z or $ZK.
// Output matches the Python twin (jubatus_amd/cmd/jubaconfig.py).
#include <stdio.h>

#include <fstream>
#include <sstream>
#include <string>

#include "jb_cmd.hpp"
#include "jb_value.hpp"

namespace {

using jb::cmd::Zk;

struct ConfigError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

std::string lock_dir(const std::string& type, const std::string& name) {
  return jb::cmd::actor_path(type, name) + "/config_lock";
}

void no_server_running(Zk& zk, const std::string& type, const std::string& name) {
  if (!zk.list(jb::cmd::actor_path(type, name) + "/nodes").empty()) throw ConfigError("any server is running");
}

void config_tozk(Zk& zk, const std::string& type, const std::string& name, const std::string& text) {
  try {
    jb::val::parse_json(text);
  } catch (const std::exception& e) {
    throw ConfigError(std::string("invalid config json: ") + e.what());
  }
  zk.prepare(type, name);
  jb::cmd::WriteLock m(zk, lock_dir(type, name));
  if (!m.try_lock(3)) throw ConfigError("any server is running: cannot lock config_lock");
  no_server_running(zk, type, name);
  const std::string path = jb::cmd::config_path(type, name);
  if (!(zk.create(path, text) && zk.set(path, text))) throw ConfigError("failed to write config: " + path);
}

std::string config_fromzk(Zk& zk, const std::string& type, const std::string& name) {
  std::string data;
  if (!zk.read(jb::cmd::config_path(type, name), &data))
    throw ConfigError("config is not found: " + jb::cmd::config_path(type, name));
  return data;
}

void remove_config(Zk& zk, const std::string& type, const std::string& name) {
  jb::cmd::WriteLock m(zk, lock_dir(type, name));
  if (!m.try_lock(3)) throw ConfigError("any server is running: cannot lock config_lock");
  no_server_running(zk, type, name);
  const std::string path = jb::cmd::config_path(type, name);
  if (!zk.exists(path)) throw ConfigError("config is not found: " + path);
  zk.remove(path);
}

}  // namespace

int main(int argc, char** argv) {
  jb::cmd::Flags f("jubaconfig");
  f.add('c', "cmd", "", "command: write|read|delete|list");
  f.add('f', "file", "", "config file to write");
  f.add('t', "type", "", "engine type (classifier, ...)");
  f.add('n', "name", "", "cluster name");
  f.add('z', "zookeeper", "", "coordinator hosts (host:port[,...]; default $ZK)");
  f.flag('d', "debug", "debug mode");
  int code = 0;
  if (!f.parse(argc, argv, &code)) return code;
  const std::string cmd = f.get("cmd"), type = f.get("type"), name = f.get("name");
  if (cmd != "write" && cmd != "read" && cmd != "delete" && cmd != "list") {
    fprintf(stderr, "-c must be one of write, read, delete, list\n");
    f.usage(stderr);
    return 1;
  }
  const std::string zkloc = jb::cmd::zk_location(f.get("zookeeper"));
  if (zkloc.empty()) {
    printf("can't get ZK location: set 'ZK' environment or specify '-z <somezkaddrs>'\n");
    return 1;
  }
  if (cmd != "list" && (type.empty() || name.empty())) {
    printf("type (-t) and name (-n) are required\n");
    return 1;
  }
  try {
    Zk zk(zkloc, 10.0);
    if (cmd == "write") {
      if (f.get("file").empty()) {
        printf("config file (-f) is required\n");
        return 1;
      }
      std::ifstream in(f.get("file"), std::ios::binary);
      if (!in) throw ConfigError("cannot open " + f.get("file"));
      std::stringstream ss;
      ss << in.rdbuf();
      config_tozk(zk, type, name, ss.str());
    } else if (cmd == "read") {
      printf("%s\n", config_fromzk(zk, type, name).c_str());
    } else if (cmd == "delete") {
      remove_config(zk, type, name);
    } else {
      for (const auto& t : zk.list(jb::cmd::kConfigBase))
        for (const auto& n : zk.list(std::string(jb::cmd::kConfigBase) + "/" + t)) {
          printf("config of %s/%s:\n", t.c_str(), n.c_str());
          printf("%s\n", config_fromzk(zk, t, n).c_str());
        }
    }
    return 0;
  } catch (const ConfigError& e) {
    printf("error: %s\n", e.what());
    return 1;
  } catch (const std::exception& e) {
    printf("error: %s\n", e.what());
    return 1;
  }
}
