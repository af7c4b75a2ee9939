// Shared pieces of the native operator tools (jubactl, jubaconfig): a
// coordinator session with uncached list / read (a tool acts on what is there
// now, not on a polled cache), the coordinator tree layout, the zkmutex
// write lock over config_lock, and the reference's flag parsing style.
//
// Reference: jubatus/server/common/membership.cpp:40-47,287-312 (paths,
// prepare_jubatus), common/zk.cpp:530-631 (zkmutex), common/config.cpp
// (config_tozk / remove_config_fromzk). The Python twins are
// jubatus_amd/common/{membership,config,lock_service}.py; both write the same
// nodes, so either tool works against servers of either runtime.
#pragma once

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "jb_coord_client.hpp"

namespace jb {
namespace cmd {

using jubatus_amd::mp::Value;

const char* const kJubatusBase = "/jubatus";
const char* const kVisorBase = "/jubatus/supervisors";
const char* const kProxyBase = "/jubatus/jubaproxies";
const char* const kActorBase = "/jubatus/actors";
const char* const kConfigBase = "/jubatus/config";

inline std::string actor_path(const std::string& type, const std::string& name) {
  return std::string(kActorBase) + "/" + type + "/" + name;
}
inline std::string config_path(const std::string& type, const std::string& name) {
  return std::string(kConfigBase) + "/" + type + "/" + name;
}

// "127.0.0.1_9199[_i]" -> host, port
inline bool revert(const std::string& loc, std::string* host, int* port) {
  const size_t u = loc.find('_');
  if (u == std::string::npos) return false;
  *host = loc.substr(0, u);
  *port = atoi(loc.c_str() + u + 1);
  return *port > 0;
}

// the coordinator location from -z or $ZK
inline std::string zk_location(const std::string& flag) {
  if (!flag.empty()) return flag;
  const char* e = getenv("ZK");
  return e ? std::string(e) : std::string();
}

class Zk {
 public:
  explicit Zk(const std::string& hosts, double timeout = 10.0) : c_(hosts, timeout, "zk") {}

  std::vector<std::string> list(const std::string& path) {
    Value r = c_.call("list", {Value::str(path)});
    std::vector<std::string> out;
    if (r.as_array().at(0).as_int() == 0)
      for (const auto& x : r.as_array().at(1).as_array()) out.push_back(x.as_str());
    std::sort(out.begin(), out.end());
    return out;
  }
  bool read(const std::string& path, std::string* data) {
    Value r = c_.call("read", {Value::str(path)});
    if (r.as_array().at(0).as_int() != 0) return false;
    *data = r.as_array().at(1).as_str();
    return true;
  }
  bool exists(const std::string& path) { return c_.exists(path); }
  // persistent node (true when created or already there)
  bool create(const std::string& path, const std::string& data = "") { return c_.create(path, data, false); }
  bool set(const std::string& path, const std::string& data) {
    return c_.call("set", {Value::str(path), Value::str(data)}).as_array().at(0).as_int() == 0;
  }
  bool remove(const std::string& path) { return c_.call("remove", {Value::str(path)}).as_int() == 0; }
  // ephemeral sequential node under dir with the prefix ("" on failure)
  std::string create_seq(const std::string& prefix) {
    Value r = c_.call("create_seq", {Value::integer(c_.session()), Value::str(prefix)});
    const auto& a = r.as_array();
    return a.at(0).as_int() == 0 ? a.at(1).as_str() : std::string();
  }

  // membership.cpp prepare_jubatus: the base tree (+ the actor's subtree)
  void prepare(const std::string& type, const std::string& name) {
    for (const std::string& p : {std::string(kJubatusBase), std::string(kVisorBase), std::string(kProxyBase),
                                 std::string(kActorBase), std::string(kConfigBase),
                                 std::string(kActorBase) + "/" + type, std::string(kConfigBase) + "/" + type,
                                 std::string(kProxyBase) + "/" + type})
      if (!create(p)) throw std::runtime_error("failed to prepare coordinator tree: " + p);
    if (name.empty()) return;
    const std::string base = actor_path(type, name);
    for (const char* s : {"", "/nodes", "/actives", "/master_lock", "/config_lock", "/id_generator", "/mix"})
      create(base + s);
  }

 private:
  cc::Coord c_;
};

// zkmutex write lock (the lowest sequence number under the lock node wins),
// tried `retry` times with a growing pause like the Python twin
class WriteLock {
 public:
  WriteLock(Zk& zk, const std::string& dir) : zk_(zk), dir_(dir) { zk_.create(dir_); }
  ~WriteLock() { unlock(); }
  bool try_lock(int retry = 3) {
    for (int i = 0; i < std::max(1, retry); ++i) {
      const std::string seq = zk_.create_seq(dir_ + "/wlock_");
      if (!seq.empty()) {
        const std::string me = seq.substr(seq.rfind('/') + 1);
        std::string low;
        int64_t lown = INT64_MAX;
        for (const auto& c : zk_.list(dir_)) {
          if (c.size() < 10) continue;
          const int64_t n = atoll(c.c_str() + c.size() - 10);
          if (n < lown) { lown = n; low = c; }
        }
        if (low == me) { held_ = seq; return true; }
        zk_.remove(seq);
      }
      usleep(100000 * (i + 1));
    }
    return false;
  }
  void unlock() {
    if (!held_.empty()) zk_.remove(held_);
    held_.clear();
  }

 private:
  Zk& zk_;
  std::string dir_;
  std::string held_;
};

// "-x value" / "--long value" / "--long=value" and boolean flags, the
// reference's cmdline style (its tools use cmdline::parser)
class Flags {
 public:
  struct Spec {
    char shortf;
    std::string longf;
    bool boolean;
    std::string dflt;
    std::string help;
  };
  explicit Flags(const std::string& prog) : prog_(prog) {}
  void add(char s, const std::string& l, const std::string& dflt, const std::string& help) {
    specs_.push_back({s, l, false, dflt, help});
    vals_[l] = dflt;
  }
  void flag(char s, const std::string& l, const std::string& help) {
    specs_.push_back({s, l, true, "", help});
    vals_[l] = "";
  }
  // false: print the usage (error or --help) and exit with the returned code
  bool parse(int argc, char** argv, int* code) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a == "-h" || a == "--help") { usage(stdout); *code = 0; return false; }
      const Spec* sp = nullptr;
      std::string val;
      bool have = false;
      for (const auto& s : specs_) {
        if (a.size() == 2 && a[0] == '-' && a[1] == s.shortf) sp = &s;
        else if (a == "--" + s.longf) sp = &s;
        else if (a.rfind("--" + s.longf + "=", 0) == 0) {
          sp = &s;
          val = a.substr(s.longf.size() + 3);
          have = true;
        }
        if (sp) break;
      }
      if (!sp) { fprintf(stderr, "unknown option: %s\n", a.c_str()); usage(stderr); *code = 1; return false; }
      if (sp->boolean) { vals_[sp->longf] = "1"; continue; }
      if (!have) {
        if (i + 1 >= argc) {
          fprintf(stderr, "option needs value: --%s\n", sp->longf.c_str());
          usage(stderr);
          *code = 1;
          return false;
        }
        val = argv[++i];
      }
      vals_[sp->longf] = val;
    }
    return true;
  }
  const std::string& get(const std::string& l) const { return vals_.at(l); }
  int num(const std::string& l) const { return atoi(vals_.at(l).c_str()); }
  bool on(const std::string& l) const { return !vals_.at(l).empty(); }
  void usage(FILE* f) const {
    fprintf(f, "usage: %s [options] ...\noptions:\n", prog_.c_str());
    for (const auto& s : specs_) {
      std::string left = std::string("  -") + s.shortf + ", --" + s.longf;
      if (!s.boolean) left += " VALUE";
      fprintf(f, "%-34s %s", left.c_str(), s.help.c_str());
      if (!s.boolean && !s.dflt.empty()) fprintf(f, " (default: %s)", s.dflt.c_str());
      fprintf(f, "\n");
    }
    fprintf(f, "  -h, --help                         print this message\n");
  }

 private:
  std::string prog_;
  std::vector<Spec> specs_;
  std::map<std::string, std::string> vals_;
};

}  // namespace cmd
}  // namespace jb
