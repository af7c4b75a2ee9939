// Coordinator node tree (ZooKeeper data model, the subset Jubatus uses).
//
// Reference: the lock_service API (jubatus/server/common/lock_service.hpp:34-119)
// implemented on ZooKeeper 3.4 by zk.cpp (create :145-177, create_seq
// :200-216, create_id :218-232, list/read, ephemeral cleanup via the session
// watcher :641-686). Semantics kept (see also jubatus_amd/common/lock_service.py,
// the Python twin used for in-process / single-node runs):
//   * create needs the parent; creating an existing node returns NODEEXISTS
//     (the client treats that as success for persistent nodes);
//   * ephemeral nodes belong to a session and vanish when it closes or its
//     heartbeat is older than its timeout; ephemerals cannot have children;
//   * create_seq appends the parent's 10-digit child counter;
//   * set bumps the data version (create_id = (prefix << 32) | version);
//   * mzxid / pzxid change on data / child changes: the client-side watch
//     poller compares them (stat_many) to fire one-shot watches.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

namespace jb {
namespace coord {

enum Rc : int {
  OK = 0, NONODE = -101, NODEEXISTS = -110, NOTEMPTY = -111, NOCHILDREN_FOR_EPHEMERALS = -108,
  BADARGS = -8, SESSION_EXPIRED = -112,
};

struct Node {
  std::string data;
  int64_t owner = 0;      // ephemeral owner session, 0 = persistent
  int64_t version = 0;    // data version
  int64_t cversion = 0;   // child version (sequence counter)
  int64_t mzxid = 0;
  int64_t pzxid = 0;
  std::set<std::string> children;
};

inline std::string parent_of(const std::string& path) {
  std::string p = path;
  while (p.size() > 1 && p.back() == '/') p.pop_back();
  const size_t k = p.rfind('/');
  if (k == std::string::npos || k == 0) return "/";
  return p.substr(0, k);
}

inline std::string base_of(const std::string& path) {
  const size_t k = path.rfind('/');
  return k == std::string::npos ? path : path.substr(k + 1);
}

inline bool valid_path(const std::string& p) {
  if (p.empty() || p[0] != '/') return false;
  if (p != "/" && p.back() == '/') return false;
  return p.find("//") == std::string::npos;
}

class ZNodeStore {
 public:
  using Clock = std::chrono::steady_clock;

  ZNodeStore() { nodes_["/"] = Node(); }

  // ---- sessions
  int64_t open_session(double timeout_sec) {
    std::lock_guard<std::mutex> g(mu_);
    const int64_t sid = next_sid_++;
    sessions_[sid] = {timeout_sec, Clock::now()};
    return sid;
  }
  bool heartbeat(int64_t sid) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = sessions_.find(sid);
    if (it == sessions_.end()) return false;
    it->second.second = Clock::now();
    return true;
  }
  void close_session(int64_t sid) {
    std::lock_guard<std::mutex> g(mu_);
    close_locked(sid);
  }
  std::vector<int64_t> expire_sessions() {
    std::lock_guard<std::mutex> g(mu_);
    const auto now = Clock::now();
    std::vector<int64_t> dead;
    for (const auto& kv : sessions_) {
      const double age = std::chrono::duration<double>(now - kv.second.second).count();
      if (age > kv.second.first) dead.push_back(kv.first);
    }
    for (int64_t sid : dead) close_locked(sid);
    return dead;
  }
  size_t nsessions() {
    std::lock_guard<std::mutex> g(mu_);
    return sessions_.size();
  }

  // ---- nodes
  int create(int64_t sid, const std::string& path, const std::string& data, bool ephemeral) {
    std::lock_guard<std::mutex> g(mu_);
    return create_locked(sid, path, data, ephemeral);
  }
  std::pair<int, std::string> create_seq(int64_t sid, const std::string& path,
                                         const std::string& data, bool ephemeral) {
    std::lock_guard<std::mutex> g(mu_);
    auto par = nodes_.find(parent_of(path));
    if (par == nodes_.end()) return {NONODE, ""};
    char suffix[32];
    std::snprintf(suffix, sizeof suffix, "%010lld", (long long)par->second.cversion);
    const std::string actual = path + suffix;
    return {create_locked(sid, actual, data, ephemeral), actual};
  }
  std::pair<int, int64_t> set(const std::string& path, const std::string& data) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = nodes_.find(path);
    if (it == nodes_.end()) return {NONODE, -1};
    it->second.data = data;
    it->second.version += 1;
    it->second.mzxid = ++zxid_;
    return {OK, it->second.version};
  }
  int remove(const std::string& path) {
    std::lock_guard<std::mutex> g(mu_);
    if (path == "/") return BADARGS;
    return remove_locked(path, false);
  }
  bool exists(const std::string& path) {
    std::lock_guard<std::mutex> g(mu_);
    return nodes_.count(path) != 0;
  }
  std::pair<int, std::vector<std::string>> list(const std::string& path) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = nodes_.find(path);
    if (it == nodes_.end()) return {NONODE, {}};
    return {OK, std::vector<std::string>(it->second.children.begin(), it->second.children.end())};
  }
  std::tuple<int, std::string, int64_t> read(const std::string& path) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = nodes_.find(path);
    if (it == nodes_.end()) return std::make_tuple((int)NONODE, std::string(), (int64_t)-1);
    return std::make_tuple((int)OK, it->second.data, it->second.version);
  }
  // (exists, mzxid, pzxid) per path: the watch poller's input
  std::vector<std::tuple<bool, int64_t, int64_t>> stat_many(const std::vector<std::string>& ps) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::tuple<bool, int64_t, int64_t>> out;
    out.reserve(ps.size());
    for (const auto& p : ps) {
      auto it = nodes_.find(p);
      if (it == nodes_.end()) out.emplace_back(false, 0, 0);
      else out.emplace_back(true, it->second.mzxid, it->second.pzxid);
    }
    return out;
  }
  std::vector<std::pair<std::string, std::string>> dump() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<std::string, std::string>> out;
    for (const auto& kv : nodes_) out.emplace_back(kv.first, kv.second.data);
    return out;
  }

 private:
  int create_locked(int64_t sid, const std::string& path, const std::string& data,
                    bool ephemeral) {
    if (!valid_path(path) || path == "/") return BADARGS;
    if (ephemeral && !sessions_.count(sid)) return SESSION_EXPIRED;
    if (nodes_.count(path)) return NODEEXISTS;
    auto par = nodes_.find(parent_of(path));
    if (par == nodes_.end()) return NONODE;
    if (par->second.owner) return NOCHILDREN_FOR_EPHEMERALS;
    const int64_t z = ++zxid_;
    Node n;
    n.data = data;
    n.owner = ephemeral ? sid : 0;
    n.mzxid = z;
    n.pzxid = z;
    par->second.children.insert(base_of(path));
    par->second.cversion += 1;
    par->second.pzxid = z;
    nodes_.emplace(path, std::move(n));
    return OK;
  }

  int remove_locked(const std::string& path, bool force) {
    auto it = nodes_.find(path);
    if (it == nodes_.end()) return NONODE;
    if (!it->second.children.empty() && !force) return NOTEMPTY;
    const std::vector<std::string> kids(it->second.children.begin(), it->second.children.end());
    for (const auto& c : kids) remove_locked(path == "/" ? "/" + c : path + "/" + c, true);
    nodes_.erase(path);
    auto par = nodes_.find(parent_of(path));
    if (par != nodes_.end()) {
      par->second.children.erase(base_of(path));
      par->second.cversion += 1;
      par->second.pzxid = ++zxid_;
    }
    return OK;
  }

  void close_locked(int64_t sid) {
    sessions_.erase(sid);
    std::vector<std::string> mine;
    for (const auto& kv : nodes_)
      if (kv.second.owner == sid) mine.push_back(kv.first);
    // deepest first (ephemerals have no children, but keep the order safe)
    std::sort(mine.begin(), mine.end(),
              [](const std::string& a, const std::string& b) { return a.size() > b.size(); });
    for (const auto& p : mine) remove_locked(p, true);
  }

  std::mutex mu_;
  std::map<std::string, Node> nodes_;
  std::map<int64_t, std::pair<double, Clock::time_point>> sessions_;
  int64_t next_sid_ = 1;
  int64_t zxid_ = 0;
};

}  // namespace coord
}  // namespace jb
