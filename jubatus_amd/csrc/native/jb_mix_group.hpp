// Native model plane of the distributed servers: the group of servers that
// mix together, its control plane, and the linear mixer loop.
//
// Reference: jubatus/server/framework/mixer/linear_mixer.cpp:358-544 (the
// stabilizer thread: counter / tick trigger, master lock, get_diff / put_diff
// over msgpack-RPC to every node), :394-410,582-611 (obsolete protocol),
// server_util.cpp:184-194 (interconnect timeout). The Python twin of this
// file is jubatus_amd/parallel/{group,linear_mixer}.py - same coordinator
// layout and epoch protocol, so either runtime reads the other's state.
//
// MI355X design (not a translation of the RPC fan-out): every server is one
// rank of a group formed per membership *epoch*:
//
//   <actor>/mix_epoch = {"epoch": e, "members": [ident...], "addr": a, "port": p}
//
// published by the leader (smallest live ident) whenever the live nodes/ set
// changes. (addr, port) is the leader's control-plane listener: the members
// connect to it and the group talks over a TCP star (Star below: small
// metadata - trigger flags, label names, counts - and the RCCL unique id).
// The tables themselves move over a Plane: RCCL all-reduce / broadcast
// between the GPUs (xGMI), or a host plane (staged through the star) when
// the members share a device or no RCCL is wanted (JUBATUS_MIX_PLANE=host).
//
// Every collective runs against the interconnect timeout; a miss aborts the
// group (RCCL comm abort, sockets closed), marks the epoch failed, and the
// survivors re-form without the stuck member once the leader publishes the
// next epoch (its node's session expires).
#pragma once

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "jb_coord_client.hpp"
#include "jb_roctx.hpp"
#include "jb_hash.hpp"

namespace jb {
namespace mix {

using cc::now_s;

struct Timeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void log(const char* level, const std::string& msg) { cc::log_tagged("mixer", level, msg); }

// ------------------------------------------------------------ sockets
inline bool wait_fd(int fd, short ev, double deadline) {
  for (;;) {
    const double left = deadline - now_s();
    if (left <= 0) return false;
    pollfd p{fd, ev, 0};
    const int r = ::poll(&p, 1, (int)(left * 1000) + 1);
    if (r > 0) return true;
    if (r < 0 && errno != EINTR) return false;
  }
}

inline void send_all(int fd, const void* p, size_t n, double dl) {
  const char* q = (const char*)p;
  while (n) {
    const ssize_t k = ::send(fd, q, n, MSG_NOSIGNAL);
    if (k > 0) { q += k; n -= (size_t)k; continue; }
    if (k < 0 && errno == EINTR) continue;
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      if (!wait_fd(fd, POLLOUT, dl)) throw Timeout("control plane send timed out");
      continue;
    }
    throw std::runtime_error("control plane peer closed (send)");
  }
}

inline void recv_all(int fd, void* p, size_t n, double dl) {
  char* q = (char*)p;
  while (n) {
    const ssize_t k = ::recv(fd, q, n, 0);
    if (k > 0) { q += k; n -= (size_t)k; continue; }
    if (k == 0) throw std::runtime_error("control plane peer closed");
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) {
      if (!wait_fd(fd, POLLIN, dl)) throw Timeout("control plane receive timed out");
      continue;
    }
    throw std::runtime_error(std::string("control plane recv: ") + strerror(errno));
  }
}

inline void send_frame(int fd, const std::string& s, double dl) {
  const uint64_t n = s.size();
  send_all(fd, &n, 8, dl);
  send_all(fd, s.data(), s.size(), dl);
}

inline std::string recv_frame(int fd, double dl) {
  uint64_t n = 0;
  recv_all(fd, &n, 8, dl);
  if (n > (1ull << 36)) throw std::runtime_error("control plane frame too large");
  std::string s(n, '\0');
  recv_all(fd, &s[0], n, dl);
  return s;
}

inline void nonblock(int fd) {
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

// the leader's control-plane listener (one per process, reused by every epoch)
class Listener {
 public:
  explicit Listener(const std::string& host) {
    fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd_ < 0) throw std::runtime_error("socket failed");
    int one = 1;
    setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = 0;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (!host.empty() && host != "0.0.0.0") inet_pton(AF_INET, host.c_str(), &a.sin_addr);
    if (::bind(fd_, (sockaddr*)&a, sizeof a) != 0 || ::listen(fd_, 64) != 0)
      throw std::runtime_error(std::string("mix listener: ") + strerror(errno));
    socklen_t len = sizeof a;
    getsockname(fd_, (sockaddr*)&a, &len);
    port_ = ntohs(a.sin_port);
    nonblock(fd_);
  }
  ~Listener() { if (fd_ >= 0) ::close(fd_); }
  int port() const { return port_; }
  // one connection, or -1 at the deadline
  int accept(double dl) {
    for (;;) {
      const int c = ::accept4(fd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (c >= 0) { nonblock(c); return c; }
      if (errno == EINTR) continue;
      if (errno != EAGAIN && errno != EWOULDBLOCK) return -1;
      if (!wait_fd(fd_, POLLIN, dl)) return -1;
    }
  }

 private:
  int fd_ = -1;
  int port_ = 0;
};

inline int connect_to(const std::string& host, int port, double dl) {
  addrinfo hints{}, *ai = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &ai) != 0 || !ai)
    throw std::runtime_error("cannot resolve " + host);
  const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  nonblock(fd);
  int rc = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
  freeaddrinfo(ai);
  if (rc != 0 && errno != EINPROGRESS) { ::close(fd); throw std::runtime_error("connect refused"); }
  if (rc != 0) {
    if (!wait_fd(fd, POLLOUT, dl)) { ::close(fd); throw Timeout("connect timed out"); }
    int err = 0;
    socklen_t len = sizeof err;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
    if (err) { ::close(fd); throw std::runtime_error(std::string("connect: ") + strerror(err)); }
  }
  return fd;
}

// ------------------------------------------------------------ control plane
// TCP star rooted at rank 0: gathers go to the leader, results come back.
// Every operation is a collective: all ranks call it in the same order.
class Star {
 public:
  Star(int rank, int world) : rank_(rank), world_(world), fds_((size_t)world, -1) {}
  ~Star() { close(); }
  Star(const Star&) = delete;
  Star& operator=(const Star&) = delete;

  // leader: accept world-1 members of this epoch (hello = epoch, rank)
  static std::unique_ptr<Star> lead(Listener& l, int64_t epoch, int world, double dl) {
    std::unique_ptr<Star> s(new Star(0, world));
    int have = 0;
    while (have < world - 1) {
      const int c = l.accept(dl);
      if (c < 0) throw Timeout("members did not join the mix group");
      int64_t hello[2] = {0, 0};
      try {
        recv_all(c, hello, sizeof hello, std::min(dl, now_s() + 5.0));
      } catch (...) {
        ::close(c);
        continue;
      }
      if (hello[0] != epoch || hello[1] <= 0 || hello[1] >= world) {
        ::close(c);   // a stale epoch's member (it retries with the new one)
        continue;
      }
      int& slot = s->fds_[(size_t)hello[1]];
      if (slot >= 0) ::close(slot);   // a member's retry replaces its earlier attempt
      else ++have;
      slot = c;
    }
    const char ok = 1;
    for (int r = 1; r < world; ++r) send_all(s->fds_[(size_t)r], &ok, 1, dl);
    return s;
  }

  static std::unique_ptr<Star> join(const std::string& host, int port, int64_t epoch, int rank, int world,
                                    double dl) {
    std::unique_ptr<Star> s(new Star(rank, world));
    const int fd = connect_to(host, port, dl);
    s->fds_[0] = fd;
    const int64_t hello[2] = {epoch, rank};
    send_all(fd, hello, sizeof hello, dl);
    char ok = 0;
    recv_all(fd, &ok, 1, dl);
    if (ok != 1) throw std::runtime_error("mix group refused");
    return s;
  }

  int rank() const { return rank_; }
  int world() const { return world_; }

  void close() {
    for (int& f : fds_)
      if (f >= 0) { ::shutdown(f, SHUT_RDWR); ::close(f); f = -1; }
  }
  // from another thread: fail every send / recv in progress at once (the
  // descriptors stay open until the owner closes them)
  void interrupt() {
    for (const int f : fds_)
      if (f >= 0) ::shutdown(f, SHUT_RDWR);
  }

  std::vector<std::string> allgather(const std::string& mine, double dl) {
    std::vector<std::string> parts((size_t)world_);
    if (world_ == 1) { parts[0] = mine; return parts; }
    if (rank_ == 0) {
      parts[0] = mine;
      for (int r = 1; r < world_; ++r) parts[(size_t)r] = recv_frame(fds_[(size_t)r], dl);
      std::string all;
      for (const auto& p : parts) {
        const uint64_t n = p.size();
        all.append((const char*)&n, 8);
        all += p;
      }
      for (int r = 1; r < world_; ++r) send_frame(fds_[(size_t)r], all, dl);
      return parts;
    }
    send_frame(fds_[0], mine, dl);
    const std::string all = recv_frame(fds_[0], dl);
    size_t o = 0;
    for (int r = 0; r < world_; ++r) {
      if (o + 8 > all.size()) throw std::runtime_error("control plane: short gather");
      uint64_t n;
      memcpy(&n, all.data() + o, 8);
      o += 8;
      if (o + n > all.size()) throw std::runtime_error("control plane: short gather");
      parts[(size_t)r] = all.substr(o, n);
      o += n;
    }
    return parts;
  }

  // element-wise reduction of n values of T (op(a, b) -> a)
  template <class T, class Op>
  void allreduce(T* v, size_t n, Op op, double dl) {
    if (world_ == 1 || n == 0) return;
    const size_t bytes = n * sizeof(T);
    if (rank_ == 0) {
      std::vector<T> tmp(n);
      for (int r = 1; r < world_; ++r) {
        recv_all(fds_[(size_t)r], tmp.data(), bytes, dl);
        for (size_t i = 0; i < n; ++i) v[i] = op(v[i], tmp[i]);
      }
      for (int r = 1; r < world_; ++r) send_all(fds_[(size_t)r], v, bytes, dl);
    } else {
      send_all(fds_[0], v, bytes, dl);
      recv_all(fds_[0], v, bytes, dl);
    }
  }

  void allreduce_max(int64_t* v, size_t n, double dl) {
    allreduce(v, n, [](int64_t a, int64_t b) { return a > b ? a : b; }, dl);
  }
  void allreduce_sum(int64_t* v, size_t n, double dl) {
    allreduce(v, n, [](int64_t a, int64_t b) { return a + b; }, dl);
  }

  // root's bytes to every rank (through the leader)
  void bcast(int root, void* p, size_t bytes, double dl) {
    if (world_ == 1 || bytes == 0) return;
    if (rank_ == 0) {
      if (root != 0) recv_all(fds_[(size_t)root], p, bytes, dl);
      for (int r = 1; r < world_; ++r)
        if (r != root) send_all(fds_[(size_t)r], p, bytes, dl);
    } else if (rank_ == root) {
      send_all(fds_[0], p, bytes, dl);
    } else {
      recv_all(fds_[0], p, bytes, dl);
    }
  }
  std::string bcast_str(int root, const std::string& s, double dl) {
    uint64_t n = s.size();
    bcast(root, &n, 8, dl);
    std::string out = rank_ == root ? s : std::string(n, '\0');
    bcast(root, &out[0], n, dl);
    return out;
  }

  // one round of a pairwise schedule (push mixers): every rank names its
  // peer (-1: none this round) and gets the bytes its peer sent it; the
  // leader routes the frames. Collective: every rank calls it once per round
  std::string permute(int peer, const std::string& mine, double dl) {
    if (world_ == 1) return std::string();
    auto frame = [](int32_t to, const std::string& b) {
      std::string f((const char*)&to, 4);
      return f + b;
    };
    if (rank_ != 0) {
      send_frame(fds_[0], frame(peer, mine), dl);
      return recv_frame(fds_[0], dl);
    }
    std::vector<std::string> in((size_t)world_);
    std::vector<int32_t> to((size_t)world_, -1);
    in[0] = mine;
    to[0] = peer;
    for (int r = 1; r < world_; ++r) {
      const std::string f = recv_frame(fds_[(size_t)r], dl);
      if (f.size() < 4) throw std::runtime_error("control plane: short permute frame");
      memcpy(&to[(size_t)r], f.data(), 4);
      in[(size_t)r] = f.substr(4);
    }
    // rank r receives what its peer addressed to it (empty if none)
    std::vector<std::string> out((size_t)world_);
    for (int r = 0; r < world_; ++r) {
      const int32_t d = to[(size_t)r];
      if (d >= 0 && d < world_ && to[(size_t)d] == r) out[(size_t)d] = in[(size_t)r];
    }
    for (int r = 1; r < world_; ++r) send_frame(fds_[(size_t)r], out[(size_t)r], dl);
    return out[0];
  }

 private:
  int rank_, world_;
  std::vector<int> fds_;
};

// ------------------------------------------------------------ data plane
// Collectives over model tables in the plane's memory space (device memory
// for the GPU planes, host memory for HostPlane). Blocking; a collective past
// the deadline throws Timeout (the group then aborts).
class Plane {
 public:
  virtual ~Plane() {}
  virtual const char* name() const = 0;
  virtual void allreduce_sum(float* p, size_t n, double dl) = 0;
  virtual void allreduce_max(uint8_t* p, size_t n, double dl) = 0;
  // bf16 SUM (the bit patterns in uint16): only the device plane has it
  // (false: not supported, the caller sends fp32)
  virtual bool allreduce_sum_bf16(uint16_t* p, size_t n, double dl) {
    (void)p; (void)n; (void)dl;
    return false;
  }
  virtual void bcast(void* p, size_t bytes, int root, double dl) = 0;
  virtual void abort() {}
  // variable-size host byte strings (row diffs, whole models): every rank's
  // bytes to every rank / the root's bytes to every rank. The default moves
  // them over the control plane; the device plane moves the payload over
  // RCCL (the sizes over the control plane)
  virtual std::vector<std::string> allgather_bytes(Star& s, const std::string& mine, double dl) {
    return s.allgather(mine, dl);
  }
  virtual std::string bcast_bytes(Star& s, int root, const std::string& b, double dl) {
    return s.bcast_str(root, b, dl);
  }
  // one round of a pairwise schedule: this rank's bytes to `peer`, the
  // peer's back (peer -1: no exchange this round, still a collective call)
  virtual std::string exchange_bytes(Star& s, int peer, const std::string& mine, double dl) {
    return s.permute(peer, mine, dl);
  }
  // one round of a pairwise schedule over tables in the plane's memory:
  // p += the peer's p / p = max(p, the peer's p). Every rank calls it once
  // per round (peer -1, n 0: sits the round out). The default moves host
  // memory over the control plane; the device plane sends point-to-point
  virtual void pair_sum(Star& s, float* p, size_t n, int peer, double dl) {
    const std::string theirs = s.permute(peer, std::string((const char*)p, peer >= 0 ? n * 4 : 0), dl);
    if (peer < 0) return;
    if (theirs.size() != n * 4) throw std::runtime_error("pair MIX: the peer's table differs in size");
    const float* q = (const float*)theirs.data();
    for (size_t i = 0; i < n; ++i) p[i] += q[i];
  }
  virtual void pair_max(Star& s, uint8_t* p, size_t n, int peer, double dl) {
    const std::string theirs = s.permute(peer, std::string((const char*)p, peer >= 0 ? n : 0), dl);
    if (peer < 0) return;
    if (theirs.size() != n) throw std::runtime_error("pair MIX: the peer's bitmap differs in size");
    for (size_t i = 0; i < n; ++i) p[i] = std::max(p[i], (uint8_t)theirs[i]);
  }
};

// host memory over the star (CPU servers, rehearsals)
class HostPlane : public Plane {
 public:
  explicit HostPlane(Star* s) : s_(s) {}
  const char* name() const override { return "host"; }
  void allreduce_sum(float* p, size_t n, double dl) override {
    s_->allreduce(p, n, [](float a, float b) { return a + b; }, dl);
  }
  void allreduce_max(uint8_t* p, size_t n, double dl) override {
    s_->allreduce(p, n, [](uint8_t a, uint8_t b) { return a > b ? a : b; }, dl);
  }
  void bcast(void* p, size_t bytes, int root, double dl) override { s_->bcast(root, p, bytes, dl); }

 private:
  Star* s_;
};

// ------------------------------------------------------------ epochs
struct Epoch {
  int64_t epoch = -1;
  std::vector<std::string> members;
  std::string addr;
  int port = 0;
};

// {"epoch": e, "members": [...], "addr": "...", "port": p} (group.py layout)
inline bool parse_epoch(const std::string& text, Epoch* e) {
  if (text.empty()) return false;
  // a flat object of known keys: scanned by hand
  auto num_after = [&](const char* key, int64_t* out) {
    const size_t k = text.find(std::string("\"") + key + "\"");
    if (k == std::string::npos) return false;
    size_t c = text.find(':', k);
    if (c == std::string::npos) return false;
    ++c;
    while (c < text.size() && text[c] == ' ') ++c;
    char* end = nullptr;
    const long long v = strtoll(text.c_str() + c, &end, 10);
    if (end == text.c_str() + c) return false;
    *out = v;
    return true;
  };
  auto str_after = [&](const char* key, std::string* out) {
    const size_t k = text.find(std::string("\"") + key + "\"");
    if (k == std::string::npos) return false;
    size_t q = text.find('"', text.find(':', k));
    if (q == std::string::npos) return false;
    const size_t q2 = text.find('"', q + 1);
    if (q2 == std::string::npos) return false;
    *out = text.substr(q + 1, q2 - q - 1);
    return true;
  };
  int64_t ep = 0, port = 0;
  if (!num_after("epoch", &ep) || !num_after("port", &port) || !str_after("addr", &e->addr)) return false;
  const size_t m = text.find("\"members\"");
  if (m == std::string::npos) return false;
  const size_t lb = text.find('[', m), rb = text.find(']', m);
  if (lb == std::string::npos || rb == std::string::npos || rb < lb) return false;
  e->members.clear();
  size_t p = lb;
  while (true) {
    const size_t q = text.find('"', p + 1);
    if (q == std::string::npos || q > rb) break;
    const size_t q2 = text.find('"', q + 1);
    if (q2 == std::string::npos || q2 > rb) return false;
    e->members.push_back(text.substr(q + 1, q2 - q - 1));
    p = q2;
  }
  e->epoch = ep;
  e->port = (int)port;
  return true;
}

inline std::string epoch_json(const Epoch& e) {
  std::string s = "{\"epoch\": " + std::to_string(e.epoch) + ", \"members\": [";
  for (size_t i = 0; i < e.members.size(); ++i) s += (i ? ", \"" : "\"") + e.members[i] + "\"";
  return s + "], \"addr\": \"" + e.addr + "\", \"port\": " + std::to_string(e.port) + "}";
}

inline std::string actor_path(const std::string& type, const std::string& name) {
  return "/jubatus/actors/" + type + "/" + name;
}

class Group;
using PlaneFactory = std::function<std::unique_ptr<Plane>(Group&, double dl)>;

// The group of the current epoch (parallel/group.py ProcessGroupManager).
class Group {
 public:
  Group(cc::Coord* coord, const std::string& type, const std::string& name, const std::string& ident,
        const std::string& eth, double rendezvous_timeout, double op_timeout, PlaneFactory pf)
      : coord_(coord), type_(type), name_(name), ident_(ident), eth_(eth),
        rdv_timeout_(rendezvous_timeout), op_timeout_(op_timeout), pf_(std::move(pf)),
        listener_(new Listener(eth == "localhost" ? "127.0.0.1" : eth)) {
    path_ = actor_path(type, name) + "/mix_epoch";
    coord_->create(path_, "", false);
  }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t epoch() const { return epoch_; }
  uint64_t aborts() const { return aborts_; }
  const std::string& plane_name() const { return plane_name_; }
  Star& star() { return *star_; }
  Plane& plane() { return *plane_; }
  double deadline() const { return now_s() + op_timeout_; }
  double op_timeout() const { return op_timeout_; }

  std::vector<std::string> live() {
    auto v = coord_->list(actor_path(type_, name_) + "/nodes");
    std::sort(v.begin(), v.end());
    return v;
  }

  void maybe_publish() {
    const auto lv = live();
    if (lv.empty() || lv[0] != ident_) return;   // not the leader
    Epoch cur;
    std::string text;
    const bool have = coord_->read(path_, &text) && parse_epoch(text, &cur);
    if (have && cur.members == lv) return;
    Epoch e;
    e.epoch = (have ? cur.epoch : 0) + 1;
    e.members = lv;
    e.addr = (eth_.empty() || eth_ == "0.0.0.0" || eth_ == "localhost") ? "127.0.0.1" : eth_;
    e.port = listener_->port();
    coord_->call("set", {cc::Value::str(path_), cc::Value::str(epoch_json(e))});
    log("INFO", "published mix group epoch " + std::to_string(e.epoch) + " (" +
                    std::to_string(lv.size()) + " members)");
  }

  // (re)join the current epoch's group; true when a new group formed
  bool ensure() {
    maybe_publish();
    Epoch cur;
    std::string text;
    if (!coord_->read(path_, &text) || !parse_epoch(text, &cur)) return false;
    if (cur.epoch == epoch_) return false;
    auto me = std::find(cur.members.begin(), cur.members.end(), ident_);
    if (me == cur.members.end()) return false;
    auto f = failed_.find(cur.epoch);
    if (f != failed_.end() && now_s() - f->second < rdv_timeout_) return false;
    const auto lv = live();
    for (const auto& m : cur.members)
      if (!std::binary_search(lv.begin(), lv.end(), m)) return false;   // wait for the next epoch
    teardown();
    const int rank = (int)(me - cur.members.begin());
    const int world = (int)cur.members.size();
    const double dl = now_s() + rdv_timeout_;
    try {
      if (world > 1) {
        std::unique_ptr<Star> st = rank == 0 ? Star::lead(*listener_, cur.epoch, world, dl)
                                             : Star::join(cur.addr, cur.port, cur.epoch, rank, world, dl);
        std::lock_guard<std::mutex> g(smu_);
        star_ = std::move(st);
      } else {
        std::lock_guard<std::mutex> g(smu_);
        star_.reset(new Star(0, 1));
      }
      rank_ = rank;
      world_ = world;
      plane_ = pf_(*this, dl);
      plane_name_ = plane_->name();
    } catch (const std::exception& e) {
      log("WARN", "failed to join mix group epoch " + std::to_string(cur.epoch) + ": " + e.what());
      failed_[cur.epoch] = now_s();
      teardown();
      return false;
    }
    epoch_ = cur.epoch;
    log("INFO", "joined mix group epoch " + std::to_string(epoch_) + " as rank " + std::to_string(rank_) +
                    "/" + std::to_string(world_) + " (" + plane_name_ + " plane)");
    return true;
  }

  // a collective failed or missed the deadline: leave the epoch
  void abort(const std::string& why) {
    ++aborts_;
    log("WARN", "aborting mix group epoch " + std::to_string(epoch_) + ": " + why);
    if (plane_) plane_->abort();
    if (epoch_ >= 0) failed_[epoch_] = now_s();
    teardown();
    epoch_ = -1;
  }

  void close() {
    teardown();
    epoch_ = -1;
  }

  // any thread (shutdown): a collective blocked on the control plane - or on
  // the host data plane, which runs over it - fails now instead of at the
  // interconnect deadline
  void interrupt() {
    std::lock_guard<std::mutex> g(smu_);
    if (star_) star_->interrupt();
  }

 private:
  void teardown() {
    plane_.reset();
    std::lock_guard<std::mutex> g(smu_);
    if (star_) star_->close();
    star_.reset();
    rank_ = -1;
    world_ = 0;
  }

  cc::Coord* coord_;
  std::string type_, name_, ident_, eth_, path_;
  double rdv_timeout_, op_timeout_;
  PlaneFactory pf_;
  std::unique_ptr<Listener> listener_;
  std::unique_ptr<Star> star_;
  std::mutex smu_;                 // star_'s lifetime vs interrupt()
  std::unique_ptr<Plane> plane_;
  std::string plane_name_ = "none";
  int rank_ = -1, world_ = 0;
  int64_t epoch_ = -1;
  uint64_t aborts_ = 0;
  std::map<int64_t, double> failed_;
};

// ------------------------------------------------------------ mixer
// What a model contributes to the linear mixer (called on the mixer thread,
// every rank in the same order).
class Mixable {
 public:
  virtual ~Mixable() {}
  // one MIX; -> bytes this rank all-reduced
  virtual uint64_t mix(Group& g) = 0;
  // obsolete protocol: rank `src` sends its whole model; apply = replace mine
  virtual void hand_over(Group& g, int src, bool apply) = 0;
  // push mixers: one round of the pairwise schedule - a symmetric exchange
  // with `peer` (-1: this rank sits the round out, but still takes part in
  // the round's collective calls); -> bytes this rank sent
  virtual uint64_t pair_mix(Group& g, int peer) {
    (void)g;
    (void)peer;
    throw std::runtime_error("this model is not push-mixable");
  }
  virtual bool push_mixable() const { return false; }
  // around the rounds of one push MIX (a model may forward what it received
  // in earlier rounds of the same MIX, then forget its diff at the end)
  virtual void push_begin() {}
  virtual void push_end() {}
};

// Pairwise schedules of the push mixers (parallel/push_mixer.py, reference
// random_mixer.hpp:45-59, broadcast_mixer.hpp:45-55, skip_mixer.hpp:46-57):
// every rank derives the same rounds from (epoch, mix count); a round is a
// perfect matching (peer -1 for a rank without one).
inline std::vector<std::vector<int>> push_schedule(const std::string& kind, int n, int64_t epoch,
                                                   uint64_t round_no) {
  std::vector<std::vector<int>> rounds;
  if (n <= 1) return rounds;
  auto tournament = [&](int limit) {
    std::vector<int> pl;
    for (int i = 0; i < n; ++i) pl.push_back(i);
    if (n % 2) pl.push_back(-1);
    const int k = (int)pl.size();
    for (int r = 0; r < k - 1 && (int)rounds.size() < limit; ++r) {
      std::vector<int> m((size_t)n, -1);
      for (int i = 0; i < k / 2; ++i) {
        const int a = pl[(size_t)i], b = pl[(size_t)(k - 1 - i)];
        if (a >= 0 && b >= 0) { m[(size_t)a] = b; m[(size_t)b] = a; }
      }
      rounds.push_back(m);
      std::vector<int> nx{pl[0], pl[(size_t)(k - 1)]};
      for (int i = 1; i < k - 1; ++i) nx.push_back(pl[(size_t)i]);
      pl.swap(nx);
    }
  };
  if (kind == "random_mixer") {
    // one random perfect matching: a shuffle seeded by (epoch, round)
    std::vector<int> order;
    for (int i = 0; i < n; ++i) order.push_back(i);
    uint64_t x = ((uint64_t)epoch << 20) ^ round_no ^ 0x9E3779B97F4A7C15ull;
    for (int i = n - 1; i > 0; --i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      std::swap(order[(size_t)i], order[(size_t)(x % (uint64_t)(i + 1))]);
    }
    std::vector<int> m((size_t)n, -1);
    for (int i = 0; i + 1 < n; i += 2) {
      m[(size_t)order[(size_t)i]] = order[(size_t)i + 1];
      m[(size_t)order[(size_t)i + 1]] = order[(size_t)i];
    }
    rounds.push_back(m);
  } else if (kind == "broadcast_mixer") {
    tournament(n);                     // every pair once
  } else {                             // skip_mixer: strides N/2, N/4, ..., 1
    int nstr = 0;
    for (int st = n / 2; st >= 1; st /= 2) ++nstr;
    if ((n & (n - 1)) == 0) {
      for (int st = n / 2; st >= 1; st /= 2) {
        std::vector<int> m((size_t)n, -1);
        for (int r = 0; r < n; ++r) m[(size_t)r] = r ^ st;   // butterfly
        rounds.push_back(m);
      }
    } else {
      tournament(std::max(1, nstr));   // log2 rounds of the tournament
    }
  }
  return rounds;
}

// fault injection (utils/fault.py rules mix_hang / mix_kill, phase and at=N)
class Faults {
 public:
  Faults() {
    const char* e = getenv("JUBATUS_FAULT");
    if (!e) return;
    std::string s(e);
    size_t p = 0;
    while (p <= s.size()) {
      size_t q = s.find(';', p);
      if (q == std::string::npos) q = s.size();
      parse_rule(s.substr(p, q - p));
      p = q + 1;
    }
  }
  // the MIX reached `phase`
  void on_mix(const std::string& phase) {
    for (Rule& r : rules_) {
      if (r.phase != "*" && r.phase != phase) continue;
      ++r.hits;
      if (r.at > 0 && r.hits != r.at) continue;
      if (r.kind == "mix_kill") {
        log("WARN", "fault injection: exiting at MIX phase " + phase);
        _exit(3);
      }
      if (r.kind == "mix_hang") {
        log("WARN", "fault injection: stalling MIX phase " + phase);
        std::this_thread::sleep_for(std::chrono::milliseconds(r.ms));
      }
    }
  }

 private:
  struct Rule {
    std::string kind, phase = "*";
    int64_t at = 0, ms = 0, hits = 0;
  };
  void parse_rule(const std::string& r) {
    const size_t c = r.find(':');
    if (c == std::string::npos) return;
    Rule x;
    x.kind = r.substr(0, c);
    if (x.kind != "mix_kill" && x.kind != "mix_hang") return;
    std::string rest = r.substr(c + 1);
    size_t p = 0;
    while (p < rest.size()) {
      size_t q = rest.find(',', p);
      if (q == std::string::npos) q = rest.size();
      const std::string kv = rest.substr(p, q - p);
      const size_t e = kv.find('=');
      if (e != std::string::npos) {
        const std::string k = kv.substr(0, e), v = kv.substr(e + 1);
        if (k == "phase") x.phase = v;
        else if (k == "at") x.at = atoll(v.c_str());
        else if (k == "ms") x.ms = atoll(v.c_str());
      }
      p = q + 1;
    }
    rules_.push_back(x);
  }
  std::vector<Rule> rules_;
};

struct MixerArgs {
  std::string kind = "linear_mixer";   // or random_mixer / broadcast_mixer / skip_mixer
  std::string type, name, eth;
  int port = 0;
  int interval_sec = 16, interval_count = 512;
  double interconnect_timeout = 10;
  int protocol_version = 1;
};

// The mixer's stabilizer loop (parallel/linear_mixer.py CollectiveMixer): the
// linear mixer (all members fold every member's diff) or, with a push kind,
// the rounds of a pairwise schedule (parallel/push_mixer.py PushMixer).
class LinearMixer {
 public:
  LinearMixer(cc::Coord* coord, const MixerArgs& a, Mixable* model, PlaneFactory pf)
      : coord_(coord), a_(a), model_(model) {
    ident_ = a.eth + "_" + std::to_string(a.port);
    group_.reset(new Group(coord, a.type, a.name, ident_, a.eth,
                           std::max(5.0, 3.0 * a.interconnect_timeout),
                           std::max(1.0, a.interconnect_timeout), std::move(pf)));
    ticktime_ = now_s();
  }
  ~LinearMixer() { stop(); }

  void start() {
    running_ = true;
    th_ = std::thread([this] { loop(); });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stop_) return;
      stop_ = true;
      cv_.notify_all();
    }
    group_->interrupt();     // a MIX in flight fails now (its peers abort their epoch)
    if (th_.joinable()) th_.join();
    running_ = false;
    group_->close();
  }

  void updated(uint64_t n) {
    std::lock_guard<std::mutex> g(mu_);
    counter_ += n;
    if (a_.interval_count > 0 && counter_ >= (uint64_t)a_.interval_count) cv_.notify_all();
  }

  // force a MIX at the next tick and wait for it (RPC do_mix)
  // a MIX that begins after this call (a MIX already under way snapshotted
  // the model before it: its end does not count)
  bool do_mix() {
    std::unique_lock<std::mutex> g(mu_);
    const uint64_t want = begun_ + 1;
    force_ = true;
    cv_.notify_all();
    const double dl = now_s() + std::max(30.0, 4 * a_.interconnect_timeout);
    while (ended_ < want && !stop_ && now_s() < dl) cv_.wait_for(g, std::chrono::milliseconds(100));
    return ended_ >= want;
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) {
    std::lock_guard<std::mutex> g(mu_);
    auto add = [&](const std::string& k, const std::string& v) { st->emplace_back(a_.kind + "." + k, v); };
    add("count", std::to_string(counter_));
    add("ticktime", std::to_string((int64_t)ticktime_wall_));
    add("is_obsolete", obsolete_ ? "1" : "0");
    add("is_running", running_ ? "1" : "0");
    add("mix_count", std::to_string(mix_count_));
    add("last_mix_bytes", std::to_string(last_bytes_));
    char b[32];
    snprintf(b, sizeof b, "%.6f", last_sec_);
    add("last_mix_sec", b);
    add("watchdog_aborts", std::to_string(group_->aborts()));
    add("group_epoch", std::to_string(group_->epoch()));
    add("group_rank", std::to_string(group_->rank()));
    add("group_size", std::to_string(group_->world()));
    add("backend", group_->plane_name());
    add("runtime", "native");
  }

 private:
  bool want_locked() const {
    if (counter_ == 0) return false;
    if (a_.interval_count > 0 && counter_ >= (uint64_t)a_.interval_count) return true;
    return a_.interval_sec > 0 && now_s() - ticktime_ > a_.interval_sec;
  }

  // a MIX begins: the force it answers is consumed (a do_mix after this
  // point waits for the next one) -> its sequence number
  uint64_t begin_locked() {
    force_ = false;
    return ++begun_;
  }
  void mixed_locked(uint64_t seq, uint64_t bytes, double sec) {
    counter_ = 0;
    ticktime_ = now_s();
    ticktime_wall_ = (double)time(nullptr);
    ++mix_count_;
    if (seq > ended_) ended_ = seq;
    last_bytes_ = bytes;
    last_sec_ = sec;
    cv_.notify_all();
  }

  void register_active() {
    const std::string base = actor_path(a_.type, a_.name) + "/actives";
    coord_->create(base, "", false);
    if (!coord_->exists(base + "/" + ident_)) coord_->create(base + "/" + ident_, "", true);
  }

  void loop() {
    while (true) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait_for(g, std::chrono::milliseconds(500));
        if (stop_) break;
      }
      try {
        tick();
      } catch (const std::exception& e) {
        if (group_->epoch() >= 0) group_->abort(std::string("collective failed: ") + e.what());
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait_for(g, std::chrono::milliseconds(500), [this] { return stop_; });
      }
    }
  }

  void tick() {
    Group& g = *group_;
    const bool formed = g.ensure();
    if (g.world() == 0) return;
    if (g.world() == 1) {
      if (obsolete_) {
        obsolete_ = false;
        register_active();
      }
      std::lock_guard<std::mutex> l(mu_);
      if (force_ || want_locked()) mixed_locked(begin_locked(), 0, 0.0);
      return;
    }
    if (formed) {
      faults_.on_mix("handover");
      hand_over();
    }
    // [wants a MIX, forced, protocol version, -version, MIX count]: the count is
    // agreed too - the push mixers derive the pairing of a round from it, and
    // members' own counts differ (solo ticks, a member that joined late, a
    // MIX that failed on one side); every member mixes round max(counts)
    int64_t flags[5];
    {
      std::lock_guard<std::mutex> l(mu_);
      flags[0] = want_locked() ? 1 : 0;
      flags[1] = force_ ? 1 : 0;
      flags[4] = (int64_t)mix_count_;
    }
    flags[2] = a_.protocol_version;
    flags[3] = -a_.protocol_version;
    g.star().allreduce_max(flags, 5, g.deadline());
    if (flags[2] != -flags[3]) {
      log("FATAL", "mix protocol version mismatch in the cluster: shutting down");
      kill(getpid(), SIGTERM);
      return;
    }
    if (!(flags[0] || flags[1])) return;
    uint64_t seq;
    {
      std::lock_guard<std::mutex> l(mu_);
      seq = begin_locked();
    }
    faults_.on_mix("allreduce");
    const double t0 = now_s();
    uint64_t bytes = 0;
    if (a_.kind == "linear_mixer") {
      jb::tx::Range tr("mix.linear");
      bytes = model_->mix(g);
    } else {
      // push mixers: the rounds of the pairwise schedule (push_mixer.cpp:335-408)
      // of the agreed round number
      const uint64_t round_no = (uint64_t)flags[4];
      model_->push_begin();
      for (const auto& m : push_schedule(a_.kind, g.world(), g.epoch(), round_no)) {
        faults_.on_mix("pair");
        jb::tx::Range tr("mix.push_round");
        bytes += model_->pair_mix(g, m[(size_t)g.rank()]);
      }
      model_->push_end();
    }
    const double sec = now_s() - t0;
    std::lock_guard<std::mutex> l(mu_);
    mix_count_ = (uint64_t)flags[4];      // every member leaves this MIX at the same count
    mixed_locked(seq, bytes, sec);
    char b[160];
    snprintf(b, sizeof b, "mixed with %d servers in %.6f secs, %llu bytes", g.world(), sec,
             (unsigned long long)bytes);
    log("INFO", b);
  }

  // a new group: obsolete members receive the lowest-rank up-to-date model
  void hand_over() {
    Group& g = *group_;
    const int64_t big = 1ll << 30;
    int64_t r[2] = {-(obsolete_ ? big : (int64_t)g.rank()), obsolete_ ? 1 : 0};
    g.star().allreduce_max(r, 2, g.deadline());
    const int64_t src = -r[0];
    if (r[1] && src < big) {
      model_->hand_over(g, (int)src, obsolete_);
      if (obsolete_) log("INFO", "model fetched from rank " + std::to_string(src));
    }
    obsolete_ = false;
    register_active();
  }

  cc::Coord* coord_;
  MixerArgs a_;
  Mixable* model_;
  std::string ident_;
  std::unique_ptr<Group> group_;
  Faults faults_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
  bool stop_ = false, force_ = false, obsolete_ = true;
  std::atomic<bool> running_{false};
  uint64_t counter_ = 0, mix_count_ = 0, last_bytes_ = 0;
  uint64_t begun_ = 0, ended_ = 0;   // MIXes this member began / finished (do_mix)
  double ticktime_ = 0, ticktime_wall_ = (double)time(nullptr), last_sec_ = 0;
};

// ------------------------------------------------------------ membership
// Distributed-mode registration of a server process (membership.py):
// the base tree, the config read lock, the actor node (ephemeral) and a
// self-fencing watch that SIGTERMs the process when its node disappears.
class ClusterNode {
 public:
  ClusterNode(const std::string& zk, double zk_timeout, const std::string& type, const std::string& name)
      : type_(type), name_(name) {
    coord_.reset(new cc::Coord(zk, zk_timeout, "cluster"));
    const std::string base = actor_path(type, name);
    for (const std::string& p : {std::string("/jubatus"), std::string("/jubatus/supervisors"),
                                 std::string("/jubatus/jubaproxies"), std::string("/jubatus/actors"),
                                 std::string("/jubatus/config"), "/jubatus/actors/" + type,
                                 "/jubatus/config/" + type, "/jubatus/jubaproxies/" + type, base,
                                 base + "/nodes", base + "/actives", base + "/master_lock",
                                 base + "/config_lock", base + "/id_generator", base + "/mix"})
      coord_->create(p, "", false);
  }
  ~ClusterNode() { leave(); }

  cc::Coord* coord() { return coord_.get(); }

  std::string config() {
    std::string text;
    if (!coord_->read("/jubatus/config/" + type_ + "/" + name_, &text))
      throw std::runtime_error("config is not found: /jubatus/config/" + type_ + "/" + name_);
    return text;
  }

  // config read lock (zkmutex rlock): no writer may precede us
  bool config_rlock() {
    const std::string dir = actor_path(type_, name_) + "/config_lock";
    for (int attempt = 0; attempt < 3; ++attempt) {
      cc::Value r = coord_->call("create_seq", {cc::Value::integer(sid()), cc::Value::str(dir + "/rlock_")});
      const auto& a = r.as_array();
      if (a.at(0).as_int() != 0) continue;
      const std::string mine = a.at(1).as_str();
      const std::string me = mine.substr(mine.rfind('/') + 1);
      const int64_t my = atoll(me.c_str() + me.size() - 10);
      bool ok = true;
      for (const auto& c : coord_->list(dir))
        if (c.compare(0, 6, "wlock_") == 0 && atoll(c.c_str() + c.size() - 10) < my) ok = false;
      if (ok) { rlock_ = mine; return true; }
      coord_->call("remove", {cc::Value::str(mine)});
    }
    return false;
  }

  void register_actor(const std::string& eth, int port) {
    node_ = actor_path(type_, name_) + "/nodes/" + eth + "_" + std::to_string(port);
    active_ = actor_path(type_, name_) + "/actives/" + eth + "_" + std::to_string(port);
    if (!coord_->create(node_, "", true)) throw std::runtime_error("Failed to register_actor");
    cc::log_tagged("cluster", "INFO", "actor created: " + node_);
    fence_ = std::thread([this] {
      while (!stop_.load()) {
        for (int i = 0; i < 10 && !stop_.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(50));
        if (stop_.load()) break;
        try {
          if (!coord_->exists(node_)) {
            cc::log_tagged("cluster", "ERROR", "own actor node deleted: shutting down");
            kill(getpid(), SIGTERM);
            return;
          }
        } catch (...) {
        }
      }
    });
  }

  void leave() {
    if (stop_.exchange(true)) return;
    if (fence_.joinable()) fence_.join();
    try {
      for (const auto& c : cht_nodes_) coord_->call("remove", {cc::Value::str(c)});
      if (!node_.empty()) coord_->call("remove", {cc::Value::str(active_)});
      if (!node_.empty()) coord_->call("remove", {cc::Value::str(node_)});
      if (!rlock_.empty()) coord_->call("remove", {cc::Value::str(rlock_)});
    } catch (...) {
    }
    coord_->close();
  }

  std::string connected() const { return coord_->connected(); }

  // CHT registration: NUM_VSERV = 8 ephemeral vnodes <actor>/cht/<md5(ip_port[_i])>
  // with payload ip_port (cht.cpp:42-93, membership.cpp:40-47)
  void register_cht(const std::string& eth, int port) {
    const std::string dir = actor_path(type_, name_) + "/cht";
    coord_->create(dir, "", false);
    const std::string loc = eth + "_" + std::to_string(port);
    for (int i = 0; i < 8; ++i) {
      const std::string key = i > 0 ? loc + "_" + std::to_string(i) : loc;
      const std::string path = dir + "/" + jb::Md5::hex(key);
      if (!coord_->create(path, loc, true)) throw std::runtime_error("Failed to register cht node: " + path);
      cht_nodes_.push_back(path);
    }
  }
  // n consecutive vnodes from lower_bound(md5(key)), wrapping (cht.cpp:107-143)
  std::vector<std::pair<std::string, int>> cht_find(const std::string& key, int n) {
    const std::string dir = actor_path(type_, name_) + "/cht";
    std::vector<std::string> h = coord_->list(dir);
    if (h.empty()) throw std::runtime_error("no server found in cht: " + name_);
    std::sort(h.begin(), h.end());
    size_t idx = (size_t)(std::lower_bound(h.begin(), h.end(), jb::Md5::hex(key)) - h.begin()) % h.size();
    std::vector<std::pair<std::string, int>> out;
    for (int i = 0; i < n; ++i) {
      std::string loc;
      if (!coord_->read(dir + "/" + h[idx], &loc)) throw std::runtime_error("failed to read CHT entry: " + dir);
      const size_t u = loc.find('_');
      out.push_back(u == std::string::npos ? std::make_pair(loc, 0)
                                           : std::make_pair(loc.substr(0, u), atoi(loc.c_str() + u + 1)));
      idx = (idx + 1) % h.size();
    }
    return out;
  }
  // every registered actor ("ip_port" children of <actor>/nodes, membership.py get_all_nodes)
  std::vector<std::pair<std::string, int>> actors() {
    std::vector<std::pair<std::string, int>> out;
    for (const auto& loc : coord_->list(actor_path(type_, name_) + "/nodes")) {
      const size_t u = loc.rfind('_');
      if (u != std::string::npos) out.emplace_back(loc.substr(0, u), atoi(loc.c_str() + u + 1));
    }
    return out;
  }
  // the whole ring, sorted by vnode hash: (md5 hex, "ip_port") - for engines
  // that place many keys at once (burst's processed keywords)
  std::vector<std::pair<std::string, std::string>> cht_ring() {
    const std::string dir = actor_path(type_, name_) + "/cht";
    std::vector<std::string> h = coord_->list(dir);
    std::sort(h.begin(), h.end());
    std::vector<std::pair<std::string, std::string>> out;
    for (const auto& x : h) {
      std::string loc;
      if (coord_->read(dir + "/" + x, &loc)) out.emplace_back(x, loc);
    }
    return out;
  }
  // global_id_generator_zk: the data version of <actor>/id_generator
  uint64_t create_id() {
    const std::string path = actor_path(type_, name_) + "/id_generator";
    cc::Value r = coord_->call("set", {cc::Value::str(path), cc::Value::str("dummy")});
    const auto& a = r.as_array();
    if (a.at(0).as_int() != 0) throw std::runtime_error("failed to increment version of node: " + path);
    return (uint64_t)a.at(1).as_int();
  }

 private:
  int64_t sid() { return coord_->session(); }
  std::string type_, name_, node_, active_, rlock_;
  std::vector<std::string> cht_nodes_;
  std::unique_ptr<cc::Coord> coord_;
  std::thread fence_;
  std::atomic<bool> stop_{false};
};

}  // namespace mix
}  // namespace jb
