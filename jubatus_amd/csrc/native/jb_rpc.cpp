// See jb_rpc.hpp.
#include "jb_rpc.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <stdexcept>

#include "jb_msgpack.hpp"
#include "jb_roctx.hpp"

namespace jb {

namespace {

double now_sec() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// Header of the msgpack token at p (p[0] = type byte, tokens other than the
// one-byte fixint / fixstr / fixarray / fixmap forms): bytes before the
// payload, for the bounds check of the slow path.
inline uint32_t header_bytes(uint8_t t) {
  switch (t) {
    case 0xd9: case 0xc4: case 0xc7: return t == 0xc7 ? 3 : 2;
    case 0xda: case 0xc5: case 0xdc: case 0xde: return 3;
    case 0xc8: return 4;
    case 0xdb: case 0xc6: case 0xdd: case 0xdf: return 5;
    case 0xc9: return 6;
    default: return 1;
  }
}

inline uint64_t be16(const uint8_t* p) { return ((uint64_t)p[0] << 8) | p[1]; }
inline uint64_t be32(const uint8_t* p) {
  return ((uint64_t)p[0] << 24) | ((uint64_t)p[1] << 16) | ((uint64_t)p[2] << 8) | p[3];
}

// Length of the token at p (header + payload, not the elements of a
// container) and the number of elements it opens; every header byte must be
// readable (header_bytes). false: not a msgpack type byte (0xc1).
inline bool token_c0(const uint8_t* p, uint64_t* adv, uint64_t* opens) {
  const uint8_t t = p[0];
  uint64_t a = 1, o = 0;
  switch (t) {
    case 0xc0: case 0xc2: case 0xc3: break;
    case 0xcc: case 0xd0: a = 2; break;
    case 0xcd: case 0xd1: a = 3; break;
    case 0xce: case 0xd2: case 0xca: a = 5; break;
    case 0xcf: case 0xd3: case 0xcb: a = 9; break;
    case 0xd4: a = 3; break;
    case 0xd5: a = 4; break;
    case 0xd6: a = 6; break;
    case 0xd7: a = 10; break;
    case 0xd8: a = 18; break;
    case 0xd9: case 0xc4: a = 2 + p[1]; break;
    case 0xda: case 0xc5: a = 3 + be16(p + 1); break;
    case 0xdb: case 0xc6: a = 5 + be32(p + 1); break;
    case 0xc7: a = 3 + p[1]; break;
    case 0xc8: a = 4 + be16(p + 1); break;
    case 0xc9: a = 6 + be32(p + 1); break;
    case 0xdc: a = 3; o = be16(p + 1); break;
    case 0xde: a = 3; o = 2 * be16(p + 1); break;
    case 0xdd: a = 5; o = be32(p + 1); break;
    case 0xdf: a = 5; o = 2 * be32(p + 1); break;
    default: return false;
  }
  *adv = a;
  *opens = o;
  return true;
}

void set_nonblock(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

}  // namespace

// The walk keeps one count, the objects still to skip (a container adds its
// elements), so its state is two integers; payloads are skipped without being
// read, so the position may run past the bytes received so far. The common
// one-byte forms (fixint, fixstr, fixarray, fixmap) are decoded inline while a
// full header is in bounds; the 9-byte guard covers every header.
int frame_resume(const uint8_t* b, size_t n, FrameState& st) {
  if (!st.started) {
    st.started = true;
    st.pos = 0;
    st.rem = 1;
  }
  uint64_t pos = st.pos, rem = st.rem;
  if (rem && pos + 9 <= n) {
    // pointer form: the chain per token is load -> length -> add (no index add)
    const uint8_t* p = b + pos;
    const uint8_t* const pend = b + n - 9;
    while (rem && p <= pend) {
      const uint8_t t = *p;
      --rem;
      if ((t & 0xe0) == 0xa0) { p += 1 + (t & 0x1f); continue; }
      if (t < 0x80 || t >= 0xe0) { ++p; continue; }
      if (t < 0xa0) { rem += (t < 0x90) ? 2u * (t & 0x0f) : (t & 0x0fu); ++p; continue; }
      uint64_t adv, opens;
      if (!token_c0(p, &adv, &opens)) return -1;
      p += adv;
      rem += opens;
    }
    pos = (uint64_t)(p - b);
  }
  while (rem) {
    if (pos >= n) break;
    const uint8_t* p = b + pos;
    const uint8_t t = p[0];
    uint64_t adv = 1, opens = 0;
    if ((t & 0xe0) == 0xa0) adv = 1 + (t & 0x1f);
    else if (t < 0x80 || t >= 0xe0) adv = 1;
    else if (t < 0xa0) opens = (t < 0x90) ? 2u * (t & 0x0f) : (t & 0x0fu);
    else {
      if (pos + header_bytes(t) > n) break;
      if (!token_c0(p, &adv, &opens)) return -1;
    }
    --rem;
    pos += adv;
    rem += opens;
  }
  st.pos = pos;
  st.rem = rem;
  if (rem > ((uint64_t)1 << 40)) return -1;    // more elements than any message has bytes
  return (rem == 0 && pos <= n) ? 1 : 0;
}

namespace {

// one token at b[pos] (9 readable bytes): advances pos, returns the change of
// the objects-remaining count (elements opened - 1); false on 0xc1
inline bool frame_step(const uint8_t* b, uint64_t* pos, int64_t* delta) {
  const uint8_t t = b[*pos];
  if ((t & 0xe0) == 0xa0) { *pos += 1 + (t & 0x1f); *delta = -1; return true; }
  if (t < 0x80 || t >= 0xe0) { *pos += 1; *delta = -1; return true; }
  if (t < 0xa0) {
    *delta = (int64_t)((t < 0x90) ? 2 * (t & 0x0f) : (t & 0x0f)) - 1;
    *pos += 1;
    return true;
  }
  uint64_t adv, opens;
  if (!token_c0(b + *pos, &adv, &opens)) return false;
  *pos += adv;
  *delta = (int64_t)opens - 1;
  return true;
}

// sequential framing of every complete message from the state st
int frame_all_seq(const uint8_t* b, size_t n, uint64_t base, FrameState& st,
                  std::vector<uint64_t>* ends) {
  for (;;) {
    const int r = frame_resume(b + base, n - base, st);
    if (r <= 0) return r;
    base += st.pos;
    ends->push_back(base);
    st.reset();
    if (base >= n) return 0;
  }
}

constexpr size_t kSpecMin = 32 << 10;      // buffers shorter than this: one walk
constexpr size_t kSpecChunk = 8 << 10;     // bytes per speculative walk
constexpr int kSpecMax = 8;                // walks
constexpr size_t kSpecWindow = 512 << 10;  // bytes framed speculatively per call

struct SpecWalk {
  std::vector<uint64_t> pos;   // token starts
  std::vector<int64_t> d;      // remaining-count change of each token
  uint64_t x = 0, end = 0;     // current position, region end
  bool live = false;
};

}  // namespace

// Speculative framing (the CPU twin of csrc/hip/scan.hip's chunk walks): a
// message's length is only known by walking every token, a chain of dependent
// loads (~7 cycles a token). Large buffers are cut into up to 8 regions; a walk
// starts at each region's first byte as if a token started there (msgpack
// re-synchronises within a few tokens) and the walks advance in lockstep, so
// the core overlaps their load chains. The true walk (from the message start)
// then follows each region's recorded tokens from the first position they
// share, and message ends are where the true remaining count reaches zero.
// Walks that decode garbage are harmless: only tokens at or after a position
// the true walk itself reached are used.
int frame_all(const uint8_t* b, size_t n, FrameState& st, std::vector<uint64_t>* ends,
              bool speculative) {
  if (!st.started) {
    st.started = true;
    st.pos = 0;
    st.rem = 1;
  }
  if (!speculative || st.pos >= n || n - st.pos < kSpecMin || st.rem == 0)
    return frame_all_seq(b, n, 0, st, ends);
  thread_local SpecWalk w[kSpecMax];
  const uint64_t p0 = st.pos;
  const uint64_t lim = std::min<uint64_t>(n, p0 + kSpecWindow);   // speculate over a window
  const int K = (int)std::min<uint64_t>(kSpecMax, (lim - p0) / kSpecChunk);
  const uint64_t span = (lim - p0) / (uint64_t)K;
  const uint64_t fast_end = lim - 9;           // a step needs 9 readable bytes
  // the true walk runs region 0 and reports message ends as it goes
  uint64_t x = p0, last_end = 0;
  int64_t L = (int64_t)st.rem;
  for (int j = 1; j < K; ++j) {
    SpecWalk& s = w[j];
    s.pos.clear();
    s.d.clear();
    s.x = p0 + span * (uint64_t)j;
    s.end = (j + 1 < K) ? p0 + span * (uint64_t)(j + 1) : fast_end;
    s.live = true;
    s.pos.reserve(span / 2);
    s.d.reserve(span / 2);
  }
  const uint64_t end0 = p0 + span;
  bool live0 = true;
  for (bool any = true; any;) {
    any = false;
    if (live0) {
      if (x < end0 && x <= fast_end) {
        int64_t dd;
        if (!frame_step(b, &x, &dd)) return -1;
        L += dd;
        if (L == 0) {
          if (x > n) { st.pos = x - last_end; st.rem = 0; return 0; }
          ends->push_back(x);
          last_end = x;
          L = 1;
        }
        any = true;
      } else {
        live0 = false;
      }
    }
    for (int j = 1; j < K; ++j) {
      SpecWalk& s = w[j];
      if (!s.live) continue;
      if (s.x >= s.end || s.x > fast_end) { s.live = false; continue; }
      const uint64_t at = s.x;
      int64_t dd;
      if (!frame_step(b, &s.x, &dd)) { s.live = false; continue; }
      s.pos.push_back(at);
      s.d.push_back(dd);
      any = true;
    }
  }
  // stitch: follow the true chain through the walks' tokens
  for (int j = 1; j < K; ++j) {
    SpecWalk& s = w[j];
    const size_t m = s.pos.size();
    if (m == 0 || s.pos[m - 1] < x) continue;
    size_t q = (size_t)(std::lower_bound(s.pos.begin(), s.pos.end(), x) - s.pos.begin());
    bool synced = false;
    for (;;) {
      while (q < m && s.pos[q] < x) ++q;
      if (q >= m) break;
      if (s.pos[q] == x) { synced = true; break; }
      if (x > fast_end) break;
      int64_t dd;
      if (!frame_step(b, &x, &dd)) return -1;
      L += dd;
      if (L == 0) {
        if (x > n) { st.pos = x - last_end; st.rem = 0; return 0; }
        ends->push_back(x);
        last_end = x;
        L = 1;
      }
    }
    if (!synced) continue;
    for (size_t t = q; t < m; ++t) {
      L += s.d[t];
      if (L == 0) {
        const uint64_t e = (t + 1 < m) ? s.pos[t + 1] : s.x;
        if (e > n) { st.pos = e - last_end; st.rem = 0; return 0; }
        ends->push_back(e);
        last_end = e;
        L = 1;
      }
    }
    x = s.x;
  }
  // the rest with bounds checks, from the true state
  st.pos = x - last_end;
  st.rem = (uint64_t)L;
  if (L < 0 || st.rem > ((uint64_t)1 << 40)) return -1;
  return frame_all_seq(b, n, last_end, st, ends);
}

uint8_t* RecvBuf::space(size_t want, size_t* got) {
  if (cap_ - tail_ < want) {
    const size_t live = tail_ - head_;
    if (head_ > 0 && cap_ - live >= want && live <= cap_ / 2) {
      memmove(d_.get(), d_.get() + head_, live);     // compact: cheap while little is live
    } else {
      size_t ncap = cap_ ? cap_ : want;
      while (ncap - live < want) ncap *= 2;
      std::unique_ptr<uint8_t[]> nd(new uint8_t[ncap]);
      if (live) memcpy(nd.get(), d_.get() + head_, live);
      d_ = std::move(nd);
      cap_ = ncap;
    }
    head_ = 0;
    tail_ = live;
  }
  *got = cap_ - tail_;
  return d_.get() + tail_;
}

int64_t msgpack_frame(const uint8_t* p, size_t n) {
  FrameState st;
  const int r = frame_resume(p, n, st);
  return r == 1 ? (int64_t)st.pos : r;
}

RpcServer::RpcServer(Handler h, int nworkers, double idle_timeout_sec)
    : handler_(std::move(h)), nworkers_(nworkers < 1 ? 1 : nworkers),
      idle_timeout_(idle_timeout_sec) {
  signal(SIGPIPE, SIG_IGN);
}

RpcServer::~RpcServer() { stop(); }

void RpcServer::set_batch(const std::vector<std::string>& methods, BatchHandler h,
                          size_t max_batch) {
  batch_methods_ = methods;
  batch_handler_ = std::move(h);
  max_batch_ = max_batch ? max_batch : 1;
}

void RpcServer::enqueue(RpcRequest&& req) {
  for (const auto& m : batch_methods_)
    if (m == req.method) {
      if (prep_) prep_(req);
      std::lock_guard<std::mutex> g(bmu_);
      bqueue_.push_back(std::move(req));
      bcv_.notify_all();  // the generic-queue thread must see it
      return;
    }
  std::lock_guard<std::mutex> g(qmu_);
  queue_.push_back(std::move(req));
  qlen_.store(queue_.size(), std::memory_order_relaxed);
  qcv_.notify_one();
}

// Drain every queued request of the method at the head of the batch queue
// and serve them with one handler call; requests arriving meanwhile form
// the next (larger) batch - adaptive batching without a timer.
void RpcServer::batch_loop(int idx) {
  const bool generic = idx == 0;
  for (;;) {
    if (arena_handler_ && arena_batch_once()) continue;
    std::vector<RpcRequest> batch;
    {
      std::unique_lock<std::mutex> g(bmu_);
      bcv_.wait_for(g, std::chrono::milliseconds(arena_handler_ ? 1 : 100), [this, generic] {
        if (!running_.load() || (generic && !bqueue_.empty())) return true;
        if (!arena_handler_) return false;
        std::lock_guard<std::mutex> a(amu_);
        for (const auto& s : slots_)
          if (!s.busy && !s.reqs.empty()) return true;
        return false;
      });
      if (!running_.load()) return;
      if (!generic || bqueue_.empty()) continue;
      const std::string method = bqueue_.front().method;
      auto ordered = [this](const std::string& m) {
        return std::find(ordered_.begin(), ordered_.end(), m) != ordered_.end();
      };
      const bool keep_order = ordered(method);
      for (auto it = bqueue_.begin(); it != bqueue_.end() && batch.size() < max_batch_;) {
        if (it->method == method) {
          batch.push_back(std::move(*it));
          it = bqueue_.erase(it);
        } else {
          if (keep_order || ordered(it->method)) break;
          ++it;
        }
      }
    }
    if (!batch_handler_) {          // arena-only server: an overflow request
      for (auto& r : batch)
        if (!r.notify) {
          std::string o("\x94\x01", 2);
          o.push_back((char)0xce);
          for (int k = 3; k >= 0; --k) o.push_back((char)((r.msgid >> (8 * k)) & 0xff));
          o += "\xa4" "busy" "\xc0";
          send_response(r.conn_id, o);
        }
      continue;
    }
    std::vector<std::string> resp;
    {
      // JUBATUS_ROCTX=1: one range per handed-over batch (rocprofv3 --marker-trace)
      const std::string tag = "rpc.batch." + batch[0].method;
      jb::tx::Range tr(tag.c_str());
      resp = batch_handler_(batch[0].method, batch);
    }
    batches_.fetch_add(1);
    served_.fetch_add(batch.size());
    std::vector<uint64_t> ids(batch.size());
    for (size_t i = 0; i < batch.size(); ++i) {
      ids[i] = batch[i].conn_id;
      if (batch[i].notify && i < resp.size()) resp[i].clear();
    }
    send_responses(ids, resp);
  }
}

int RpcServer::listen(const std::string& addr, int port) {
  listen_fd_ = socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (addr.empty() || addr == "0.0.0.0") sa.sin_addr.s_addr = htonl(INADDR_ANY);
  else if (inet_pton(AF_INET, addr.c_str(), &sa.sin_addr) != 1)
    throw std::runtime_error("bad bind address: " + addr);
  if (::bind(listen_fd_, (sockaddr*)&sa, sizeof(sa)) != 0) {
    int e = errno;
    ::close(listen_fd_);
    listen_fd_ = -1;
    throw std::runtime_error(std::string("bind failed: ") + strerror(e));
  }
  if (::listen(listen_fd_, 1024) != 0) throw std::runtime_error("listen failed");
  set_nonblock(listen_fd_);
  socklen_t len = sizeof(sa);
  getsockname(listen_fd_, (sockaddr*)&sa, &len);
  return ntohs(sa.sin_port);
}

void RpcServer::start() {
  if (listen_fd_ < 0) throw std::runtime_error("listen() first");
  running_.store(true);
  for (int i = 0; i < nio_; ++i) {
    std::unique_ptr<Loop> L(new Loop());
    L->epfd = epoll_create1(0);
    L->wake_fd = eventfd(0, EFD_NONBLOCK);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = UINT64_MAX;  // wakeup
    epoll_ctl(L->epfd, EPOLL_CTL_ADD, L->wake_fd, &ev);
    if (i == 0) {
      ev.data.u64 = 0;  // listen socket lives in loop 0
      epoll_ctl(L->epfd, EPOLL_CTL_ADD, listen_fd_, &ev);
    }
    loops_.push_back(std::move(L));
  }
  // named threads: per-thread CPU time is attributable (/proc/<pid>/task/*/comm)
  for (int i = 0; i < nio_; ++i)
    loops_[i]->th = std::thread([this, i] {
      pthread_setname_np(pthread_self(), "jb-rpc-io");
      io_loop(i);
    });
  for (int i = 0; i < nworkers_; ++i)
    workers_.emplace_back([this] {
      pthread_setname_np(pthread_self(), "jb-rpc-worker");
      worker_loop();
    });
  if (batch_handler_ || arena_handler_)
    for (int i = 0; i < nbatch_; ++i)
      batchers_.emplace_back([this, i] {
        pthread_setname_np(pthread_self(), "jb-rpc-batch");
        batch_loop(i);
      });
}

void RpcServer::stop() {
  if (!running_.exchange(false)) return;
  uint64_t one = 1;
  for (auto& L : loops_)
    if (L->wake_fd >= 0) { ssize_t r = write(L->wake_fd, &one, 8); (void)r; }
  qcv_.notify_all();
  {
    std::lock_guard<std::mutex> g(bmu_);
    bcv_.notify_all();
  }
  for (auto& L : loops_)
    if (L->th.joinable()) L->th.join();
  for (auto& b : batchers_)
    if (b.joinable()) b.join();
  batchers_.clear();
  for (auto& w : workers_) if (w.joinable()) w.join();
  workers_.clear();
  {
    std::lock_guard<std::mutex> g(cmu_);
    for (auto& kv : conns_) ::close(kv.second->fd);
    conns_.clear();
  }
  if (listen_fd_ >= 0) ::close(listen_fd_);
  for (auto& L : loops_) {
    if (L->epfd >= 0) ::close(L->epfd);
    if (L->wake_fd >= 0) ::close(L->wake_fd);
  }
  loops_.clear();
  listen_fd_ = -1;
}

void RpcServer::close_conn(uint64_t id) {
  std::shared_ptr<Conn> c;
  {
    std::lock_guard<std::mutex> g(cmu_);
    auto it = conns_.find(id);
    if (it == conns_.end()) return;
    c = it->second;
    conns_.erase(it);
  }
  {
    std::lock_guard<std::mutex> g(c->wmu);
    c->closed = true;
  }
  epoll_ctl(loops_[c->loop]->epfd, EPOLL_CTL_DEL, c->fd, nullptr);
  ::close(c->fd);
  nconn_.fetch_sub(1);
}

void RpcServer::io_loop(int li) {
  Loop& L = *loops_[li];
  epoll_event evs[256];
  double last_sweep = now_sec();
  while (running_.load()) {
    int n = epoll_wait(L.epfd, evs, 256, 100);
    for (int i = 0; i < n; ++i) {
      const uint64_t key = evs[i].data.u64;
      if (key == UINT64_MAX) {
        uint64_t v;
        ssize_t r = read(L.wake_fd, &v, 8);
        (void)r;
        std::vector<uint64_t> ids;
        {
          std::lock_guard<std::mutex> g(L.wq_mu);
          ids.swap(L.want_write);
        }
        for (uint64_t id : ids) {
          std::shared_ptr<Conn> c;
          {
            std::lock_guard<std::mutex> g(cmu_);
            auto it = conns_.find(id);
            if (it != conns_.end()) c = it->second;
          }
          if (!c) continue;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLOUT;
          ev.data.u64 = id;
          epoll_ctl(L.epfd, EPOLL_CTL_MOD, c->fd, &ev);
        }
        continue;
      }
      if (key == 0) {  // accept
        for (;;) {
          int fd = accept(listen_fd_, nullptr, nullptr);
          if (fd < 0) break;
          set_nonblock(fd);
          int one = 1;
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          auto c = std::make_shared<Conn>();
          c->fd = fd;
          c->last_active = now_sec();
          c->loop = (int)(next_loop_.fetch_add(1) % (uint64_t)nio_);
          {
            std::lock_guard<std::mutex> g(cmu_);
            c->id = next_id_++;
            conns_[c->id] = c;
          }
          nconn_.fetch_add(1);
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.u64 = c->id;
          epoll_ctl(loops_[c->loop]->epfd, EPOLL_CTL_ADD, fd, &ev);
        }
        continue;
      }
      std::shared_ptr<Conn> c;
      {
        std::lock_guard<std::mutex> g(cmu_);
        auto it = conns_.find(key);
        if (it != conns_.end()) c = it->second;
      }
      if (!c) continue;
      if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
        // drain what is readable first (a peer may send then close)
        on_readable(c);
        close_conn(key);
        continue;
      }
      if (evs[i].events & EPOLLIN) on_readable(c);
      if (evs[i].events & EPOLLOUT) {
        flush(c);
        std::lock_guard<std::mutex> g(c->wmu);
        if (c->wbuf.empty() && !c->closed) {
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.u64 = c->id;
          epoll_ctl(L.epfd, EPOLL_CTL_MOD, c->fd, &ev);
          c->want_write = false;
        }
      }
    }
    const double t = now_sec();
    if (idle_timeout_ > 0 && t - last_sweep > 1.0) {
      last_sweep = t;
      std::vector<uint64_t> idle;
      {
        std::lock_guard<std::mutex> g(cmu_);
        for (auto& kv : conns_)
          if (kv.second->loop == li && t - kv.second->last_active > idle_timeout_)
            idle.push_back(kv.first);
      }
      for (uint64_t id : idle) close_conn(id);
    }
  }
}

void RpcServer::on_readable(const std::shared_ptr<Conn>& c) {
  bool eof = false;
  for (;;) {
    size_t room;
    uint8_t* dst = c->rbuf.space(65536, &room);
    ssize_t r = ::read(c->fd, dst, room);
    if (r > 0) {
      c->rbuf.produced((size_t)r);
      if ((size_t)r < room) break;      // drained (the next read would say EAGAIN)
      continue;
    }
    if (r == 0) eof = true;
    else if (errno == EINTR) continue;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
    break;
  }
  c->last_active = now_sec();
  const uint8_t* base = c->rbuf.data();
  const size_t total = c->rbuf.size();
  thread_local std::vector<uint64_t> ends;
  ends.clear();
  if (frame_all(base, total, c->fs, &ends) < 0) eof = true;
  if (c->fs.started && (c->fs.pos > max_message_ ||
                        total - (ends.empty() ? 0 : ends.back()) > max_message_))
    eof = true;                                  // refuse oversized messages
  size_t pos = 0;
  for (const uint64_t e : ends) {
    const uint8_t* p = base + pos;
    const int64_t len = (int64_t)(e - pos);
    Cursor cur{p, p + len};
    uint32_t n;
    double type = -1, msgid = 0;
    const uint8_t* m = nullptr;
    uint32_t mlen = 0;
    bool ok = cur.array(&n) && (n == 4 || n == 3) && cur.number(&type);
    if (ok && n == 4 && type == 0) {
      ok = cur.number(&msgid) && cur.raw(&m, &mlen);
      if (ok) {
        bool taken = false;
        if (!arena_method_.empty() && mlen == arena_method_.size() &&
            memcmp(m, arena_method_.data(), mlen) == 0) {
          // params = [name, body]: the body goes straight into an arena slot
          Cursor pc{cur.p, p + len};
          uint32_t np;
          const uint8_t* nm;
          uint32_t nlen;
          if (pc.array(&np) && np == 2 && pc.raw(&nm, &nlen))
            taken = arena_take(c->id, (uint32_t)msgid, pc.p, (size_t)(p + len - pc.p));
        }
        if (!taken)
          enqueue(RpcRequest{c->id, (uint32_t)msgid, false, std::string((const char*)m, mlen),
                             std::string((const char*)cur.p, (size_t)(p + len - cur.p))});
      }
    } else if (ok && n == 3 && type == 2) {
      ok = cur.raw(&m, &mlen);
      if (ok) {
        enqueue(RpcRequest{c->id, 0, true, std::string((const char*)m, mlen),
                           std::string((const char*)cur.p, (size_t)(p + len - cur.p))});
      }
    } else if (ok && n == 4 && type == 1) {
      ok = true;   // responses sent to a server are ignored
    }
    if (!ok) { eof = true; break; }   // not an RPC envelope: no msgid to answer, drop the peer
    pos += (size_t)len;
  }
  if (pos) c->rbuf.consume(pos);
  if (eof) close_conn(c->id);
}

// ---------------------------------------------------------- arena batching
void RpcServer::set_arena_batch(const std::string& method, const std::vector<uint8_t*>& slots,
                                size_t slot_bytes, ArenaHandler h) {
  arena_method_ = method;
  arena_handler_ = std::move(h);
  slot_bytes_ = slot_bytes;
  slots_.assign(slots.size(), Slot());
  for (size_t i = 0; i < slots.size(); ++i) slots_[i].base = slots[i];
  open_ = -1;
}

void RpcServer::release_slot(int slot) {
  std::lock_guard<std::mutex> g(amu_);
  if (slot < 0 || slot >= (int)slots_.size()) return;
  slots_[slot].busy = false;
  slots_[slot].used = 0;
  slots_[slot].reqs.clear();
  acv_.notify_all();
}

// IO thread: reserve room in the open slot (opening a free one if needed),
// copy the body outside the lock. false: no room anywhere (caller falls
// back to the ordinary batch path).
bool RpcServer::arena_take(uint64_t conn_id, uint32_t msgid, const uint8_t* body, size_t len) {
  const uint64_t need = (len + 15) & ~(uint64_t)15;
  if (need > slot_bytes_) return false;
  int k;
  uint64_t off;
  bool first;
  {
    std::lock_guard<std::mutex> g(amu_);
    if (open_ >= 0 && slots_[open_].used + need > slot_bytes_) open_ = -1;   // full: batcher seals it
    if (open_ < 0) {
      for (size_t i = 0; i < slots_.size(); ++i) {
        Slot& s = slots_[i];
        if (!s.busy && s.reqs.empty() && s.writers == 0) { open_ = (int)i; break; }
      }
      if (open_ < 0) return false;
    }
    k = open_;
    Slot& s = slots_[k];
    off = s.used;
    s.used += need;
    ++s.writers;
    s.reqs.push_back(ArenaReq{conn_id, msgid, off, (uint64_t)len});
    first = s.reqs.size() == 1;
  }
  memcpy(slots_[k].base + off, body, len);
  {
    std::lock_guard<std::mutex> g(amu_);
    if (--slots_[k].writers == 0) acv_.notify_all();
  }
  if (first) {     // a batch thread looks at non-empty slots; later arrivals need no wakeup
    std::lock_guard<std::mutex> g(bmu_);
    bcv_.notify_one();
  }
  return true;
}

// Batch thread: seal the fullest slot that holds requests (the open one
// included), wait until its copies landed, hand it to the handler.
bool RpcServer::arena_batch_once() {
  int k = -1;
  std::vector<ArenaReq> reqs;
  {
    std::unique_lock<std::mutex> g(amu_);
    for (size_t i = 0; i < slots_.size(); ++i)
      if (!slots_[i].busy && !slots_[i].reqs.empty() &&
          (k < 0 || slots_[i].used > slots_[k].used))
        k = (int)i;
    if (k < 0) return false;
    if (open_ == k) open_ = -1;                 // sealed: new bodies go elsewhere
    Slot& s = slots_[k];
    s.busy = true;
    acv_.wait(g, [&] { return s.writers == 0; });
    reqs.swap(s.reqs);
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::string> resp;
  {
    jb::tx::Range tr("rpc.arena_batch");
    resp = arena_handler_(k, reqs);
  }
  const auto t1 = std::chrono::steady_clock::now();
  batches_.fetch_add(1);
  served_.fetch_add(reqs.size());
  std::vector<uint64_t> ids(reqs.size());
  for (size_t i = 0; i < reqs.size(); ++i) ids[i] = reqs[i].conn_id;
  send_responses(ids, resp);
  const auto t2 = std::chrono::steady_clock::now();
  arena_handler_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
  arena_send_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count());
  return true;
}

// Responses of one batch: those of a connection are joined and written
// with one send (a batch of ~hundreds of requests from tens of connections
// costs tens of syscalls, not hundreds).
void RpcServer::send_responses(const std::vector<uint64_t>& conn_ids,
                               const std::vector<std::string>& resp) {
  const size_t n = std::min(conn_ids.size(), resp.size());
  std::vector<std::pair<uint64_t, size_t>> order;
  order.reserve(n);
  for (size_t i = 0; i < n; ++i)
    if (!resp[i].empty()) order.emplace_back(conn_ids[i], i);
  std::stable_sort(order.begin(), order.end(),
                   [](const std::pair<uint64_t, size_t>& a, const std::pair<uint64_t, size_t>& b) {
                     return a.first < b.first;
                   });
  std::string joined;
  for (size_t i = 0; i < order.size();) {
    size_t j = i;
    joined.clear();
    while (j < order.size() && order[j].first == order[i].first) joined += resp[order[j++].second];
    send_response(order[i].first, joined);
    i = j;
  }
}

void RpcServer::flush(const std::shared_ptr<Conn>& c) {
  std::lock_guard<std::mutex> g(c->wmu);
  while (!c->wbuf.empty() && !c->closed) {
    ssize_t w = ::send(c->fd, c->wbuf.data(), c->wbuf.size(), MSG_NOSIGNAL);
    if (w > 0) { c->wbuf.erase(0, (size_t)w); continue; }
    if (w < 0 && errno == EINTR) continue;
    break;  // EAGAIN or error: the IO thread retries on EPOLLOUT / HUP
  }
}

void RpcServer::send_response(uint64_t conn_id, const std::string& bytes) {
  std::shared_ptr<Conn> c;
  {
    std::lock_guard<std::mutex> g(cmu_);
    auto it = conns_.find(conn_id);
    if (it == conns_.end()) return;  // client went away
    c = it->second;
  }
  bool arm = false;
  {
    std::lock_guard<std::mutex> g(c->wmu);
    if (c->closed) return;
    c->wbuf.append(bytes);
  }
  flush(c);
  {
    std::lock_guard<std::mutex> g(c->wmu);
    if (!c->wbuf.empty() && !c->want_write) { c->want_write = true; arm = true; }
  }
  if (arm) {
    Loop& L = *loops_[c->loop];
    {
      std::lock_guard<std::mutex> g(L.wq_mu);
      L.want_write.push_back(conn_id);
    }
    uint64_t one = 1;
    ssize_t r = write(L.wake_fd, &one, 8);
    (void)r;
  }
}

void RpcServer::worker_loop() {
  bool busy = false;
  for (;;) {
    RpcRequest req;
    if (busy) {
      // spin briefly after a request before parking on the condition
      // variable: back-to-back requests skip the futex wakeup (~10-20 us)
      const double t0 = now_sec();
      while (qlen_.load(std::memory_order_relaxed) == 0 && running_.load(std::memory_order_relaxed) &&
             now_sec() - t0 < 50e-6)
        __builtin_ia32_pause();
    }
    {
      std::unique_lock<std::mutex> g(qmu_);
      qcv_.wait(g, [this] { return !queue_.empty() || !running_.load(); });
      if (!running_.load()) return;
      req = std::move(queue_.front());
      queue_.pop_front();
      qlen_.store(queue_.size(), std::memory_order_relaxed);
    }
    busy = true;
    std::string resp;
    if (jb::tx::enabled()) {
      const std::string tag = "rpc." + req.method;
      jb::tx::Range tr(tag.c_str());
      resp = handler_(req);
    } else {
      resp = handler_(req);
    }
    served_.fetch_add(1);
    if (!req.notify && !resp.empty()) send_response(req.conn_id, resp);
  }
}

}  // namespace jb
