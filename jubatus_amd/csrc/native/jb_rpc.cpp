// See jb_rpc.hpp.
#include "jb_rpc.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <stdexcept>

#include "jb_msgpack.hpp"

namespace jb {

namespace {

double now_sec() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// skip one object: 1 ok, 0 incomplete, -1 malformed
int skip_status(Cursor& c, int depth) {
  if (depth > 128) return -1;
  if (!c.need(1)) return 0;
  const uint8_t t = *c.p;
  auto take = [&](uint64_t n) -> int {
    if (!c.need(n)) return 0;
    c.p += n;
    return 1;
  };
  auto be = [&](int off, int nb) -> uint64_t {
    uint64_t v = 0;
    for (int i = 0; i < nb; ++i) v = (v << 8) | c.p[off + i];
    return v;
  };
  if (t <= 0x7f || t >= 0xe0 || t == 0xc0 || t == 0xc2 || t == 0xc3) return take(1);
  if ((t & 0xe0) == 0xa0) return take(1 + (t & 0x1f));
  if ((t & 0xf0) == 0x90 || (t & 0xf0) == 0x80) {
    uint64_t n = (t & 0x0f) * (((t & 0xf0) == 0x80) ? 2 : 1);
    c.p += 1;
    for (uint64_t i = 0; i < n; ++i) {
      int r = skip_status(c, depth + 1);
      if (r <= 0) return r;
    }
    return 1;
  }
  switch (t) {
    case 0xcc: case 0xd0: return take(2);
    case 0xcd: case 0xd1: return take(3);
    case 0xce: case 0xd2: case 0xca: return take(5);
    case 0xcf: case 0xd3: case 0xcb: return take(9);
    case 0xd9: case 0xc4: if (!c.need(2)) return 0; return take(2 + be(1, 1));
    case 0xda: case 0xc5: if (!c.need(3)) return 0; return take(3 + be(1, 2));
    case 0xdb: case 0xc6: if (!c.need(5)) return 0; return take(5 + be(1, 4));
    case 0xd4: return take(3); case 0xd5: return take(4); case 0xd6: return take(6);
    case 0xd7: return take(10); case 0xd8: return take(18);
    case 0xc7: if (!c.need(2)) return 0; return take(3 + be(1, 1));
    case 0xc8: if (!c.need(3)) return 0; return take(4 + be(1, 2));
    case 0xc9: if (!c.need(5)) return 0; return take(6 + be(1, 4));
    case 0xdc: case 0xdd: case 0xde: case 0xdf: {
      const int nb = (t == 0xdc || t == 0xde) ? 2 : 4;
      if (!c.need(1 + nb)) return 0;
      uint64_t n = be(1, nb) * ((t == 0xde || t == 0xdf) ? 2 : 1);
      c.p += 1 + nb;
      for (uint64_t i = 0; i < n; ++i) {
        int r = skip_status(c, depth + 1);
        if (r <= 0) return r;
      }
      return 1;
    }
    default: return -1;
  }
}

void set_nonblock(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

}  // namespace

int frame_resume(const uint8_t* b, size_t n, FrameState& st) {
  for (;;) {
    if (st.started && st.stack.empty()) return 1;
    if (st.pos >= n) return 0;
    const uint8_t* p = b + st.pos;
    const uint8_t t = p[0];
    auto have = [&](uint64_t k) { return st.pos + k <= n; };
    auto be = [&](int off, int nb) -> uint64_t {
      uint64_t v = 0;
      for (int i = 0; i < nb; ++i) v = (v << 8) | p[off + i];
      return v;
    };
    uint64_t hdr = 1, payload = 0, count = 0;
    bool container = false;
    if (t <= 0x7f || t >= 0xe0 || t == 0xc0 || t == 0xc2 || t == 0xc3) {
    } else if ((t & 0xe0) == 0xa0) {
      payload = t & 0x1f;
    } else if ((t & 0xf0) == 0x90) {
      container = true; count = t & 0x0f;
    } else if ((t & 0xf0) == 0x80) {
      container = true; count = 2u * (t & 0x0f);
    } else {
      switch (t) {
        case 0xcc: case 0xd0: payload = 1; break;
        case 0xcd: case 0xd1: payload = 2; break;
        case 0xce: case 0xd2: case 0xca: payload = 4; break;
        case 0xcf: case 0xd3: case 0xcb: payload = 8; break;
        case 0xd9: case 0xc4: if (!have(2)) return 0; hdr = 2; payload = be(1, 1); break;
        case 0xda: case 0xc5: if (!have(3)) return 0; hdr = 3; payload = be(1, 2); break;
        case 0xdb: case 0xc6: if (!have(5)) return 0; hdr = 5; payload = be(1, 4); break;
        case 0xd4: payload = 2; break;
        case 0xd5: payload = 3; break;
        case 0xd6: payload = 5; break;
        case 0xd7: payload = 9; break;
        case 0xd8: payload = 17; break;
        case 0xc7: if (!have(2)) return 0; hdr = 2; payload = 1 + be(1, 1); break;
        case 0xc8: if (!have(3)) return 0; hdr = 3; payload = 1 + be(1, 2); break;
        case 0xc9: if (!have(5)) return 0; hdr = 5; payload = 1 + be(1, 4); break;
        case 0xdc: case 0xde:
          if (!have(3)) return 0;
          hdr = 3; container = true; count = be(1, 2) * (t == 0xde ? 2 : 1); break;
        case 0xdd: case 0xdf:
          if (!have(5)) return 0;
          hdr = 5; container = true; count = be(1, 4) * (t == 0xdf ? 2 : 1); break;
        default: return -1;
      }
    }
    if (!have(hdr + payload)) return 0;
    st.pos += hdr + payload;
    st.started = true;
    if (container && count > 0) {
      if (st.stack.size() >= 128) return -1;
      st.stack.push_back(count);
      continue;
    }
    while (!st.stack.empty()) {        // one element done
      if (--st.stack.back() > 0) break;
      st.stack.pop_back();
    }
  }
}

int64_t msgpack_frame(const uint8_t* p, size_t n) {
  Cursor c{p, p + n};
  int r = skip_status(c, 0);
  if (r == 0) return 0;
  if (r < 0) return -1;
  return (int64_t)(c.p - p);
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
      std::lock_guard<std::mutex> g(bmu_);
      bqueue_.push_back(std::move(req));
      bcv_.notify_one();
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
void RpcServer::batch_loop() {
  for (;;) {
    if (arena_handler_ && arena_batch_once()) continue;
    std::vector<RpcRequest> batch;
    {
      std::unique_lock<std::mutex> g(bmu_);
      bcv_.wait_for(g, std::chrono::milliseconds(arena_handler_ ? 1 : 100), [this] {
        if (!bqueue_.empty() || !running_.load()) return true;
        if (!arena_handler_) return false;
        std::lock_guard<std::mutex> a(amu_);
        for (const auto& s : slots_)
          if (!s.busy && !s.reqs.empty()) return true;
        return false;
      });
      if (!running_.load()) return;
      if (bqueue_.empty()) continue;
      const std::string method = bqueue_.front().method;
      for (auto it = bqueue_.begin(); it != bqueue_.end() && batch.size() < max_batch_;) {
        if (it->method == method) {
          batch.push_back(std::move(*it));
          it = bqueue_.erase(it);
        } else {
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
          o += "\xa4busy\xc0";
          send_response(r.conn_id, o);
        }
      continue;
    }
    std::vector<std::string> resp = batch_handler_(batch[0].method, batch);
    batches_.fetch_add(1);
    served_.fetch_add(batch.size());
    for (size_t i = 0; i < batch.size() && i < resp.size(); ++i)
      if (!batch[i].notify && !resp[i].empty()) send_response(batch[i].conn_id, resp[i]);
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
  for (int i = 0; i < nio_; ++i) loops_[i]->th = std::thread([this, i] { io_loop(i); });
  for (int i = 0; i < nworkers_; ++i) workers_.emplace_back([this] { worker_loop(); });
  if (batch_handler_ || arena_handler_)
    for (int i = 0; i < nbatch_; ++i) batchers_.emplace_back([this] { batch_loop(); });
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
  char tmp[65536];
  bool eof = false;
  for (;;) {
    ssize_t r = ::read(c->fd, tmp, sizeof(tmp));
    if (r > 0) { c->rbuf.append(tmp, (size_t)r); continue; }
    if (r == 0) eof = true;
    else if (errno == EINTR) continue;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
    break;
  }
  c->last_active = now_sec();
  size_t pos = 0;
  while (pos < c->rbuf.size()) {
    const uint8_t* p = (const uint8_t*)c->rbuf.data() + pos;
    const size_t avail = c->rbuf.size() - pos;
    const int fr = frame_resume(p, avail, c->fs);
    if (fr == 0) {
      // incomplete: keep the walk's state; refuse oversized messages
      if (c->fs.pos > max_message_ || avail > max_message_) eof = true;
      break;
    }
    if (fr < 0) { eof = true; break; }
    const int64_t len = (int64_t)c->fs.pos;
    c->fs.reset();
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
  if (pos) c->rbuf.erase(0, pos);
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
  }
  memcpy(slots_[k].base + off, body, len);
  {
    std::lock_guard<std::mutex> g(amu_);
    if (--slots_[k].writers == 0) acv_.notify_all();
  }
  {
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
  std::vector<std::string> resp = arena_handler_(k, reqs);
  batches_.fetch_add(1);
  served_.fetch_add(reqs.size());
  for (size_t i = 0; i < reqs.size() && i < resp.size(); ++i)
    if (!resp[i].empty()) send_response(reqs[i].conn_id, resp[i]);
  return true;
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
    std::string resp = handler_(req);
    served_.fetch_add(1);
    if (!req.notify && !resp.empty()) send_response(req.conn_id, resp);
  }
}

}  // namespace jb
