// jubaloadgen: native msgpack-RPC load generator (benchmarks of the servers'
// request path without a Python client in the way).
//
// Sends pre-encoded requests (params = msgpack arrays read from a file, e.g.
// ["", [[label, datum]...]] for train; several params objects concatenated in
// the file are sent in turn, each connection starting at its own one) on C
// connections, each keeping D requests in flight, for T seconds; prints one
// JSON line with the request rate and the per-request latency distribution.
// Any error response aborts. Every request the in-flight window allows goes
// out in one sendmsg (envelope + params iovecs, no per-request copy of the
// params), as a pipelining client library would write them.
//
// -o 1 (once): every params object is sent exactly once - connection i takes
// the i-th contiguous share of the file - and the run ends when all replied
// (bulk loads: each row once, in file order per connection).
//
// -r SEED (fresh, with -t): train params only ([name, [[label, datum]...]]).
// Every sample sent carries freshly drawn values: the first float64 of its
// datum's num_values becomes v + N(0, 1/4) and the digits of its last string
// value are redrawn (a new token of the same length: a feature the model has
// likely not seen), from a per-connection splitmix64 stream. Each connection
// owns `depth` private copies of params objects and refreshes one in place
// just before it goes out, so no two samples of a run are alike - the model
// keeps meeting data it has not seen, as in the in-process bench's
// non-repeating stream - at the cost of a few draws per sample, no copy.
//
// -u N (with -r): N per mille of the samples sent get new digits in every
// string value instead (all their tokens unseen: the model updates on them) -
// a stream that keeps learning.
//
// Usage: jubaloadgen -p PORT -m METHOD -f PARAMS.bin [-H HOST] [-c CONNS] [-d DEPTH] [-t SECONDS]
//                    [-o 1] [-r SEED [-u N]]
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/tcp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "jb_msgpack.hpp"
#include "jb_rpc.hpp"

namespace {

using Clock = std::chrono::steady_clock;

// envelope head [0, msgid, method, (params follow)
std::string request_head(uint32_t msgid, const std::string& method) {
  std::string o;
  o.push_back((char)0x94);
  o.push_back((char)0x00);
  o.push_back((char)0xce);
  for (int k = 3; k >= 0; --k) o.push_back((char)((msgid >> (8 * k)) & 0xff));
  const size_t n = method.size();
  if (n < 32) o.push_back((char)(0xa0 | n));
  else { o.push_back((char)0xda); o.push_back((char)(n >> 8)); o.push_back((char)n); }
  o += method;
  return o;
}

// several requests (head + params each) with as few sendmsg calls as the
// socket takes
bool send_many(int fd, const std::vector<std::string>& heads,
               const std::vector<const std::string*>& bodies) {
  std::vector<iovec> iov;
  iov.reserve(2 * heads.size());
  for (size_t i = 0; i < heads.size(); ++i) {
    iov.push_back(iovec{(void*)heads[i].data(), heads[i].size()});
    iov.push_back(iovec{(void*)bodies[i]->data(), bodies[i]->size()});
  }
  size_t k = 0;
  while (k < iov.size()) {
    msghdr m{};
    m.msg_iov = iov.data() + k;
    m.msg_iovlen = std::min<size_t>(iov.size() - k, 1024);
    const ssize_t w = sendmsg(fd, &m, MSG_NOSIGNAL);
    if (w <= 0) return false;
    size_t left = (size_t)w;
    while (left > 0 && k < iov.size()) {            // drop what went out
      if (left >= iov[k].iov_len) { left -= iov[k].iov_len; ++k; continue; }
      iov[k].iov_base = (char*)iov[k].iov_base + left;
      iov[k].iov_len -= left;
      left = 0;
    }
  }
  return true;
}

int connect_to(const std::string& host, int port) {
  addrinfo hints{}, *ai = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &ai) != 0) return -1;
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0 || connect(fd, ai->ai_addr, ai->ai_addrlen) != 0) {
    freeaddrinfo(ai);
    if (fd >= 0) close(fd);
    return -1;
  }
  freeaddrinfo(ai);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  return fd;
}

// what a fresh send redraws in a train params object: the float64 payload
// of the first numeric value of every sample, and the decimal digits of the
// last string value of every sample (empty: not that layout)
struct FreshSlots {
  std::vector<uint32_t> f64;                          // payload offsets
  std::vector<std::pair<uint32_t, uint32_t>> digits;  // (offset, length) runs
  // -u: the digit runs of every string value, per sample [all_begin[i], all_begin[i + 1])
  std::vector<std::pair<uint32_t, uint32_t>> all;
  std::vector<uint32_t> all_begin{0};
  bool empty() const { return f64.empty(); }
};

FreshSlots fresh_slots(const std::string& prm) {
  FreshSlots out;
  const uint8_t* b = (const uint8_t*)prm.data();
  jb::Cursor c{b, b + prm.size()};
  uint32_t n, ns;
  const uint8_t* s;
  if (!c.array(&n) || n != 2 || !c.raw(&s, &n) || !c.array(&ns)) return {};
  for (uint32_t i = 0; i < ns; ++i) {
    uint32_t two, three, nn, sn;
    if (!c.array(&two) || two != 2 || !c.raw(&s, &n) || !c.array(&three) || three < 2) return {};
    if (!c.array(&sn)) return {};                   // string_values
    for (uint32_t j = 0; j < sn; ++j) {
      uint32_t kv;
      if (!c.array(&kv) || kv != 2 || !c.raw(&s, &n) || !c.raw(&s, &n)) return {};
      uint32_t k = 0;
      while (k < n && !(s[k] >= '0' && s[k] <= '9')) ++k;
      uint32_t e = k;
      while (e < n && s[e] >= '0' && s[e] <= '9') ++e;
      if (e > k) {
        out.all.emplace_back((uint32_t)(s + k - b), e - k);
        if (j + 1 == sn) out.digits.emplace_back((uint32_t)(s + k - b), e - k);   // the last value's digits
      }
    }
    out.all_begin.push_back((uint32_t)out.all.size());
    if (!c.array(&nn)) return {};
    for (uint32_t j = 0; j < nn; ++j) {
      uint32_t kv;
      if (!c.array(&kv) || kv != 2 || !c.raw(&s, &n) || !c.need(1)) return {};
      if (j == 0 && *c.p == 0xcb) out.f64.push_back((uint32_t)(c.p + 1 - b));
      double d;
      if (!c.number(&d)) return {};
    }
    for (uint32_t k = 2; k < three; ++k)
      if (!c.skip()) return {};
  }
  return out;
}

struct Fresh {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  // N(0, 1/4) from the sum of four 16-bit uniforms (Irwin-Hall, variance 1/3
  // each -> scaled)
  double half_gauss() {
    const uint64_t r = next();
    const double u = (double)(r & 0xffff) + (double)((r >> 16) & 0xffff) +
                     (double)((r >> 32) & 0xffff) + (double)(r >> 48);
    return (u / 65536.0 - 2.0) * 0.8660254037844386;   // sqrt(3)/2: sd 0.5
  }
};

inline double get_f64(const uint8_t* p) {
  uint64_t u = 0;
  for (int k = 0; k < 8; ++k) u = (u << 8) | p[k];
  double v;
  memcpy(&v, &u, 8);
  return v;
}

// One private request of a connection in fresh mode: a copy of a params
// object refreshed in place before every send (the kernel has copied the
// bytes when sendmsg returns, so the buffer is free again)
struct FreshReq {
  std::string buf;
  std::vector<double> base;          // the template's float64 values
  const FreshSlots* slots = nullptr;
  void init(const std::string& src, const FreshSlots* sl) {
    buf = src;
    slots = sl;
    base.clear();
    for (const uint32_t o : sl->f64) base.push_back(get_f64((const uint8_t*)src.data() + o));
  }
  // noise_pm: per mille of the samples whose every string value gets new
  // digits (tokens the model has not seen: the sample updates the model)
  void refresh(Fresh* rng, int noise_pm) {
    uint8_t* b = (uint8_t*)&buf[0];
    if (noise_pm > 0)
      for (size_t i = 0; i + 1 < slots->all_begin.size(); ++i) {
        if ((int)(rng->next() % 1000) >= noise_pm) continue;
        for (uint32_t q = slots->all_begin[i]; q < slots->all_begin[i + 1]; ++q) {
          const auto& d = slots->all[q];
          uint64_t r = rng->next();
          for (uint32_t k = 0; k < d.second; ++k, r /= 10) b[d.first + k] = (uint8_t)('0' + r % 10);
        }
      }
    for (size_t i = 0; i < slots->f64.size(); ++i) {
      const double v = base[i] + rng->half_gauss();
      uint64_t u;
      memcpy(&u, &v, 8);
      uint8_t* p = b + slots->f64[i];
      for (int k = 7; k >= 0; --k) { p[k] = (uint8_t)u; u >>= 8; }
    }
    for (const auto& d : slots->digits) {
      uint64_t r = rng->next();
      for (uint32_t k = 0; k < d.second; ++k, r /= 10) b[d.first + k] = (uint8_t)('0' + r % 10);
    }
  }
};

struct Result {
  uint64_t done = 0;
  std::vector<double> lat_us;
  std::string error;
};

void run_conn(const std::string& host, int port, const std::string& method,
              const std::vector<std::string>* params, const std::vector<FreshSlots>* fresh,
              uint64_t seed, size_t first, size_t last, bool once, int depth, double secs, int noise_pm,
              Result* r) {
  const int fd = connect_to(host, port);
  if (fd < 0) { r->error = "connect failed"; return; }
  std::vector<Clock::time_point> sent(1 << 16);
  uint32_t next = 1;
  size_t which = first;
  int inflight = 0;
  std::string rbuf;
  const auto t_end = Clock::now() + std::chrono::duration<double>(secs);
  bool sending = true;
  char buf[1 << 16];
  std::vector<std::string> heads;
  std::vector<const std::string*> bodies;
  // fresh mode: the connection's depth private requests (templates
  // first, first + 1, ... of the params), each refreshed before it goes out
  std::vector<FreshReq> priv(fresh ? (size_t)depth : 0);
  for (size_t j = 0; j < priv.size(); ++j) {
    const size_t t = (first + j) % params->size();
    priv[j].init((*params)[t], &(*fresh)[t]);
  }
  Fresh rng{seed * 0xD1B54A32D192ED03ull + first};
  while (sending || inflight > 0) {
    // every request the window allows goes out in one sendmsg
    heads.clear();
    bodies.clear();
    const auto now = Clock::now();
    if (sending && !once && now >= t_end) sending = false;
    if (sending && once && which >= last) sending = false;
    while (sending && inflight < depth && !(once && which >= last)) {
      heads.push_back(request_head(next, method));
      if (fresh) {
        FreshReq& f = priv[heads.size() - 1];
        f.refresh(&rng, noise_pm);
        bodies.push_back(&f.buf);
      } else {
        bodies.push_back(&(*params)[which]);
      }
      sent[next & 0xffff] = now;
      which = once ? which + 1 : (which + 1) % params->size();
      ++next;
      ++inflight;
    }
    if (!heads.empty() && !send_many(fd, heads, bodies)) {
      r->error = "send failed";
      close(fd);
      return;
    }
    if (inflight == 0) break;
    ssize_t k = recv(fd, buf, sizeof buf, 0);
    if (k <= 0) { r->error = "connection closed"; close(fd); return; }
    rbuf.append(buf, (size_t)k);
    for (;;) {
      const int64_t f = jb::msgpack_frame((const uint8_t*)rbuf.data(), rbuf.size());
      if (f < 0) { r->error = "malformed response"; close(fd); return; }
      if (f == 0) break;
      jb::Cursor c{(const uint8_t*)rbuf.data(), (const uint8_t*)rbuf.data() + f};
      uint32_t n;
      double type, id;
      if (!c.array(&n) || n != 4 || !c.number(&type) || !c.number(&id)) {
        r->error = "bad response";
        close(fd);
        return;
      }
      if (*c.p != 0xc0) { r->error = "error response from server"; close(fd); return; }
      const auto now = Clock::now();
      r->lat_us.push_back(std::chrono::duration<double, std::micro>(now - sent[(uint32_t)id & 0xffff]).count());
      ++r->done;
      --inflight;
      rbuf.erase(0, (size_t)f);
    }
  }
  close(fd);
}

}  // namespace

int main(int argc, char** argv) {
  std::string host = "127.0.0.1", method, file;
  int port = 0, conns = 8, depth = 4;
  bool once = false;
  double secs = 3.0;
  long long fresh_seed = -1;
  int noise_pm = 0;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string a = argv[i], v = argv[i + 1];
    if (a == "-H") host = v;
    else if (a == "-p") port = atoi(v.c_str());
    else if (a == "-m") method = v;
    else if (a == "-f") file = v;
    else if (a == "-c") conns = atoi(v.c_str());
    else if (a == "-d") depth = atoi(v.c_str());
    else if (a == "-t") secs = atof(v.c_str());
    else if (a == "-o") once = atoi(v.c_str()) != 0;
    else if (a == "-r") fresh_seed = atoll(v.c_str());
    else if (a == "-u") noise_pm = atoi(v.c_str());
    else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 1; }
  }
  if (!port || method.empty() || file.empty() || conns < 1 || depth < 1) {
    fprintf(stderr,
            "usage: jubaloadgen -p PORT -m METHOD -f PARAMS.bin [-H HOST] [-c CONNS] [-d DEPTH]"
            " [-t SECONDS] [-o 1] [-r SEED [-u NOISE_PER_MILLE]]\n");
    return 1;
  }
  std::ifstream ifs(file, std::ios::binary);
  std::stringstream ss;
  ss << ifs.rdbuf();
  const std::string all = ss.str();
  std::vector<std::string> params;
  for (size_t pos = 0; pos < all.size();) {
    const int64_t f = jb::msgpack_frame((const uint8_t*)all.data() + pos, all.size() - pos);
    if (f <= 0) { fprintf(stderr, "params file: bad msgpack at byte %zu\n", pos); return 1; }
    params.push_back(all.substr(pos, (size_t)f));
    pos += (size_t)f;
  }
  if (params.empty()) { fprintf(stderr, "empty params file\n"); return 1; }
  std::vector<FreshSlots> slots;
  if (fresh_seed >= 0) {
    if (once) { fprintf(stderr, "-r: not with -o\n"); return 1; }
    for (const auto& p : params) {
      slots.push_back(fresh_slots(p));
      if (slots.back().empty()) { fprintf(stderr, "-r: params without float64 num values\n"); return 1; }
    }
  }
  std::vector<Result> res(conns);
  std::vector<std::thread> ts;
  const auto t0 = Clock::now();
  for (int i = 0; i < conns; ++i)
    ts.emplace_back(run_conn, host, port, method, &params, fresh_seed >= 0 ? &slots : nullptr,
                    (uint64_t)(fresh_seed >= 0 ? fresh_seed : 0),
                    (size_t)i * params.size() / (size_t)conns,
                    (size_t)(i + 1) * params.size() / (size_t)conns, once, depth, secs, noise_pm, &res[i]);
  for (auto& t : ts) t.join();
  const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
  uint64_t done = 0;
  std::vector<double> lat;
  for (auto& r : res) {
    if (!r.error.empty()) { fprintf(stderr, "jubaloadgen: %s\n", r.error.c_str()); return 2; }
    done += r.done;
    lat.insert(lat.end(), r.lat_us.begin(), r.lat_us.end());
  }
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double q) { return lat.empty() ? 0.0 : lat[(size_t)(q * (lat.size() - 1))]; };
  printf("{\"requests\": %llu, \"seconds\": %.3f, \"requests_per_s\": %.1f, \"connections\": %d, "
         "\"depth\": %d, \"distinct_requests\": %zu, \"fresh_values\": %s, \"noise_per_mille\": %d, "
         "\"p50_us\": %.1f, \"p99_us\": %.1f}\n",
         (unsigned long long)done, dt, done / dt, conns, depth, params.size(),
         fresh_seed >= 0 ? "true" : "false", noise_pm, pct(0.5), pct(0.99));
  return 0;
}
