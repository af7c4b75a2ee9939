// Synthetic train-request generator for the benchmark (bench.py) and the
// kernel micro-benchmarks: msgpack list<labeled_datum> bodies (old-spec RAW,
// the wire layout of jubatus/client/common/datum.hpp:42-46) written straight
// into a caller-owned (pinned) arena, multi-threaded.
//
// Request k is generated from its own splitmix64 stream seeded by
// (seed, k), so a batch is reproducible and any two (seed, k) pairs give
// independent data: the benchmark's timed steps never replay a sample.
// Each datum: label "label<y>", n_str string values s<j> -> t<tok> where tok
// is label-correlated (y*131 + [0, hot)) with probability p_corr and
// uniform in [0, vocab) otherwise, n_num numeric values n<j> ->
// (y - nlabels/2) * 0.05 + N(0, 1) (float64).
#include <pybind11/pybind11.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  double gauss() {
    double u = unit();
    if (u < 1e-300) u = 1e-300;
    return std::sqrt(-2.0 * std::log(u)) * std::cos(6.283185307179586 * unit());
  }
};

struct Spec {
  uint64_t seed;
  int per_req, nlabels, n_str, n_num;
  uint32_t vocab, hot;
  double p_corr;
};

int ndigits(uint64_t v) {
  int n = 1;
  while (v >= 10) { v /= 10; ++n; }
  return n;
}

// writer that only counts when out == nullptr
struct W {
  uint8_t* p;
  int64_t n = 0;
  void byte(uint8_t b) { if (p) p[n] = b; ++n; }
  void raw_hdr(int len) {           // old-spec RAW: fixraw / raw16
    if (len < 32) byte((uint8_t)(0xa0 | len));
    else { byte(0xda); byte((uint8_t)(len >> 8)); byte((uint8_t)len); }
  }
  void arr_hdr(int len) {
    if (len < 16) byte((uint8_t)(0x90 | len));
    else if (len < 65536) { byte(0xdc); byte((uint8_t)(len >> 8)); byte((uint8_t)len); }
    else { byte(0xdd); for (int s = 24; s >= 0; s -= 8) byte((uint8_t)(len >> s)); }
  }
  void prefixed_num(char c, uint64_t v) {   // RAW "<c><decimal v>"
    const int d = ndigits(v);
    raw_hdr(1 + d);
    byte((uint8_t)c);
    if (p) {
      uint64_t x = v;
      for (int i = d - 1; i >= 0; --i) { p[n + i] = (uint8_t)('0' + x % 10); x /= 10; }
    }
    n += d;
  }
  void label(uint64_t y) {         // RAW "label<y>"
    const int d = ndigits(y);
    raw_hdr(5 + d);
    static const char kL[] = "label";
    for (int i = 0; i < 5; ++i) byte((uint8_t)kL[i]);
    if (p) {
      uint64_t x = y;
      for (int i = d - 1; i >= 0; --i) { p[n + i] = (uint8_t)('0' + x % 10); x /= 10; }
    }
    n += d;
  }
  void f64(double v) {
    uint64_t u;
    std::memcpy(&u, &v, 8);
    byte(0xcb);
    for (int s = 56; s >= 0; s -= 8) byte((uint8_t)(u >> s));
  }
};

int64_t one_request(const Spec& sp, uint64_t k, uint8_t* out) {
  Rng r{sp.seed * 0x632BE59BD9B4E019ull ^ (k + 1) * 0x9E3779B97F4A7C15ull};
  W w{out};
  w.arr_hdr(sp.per_req);
  for (int i = 0; i < sp.per_req; ++i) {
    const uint32_t y = r.below((uint32_t)sp.nlabels);
    w.arr_hdr(2);
    w.label(y);
    w.arr_hdr(3);
    w.arr_hdr(sp.n_str);
    for (int j = 0; j < sp.n_str; ++j) {
      uint64_t tok;
      if (r.unit() < sp.p_corr) tok = (uint64_t)y * 131 + r.below(sp.hot ? sp.hot : 1);
      else tok = r.below(sp.vocab ? sp.vocab : 1);
      w.arr_hdr(2);
      w.prefixed_num('s', (uint64_t)j);
      w.prefixed_num('t', tok);
    }
    w.arr_hdr(sp.n_num);
    for (int j = 0; j < sp.n_num; ++j) {
      w.arr_hdr(2);
      w.prefixed_num('n', (uint64_t)j);
      w.f64(((double)y - sp.nlabels / 2.0) * 0.05 + r.gauss());
    }
    w.arr_hdr(0);
  }
  return w.n;
}

// -> bytes used (bodies 16-B aligned like RequestArena.append), -1 if the
// arena is too small. offs / lens: int64[nreq] outputs.
int64_t synth_requests(uintptr_t base, int64_t cap, uintptr_t offs_p, uintptr_t lens_p,
                       uint64_t seed, int64_t first_req, int64_t nreq, int per_req, int nlabels,
                       int n_str, int n_num, uint32_t vocab, uint32_t hot, double p_corr,
                       int nthreads) {
  Spec sp{seed, per_req, nlabels, n_str, n_num, vocab, hot, p_corr};
  int64_t* offs = (int64_t*)offs_p;
  int64_t* lens = (int64_t*)lens_p;
  uint8_t* out = (uint8_t*)base;
  nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<int64_t>(1, nreq / 4)));
  py::gil_scoped_release nogil;
  auto run = [&](auto&& fn) {
    std::atomic<int64_t> next{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < nthreads; ++t)
      ts.emplace_back([&] {
        for (int64_t k; (k = next.fetch_add(16)) < nreq;)
          for (int64_t j = k; j < std::min(nreq, k + 16); ++j) fn(j);
      });
    for (auto& t : ts) t.join();
  };
  run([&](int64_t k) { lens[k] = one_request(sp, (uint64_t)(first_req + k), nullptr); });
  int64_t used = 0;
  for (int64_t k = 0; k < nreq; ++k) {
    const int64_t off = (used + 15) & ~(int64_t)15;
    offs[k] = off;
    used = off + lens[k];
  }
  if (used > cap) return -1;
  run([&](int64_t k) { one_request(sp, (uint64_t)(first_req + k), out + offs[k]); });
  return used;
}

}  // namespace

void register_synth(py::module_& m) {
  m.def("synth_requests", &synth_requests,
        "generate synthetic msgpack train bodies into an arena -> bytes used (-1: too small)",
        py::arg("base"), py::arg("cap"), py::arg("offs"), py::arg("lens"), py::arg("seed"),
        py::arg("first_req"), py::arg("nreq"), py::arg("per_req"), py::arg("nlabels"),
        py::arg("n_str"), py::arg("n_num"), py::arg("vocab"), py::arg("hot"), py::arg("p_corr"),
        py::arg("nthreads"));
}
