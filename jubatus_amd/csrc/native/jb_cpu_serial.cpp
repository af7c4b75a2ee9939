// Host serial trainer: the in-house CPU baseline of the classifier's default
// (serial-equivalent, "exact") training semantics, and the host oracle the
// GPU committer's design is studied against.
//
// The reference trains one sample at a time under the model's write lock
// (jubatus/server/server/classifier_serv.cpp:138-144); this is that loop in
// native C++ over the hashed feature vectors of the GPU path (same hasher,
// jb_hostfv.hpp; same update rules as jubatus_amd/models/linear_oracle.py and
// csrc/hip/jb_linear.hpp step_coeffs / dprec, fp32 arithmetic):
//
//   cpu_hash_arena      request spans -> (row_ptr, idx, val, labels)
//   cpu_serial_train    CSR + labels -> W / P updated in order; optionally the
//                       per-update step magnitudes (max(|dW_y|, |dW_l*|) per
//                       feature slot, 0 for a sample that did not update)
//   cpu_train_arena     the whole path on the host: parse + hash (nthreads
//                       workers, request order preserved) and the serial train
//                       (one thread - the semantics are sequential), pipelined
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "jb_host_linear.hpp"
#include "jb_hostfv.hpp"
#include "jb_msgpack.hpp"
#include "jb_pack.hpp"

namespace py = pybind11;

namespace {

using jb::hl::Trainer;

// parsed + hashed requests: one request's samples
struct Parsed {
  std::vector<int64_t> rp{0};
  std::vector<int32_t> ix;
  std::vector<float> val;
  std::vector<std::pair<const uint8_t*, uint32_t>> lab;   // label bytes (resolved in order)
  int err = 0;
};

int parse_request(const jb::HostFvHasher& h, const uint8_t* p, uint64_t len, Parsed& out) {
  out.rp.assign(1, 0);
  out.ix.clear();
  out.val.clear();
  out.lab.clear();
  jb::Cursor c{p, p + len};
  uint32_t cnt;
  if (!c.array(&cnt)) return 1;
  for (uint32_t i = 0; i < cnt; ++i) {
    uint32_t two;
    const uint8_t* lb;
    uint32_t ln;
    if (!c.array(&two) || two != 2 || !c.raw(&lb, &ln)) return 1;
    out.lab.emplace_back(lb, ln);
    int64_t slots = (int64_t)out.ix.size();
    for (;;) {
      const int64_t cap = (int64_t)out.ix.size() + 256;
      out.ix.resize((size_t)cap);
      out.val.resize((size_t)cap);
      jb::Cursor save = c;
      const int rc = h.hash_datum(c, out.ix.data(), out.val.data(), cap, &slots);
      if (rc == 2) {          // a datum wider than 256 slots: grow and re-hash
        c = save;
        slots = out.rp.back();
        out.ix.resize((size_t)cap * 2);
        continue;
      }
      if (rc) return rc;
      break;
    }
    out.ix.resize((size_t)slots);
    out.val.resize((size_t)slots);
    out.rp.push_back(slots);
  }
  return 0;
}

py::tuple cpu_hash_arena(const jb::HostFvHasher& h, uintptr_t base, py::array_t<int64_t> offs,
                         py::array_t<int64_t> lens, jb::LabelTable* table) {
  const int64_t nreq = offs.size();
  std::vector<int64_t> rp{0};
  std::vector<int32_t> ix;
  std::vector<float> val;
  std::vector<int32_t> labels;
  Parsed pr;
  for (int64_t k = 0; k < nreq; ++k) {
    if (parse_request(h, (const uint8_t*)base + offs.at(k), (uint64_t)lens.at(k), pr))
      throw std::invalid_argument("malformed train request " + std::to_string(k));
    for (size_t i = 0; i + 1 < pr.rp.size(); ++i) {
      labels.push_back(table->get_or_add((const char*)pr.lab[i].first, pr.lab[i].second));
      const int64_t o = (int64_t)ix.size();
      ix.insert(ix.end(), pr.ix.begin() + pr.rp[i], pr.ix.begin() + pr.rp[i + 1]);
      val.insert(val.end(), pr.val.begin() + pr.rp[i], pr.val.begin() + pr.rp[i + 1]);
      rp.push_back(o + (pr.rp[i + 1] - pr.rp[i]));
    }
  }
  py::array_t<int64_t> a_rp((py::ssize_t)rp.size());
  py::array_t<int32_t> a_ix((py::ssize_t)ix.size()), a_lab((py::ssize_t)labels.size());
  py::array_t<float> a_val((py::ssize_t)val.size());
  memcpy(a_rp.mutable_data(), rp.data(), rp.size() * 8);
  if (!ix.empty()) {
    memcpy(a_ix.mutable_data(), ix.data(), ix.size() * 4);
    memcpy(a_val.mutable_data(), val.data(), val.size() * 4);
  }
  if (!labels.empty()) memcpy(a_lab.mutable_data(), labels.data(), labels.size() * 4);
  return py::make_tuple(a_rp, a_ix, a_val, a_lab);
}

// -> (updates, seconds); mag (optional, float32[nnz]) gets the step magnitudes
py::tuple cpu_serial_train(int method, float C, int LC, py::array_t<int64_t> row_ptr,
                           py::array_t<int32_t> idx, py::array_t<float> val, py::array_t<int32_t> labels,
                           py::array_t<uint8_t> active, uintptr_t W, uintptr_t P, py::object mag) {
  const int64_t n = row_ptr.size() - 1;
  if (n < 0 || labels.size() < n) throw std::invalid_argument("row_ptr / labels sizes");
  if (active.size() < LC) throw std::invalid_argument("active shorter than LC");
  const int64_t* rp = row_ptr.data();
  if (idx.size() < rp[n] || val.size() < rp[n]) throw std::invalid_argument("CSR shorter than row_ptr");
  float* mg = nullptr;
  if (!mag.is_none()) {
    auto m = mag.cast<py::array_t<float>>();
    if (m.size() < rp[n]) throw std::invalid_argument("mag shorter than the CSR");
    mg = m.mutable_data();
  }
  Trainer t(method, C, LC, active.data(), (float*)W, (float*)P);
  const int32_t* ix = idx.data();
  const float* vx = val.data();
  const int32_t* lab = labels.data();
  int64_t upd = 0;
  const auto t0 = std::chrono::steady_clock::now();
  {
    py::gil_scoped_release nogil;
    for (int64_t i = 0; i < n; ++i) {
      if (i + 1 < n) t.prefetch(ix + rp[i + 1], (int)(rp[i + 2] - rp[i + 1]));
      const int y = lab[i];
      const int nf = (int)(rp[i + 1] - rp[i]);
      if (y < 0 || y >= LC) {
        if (mg != nullptr) std::fill(mg + rp[i], mg + rp[i + 1], 0.f);
        continue;
      }
      upd += t.step(ix + rp[i], vx + rp[i], nf, y, mg != nullptr ? mg + rp[i] : nullptr) ? 1 : 0;
    }
  }
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return py::make_tuple(upd, sec);
}

// the whole host path; -> (samples, updates, seconds)
py::tuple cpu_train_arena(const jb::HostFvHasher& h, uintptr_t base, py::array_t<int64_t> offs,
                          py::array_t<int64_t> lens, jb::LabelTable* table, int method, float C, int LC,
                          uintptr_t W, uintptr_t P, py::array_t<uint8_t> active, int nthreads) {
  const int64_t nreq = offs.size();
  if (lens.size() < nreq) throw std::invalid_argument("lens shorter than offs");
  if (active.size() < LC) throw std::invalid_argument("active shorter than LC");
  const int64_t* o = offs.data();
  const int64_t* l = lens.data();
  Trainer t(method, C, LC, active.data(), (float*)W, (float*)P);
  int64_t samples = 0, upd = 0;
  int bad = 0;
  const auto t0 = std::chrono::steady_clock::now();
  {
    py::gil_scoped_release nogil;
    auto train = [&](Parsed& pr) {
      const int64_t m = (int64_t)pr.rp.size() - 1;
      for (int64_t i = 0; i < m; ++i) {
        if (i + 1 < m) t.prefetch(pr.ix.data() + pr.rp[i + 1], (int)(pr.rp[i + 2] - pr.rp[i + 1]));
        const int y = table->get_or_add((const char*)pr.lab[(size_t)i].first, pr.lab[(size_t)i].second);
        ++samples;
        if (y < 0 || y >= LC) continue;
        upd += t.step(pr.ix.data() + pr.rp[i], pr.val.data() + pr.rp[i], (int)(pr.rp[i + 1] - pr.rp[i]), y,
                      nullptr) ? 1 : 0;
      }
    };
    if (nthreads <= 1) {
      Parsed pr;
      for (int64_t k = 0; k < nreq && !bad; ++k) {
        if (parse_request(h, (const uint8_t*)base + o[k], (uint64_t)l[k], pr)) { bad = 1; break; }
        train(pr);
      }
    } else {
      // nthreads - 1 workers parse + hash requests round-robin into a ring of
      // slots (the calling thread, which trains them in request order, keeps
      // a core of its own). Hand-offs block on condition variables: a request
      // is ~100 us of training, so a wake-up per request costs little, and
      // spinning waiters would take the trainer's core (the round-5 ring
      // yield-spun 16 workers over adjacent atomics: all threads ran slower
      // than one).
      const int nw = std::max(1, nthreads - 1);
      const int64_t ring = 4 * (int64_t)nw;
      struct alignas(64) Slot {
        Parsed pr;
        int64_t k = -1;   // request index parsed into the slot
      };
      std::vector<Slot> slot((size_t)ring);
      std::mutex mu;
      std::condition_variable room, ready;
      int64_t consumed = 0;
      bool stop = false;
      std::vector<std::thread> th;
      for (int w = 0; w < nw; ++w)
        th.emplace_back([&, w] {
          for (int64_t k = w; k < nreq; k += nw) {
            {
              std::unique_lock<std::mutex> g(mu);
              room.wait(g, [&] { return stop || k - consumed < ring; });
              if (stop) return;
            }
            Slot& sl = slot[(size_t)(k % ring)];
            sl.pr.err = parse_request(h, (const uint8_t*)base + o[k], (uint64_t)l[k], sl.pr);
            {
              std::lock_guard<std::mutex> g(mu);
              sl.k = k;
            }
            ready.notify_one();
          }
        });
      for (int64_t k = 0; k < nreq; ++k) {
        Slot& sl = slot[(size_t)(k % ring)];
        {
          std::unique_lock<std::mutex> g(mu);
          ready.wait(g, [&] { return sl.k == k; });
        }
        if (sl.pr.err) { bad = 1; break; }
        train(sl.pr);
        {
          std::lock_guard<std::mutex> g(mu);
          sl.k = -1;
          consumed = k + 1;
        }
        room.notify_all();
      }
      {
        std::lock_guard<std::mutex> g(mu);
        stop = true;
      }
      room.notify_all();
      for (auto& x : th) x.join();
    }
  }
  if (bad) throw std::invalid_argument("malformed train request");
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return py::make_tuple(samples, upd, sec);
}

}  // namespace

void register_cpu_serial(py::module_& m) {
  m.def("cpu_hash_arena", &cpu_hash_arena, "request spans [[label, datum], ...] -> (row_ptr, idx, val, labels)",
        py::arg("hasher"), py::arg("base"), py::arg("offs"), py::arg("lens"), py::arg("table"));
  m.def("cpu_serial_train", &cpu_serial_train,
        "serial online training of a hashed batch on the host -> (updates, seconds)", py::arg("method"),
        py::arg("C"), py::arg("LC"), py::arg("row_ptr"), py::arg("idx"), py::arg("val"), py::arg("labels"),
        py::arg("active"), py::arg("W"), py::arg("P"), py::arg("mag") = py::none());
  m.def("cpu_train_arena", &cpu_train_arena,
        "parse + hash (nthreads workers) + serial train of request spans on the host -> (samples, updates, s)",
        py::arg("hasher"), py::arg("base"), py::arg("offs"), py::arg("lens"), py::arg("table"),
        py::arg("method"), py::arg("C"), py::arg("LC"), py::arg("W"), py::arg("P"), py::arg("active"),
        py::arg("nthreads") = 1);
}
