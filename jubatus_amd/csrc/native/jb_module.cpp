// Python bindings of the host-native runtime (_jubatus_native).
#include <algorithm>
#include <vector>

#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include "jb_hash.hpp"
#include "jb_hostfv.hpp"
#include "jb_hostfv_wide.hpp"
#include "jb_pyrandom.hpp"
#include "jb_pack.hpp"
#include "jb_rpc.hpp"

namespace py = pybind11;

namespace {

py::tuple pack(py::list reqs, int labeled, int sps, int spn, jb::LabelTable* table,
               uintptr_t staging, uint64_t staging_cap, uintptr_t datum_off, uintptr_t datum_len,
               uintptr_t labels, uintptr_t row_ptr, uintptr_t stream_ptr, int64_t max_samples,
               int nthreads) {
  std::vector<jb::RequestView> views;
  std::vector<py::buffer_info> keep;
  views.reserve(reqs.size());
  keep.reserve(reqs.size());
  for (auto item : reqs) {
    py::buffer b = py::reinterpret_borrow<py::buffer>(item);
    keep.emplace_back(b.request());
    const py::buffer_info& bi = keep.back();
    views.push_back({(const uint8_t*)bi.ptr, (uint64_t)(bi.size * bi.itemsize)});
  }
  jb::PackOut out{(uint8_t*)staging, nullptr, staging_cap, (int64_t*)datum_off,
                  (int32_t*)datum_len, (int32_t*)labels,
                  (int64_t*)row_ptr, (int64_t*)stream_ptr, max_samples};
  jb::PackResult r;
  {
    py::gil_scoped_release nogil;
    r = jb::pack_requests(views, labeled, sps, spn, table, out, nthreads);
  }
  return py::make_tuple(r.n_samples, r.n_bytes, r.n_slots, r.error, r.error_request);
}

// zero-copy variant: requests are spans [offs[k], offs[k]+lens[k]) of one
// pinned arena at `base` (e.g. the RPC receive arena); nothing is copied.
py::tuple pack_spans(uintptr_t base, uintptr_t offs, uintptr_t lens, int64_t nreq, int labeled,
                     int sps, int spn, jb::LabelTable* table, uintptr_t datum_off,
                     uintptr_t datum_len, uintptr_t labels, uintptr_t row_ptr, uintptr_t stream_ptr,
                     int64_t max_samples, int nthreads) {
  std::vector<jb::RequestView> views((size_t)nreq);
  const int64_t* o = (const int64_t*)offs;
  const int64_t* l = (const int64_t*)lens;
  for (int64_t k = 0; k < nreq; ++k) views[k] = {(const uint8_t*)base + o[k], (uint64_t)l[k]};
  jb::PackOut out{nullptr, (const uint8_t*)base, 0, (int64_t*)datum_off, (int32_t*)datum_len,
                  (int32_t*)labels,
                  (int64_t*)row_ptr, (int64_t*)stream_ptr, max_samples};
  jb::PackResult r;
  {
    py::gil_scoped_release nogil;
    r = jb::pack_requests(views, labeled, sps, spn, table, out, nthreads);
  }
  return py::make_tuple(r.n_samples, r.n_bytes, r.n_slots, r.error, r.error_request);
}

uint32_t crc32(py::buffer b, uint32_t init) {
  py::buffer_info bi = b.request();
  return jb::crc32_update(init, (const uint8_t*)bi.ptr, (size_t)(bi.size * bi.itemsize));
}

std::string md5_hex(const std::string& s) { return jb::Md5::hex(s); }

int64_t feature_index(py::bytes name, uint64_t H) {
  std::string s = name;
  return jb::hash_to_index(jb::fnv_bytes(jb::kFnvOffset, (const uint8_t*)s.data(), s.size()), H);
}

uint64_t fnv1a64(py::bytes name) {
  std::string s = name;
  return jb::fnv_bytes(jb::kFnvOffset, (const uint8_t*)s.data(), s.size());
}

// Python face of jb::RpcServer. handler(method: str, params: bytes,
// msgid: int, notify: bool) -> bytes | None (the complete encoded response).
class PyRpcServer {
 public:
  PyRpcServer(py::object handler, int nworkers, double idle_timeout)
      : handler_(std::move(handler)) {
    srv_.reset(new jb::RpcServer(
        [this](const jb::RpcRequest& r) -> std::string {
          py::gil_scoped_acquire gil;
          try {
            py::object res = handler_(py::str(r.method), py::bytes(r.params), r.msgid, r.notify);
            if (res.is_none()) return std::string();
            return res.cast<std::string>();
          } catch (py::error_already_set& e) {
            // last-resort error response: [1, msgid, "<error>", nil] (fixarray 4)
            std::string what = e.what();
            if (what.size() > 255) what.resize(255);
            std::string out;
            out.push_back((char)0x94);
            out.push_back((char)0x01);
            out.push_back((char)0xce);
            for (int i = 3; i >= 0; --i) out.push_back((char)((r.msgid >> (8 * i)) & 0xff));
            out.push_back((char)0xd9);
            out.push_back((char)what.size());
            out += what;
            out.push_back((char)0xc0);
            return r.notify ? std::string() : out;
          }
        },
        nworkers, idle_timeout));
  }
  ~PyRpcServer() {
    py::gil_scoped_release nogil;
    srv_.reset();
  }
  // fn(method: str, params: list[bytes], msgids: list[int]) -> list[bytes | None]
  void set_batch(std::vector<std::string> methods, py::object fn, size_t max_batch) {
    batch_fn_ = std::move(fn);
    srv_->set_batch(
        methods,
        [this](const std::string& method, std::vector<jb::RpcRequest>& reqs) {
          std::vector<std::string> out(reqs.size());
          py::gil_scoped_acquire gil;
          try {
            py::list params, ids;
            for (auto& r : reqs) {
              params.append(py::bytes(r.params));
              ids.append(r.msgid);
            }
            py::list res = batch_fn_(py::str(method), params, ids);
            for (size_t i = 0; i < reqs.size() && i < (size_t)py::len(res); ++i)
              if (!res[i].is_none()) out[i] = res[i].cast<std::string>();
          } catch (py::error_already_set& e) {
            // every request of the batch gets the error string
            std::string what = e.what();
            if (what.size() > 255) what.resize(255);
            for (size_t i = 0; i < reqs.size(); ++i) {
              std::string& o = out[i];
              o.push_back((char)0x94);
              o.push_back((char)0x01);
              o.push_back((char)0xce);
              for (int k = 3; k >= 0; --k) o.push_back((char)((reqs[i].msgid >> (8 * k)) & 0xff));
              o.push_back((char)0xd9);
              o.push_back((char)what.size());
              o += what;
              o.push_back((char)0xc0);
            }
          }
          return out;
        },
        max_batch);
  }
  // Arena batching (jb_rpc.hpp): fn(slot: int, offs: int64[n], lens: int64[n])
  // -> (results: int64[n], errors: dict[int, str]); results[i] >= 0 is the
  // reply value, -1 ARGUMENT_ERROR, -2 the message errors[i], -3 no reply.
  // Responses are encoded here (old-spec msgpack), not in Python.
  void set_arena_batch(const std::string& method, std::vector<uintptr_t> slots, size_t slot_bytes,
                       py::object fn) {
    arena_fn_ = std::move(fn);
    std::vector<uint8_t*> ptrs;
    for (auto p : slots) ptrs.push_back((uint8_t*)p);
    srv_->set_arena_batch(method, ptrs, slot_bytes,
                          [this](int slot, const std::vector<jb::ArenaReq>& reqs) {
      const size_t n = reqs.size();
      std::vector<std::string> out(n);
      std::vector<int64_t> res(n, -2);
      std::vector<std::string> msg(n);
      {
        py::gil_scoped_acquire gil;
        try {
          py::array_t<int64_t> offs(n), lens(n);
          auto o = offs.mutable_unchecked<1>();
          auto l = lens.mutable_unchecked<1>();
          for (size_t i = 0; i < n; ++i) { o(i) = (int64_t)reqs[i].off; l(i) = (int64_t)reqs[i].len; }
          py::tuple r = arena_fn_(slot, offs, lens);
          py::array_t<int64_t> vals = r[0].cast<py::array_t<int64_t>>();
          auto v = vals.unchecked<1>();
          for (size_t i = 0; i < n && i < (size_t)v.shape(0); ++i) res[i] = v(i);
          py::dict errs = r[1].cast<py::dict>();
          for (auto kv : errs) {
            const size_t i = kv.first.cast<size_t>();
            if (i < n) msg[i] = py::str(kv.second).cast<std::string>();
          }
        } catch (py::error_already_set& e) {
          for (size_t i = 0; i < n; ++i) msg[i] = e.what();
        }
      }
      for (size_t i = 0; i < n; ++i) {
        if (res[i] == -3) continue;
        std::string& b = out[i];
        b.push_back((char)0x94);
        b.push_back((char)0x01);
        b.push_back((char)0xce);
        for (int k = 3; k >= 0; --k) b.push_back((char)((reqs[i].msgid >> (8 * k)) & 0xff));
        if (res[i] >= 0) {
          b.push_back((char)0xc0);
          const uint64_t x = (uint64_t)res[i];
          if (x < 128) {
            b.push_back((char)x);
          } else if (x < 65536) {
            b.push_back((char)0xcd); b.push_back((char)(x >> 8)); b.push_back((char)x);
          } else if (x < (1ull << 32)) {
            b.push_back((char)0xce);
            for (int k = 3; k >= 0; --k) b.push_back((char)(x >> (8 * k)));
          } else {
            b.push_back((char)0xcf);
            for (int k = 7; k >= 0; --k) b.push_back((char)(x >> (8 * k)));
          }
        } else if (res[i] == -1) {
          b.push_back((char)0x02);          // ARGUMENT_ERROR
          b.push_back((char)0xc0);
        } else {
          std::string m = msg[i].empty() ? std::string("error") : msg[i];
          if (m.size() > 65535) m.resize(65535);
          if (m.size() < 32) b.push_back((char)(0xa0 | m.size()));
          else { b.push_back((char)0xda); b.push_back((char)(m.size() >> 8)); b.push_back((char)m.size()); }
          b += m;
          b.push_back((char)0xc0);
        }
      }
      return out;
    });
  }
  void release_slot(int slot) { srv_->release_slot(slot); }
  void set_max_message(uint64_t n) { srv_->set_max_message(n); }
  uint64_t batches() const { return srv_->batches(); }
  py::tuple arena_ns() const {
    return py::make_tuple(srv_->arena_handler_ns(), srv_->arena_send_ns());
  }
  void set_io_threads(int n) { srv_->set_io_threads(n); }
  void set_batch_threads(int n) { srv_->set_batch_threads(n); }
  void set_ordered(std::vector<std::string> methods) { srv_->set_ordered(methods); }
  int listen(const std::string& addr, int port) { return srv_->listen(addr, port); }
  void start() { srv_->start(); }
  void stop() {
    py::gil_scoped_release nogil;
    srv_->stop();
  }
  bool running() const { return srv_->running(); }
  uint64_t served() const { return srv_->requests_served(); }
  uint64_t connections() const { return srv_->connections(); }

 private:
  py::object handler_;
  py::object batch_fn_;
  py::object arena_fn_;
  std::unique_ptr<jb::RpcServer> srv_;
};

jb::HostFvHasher* make_hasher(py::buffer srules, int n_srules, py::buffer nrules, int n_nrules,
                              py::buffer blob, uint64_t H) {
  py::buffer_info s = srules.request(), n = nrules.request(), b = blob.request();
  if ((size_t)s.size * s.itemsize < sizeof(jb::HostRule) * (size_t)n_srules ||
      (size_t)n.size * n.itemsize < sizeof(jb::HostRule) * (size_t)n_nrules)
    throw std::invalid_argument("rule table shorter than its rule count");
  return new jb::HostFvHasher((const uint8_t*)s.ptr, n_srules, (const uint8_t*)n.ptr, n_nrules,
                              (const uint8_t*)b.ptr, (size_t)(b.size * b.itemsize), H);
}

jb::HostFvWide* make_wide(py::buffer srules, int n_srules, py::buffer nrules, int n_nrules,
                          py::buffer crules, int n_crules, py::buffer blob, uint64_t H) {
  py::buffer_info s = srules.request(), n = nrules.request(), c = crules.request(),
                  b = blob.request();
  if ((size_t)s.size * s.itemsize < sizeof(jb::HostRule) * (size_t)n_srules ||
      (size_t)n.size * n.itemsize < sizeof(jb::HostRule) * (size_t)n_nrules ||
      (size_t)c.size * c.itemsize < sizeof(jb::HostRule) * 2 * (size_t)n_crules)
    throw std::invalid_argument("rule table shorter than its rule count");
  return new jb::HostFvWide((const uint8_t*)s.ptr, n_srules, (const uint8_t*)n.ptr, n_nrules,
                            (const uint8_t*)c.ptr, n_crules, (const uint8_t*)b.ptr,
                            (size_t)(b.size * b.itemsize), H);
}

py::tuple wide_hash(jb::HostFvWide& h, py::list reqs, uintptr_t idx, uintptr_t val,
                    uintptr_t row_ptr, int64_t max_samples, int64_t max_slots, bool update) {
  int64_t n = 0, slots = 0;
  int64_t* rp = (int64_t*)row_ptr;
  rp[0] = 0;
  h.begin();
  for (auto item : reqs) {
    py::buffer b = py::reinterpret_borrow<py::buffer>(item);
    py::buffer_info bi = b.request();
    int rc = h.hash_body((const uint8_t*)bi.ptr, (size_t)(bi.size * bi.itemsize), (int32_t*)idx,
                         (float*)val, rp, max_samples, max_slots, &n, &slots, update);
    if (rc) {
      if (update && h.needs_weights()) h.rollback();   // no partial statistics
      return py::make_tuple(n, slots, rc);
    }
  }
  return py::make_tuple(n, slots, 0);
}

// One body (msgpack list<datum>) with feature names: -> (error, row_ptr
// int64 [n+1], idx int32, val float32, names bytes, name_end int64 [slots],
// datum spans int64 [n][2] relative to the body). error 1: malformed (no
// statistics were updated).
py::tuple wide_hash_named(jb::HostFvWide& h, py::buffer body, bool update) {
  py::buffer_info bi = body.request();
  const uint8_t* p = (const uint8_t*)bi.ptr;
  const size_t len = (size_t)(bi.size * bi.itemsize);
  int64_t cap_n = 256, cap_s = 4096;
  for (;;) {
    std::vector<int64_t> rp((size_t)cap_n + 1, 0), name_end, spans;
    std::vector<int32_t> idx((size_t)cap_s);
    std::vector<float> val((size_t)cap_s);
    std::string names;
    int64_t n = 0, slots = 0;
    h.begin();
    h.set_sinks(&names, &name_end, &spans);
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = h.hash_body(p, len, idx.data(), val.data(), rp.data(), cap_n, cap_s, &n, &slots, update);
    }
    h.set_sinks(nullptr, nullptr, nullptr);
    if (rc == 2) {
      if (update && h.needs_weights()) h.rollback();
      cap_n *= 4;
      cap_s *= 4;
      continue;
    }
    if (rc) {
      if (update && h.needs_weights()) h.rollback();
      return py::make_tuple(rc, py::none(), py::none(), py::none(), py::none(), py::none(), py::none());
    }
    py::array_t<int64_t> a_rp(n + 1), a_ne(slots), a_sp(2 * n);
    py::array_t<int32_t> a_idx(slots);
    py::array_t<float> a_val(slots);
    memcpy(a_rp.mutable_data(), rp.data(), 8 * (size_t)(n + 1));
    if (slots) {
      memcpy(a_idx.mutable_data(), idx.data(), 4 * (size_t)slots);
      memcpy(a_val.mutable_data(), val.data(), 4 * (size_t)slots);
      memcpy(a_ne.mutable_data(), name_end.data(), 8 * (size_t)slots);
    }
    if (n) memcpy(a_sp.mutable_data(), spans.data(), 16 * (size_t)n);
    return py::make_tuple(0, a_rp, a_idx, a_val, py::bytes(names), a_ne, a_sp);
  }
}

// -> (n_samples, n_slots, error): 0 ok, 1 malformed request, 2 capacity
py::tuple hasher_hash(const jb::HostFvHasher& h, py::list reqs, uintptr_t idx, uintptr_t val,
                      uintptr_t row_ptr, int64_t max_samples, int64_t max_slots, bool update) {
  (void)update;    // no global weights on this rule set
  int64_t n = 0, slots = 0;
  int64_t* rp = (int64_t*)row_ptr;
  rp[0] = 0;
  for (auto item : reqs) {
    py::buffer b = py::reinterpret_borrow<py::buffer>(item);
    py::buffer_info bi = b.request();
    int rc = h.hash_body((const uint8_t*)bi.ptr, (size_t)(bi.size * bi.itemsize), (int32_t*)idx,
                         (float*)val, rp, max_samples, max_slots, &n, &slots);
    if (rc) return py::make_tuple(n, slots, rc);
  }
  return py::make_tuple(n, slots, 0);
}

// Per row of a CSR: drop idx < 0, sort by feature (stable), sum repeated
// features in double, store float; squared norm in double of the stored
// floats. Twin of models/similarity.py normalize_csr for the latency path
// (one small query: ~1 us here vs ~40 us of numpy calls).
py::tuple csr_normalize(py::array_t<int64_t, py::array::c_style | py::array::forcecast> rp,
                        py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx,
                        py::array_t<float, py::array::c_style | py::array::forcecast> val) {
  const int64_t n = rp.size() - 1;
  if (n < 0) throw std::invalid_argument("row_ptr is empty");
  const int64_t* r = rp.data();
  const int64_t nnz = r[n];
  if (idx.size() < nnz || val.size() < nnz) throw std::invalid_argument("CSR shorter than row_ptr");
  const int64_t* ix = idx.data();
  const float* vx = val.data();
  py::array_t<int64_t> lens(n);
  py::array_t<double> n2(n);
  std::vector<int32_t> oi;
  std::vector<float> ov;
  oi.reserve(nnz);
  ov.reserve(nnz);
  std::vector<int64_t> ord;
  auto* L = lens.mutable_data();
  auto* N2 = n2.mutable_data();
  for (int64_t i = 0; i < n; ++i) {
    ord.clear();
    for (int64_t j = r[i]; j < r[i + 1]; ++j)
      if (ix[j] >= 0) ord.push_back(j);
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return ix[a] < ix[b]; });
    const size_t start = oi.size();
    double sq = 0.0;
    for (size_t k = 0; k < ord.size();) {
      const int64_t f = ix[ord[k]];
      double acc = 0.0;
      while (k < ord.size() && ix[ord[k]] == f) acc += (double)vx[ord[k++]];
      const float v32 = (float)acc;
      oi.push_back((int32_t)f);
      ov.push_back(v32);
      sq += (double)v32 * (double)v32;
    }
    L[i] = (int64_t)(oi.size() - start);
    N2[i] = sq;
  }
  py::array_t<int32_t> ai((py::ssize_t)oi.size());
  py::array_t<float> av((py::ssize_t)ov.size());
  if (!oi.empty()) {
    memcpy(ai.mutable_data(), oi.data(), oi.size() * 4);
    memcpy(av.mutable_data(), ov.data(), ov.size() * 4);
  }
  return py::make_tuple(lens, ai, av, n2);
}

int64_t frame(py::buffer b) {
  py::buffer_info bi = b.request();
  return jb::msgpack_frame((const uint8_t*)bi.ptr, (size_t)(bi.size * bi.itemsize));
}

}  // namespace

void register_synth(py::module_& m);   // jb_synth.cpp
void register_cpu_serial(py::module_& m);   // jb_cpu_serial.cpp

PYBIND11_MODULE(_jubatus_native, m) {
  register_synth(m);
  register_cpu_serial(m);
  m.def("csr_normalize", &csr_normalize, "sort / merge / drop-negative a CSR per row, with norms");
  m.doc() = "jubatus_amd host-native runtime: request scanning, hashing, CRC32, MD5";
  py::class_<jb::LabelTable>(m, "LabelTable")
      .def(py::init<>())
      .def("get_or_add", [](jb::LabelTable& t, const std::string& s) { return t.get_or_add(s.data(), s.size()); })
      .def("lookup", &jb::LabelTable::lookup)
      .def("remove", &jb::LabelTable::remove)
      .def("clear", &jb::LabelTable::clear)
      .def("size", &jb::LabelTable::size)
      .def("names", &jb::LabelTable::names)
      .def("alive", &jb::LabelTable::alive)
      .def("version", &jb::LabelTable::version)
      .def("count", &jb::LabelTable::count)
      .def("set_count", &jb::LabelTable::set_count)
      .def("add_count", &jb::LabelTable::add_count);
  py::class_<jb::HostFvHasher>(m, "HostFvHasher")
      .def(py::init(&make_hasher))
      .def("hash", &hasher_hash, "hash msgpack list<datum> bodies into CSR (idx, val, row_ptr)",
           py::arg("reqs"), py::arg("idx"), py::arg("val"), py::arg("row_ptr"),
           py::arg("max_samples"), py::arg("max_slots"), py::arg("update") = false);
  py::class_<jb::PyRandom>(m, "PyRandom", "CPython random.Random twin (jb_pyrandom.hpp)")
      .def(py::init<int64_t>())
      .def("random", &jb::PyRandom::random)
      .def("getrandbits", &jb::PyRandom::getrandbits)
      .def("randbelow", &jb::PyRandom::randbelow)
      .def("sample_range", &jb::PyRandom::sample_range)
      .def("choice_weighted", &jb::PyRandom::choice_weighted);
  py::class_<jb::HostFvWide>(m, "HostFvWide")
      .def(py::init(&make_wide))
      .def("set_weights", [](jb::HostFvWide& h, uintptr_t df, uintptr_t diff, uintptr_t counts) {
        h.set_weights((int64_t*)df, (int64_t*)diff, (int64_t*)counts);
      })
      .def("needs_weights", &jb::HostFvWide::needs_weights)
      .def("hash", &wide_hash, "wide-rule converter: msgpack list<datum> bodies -> CSR",
           py::arg("reqs"), py::arg("idx"), py::arg("val"), py::arg("row_ptr"),
           py::arg("max_samples"), py::arg("max_slots"), py::arg("update") = false)
      .def("hash_named", &wide_hash_named,
           "one list<datum> body -> (err, row_ptr, idx, val, names, name_end, datum spans)",
           py::arg("body"), py::arg("update") = false);
  m.def("pack_requests", &pack, "scan msgpack request bodies into a device-ready batch");
  m.def("pack_spans", &pack_spans, "zero-copy scan of request spans inside one pinned arena");
  py::class_<PyRpcServer>(m, "RpcServer")
      .def(py::init<py::object, int, double>(), py::arg("handler"), py::arg("nworkers") = 2,
           py::arg("idle_timeout") = 0.0)
      .def("set_batch", &PyRpcServer::set_batch, py::arg("methods"), py::arg("fn"),
           py::arg("max_batch") = 4096)
      .def("batches", &PyRpcServer::batches)
      .def("set_arena_batch", &PyRpcServer::set_arena_batch, py::arg("method"), py::arg("slots"),
           py::arg("slot_bytes"), py::arg("fn"))
      .def("release_slot", &PyRpcServer::release_slot)
      .def("set_max_message", &PyRpcServer::set_max_message)
      .def("set_io_threads", &PyRpcServer::set_io_threads)
      .def("set_batch_threads", &PyRpcServer::set_batch_threads)
      .def("set_ordered", &PyRpcServer::set_ordered, py::arg("methods"))
      .def("arena_ns", &PyRpcServer::arena_ns)
      .def("listen", &PyRpcServer::listen)
      .def("start", &PyRpcServer::start)
      .def("stop", &PyRpcServer::stop)
      .def("running", &PyRpcServer::running)
      .def("served", &PyRpcServer::served)
      .def("connections", &PyRpcServer::connections);
  m.def("msgpack_frame", &frame, "length of the first complete msgpack object (0: incomplete, -1: bad)");
  m.def("frame_stream",
        [](py::buffer b, size_t cut, bool speculative) {
          // tests: frame a byte stream delivered in two reads ([0, cut), then
          // the rest) -> (message ends, rc, pending pos, pending rem)
          py::buffer_info bi = b.request();
          const uint8_t* p = (const uint8_t*)bi.ptr;
          const size_t n = (size_t)(bi.size * bi.itemsize);
          std::vector<uint64_t> ends;
          jb::FrameState st;
          int rc = 0;
          uint64_t base = 0;
          for (size_t upto : {std::min(cut, n), n}) {
            if (upto <= base) continue;
            std::vector<uint64_t> e;
            if (speculative) {
              rc = jb::frame_all(p + base, upto - base, st, &e, true);
            } else {
              for (;;) {
                const uint64_t off = e.empty() ? 0 : e.back();
                rc = jb::frame_resume(p + base + off, upto - base - off, st);
                if (rc <= 0) break;
                e.push_back(off + st.pos);
                st.reset();
              }
            }
            for (auto x : e) ends.push_back(base + x);
            if (!e.empty()) base += e.back();
            if (rc < 0) break;
          }
          if (!st.started) { st.pos = 0; st.rem = 1; }    // a fresh message: nothing pending
          return py::make_tuple(ends, rc, st.pos, st.rem);
        },
        py::arg("buf"), py::arg("cut"), py::arg("speculative"));
  m.def("crc32", &crc32, py::arg("data"), py::arg("init") = 0u);
  m.def("md5_hex", &md5_hex);
  m.def("feature_index", &feature_index);
  m.def("fnv1a64", &fnv1a64);
}
