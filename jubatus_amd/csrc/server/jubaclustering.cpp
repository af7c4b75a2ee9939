// jubaclustering, native: the clustering server without Python.
//
// Reference: jubatus/server/server/clustering_serv.cpp:71-151 (push,
// get_revision, get_core_members, get_k_center, get_nearest_center,
// get_nearest_members, clear) over jubatus_core's clustering (EXTERNAL).
// The engine is models/clustering.py's, step for step: points converted by
// the native wide converter in one call per push into a point set (weights,
// CSR of hashed feature keys, raw datum bytes, feature names recorded once
// per key); full buckets compressed (simple: the Python RNG's sample;
// compressive: k-means++ representatives weighted by the points they absorb,
// csrc/hip/clustering.hip), forgetting and merging of coresets, then
// k-means++ / Lloyd / GMM EM over every coreset point in single-workgroup HIP
// launches. The random stream is CPython's (csrc/native/jb_pyrandom.hpp), so
// the native and the Python server draw the same seeds. Model files are
// shared with the Python server (Clustering.pack(): pending / buckets /
// others as [weight, {feature: value}, datum]). idf / bm25 global weights
// count documents in the converter's hash_max_size rows (DocStats, MIXed
// with the coresets and kept in the model file under "weights"); converters
// outside the wide rule set go to the Python server.
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "jb_host_server.hpp"
#include "jb_linear_conv.hpp"
#include "jb_mix_device.hpp"
#include "jb_msgpack.hpp"
#include "jb_pyrandom.hpp"
#include "jb_wide_rules.hpp"

extern "C" int jb_argmin_rows(const float* D, int64_t n, int k, int32_t* out, hipStream_t stream);
extern "C" int jb_sqdist_mfma(const float* X, int64_t n, const float* C, int k, int d, const float* xn2,
                              const float* cn2, float* out, hipStream_t stream);
extern "C" int jb_kmeanspp(const float* X, int n, int d, const float* w, const double* u, int m, float* d2,
                           float* prob, int32_t* out, int32_t* status, hipStream_t stream);
extern "C" int jb_lloyd(const float* X, int n, int d, const float* w, float* C, int k, int iters, float atol,
                        float rtol, int32_t* assign, float* S, int32_t* done_iters, hipStream_t stream);
extern "C" int jb_gmm_em(const float* X, int n, int d, const float* w, float* C, float* var, float* pi, int k,
                         int iters, int32_t* assign, hipStream_t stream);

namespace {

using namespace jb::srv;

constexpr uint64_t kKeySpace = (1ull << 31) - 1;   // models/clustering.py KEY_SPACE

struct Params {
  std::string method;
  int k = 3;
  std::string compressor = "simple";
  int64_t bucket_size = 1000, compressed = 100, bicriteria = 10, bucket_length = 2;
  double forgetting_factor = 0.0, forgetting_threshold = 0.5;
  int64_t seed = 0;
  std::vector<jb::HostRule> s, n, c;
  std::string blob;
  uint64_t H = 1ull << 20;
  bool global = false;
  std::shared_ptr<jb::WideExt> ext;   // plug-ins, filters, binary rules
};

double num_or(const Value* p, const char* k, double d) {
  const Value* v = p ? p->get(k) : nullptr;
  if (!v) return d;
  if (v->is_num()) return v->num();
  if (v->is_str()) return atof(v->s.c_str());
  return d;
}

bool check_config(const std::string& text, std::string* why, Params* out) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  Params p;
  p.method = v.str_or("method", "");
  if (p.method != "kmeans" && p.method != "gmm") { *why = "unsupported clustering method: " + p.method; return false; }
  const Value* par = v.get("parameter");
  p.k = (int)num_or(par, "k", 3);
  if (const Value* c = par ? par->get("compressor_method") : nullptr) p.compressor = c->s;
  if (p.compressor != "simple" && p.compressor != "compressive_kmeans" && p.compressor != "compressive_gmm") {
    *why = "unknown compressor_method: " + p.compressor;
    return false;
  }
  p.bucket_size = (int64_t)num_or(par, "bucket_size", 1000);
  p.compressed = (int64_t)num_or(par, "compressed_bucket_size", 100);
  p.bicriteria = (int64_t)num_or(par, "bicriteria_base_size", 10);
  p.bucket_length = (int64_t)num_or(par, "bucket_length", 2);
  p.forgetting_factor = num_or(par, "forgetting_factor", 0.0);
  p.forgetting_threshold = num_or(par, "forgetting_threshold", 0.5);
  p.seed = (int64_t)num_or(par, "seed", 0);
  if (p.k <= 0 || p.bucket_size <= 0 || !(0 < p.compressed && p.compressed <= p.bucket_size)) {
    *why = "invalid clustering parameter (k, bucket_size, compressed_bucket_size)";
    return false;
  }
  if (p.bucket_length < 1) { *why = "bucket_length must be positive"; return false; }
  const Value* conv = v.get("converter");
  Value empty;
  empty.kind = Value::MAP;
  if (!jb::row::build_wide_rules(conv ? *conv : empty, &p.s, &p.n, &p.c, &p.blob, &p.H, &p.global, why, &p.ext))
    return false;
  if (out) *out = std::move(p);
  return true;
}

// ------------------------------------------------------------ point sets
struct PointSet {
  std::vector<double> w;
  std::vector<int64_t> rp{0};
  std::vector<int64_t> key;
  std::vector<float> val;
  std::vector<std::string> raw;     // msgpack of each point's datum

  size_t size() const { return w.size(); }
  void append(const PointSet& o) {
    const int64_t off = rp.back();
    for (size_t i = 1; i < o.rp.size(); ++i) rp.push_back(o.rp[i] + off);
    w.insert(w.end(), o.w.begin(), o.w.end());
    key.insert(key.end(), o.key.begin(), o.key.end());
    val.insert(val.end(), o.val.begin(), o.val.end());
    raw.insert(raw.end(), o.raw.begin(), o.raw.end());
  }
  PointSet take(const std::vector<int64_t>& rows, const std::vector<double>* nw = nullptr) const {
    PointSet o;
    for (size_t t = 0; t < rows.size(); ++t) {
      const int64_t r = rows[t];
      o.w.push_back(nw ? (*nw)[t] : w[(size_t)r]);
      for (int64_t s = rp[(size_t)r]; s < rp[(size_t)r + 1]; ++s) {
        o.key.push_back(key[(size_t)s]);
        o.val.push_back(val[(size_t)s]);
      }
      o.rp.push_back((int64_t)o.key.size());
      o.raw.push_back(raw[(size_t)r]);
    }
    return o;
  }
};

void put_value(MsgpackWriter& w, const Value& v) {
  switch (v.kind) {
    case Value::NIL: w.nil(); break;
    case Value::BOOL: w.boolean(v.b); break;
    case Value::INT: w.sint(v.i); break;
    case Value::UINT: w.uint(v.u); break;
    case Value::DBL: w.dbl(v.d); break;
    case Value::STR: w.raw(v.s); break;
    case Value::BIN: w.bin(v.s.data(), v.s.size()); break;
    case Value::ARR:
      w.arr(v.a.size());
      for (const Value& x : v.a) put_value(w, x);
      break;
    case Value::MAP:
      w.map(v.o.size());
      for (const auto& kv : v.o) { w.raw(kv.first); put_value(w, kv.second); }
      break;
  }
}

template <class T>
struct Dev {
  T* p = nullptr;
  size_t cap = 0;
  ~Dev() { if (p) (void)hipFree(p); }
  T* get(size_t n) {
    if (n > cap) {
      if (p) HIPCHK(hipFree(p));
      HIPCHK(hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T)));
      cap = n;
    }
    return p;
  }
};

class Clustering : public HostEngine {
 public:
  explicit Clustering(Params p) : p_(std::move(p)), rng_(p_.seed) {
    hw_.reset(new jb::HostFvWide((const uint8_t*)p_.s.data(), (int)p_.s.size(), (const uint8_t*)p_.n.data(),
                                 (int)p_.n.size(), (const uint8_t*)p_.c.data(), (int)p_.c.size() / 2,
                                 (const uint8_t*)p_.blob.data(), p_.blob.size(), kKeySpace));
    hw_->set_ext(p_.ext);
    if (p_.global) {   // document statistics over the converter's table height
      stats_.reset(p_.H);
      stats_.attach(hw_.get());
      hw_->set_df_height(p_.H);
    }
    HIPCHK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&mix_st_, hipStreamNonBlocking));
    HIPCHK(hipGetDevice(&device_));
    token_ = std::to_string((uint64_t)getpid() * 0x9E3779B97F4A7C15ull ^ (uint64_t)time(nullptr) ^
                            (uint64_t)(uintptr_t)this);
  }
  ~Clustering() override {
    (void)hipStreamDestroy(st_);
    (void)hipStreamDestroy(mix_st_);
  }

  // ---------------------------------------------------------- MIX
  // models/clustering.py get_diff / mix_diff / put_diff: every member ships
  // its coresets (all buckets) under its token; each member clusters its
  // own coresets plus every other member's (clustering_serv.cpp:108-142)
  bool mixable() const override { return true; }
  std::unique_ptr<jb::mix::Plane> make_plane(jb::mix::Star& s, double dl) override {
    return jb::mix::make_device_plane(s, device_, mix_st_, dl);
  }
  // The members agree on the clustering of a MIX: every member clusters the
  // coresets in rank order (its own at its rank) and seeds k-means++ from
  // the largest revision among them, so the centers are the same everywhere.
  std::string get_diff() override {
    PointSet all;
    for (const auto& b : buckets_) all.append(b);
    MsgpackWriter u;
    u.arr(4);
    u.str(token_);
    wire(u, all);
    u.uint(revision_);
    if (p_.global) u.out += stats_.get_diff();   // the weight manager's diff (encoded)
    else u.nil();
    return std::move(u.out);
  }
  void put_diffs(const std::vector<Value>& parts) override {
    PointSet before, after, others;
    bool mine = false;
    uint64_t rev = revision_;
    std::vector<Value> wd;
    for (const Value& d : parts) {
      if (d.kind != Value::ARR || d.a.size() < 3) throw std::runtime_error("mix: malformed clustering diff");
      if (d.a.size() > 3 && d.a[3].kind == Value::ARR) wd.push_back(d.a[3]);
      rev = std::max<uint64_t>(rev, (uint64_t)d.a[2].num());
      if (d.a[0].s == token_) { mine = true; continue; }
      PointSet ps = unwire(d.a[1]);
      others.append(ps);
      (mine ? after : before).append(ps);
    }
    others_ = std::move(others);
    revision_ = rev;
    if (p_.global && !wd.empty()) stats_.put_diffs(wd);
    if (!buckets_.empty() || others_.size()) recluster(&before, &after);
  }

  void set_lock(std::shared_mutex* mu) override { mu_ = mu; }

  std::vector<HostMethod> methods() override {
    std::vector<HostMethod> m = {
        {"push", 2, true, nullptr, [this](const std::string& params, MsgpackWriter* w) { push_raw(params, w); },
         true},
        {"get_revision", 1, false, [this](const std::vector<Value>&, MsgpackWriter* w) { w->uint(revision_); }},
        {"get_core_members", 1, false,
         [this](const std::vector<Value>&, MsgpackWriter* w) { core_members(w); }},
        {"get_k_center", 1, false, [this](const std::vector<Value>&, MsgpackWriter* w) { k_center(w); }},
        {"get_nearest_center", 2, false,
         [this](const std::vector<Value>& a, MsgpackWriter* w) { center_datum(nearest(a[0]), w); }},
        {"get_nearest_members", 2, false,
         [this](const std::vector<Value>& a, MsgpackWriter* w) { members_of(nearest(a[0]), w); }},
        {"clear", 1, true, [this](const std::vector<Value>&, MsgpackWriter* w) {
           clear();
           w->boolean(true);
         }},
    };
    return m;
  }

  void clear() override {
    pending_ = PointSet();
    buckets_.clear();
    others_ = PointSet();
    core_ = PointSet();
    revision_ = 0;
    centers_.clear();
    var_.clear();
    pi_.clear();
    dims_.clear();
    dim_keys_.clear();
    assign_.clear();
    rng_ = jb::PyRandom(p_.seed);
    stats_.clear();
  }

  // ---------------------------------------------------------- persist
  std::string pack() override {
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(p_.global ? 6 : 5);
    u.str("method"); u.str(p_.method);
    u.str("revision"); u.uint(revision_);
    u.str("pending"); wire(u, pending_);
    u.str("buckets"); u.arr(buckets_.size());
    for (const auto& b : buckets_) wire(u, b);
    u.str("others"); wire(u, others_);
    if (p_.global) { u.str("weights"); stats_.pack(u); }
    return std::move(u.out);
  }

  void unpack(const Value& obj) override {
    const Value* pv = obj.get("pending");
    const Value* bv = obj.get("buckets");
    const Value* ov = obj.get("others");
    const Value* rv = obj.get("revision");
    if (!pv || !bv || !ov || !rv || bv->kind != Value::ARR) throw std::runtime_error("broken model data: clustering");
    clear();
    pending_ = unwire(*pv);
    for (const Value& b : bv->a) buckets_.push_back(unwire(b));
    others_ = unwire(*ov);
    if (p_.global) stats_.unpack(obj.get("weights"));
    const uint64_t rev = (uint64_t)rv->num();
    if (!buckets_.empty() || others_.size()) recluster();
    revision_ = rev;
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) override {
    st->emplace_back("method", p_.method);
    st->emplace_back("k", std::to_string(p_.k));
    st->emplace_back("revision", std::to_string(revision_));
    st->emplace_back("pending", std::to_string(pending_.size()));
    st->emplace_back("buckets", std::to_string(buckets_.size()));
    st->emplace_back("compressor_method", p_.compressor);
    st->emplace_back("storage", "hbm");
    st->emplace_back("converter", "native");
    st->emplace_back("server_runtime", "native");
  }

 private:
  // ---------------------------------------------------------- convert
  // hashing scratch of one converter
  struct Conv {
    jb::HostFvWide* h = nullptr;
    std::unique_ptr<jb::HostFvWide> own;   // a pooled converter's hasher
    std::vector<int32_t> idx;
    std::vector<float> fv;
    std::vector<int64_t> rp;
  };
  // one msgpack list<datum> body -> points (weight 1); false: malformed.
  // names: the (key, name) of each distinct feature key the body holds
  bool convert(Conv& cv, const uint8_t* body, size_t len, bool update, PointSet* out,
               std::vector<std::pair<int64_t, std::string>>* names_out) {
    std::string names;
    std::vector<int64_t> name_end, spans;
    cv.idx.resize(std::max<size_t>(cv.idx.size(), 4096));
    cv.fv.resize(cv.idx.size());
    cv.rp.resize(std::max<size_t>(cv.rp.size(), 1025));
    jb::HostFvWide& h = *cv.h;
    int rc;
    int64_t n = 0, slots = 0;
    for (;;) {
      n = slots = 0;
      names.clear();
      name_end.clear();
      spans.clear();
      cv.rp[0] = 0;
      h.set_sinks(&names, &name_end, &spans);
      if (p_.global) h.begin();
      rc = h.hash_body(body, len, cv.idx.data(), cv.fv.data(), cv.rp.data(), (int64_t)cv.rp.size() - 1,
                       (int64_t)cv.idx.size(), &n, &slots, update);
      h.set_sinks(nullptr, nullptr, nullptr);
      if (rc != 0 && p_.global) h.rollback();   // a retry / a malformed body counts nothing
      if (rc != 2) break;
      cv.idx.resize(cv.idx.size() * 4);
      cv.fv.resize(cv.idx.size());
      cv.rp.resize(cv.rp.size() * 4);
    }
    if (rc) return false;
    int64_t st = 0;
    for (int64_t s = 0; s < slots; ++s) {
      const int64_t k = cv.idx[(size_t)s];
      bool seen = false;   // (a body holds a handful of distinct keys)
      for (const auto& kv : *names_out)
        if (kv.first == k) { seen = true; break; }
      if (!seen) names_out->emplace_back(k, names.substr((size_t)st, (size_t)(name_end[(size_t)s] - st)));
      st = name_end[(size_t)s];
      out->key.push_back(k);
      out->val.push_back(cv.fv[(size_t)s]);
    }
    const int64_t off = out->rp.back();
    for (int64_t i = 0; i < n; ++i) {
      out->rp.push_back(off + cv.rp[(size_t)i + 1]);
      out->w.push_back(1.0);
      out->raw.emplace_back((const char*)body + spans[2 * (size_t)i],
                            (size_t)(spans[2 * (size_t)i + 1] - spans[2 * (size_t)i]));
    }
    return true;
  }
  // the engine's own converter (hw_: the document statistics hang off it)
  bool convert(const uint8_t* body, size_t len, bool update, PointSet* out) {
    main_.h = hw_.get();
    std::vector<std::pair<int64_t, std::string>> nm;
    if (!convert(main_, body, len, update, out, &nm)) return false;
    for (auto& kv : nm)
      if (!names_.count(kv.first)) names_[kv.first] = std::move(kv.second);
    return true;
  }
  // converters for pushes hashed outside the model lock (no document
  // statistics: p_.global is false), one per push in flight
  std::unique_ptr<Conv> take_conv() {
    {
      std::lock_guard<std::mutex> g(conv_mu_);
      if (!conv_pool_.empty()) {
        std::unique_ptr<Conv> c = std::move(conv_pool_.back());
        conv_pool_.pop_back();
        return c;
      }
    }
    std::unique_ptr<Conv> c(new Conv);
    c->own.reset(new jb::HostFvWide((const uint8_t*)p_.s.data(), (int)p_.s.size(), (const uint8_t*)p_.n.data(),
                                    (int)p_.n.size(), (const uint8_t*)p_.c.data(), (int)p_.c.size() / 2,
                                    (const uint8_t*)p_.blob.data(), p_.blob.size(), kKeySpace));
    c->own->set_ext(p_.ext);
    c->h = c->own.get();
    return c;
  }
  void give_conv(std::unique_ptr<Conv> c) {
    std::lock_guard<std::mutex> g(conv_mu_);
    conv_pool_.push_back(std::move(c));
  }

  // push: HostMethod::self_lock - without document statistics the points
  // are hashed before the model lock (pushes in flight hash in parallel on
  // the RPC workers while one closes a bucket), then appended under it
  void push_raw(const std::string& params, MsgpackWriter* w) {
    jb::Cursor c{(const uint8_t*)params.data(), (const uint8_t*)params.data() + params.size()};
    uint32_t two;
    const uint8_t* nm;
    uint32_t nn;
    if (!c.array(&two) || two != 2 || !c.raw(&nm, &nn)) throw std::invalid_argument("push");
    PointSet ps;
    auto t0 = Clock::now();
    if (!p_.global && mu_ != nullptr) {
      std::unique_ptr<Conv> cv = take_conv();
      std::vector<std::pair<int64_t, std::string>> names;
      const bool ok = convert(*cv, c.p, (size_t)(c.end - c.p), true, &ps, &names);
      give_conv(std::move(cv));
      if (!ok) throw std::invalid_argument("push: malformed points");
      const double conv_us = since_us(t0);
      std::unique_lock<std::shared_mutex> g(*mu_);
      if (prof_.on) prof_.us[5] += conv_us;
      for (auto& kv : names)
        if (!names_.count(kv.first)) names_[kv.first] = std::move(kv.second);
      append_points(std::move(ps));
    } else {
      std::unique_lock<std::shared_mutex> g;
      if (mu_ != nullptr) g = std::unique_lock<std::shared_mutex>(*mu_);
      if (!convert(c.p, (size_t)(c.end - c.p), true, &ps)) throw std::invalid_argument("push: malformed points");
      if (prof_.on) prof_.us[5] += since_us(t0);
      append_points(std::move(ps));
    }
    w->boolean(true);
  }
  // (model lock held) the points join the pending bucket; full buckets close
  void append_points(PointSet&& ps) {
    auto t0 = Clock::now();
    if (pending_.size() == 0) pending_ = std::move(ps);
    else pending_.append(ps);
    while ((int64_t)pending_.size() >= p_.bucket_size) {
      PointSet full;
      if ((int64_t)pending_.size() == p_.bucket_size) {   // the common case: a whole bucket, no copies
        full = std::move(pending_);
        pending_ = PointSet();
      } else {
        std::vector<int64_t> head((size_t)p_.bucket_size), tail(pending_.size() - (size_t)p_.bucket_size);
        std::iota(head.begin(), head.end(), 0);
        std::iota(tail.begin(), tail.end(), p_.bucket_size);
        full = pending_.take(head);
        pending_ = pending_.take(tail);
      }
      if (prof_.on) prof_.us[6] += since_us(t0);
      close_bucket(full);
      t0 = Clock::now();
    }
    if (prof_.on) prof_.us[6] += since_us(t0);
  }

  // ---------------------------------------------------------- dense
  // feature keys of a set ordered by name, and those names
  void columns(const PointSet& ps, std::vector<int64_t>* keys, std::vector<std::string>* dims) {
    // distinct keys: a linear scan while there are few (a bucket's points
    // share a handful of columns), a sort past that
    std::vector<int64_t> k;
    bool few = true;
    for (int64_t x : ps.key) {
      if (std::find(k.begin(), k.end(), x) != k.end()) continue;
      k.push_back(x);
      if (k.size() > 32) { few = false; break; }
    }
    if (!few) {
      k = ps.key;
      std::sort(k.begin(), k.end());
      k.erase(std::unique(k.begin(), k.end()), k.end());
    }
    std::vector<size_t> order(k.size());
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return names_[k[a]] < names_[k[b]]; });
    keys->clear();
    dims->clear();
    for (size_t i : order) { keys->push_back(k[i]); dims->push_back(names_[k[i]]); }
  }

  std::vector<float> dense(const PointSet& ps, const std::vector<int64_t>& keys) {
    const size_t m = ps.size(), D = keys.size();
    std::vector<float> X(m * D, 0.f);
    if (D <= 32) {   // few columns: a linear scan beats hashing
      for (size_t r = 0; r < m; ++r)
        for (int64_t s = ps.rp[r]; s < ps.rp[r + 1]; ++s) {
          const int64_t kk = ps.key[(size_t)s];
          for (size_t j = 0; j < D; ++j)
            if (keys[j] == kk) { X[r * D + j] += ps.val[(size_t)s]; break; }
        }
      return X;
    }
    std::unordered_map<int64_t, size_t> col;
    for (size_t j = 0; j < D; ++j) col[keys[j]] = j;
    for (size_t r = 0; r < m; ++r)
      for (int64_t s = ps.rp[r]; s < ps.rp[r + 1]; ++s) {
        auto it = col.find(ps.key[(size_t)s]);
        if (it != col.end()) X[r * D + it->second] += ps.val[(size_t)s];
      }
    return X;
  }

  // squared distances [n][m] of rows X to rows C on the matrix cores
  std::vector<float> sqdist(const std::vector<float>& X, size_t n, const std::vector<float>& C, size_t m,
                            size_t D) {
    std::vector<float> xn(n, 0.f), cn(m, 0.f), out(n * m);
    for (size_t i = 0; i < n; ++i)
      for (size_t q = 0; q < D; ++q) xn[i] += X[i * D + q] * X[i * D + q];
    for (size_t j = 0; j < m; ++j)
      for (size_t q = 0; q < D; ++q) cn[j] += C[j * D + q] * C[j * D + q];
    float* dx = dX_.get(n * D);
    float* dc = dC_.get(m * D);
    float* dxn = dXn_.get(n);
    float* dcn = dCn_.get(m);
    float* dout = dOut_.get(n * m);
    h2d(dx, X.data(), 4 * n * D);
    h2d(dc, C.data(), 4 * m * D);
    h2d(dxn, xn.data(), 4 * n);
    h2d(dcn, cn.data(), 4 * m);
    if (jb_sqdist_mfma(dx, (int64_t)n, dc, (int)m, (int)D, dxn, dcn, dout, st_) != 0)
      throw std::runtime_error("jb_sqdist_mfma failed");
    d2h(out.data(), dout, 4 * n * m);
    sync();
    return out;
  }

  // nearest row of C [m][D] for every row of X (the sqdist values and the
  // first-minimum rule of sqdist + argmin), computed and reduced on the
  // device: n indices come back instead of n x m distances. x_dev: X is in
  // dX_ already (the k-means++ call just uploaded it)
  std::vector<int32_t> nearest(const std::vector<float>& X, size_t n, const std::vector<float>& C, size_t m,
                               size_t D, bool x_dev) {
    std::vector<float> xn(n, 0.f), cn(m, 0.f);
    for (size_t i = 0; i < n; ++i)
      for (size_t q = 0; q < D; ++q) xn[i] += X[i * D + q] * X[i * D + q];
    for (size_t j = 0; j < m; ++j)
      for (size_t q = 0; q < D; ++q) cn[j] += C[j * D + q] * C[j * D + q];
    float* dx = dX_.get(n * D);
    float* dc = dC_.get(m * D);
    float* dxn = dXn_.get(n);
    float* dcn = dCn_.get(m);
    float* dout = dOut_.get(n * m);
    int32_t* da = dA_.get(n);
    if (!x_dev) h2d(dx, X.data(), 4 * n * D);
    h2d(dc, C.data(), 4 * m * D);
    h2d(dxn, xn.data(), 4 * n);
    h2d(dcn, cn.data(), 4 * m);
    if (jb_sqdist_mfma(dx, (int64_t)n, dc, (int)m, (int)D, dxn, dcn, dout, st_) != 0 ||
        jb_argmin_rows(dout, (int64_t)n, (int)m, da, st_) != 0)
      throw std::runtime_error("jb_sqdist_mfma failed");
    std::vector<int32_t> a(n);
    d2h(a.data(), da, 4 * n);
    sync();
    return a;
  }

  // k-means++ over rows of X (models/clustering.py _kmeanspp: one uniform per
  // draw for the device kernel, the host draws after a zero-mass stop)
  std::vector<int64_t> kmeanspp(const std::vector<float>& X, const std::vector<float>& w, size_t n, size_t D,
                                int64_t m, jb::PyRandom& rng) {
    m = std::min<int64_t>(m, (int64_t)n);
    std::vector<double> u((size_t)m);
    for (auto& x : u) x = rng.random();
    float* dx = dX_.get(n * D);
    float* dw = dW_.get(n);
    double* du = dU_.get((size_t)m);
    float* scr = dScr_.get(2 * n);
    int32_t* dout = dI_.get((size_t)m + 1);
    h2d(dx, X.data(), 4 * n * D);
    h2d(dw, w.data(), 4 * n);
    h2d(du, u.data(), 8 * (size_t)m);
    if (jb_kmeanspp(dx, (int)n, (int)D, dw, du, (int)m, scr, scr + n, dout, dout + m, st_) != 0)
      throw std::runtime_error("jb_kmeanspp failed");
    std::vector<int32_t> o((size_t)m + 1);
    d2h(o.data(), dout, 4 * ((size_t)m + 1));
    sync();
    const int status = o[(size_t)m];
    std::vector<int64_t> chosen;
    if (status == 0) {
      for (int64_t j = 0; j < m; ++j) chosen.push_back(o[(size_t)j]);
      return chosen;
    }
    for (int j = 0; j < status - 1; ++j) chosen.push_back(o[(size_t)j]);
    if (chosen.empty()) {
      std::vector<double> wd(w.begin(), w.end());
      chosen.push_back(rng.choice_weighted(wd));
    }
    std::vector<float> d2(n, INFINITY);
    auto relax = [&](int64_t c) {
      std::vector<float> C(X.begin() + c * (int64_t)D, X.begin() + (c + 1) * (int64_t)D);
      const auto dd = sqdist(X, n, C, 1, D);
      for (size_t i = 0; i < n; ++i) d2[i] = std::min(d2[i], dd[i]);
    };
    for (int64_t c : chosen) relax(c);
    while ((int64_t)chosen.size() < m) {
      std::vector<double> prob(n);
      double s = 0;
      for (size_t i = 0; i < n; ++i) { prob[i] = (double)(d2[i] * w[i]); s += prob[i]; }
      int64_t nxt;
      if (s <= 0) {
        std::vector<int64_t> rest;
        for (size_t i = 0; i < n; ++i)
          if (std::find(chosen.begin(), chosen.end(), (int64_t)i) == chosen.end()) rest.push_back((int64_t)i);
        if (rest.empty()) break;
        nxt = rest[(size_t)rng.choice_index((int64_t)rest.size())];
      } else {
        nxt = rng.choice_weighted(prob);
      }
      chosen.push_back(nxt);
      relax(nxt);
    }
    return chosen;
  }

  PointSet compress(const PointSet& ps, int64_t m) {
    if ((int64_t)ps.size() <= m) return ps;
    if (p_.compressor == "simple") {
      const auto idx = rng_.sample_range((int64_t)ps.size(), m);
      double tot = 0, sel = 0;
      for (double x : ps.w) tot += x;
      for (int64_t i : idx) sel += ps.w[(size_t)i];
      const double scale = tot / sel;
      std::vector<double> nw;
      for (int64_t i : idx) nw.push_back(ps.w[(size_t)i] * scale);
      return ps.take(idx, &nw);
    }
    std::vector<int64_t> keys;
    std::vector<std::string> dims;
    columns(ps, &keys, &dims);
    const size_t n = ps.size(), D = keys.size();
    const auto X = dense(ps, keys);
    std::vector<float> w(ps.w.begin(), ps.w.end());
    auto t0 = Clock::now();
    const auto reps = kmeanspp(X, w, n, D, m, rng_);
    if (prof_.on) prof_.us[7] += since_us(t0);
    t0 = Clock::now();
    std::vector<float> C;
    for (int64_t r : reps) C.insert(C.end(), X.begin() + r * (int64_t)D, X.begin() + (r + 1) * (int64_t)D);
    // (X is in dX_ from the k-means++ call: its kernel path uploaded it, and
    // its host fallback's sqdist calls upload the same rows)
    const auto asg = nearest(X, n, C, reps.size(), D, true);
    if (prof_.on) prof_.us[8] += since_us(t0);
    std::vector<float> ws(reps.size(), 0.f);
    for (size_t i = 0; i < n; ++i) ws[(size_t)asg[i]] += w[i];
    std::vector<int64_t> keep;
    std::vector<double> nw;
    for (size_t j = 0; j < reps.size(); ++j)
      if (ws[j] > 0) { keep.push_back(reps[j]); nw.push_back((double)ws[j]); }
    return ps.take(keep, &nw);
  }

  // JB_CLUSTER_PROF=1: wall time per phase of a closed bucket, logged every
  // 50 buckets (compress, merge-compress, k-means++, Lloyd, EM)
  struct Prof {
    bool on = false;
    // compress, merge, k-means++, Lloyd, EM; push conversion, the bucket
    // hand-over, compress's k-means++ and nearest calls
    double us[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int64_t buckets = 0;
  } prof_;
  using Clock = std::chrono::steady_clock;
  static double since_us(Clock::time_point t0) {
    return std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
  }

  void close_bucket(const PointSet& full) {
    static const bool prof_on = [] {
      const char* e = getenv("JB_CLUSTER_PROF");
      return e != nullptr && e[0] == '1';
    }();
    prof_.on = prof_on;
    auto t0 = Clock::now();
    PointSet core = compress(full, p_.compressed);
    if (prof_.on) prof_.us[0] += since_us(t0);
    if (p_.forgetting_factor > 0) {
      const double f = exp(-p_.forgetting_factor);
      std::vector<PointSet> out;
      for (const auto& b : buckets_) {
        std::vector<int64_t> keep;
        std::vector<double> nw;
        for (size_t i = 0; i < b.size(); ++i) {
          const double x = b.w[i] * f;
          if (x >= p_.forgetting_threshold) { keep.push_back((int64_t)i); nw.push_back(x); }
        }
        if (!keep.empty()) out.push_back(b.take(keep, &nw));
      }
      buckets_.swap(out);
    }
    buckets_.push_back(std::move(core));
    t0 = Clock::now();
    while ((int64_t)buckets_.size() > p_.bucket_length) {
      PointSet both = buckets_[0];
      both.append(buckets_[1]);
      PointSet merged = compress(both, p_.compressed);
      buckets_.erase(buckets_.begin(), buckets_.begin() + 2);
      buckets_.insert(buckets_.begin(), std::move(merged));
    }
    if (prof_.on) prof_.us[1] += since_us(t0);
    recluster();
    if (prof_.on && ++prof_.buckets % 50 == 0)
      fprintf(stderr,
              "cluster prof: %lld buckets, us per bucket: compress %.1f merge %.1f kmeans++ %.1f lloyd %.1f "
              "em %.1f convert %.1f hand-over %.1f compress.kmeans++ %.1f compress.nearest %.1f\n",
              (long long)prof_.buckets, prof_.us[0] / prof_.buckets, prof_.us[1] / prof_.buckets,
              prof_.us[2] / prof_.buckets, prof_.us[3] / prof_.buckets, prof_.us[4] / prof_.buckets,
              prof_.us[5] / prof_.buckets, prof_.us[6] / prof_.buckets, prof_.us[7] / prof_.buckets,
              prof_.us[8] / prof_.buckets);
  }

  // ---------------------------------------------------------- cluster
  // over this member's coresets and the others' (a MIX passes the others
  // split around this member's rank: the rank order every member shares)
  void recluster(const PointSet* before = nullptr, const PointSet* after = nullptr) {
    PointSet pts;
    if (before) pts.append(*before);
    for (const auto& b : buckets_) pts.append(b);
    pts.append(after ? *after : others_);
    if ((int64_t)pts.size() < p_.k) return;
    std::vector<int64_t> keys;
    std::vector<std::string> dims;
    columns(pts, &keys, &dims);
    const size_t n = pts.size(), D = keys.size(), k = (size_t)p_.k;
    const auto X = dense(pts, keys);
    std::vector<float> w(pts.w.begin(), pts.w.end());
    jb::PyRandom rng(p_.seed + (int64_t)revision_);
    auto t0 = Clock::now();
    const auto seeds = kmeanspp(X, w, n, D, (int64_t)k, rng);
    if (prof_.on) prof_.us[2] += since_us(t0);
    t0 = Clock::now();
    std::vector<float> C;
    for (int64_t r : seeds) C.insert(C.end(), X.begin() + r * (int64_t)D, X.begin() + (r + 1) * (int64_t)D);
    const size_t kk = seeds.size();
    std::vector<int32_t> assign(n, 0);
    // Lloyd on the device (models/clustering.py: 100 iterations, allclose 1e-6 / 1e-5)
    float* dx = dX_.get(n * D);
    float* dw = dW_.get(n);
    float* dc = dC_.get(kk * D);
    int32_t* da = dA_.get(n);
    int32_t* dd = dI_.get(1);
    h2d(dx, X.data(), 4 * n * D);
    h2d(dw, w.data(), 4 * n);
    h2d(dc, C.data(), 4 * kk * D);
    int rc = jb_lloyd(dx, (int)n, (int)D, dw, dc, (int)kk, 100, 1e-6f, 1e-5f, da, nullptr, dd, st_);
    const bool gmm = p_.method == "gmm";
    const bool lloyd_dev = rc != -2;    // Lloyd's centers are in dc
    if (prof_.on && gmm) {   // (kmeans: the Lloyd time includes the read-back below)
      sync();
      prof_.us[3] += since_us(t0);
      t0 = Clock::now();
    }
    if (rc == -2) {
      host_lloyd(X, w, n, D, kk, &C, &assign);   // k x dims beyond the kernel's LDS
    } else {
      if (rc) throw std::runtime_error("jb_lloyd failed");
      if (!gmm) {   // GMM's EM starts from Lloyd's centers where they are (no round trip)
        d2h(C.data(), dc, 4 * kk * D);
        d2h(assign.data(), da, 4 * n);
        sync();
      }
    }
    if (gmm) {
      std::vector<float> var(kk * D, 1.f), pi(kk, 1.f / (float)kk);
      float* dv = dV_.get(kk * D);
      float* dp = dP_.get(kk);
      if (rc == -2) h2d(dc, C.data(), 4 * kk * D);
      h2d(dv, var.data(), 4 * kk * D);
      h2d(dp, pi.data(), 4 * kk);
      rc = jb_gmm_em(dx, (int)n, (int)D, dw, dc, dv, dp, (int)kk, 50, da, st_);
      if (rc == -2) {
        if (lloyd_dev) {
          d2h(C.data(), dc, 4 * kk * D);
          sync();
        }
        host_em(X, w, n, D, kk, &C, &var, &pi, &assign);
      } else {
        if (rc) throw std::runtime_error("jb_gmm_em failed");
        d2h(C.data(), dc, 4 * kk * D);
        d2h(var.data(), dv, 4 * kk * D);
        d2h(pi.data(), dp, 4 * kk);
        d2h(assign.data(), da, 4 * n);
        sync();
      }
      var_ = var;
      pi_ = pi;
      if (prof_.on) prof_.us[4] += since_us(t0);
    } else if (prof_.on) {
      prof_.us[3] += since_us(t0);
    }
    centers_ = C;
    ncenters_ = kk;
    dims_ = dims;
    dim_keys_ = keys;
    core_ = std::move(pts);
    assign_ = assign;
    ++revision_;
  }

  // models/clustering.py's host loops, for k x dims beyond the kernels' LDS
  void host_lloyd(const std::vector<float>& X, const std::vector<float>& w, size_t n, size_t D, size_t k,
                  std::vector<float>* C, std::vector<int32_t>* assign) {
    for (int it = 0; it < 100; ++it) {
      const auto dd = sqdist(X, n, *C, k, D);
      std::vector<double> ws(k, 0.0), S(k * D, 0.0);
      for (size_t i = 0; i < n; ++i) {
        size_t a = 0;
        for (size_t j = 1; j < k; ++j)
          if (dd[i * k + j] < dd[i * k + a]) a = j;
        (*assign)[i] = (int32_t)a;
        ws[a] += w[i];
        for (size_t t = 0; t < D; ++t) S[a * D + t] += (double)X[i * D + t] * w[i];
      }
      bool done = true;
      for (size_t j = 0; j < k; ++j)
        for (size_t t = 0; t < D; ++t) {
          const float old = (*C)[j * D + t];
          const float nv = ws[j] > 0 ? (float)(S[j * D + t] / std::max(ws[j], 1e-12)) : old;
          if (fabsf(nv - old) > 1e-6f + 1e-5f * fabsf(old)) done = false;
          (*C)[j * D + t] = nv;
        }
      if (done) break;
    }
    const auto dd = sqdist(X, n, *C, k, D);
    for (size_t i = 0; i < n; ++i) {
      size_t a = 0;
      for (size_t j = 1; j < k; ++j)
        if (dd[i * k + j] < dd[i * k + a]) a = j;
      (*assign)[i] = (int32_t)a;
    }
  }

  double log_resp(const float* x, size_t j, size_t D, const std::vector<float>& C, const std::vector<float>& var,
                  const std::vector<float>& pi) const {
    double q2 = 0, ld = 0;
    for (size_t t = 0; t < D; ++t) {
      const double df = (double)x[t] - C[j * D + t];
      q2 += df * df / var[j * D + t];
      ld += log(2 * M_PI * var[j * D + t]);
    }
    return -0.5 * (q2 + ld) + log(std::max(1e-12, (double)pi[j]));
  }

  void host_em(const std::vector<float>& X, const std::vector<float>& w, size_t n, size_t D, size_t k,
               std::vector<float>* C, std::vector<float>* var, std::vector<float>* pi,
               std::vector<int32_t>* assign) {
    std::vector<double> r(k);
    for (int it = 0; it < 50; ++it) {
      std::vector<double> nk(k, 0.0), S1(k * D, 0.0), S2(k * D, 0.0);
      for (size_t i = 0; i < n; ++i) {
        double mx = -INFINITY, z = 0;
        for (size_t j = 0; j < k; ++j) mx = std::max(mx, r[j] = log_resp(&X[i * D], j, D, *C, *var, *pi));
        for (size_t j = 0; j < k; ++j) z += r[j] = exp(r[j] - mx);
        for (size_t j = 0; j < k; ++j) {
          const double q = r[j] / z * w[i];
          nk[j] += q;
          for (size_t t = 0; t < D; ++t) {
            S1[j * D + t] += q * X[i * D + t];
            S2[j * D + t] += q * X[i * D + t] * X[i * D + t];
          }
        }
      }
      double tot = 0;
      for (size_t j = 0; j < k; ++j) tot += nk[j] = std::max(nk[j], 1e-9);
      for (size_t j = 0; j < k; ++j) {
        for (size_t t = 0; t < D; ++t) {
          const double c = S1[j * D + t] / nk[j];
          (*C)[j * D + t] = (float)c;
          (*var)[j * D + t] = (float)std::max(S2[j * D + t] / nk[j] - c * c, 1e-6);
        }
        (*pi)[j] = (float)(nk[j] / tot);
      }
    }
    for (size_t i = 0; i < n; ++i) {
      size_t a = 0;
      double bv = -INFINITY;
      for (size_t j = 0; j < k; ++j) {
        const double v = log_resp(&X[i * D], j, D, *C, *var, *pi);
        if (v > bv) { bv = v; a = j; }
      }
      (*assign)[i] = (int32_t)a;
    }
  }

  // ---------------------------------------------------------- queries
  void check() const {
    if (centers_.empty()) throw std::runtime_error("clustering is not performed yet");
  }

  size_t nearest(const Value& datum) {
    check();
    if (datum.kind != Value::ARR || datum.a.size() < 2) throw std::invalid_argument("datum expected");
    MsgpackWriter body;
    body.arr(1);
    put_value(body, datum);
    PointSet q;
    if (!convert((const uint8_t*)body.out.data(), body.out.size(), false, &q))
      throw std::invalid_argument("malformed datum");
    const auto x = dense(q, dim_keys_);
    const size_t D = dim_keys_.size();
    size_t best = 0;
    if (p_.method == "gmm") {           // argmax log N(x | C_j, var_j) + log pi_j
      double bv = -INFINITY;
      for (size_t j = 0; j < ncenters_; ++j) {
        const double v = log_resp(x.data(), j, D, centers_, var_, pi_);
        if (v > bv) { bv = v; best = j; }
      }
      return best;
    }
    if (D == 0) return 0;
    // one query against k centers is k x D host flops: a device launch (and
    // its two copies) would cost more than the whole RPC. Double precision,
    // as the reference's host distance (the batched paths use the matrix cores).
    double bd = INFINITY;
    for (size_t j = 0; j < ncenters_; ++j) {
      double d = 0.0;
      const float* c = &centers_[j * D];
      for (size_t t = 0; t < D; ++t) {
        const double e = (double)x[t] - (double)c[t];
        d += e * e;
      }
      if (d < bd) { bd = d; best = j; }
    }
    return best;
  }

  void center_datum(size_t j, MsgpackWriter* w) {
    const size_t D = dim_keys_.size();
    size_t nz = 0;
    for (size_t t = 0; t < D; ++t) nz += centers_[j * D + t] != 0.f;
    w->arr(3);
    w->arr(0);
    w->arr(nz);
    for (size_t t = 0; t < D; ++t)
      if (centers_[j * D + t] != 0.f) { w->arr(2); w->raw(dims_[t]); w->dbl((double)centers_[j * D + t]); }
    w->arr(0);
  }

  void k_center(MsgpackWriter* w) {
    check();
    w->arr(ncenters_);
    for (size_t j = 0; j < ncenters_; ++j) center_datum(j, w);
  }

  void members_of(size_t j, MsgpackWriter* w) {
    size_t n = 0;
    for (int32_t a : assign_) n += (size_t)a == j;
    w->arr(n);
    for (size_t i = 0; i < assign_.size(); ++i)
      if ((size_t)assign_[i] == j) {
        w->arr(2);
        w->dbl(core_.w[i]);
        w->out += core_.raw[i];       // the datum as the client sent it
      }
  }

  void core_members(MsgpackWriter* w) {
    check();
    w->arr(ncenters_);
    for (size_t j = 0; j < ncenters_; ++j) members_of(j, w);
  }

  // ---------------------------------------------------------- wire
  void wire(MsgpackWriter& u, const PointSet& ps) {
    u.arr(ps.size());
    for (size_t i = 0; i < ps.size(); ++i) {
      u.arr(3);
      u.dbl(ps.w[i]);
      std::vector<std::pair<std::string, double>> fv;
      for (int64_t s = ps.rp[i]; s < ps.rp[i + 1]; ++s) {
        const std::string& nm = names_[ps.key[(size_t)s]];
        bool found = false;
        for (auto& kv : fv)
          if (kv.first == nm) { kv.second += (double)ps.val[(size_t)s]; found = true; break; }
        if (!found) fv.emplace_back(nm, (double)ps.val[(size_t)s]);
      }
      u.map(fv.size());
      for (const auto& kv : fv) { u.raw(kv.first); u.dbl(kv.second); }
      u.out += ps.raw[i];
    }
  }

  PointSet unwire(const Value& v) {
    if (v.kind != Value::ARR) throw std::runtime_error("broken model data: points");
    PointSet ps;
    for (const Value& p : v.a) {
      if (p.kind != Value::ARR || p.a.size() != 3 || p.a[1].kind != Value::MAP)
        throw std::runtime_error("broken model data: point");
      ps.w.push_back(p.a[0].num());
      for (const auto& kv : p.a[1].o) {
        const int64_t k = (int64_t)jb::hash_to_index(jb::fnv_bytes(jb::kFnvOffset, (const uint8_t*)kv.first.data(),
                                                                   kv.first.size()), kKeySpace);
        if (!names_.count(k)) names_[k] = kv.first;
        ps.key.push_back(k);
        ps.val.push_back((float)kv.second.num());
      }
      ps.rp.push_back((int64_t)ps.key.size());
      MsgpackWriter d;
      put_value(d, p.a[2]);
      ps.raw.push_back(std::move(d.out));
    }
    return ps;
  }

  Params p_;
  jb::PyRandom rng_;
  std::unique_ptr<jb::HostFvWide> hw_;
  DocStats stats_;   // idf / bm25 document statistics (p_.global)
  hipStream_t st_ = nullptr;
  hipStream_t mix_st_ = nullptr;   // the RCCL plane of the MIX
  int device_ = 0;
  std::string token_;              // this member's coresets in a MIX
  std::unordered_map<int64_t, std::string> names_;
  PointSet pending_, others_, core_;
  std::vector<PointSet> buckets_;
  uint64_t revision_ = 0;
  std::vector<float> centers_, var_, pi_;
  size_t ncenters_ = 0;
  std::vector<std::string> dims_;
  std::vector<int64_t> dim_keys_;
  std::vector<int32_t> assign_;
  Conv main_;                       // hw_'s scratch (queries, pushes with statistics)
  std::shared_mutex* mu_ = nullptr;  // the server's model lock (set_lock)
  std::mutex conv_mu_;
  std::vector<std::unique_ptr<Conv>> conv_pool_;
  Dev<float> dX_, dW_, dC_, dXn_, dCn_, dOut_, dScr_, dV_, dP_;
  Dev<double> dU_;
  Dev<int32_t> dI_, dA_;

  // Copies through page-locked staging: from pageable memory the runtime
  // stages each copy through a buffer of its own and waits for it (27 such
  // copies per 1000-point push). Offsets grow until sync(), which waits for
  // the stream, hands the device-to-host results to their vectors and
  // resets the staging.
  PinBuf<uint8_t> pin_;
  size_t pin_off_ = 0;
  struct Pending { void* dst; const uint8_t* src; size_t n; };
  std::vector<Pending> back_;
  uint8_t* stage(size_t n) {
    const size_t a = (pin_off_ + 255) & ~(size_t)255;
    if (pin_.p == nullptr || a + n > pin_.cap) {
      sync();                       // everything staged so far is done with
      pin_.get(std::max<size_t>(2 * pin_.cap, n + 4096));
      pin_off_ = n;
      return pin_.p;
    }
    pin_off_ = a + n;
    return pin_.p + a;
  }
  void h2d(void* dst, const void* src, size_t n) {
    uint8_t* b = stage(n);
    memcpy(b, src, n);
    HIPCHK(hipMemcpyAsync(dst, b, n, hipMemcpyHostToDevice, st_));
  }
  void d2h(void* dst, const void* src, size_t n) {
    uint8_t* b = stage(n);
    HIPCHK(hipMemcpyAsync(b, src, n, hipMemcpyDeviceToHost, st_));
    back_.push_back({dst, b, n});
  }
  void sync() {
    HIPCHK(hipStreamSynchronize(st_));
    for (const Pending& q : back_) memcpy(q.dst, q.src, q.n);
    back_.clear();
    pin_off_ = 0;
  }
};

}  // namespace

int main(int argc, char** argv) {
  set_engine("clustering");
  Args a;
  std::string text;
  const int rc = startup(argc, argv, &a, &text,
                         [](const std::string& t, std::string* why) { return check_config(t, why, nullptr); },
                         /*needs_gpu=*/true, /*native_dist=*/true, /*native_push=*/true);
  if (rc >= 0) return rc;
  try {
    const int device = device_and_signals(a);
    HIPCHK(hipSetDevice(device));
    logf_("INFO", "starting jubaclustering %s RPC server at %s:%d (native, device %d)", kVersion, a.eth.c_str(),
          a.port, device);
    HostServer srv(a, text, [](const std::string& t) -> std::unique_ptr<HostEngine> {
      Params p;
      std::string why;
      if (!check_config(t, &why, &p)) throw std::runtime_error(why);
      return std::unique_ptr<HostEngine>(new Clustering(std::move(p)));
    });
    if (!a.zookeeper.empty())
      srv.join_cluster(std::unique_ptr<jb::mix::ClusterNode>(
          new jb::mix::ClusterNode(a.zookeeper, std::max(1, a.zk_timeout), "clustering", a.name)));
    if (!a.model_file.empty()) srv.load_file(a.model_file);
    return srv.run();
  } catch (const std::exception& e) {
    logf_("FATAL", "failed to start clustering: %s", e.what());
    return 1;
  }
}
