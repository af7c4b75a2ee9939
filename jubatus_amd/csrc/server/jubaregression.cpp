// jubaregression, native: the PA regression server without Python.
//
// Reference: jubatus/server/server/regression_serv.cpp (train :95-130,
// estimate :132-148, clear), regression_impl.cpp (RPC table) over
// jubatus_core's PA regression; the update rule and its oracle are in
// models/regression.py, the kernels in csrc/hip/regression.hip.
//
// Scope: standalone and distributed servers (linear and push mixers over the
// native MIX plane, csrc/native/jb_mix_group.hpp), fixed-slot converters and
// the wide rule set (bigram / combination, idf with MIXed document
// statistics); --cpu and hosts without a GPU go to the Python server (exec
// before any GPU call).
//
// Data path: the batch of queued train RPCs is validated and hashed on the
// host (jb_hostfv.hpp, bit-identical to fv_hash.hip), one request per
// update stream, and trained by ONE jb_regression_train launch (concurrent
// streams when the batch holds several requests, like the Python server's
// train_requests); estimate batches are hashed the same way and scored by
// jb_regression_estimate. Model files are byte-compatible with the Python
// server's (models/regression.py pack()).
#include <signal.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "jb_hostfv.hpp"
#include "jb_linear_conv.hpp"
#include "jb_mix_device.hpp"
#include "jb_msgpack.hpp"
#include "jb_rpc.hpp"
#include "jb_server_common.hpp"
#include "jb_value.hpp"

extern "C" int jb_mix_gather(const float* W, const float* S, int LC, const int64_t* rows, int64_t n,
                             const int32_t* map, int Lc, float* snap, hipStream_t st);
extern "C" int jb_mix_fold(float* W, float* S, int LC, const int64_t* rows, int64_t n, const int32_t* map,
                           int Lc, const float* snap, const float* red, float inv_n, hipStream_t st);

extern "C" int jb_regression_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                   const float* targets, const int64_t* stream_ptr, int nstreams,
                                   float* W, float* stats, float C, float eps, int concurrent,
                                   hipStream_t stream);
extern "C" int jb_regression_estimate(const int64_t* row_ptr, const int32_t* fidx,
                                      const float* fval, int n, const float* W, float* out,
                                      hipStream_t stream);

namespace {

using namespace jb::srv;

struct Config {
  std::string text;
  float eps = 0.1f, C = 3.40282e+38f;
  Rules rules;
  bool wide = false;     // the wide rule set on the host (bigram / combinations)
  WideRules wrules;
};

// models/regression.py PARegression.__init__ + the fixed-slot converter check
bool parse_config(const std::string& text, Config* c, std::string* why) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  if (v.kind != Value::MAP) { *why = "configuration must be a JSON object"; return false; }
  if (v.str_or("method", "") != "PA") { *why = "method " + v.str_or("method", "") + " is not PA"; return false; }
  if (const Value* p = v.get("parameter")) {
    if (const Value* s = p->get("sensitivity")) {
      if (!s->is_num()) { *why = "sensitivity"; return false; }
      c->eps = (float)s->num();
    }
    if (const Value* r = p->get("regularization_weight")) {
      if (!r->is_num()) { *why = "regularization_weight"; return false; }
      c->C = (float)r->num();
    }
  }
  if (c->eps < 0 || !(c->C > 0)) { *why = "sensitivity must be >= 0 and regularization_weight > 0"; return false; }
  const Value* conv = v.get("converter");
  Value empty;
  empty.kind = Value::MAP;
  c->rules.H = device_hash_max_size();   // unless the converter names hash_max_size
  if (!build_linear_rules(conv ? *conv : empty, &c->rules, &c->wide, &c->wrules, why)) return false;
  c->text = text;
  return true;
}

template <class T>
struct HostVec {   // growable host array (realloc keeps the contents)
  T* p = nullptr;
  size_t cap = 0;
  T* get(size_t n) {
    if (n > cap) {
      T* np = (T*)realloc(p, n * sizeof(T));
      if (!np) throw std::bad_alloc();
      p = np;
      cap = n;
    }
    return p;
  }
};

class Regression : public jb::mix::Mixable {
 public:
  std::atomic<uint64_t> update_count{0}, train_calls{0}, train_batches{0};

  Regression(const Config& cfg, int device) : device_(device) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    configure(cfg);
  }

  void configure(const Config& cfg) {
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipStreamSynchronize(stream_));
    ++gen_;
    cfg_ = cfg;
    const Rules& r = cfg.rules;
    conv_.configure(r, cfg.wide, cfg.wrules);
    if (w_) HIPCHK(hipFree(w_));
    if (stats_) HIPCHK(hipFree(stats_));
    HIPCHK(hipMalloc((void**)&w_, r.H * 4));
    HIPCHK(hipMalloc((void**)&stats_, 3 * 4));
    clear_locked();
  }

  const std::string& config_text() const { return cfg_.text; }

  // train bodies (list<scored_datum>): res[k] = samples, or -1 ARGUMENT_ERROR
  void train(const std::vector<std::pair<const uint8_t*, size_t>>& bodies, std::vector<int64_t>* res) {
    const size_t R = bodies.size();
    res->assign(R, -1);
    train_calls += R;
    train_batches += 1;
    update_count += R;
    std::lock_guard<std::mutex> g(mu_);
    int64_t n = 0, slots = 0;
    std::vector<int64_t> sp(1, 0);
    row_.get(1024)[0] = 0;
    for (size_t k = 0; k < R; ++k) {
      const int64_t n0 = n, s0 = slots;
      if (parse_scored(bodies[k].first, bodies[k].second, &n, &slots)) {
        (*res)[k] = n - n0;
        if (n > n0) sp.push_back(n);
      } else {
        n = n0;
        slots = s0;
      }
    }
    const int ns = (int)sp.size() - 1;
    if (n == 0 || ns == 0) return;
    upload(n, slots);
    HIPCHK(hipMemcpyAsync(d_tgt_.get(n), tgt_.p, 4 * (size_t)n, hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_sp_.get(sp.size()), sp.data(), 8 * sp.size(), hipMemcpyHostToDevice, stream_));
    const int rc = jb_regression_train(d_row_.p, d_idx_.p, d_val_.p, d_tgt_.p, d_sp_.p, ns, w_, stats_,
                                       cfg_.C, cfg_.eps, ns > 1 ? 1 : 0, stream_);
    if (rc != 0) throw std::runtime_error("jb_regression_train failed: " + std::to_string(rc));
    HIPCHK(hipStreamSynchronize(stream_));
    samples_ += (uint64_t)n;
  }

  // estimate bodies (list<datum>): per body the estimates, ok[k] false on a malformed body
  std::vector<std::vector<float>> estimate(const std::vector<std::pair<const uint8_t*, size_t>>& bodies,
                                           std::vector<bool>* ok) {
    const size_t R = bodies.size();
    ok->assign(R, true);
    std::vector<int64_t> first(R + 1, 0);
    std::lock_guard<std::mutex> g(mu_);
    int64_t n = 0, slots = 0;
    idx_.get(std::max<size_t>(idx_.cap, 1024));
    val_.get(idx_.cap);
    row_.get(std::max<size_t>(row_.cap, 1024));
    row_.p[0] = 0;
    for (size_t k = 0; k < R; ++k) {
      first[k] = n;
      const int64_t n0 = n, s0 = slots;
      while (true) {
        int rc = conv_.hash_body(bodies[k].first, bodies[k].second, idx_.p, val_.p, row_.p,
                                    (int64_t)row_.cap - 1, (int64_t)idx_.cap, &n, &slots);
        if (rc == 2) {
          n = n0;
          slots = s0;
          idx_.get(2 * idx_.cap);
          val_.get(idx_.cap);
          row_.get(2 * row_.cap);
          continue;
        }
        if (rc == 1) { (*ok)[k] = false; n = n0; slots = s0; }
        break;
      }
    }
    first[R] = n;
    std::vector<float> out(n);
    if (n > 0) {
      upload(n, slots);
      const int rc = jb_regression_estimate(d_row_.p, d_idx_.p, d_val_.p, (int)n, w_, d_out_.get(n), stream_);
      if (rc != 0) throw std::runtime_error("jb_regression_estimate failed: " + std::to_string(rc));
      HIPCHK(hipMemcpyAsync(out.data(), d_out_.p, 4 * (size_t)n, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
    }
    std::vector<std::vector<float>> res(R);
    for (size_t k = 0; k < R; ++k) res[k].assign(out.begin() + first[k], out.begin() + first[k + 1]);
    return res;
  }

  void clear() {
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    ++gen_;
    clear_locked();
  }

  // ------------------------------------------------------------ MIX
  // distributed mode: the linear mixer (jb_mix_group.hpp) runs mix() /
  // hand_over() on its thread. The model is small and dense (w[H] + the 3
  // target statistics), so a MIX is the mean of the whole table, as the
  // Python twin's (models/regression.py mix: all-reduce mean of w and stats;
  // reference: regression's linear mixable, get_diff / put_diff of w).
  // Training goes on during the collective: the table is snapshotted behind
  // the queued training, the snapshot is SUM-reduced, and the fold adds
  // mean - snapshot, so updates made meanwhile are kept.
  void enable_mix() {
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipStreamCreateWithFlags(&mixs_, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&mix_ev_, hipEventDisableTiming));
    const int32_t zero = 0;
    HIPCHK(hipMemcpy(map_.get(1), &zero, 4, hipMemcpyHostToDevice));
    mixing_ = true;
  }
  bool distributed() const { return mixing_; }

  std::unique_ptr<jb::mix::Plane> make_plane(jb::mix::Star& star, double dl) {
    return jb::mix::make_device_plane(star, device_, mixs_, dl);
  }

  uint64_t mix(jb::mix::Group& grp) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    uint64_t gen, H;
    {
      std::lock_guard<std::mutex> g(mu_);
      gen = gen_;
      H = cfg_.rules.H;
      // snapshot (behind the queued training): [w | stats] -> snap, red
      if (jb_mix_gather(w_, nullptr, 1, nullptr, (int64_t)H, map_.p, 1, snap_.get(H + 3), stream_) != 0)
        throw std::runtime_error("jb_mix_gather failed");
      HIPCHK(hipMemcpyAsync(snap_.p + H, stats_, 12, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(red_.get(H + 3), snap_.p, (H + 3) * 4, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipEventRecord(mix_ev_, stream_));
      HIPCHK(hipStreamWaitEvent(mixs_, mix_ev_, 0));
    }
    // every member checks the layout (a different table height cannot mix),
    // and a member whose tables were replaced since its snapshot makes the
    // whole group skip the fold (slot 2: max of "replaced")
    int64_t hh[3] = {(int64_t)H, -(int64_t)H, 0};
    {
      std::lock_guard<std::mutex> g(mu_);
      hh[2] = gen != gen_ ? 1 : 0;
    }
    star.allreduce_max(hh, 3, grp.deadline());
    if (hh[0] != -hh[1]) throw std::runtime_error("mix: members disagree on hash_max_size");
    uint64_t wbytes = 0;
    if (conv_.global()) {   // the document statistics of idf / bm25 converters
      std::string dm;
      {
        std::lock_guard<std::mutex> g(mu_);
        dm = conv_.get_diff();
      }
      const auto parts = pl.allgather_bytes(star, dm, grp.deadline());
      std::lock_guard<std::mutex> g(mu_);
      conv_.put_diffs(parts);
      wbytes = dm.size();
    }
    if (hh[2] != 0) {
      last_applied_ = false;
      return 24 + wbytes;
    }
    pl.allreduce_sum(red_.p, H + 3, grp.deadline());
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipEventRecord(mix_ev_, mixs_));
    HIPCHK(hipStreamWaitEvent(stream_, mix_ev_, 0));
    if (gen != gen_) {          // cleared / reconfigured / loaded meanwhile: nothing to fold into
      last_applied_ = false;
      return (H + 3) * 4;
    }
    const float inv = 1.f / (float)grp.world();
    if (jb_mix_fold(w_, nullptr, 1, nullptr, (int64_t)H, map_.p, 1, snap_.p, red_.p, inv, stream_) != 0)
      throw std::runtime_error("jb_mix_fold failed");
    float sn[3], rd[3], cur[3];
    HIPCHK(hipMemcpyAsync(sn, snap_.p + H, 12, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipMemcpyAsync(rd, red_.p + H, 12, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipMemcpyAsync(cur, stats_, 12, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    for (int i = 0; i < 3; ++i) cur[i] += rd[i] * inv - sn[i];
    HIPCHK(hipMemcpy(stats_, cur, 12, hipMemcpyHostToDevice));
    last_applied_ = true;
    ++mixes_;
    return (H + 3) * 4;
  }

  // push mixers (random / broadcast / skip, push_mixer.cpp:335-408): one
  // round = the pairwise mean of [w | stats] with the peer (point-to-point),
  // folded like mix() so training meanwhile is kept. Python twin:
  // models/regression.py through parallel/mixable.py pair_exchange.
  bool push_mixable() const override { return true; }
  void push_end() override {
    std::lock_guard<std::mutex> g(mu_);
    conv_.clear_diff();              // the own statistics went to every partner of this MIX
  }
  uint64_t pair_mix(jb::mix::Group& grp, int peer) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    const double dl = grp.deadline();
    uint64_t gen = 0, H = 0;
    if (peer >= 0) {
      std::lock_guard<std::mutex> g(mu_);
      gen = gen_;
      H = cfg_.rules.H;
      if (jb_mix_gather(w_, nullptr, 1, nullptr, (int64_t)H, map_.p, 1, snap_.get(H + 3), stream_) != 0)
        throw std::runtime_error("jb_mix_gather failed");
      HIPCHK(hipMemcpyAsync(snap_.p + H, stats_, 12, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(red_.get(H + 3), snap_.p, (H + 3) * 4, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipEventRecord(mix_ev_, stream_));
      HIPCHK(hipStreamWaitEvent(mixs_, mix_ev_, 0));
    }
    // the pair checks the layout and whether both can fold; every call below
    // is one of the round's collectives (a rank without a peer sends nothing)
    std::string me;
    if (peer >= 0) me = std::to_string(H) + (gen != gen_ ? " 1" : " 0");
    const std::string th = pl.exchange_bytes(star, peer, me, dl);
    bool fold = peer >= 0 && gen == gen_;
    if (peer >= 0) {
      if (th.substr(0, th.find(' ')) != std::to_string(H))
        throw std::runtime_error("mix: members disagree on hash_max_size");
      fold = fold && th.size() > 2 && th.back() == '0';
    }
    uint64_t wbytes = 0;
    if (conv_.global()) {
      std::string dm;
      if (peer >= 0) {
        std::lock_guard<std::mutex> g(mu_);
        dm = conv_.get_diff();
      }
      const std::string td = pl.exchange_bytes(star, peer, dm, dl);
      if (peer >= 0) {
        std::lock_guard<std::mutex> g(mu_);
        conv_.put_diffs(grp.rank() < peer ? std::vector<std::string>{dm, td} : std::vector<std::string>{td, dm},
                      true);
        wbytes = dm.size();
      }
    }
    pl.pair_sum(star, fold ? red_.p : nullptr, fold ? H + 3 : 0, fold ? peer : -1, dl);
    if (!fold) {
      if (peer >= 0) last_applied_ = false;
      return wbytes;
    }
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipEventRecord(mix_ev_, mixs_));
    HIPCHK(hipStreamWaitEvent(stream_, mix_ev_, 0));
    if (gen != gen_) {
      last_applied_ = false;
      return (H + 3) * 4 + wbytes;
    }
    if (jb_mix_fold(w_, nullptr, 1, nullptr, (int64_t)H, map_.p, 1, snap_.p, red_.p, 0.5f, stream_) != 0)
      throw std::runtime_error("jb_mix_fold failed");
    float sn[3], rd[3], cur[3];
    HIPCHK(hipMemcpyAsync(sn, snap_.p + H, 12, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipMemcpyAsync(rd, red_.p + H, 12, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipMemcpyAsync(cur, stats_, 12, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    for (int i = 0; i < 3; ++i) cur[i] += rd[i] * 0.5f - sn[i];
    HIPCHK(hipMemcpy(stats_, cur, 12, hipMemcpyHostToDevice));
    last_applied_ = true;
    ++mixes_;
    return (H + 3) * 4 + wbytes;
  }

  // obsolete protocol: rank src sends w and stats; apply = take them
  void hand_over(jb::mix::Group& grp, int src, bool apply) override {
    jb::mix::Plane& pl = grp.plane();
    uint64_t H;
    {
      std::lock_guard<std::mutex> g(mu_);
      H = cfg_.rules.H;
      if (grp.rank() == src) {
        HIPCHK(hipMemcpyAsync(red_.get(H + 3), w_, H * 4, hipMemcpyDeviceToDevice, stream_));
        HIPCHK(hipMemcpyAsync(red_.p + H, stats_, 12, hipMemcpyDeviceToDevice, stream_));
      } else {
        red_.get(H + 3);
      }
      HIPCHK(hipStreamSynchronize(stream_));
    }
    int64_t hh[2] = {(int64_t)H, -(int64_t)H};
    grp.star().allreduce_max(hh, 2, grp.deadline());
    if (hh[0] != -hh[1]) throw std::runtime_error("hand-over: members disagree on hash_max_size");
    pl.bcast(red_.p, (H + 3) * 4, src, grp.deadline());
    if (!apply || grp.rank() == src) return;
    std::lock_guard<std::mutex> g(mu_);
    ++gen_;
    HIPCHK(hipMemcpyAsync(w_, red_.p, H * 4, hipMemcpyDeviceToDevice, stream_));
    HIPCHK(hipMemcpyAsync(stats_, red_.p + H, 12, hipMemcpyDeviceToDevice, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
  }

  // models/regression.py pack(): the nonzero rows of w, the target statistics
  std::string pack_user_data() {
    std::lock_guard<std::mutex> g(mu_);
    const uint64_t H = cfg_.rules.H;
    std::vector<float> w(H);
    float st[3];
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(w.data(), w_, H * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(st, stats_, sizeof st, hipMemcpyDeviceToHost));
    std::vector<int64_t> rows;
    std::vector<float> vals;
    for (uint64_t h = 0; h < H; ++h)
      if (w[h] != 0.f) { rows.push_back((int64_t)h); vals.push_back(w[h]); }
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(6);
    u.str("method"); u.str("PA");
    u.str("H"); u.uint(H);
    u.str("rows"); u.bin(rows.data(), rows.size() * 8);
    u.str("w"); u.bin(vals.data(), vals.size() * 4);
    u.str("stats"); u.arr(3);
    for (float x : st) u.dbl((double)x);
    u.str("weights");
    conv_.pack(u);
    return std::move(u.out);
  }

  void unpack(const Value& obj) {
    const Value* H = obj.get("H");
    const Value* rv = obj.get("rows");
    const Value* wv = obj.get("w");
    const Value* sv = obj.get("stats");
    if (!H || !H->is_num() || (uint64_t)H->num() != cfg_.rules.H)
      throw std::runtime_error("model hash_max_size differs from the configuration");
    if (!rv || !wv || rv->s.size() / 8 != wv->s.size() / 4 || !sv || sv->kind != Value::ARR || sv->a.size() != 3)
      throw std::runtime_error("broken model data: regression tables");
    std::lock_guard<std::mutex> g(mu_);
    ++gen_;
    const uint64_t Hn = cfg_.rules.H;
    std::vector<float> w(Hn, 0.f);
    const int64_t* rows = (const int64_t*)rv->s.data();
    const float* vals = (const float*)wv->s.data();
    for (size_t k = 0; k < rv->s.size() / 8; ++k) {
      if (rows[k] < 0 || (uint64_t)rows[k] >= Hn) throw std::runtime_error("broken model data: row index");
      w[rows[k]] = vals[k];
    }
    float st[3] = {(float)sv->a[0].num(), (float)sv->a[1].num(), (float)sv->a[2].num()};
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(w_, w.data(), Hn * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(stats_, st, sizeof st, hipMemcpyHostToDevice));
    conv_.unpack(obj.get("weights"));
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) {
    auto add = [&](const char* k, const std::string& v) { st->emplace_back(k, v); };
    add("num_features", std::to_string(cfg_.rules.H));
    add("method", "PA");
    add("storage", "hbm");
    add("fv_path", "gpu");
    add("server_runtime", "native");
    add("batching.train.calls", std::to_string(train_calls.load()));
    add("batching.train.launches", std::to_string(train_batches.load()));
    add("train.samples_trained", std::to_string(samples_));
    add("device", "cuda:" + std::to_string(device_));
    if (mixing_) {
      add("mix.mode", "dense");
      add("mix.last_applied", last_applied_ ? "1" : "0");
      add("mix.applied_count", std::to_string(mixes_));
    }
  }

 private:
  void clear_locked() {
    conv_.clear();
    HIPCHK(hipMemsetAsync(w_, 0, cfg_.rules.H * 4, stream_));
    HIPCHK(hipMemsetAsync(stats_, 0, 3 * 4, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
  }

  // one list<[score, datum]> body appended to the host CSR (validated as a
  // whole: false leaves nothing behind)
  // (the wide converter's document statistics of a body that fails are undone)
  bool parse_scored(const uint8_t* b, size_t len, int64_t* n, int64_t* slots) {
    conv_.begin();
    const int64_t n0 = *n, s0 = *slots;
    for (;;) {
      const int rc = parse_scored_once(b, len, n, slots);
      if (rc == 0) return true;
      conv_.rollback();
      *n = n0;
      *slots = s0;
      if (rc != 2) return false;
      const size_t cap = std::max<size_t>(idx_.cap, 256);   // out of slots: grow, hash the body again
      idx_.get(2 * cap);
      val_.get(2 * cap);
      conv_.begin();
    }
  }
  // -> 0 ok, 1 malformed, 2 out of slots
  int parse_scored_once(const uint8_t* b, size_t len, int64_t* n, int64_t* slots) {
    jb::Cursor c{b, b + len};
    uint32_t cnt;
    if (!c.array(&cnt) || cnt > len) return 1;
    row_.get((size_t)*n + cnt + 1);
    tgt_.get((size_t)*n + cnt + 1);
    for (uint32_t k = 0; k < cnt; ++k) {
      uint32_t two;
      double y;
      if (!c.array(&two) || two != 2) return 1;
      if (c.p < c.end && (*c.p == 0xc2 || *c.p == 0xc3)) return 1;   // bool is not a score
      if (!c.number(&y)) return 1;
      const int64_t cap = (int64_t)std::max<size_t>(idx_.cap, 256);
      idx_.get(cap);
      val_.get(cap);
      const int rc = conv_.hash_datum(c, idx_.p, val_.p, cap, slots, true);
      if (rc != 0) return rc;
      tgt_.p[*n] = (float)y;
      row_.p[++*n] = *slots;
    }
    return c.p == c.end ? 0 : 1;
  }

  void upload(int64_t n, int64_t slots) {
    const int64_t nnz = std::max<int64_t>(slots, 1);
    HIPCHK(hipMemcpyAsync(d_row_.get(n + 1), row_.p, 8 * ((size_t)n + 1), hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_idx_.get(nnz), idx_.p, 4 * (size_t)slots, hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_val_.get(nnz), val_.p, 4 * (size_t)slots, hipMemcpyHostToDevice, stream_));
  }

  std::mutex mu_;
  Config cfg_;
  int device_;
  hipStream_t stream_;
  // MIX state: table generation (bumped when the tables are replaced), the
  // mixer's stream / event, snapshot and reduction buffers [w | stats]
  uint64_t gen_ = 0, mixes_ = 0;
  bool mixing_ = false, last_applied_ = false;
  hipStream_t mixs_ = nullptr;
  hipEvent_t mix_ev_ = nullptr;
  DevBuf<float> snap_, red_;
  DevBuf<int32_t> map_;
  float* w_ = nullptr;
  float* stats_ = nullptr;
  uint64_t samples_ = 0;
  LinearConv conv_;
  HostVec<int32_t> idx_;
  HostVec<float> val_, tgt_;
  HostVec<int64_t> row_;
  DevBuf<int64_t> d_row_, d_sp_;
  DevBuf<int32_t> d_idx_;
  DevBuf<float> d_val_, d_tgt_, d_out_;
};

class Server {
 public:
  Server(const Args& a, const Config& cfg, int device) : a_(a) { reg_.reset(new Regression(cfg, device)); }

  void load_file(const std::string& path) { load_impl(path, true); }

  int run() {
    rpc_.reset(new jb::RpcServer([this](const jb::RpcRequest& r) { return dispatch(r); }, a_.threads, 0.0));
    rpc_->set_io_threads(std::max(1, a_.threads / 4));
    rpc_->set_batch({"estimate", "train"},
                    [this](const std::string& m, std::vector<jb::RpcRequest>& reqs) { return batch(m, reqs); },
                    4096);
    int port;
    try {
      port = rpc_->listen(a_.bind, a_.port);
    } catch (const std::exception& e) {
      logf_("FATAL", "server failed to start: any process using port %d? (%s)", a_.port, e.what());
      return 1;
    }
    a_.port = port;
    logf_("INFO", "start listening at port %d", port);
    cs_.start_time = time(nullptr);
    rpc_->start();
    if (node_) {   // distributed mode: register, then the mixer thread
      node_->register_actor(a_.eth, a_.port);
      jb::mix::MixerArgs ma;
      ma.type = "regression";
      ma.name = a_.name;
      ma.eth = a_.eth;
      ma.port = a_.port;
      ma.interval_sec = a_.interval_sec;
      ma.interval_count = a_.interval_count;
      ma.interconnect_timeout = a_.ic_timeout;
      Regression* r = reg_.get();
      mixer_.reset(new jb::mix::LinearMixer(node_->coord(), ma, r, [r](jb::mix::Group& g, double dl) {
        return r->make_plane(g.star(), dl);
      }));
      mixer_->start();
      logf_("INFO", "registered group membership as %s (native linear_mixer)", ident().c_str());
    }
    logf_("INFO", "jubaregression RPC server startup (native)");
    wait_for_term();
    if (mixer_) {
      logf_("INFO", "stopping mixer thread");
      mixer_->stop();
    }
    if (node_) node_->leave();
    logf_("INFO", "stopping RPC server");
    rpc_->stop();
    return 0;
  }

  // distributed mode (-z): coordinator session, config lock, MIX state
  void join_cluster(std::unique_ptr<jb::mix::ClusterNode> node) {
    node_ = std::move(node);
    a_.connected_zookeeper = node_->connected();
    if (!node_->config_rlock()) throw std::runtime_error("failed to get config lock");
    reg_->enable_mix();
  }

 private:
  std::string ident() const { return a_.eth + "_" + std::to_string(a_.port); }

  static bool name_and_body(const std::string& params, const uint8_t** b, size_t* n) {
    jb::Cursor c{(const uint8_t*)params.data(), (const uint8_t*)params.data() + params.size()};
    uint32_t two;
    const uint8_t* s;
    uint32_t sn;
    if (!c.array(&two) || two != 2 || !c.raw(&s, &sn)) return false;
    *b = c.p;
    *n = (size_t)(c.end - c.p);
    return true;
  }

  std::vector<std::string> batch(const std::string& method, std::vector<jb::RpcRequest>& reqs) {
    std::vector<std::string> out(reqs.size());
    std::vector<std::pair<const uint8_t*, size_t>> bodies;
    std::vector<size_t> where;
    for (size_t k = 0; k < reqs.size(); ++k) {
      const uint8_t* b;
      size_t n;
      if (!name_and_body(reqs[k].params, &b, &n)) {
        out[k] = jb::val::response_code(reqs[k].msgid, kArgumentError);
        continue;
      }
      bodies.emplace_back(b, n);
      where.push_back(k);
    }
    try {
      if (method == "train") {
        if (mixer_) mixer_->updated(bodies.size());
        std::vector<int64_t> res;
        reg_->train(bodies, &res);
        for (size_t j = 0; j < where.size(); ++j) {
          const uint32_t id = reqs[where[j]].msgid;
          if (res[j] < 0) {
            out[where[j]] = jb::val::response_code(id, kArgumentError);
          } else {
            MsgpackWriter w;
            w.uint((uint64_t)res[j]);
            out[where[j]] = jb::val::response_ok(id, w.out);
          }
        }
      } else {
        std::vector<bool> ok;
        auto res = reg_->estimate(bodies, &ok);
        for (size_t j = 0; j < where.size(); ++j) {
          const uint32_t id = reqs[where[j]].msgid;
          if (!ok[j]) {
            out[where[j]] = jb::val::response_code(id, kArgumentError);
            continue;
          }
          MsgpackWriter w;
          w.arr(res[j].size());
          for (float x : res[j]) w.dbl((double)x);
          out[where[j]] = jb::val::response_ok(id, w.out);
        }
      }
    } catch (const std::exception& e) {
      for (size_t j = 0; j < where.size(); ++j)
        out[where[j]] = jb::val::response_msg(reqs[where[j]].msgid, e.what());
    }
    for (size_t k = 0; k < reqs.size(); ++k)
      if (reqs[k].notify) out[k].clear();
    return out;
  }

  std::string dispatch(const jb::RpcRequest& r) {
    Value args;
    try {
      args = MsgpackReader((const uint8_t*)r.params.data(), r.params.size()).read();
    } catch (const std::exception&) {
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    }
    if (args.kind != Value::ARR) return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    const std::string& m = r.method;
    static const std::vector<std::pair<std::string, size_t>> arity = {
        {"get_config", 1}, {"save", 2}, {"load", 2}, {"get_status", 1}, {"clear", 1},
        {"train", 2}, {"estimate", 2}};
    size_t want = 0;
    for (const auto& x : arity)
      if (x.first == m) want = x.second;
    if (m == "do_mix" && mixer_) want = 1;
    if (want == 0) return r.notify ? std::string() : jb::val::response_code(r.msgid, kNoMethodError);
    if (args.a.size() != want || ((m == "save" || m == "load") && !args.a[1].is_str()))
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    MsgpackWriter w;
    try {
      if (m == "get_config") {
        w.raw(reg_->config_text());
      } else if (m == "clear") {
        reg_->clear();
        w.boolean(true);
      } else if (m == "save") {
        const std::string& id = args.a[1].s;
        if (id.empty()) throw std::runtime_error("empty id is not allowed");
        const std::string path = local_path(id);
        write_model_file(path, "regression", id, reg_->config_text(), reg_->pack_user_data());
        {
          std::lock_guard<std::mutex> g(st_mu_);
          cs_.last_saved = time(nullptr);
          cs_.last_saved_path = path;
        }
        logf_("INFO", "saved to %s", path.c_str());
        w.map(1);
        w.raw(ident());
        w.raw(path);
      } else if (m == "load") {
        if (args.a[1].s.empty()) throw std::runtime_error("empty id is not allowed");
        load_impl(local_path(args.a[1].s), false);
        w.boolean(true);
      } else if (m == "get_status") {
        std::vector<std::pair<std::string, std::string>> st;
        {
          std::lock_guard<std::mutex> g(st_mu_);
          common_status(a_, cs_, reg_->update_count.load(), &st);
        }
        reg_->status(&st);
        if (mixer_) mixer_->status(&st);
        w.map(1);
        w.raw(ident());
        w.map(st.size());
        for (auto& kv : st) { w.raw(kv.first); w.raw(kv.second); }
      } else if (m == "do_mix") {
        w.boolean(mixer_->do_mix());
      } else {   // train / estimate outside the batch path (not reached: batched methods)
        std::vector<jb::RpcRequest> one{r};
        return batch(m, one)[0];
      }
    } catch (const std::exception& e) {
      return r.notify ? std::string() : jb::val::response_msg(r.msgid, e.what());
    }
    return r.notify ? std::string() : jb::val::response_ok(r.msgid, w.out);
  }

  std::string local_path(const std::string& id) const {
    return a_.datadir + "/" + a_.eth + "_" + std::to_string(a_.port) + "_regression_" + id + ".jubatus";
  }

  void load_impl(const std::string& path, bool overwrite_config) {
    std::string bytes;
    if (!read_file(path, &bytes)) throw std::runtime_error("cannot open input file: " + path + ": " + strerror(errno));
    ModelFile mf;
    const std::string err = read_model_file(bytes, &mf);
    if (!err.empty()) throw std::runtime_error(err);
    if (mf.type != "regression")
      throw std::runtime_error("invalid model type: saved type: " + mf.type + ", expected type: regression");
    const std::string current = reg_->config_text();
    if (!overwrite_config && !jb::val::same_config(mf.config, current))
      throw std::runtime_error("model config mismatched with the running config");
    if (mf.user_version != 1)
      throw std::runtime_error("user data version mismatched: " + std::to_string(mf.user_version) +
                               ", current version: 1");
    if (overwrite_config && !jb::val::same_config(mf.config, current)) {
      Config cfg;
      std::string why;
      if (!parse_config(mf.config, &cfg, &why)) throw std::runtime_error("model config is not served natively: " + why);
      reg_->configure(cfg);
    }
    reg_->unpack(mf.user);
    std::lock_guard<std::mutex> g(st_mu_);
    cs_.last_loaded = time(nullptr);
    cs_.last_loaded_path = path;
    logf_("INFO", "loaded from %s", path.c_str());
  }

  Args a_;
  std::unique_ptr<Regression> reg_;
  std::unique_ptr<jb::mix::ClusterNode> node_;
  std::unique_ptr<jb::mix::LinearMixer> mixer_;
  std::unique_ptr<jb::RpcServer> rpc_;
  std::mutex st_mu_;
  CommonStatus cs_;
};

}  // namespace

int main(int argc, char** argv) {
  set_engine("regression");
  Args a;
  std::string text;
  Config cfg;
  const int rc = startup(argc, argv, &a, &text, [&cfg](const std::string& t, std::string* why) {
    return parse_config(t, &cfg, why);
  }, true, /*native_dist=*/true, /*native_push=*/true);
  if (rc >= 0) return rc;
  // below this line the process owns the GPU: no exec
  try {
    const int device = device_and_signals(a);
    logf_("INFO", "starting jubaregression %s RPC server at %s:%d (native, device %d)", kVersion,
          a.eth.c_str(), a.port, device);
    Server srv(a, cfg, device);
    if (!a.zookeeper.empty()) {
      srv.join_cluster(std::unique_ptr<jb::mix::ClusterNode>(
          new jb::mix::ClusterNode(a.zookeeper, std::max(1, a.zk_timeout), "regression", a.name)));
    } else if (!a.model_file.empty()) {
      srv.load_file(a.model_file);
    }
    return srv.run();
  } catch (const std::exception& e) {
    logf_("FATAL", "failed to start regression: %s", e.what());
    return 1;
  }
}
