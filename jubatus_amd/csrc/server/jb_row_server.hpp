// The RPC server of the native row engines: jubarecommender,
// jubanearest_neighbor and jubaanomaly (one binary each, csrc/server/
// juba{recommender,nearest_neighbor,anomaly}.cpp), and jubaclassifier's
// nearest-neighbor methods (NN over lsh / euclid_lsh / minhash, cosine,
// euclidean: models/nn_classifier.py), no Python in the process.
//
// Reference: jubatus/server/server/recommender_serv.cpp:126-224,
// recommender_impl.cpp (RPC table), nearest_neighbor_serv.cpp:121-178,
// nearest_neighbor_impl.cpp, anomaly_serv.cpp:149-320 (standalone add with
// the id counter, update / overwrite, calc_score, the id reset on load);
// the Python twins are server/{recommender,nearest_neighbor,anomaly}_serv.py
// over models/recommender.py and models/anomaly.py.
//
// Scope: servers whose converter runs on the native hashers
// (jb_row_engine.hpp Converter), standalone or distributed with the linear
// mixer: the row diffs of a MIX move as one byte buffer per rank over the
// group's plane (RCCL all-gather over xGMI between GPUs, the control plane
// when members share a device), newest version wins (parallel/row_mix.py's
// protocol); CHT registration, and anomaly's add over the coordinator's id
// generator + CHT owners with server-to-server update (anomaly_serv.cpp:
// 178-211,275-297), push mixers (pairwise row diffs). Other configurations,
// --cpu and hosts without a GPU go to the Python server (exec before any GPU
// call).
//
// Concurrency (the reference: nearest_neighbor analysis lock-free,
// ChangeLog.rst:102, nearest_neighbor_serv.cpp:138-172 NOLOCK; recommender
// analysis read-locked, recommender_serv.cpp:170-224 JRLOCK): updates take
// the model lock exclusively; analysis takes it shared. Every query that
// needs the device (similar_row_* / neighbor_row_* / calc_score) is handed
// to ONE batcher thread, which takes all the queries the RPC threads have
// queued, hashes them and scores up to 8 at one k in a single pass over the
// index (LSH signatures: lsh.hip + topk.hip; inverted index: sparse_pool.hip
// pool_rows_kernel), so concurrent clients share the table scan.
#pragma once
#include <time.h>

#include <math.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <random>
#include <set>
#include <deque>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "jb_lof_state.hpp"
#include "jb_roctx.hpp"
#include "jb_mix_device.hpp"
#include "jb_mix_group.hpp"
#include "jb_msgpack.hpp"
#include "jb_row_engine.hpp"
#include "jb_rpc.hpp"
#include "jb_server_common.hpp"
#include "jb_value.hpp"

namespace jb {
namespace rowsrv {

using namespace jb::srv;
using jb::row::ArgError;
using jb::row::Datum;
using jb::row::Hit;
using jb::row::RowEngine;

constexpr int kCompleteK = 10;   // models/recommender.py COMPLETE_K

enum class Kind { kRecommender, kNearestNeighbor, kAnomaly, kClassifier };

inline const char* kind_name(Kind k) {
  return k == Kind::kRecommender ? "recommender"
         : k == Kind::kNearestNeighbor ? "nearest_neighbor"
         : k == Kind::kAnomaly ? "anomaly" : "classifier";
}

struct Config {
  std::string text;
  std::string outer;     // config "method" (status)
  std::string inner;     // the similarity method of the index
  Value param;           // parameters of the index (hash_num, seed, unlearner...)
  Value conv;
  // anomaly (models/anomaly.py LOF)
  int k = 10, rnn = 30;
  bool ignore_kth_same = false;
  // classifier (models/nn_classifier.py): k nearest rows, label score
  // sum exp(-alpha d) (NN, euclidean) or summed similarity (cosine)
  int nn_k = 128;
  double alpha = 1.0;
  bool similar = false;
};

inline bool is_nn_classifier(const std::string& m) {
  return m == "NN" || m == "nearest_neighbor" || m == "cosine" || m == "euclidean";
}

inline bool is_lsh(const std::string& m) { return m == "lsh" || m == "euclid_lsh" || m == "minhash"; }

// models/recommender.py Recommender / NearestNeighbor __init__ + the
// converter check
inline bool parse_config(Kind kind, const std::string& text, Config* c, std::string* why) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  if (v.kind != Value::MAP) { *why = "configuration must be a JSON object"; return false; }
  c->outer = v.str_or("method", "");
  const Value* p = v.get("parameter");
  Value empty;
  empty.kind = Value::MAP;
  c->param = p && p->kind == Value::MAP ? *p : empty;
  c->inner = c->outer;
  if (kind == Kind::kNearestNeighbor) {
    if (!is_lsh(c->outer)) { *why = "nearest_neighbor method " + c->outer; return false; }
  } else if (kind == Kind::kClassifier) {
    if (!is_nn_classifier(c->outer)) {
      *why = "classifier method " + c->outer + " is not a nearest-neighbor one";
      return false;
    }
    auto num = [&](const char* key, double d) {
      const Value* x = c->param.get(key);
      return x && x->is_num() ? x->num() : d;
    };
    c->nn_k = (int)num("nearest_neighbor_num", 128);
    c->alpha = num("local_sensitivity", 1.0);
    if (c->nn_k <= 0 || c->alpha < 0) {
      *why = "nearest_neighbor_num must be positive, local_sensitivity >= 0";
      return false;
    }
    Value inner = empty;
    if (c->outer == "cosine") {
      c->inner = "inverted_index";
      c->similar = true;
    } else if (c->outer == "euclidean") {
      c->inner = "inverted_index_euclid";
    } else {
      c->inner = c->param.str_or("method", "lsh");
      if (!is_lsh(c->inner)) { *why = "unknown nearest neighbor method: " + c->inner; return false; }
      if (const Value* ip = c->param.get("parameter"))
        if (ip->kind == Value::MAP) inner = *ip;
    }
    for (const char* key : {"unlearner", "unlearner_parameter"})
      if (const Value* x = c->param.get(key)) inner.o.emplace_back(key, *x);
    c->param = inner;
  } else if (kind == Kind::kAnomaly) {
    // lof: any recommender backend; light_lof: the nearest_neighbor (LSH) ones
    if (c->outer != "lof" && c->outer != "light_lof") { *why = "anomaly method " + c->outer; return false; }
    c->inner = c->param.str_or("method", "");
    const bool ok = is_lsh(c->inner) ||
                    (c->outer == "lof" && (c->inner == "inverted_index" || c->inner == "inverted_index_euclid"));
    if (!ok) { *why = c->outer + ": parameter.method " + c->inner; return false; }
    auto num = [&](const char* key, double d) {
      const Value* x = c->param.get(key);
      return x && x->is_num() ? x->num() : d;
    };
    c->k = (int)num("nearest_neighbor_num", 10);
    c->rnn = (int)num("reverse_nearest_neighbor_num", 30);
    if (c->k <= 0 || c->rnn < c->k) { *why = "nearest_neighbor_num / reverse_nearest_neighbor_num"; return false; }
    if (c->k > jb::row::kLofMaxK) {
      *why = "nearest_neighbor_num beyond the device limit";
      return false;
    }
    if (const Value* b = c->param.get("ignore_kth_same_point"))
      c->ignore_kth_same = b->kind == Value::BOOL ? b->b : b->num() != 0;
    Value inner = empty;
    if (const Value* ip = c->param.get("parameter"))
      if (ip->kind == Value::MAP) inner = *ip;
    for (const char* key : {"unlearner", "unlearner_parameter"})
      if (const Value* x = c->param.get(key)) inner.o.emplace_back(key, *x);
    c->param = inner;
  } else if (c->outer == "nearest_neighbor_recommender") {
    c->inner = c->param.str_or("method", "");
    if (!is_lsh(c->inner)) { *why = "nearest_neighbor_recommender inner method"; return false; }
    // the unlearner of the outer parameters applies (Recommender.__init__)
    Value inner = empty;
    if (const Value* ip = c->param.get("parameter"))
      if (ip->kind == Value::MAP) inner = *ip;
    for (const char* k : {"unlearner", "unlearner_parameter"})
      if (const Value* x = c->param.get(k)) inner.o.emplace_back(k, *x);
    c->param = inner;
  } else if (!is_lsh(c->outer) && c->outer != "inverted_index" && c->outer != "inverted_index_euclid") {
    *why = "recommender method " + c->outer;
    return false;
  }
  if (const Value* h = c->param.get("hash_num"))
    if (!h->is_num() || h->num() <= 0) { *why = "hash_num"; return false; }
  if (const Value* u = c->param.get("unlearner")) {
    if (u->kind != Value::NIL && !(u->is_str() && u->s == "lru")) { *why = "unlearner"; return false; }
    if (u->is_str()) {
      const Value* up = c->param.get("unlearner_parameter");
      const Value* ms = up ? up->get("max_size") : nullptr;
      if (!ms || !ms->is_num() || ms->num() <= 0) { *why = "unlearner_parameter.max_size"; return false; }
    }
  }
  const Value* conv = v.get("converter");
  c->conv = conv ? *conv : empty;
  jb::row::Converter probe;
  if (!probe.configure(c->conv, why)) return false;
  c->text = text;
  return true;
}

class Model : public jb::mix::Mixable {
 public:
  std::atomic<uint64_t> update_count{0};
  uint64_t clear_row_cnt = 0, update_row_cnt = 0;

  Model(Kind kind, const Config& cfg, int device) : kind_(kind), device_(device) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    // the LOF state's own stream: a batch's one-wave add kernel runs while
    // the next batch's neighbour queries run on stream_ (add_many); the
    // state only takes host-staged candidates, no stream_ results
    HIPCHK(hipStreamCreateWithFlags(&lof_stream_, hipStreamNonBlocking));
    configure(cfg);
    HIPCHK(hipStreamCreateWithFlags(&mix_stream_, hipStreamNonBlocking));
    batcher_ = std::thread([this] {
      HIPCHK(hipSetDevice(device_));
      batch_loop();
    });
  }

  // ------------------------------------------------------------- MIX
  std::unique_ptr<jb::mix::Plane> make_plane(jb::mix::Star& star, double dl) {
    return jb::mix::make_device_plane(star, device_, mix_stream_, dl);
  }
  // one MIX (all ranks): the model is held exclusively from packing this
  // server's diff to applying the cluster's (the reference's put_diff takes
  // the model write lock, linear_mixer.cpp:613-662)
  uint64_t mix(jb::mix::Group& g) override {
    std::unique_lock<std::shared_mutex> lk(mu_);
    MsgpackWriter w;
    pack_mix(w);
    const auto raw = g.plane().allgather_bytes(g.star(), w.out, g.deadline());
    std::vector<Value> parts;
    parts.reserve(raw.size());
    for (const auto& r : raw) parts.push_back(MsgpackReader((const uint8_t*)r.data(), r.size()).read());
    const size_t n = apply_mix(parts, false);
    // LOF: the neighbour lists are caches of the row set; rows written by the
    // MIX invalidate them (rebuilt on demand against the mixed rows)
    if (kind_ == Kind::kAnomaly && n > 0) lof_.reset();
    HIPCHK(hipStreamSynchronize(stream_));
    last_mix_rows_ = n;
    uint64_t bytes = 0;
    for (const auto& r : raw) bytes += r.size();
    return bytes;
  }
  // push mixers: the pair folds its two row diffs, lower rank first
  uint64_t pair_mix(jb::mix::Group& g, int peer) override {
    std::unique_lock<std::shared_mutex> lk(mu_);
    std::string mine;
    if (peer >= 0) {
      MsgpackWriter w;
      pack_mix(w);
      mine = std::move(w.out);
    }
    const std::string theirs = g.plane().exchange_bytes(g.star(), peer, mine, g.deadline());
    if (peer < 0) return 0;
    Value a = MsgpackReader((const uint8_t*)mine.data(), mine.size()).read();
    Value b = MsgpackReader((const uint8_t*)theirs.data(), theirs.size()).read();
    std::vector<Value> parts;
    if (g.rank() < peer) { parts.push_back(std::move(a)); parts.push_back(std::move(b)); }
    else { parts.push_back(std::move(b)); parts.push_back(std::move(a)); }
    const size_t n = apply_mix(parts, true);
    if (kind_ == Kind::kAnomaly && n > 0) lof_.reset();
    HIPCHK(hipStreamSynchronize(stream_));
    last_mix_rows_ = n;
    return mine.size();
  }
  bool push_mixable() const override { return true; }
  void push_end() override {
    std::unique_lock<std::shared_mutex> lk(mu_);
    eng_->mix_done();
  }

  // obsolete protocol: rank src's whole model replaces an obsolete member's
  void hand_over(jb::mix::Group& g, int src, bool apply) override {
    std::string mine;
    if (g.rank() == src) mine = pack_user_data();
    const std::string got = g.plane().bcast_bytes(g.star(), src, mine, g.deadline());
    if (apply) {
      const Value v = MsgpackReader((const uint8_t*)got.data(), got.size()).read();
      if (v.kind != Value::ARR || v.a.size() != 2) throw std::runtime_error("hand-over: malformed model");
      unpack(v.a[1]);
    }
  }
  size_t last_mix_rows() const { return last_mix_rows_; }
  ~Model() {
    {
      std::lock_guard<std::mutex> lk(qmu_);
      stop_ = true;
    }
    qcv_.notify_all();
    if (batcher_.joinable()) batcher_.join();
  }
  uint64_t batches() const { return n_batches_.load(); }
  uint64_t n_write_batches_ = 0, n_write_rows_ = 0;   // (under mu_)
  // batched anomaly adds (under mu_): chunks, wall microseconds preparing
  // (rows set, neighbour queries) and finishing (LOF wait, stopped adds)
  uint64_t ab_chunks_ = 0;
  double ab_us_[2] = {0, 0};
  // wall microseconds of the write batches (under mu_): parse / hash outside
  // the lock, the locked apply, the device flush; the RPC side adds the
  // argument decoding (status key write_batch_us)
  double wb_us_[4] = {0, 0, 0, 0};
  // the stateless hasher of the current converter (prep_write; atomic
  // shared_ptr access: the IO threads read it without the model lock)
  std::shared_ptr<const jb::HostFvHasher> prep_h_;
  uint64_t batched_queries() const { return n_batched_.load(); }

  void configure(const Config& cfg) {
    std::unique_lock<std::shared_mutex> g(mu_);
    HIPCHK(hipStreamSynchronize(stream_));
    lof_.reset();
    eng_.reset(new RowEngine(cfg.inner, &cfg.param, stream_));
    std::string why;
    if (!eng_->conv.configure(cfg.conv, &why)) throw std::runtime_error("converter: " + why);
    std::atomic_store(&prep_h_, eng_->conv.stateless());
    cfg_ = cfg;
    if (kind_ == Kind::kAnomaly)   // LOF._remove: a removed row's dependants go stale
      eng_->on_remove = [this](int32_t s) { if (lof_) lof_->moved({s}); };
    if (kind_ == Kind::kClassifier) {   // an evicted / removed row loses its label (NNClassifier._gc)
      eng_->on_remove = [this](int32_t s) { row_label_.erase(eng_->at(s).id); };
      row_label_.clear();
      labels_.clear();
      label_order_.clear();
      seq_ = 0;
      if (prefix_.empty()) {
        std::random_device rd;
        char b[16];
        snprintf(b, sizeof b, "%08x", (unsigned)rd());
        prefix_ = b;
      }
    }
  }

  // ------------------------------------------------------------ classifier
  // models/nn_classifier.py train: each example a row "<prefix>-<seq>"
  // tagged with its label
  int64_t nn_train(const Value& data) {
    std::vector<std::pair<std::string, Datum>> ex;
    for (const Value& x : data.a) {
      if (x.kind != Value::ARR || x.a.size() != 2 || !x.a[0].is_str()) throw ArgError("labeled_datum expected");
      Datum d;
      jb::row::parse_datum(x.a[1], &d);
      ex.emplace_back(x.a[0].s, std::move(d));
    }
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    for (auto& e : ex) {
      const std::string rid = prefix_ + "-" + std::to_string(seq_++);
      eng_->set(rid, std::move(e.second));
      if (eng_->slot(rid) >= 0) row_label_[rid] = e.first;
      add_label(e.first, 1);
    }
    return (int64_t)ex.size();
  }
  // every known label, scored over the query's k nearest rows
  std::vector<std::vector<std::pair<std::string, double>>> nn_classify(const Value& data) {
    const size_t n = data.a.size();
    std::vector<QReq> rs(n);
    for (size_t i = 0; i < n; ++i) {
      Datum chk;
      jb::row::parse_datum(data.a[i], &chk);
      MsgpackWriter w;
      write_value(w, data.a[i]);
      rs[i].kind = QReq::kDatum;
      rs[i].datum = std::move(w.out);
      rs[i].k = cfg_.nn_k;
      rs[i].similar = cfg_.similar;
    }
    std::vector<QReq*> ps;
    for (auto& r : rs) ps.push_back(&r);
    submit_many(ps);
    std::shared_lock<std::shared_mutex> g(mu_);
    std::vector<std::vector<std::pair<std::string, double>>> out(n);
    for (size_t i = 0; i < n; ++i) {
      std::unordered_map<std::string, double> sc;
      for (const auto& lab : label_order_) sc[lab] = 0.0;
      std::vector<std::string> extra;
      for (const auto& hv : rs[i].res) {
        auto it = row_label_.find(hv.first);
        if (it == row_label_.end()) continue;
        if (!sc.count(it->second)) extra.push_back(it->second);
        sc[it->second] += cfg_.similar ? hv.second : exp(-cfg_.alpha * hv.second);
      }
      for (const auto& lab : label_order_) out[i].emplace_back(lab, sc[lab]);
      for (const auto& lab : extra) out[i].emplace_back(lab, sc[lab]);
    }
    return out;
  }
  std::vector<std::pair<std::string, uint64_t>> nn_labels() {
    std::shared_lock<std::shared_mutex> g(mu_);
    std::vector<std::pair<std::string, uint64_t>> out;
    for (const auto& lab : label_order_) out.emplace_back(lab, labels_.at(lab));
    return out;
  }
  bool nn_set_label(const std::string& lab) {
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    if (labels_.count(lab)) return false;
    add_label(lab, 0);
    return true;
  }
  bool nn_delete_label(const std::string& lab) {
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    if (!labels_.count(lab)) return false;
    std::vector<std::string> drop;
    for (const auto& kv : row_label_)
      if (kv.second == lab) drop.push_back(kv.first);
    for (const auto& rid : drop) eng_->remove(rid);   // on_remove drops the tag
    labels_.erase(lab);
    label_order_.erase(std::find(label_order_.begin(), label_order_.end(), lab));
    return true;
  }
  const std::string& config_text() const { return cfg_.text; }

  // ------------------------------------------------------------- updates
  bool clear_row(const std::string& id) {
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    ++clear_row_cnt;
    return eng_->remove(id);
  }
  // recommender update_row: merge into the stored datum (RowEngine.update_row)
  bool update_row(const std::string& id, const Value& dv) {
    Datum nd;
    jb::row::parse_datum(dv, &nd);
    std::unique_lock<std::shared_mutex> g(mu_);
    update_row_locked(id, std::move(nd));
    return true;
  }
  void update_row_locked(const std::string& id, Datum&& nd) {
    ++update_count;
    ++update_row_cnt;
    if (const jb::row::Row* r = eng_->find(id)) {
      Datum m = r->d;
      for (auto& kv : nd.sv) m.sv[kv.first] = kv.second;
      for (auto& kv : nd.nv) m.nv[kv.first] = kv.second;
      for (auto& kv : nd.bv) m.bv[kv.first] = kv.second;
      nd = std::move(m);
    }
    eng_->set(id, std::move(nd));
  }

  // A batch of queued writes of one method (the RPC batch thread, see
  // Server::run): the datums parse outside the model lock, the writes apply
  // in arrival order under ONE exclusive section, and the LSH signatures of
  // the whole batch go to the device in one staged launch (LshIndex
  // set_defer) instead of one launch per row. kind: 0 update_row, 1
  // set_row, 2 clear_row. -> per write: 1 / 0 (clear_row of an unknown id),
  // or the exception it raised
  // a write decoded and hashed on the RPC IO thread (prep_write)
  struct PrepWrite {
    std::shared_ptr<const jb::HostFvHasher> h;   // the hasher it used (null: parsed only)
    std::string id;
    Datum d;
    std::vector<int32_t> idx;
    std::vector<float> val;
  };
  struct Write {
    const std::string* id;
    const Value* dv;          // or:
    PrepWrite* pre = nullptr;
    int result = 0;
    std::exception_ptr err;
  };
  // IO thread, no model lock (the hasher is an immutable snapshot): decode
  // an update_row / set_row and hash its datum as a row of its own - or only
  // decode it when the converter keeps statistics (they change under the
  // lock); null when the request is not well formed (the batch path decodes
  // it again and answers the error)
  std::shared_ptr<PrepWrite> prep_write(const std::string& params) const {
    std::shared_ptr<const jb::HostFvHasher> h = std::atomic_load(&prep_h_);
    try {
      Value a = MsgpackReader((const uint8_t*)params.data(), params.size()).read();
      if (a.kind != Value::ARR || a.a.size() != 3 || !a.a[0].is_str() || !a.a[1].is_str() ||
          a.a[2].kind != Value::ARR)
        return nullptr;
      auto p = std::make_shared<PrepWrite>();
      jb::row::parse_datum(a.a[2], &p->d);
      if (h) {
        MsgpackWriter w;
        jb::row::write_datum(w, p->d);
        jb::row::Converter::hash_with(*h, (const uint8_t*)w.out.data(), w.out.size(), &p->idx, &p->val);
      }
      p->id = std::move(a.a[1].s);
      p->h = std::move(h);
      return p;
    } catch (...) {
      return nullptr;
    }
  }
  void write_many(int kind, std::vector<Write>& ws) {
    // parse each datum, and with a stateless converter hash it as a row of
    // its own (a write whose id turns out to be stored merges and hashes
    // again under the lock); the IO threads did both for most writes
    std::vector<Datum> ds(ws.size());
    std::vector<std::vector<int32_t>> hi(ws.size());
    std::vector<std::vector<float>> hv(ws.size());
    std::vector<uint8_t> pre(ws.size(), 0);
    using Clk = std::chrono::steady_clock;
    const auto t0 = Clk::now();
    if (kind != 2) {
      std::shared_lock<std::shared_mutex> rd(mu_);   // (the converter stays as it is)
      const std::shared_ptr<const jb::HostFvHasher> h = eng_->conv.stateless();
      for (size_t i = 0; i < ws.size(); ++i) {
        try {
          if (PrepWrite* p = ws[i].pre) {
            ds[i] = std::move(p->d);
            if (p->h != nullptr && p->h == h) {
              hi[i] = std::move(p->idx);
              hv[i] = std::move(p->val);
              pre[i] = 1;
              continue;
            }
          } else {
            jb::row::parse_datum(*ws[i].dv, &ds[i]);
          }
          if (h) {
            MsgpackWriter w;
            jb::row::write_datum(w, ds[i]);
            jb::row::Converter::hash_with(*h, (const uint8_t*)w.out.data(), w.out.size(), &hi[i], &hv[i]);
            pre[i] = 1;
          }
        } catch (...) {
          ws[i].err = std::current_exception();
        }
      }
    }
    const auto t1 = Clk::now();
    std::unique_lock<std::shared_mutex> g(mu_);
    eng_->defer_writes(true);
    for (size_t i = 0; i < ws.size(); ++i) {
      if (ws[i].err) continue;
      try {
        if (kind == 0 && (!pre[i] || eng_->find(*ws[i].id) != nullptr)) {
          update_row_locked(*ws[i].id, std::move(ds[i]));
          ws[i].result = 1;
        } else if (kind != 2) {
          ++update_count;
          if (kind == 0) ++update_row_cnt;
          if (pre[i]) eng_->store(*ws[i].id, std::move(ds[i]), hi[i], hv[i], true);
          else eng_->set(*ws[i].id, std::move(ds[i]));
          ws[i].result = 1;
        } else {
          ++update_count;
          ++clear_row_cnt;
          ws[i].result = eng_->remove(*ws[i].id) ? 1 : 0;
        }
      } catch (...) {
        ws[i].err = std::current_exception();
      }
    }
    const auto t2 = Clk::now();
    eng_->defer_writes(false);
    const auto t3 = Clk::now();
    wb_us_[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
    wb_us_[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
    wb_us_[2] += std::chrono::duration<double, std::micro>(t3 - t2).count();
    ++n_write_batches_;
    n_write_rows_ += ws.size();
  }
  uint64_t write_batches() const { return n_write_batches_; }
  void add_decode_us(double us) {
    std::unique_lock<std::shared_mutex> g(mu_);
    wb_us_[3] += us;
  }
  uint64_t write_rows() const { return n_write_rows_; }
  // nearest_neighbor set_row: replace
  bool set_row(const std::string& id, const Value& dv) {
    Datum nd;
    jb::row::parse_datum(dv, &nd);
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    eng_->set(id, std::move(nd));
    return true;
  }
  void clear() {
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    clear_row_cnt = update_row_cnt = 0;
    eng_->clear();
    lof_.reset();
    next_id_ = 0;
    row_label_.clear();
    labels_.clear();
    label_order_.clear();
    seq_ = 0;
  }

  // ------------------------------------------------------------- anomaly
  // anomaly_serv.cpp add (standalone): a new id from the counter, insert
  std::pair<std::string, double> add(const Value& dv) {
    Datum d;
    jb::row::parse_datum(dv, &d);
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    const std::string id = std::to_string(next_id_++);
    return {id, (double)insert(id, std::move(d))};
  }
  // A batch of anomaly adds (Server::add_batch; anomaly_serv.cpp:157-176 per
  // add): the rows are set with one staged signature launch, their
  // neighbours come from multi-query passes over the table holding the whole
  // batch (k = rnn + batch, then each add drops itself and the rows added
  // after it - exactly its sequential candidate list), and the LOF inserts
  // run as one enqueue (LofState::add_many). Ids, candidates and scores are
  // those of the adds one by one, in arrival order.
  struct AddReq {
    const Value* dv = nullptr;
    std::string id;
    double score = 0;
    bool scored = false;   // the add finished (a chunk that throws fails the rest)
    std::exception_ptr err;
  };
  void add_many(std::vector<AddReq>& rs) {
    std::vector<Datum> ds(rs.size());
    for (size_t i = 0; i < rs.size(); ++i) {
      try {
        jb::row::parse_datum(*rs[i].dv, &ds[i]);
      } catch (...) {
        rs[i].err = std::current_exception();
      }
    }
    std::unique_lock<std::shared_mutex> g(mu_);
    // JB_LOF_CHUNK: adds per LOF launch, default 8 - one neighbour query
    // pass (kQueryMax queries) per chunk, and the pipeline below overlaps it
    // with the previous chunk's kernel. Measured (100K-row fill, 16 x 8 in
    // flight): 64 -> 40K adds/s, 16 -> 53K, 8 -> 58K
    static const int chunk_env = [] {
      const char* e = getenv("JB_LOF_CHUNK");
      return e != nullptr && atoi(e) > 0 ? atoi(e) : 8;
    }();
    const int cmax = std::max(1, std::min(jb::row::kLofBatchMax, 128 - cfg_.rnn));
    const size_t chunk = (size_t)std::min(chunk_env, cmax);
    using Clk = std::chrono::steady_clock;
    auto us = [](Clk::time_point a, Clk::time_point b) {
      return std::chrono::duration<double, std::micro>(b - a).count();
    };
    std::vector<size_t> todo;
    for (size_t i = 0; i < rs.size(); ++i)
      if (!rs[i].err) todo.push_back(i);
    // pipelined: chunk c's rows are set and its neighbours queried (stream_)
    // while chunk c - 1's LOF kernel runs (lof_stream_); c - 1 finishes
    // before c's kernel starts, so the adds still apply in arrival order
    auto fail = [&rs](const std::vector<size_t>& ids) {
      for (size_t i : ids)
        if (!rs[i].err && !rs[i].scored) rs[i].err = std::current_exception();
    };
    std::unique_ptr<AddChunk> prev;
    auto finish_prev = [&](const std::vector<int32_t>& later, AddChunk* next) {
      if (!prev) return;
      const auto t0 = Clk::now();
      try {
        finish_chunk(rs, *prev, later, next);
      } catch (...) {
        fail(prev->idx);
      }
      prev.reset();
      ab_us_[1] += us(t0, Clk::now());
    };
    for (size_t c0 = 0; c0 < todo.size(); c0 += chunk) {
      const size_t c1 = std::min(todo.size(), c0 + chunk);
      std::unique_ptr<AddChunk> cur(new AddChunk);
      cur->idx.assign(todo.begin() + c0, todo.begin() + c1);
      if (!batchable(cur->idx.size())) {
        finish_prev({}, nullptr);
        try {
          for (size_t i : cur->idx) {
            ++update_count;
            rs[i].id = std::to_string(next_id_++);
            rs[i].score = (double)insert(rs[i].id, std::move(ds[i]));
            rs[i].scored = true;
          }
        } catch (...) {
          fail(cur->idx);
        }
        continue;
      }
      bool ok = true;
      const auto t0 = Clk::now();
      try {
        prepare_chunk(rs, ds, cur.get());
      } catch (...) {
        fail(cur->idx);
        ok = false;
      }
      ab_us_[0] += us(t0, Clk::now());
      ++ab_chunks_;
      if (!ok) {
        finish_prev({}, nullptr);
        continue;
      }
      // a previous chunk whose batch did not run (queued behind one that
      // stopped) reruns first, alone: nothing may queue ahead of its adds
      if (prev && !prev->launched) finish_prev(cur->slots, nullptr);
      // queued behind the previous chunk's kernel: it starts when that one
      // ends (or does not run if that one stops - finish_chunk reruns it)
      std::exception_ptr lerr;
      try {
        state().launch_many(cur->slots, cur->cs, cur->cd);
        cur->launched = true;
      } catch (...) {
        lerr = std::current_exception();
      }
      finish_prev(cur->slots, cur.get());
      if (lerr) {
        for (size_t i : cur->idx)
          if (!rs[i].err && !rs[i].scored) rs[i].err = lerr;
        continue;
      }
      prev = std::move(cur);
    }
    finish_prev({}, nullptr);
  }
  // update merges into the stored datum, overwrite replaces it
  double update(const std::string& id, const Value& dv, bool merge) {
    Datum nd;
    jb::row::parse_datum(dv, &nd);
    std::unique_lock<std::shared_mutex> g(mu_);
    ++update_count;
    if (merge)
      if (const jb::row::Row* r = eng_->find(id)) {
        Datum m = r->d;
        for (auto& kv : nd.sv) m.sv[kv.first] = kv.second;
        for (auto& kv : nd.nv) m.nv[kv.first] = kv.second;
        for (auto& kv : nd.bv) m.bv[kv.first] = kv.second;
        nd = std::move(m);
      }
    return (double)insert(id, std::move(nd));
  }
  // models/anomaly.py calc_score: the k nearest stored rows, then LOF
  // (batched: the neighbours of every queued calc_score in one pass)
  double calc_score(const Value& dv) {
    Datum chk;
    jb::row::parse_datum(dv, &chk);
    QReq r;
    r.kind = QReq::kScore;
    MsgpackWriter w;
    write_value(w, dv);
    r.datum = std::move(w.out);
    r.k = cfg_.k;
    submit(&r);
    return r.score;
  }

  // ------------------------------------------------------------- queries
  // Analysis calls handed over by the RPC batch thread (every queued
  // similar_row_* / neighbor_row_* / calc_score of one method): validated
  // here, then run as ONE batch on this thread - no RPC worker blocks on a
  // query, so the batch size follows the requests in flight, not the -c
  // worker count.
  enum CallKind { kCallDatum = 0, kCallId = 1, kCallScore = 2 };
  struct Call {
    CallKind what = kCallDatum;
    const Value* dv = nullptr;   // kCallDatum, kCallScore
    std::string id;              // kCallId
    int64_t k = 0;
    bool similar = true;
    std::vector<std::pair<std::string, double>> res;
    double score = 0.0;
    std::exception_ptr err;
  };
  void run_calls(std::vector<Call>& cs) {
    jb::tx::Range tr("rows.query_batch");
    std::vector<QReq> reqs(cs.size());
    std::vector<QReq*> ptrs;
    for (size_t i = 0; i < cs.size(); ++i) {
      Call& c = cs[i];
      QReq& r = reqs[i];
      try {
        if (c.what == kCallId) {
          r.kind = QReq::kId;
          r.id = c.id;
          r.k = c.k <= 0 ? 0 : clamp_k(c.k);
          r.neg_k = c.k <= 0;
          r.similar = c.similar;
        } else {
          Datum chk;
          jb::row::parse_datum(*c.dv, &chk);           // validate first (ARGUMENT_ERROR)
          if (c.what == kCallDatum && c.k <= 0) continue;
          MsgpackWriter w;
          write_value(w, *c.dv);
          r.datum = std::move(w.out);
          r.kind = c.what == kCallScore ? (int)QReq::kScore : (int)QReq::kDatum;
          r.k = c.what == kCallScore ? cfg_.k : clamp_k(c.k);
          r.similar = c.similar;
        }
        ptrs.push_back(&r);
      } catch (...) {
        c.err = std::current_exception();
      }
    }
    if (!ptrs.empty()) {
      std::lock_guard<std::mutex> g(run_mu_);
      run_batch(ptrs);
    }
    for (size_t i = 0; i < cs.size(); ++i) {
      if (cs[i].err) continue;
      cs[i].err = reqs[i].err;
      cs[i].res = std::move(reqs[i].res);
      cs[i].score = reqs[i].score;
    }
  }

  std::vector<std::pair<std::string, double>> query_id(const std::string& id, int64_t k, bool similar) {
    QReq r;
    r.kind = QReq::kId;
    r.id = id;
    r.k = k <= 0 ? 0 : clamp_k(k);
    r.neg_k = k <= 0;
    r.similar = similar;
    submit(&r);
    return std::move(r.res);
  }
  std::vector<std::pair<std::string, double>> query_datum(const Value& dv, int64_t k, bool similar) {
    Datum chk;
    jb::row::parse_datum(dv, &chk);                  // validate first (ARGUMENT_ERROR)
    if (k <= 0) return {};
    QReq r;
    r.kind = QReq::kDatum;
    MsgpackWriter w;
    write_value(w, dv);
    r.datum = std::move(w.out);
    r.k = clamp_k(k);
    r.similar = similar;
    submit(&r);
    return std::move(r.res);
  }

  Datum decode_row(const std::string& id) {
    std::shared_lock<std::shared_mutex> g(mu_);
    const jb::row::Row* r = eng_->find(id);
    return r ? r->d : Datum();
  }
  std::vector<std::string> get_all_rows() {
    std::shared_lock<std::shared_mutex> g(mu_);
    return eng_->all_ids();
  }

  // models/recommender.py complete_row_from_id / _from_datum / _complete
  Datum complete_row_from_id(const std::string& id) {
    std::unique_lock<std::shared_mutex> g(mu_);
    const jb::row::Row* r = eng_->find(id);
    if (!r) return Datum();
    const std::vector<int32_t> idx = r->idx;
    const std::vector<float> val = r->val;
    const std::map<std::string, double> base = r->d.nv;
    auto nb = eng_->results(eng_->query_fv(idx, val, kCompleteK + 1), true);
    std::vector<std::pair<std::string, double>> keep;
    for (auto& x : nb)
      if (x.first != id) keep.push_back(x);
    if (keep.size() > (size_t)kCompleteK) keep.resize(kCompleteK);
    return complete(base, keep);
  }
  Datum complete_row_from_datum(const Value& dv) {
    Datum d;
    jb::row::parse_datum(dv, &d);
    auto nb = query_datum(dv, kCompleteK, true);
    std::shared_lock<std::shared_mutex> g(mu_);
    return complete(d.nv, nb);
  }

  double calc_similarity(const Value& a, const Value& b) {
    std::vector<int32_t> ai, bi;
    std::vector<float> av, bv;
    fv_of(a, &ai, &av);
    fv_of(b, &bi, &bv);
    std::shared_lock<std::shared_mutex> g(mu_);
    return eng_->calc_similarity(ai, av, bi, bv);
  }
  double calc_l2norm(const Value& a) {
    std::vector<int32_t> ai;
    std::vector<float> av;
    fv_of(a, &ai, &av);
    double s = 0.0;
    for (size_t i = 0; i < ai.size(); ++i)
      if (ai[i] >= 0) s += (double)av[i] * (double)av[i];
    return sqrt(s);
  }

  // ------------------------------------------------------------ persist
  std::string pack_user_data() {
    std::unique_lock<std::shared_mutex> g(mu_);
    HIPCHK(hipStreamSynchronize(stream_));
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    if (kind_ == Kind::kClassifier) {   // NNClassifier.pack()
      u.map(5);
      u.str("method"); u.str(cfg_.outer);
      u.str("engine"); eng_->pack(u, eng_->method());
      u.str("row_label"); u.map(row_label_.size());
      for (const auto& kv : row_label_) { u.str(kv.first); u.str(kv.second); }
      u.str("labels"); u.map(label_order_.size());
      for (const auto& lab : label_order_) { u.str(lab); u.uint(labels_.at(lab)); }
      u.str("seq"); u.uint(seq_);
      return std::move(u.out);
    }
    eng_->pack(u, eng_->method());
    return std::move(u.out);
  }
  void unpack(const Value& obj) {
    std::unique_lock<std::shared_mutex> g(mu_);
    lof_.reset();                  // LOF.unpack: lists rebuilt on demand
    if (kind_ == Kind::kClassifier) {
      const Value* ev = obj.get("engine");
      const Value* rl = obj.get("row_label");
      const Value* lv = obj.get("labels");
      const Value* sq = obj.get("seq");
      if (!ev || !rl || rl->kind != Value::MAP || !lv || lv->kind != Value::MAP)
        throw std::runtime_error("broken model data: nn classifier");
      eng_->unpack(*ev);
      row_label_.clear();
      for (const auto& kv : rl->o) row_label_[kv.first] = kv.second.s;
      labels_.clear();
      label_order_.clear();
      for (const auto& kv : lv->o) add_label(kv.first, (uint64_t)kv.second.num());
      seq_ = sq && sq->is_num() ? (uint64_t)sq->num() : 0;
      HIPCHK(hipStreamSynchronize(stream_));
      return;
    }
    eng_->unpack(obj);
    lof_.reset();
    HIPCHK(hipStreamSynchronize(stream_));
    if (kind_ == Kind::kAnomaly) {
      // anomaly_serv.cpp:299-320: the id counter restarts past the largest
      // all-digit id
      int64_t m = -1;
      for (const std::string& id : eng_->all_ids()) {
        if (id.empty() || id.size() > 18 || id.find_first_not_of("0123456789") != std::string::npos) continue;
        m = std::max<int64_t>(m, std::stoll(id));
      }
      next_id_ = m + 1;
    }
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) {
    std::shared_lock<std::shared_mutex> g(mu_);
    auto add = [&](const char* k, const std::string& v) { st->emplace_back(k, v); };
    add("method", kind_ == Kind::kNearestNeighbor ? eng_->method() : cfg_.outer);
    add("write_batches", std::to_string(n_write_batches_));   // Model::write_many
    add("write_batch_rows", std::to_string(n_write_rows_));
    {   // decode (RPC args), prep (parse / hash), apply (locked), flush (device)
      char b[160];
      snprintf(b, sizeof b, "decode %.0f prep %.0f apply %.0f flush %.0f", wb_us_[3], wb_us_[0], wb_us_[1],
               wb_us_[2]);
      add("write_batch_us", b);
    }
    if (ab_chunks_) {
      char b[160];
      snprintf(b, sizeof b, "chunks %llu prepare %.0f finish %.0f", (unsigned long long)ab_chunks_, ab_us_[0],
               ab_us_[1]);
      add("add_batch_us", b);
    }
    if (kind_ == Kind::kClassifier) {
      add("num_labels", std::to_string(labels_.size()));
      add("nearest_neighbor_num", std::to_string(cfg_.nn_k));
      char b[40];
      snprintf(b, sizeof b, "%.17g", cfg_.alpha);
      add("local_sensitivity", b);
      add("nn.method", eng_->method());
    }
    if (kind_ == Kind::kAnomaly) add("backend", eng_->method());
    add("num_rows", std::to_string(eng_->size()));
    add("storage", "hbm");
    add("unlearner", eng_->lru() ? "lru" : "none");
    add("device", "cuda:" + std::to_string(device_));
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) add("hbm_used_bytes", std::to_string(tot - fr));
    add("server_runtime", "native");
    add("query_batches", std::to_string(n_batches_.load()));
    add("batched_queries", std::to_string(n_batched_.load()));
    if (kind_ == Kind::kRecommender) {
      add("clear_row_cnt", std::to_string(clear_row_cnt));
      add("update_row_cnt", std::to_string(update_row_cnt));
    }
  }

 private:
  int clamp_k(int64_t k) const { return (int)std::min<int64_t>(k, 1 << 30); }

  void add_label(const std::string& lab, uint64_t n) {   // mu_ held
    auto it = labels_.find(lab);
    if (it == labels_.end()) {
      labels_[lab] = n;
      label_order_.push_back(lab);
    } else {
      it->second += n;
    }
  }

  // the MIX payload: the row diff (jb_row_mix.hpp); the classifier adds the
  // labels of the rows in it and its label counts (NNClassifier.get_diff)
  void pack_mix(MsgpackWriter& w) {
    if (kind_ != Kind::kClassifier) {
      eng_->pack_diff(w);
      return;
    }
    w.arr(3);
    eng_->pack_diff(w);
    const std::vector<std::string> ids = eng_->mix_ids();
    size_t nt = 0;
    for (const auto& id : ids) nt += row_label_.count(id);
    w.map(nt);
    for (const auto& id : ids) {
      auto it = row_label_.find(id);
      if (it != row_label_.end()) { w.str(id); w.str(it->second); }
    }
    w.map(label_order_.size());
    for (const auto& lab : label_order_) { w.str(lab); w.uint(labels_.at(lab)); }
  }
  // mix_diff folded in rank order + put_diff; -> rows applied
  size_t apply_mix(const std::vector<Value>& parts, bool forward) {
    std::vector<int32_t> changed;
    if (kind_ != Kind::kClassifier) return eng_->apply_diffs(parts, &changed, forward);
    std::vector<Value> rows;
    std::vector<std::pair<std::string, std::string>> tags;
    std::vector<std::string> lorder;
    std::set<std::string> lseen;
    for (const Value& p : parts) {
      if (p.kind != Value::ARR || p.a.size() != 3 || p.a[1].kind != Value::MAP || p.a[2].kind != Value::MAP)
        throw std::runtime_error("mix: malformed nn classifier diff");
      rows.push_back(p.a[0]);
      for (const auto& kv : p.a[1].o) tags.emplace_back(kv.first, kv.second.s);
      for (const auto& kv : p.a[2].o)
        if (lseen.insert(kv.first).second) lorder.push_back(kv.first);
    }
    const size_t n = eng_->apply_diffs(rows, &changed, forward);
    for (const auto& t : tags)
      if (eng_->slot(t.first) >= 0) row_label_[t.first] = t.second;
    // counts: the labels of the rows held now (put_diff), every label known
    std::vector<std::string> order = lorder;
    for (const auto& lab : label_order_)
      if (!lseen.count(lab)) order.push_back(lab);
    labels_.clear();
    label_order_.clear();
    for (const auto& lab : order) add_label(lab, 0);
    for (const auto& kv : row_label_) add_label(kv.second, 1);
    return n;
  }

  void fv_of(const Value& dv, std::vector<int32_t>* idx, std::vector<float>* val) {
    Datum chk;
    jb::row::parse_datum(dv, &chk);
    MsgpackWriter w;
    write_value(w, dv);
    std::shared_lock<std::shared_mutex> g(mu_);
    std::lock_guard<std::mutex> h(hash_mu_);
    eng_->conv.hash((const uint8_t*)w.out.data(), w.out.size(), idx, val, false);
  }

  Datum complete(const std::map<std::string, double>& base,
                 const std::vector<std::pair<std::string, double>>& nb) {
    const std::string& m = eng_->method();
    const bool raw_w = m == "inverted_index" || m == "lsh" || m == "minhash";
    std::map<std::string, double> acc, wsum;
    for (const auto& x : nb) {
      const jb::row::Row* r = eng_->find(x.first);
      if (!r) continue;
      const double w = raw_w ? x.second : 1.0 / (1.0 + std::max(0.0, -x.second));
      if (w <= 0) continue;
      for (const auto& kv : r->d.nv) {
        acc[kv.first] += w * kv.second;
        wsum[kv.first] += w;
      }
    }
    Datum out;
    for (const auto& kv : acc)
      if (wsum[kv.first] > 0) out.nv[kv.first] = kv.second / wsum[kv.first];
    for (const auto& kv : base) out.nv[kv.first] = kv.second;
    return out;
  }

  // re-encode a decoded datum Value (the query's own order kept)
 public:
  static void write_value(MsgpackWriter& w, const Value& v) {
    switch (v.kind) {
      case Value::NIL: w.nil(); break;
      case Value::BOOL: w.boolean(v.b); break;
      case Value::INT: w.sint(v.i); break;
      case Value::UINT: w.uint(v.u); break;
      case Value::DBL: w.dbl(v.d); break;
      case Value::STR: case Value::BIN: w.raw(v.s); break;
      case Value::ARR:
        w.arr(v.a.size());
        for (const Value& x : v.a) write_value(w, x);
        break;
      case Value::MAP:
        w.map(v.o.size());
        for (const auto& kv : v.o) { w.raw(kv.first); write_value(w, kv.second); }
        break;
    }
  }
 private:


  // ------------------------------------------------------------ batcher
  struct QReq {
    enum { kDatum = 0, kScore = 1, kId = 2 };
    int kind = kDatum;
    std::string datum;        // msgpack of the query datum (kDatum, kScore)
    std::string id;           // kId
    int k = 0;
    bool neg_k = false;       // kId with k <= 0: only the existence check
    bool similar = true;
    std::vector<std::pair<std::string, double>> res;
    double score = 0.0;
    std::exception_ptr err;
    bool done = false;
  };

  void submit(QReq* r) {
    std::unique_lock<std::mutex> lk(qmu_);
    q_.push_back(r);
    qcv_.notify_one();
    dcv_.wait(lk, [&] { return r->done; });
    if (r->err) std::rethrow_exception(r->err);
  }
  // several queries of one call: queued together, so they share a pass
  void submit_many(const std::vector<QReq*>& rs) {
    if (rs.empty()) return;
    std::unique_lock<std::mutex> lk(qmu_);
    for (QReq* r : rs) q_.push_back(r);
    qcv_.notify_one();
    dcv_.wait(lk, [&] {
      for (QReq* r : rs)
        if (!r->done) return false;
      return true;
    });
    for (QReq* r : rs)
      if (r->err) std::rethrow_exception(r->err);
  }

  void batch_loop() {
    std::vector<QReq*> take;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(qmu_);
        qcv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;   // stop_ and drained
        take.assign(q_.begin(), q_.end());
        q_.clear();
      }
      {
        std::lock_guard<std::mutex> g(run_mu_);
        run_batch(take);
      }
      {
        std::lock_guard<std::mutex> lk(qmu_);
        for (QReq* r : take) r->done = true;
      }
      dcv_.notify_all();
    }
  }

  // one batch under the shared model lock: the batcher is the only reader
  // that touches the device index / LOF state (updates hold the lock
  // exclusively)
  void run_batch(std::vector<QReq*>& rs) {
    std::shared_lock<std::shared_mutex> g(mu_);
    ++n_batches_;
    n_batched_ += rs.size();
    const size_t n = rs.size();
    std::vector<std::vector<int32_t>> idx(n);
    std::vector<std::vector<float>> val(n);
    std::map<int, std::vector<size_t>> byk;
    {
      std::lock_guard<std::mutex> h(hash_mu_);
      for (size_t i = 0; i < n; ++i) {
        QReq* r = rs[i];
        if (r->kind == QReq::kId) continue;
        if (eng_->nslots() == 0) continue;        // nothing stored: no query
        try {
          eng_->conv.hash((const uint8_t*)r->datum.data(), r->datum.size(), &idx[i], &val[i], false);
          byk[r->k].push_back(i);
        } catch (...) {
          r->err = std::current_exception();
        }
      }
    }
    std::vector<std::vector<Hit>> hits(n);
    for (auto& kv : byk) {
      std::vector<const std::vector<int32_t>*> pi;
      std::vector<const std::vector<float>*> pv;
      for (size_t i : kv.second) { pi.push_back(&idx[i]); pv.push_back(&val[i]); }
      try {
        auto h = eng_->query_fv_many(pi, pv, kv.first);
        for (size_t q = 0; q < kv.second.size(); ++q) hits[kv.second[q]] = std::move(h[q]);
      } catch (...) {
        for (size_t i : kv.second) rs[i]->err = std::current_exception();
      }
    }
    // the batch's calc_score queries: one LOF launch each, one wait; a query
    // that meets rows without a valid list is finished alone below
    std::vector<size_t> sq;
    std::vector<std::vector<int32_t>> sts;
    std::vector<std::vector<float>> std_;
    std::vector<float> ssc;
    std::vector<char> sdone;
    for (size_t i = 0; i < n; ++i) {
      QReq* r = rs[i];
      if (r->err || r->kind != QReq::kScore) continue;
      sq.push_back(i);
      sts.emplace_back();
      std_.emplace_back();
      for (const Hit& hh : hits[i])
        if (live(hh.slot)) { sts.back().push_back(hh.slot); std_.back().push_back(hh.dist); }
    }
    if (sq.size() > 1) {
      try {
        state().score_many(sts, std_, &ssc, &sdone);
      } catch (...) {
        for (size_t i : sq) rs[i]->err = std::current_exception();
      }
    }
    for (size_t j = 0; j < sq.size(); ++j) {
      QReq* r = rs[sq[j]];
      if (r->err) continue;
      try {
        if (sq.size() > 1 && sdone[j]) r->score = (double)ssc[j];
        else if (sts[j].empty()) r->score = 1.0;
        else r->score = (double)score_from(sts[j], std_[j], -1);
      } catch (...) {
        r->err = std::current_exception();
      }
    }
    for (size_t i = 0; i < n; ++i) {
      QReq* r = rs[i];
      if (r->err || r->kind == QReq::kScore) continue;
      try {
        if (r->kind == QReq::kDatum) {
          r->res = eng_->results(hits[i], r->similar);
        } else {
          const int32_t s = eng_->slot(r->id);
          if (s < 0) throw std::runtime_error("'row not found: " + r->id + "'");   // str(KeyError)
          if (!r->neg_k) r->res = eng_->results(eng_->query_slot(s, r->k), r->similar);
        }
      } catch (...) {
        r->err = std::current_exception();
      }
    }
  }

  bool live(int32_t s) const { return s >= 0 && s < eng_->nslots() && eng_->at(s).live; }

  jb::row::LofState& state() {
    if (!lof_) lof_.reset(new jb::row::LofState(cfg_.k, cfg_.ignore_kth_same, lof_stream_));
    lof_->ensure(eng_->nslots());
    return *lof_;
  }

  // row_engine.query_slot_lists: each row's nearest (itself included), live
  // rows; absent: rows a batch of adds set but has not added yet
  std::vector<std::vector<std::pair<int32_t, float>>> slot_lists(const std::vector<int32_t>& slots, int k,
                                                                 const std::unordered_set<int32_t>* absent = nullptr) {
    std::vector<std::vector<std::pair<int32_t, float>>> out;
    const int kq = k + (absent ? (int)absent->size() : 0);
    for (int32_t s : slots) {
      std::vector<std::pair<int32_t, float>> l;
      for (const Hit& h : eng_->query_slot(s, std::min(kq, 128))) {
        if (!live(h.slot) || (absent && absent->count(h.slot))) continue;
        if ((int)l.size() >= k) break;
        l.push_back({h.slot, h.dist});
      }
      out.push_back(std::move(l));
    }
    return out;
  }

  // LOF._score_from: refresh missing neighbour lists until the score resolves
  float score_from(const std::vector<int32_t>& ts, const std::vector<float>& td, int32_t store,
                   const std::unordered_set<int32_t>* absent = nullptr) {
    jb::row::LofState& st = state();
    std::vector<int32_t> missing;
    for (int it = 0; it < 1 + 2 * cfg_.k; ++it) {
      float sc;
      if (st.score(ts, td, store, &sc, &missing)) return sc;
      st.set_lists(missing, slot_lists(missing, cfg_.k + 1, absent));
    }
    throw std::runtime_error("lof: neighbour lists did not converge");
  }

  // one chunk of add_many (mu_ held exclusively): its rows set, their
  // candidate lists (each add's rnn nearest among the rows before it)
  struct AddChunk {
    std::vector<size_t> idx;   // positions in the request batch
    std::vector<int32_t> slots;
    std::vector<std::vector<int32_t>> cs;
    std::vector<std::vector<float>> cd;
    bool launched = false;     // its first LOF launch is in flight
  };
  // fresh ids only (an id a client set with update / overwrite takes the
  // sequential path), more than one add, no unlearner
  bool batchable(size_t B) const {
    if (B <= 1 || eng_->lru()) return false;
    for (size_t j = 0; j < B; ++j)
      if (eng_->slot(std::to_string(next_id_ + (int64_t)j)) >= 0) return false;
    return true;
  }
  void prepare_chunk(std::vector<AddReq>& rs, std::vector<Datum>& ds, AddChunk* ch) {
    const size_t B = ch->idx.size();
    ch->slots.assign(B, -1);
    // deferral always ends (a failed set must not leave the index deferred)
    struct DeferGuard {
      RowEngine* e;
      ~DeferGuard() { e->defer_writes(false); }
    };
    {
      eng_->defer_writes(true);
      DeferGuard guard{eng_.get()};
      for (size_t j = 0; j < B; ++j) {
        const size_t i = ch->idx[j];
        ++update_count;
        rs[i].id = std::to_string(next_id_++);
        eng_->set(rs[i].id, std::move(ds[i]));
        ch->slots[j] = eng_->slot(rs[i].id);
      }
    }
    std::unordered_map<int32_t, size_t> order;
    for (size_t j = 0; j < B; ++j) order[ch->slots[j]] = j;
    std::vector<const std::vector<int32_t>*> qi;
    std::vector<const std::vector<float>*> qv;
    for (int32_t s : ch->slots) {
      qi.push_back(&eng_->at(s).idx);
      qv.push_back(&eng_->at(s).val);
    }
    const auto hits = eng_->query_fv_many(qi, qv, cfg_.rnn + (int)B);
    ch->cs.assign(B, {});
    ch->cd.assign(B, {});
    for (size_t j = 0; j < B; ++j)
      for (const Hit& h : hits[j]) {
        if (!live(h.slot) || h.slot == ch->slots[j]) continue;
        auto it = order.find(h.slot);
        if (it != order.end() && it->second > j) continue;   // added after j
        if ((int)ch->cs[j].size() >= cfg_.rnn) break;
        ch->cs[j].push_back(h.slot);
        ch->cd[j].push_back(h.dist);
      }
  }
  // the LOF adds of a prepared chunk (the first launch may be in flight);
  // later: rows set by the next chunk already, not added yet
  // next: the chunk queued behind this one (its batch does not run when
  // this one stops: it is marked for a rerun)
  void finish_chunk(std::vector<AddReq>& rs, AddChunk& ch, const std::vector<int32_t>& later, AddChunk* next) {
    const size_t B = ch.idx.size();
    jb::row::LofState& st = state();
    size_t j = 0;
    while (j < B) {
      std::vector<float> sc;
      std::vector<int32_t> missing;
      size_t m;
      if (ch.launched) {
        ch.launched = false;
        size_t dropped = 0;
        m = st.finish_many(&sc, &missing, &dropped);
        if (dropped > 0 && next != nullptr) next->launched = false;
      } else {
        std::vector<int32_t> ps(ch.slots.begin() + j, ch.slots.end());
        std::vector<std::vector<int32_t>> c(ch.cs.begin() + j, ch.cs.end());
        std::vector<std::vector<float>> d(ch.cd.begin() + j, ch.cd.end());
        m = st.add_many(ps, c, d, &sc, &missing);
      }
      for (size_t q = 0; q < m; ++q) {
        rs[ch.idx[j + q]].score = (double)sc[q];
        rs[ch.idx[j + q]].scored = true;
      }
      j += m;
      if (j < B) {   // add j stopped on lists to install: finish it as insert() does
        std::unordered_set<int32_t> absent(ch.slots.begin() + j + 1, ch.slots.end());
        absent.insert(later.begin(), later.end());
        const size_t kk = std::min<size_t>(ch.cs[j].size(), (size_t)cfg_.k);
        rs[ch.idx[j]].score = (double)score_from(std::vector<int32_t>(ch.cs[j].begin(), ch.cs[j].begin() + kk),
                                                 std::vector<float>(ch.cd[j].begin(), ch.cd[j].begin() + kk),
                                                 ch.slots[j], &absent);
        rs[ch.idx[j]].scored = true;
        ++j;
      }
    }
  }

  // LOF._insert
  float insert(const std::string& id, Datum&& d) {
    const bool existed = eng_->slot(id) >= 0;
    eng_->set(id, std::move(d));
    const int32_t s = eng_->slot(id);
    jb::row::LofState& st = state();
    if (existed) st.moved({s});
    std::vector<int32_t> cs;
    std::vector<float> cd;
    for (const Hit& h : eng_->query_slot(s, cfg_.rnn + 1)) {
      if (!live(h.slot) || h.slot == s) continue;
      if ((int)cs.size() >= cfg_.rnn) break;
      cs.push_back(h.slot);
      cd.push_back(h.dist);
    }
    float sc;
    std::vector<int32_t> missing;
    if (st.add(s, cs, cd, &sc, &missing)) return sc;
    const size_t kk = std::min<size_t>(cs.size(), (size_t)cfg_.k);
    return score_from(std::vector<int32_t>(cs.begin(), cs.begin() + kk),
                      std::vector<float>(cd.begin(), cd.begin() + kk), s);
  }

  Kind kind_;
  int device_;
  hipStream_t stream_;
  hipStream_t lof_stream_ = nullptr;
  hipStream_t mix_stream_ = nullptr;   // the RCCL plane's collectives
  size_t last_mix_rows_ = 0;
  std::shared_mutex mu_;      // the model: updates exclusive, analysis shared
  std::mutex hash_mu_;        // the converter's hashers (scratch state) under a shared lock
  std::mutex qmu_;            // the batcher's queue
  std::mutex run_mu_;         // one run_batch at a time (the engine's query buffers, the stream)
  std::condition_variable qcv_, dcv_;
  std::deque<QReq*> q_;
  bool stop_ = false;
  std::thread batcher_;
  std::atomic<uint64_t> n_batches_{0}, n_batched_{0};
  Config cfg_;
  std::unique_ptr<RowEngine> eng_;
  std::unique_ptr<jb::row::LofState> lof_;
  int64_t next_id_ = 0;
  // classifier: row -> label, label counts in first-seen order, row sequence
  std::unordered_map<std::string, std::string> row_label_;
  std::unordered_map<std::string, uint64_t> labels_;
  std::vector<std::string> label_order_;
  uint64_t seq_ = 0;
  std::string prefix_;
};

inline void write_pairs(MsgpackWriter& w, const std::vector<std::pair<std::string, double>>& r) {
  w.arr(r.size());
  for (const auto& x : r) {
    w.arr(2);
    w.raw(x.first);
    w.dbl(x.second);
  }
}

class Server {
 public:
  Server(Kind kind, const Args& a, const Config& cfg, int device) : kind_(kind), a_(a) {
    model_.reset(new Model(kind, cfg, device));
  }

  void load_file(const std::string& path) { load_impl(path, true); }

  // distributed mode (-z): coordinator session, config read lock
  void join_cluster(std::unique_ptr<jb::mix::ClusterNode> node) {
    node_ = std::move(node);
    a_.connected_zookeeper = node_->connected();
    if (!node_->config_rlock()) throw std::runtime_error("failed to get config lock");
  }

  int run() {
    rpc_.reset(new jb::RpcServer([this](const jb::RpcRequest& r) { return dispatch(r); }, a_.threads, 0.0));
    rpc_->set_io_threads(std::max(1, a_.threads / 4));
    // analysis RPCs bypass the workers: the batch thread serves everything
    // queued of one method with one device pass (Model::run_calls)
    std::vector<std::string> qm;
    if (kind_ == Kind::kRecommender || kind_ == Kind::kNearestNeighbor)
      qm = {"similar_row_from_datum", "similar_row_from_id"};
    if (kind_ == Kind::kNearestNeighbor) {
      qm.push_back("neighbor_row_from_datum");
      qm.push_back("neighbor_row_from_id");
    }
    if (kind_ == Kind::kAnomaly) qm = {"calc_score"};
    // standalone anomaly adds: one LOF pass per queued batch (Model::add_many);
    // in a cluster an add goes to its CHT owners one by one (add_zk)
    if (kind_ == Kind::kAnomaly && !node_) qm.push_back("add");
    // writes of the similarity engines: one exclusive section and one device
    // launch per batch of queued writes (Model::write_many)
    if (kind_ == Kind::kRecommender) {
      qm.push_back("update_row");
      qm.push_back("clear_row");
    }
    if (kind_ == Kind::kNearestNeighbor) qm.push_back("set_row");
    rpc_->set_ordered({"update_row", "clear_row", "set_row", "add"});
    if (kind_ == Kind::kRecommender || kind_ == Kind::kNearestNeighbor)
      rpc_->set_prep([this](jb::RpcRequest& r) {
        if (r.method == (kind_ == Kind::kRecommender ? "update_row" : "set_row"))
          r.prep = model_->prep_write(r.params);
      });
    if (!qm.empty())
      rpc_->set_batch(qm, [this](const std::string& m, std::vector<jb::RpcRequest>& rs) {
        if (m == "update_row" || m == "set_row" || m == "clear_row") return write_batch(m, rs);
        if (m == "add") return add_batch(rs);
        return query_batch(m, rs);
      }, 1024);
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
    if (node_) {   // distributed mode: actor + CHT vnodes, then the mixer thread
      node_->register_actor(a_.eth, a_.port);
      node_->register_cht(a_.eth, a_.port);
      jb::mix::MixerArgs ma;
      ma.kind = a_.mixer;
      ma.type = type();
      ma.name = a_.name;
      ma.eth = a_.eth;
      ma.port = a_.port;
      ma.interval_sec = a_.interval_sec;
      ma.interval_count = a_.interval_count;
      ma.interconnect_timeout = a_.ic_timeout;
      Model* m = model_.get();
      mixer_.reset(new jb::mix::LinearMixer(node_->coord(), ma, m, [m](jb::mix::Group& g, double dl) {
        return m->make_plane(g.star(), dl);
      }));
      mixer_->start();
      logf_("INFO", "registered group membership as %s (native %s)", ident().c_str(), a_.mixer.c_str());
    }
    logf_("INFO", "%s RPC server startup (native)", prog_name());
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

 private:
  std::string ident() const { return a_.eth + "_" + std::to_string(a_.port); }
  const char* type() const { return kind_name(kind_); }

  // one batch of writes of method m (see run()): malformed ones answer as
  // dispatch() would, the rest apply as one Model::write_many
  std::vector<std::string> write_batch(const std::string& m, std::vector<jb::RpcRequest>& rs) {
    std::vector<std::string> out(rs.size());
    const auto td = std::chrono::steady_clock::now();
    std::vector<Value> args(rs.size());
    std::vector<Model::Write> ws;
    std::vector<size_t> at;
    const bool clr = m == "clear_row";
    for (size_t i = 0; i < rs.size(); ++i) {
      const jb::RpcRequest& r = rs[i];
      if (r.prep) {   // decoded and hashed on the IO thread
        Model::Write w;
        w.pre = static_cast<Model::PrepWrite*>(r.prep.get());
        w.id = &w.pre->id;
        w.dv = nullptr;
        ws.push_back(w);
        at.push_back(i);
        continue;
      }
      bool ok = true;
      try {
        args[i] = MsgpackReader((const uint8_t*)r.params.data(), r.params.size()).read();
      } catch (const std::exception&) {
        ok = false;
      }
      const Value& a = args[i];
      ok = ok && a.kind == Value::ARR && a.a.size() == (clr ? 2u : 3u) && a.a[0].is_str() && a.a[1].is_str() &&
           (clr || a.a[2].kind == Value::ARR);
      if (!ok) {
        out[i] = r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
        continue;
      }
      Model::Write w;
      w.id = &a.a[1].s;
      w.dv = clr ? nullptr : &a.a[2];
      ws.push_back(w);
      at.push_back(i);
    }
    model_->add_decode_us(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - td).count());
    if (ws.empty()) return out;
    if (mixer_) mixer_->updated(ws.size());   // event_model_updated, once per write
    model_->write_many(m == "update_row" ? 0 : m == "set_row" ? 1 : 2, ws);
    for (size_t j = 0; j < ws.size(); ++j) {
      const jb::RpcRequest& r = rs[at[j]];
      if (r.notify) continue;
      try {
        if (ws[j].err) std::rethrow_exception(ws[j].err);
        MsgpackWriter w;
        w.boolean(ws[j].result != 0);
        out[at[j]] = jb::val::response_ok(r.msgid, w.out);
      } catch (const ArgError&) {
        out[at[j]] = jb::val::response_code(r.msgid, kArgumentError);
      } catch (const std::exception& e) {
        out[at[j]] = jb::val::response_msg(r.msgid, e.what());
      }
    }
    return out;
  }

  // one batch of anomaly adds (see run()): malformed ones answer as
  // dispatch() would, the rest run as one Model::add_many in arrival order
  std::vector<std::string> add_batch(std::vector<jb::RpcRequest>& rs) {
    jb::tx::Range tr("rows.lof_add_batch");
    std::vector<std::string> out(rs.size());
    std::vector<Value> args(rs.size());
    std::vector<Model::AddReq> reqs;
    std::vector<size_t> at;
    for (size_t i = 0; i < rs.size(); ++i) {
      const jb::RpcRequest& r = rs[i];
      bool ok = true;
      try {
        args[i] = MsgpackReader((const uint8_t*)r.params.data(), r.params.size()).read();
      } catch (const std::exception&) {
        ok = false;
      }
      const Value& a = args[i];
      ok = ok && a.kind == Value::ARR && a.a.size() == 2 && a.a[0].is_str() && a.a[1].kind == Value::ARR;
      if (!ok) {
        out[i] = r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
        continue;
      }
      Model::AddReq q;
      q.dv = &a.a[1];
      reqs.push_back(q);
      at.push_back(i);
    }
    if (reqs.empty()) return out;
    if (mixer_) mixer_->updated(reqs.size());   // event_model_updated, once per add
    model_->add_many(reqs);
    for (size_t j = 0; j < reqs.size(); ++j) {
      const jb::RpcRequest& r = rs[at[j]];
      if (r.notify) continue;
      try {
        if (reqs[j].err) std::rethrow_exception(reqs[j].err);
        MsgpackWriter w;
        w.arr(2);
        w.raw(reqs[j].id);
        w.dbl(reqs[j].score);
        out[at[j]] = jb::val::response_ok(r.msgid, w.out);
      } catch (const ArgError&) {
        out[at[j]] = jb::val::response_code(r.msgid, kArgumentError);
      } catch (const std::exception& e) {
        out[at[j]] = jb::val::response_msg(r.msgid, e.what());
      }
    }
    return out;
  }

  // one batch of analysis requests of method m (see run()): malformed ones
  // answer as dispatch() would, the rest run as one Model::run_calls
  std::vector<std::string> query_batch(const std::string& m, std::vector<jb::RpcRequest>& rs) {
    std::vector<std::string> out(rs.size());
    std::vector<Value> args(rs.size());
    std::vector<Model::Call> calls;
    std::vector<size_t> at;
    const bool score = m == "calc_score";
    const bool by_id = m == "similar_row_from_id" || m == "neighbor_row_from_id";
    for (size_t i = 0; i < rs.size(); ++i) {
      const jb::RpcRequest& r = rs[i];
      bool ok = true;
      try {
        args[i] = MsgpackReader((const uint8_t*)r.params.data(), r.params.size()).read();
      } catch (const std::exception&) {
        ok = false;
      }
      const Value& a = args[i];
      ok = ok && a.kind == Value::ARR && a.a.size() == (score ? 2u : 3u) && a.a[0].is_str() &&
           (by_id ? a.a[1].is_str() : a.a[1].kind == Value::ARR) &&
           (score || a.a[2].kind == Value::INT || a.a[2].kind == Value::UINT);
      if (!ok) {
        out[i] = r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
        continue;
      }
      Model::Call c;
      c.what = score ? Model::kCallScore : by_id ? Model::kCallId : Model::kCallDatum;
      if (by_id) c.id = a.a[1].s; else c.dv = &a.a[1];
      if (!score) {
        const Value& x = a.a[2];
        c.k = x.kind == Value::UINT ? (int64_t)std::min<uint64_t>(x.u, (uint64_t)INT64_MAX) : x.i;
      }
      c.similar = m.compare(0, 7, "similar") == 0;
      calls.push_back(std::move(c));
      at.push_back(i);
    }
    model_->run_calls(calls);
    for (size_t j = 0; j < calls.size(); ++j) {
      const jb::RpcRequest& r = rs[at[j]];
      if (r.notify) continue;
      try {
        if (calls[j].err) std::rethrow_exception(calls[j].err);
        MsgpackWriter w;
        if (score) w.dbl(calls[j].score); else write_pairs(w, calls[j].res);
        out[at[j]] = jb::val::response_ok(r.msgid, w.out);
      } catch (const ArgError&) {
        out[at[j]] = jb::val::response_code(r.msgid, kArgumentError);
      } catch (const std::exception& e) {
        out[at[j]] = jb::val::response_msg(r.msgid, e.what());
      }
    }
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
    // arity including the leading cluster name; argument kinds (s: string,
    // d: datum, k: size)
    static const std::vector<std::pair<std::string, std::string>> rec = {
        {"get_config", ""}, {"save", "s"}, {"load", "s"}, {"get_status", ""}, {"clear", ""},
        {"clear_row", "s"}, {"update_row", "sd"}, {"complete_row_from_id", "s"},
        {"complete_row_from_datum", "d"}, {"similar_row_from_id", "sk"}, {"similar_row_from_datum", "dk"},
        {"decode_row", "s"}, {"get_all_rows", ""}, {"calc_similarity", "dd"}, {"calc_l2norm", "d"},
        {"do_mix", ""}};
    static const std::vector<std::pair<std::string, std::string>> nn = {
        {"get_config", ""}, {"save", "s"}, {"load", "s"}, {"get_status", ""}, {"clear", ""},
        {"set_row", "sd"}, {"neighbor_row_from_id", "sk"}, {"neighbor_row_from_datum", "dk"},
        {"similar_row_from_id", "sk"}, {"similar_row_from_datum", "dk"}, {"get_all_rows", ""},
        {"do_mix", ""}};
    static const std::vector<std::pair<std::string, std::string>> an = {
        {"get_config", ""}, {"save", "s"}, {"load", "s"}, {"get_status", ""}, {"clear", ""},
        {"clear_row", "s"}, {"add", "d"}, {"update", "sd"}, {"overwrite", "sd"}, {"calc_score", "d"},
        {"get_all_rows", ""}, {"do_mix", ""}};
    static const std::vector<std::pair<std::string, std::string>> cl = {
        {"get_config", ""}, {"save", "s"}, {"load", "s"}, {"get_status", ""}, {"clear", ""},
        {"train", "l"}, {"classify", "l"}, {"get_labels", ""}, {"set_label", "s"}, {"delete_label", "s"},
        {"do_mix", ""}};
    const auto& table = kind_ == Kind::kRecommender ? rec
                        : kind_ == Kind::kNearestNeighbor ? nn
                        : kind_ == Kind::kAnomaly ? an : cl;
    const std::string* sig = nullptr;
    for (const auto& x : table)
      if (x.first == m) sig = &x.second;
    if (!sig || (m == "do_mix" && !mixer_))
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kNoMethodError);
    bool ok = args.a.size() == sig->size() + 1 && args.a[0].is_str();
    for (size_t k = 0; ok && k < sig->size(); ++k) {
      const Value& x = args.a[k + 1];
      const char c = (*sig)[k];
      // s: string, k: size, d / l: arrays
      ok = c == 's' ? x.is_str() : c == 'k' ? (x.kind == Value::INT || x.kind == Value::UINT) : x.kind == Value::ARR;
    }
    if (!ok) return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    auto size_arg = [&](size_t i) -> int64_t {
      const Value& x = args.a[i];
      return x.kind == Value::UINT ? (int64_t)std::min<uint64_t>(x.u, (uint64_t)INT64_MAX) : x.i;
    };
    MsgpackWriter w;
    // update calls drive the MIX trigger (event_model_updated)
    static const char* const kUpdates[] = {"clear", "clear_row", "update_row", "set_row", "add", "update",
                                           "overwrite", "load", "train", "set_label", "delete_label"};
    if (mixer_)
      for (const char* u : kUpdates)
        if (m == u && !(m == "add" && node_)) { mixer_->updated(1); break; }
    try {
      if (m == "get_config") {
        w.raw(model_->config_text());
      } else if (m == "do_mix") {
        w.boolean(mixer_->do_mix());
      } else if (m == "clear") {
        model_->clear();
        w.boolean(true);
      } else if (m == "clear_row") {
        w.boolean(model_->clear_row(args.a[1].s));
      } else if (m == "add") {
        const auto r = node_ ? add_zk(args.a[1]) : model_->add(args.a[1]);
        w.arr(2);
        w.raw(r.first);
        w.dbl(r.second);
      } else if (m == "update" || m == "overwrite") {
        w.dbl(model_->update(args.a[1].s, args.a[2], m == "update"));
      } else if (m == "calc_score") {
        w.dbl(model_->calc_score(args.a[1]));
      } else if (m == "update_row") {
        w.boolean(model_->update_row(args.a[1].s, args.a[2]));
      } else if (m == "set_row") {
        w.boolean(model_->set_row(args.a[1].s, args.a[2]));
      } else if (m == "similar_row_from_id") {
        write_pairs(w, model_->query_id(args.a[1].s, size_arg(2), true));
      } else if (m == "neighbor_row_from_id") {
        write_pairs(w, model_->query_id(args.a[1].s, size_arg(2), false));
      } else if (m == "similar_row_from_datum") {
        write_pairs(w, model_->query_datum(args.a[1], size_arg(2), true));
      } else if (m == "neighbor_row_from_datum") {
        write_pairs(w, model_->query_datum(args.a[1], size_arg(2), false));
      } else if (m == "complete_row_from_id") {
        jb::row::write_datum(w, model_->complete_row_from_id(args.a[1].s));
      } else if (m == "complete_row_from_datum") {
        jb::row::write_datum(w, model_->complete_row_from_datum(args.a[1]));
      } else if (m == "decode_row") {
        jb::row::write_datum(w, model_->decode_row(args.a[1].s));
      } else if (m == "train") {
        w.sint(model_->nn_train(args.a[1]));
      } else if (m == "classify") {
        const auto res = model_->nn_classify(args.a[1]);
        w.arr(res.size());
        for (const auto& r : res) write_pairs(w, r);
      } else if (m == "get_labels") {
        const auto ls = model_->nn_labels();
        w.map(ls.size());
        for (const auto& kv : ls) { w.raw(kv.first); w.uint(kv.second); }
      } else if (m == "set_label") {
        w.boolean(model_->nn_set_label(args.a[1].s));
      } else if (m == "delete_label") {
        w.boolean(model_->nn_delete_label(args.a[1].s));
      } else if (m == "get_all_rows") {
        const auto ids = model_->get_all_rows();
        w.arr(ids.size());
        for (const auto& s : ids) w.raw(s);
      } else if (m == "calc_similarity") {
        w.dbl(model_->calc_similarity(args.a[1], args.a[2]));
      } else if (m == "calc_l2norm") {
        w.dbl(model_->calc_l2norm(args.a[1]));
      } else if (m == "save") {
        const std::string& id = args.a[1].s;
        if (id.empty()) throw std::runtime_error("empty id is not allowed");
        const std::string path = local_path(id);
        write_model_file(path, type(), id, model_->config_text(), model_->pack_user_data());
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
          common_status(a_, cs_, model_->update_count.load(), &st);
        }
        model_->status(&st);
        if (mixer_) mixer_->status(&st);
        w.map(1);
        w.raw(ident());
        w.map(st.size());
        for (auto& kv : st) { w.raw(kv.first); w.raw(kv.second); }
      }
    } catch (const ArgError&) {
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    } catch (const std::exception& e) {
      return r.notify ? std::string() : jb::val::response_msg(r.msgid, e.what());
    }
    return r.notify ? std::string() : jb::val::response_ok(r.msgid, w.out);
  }

  // anomaly_serv.cpp:178-211 add_zk: a cluster-wide id, the CHT(2) owners of
  // it; the first owner's update must succeed, the replica is best effort
  std::pair<std::string, double> add_zk(const Value& dv) {
    Datum chk;
    jb::row::parse_datum(dv, &chk);
    const std::string id = std::to_string(node_->create_id());
    const auto owners = node_->cht_find(id, 2);
    if (owners.empty()) throw std::runtime_error("no server found in cht: " + a_.name);
    double score;
    try {
      score = selective_update(owners[0], id, dv);
    } catch (const std::exception& e) {
      throw std::runtime_error("failed to add ID " + id + " (" + e.what() + "): " + owners[0].first + ":" +
                               std::to_string(owners[0].second));
    }
    for (size_t i = 1; i < owners.size(); ++i) {
      try {
        selective_update(owners[i], id, dv);
      } catch (const std::exception& e) {
        logf_("WARN", "cannot create %zuth replica (%s): %s:%d", i, e.what(), owners[i].first.c_str(),
              owners[i].second);
      }
    }
    return {id, score};
  }
  // anomaly_serv.cpp:275-297: locally when this server owns the id, else a
  // server-to-server update RPC
  double selective_update(const std::pair<std::string, int>& owner, const std::string& id, const Value& dv) {
    if (owner.first == a_.eth && owner.second == a_.port) {
      if (mixer_) mixer_->updated(1);
      return model_->update(id, dv, true);
    }
    const double tmo = std::max(1, a_.ic_timeout);
    jb::cc::Conn c(owner.first, owner.second, tmo);
    MsgpackWriter w;
    w.arr(3);
    w.raw(a_.name);
    w.raw(id);
    Model::write_value(w, dv);
    const double dl = jb::cc::now_s() + tmo;
    const uint32_t mid = c.send_request("update", w.out, dl);
    jb::cc::CallResult res;
    c.recv_response(mid, dl, &res);
    if (!res.err.empty()) throw std::runtime_error("server-to-server update failed");
    return MsgpackReader((const uint8_t*)res.res.data(), res.res.size()).read().num();
  }

  std::string local_path(const std::string& id) const {
    return a_.datadir + "/" + a_.eth + "_" + std::to_string(a_.port) + "_" + type() + "_" + id + ".jubatus";
  }

  void load_impl(const std::string& path, bool overwrite_config) {
    std::string bytes;
    if (!read_file(path, &bytes)) throw std::runtime_error("cannot open input file: " + path + ": " + strerror(errno));
    ModelFile mf;
    const std::string err = read_model_file(bytes, &mf);
    if (!err.empty()) throw std::runtime_error(err);
    if (mf.type != type())
      throw std::runtime_error("invalid model type: saved type: " + mf.type + ", expected type: " + type());
    const std::string current = model_->config_text();
    if (!overwrite_config && !jb::val::same_config(mf.config, current))
      throw std::runtime_error("model config mismatched with the running config");
    if (mf.user_version != 1)
      throw std::runtime_error("user data version mismatched: " + std::to_string(mf.user_version) +
                               ", current version: 1");
    if (overwrite_config && !jb::val::same_config(mf.config, current)) {
      Config cfg;
      std::string why;
      if (!parse_config(kind_, mf.config, &cfg, &why))
        throw std::runtime_error("model config is not served natively: " + why);
      model_->configure(cfg);
    }
    model_->unpack(mf.user);
    std::lock_guard<std::mutex> g(st_mu_);
    cs_.last_loaded = time(nullptr);
    cs_.last_loaded_path = path;
    logf_("INFO", "loaded from %s", path.c_str());
  }

  Kind kind_;
  Args a_;
  std::unique_ptr<Model> model_;
  std::unique_ptr<jb::mix::ClusterNode> node_;
  std::unique_ptr<jb::mix::LinearMixer> mixer_;
  std::unique_ptr<jb::RpcServer> rpc_;
  std::mutex st_mu_;
  CommonStatus cs_;
};

// after startup(): serve (the process owns the GPU from here: no exec)
inline int row_serve(Kind kind, Args& a, const Config& cfg) {
  try {
    const int device = device_and_signals(a);
    logf_("INFO", "starting %s %s RPC server at %s:%d (native, device %d)", prog_name(), kVersion,
          a.eth.c_str(), a.port, device);
    Server srv(kind, a, cfg, device);
    if (!a.zookeeper.empty())
      srv.join_cluster(std::unique_ptr<jb::mix::ClusterNode>(
          new jb::mix::ClusterNode(a.zookeeper, std::max(1, a.zk_timeout), kind_name(kind), a.name)));
    if (!a.model_file.empty()) srv.load_file(a.model_file);
    return srv.run();
  } catch (const std::exception& e) {
    logf_("FATAL", "failed to start %s: %s", engine_name(), e.what());
    return 1;
  }
}

inline int row_main(int argc, char** argv, Kind kind) {
  set_engine(kind_name(kind));
  Args a;
  std::string text;
  Config cfg;
  const int rc = startup(argc, argv, &a, &text, [&cfg, kind](const std::string& t, std::string* why) {
    return parse_config(kind, t, &cfg, why);
  }, true, /*native_dist=*/true, /*native_push=*/true);
  if (rc >= 0) return rc;
  return row_serve(kind, a, cfg);
}

}  // namespace rowsrv
}  // namespace jb
