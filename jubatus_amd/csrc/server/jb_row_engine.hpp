// Native core of the row-oriented GPU engines (jubarecommender,
// jubanearest_neighbor; csrc/server): the C++ twin of models/rows.py
// (RowStore, lru Unlearner), models/similarity.py (LshIndex, the HBM
// InvertedIndex pool) and the parts of models/row_engine.py the servers
// call, driving the kernels of csrc/hip (lsh.hip signatures, topk.hip
// fused scan + exact top-k, sparse_pool.hip inverted-index pool) directly.
//
// Reference: the row engines' glue jubatus/server/server/
// recommender_serv.cpp:126-224 and nearest_neighbor_serv.cpp:121-178 over
// jubatus_core's column tables (EXTERNAL). Semantics follow the Python
// drivers call for call (tests/test_native_row_servers.py compares every
// answer), and model files interchange both ways (RowEngine.pack layout:
// {"method", "rows": {id: [version, [sv, nv, bv]]}, "weights"}).
//
// Converter: the fixed-slot host hasher (jb_hostfv.hpp) when the config is
// eligible for it, else the wide rule set (jb_hostfv_wide.hpp: ngram /
// space splitters, tf / idf / bm25 with document frequencies owned here,
// add / mul combinations) - the same choice as RowEngine._hasher. Stored
// rows are hashed from their datum with sorted keys (rows.py dicts_wire),
// queries from the datum as received.
#pragma once
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "jb_hostfv.hpp"
#include "jb_hostfv_wide.hpp"
#include "jb_row_mix.hpp"
#include "jb_server_common.hpp"
#include "jb_wide_rules.hpp"
#include "jb_value.hpp"

extern "C" {
int jb_signature(const int64_t* row_ptr, const int32_t* fidx, const float* fval, int n,
                 int hash_num, uint64_t seed, int mode, uint64_t* bits, float* norms,
                 hipStream_t stream);
int jb_hamming_scan(const uint64_t* qbits, const float* qnorm, int nq, const uint64_t* tbits,
                    const float* tnorm, const uint8_t* valid, int64_t nrows, int words,
                    int hash_num, int metric, float* out, hipStream_t stream);
int jb_lsh_query_direct(const int32_t* idx, const float* val, const int64_t* row_ptr, int nq,
                        int hash_num, uint64_t seed, int mode, int metric, const uint64_t* tbits,
                        const float* tnorm, const uint8_t* valid, int64_t nrows, int k,
                        uint64_t* qbits_scratch, float* qnorm_scratch, float* scratch_d,
                        int32_t* scratch_i, float* out_d_host, int32_t* out_i_host,
                        uint32_t* done_host, hipStream_t stream);
int jb_lsh_set_rows_direct(const int32_t* idx, const float* val, const int64_t* row_ptr, int n,
                           const int64_t* slots, int hash_num, uint64_t seed, int mode,
                           uint64_t* tbits, float* tnorm, uint8_t* valid, hipStream_t stream);
int jb_lsh_set_rows_staged(const int64_t* rp, const int64_t* slots, const int32_t* idx, const float* val, int n,
                           int hash_num, uint64_t seed, int mode, uint64_t* tbits, float* tnorm, uint8_t* valid,
                           hipStream_t stream);
int jb_topk_direct_query(const uint64_t* qbits, const float* qnorm, int nq, const uint64_t* tbits,
                         const float* tnorm, const uint8_t* valid, int64_t nrows, int words,
                         int hash_num, int metric, int k, float* scratch_d, int32_t* scratch_i,
                         float* out_d_host, int32_t* out_i_host, uint32_t* done_host,
                         hipStream_t stream);
int jb_topk_blocks(int64_t nrows, int k);
int64_t jb_topk_direct_scratch(int nq);
int jb_topk_scratch_init(int32_t* scratch_i, hipStream_t stream);
int jb_pool_scan(const int64_t* qptr, const int32_t* qidx, const float* qval, const double* qn2,
                 const int32_t* qslots, int nq, int qtot, const int64_t* r_off,
                 const int32_t* r_len, const double* r_n2, const uint8_t* valid, int64_t nrows,
                 const int32_t* p_idx, const float* p_val, int metric, int lpr, float* out,
                 hipStream_t stream);
int jb_pool_query_direct(const int32_t* idx, const float* val, const int64_t* row_ptr,
                         const int32_t* qslots, const int64_t* slot_len, int nq,
                         const int64_t* r_off, const int32_t* r_len, const double* r_n2,
                         const uint8_t* valid, int64_t nrows, const int32_t* p_idx,
                         const float* p_val, int metric, int lpr, int k, float* scores,
                         float* scratch_d, int32_t* scratch_i, float* out_d_host,
                         int32_t* out_i_host, uint32_t* done_host, hipStream_t stream);
int jb_pool_append(const uint8_t* pack, int n, int64_t nnz, int64_t base, int64_t* r_off,
                   int32_t* r_len, double* r_n2, uint8_t* valid, int32_t* p_idx, float* p_val,
                   hipStream_t stream);
void* jb_host_alloc(int64_t nbytes);
int jb_host_free(void* p);
}

namespace jb {
namespace row {

using jb::val::MsgpackReader;
using jb::val::MsgpackWriter;
using jb::val::Value;
using jb::srv::DevBuf;
using jb::srv::PinBuf;

constexpr int kTopMaxK = 128;        // csrc/hip/topk.hip kTopMaxK
constexpr int kQueryMax = 8;         // lsh.hip kQueryMax
constexpr int kQuerySlots = 256;     // lsh.hip kQuerySlots (direct paths)
constexpr int kPoolMaxQ = 8;          // sparse_pool.hip kPoolMaxQ (queries per pass)
constexpr int kPoolMaxQEntries = 4096;

// datum -> hashed feature vector; owns the document-frequency statistics of
// the idf / bm25 weights (fv_converter/converter.py WeightManager layout)
class Converter {
 public:
  bool configure(const Value& conv, std::string* why) {
    jb::srv::Rules r;
    std::string w1;
    if (jb::srv::build_rules(conv, &r, &w1)) {   // RowEngine._hasher: fixed-slot first
      fast_.reset(new HostFvHasher((const uint8_t*)r.s.data(), (int)r.s.size(),
                                   (const uint8_t*)r.n.data(), (int)r.n.size(),
                                   (const uint8_t*)r.blob.data(), r.blob.size(), r.H));
      H_ = r.H;
      global_ = false;
      return true;
    }
    std::vector<HostRule> s, n, c;
    std::string blob;
    uint64_t H = 1ull << 20;
    std::shared_ptr<WideExt> ext;
    if (!build_wide_rules(conv, &s, &n, &c, &blob, &H, &global_, why, &ext)) return false;
    H_ = H;
    wide_.reset(new HostFvWide((const uint8_t*)s.data(), (int)s.size(), (const uint8_t*)n.data(),
                               (int)n.size(), (const uint8_t*)c.data(), (int)c.size() / 2,
                               (const uint8_t*)blob.data(), blob.size(), H));
    wide_->set_ext(ext);
    if (wide_->needs_weights()) {
      df_.assign(H, 0);
      diff_.assign(H, 0);
      wide_->set_weights(df_.data(), diff_.data(), counts_);
    }
    return true;
  }

  uint64_t H() const { return H_; }
  bool global() const { return global_; }

  // one datum (msgpack bytes of the datum itself) -> (idx, val); idx < 0
  // entries kept as the hasher leaves them. update: count the document in
  // the idf / bm25 statistics (set / update of a stored row)
  void hash(const uint8_t* d, size_t n, std::vector<int32_t>* idx, std::vector<float>* val,
            bool update) {
    // the hashers take a list<datum> body: a one-element array header in front
    body_.assign(1, (char)0x91);
    body_.append((const char*)d, n);
    size_t cap = std::max<size_t>(256, n / 2 + 64);
    for (;;) {
      idx->resize(cap);
      val->resize(cap);
      int64_t rp[2] = {0, 0}, nn = 0, slots = 0;
      int rc;
      if (fast_) {
        rc = fast_->hash_body((const uint8_t*)body_.data(), body_.size(), idx->data(), val->data(), rp, 1,
                              (int64_t)cap, &nn, &slots);
      } else {
        wide_->begin();
        rc = wide_->hash_body((const uint8_t*)body_.data(), body_.size(), idx->data(), val->data(), rp, 1,
                              (int64_t)cap, &nn, &slots, update);
        if (rc != 0) wide_->rollback();
      }
      if (rc == 2) { cap *= 4; continue; }
      if (rc != 0 || nn != 1) throw ArgError("malformed datum");
      idx->resize((size_t)rp[1]);
      val->resize((size_t)rp[1]);
      return;
    }
  }

  // the fixed-slot hasher, which keeps no document statistics (null: this
  // converter keeps statistics). Immutable and shared: the RPC IO threads
  // hash write datums with it outside the model lock (Model::prep_write)
  std::shared_ptr<const HostFvHasher> stateless() const { return fast_; }
  // one datum's msgpack bytes -> (idx, val) with such a hasher
  static void hash_with(const HostFvHasher& h, const uint8_t* d, size_t n, std::vector<int32_t>* idx,
                        std::vector<float>* val) {
    std::string body(1, (char)0x91);
    body.append((const char*)d, n);
    size_t cap = std::max<size_t>(256, n / 2 + 64);
    for (;;) {
      idx->resize(cap);
      val->resize(cap);
      int64_t rp[2] = {0, 0}, nn = 0, slots = 0;
      const int rc = h.hash_body((const uint8_t*)body.data(), body.size(), idx->data(), val->data(), rp, 1,
                                 (int64_t)cap, &nn, &slots);
      if (rc == 2) { cap *= 4; continue; }
      if (rc != 0 || nn != 1) throw ArgError("malformed datum");
      idx->resize((size_t)rp[1]);
      val->resize((size_t)rp[1]);
      return;
    }
  }

  // document statistics of the MIX (WeightManager.get_diff / put_diff):
  // this server's contribution since the last MIX, then the cluster's sum
  // replaces it
  bool uses_weights() const { return !df_.empty(); }
  void get_diff(int64_t* docs, int64_t* len, std::vector<int64_t>* idx, std::vector<int64_t>* cnt) const {
    *docs = counts_[2];
    *len = counts_[3];
    idx->clear();
    cnt->clear();
    for (size_t i = 0; i < diff_.size(); ++i)
      if (diff_[i] != 0) { idx->push_back((int64_t)i); cnt->push_back(diff_[i]); }
  }
  // the sum of the members' diffs (this member's included) replaces its own
  // contribution. keep_own: one round of a push MIX - the own diff stays, so
  // the MIX's later partners get it too (each round adds just the partner's
  // counts; clear_diff() when the MIX ends). Under broadcast_mixer (every pair
  // once per MIX) every member ends with every member's counts exactly once;
  // random / skip mixers reach the MIX's partners only (the statistics carry
  // no versions to forward them without double counting).
  void put_diff(int64_t docs, int64_t len, const std::vector<int64_t>& idx, const std::vector<int64_t>& cnt,
                bool keep_own = false) {
    if (df_.empty()) return;
    counts_[0] += docs - counts_[2];
    counts_[1] += len - counts_[3];
    for (size_t i = 0; i < df_.size(); ++i) df_[i] -= diff_[i];
    for (size_t k = 0; k < idx.size() && k < cnt.size(); ++k)
      if (idx[k] >= 0 && (uint64_t)idx[k] < H_) df_[(size_t)idx[k]] += cnt[k];
    for (auto& x : df_) x = std::max<int64_t>(x, 0);
    if (keep_own) return;
    std::fill(diff_.begin(), diff_.end(), 0);
    counts_[2] = counts_[3] = 0;
  }
  void clear_diff() {
    if (df_.empty()) return;
    std::fill(diff_.begin(), diff_.end(), 0);
    counts_[2] = counts_[3] = 0;
  }

  void clear() {
    if (!df_.empty()) {
      std::fill(df_.begin(), df_.end(), 0);
      std::fill(diff_.begin(), diff_.end(), 0);
    }
    memset(counts_, 0, sizeof counts_);
  }

  // WeightManager.pack(): [doc_count, total_len, {"idx": [...], "df": [...]}]
  void pack(MsgpackWriter& w) const {
    w.arr(3);
    w.sint(counts_[0]);
    w.sint(counts_[1]);
    w.map(2);
    std::vector<int64_t> nz;
    for (size_t i = 0; i < df_.size(); ++i)
      if (df_[i] != 0) nz.push_back((int64_t)i);
    w.str("idx");
    w.arr(nz.size());
    for (int64_t i : nz) w.sint(i);
    w.str("df");
    w.arr(nz.size());
    for (int64_t i : nz) w.sint(df_[i]);
  }

  void unpack(const Value& v) {
    clear();
    if (v.kind != Value::ARR || v.a.size() != 3) throw std::runtime_error("broken model data: weights");
    counts_[0] = (int64_t)v.a[0].num();
    counts_[1] = (int64_t)v.a[1].num();
    const Value* ix = v.a[2].get("idx");
    const Value* df = v.a[2].get("df");
    if (!ix || !df || ix->kind != Value::ARR || df->kind != Value::ARR || ix->a.size() != df->a.size())
      throw std::runtime_error("broken model data: weights table");
    if (ix->a.empty()) return;
    if (df_.empty()) throw std::runtime_error("model carries document frequencies the converter does not use");
    for (size_t k = 0; k < ix->a.size(); ++k) {
      const int64_t i = (int64_t)ix->a[k].num();
      if (i < 0 || (uint64_t)i >= H_) throw std::runtime_error("broken model data: weights index");
      df_[i] += (int64_t)df->a[k].num();
    }
  }

 private:
  std::shared_ptr<HostFvHasher> fast_;
  std::unique_ptr<HostFvWide> wide_;
  std::vector<int64_t> df_, diff_;
  int64_t counts_[4] = {0, 0, 0, 0};
  uint64_t H_ = 1ull << 20;
  bool global_ = false;
  std::string body_;
};

// ------------------------------------------------------------ result views
struct Hit {
  int32_t slot;
  float dist;
};

// pinned outputs + device scratch of the latency paths (ops/hip.py
// DirectQueryBuffers / _topk_scratch)
struct QueryBufs {
  float* out_d = nullptr;
  int32_t* out_i = nullptr;
  uint32_t* done = nullptr;
  DevBuf<uint64_t> qbits;
  DevBuf<float> qnorm;
  DevBuf<float> sd;
  DevBuf<int32_t> si;
  DevBuf<float> scores;
  void init() {
    out_d = (float*)jb_host_alloc((int64_t)kQueryMax * kTopMaxK * 4);
    out_i = (int32_t*)jb_host_alloc((int64_t)kQueryMax * kTopMaxK * 4);
    done = (uint32_t*)jb_host_alloc(kQueryMax * 4);
    if (!out_d || !out_i || !done) throw std::runtime_error("hipHostMalloc failed");
    memset(done, 0, kQueryMax * 4);
  }
  void scratch(int64_t nrows, int k, int nq) {
    const int64_t a = (int64_t)nq * jb_topk_blocks(nrows, k) * k;
    const int64_t b = jb_topk_direct_scratch(nq);
    const size_t n = (size_t)std::max<int64_t>(std::max(a, b), 1 << 16);
    sd.get(n);
    int32_t* before = si.p;
    si.get(n);
    // the one-launch score top-k expects its state region zeroed
    if (si.p != before && jb_topk_scratch_init(si.p, nullptr) != 0)
      throw std::runtime_error("jb_topk_scratch_init failed");
  }
};

// hits of the latency path -> ascending list, stopping at the first
// non-finite distance (similarity.py _pairs)
inline std::vector<Hit> direct_hits(const QueryBufs& b, int q, int k) {
  std::vector<Hit> out;
  for (int j = 0; j < k; ++j) {
    const float d = b.out_d[q * k + j];
    if (!std::isfinite(d)) break;
    out.push_back({b.out_i[q * k + j], d});
  }
  return out;
}

// exact top-k of a full host distance vector (k beyond the fused kernel)
inline std::vector<Hit> host_topk(const std::vector<float>& d, int k) {
  std::vector<Hit> all;
  for (size_t i = 0; i < d.size(); ++i)
    if (std::isfinite(d[i])) all.push_back({(int32_t)i, d[i]});
  std::stable_sort(all.begin(), all.end(), [](const Hit& a, const Hit& b) { return a.dist < b.dist; });
  if ((int)all.size() > k) all.resize((size_t)k);
  return all;
}

// ------------------------------------------------------------- LSH index
// similarity.py LshIndex: signatures (bits [cap][words]), norms, valid in HBM
class LshIndex {
 public:
  LshIndex(const std::string& method, int hash_num, uint64_t seed, hipStream_t st)
      : hash_num_(hash_num), seed_(seed), stream_(st) {
    metric_ = method == "lsh" ? 0 : method == "euclid_lsh" ? 1 : 2;
    mode_ = method == "minhash" ? 1 : 0;
    words_ = (hash_num + 63) / 64;
    bufs_.init();
    alloc(1024);
    for (auto& e : stage_ev_) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  ~LshIndex() {
    for (auto& e : stage_ev_)
      if (e != nullptr) (void)hipEventDestroy(e);
  }
  LshIndex(const LshIndex&) = delete;
  LshIndex& operator=(const LshIndex&) = delete;
  int metric() const { return metric_; }

  void clear() {
    pend_slot_.clear();
    pend_rp_.assign(1, 0);
    pend_idx_.clear();
    pend_val_.clear();
    cap_ = 0;
    bits_.p = nullptr; bits_.cap = 0;
    alloc(1024);
  }

  // batched writes (the row server's write batches): rows set while deferred
  // are kept on the host and written by one staged launch in flush(); every
  // other access flushes first, so nothing observes the deferral
  void set_defer(bool on) {
    if (!on) flush();
    defer_ = on;
  }
  void flush() {
    if (pend_slot_.empty()) return;
    // the last write of a slot wins (rows of one launch must be distinct)
    std::unordered_map<int32_t, size_t> last;
    for (size_t i = 0; i < pend_slot_.size(); ++i) last[pend_slot_[i]] = i;
    std::vector<size_t> keep;
    for (size_t i = 0; i < pend_slot_.size(); ++i)
      if (last[pend_slot_[i]] == i) keep.push_back(i);
    const size_t n = keep.size();
    size_t nnz = 0;
    for (size_t i : keep) nnz += pend_rp_[i + 1] - pend_rp_[i];
    const size_t bytes = 8 * (2 * n + 1) + 8 * nnz + 16;
    // a ring of staging buffers: a batch's launch runs while the RPC answers
    // go out and the next batch stages (a stream sync per batch waited for
    // each launch on the write path); a buffer is reused once its launch ended
    const int k = stage_next_;
    stage_next_ = (stage_next_ + 1) % kStageRing;
    if (stage_used_[k]) HIPCHK(hipEventSynchronize(stage_ev_[k]));
    uint8_t* h = stage_host_[k].get(bytes);
    int64_t* rp = (int64_t*)h;
    int64_t* sl = rp + n + 1;
    int32_t* ix = (int32_t*)(sl + n);
    float* vx = (float*)(ix + nnz);
    rp[0] = 0;
    size_t o = 0;
    for (size_t q = 0; q < n; ++q) {
      const size_t i = keep[q];
      const size_t b = pend_rp_[i], e = pend_rp_[i + 1];
      memcpy(ix + o, pend_idx_.data() + b, 4 * (e - b));
      memcpy(vx + o, pend_val_.data() + b, 4 * (e - b));
      o += e - b;
      rp[q + 1] = (int64_t)o;
      sl[q] = pend_slot_[i];
    }
    uint8_t* d = stage_dev_[k].get(bytes);
    HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream_));
    const int64_t* drp = (const int64_t*)d;
    const int rc = jb_lsh_set_rows_staged(drp, drp + n + 1, (const int32_t*)(drp + 2 * n + 1),
                                          (const float*)((const int32_t*)(drp + 2 * n + 1) + nnz), (int)n, hash_num_,
                                          seed_, mode_, (uint64_t*)bits_.p, norms_.p, valid_.p, stream_);
    if (rc != 0) throw std::runtime_error("lsh staged set failed: " + std::to_string(rc));
    HIPCHK(hipEventRecord(stage_ev_[k], stream_));   // (later work on stream_ sees the rows)
    stage_used_[k] = true;
    pend_slot_.clear();
    pend_rp_.assign(1, 0);
    pend_idx_.clear();
    pend_val_.clear();
    ++flushes_;
  }
  uint64_t flushes() const { return flushes_; }

  void set(int32_t slot, const std::vector<int32_t>& idx, const std::vector<float>& val) {
    grow(slot + 1);
    if (defer_) {
      pend_slot_.push_back(slot);
      pend_idx_.insert(pend_idx_.end(), idx.begin(), idx.end());
      pend_val_.insert(pend_val_.end(), val.begin(), val.end());
      pend_rp_.push_back(pend_idx_.size());
      if (pend_slot_.size() >= 4096) flush();
      return;
    }
    const int64_t rp[2] = {0, (int64_t)idx.size()};
    const int64_t sl = slot;
    int rc = jb_lsh_set_rows_direct(idx.data(), val.data(), rp, 1, &sl, hash_num_, seed_, mode_,
                                    (uint64_t*)bits_.p, norms_.p, valid_.p, stream_);
    if (rc == 1) {        // wider than the kernel arguments: one staged launch
      upload_csr(idx, val);
      rc = jb_signature(d_rp_.p, d_idx_.p, d_val_.p, 1, hash_num_, seed_, mode_,
                        (uint64_t*)bits_.p + (size_t)slot * words_, norms_.p + slot, stream_);
      if (rc == 0) HIPCHK(hipMemsetAsync(valid_.p + slot, 1, 1, stream_));
      HIPCHK(hipStreamSynchronize(stream_));   // the staging buffers are reused
    }
    if (rc != 0) throw std::runtime_error("lsh signature launch failed: " + std::to_string(rc));
  }

  void remove(int32_t slot) {
    flush();
    if (slot < cap_) HIPCHK(hipMemsetAsync(valid_.p + slot, 0, 1, stream_));
  }

  // k nearest rows of a hashed feature vector (ascending distance)
  std::vector<Hit> query_fv(const std::vector<int32_t>& idx, const std::vector<float>& val,
                            int64_t nrows, int k) {
    flush();
    if (nrows <= 0 || k <= 0) return {};
    if (k <= kTopMaxK) {
      bufs_.scratch(nrows, k, 1);
      const int64_t rp[2] = {0, (int64_t)idx.size()};
      const int rc = jb_lsh_query_direct(idx.data(), val.data(), rp, 1, hash_num_, seed_, mode_, metric_,
                                         (const uint64_t*)bits_.p, norms_.p, valid_.p, nrows, k,
                                         q_bits(), q_norm(), bufs_.sd.p, bufs_.si.p, bufs_.out_d,
                                         bufs_.out_i, bufs_.done, stream_);
      if (rc == 0) return direct_hits(bufs_, 0, k);
      if (rc != 1) throw std::runtime_error("lsh query failed: " + std::to_string(rc));
    }
    // wide query or large k: device signature, then the top-k
    upload_csr(idx, val);
    const int rc = jb_signature(d_rp_.p, d_idx_.p, d_val_.p, 1, hash_num_, seed_, mode_, q_bits(),
                                q_norm(), stream_);
    if (rc != 0) throw std::runtime_error("lsh signature launch failed: " + std::to_string(rc));
    return query_sig(q_bits(), q_norm(), nrows, k);
  }

  // up to kQueryMax hashed vectors in ONE launch sequence (signatures, the
  // fused scan + top-k of every query in one pass over the table); false
  // when they do not fit the kernel arguments (the caller goes one by one)
  bool query_fv_many(const std::vector<const std::vector<int32_t>*>& idx,
                     const std::vector<const std::vector<float>*>& val, int64_t nrows, int k,
                     std::vector<std::vector<Hit>>* out) {
    flush();
    const int nq = (int)idx.size();
    if (nq <= 0 || nq > kQueryMax || nrows <= 0 || k <= 0 || k > kTopMaxK) return false;
    std::vector<int64_t> rp(1, 0);
    std::vector<int32_t> ci;
    std::vector<float> cv;
    for (int q = 0; q < nq; ++q) {
      ci.insert(ci.end(), idx[q]->begin(), idx[q]->end());
      cv.insert(cv.end(), val[q]->begin(), val[q]->end());
      rp.push_back((int64_t)ci.size());
    }
    if ((int64_t)ci.size() > kQuerySlots) return false;
    bufs_.scratch(nrows, k, nq);
    const int rc = jb_lsh_query_direct(ci.data(), cv.data(), rp.data(), nq, hash_num_, seed_, mode_, metric_,
                                       (const uint64_t*)bits_.p, norms_.p, valid_.p, nrows, k, q_bits(), q_norm(),
                                       bufs_.sd.p, bufs_.si.p, bufs_.out_d, bufs_.out_i, bufs_.done, stream_);
    if (rc == 1) return false;
    if (rc != 0) throw std::runtime_error("lsh query failed: " + std::to_string(rc));
    out->resize((size_t)nq);
    for (int q = 0; q < nq; ++q) (*out)[(size_t)q] = direct_hits(bufs_, q, k);
    return true;
  }

  std::vector<Hit> query_slot(int32_t slot, int64_t nrows, int k) {
    flush();
    if (nrows <= 0 || k <= 0) return {};
    return query_sig((const uint64_t*)bits_.p + (size_t)slot * words_, norms_.p + slot, nrows, k);
  }

  // distance -> similarity as similar_row_* reports it (float arithmetic,
  // as the Python path: 1 - d for lsh / minhash, -d for euclid_lsh)
  double similarity(float d) const { return metric_ == 1 ? (double)(-d) : (double)(1.0f - d); }

  // models/recommender.py calc_similarity over host signatures
  // (similarity.py signature_host: float32 products summed in row order)
  double calc_similarity(const std::vector<int32_t>& ai, const std::vector<float>& av,
                         const std::vector<int32_t>& bi, const std::vector<float>& bv) const {
    std::vector<uint64_t> ba, bb;
    const double na = host_signature(ai, av, &ba), nb = host_signature(bi, bv, &bb);
    int ham = 0;
    for (int w = 0; w < words_; ++w) ham += __builtin_popcountll(ba[w] ^ bb[w]);
    const double frac = (double)ham / hash_num_;
    if (metric_ == 1) return -sqrt(std::max(0.0, na * na + nb * nb - 2 * na * nb * cos(M_PI * frac)));
    return 1.0 - frac;
  }

  // model files: signatures are recomputed from the stored rows on load
 private:
  static uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
  }
  static float gauss(uint64_t h) {
    const double u1 = ((double)(h >> 40) + 1.0) / 16777217.0;
    const double u2 = (double)(h & 0xFFFFFF) / 16777216.0;
    return (float)(sqrt(-2.0 * log(u1)) * cos(6.2831853 * u2));
  }
  double host_signature(const std::vector<int32_t>& idx, const std::vector<float>& val,
                        std::vector<uint64_t>* out) const {
    const int B = words_ * 64;
    std::vector<uint8_t> bit(B, 0);
    std::vector<int32_t> fi;
    std::vector<float> fv;
    for (size_t i = 0; i < idx.size(); ++i)
      if (idx[i] >= 0) { fi.push_back(idx[i]); fv.push_back(val[i]); }
    double n2 = 0.0;
    for (float v : fv) n2 += (double)v * (double)v;
    if (!fi.empty()) {
      if (mode_ == 0) {
        for (int j = 0; j < B; ++j) {
          float acc = 0.f;
          for (size_t i = 0; i < fi.size(); ++i) {
            const uint64_t h = splitmix(seed_ ^ splitmix(((uint64_t)(uint32_t)fi[i] << 20) ^ (uint64_t)j));
            acc += fv[i] * gauss(h);
          }
          bit[j] = acc > 0.f;
        }
      } else {
        bool any = false;
        for (float v : fv) any |= v != 0.f;
        for (int j = 0; j < B; ++j) {
          if (!any) { bit[j] = 1; continue; }
          uint64_t mn = ~0ull;
          for (size_t i = 0; i < fi.size(); ++i) {
            if (fv[i] == 0.f) continue;
            const uint64_t h = splitmix(seed_ ^ splitmix(((uint64_t)(uint32_t)fi[i] << 20) ^ (uint64_t)j));
            mn = std::min(mn, h);
          }
          bit[j] = (mn & 1) != 0;
        }
      }
    }
    out->assign(words_, 0);
    for (int j = 0; j < hash_num_; ++j)
      if (bit[j]) (*out)[j / 64] |= 1ull << (j % 64);
    return sqrt(n2);
  }

  uint64_t* q_bits() { return bufs_.qbits.get((size_t)kQueryMax * words_); }
  float* q_norm() { return bufs_.qnorm.get(kQueryMax); }

  std::vector<Hit> query_sig(const uint64_t* qb, const float* qn, int64_t nrows, int k) {
    if (k <= kTopMaxK && words_ <= 16) {
      bufs_.scratch(nrows, k, 1);
      const int rc = jb_topk_direct_query(qb, qn, 1, (const uint64_t*)bits_.p, norms_.p, valid_.p, nrows,
                                          words_, hash_num_, metric_, k, bufs_.sd.p, bufs_.si.p,
                                          bufs_.out_d, bufs_.out_i, bufs_.done, stream_);
      if (rc != 0) throw std::runtime_error("lsh top-k failed: " + std::to_string(rc));
      return direct_hits(bufs_, 0, k);
    }
    float* out = bufs_.scores.get((size_t)nrows);
    const int rc = jb_hamming_scan(qb, qn, 1, (const uint64_t*)bits_.p, norms_.p, valid_.p, nrows, words_,
                                   hash_num_, metric_, out, stream_);
    if (rc != 0) throw std::runtime_error("lsh scan failed: " + std::to_string(rc));
    std::vector<float> h((size_t)nrows);
    HIPCHK(hipMemcpyAsync(h.data(), out, 4 * (size_t)nrows, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    return host_topk(h, k);
  }

  void upload_csr(const std::vector<int32_t>& idx, const std::vector<float>& val) {
    const size_t n = std::max<size_t>(idx.size(), 1);
    const int64_t rp[2] = {0, (int64_t)idx.size()};
    HIPCHK(hipMemcpyAsync(d_rp_.get(2), rp, sizeof rp, hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_idx_.get(n), idx.data(), 4 * idx.size(), hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_val_.get(n), val.data(), 4 * val.size(), hipMemcpyHostToDevice, stream_));
    HIPCHK(hipStreamSynchronize(stream_));   // pageable sources
  }

  void alloc(int64_t cap) {
    DevBuf<uint64_t> b;
    DevBuf<float> nm;
    DevBuf<uint8_t> v;
    b.get((size_t)cap * words_);
    nm.get((size_t)cap);
    v.get((size_t)cap);
    HIPCHK(hipMemsetAsync(b.p, 0, (size_t)cap * words_ * 8, stream_));
    HIPCHK(hipMemsetAsync(nm.p, 0, (size_t)cap * 4, stream_));
    HIPCHK(hipMemsetAsync(v.p, 0, (size_t)cap, stream_));
    if (cap_) {
      HIPCHK(hipMemcpyAsync(b.p, bits_.p, (size_t)cap_ * words_ * 8, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(nm.p, norms_.p, (size_t)cap_ * 4, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(v.p, valid_.p, (size_t)cap_, hipMemcpyDeviceToDevice, stream_));
    }
    HIPCHK(hipStreamSynchronize(stream_));
    if (bits_.p) HIPCHK(hipFree(bits_.p));
    if (norms_.p) HIPCHK(hipFree(norms_.p));
    if (valid_.p) HIPCHK(hipFree(valid_.p));
    bits_ = b; norms_ = nm; valid_ = v;
    cap_ = cap;
  }
  void grow(int64_t need) {
    if (need <= cap_) return;
    int64_t c = cap_ ? cap_ : 1024;
    while (c < need) c *= 2;
    alloc(c);
  }

  int hash_num_, words_, metric_, mode_;
  uint64_t seed_;
  hipStream_t stream_;
  int64_t cap_ = 0;
  DevBuf<uint64_t> bits_;
  DevBuf<float> norms_;
  DevBuf<uint8_t> valid_;
  DevBuf<int64_t> d_rp_;
  DevBuf<int32_t> d_idx_;
  DevBuf<float> d_val_;
  QueryBufs bufs_;
  // deferred writes (set_defer)
  bool defer_ = false;
  std::vector<int32_t> pend_slot_;
  std::vector<size_t> pend_rp_{0};
  std::vector<int32_t> pend_idx_;
  std::vector<float> pend_val_;
  static constexpr int kStageRing = 4;
  PinBuf<uint8_t> stage_host_[kStageRing];
  DevBuf<uint8_t> stage_dev_[kStageRing];
  hipEvent_t stage_ev_[kStageRing] = {};
  bool stage_used_[kStageRing] = {};
  int stage_next_ = 0;
  uint64_t flushes_ = 0;
};

// ------------------------------------------------------- inverted index
// similarity.py InvertedIndex on the device (DevicePool): append-only runs
// of (feature, value) per slot + per-slot offset / length / squared norm /
// valid; exact cosine (metric 0) or euclidean distance (metric 1)
class PoolIndex {
 public:
  PoolIndex(bool euclid, hipStream_t st) : euclid_(euclid), stream_(st) {
    bufs_.init();
    reset();
  }
  int metric() const { return euclid_ ? 1 : 0; }

  void clear() {
    pend_meta_.clear();
    pend_idx_.clear();
    pend_val_.clear();
    reset();
  }

  // batched writes (the row server's write batches): the runs of rows set
  // while deferred are appended on the host (their pool offsets are taken at
  // once) and go to the device in one staged jb_pool_append in flush(); every
  // read of the pool flushes first
  void set_defer(bool on) {
    if (!on) flush();
    defer_ = on;
  }
  void flush() {
    if (pend_meta_.empty()) return;
    // the last write of a slot wins (one launch writes each slot's row once);
    // the runs of earlier writes stay in the pool as dead entries
    const size_t nw = pend_meta_.size() / 4;
    std::unordered_map<int64_t, size_t> last;
    for (size_t i = 0; i < nw; ++i) last[pend_meta_[4 * i]] = i;
    std::vector<int64_t> meta;
    meta.reserve(4 * last.size());
    for (size_t i = 0; i < nw; ++i)
      if (last[pend_meta_[4 * i]] == i)
        meta.insert(meta.end(), pend_meta_.begin() + 4 * i, pend_meta_.begin() + 4 * i + 4);
    const int n = (int)(meta.size() / 4);
    const int64_t nnz = (int64_t)pend_idx_.size();
    stage_append(meta.data(), n, pend_idx_.data(), pend_val_.data(), nnz, pend_base_);
    pend_meta_.clear();
    pend_idx_.clear();
    pend_val_.clear();
  }

  // csr_normalize of one row + jb_pool_append (latency path: pinned staging)
  void set(int32_t slot, const std::vector<int32_t>& idx, const std::vector<float>& val) {
    std::vector<std::pair<int32_t, int>> ord;
    for (size_t i = 0; i < idx.size(); ++i)
      if (idx[i] >= 0) ord.push_back({idx[i], (int)i});
    std::stable_sort(ord.begin(), ord.end(), [](const std::pair<int32_t, int>& a, const std::pair<int32_t, int>& b) {
      return a.first < b.first;
    });
    std::vector<int32_t> ni;
    std::vector<float> nv;
    double sq = 0.0;
    for (size_t k = 0; k < ord.size();) {
      const int32_t f = ord[k].first;
      double acc = 0.0;
      while (k < ord.size() && ord[k].first == f) acc += (double)val[ord[k++].second];
      const float v32 = (float)acc;
      ni.push_back(f);
      nv.push_back(v32);
      sq += (double)v32 * (double)v32;
    }
    const int64_t nnz = (int64_t)ni.size();
    grow_rows(slot + 1);
    if (end_ + nnz > cap_entries_ && end_ - live_ > live_) {
      flush();   // the compaction reads the pool back
      compact();
    }
    grow_entries(end_ + nnz);
    // meta: [slot, len, n2 bits, run offset from the launch's base]
    int64_t meta[4] = {slot, nnz, 0, 0};
    memcpy(&meta[2], &sq, 8);
    if (defer_) {
      if (pend_meta_.empty()) pend_base_ = end_;
      meta[3] = end_ - pend_base_;
      pend_meta_.insert(pend_meta_.end(), meta, meta + 4);
      pend_idx_.insert(pend_idx_.end(), ni.begin(), ni.end());
      pend_val_.insert(pend_val_.end(), nv.begin(), nv.end());
    } else {
      stage_append(meta, 1, ni.data(), nv.data(), nnz, end_);
    }
    live_ += nnz - len_h_[slot];
    if (!has_h_[slot]) { ++nlive_; has_h_[slot] = 1; }
    off_h_[slot] = end_;
    len_h_[slot] = nnz;
    end_ += nnz;
    if (defer_ && pend_meta_.size() >= 4 * 4096) flush();
  }

  void remove(int32_t slot) {
    flush();
    if (slot < 0 || slot >= cap_rows_) return;
    live_ -= len_h_[slot];
    if (has_h_[slot]) { --nlive_; has_h_[slot] = 0; }
    len_h_[slot] = 0;
    HIPCHK(hipMemsetAsync(valid_.p + slot, 0, 1, stream_));
  }

  std::vector<Hit> query_fv(const std::vector<int32_t>& idx, const std::vector<float>& val,
                            int64_t nrows, int k) {
    flush();
    if (nrows <= 0 || k <= 0) return {};
    if (k <= kTopMaxK) {
      bufs_.scratch(nrows, k, 1);
      const int64_t rp[2] = {0, (int64_t)idx.size()};
      const int rc = jb_pool_query_direct(idx.data(), val.data(), rp, nullptr, nullptr, 1, r_off_.p,
                                          r_len_.p, r_n2_.p, valid_.p, nrows, p_idx_.p, p_val_.p,
                                          metric(), lanes_per_row(1), k, bufs_.scores.get((size_t)nrows),
                                          bufs_.sd.p, bufs_.si.p, bufs_.out_d, bufs_.out_i, bufs_.done,
                                          stream_);
      if (rc == 0) return direct_hits(bufs_, 0, k);
      if (rc != 1) throw std::runtime_error("pool query failed: " + std::to_string(rc));
    }
    // a query wider than the kernel arguments / k beyond the fused top-k
    std::vector<std::pair<int32_t, int>> ord;
    for (size_t i = 0; i < idx.size(); ++i)
      if (idx[i] >= 0) ord.push_back({idx[i], (int)i});
    std::stable_sort(ord.begin(), ord.end(), [](const std::pair<int32_t, int>& a, const std::pair<int32_t, int>& b) {
      return a.first < b.first;
    });
    std::vector<int32_t> qi;
    std::vector<float> qv;
    double q2 = 0.0;
    for (size_t k2 = 0; k2 < ord.size();) {
      const int32_t f = ord[k2].first;
      double acc = 0.0;
      while (k2 < ord.size() && ord[k2].first == f) acc += (double)val[ord[k2++].second];
      qi.push_back(f);
      qv.push_back((float)acc);
      q2 += (double)(float)acc * (double)(float)acc;
    }
    if ((int64_t)qi.size() > kPoolMaxQEntries) throw std::runtime_error("query has more than 4096 features");
    const int64_t qptr[2] = {0, (int64_t)qi.size()};
    const size_t qn = std::max<size_t>(qi.size(), 1);
    HIPCHK(hipMemcpyAsync(d_qptr_.get(2), qptr, sizeof qptr, hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_qidx_.get(qn), qi.data(), 4 * qi.size(), hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_qval_.get(qn), qv.data(), 4 * qv.size(), hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(d_qn2_.get(1), &q2, 8, hipMemcpyHostToDevice, stream_));
    float* out = bufs_.scores.get((size_t)nrows);
    int rc = jb_pool_scan(d_qptr_.p, d_qidx_.p, d_qval_.p, d_qn2_.p, nullptr, 1, (int)qi.size(), r_off_.p,
                          r_len_.p, r_n2_.p, valid_.p, nrows, p_idx_.p, p_val_.p, metric(), lanes_per_row(1),
                          out, stream_);
    if (rc != 0) throw std::runtime_error("pool scan failed: " + std::to_string(rc));
    return scores_topk(out, nrows, k);
  }

  // up to kPoolMaxQ hashed vectors scored in ONE pass over the pool
  // (pool_rows_kernel), each with its own fused top-k; false when they do
  // not fit the kernel arguments (the caller goes one by one)
  bool query_fv_many(const std::vector<const std::vector<int32_t>*>& idx,
                     const std::vector<const std::vector<float>*>& val, int64_t nrows, int k,
                     std::vector<std::vector<Hit>>* out) {
    flush();
    const int nq = (int)idx.size();
    if (nq <= 0 || nq > kPoolMaxQ || nrows <= 0 || k <= 0 || k > kTopMaxK) return false;
    std::vector<int64_t> rp(1, 0);
    std::vector<int32_t> ci;
    std::vector<float> cv;
    for (int q = 0; q < nq; ++q) {
      ci.insert(ci.end(), idx[q]->begin(), idx[q]->end());
      cv.insert(cv.end(), val[q]->begin(), val[q]->end());
      rp.push_back((int64_t)ci.size());
    }
    bufs_.scratch(nrows, k, nq);
    const int rc = jb_pool_query_direct(ci.data(), cv.data(), rp.data(), nullptr, nullptr, nq, r_off_.p,
                                        r_len_.p, r_n2_.p, valid_.p, nrows, p_idx_.p, p_val_.p, metric(),
                                        lanes_per_row(nq), k, bufs_.scores.get((size_t)nrows * nq), bufs_.sd.p,
                                        bufs_.si.p, bufs_.out_d, bufs_.out_i, bufs_.done, stream_);
    if (rc == 1) return false;
    if (rc != 0) throw std::runtime_error("pool query failed: " + std::to_string(rc));
    out->resize((size_t)nq);
    for (int q = 0; q < nq; ++q) (*out)[(size_t)q] = direct_hits(bufs_, q, k);
    return true;
  }

  std::vector<Hit> query_slot(int32_t slot, int64_t nrows, int k) {
    flush();
    if (nrows <= 0 || k <= 0) return {};
    if (k <= kTopMaxK && len_h_[slot] <= kPoolMaxQEntries) {
      bufs_.scratch(nrows, k, 1);
      const int64_t sl = len_h_[slot];
      const int rc = jb_pool_query_direct(nullptr, nullptr, nullptr, &slot, &sl, 1, r_off_.p, r_len_.p,
                                          r_n2_.p, valid_.p, nrows, p_idx_.p, p_val_.p, metric(),
                                          lanes_per_row(1), k, bufs_.scores.get((size_t)nrows), bufs_.sd.p,
                                          bufs_.si.p, bufs_.out_d, bufs_.out_i, bufs_.done, stream_);
      if (rc == 0) return direct_hits(bufs_, 0, k);
      if (rc != 1) throw std::runtime_error("pool query failed: " + std::to_string(rc));
    }
    if (len_h_[slot] > kPoolMaxQEntries) throw std::runtime_error("query batch has more than 4096 features");
    HIPCHK(hipMemcpyAsync(d_qslot_.get(1), &slot, 4, hipMemcpyHostToDevice, stream_));
    float* out = bufs_.scores.get((size_t)nrows);
    int rc = jb_pool_scan(nullptr, nullptr, nullptr, nullptr, d_qslot_.p, 1, (int)len_h_[slot], r_off_.p,
                          r_len_.p, r_n2_.p, valid_.p, nrows, p_idx_.p, p_val_.p, metric(), lanes_per_row(1),
                          out, stream_);
    if (rc != 0) throw std::runtime_error("pool scan failed: " + std::to_string(rc));
    return scores_topk(out, nrows, k);
  }

  // similarity.py InvertedIndex._direct_pairs: double arithmetic
  double similarity(float d) const { return euclid_ ? -(double)d : 1.0 - (double)d; }

 private:
  static constexpr int kStages = 4;
  struct Stage {
    jb::srv::PinBuf<uint8_t> host;
    DevBuf<uint8_t> dev;
    hipEvent_t ev;
    bool used = false;
  };

  // n rows' meta + their runs (nnz entries from pool offset base) through
  // a pinned staging buffer of the ring, one jb_pool_append launch
  void stage_append(const int64_t* meta, int n, const int32_t* ni, const float* nv, int64_t nnz, int64_t base) {
    // pack: [slot, len, n2 bits, run] int64 x n | idx int32 | val f32
    const size_t bytes = 32 * (size_t)n + 8 * (size_t)nnz;
    Stage& s = stage_[turn_];
    turn_ = (turn_ + 1) % kStages;
    if (s.used) HIPCHK(hipEventSynchronize(s.ev));
    uint8_t* p = s.host.get(bytes);
    memcpy(p, meta, 32 * (size_t)n);
    if (nnz) {
      memcpy(p + 32 * (size_t)n, ni, 4 * (size_t)nnz);
      memcpy(p + 32 * (size_t)n + 4 * (size_t)nnz, nv, 4 * (size_t)nnz);
    }
    uint8_t* d = s.dev.get(bytes);
    HIPCHK(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, stream_));
    const int rc = jb_pool_append(d, n, nnz, base, r_off_.p, r_len_.p, r_n2_.p, valid_.p, p_idx_.p, p_val_.p,
                                  stream_);
    if (rc != 0) throw std::runtime_error("pool append failed: " + std::to_string(rc));
    HIPCHK(hipEventRecord(s.ev, stream_));
    s.used = true;
  }

  // scores (cosine similarity / euclidean distance) -> k smallest distances
  std::vector<Hit> scores_topk(const float* scores, int64_t nrows, int k) {
    std::vector<float> h((size_t)nrows);
    HIPCHK(hipMemcpyAsync(h.data(), scores, 4 * (size_t)nrows, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (!euclid_)
      for (float& x : h) x = std::isfinite(x) ? 1.0f - x : INFINITY;
    return host_topk(h, k);
  }

  // similarity.py DevicePool.lanes_per_row
  int lanes_per_row(int nq) const {
    static const int forced = [] {         // diagnostics: JB_POOL_LPR = 1 / 4 / 16
      const char* e = getenv("JB_POOL_LPR");
      const int v = e != nullptr ? atoi(e) : 0;
      return (v == 1 || v == 4 || v == 16) ? v : 0;
    }();
    if (forced) return forced;
    const int64_t rows = std::max<int64_t>(1, nlive_);
    const double mean = (double)live_ / (double)rows;
    if (nq >= 4 && mean <= 24) return 1;
    return mean <= 8 ? 1 : mean <= 64 ? 4 : 16;
  }

  void reset() {
    HIPCHK(hipStreamSynchronize(stream_));
    for (DevBuf<int64_t>* b : {&r_off_}) if (b->p) { HIPCHK(hipFree(b->p)); b->p = nullptr; b->cap = 0; }
    if (r_len_.p) { HIPCHK(hipFree(r_len_.p)); r_len_.p = nullptr; r_len_.cap = 0; }
    if (r_n2_.p) { HIPCHK(hipFree(r_n2_.p)); r_n2_.p = nullptr; r_n2_.cap = 0; }
    if (valid_.p) { HIPCHK(hipFree(valid_.p)); valid_.p = nullptr; valid_.cap = 0; }
    if (p_idx_.p) { HIPCHK(hipFree(p_idx_.p)); p_idx_.p = nullptr; p_idx_.cap = 0; }
    if (p_val_.p) { HIPCHK(hipFree(p_val_.p)); p_val_.p = nullptr; p_val_.cap = 0; }
    cap_rows_ = cap_entries_ = 0;
    end_ = live_ = nlive_ = 0;
    off_h_.clear(); len_h_.clear(); has_h_.clear();
    for (Stage& s : stage_)
      if (!s.used) HIPCHK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
    grow_rows(1024);
    grow_entries(1 << 16);
  }

  template <class T>
  void regrow(DevBuf<T>& b, int64_t old, int64_t cap) {
    T* np = nullptr;
    HIPCHK(hipMalloc((void**)&np, (size_t)cap * sizeof(T)));
    HIPCHK(hipMemsetAsync(np, 0, (size_t)cap * sizeof(T), stream_));
    if (old > 0 && b.p) HIPCHK(hipMemcpyAsync(np, b.p, (size_t)old * sizeof(T), hipMemcpyDeviceToDevice, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (b.p) HIPCHK(hipFree(b.p));
    b.p = np;
    b.cap = (size_t)cap;
  }

  void grow_rows(int64_t need) {
    int64_t cap = std::max<int64_t>(1024, cap_rows_);
    while (cap < need) cap *= 2;
    if (cap == cap_rows_) return;
    regrow(r_off_, cap_rows_, cap);
    regrow(r_len_, cap_rows_, cap);
    regrow(r_n2_, cap_rows_, cap);
    regrow(valid_, cap_rows_, cap);
    off_h_.resize((size_t)cap, 0);
    len_h_.resize((size_t)cap, 0);
    has_h_.resize((size_t)cap, 0);
    cap_rows_ = cap;
  }

  void grow_entries(int64_t need) {
    int64_t cap = std::max<int64_t>(1 << 16, cap_entries_);
    while (cap < need) cap *= 2;
    if (cap == cap_entries_) return;
    regrow(p_idx_, end_, cap);
    regrow(p_val_, end_, cap);
    cap_entries_ = cap;
  }

  // rewrite the live runs contiguously (DevicePool.compact), on the host
  void compact() {
    HIPCHK(hipStreamSynchronize(stream_));
    std::vector<int32_t> pi((size_t)end_);
    std::vector<float> pv((size_t)end_);
    if (end_) {
      HIPCHK(hipMemcpy(pi.data(), p_idx_.p, 4 * (size_t)end_, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(pv.data(), p_val_.p, 4 * (size_t)end_, hipMemcpyDeviceToHost));
    }
    std::vector<int32_t> ni;
    std::vector<float> nv;
    ni.reserve((size_t)live_);
    nv.reserve((size_t)live_);
    for (int64_t s = 0; s < cap_rows_; ++s) {
      if (len_h_[s] <= 0) continue;
      const int64_t o = off_h_[s];
      off_h_[s] = (int64_t)ni.size();
      ni.insert(ni.end(), pi.begin() + o, pi.begin() + o + len_h_[s]);
      nv.insert(nv.end(), pv.begin() + o, pv.begin() + o + len_h_[s]);
    }
    if (!ni.empty()) {
      HIPCHK(hipMemcpy(p_idx_.p, ni.data(), 4 * ni.size(), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(p_val_.p, nv.data(), 4 * nv.size(), hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemcpy(r_off_.p, off_h_.data(), 8 * (size_t)cap_rows_, hipMemcpyHostToDevice));
    end_ = live_ = (int64_t)ni.size();
  }

  bool euclid_;
  hipStream_t stream_;
  int64_t cap_rows_ = 0, cap_entries_ = 0, end_ = 0, live_ = 0, nlive_ = 0;
  std::vector<int64_t> off_h_, len_h_;
  std::vector<uint8_t> has_h_;
  DevBuf<int64_t> r_off_;
  DevBuf<int32_t> r_len_;
  DevBuf<double> r_n2_;
  DevBuf<uint8_t> valid_;
  DevBuf<int32_t> p_idx_;
  DevBuf<float> p_val_;
  DevBuf<int64_t> d_qptr_;
  DevBuf<int32_t> d_qidx_, d_qslot_;
  DevBuf<float> d_qval_;
  DevBuf<double> d_qn2_;
  Stage stage_[kStages];
  int turn_ = 0;
  QueryBufs bufs_;
  // deferred writes (set_defer)
  bool defer_ = false;
  int64_t pend_base_ = 0;
  std::vector<int64_t> pend_meta_;
  std::vector<int32_t> pend_idx_;
  std::vector<float> pend_val_;
};

// ------------------------------------------------------------- row store
// models/rows.py RowStore + Unlearner("lru") + the index of the engine
struct Row {
  std::string id;
  Datum d;
  std::vector<int32_t> idx;   // hashed feature vector (idx >= 0 entries)
  std::vector<float> val;
  bool live = false;
};

class RowEngine {
 public:
  // method: lsh / euclid_lsh / minhash / inverted_index / inverted_index_euclid
  RowEngine(const std::string& method, const Value* param, hipStream_t st) : method_(method), stream_(st) {
    auto num = [&](const char* k, double d) {
      const Value* v = param ? param->get(k) : nullptr;
      return v && v->is_num() ? v->num() : d;
    };
    if (method == "lsh" || method == "euclid_lsh" || method == "minhash") {
      const int hash_num = (int)num("hash_num", 64);
      if (hash_num <= 0) throw std::runtime_error("hash_num must be positive");
      lsh_.reset(new LshIndex(method, hash_num, (uint64_t)(int64_t)num("seed", 1091), st));
    } else if (method == "inverted_index" || method == "inverted_index_euclid") {
      pool_.reset(new PoolIndex(method == "inverted_index_euclid", st));
    } else {
      throw std::runtime_error("unknown similarity method: " + method);
    }
    // the id tables sized for a million rows up front: growing them rehashes
    // every node (a cache miss each) at every doubling, on the write path
    slot_of_.reserve((size_t)1 << 20);
    version_.reserve((size_t)1 << 20);
    dirty_.reserve((size_t)1 << 20);
    const Value* unl = param ? param->get("unlearner") : nullptr;
    if (unl && unl->kind != Value::NIL) {
      if (!unl->is_str() || unl->s != "lru") throw std::runtime_error("unknown unlearner");
      const Value* up = param->get("unlearner_parameter");
      const Value* ms = up ? up->get("max_size") : nullptr;
      max_size_ = ms && ms->is_num() ? (int64_t)ms->num() : 0;
      if (max_size_ <= 0) throw std::runtime_error("unlearner_parameter.max_size must be positive");
      lru_ = true;
    }
  }

  Converter conv;
  const std::string& method() const { return method_; }
  bool is_lsh() const { return (bool)lsh_; }
  bool lru() const { return lru_; }
  int64_t nslots() const { return (int64_t)rows_.size(); }
  size_t size() const { return slot_of_.size(); }

  const Row* find(const std::string& id) const {
    auto it = slot_of_.find(id);
    return it == slot_of_.end() ? nullptr : &rows_[(size_t)it->second.first];
  }
  int32_t slot(const std::string& id) const {
    auto it = slot_of_.find(id);
    return it == slot_of_.end() ? -1 : it->second.first;
  }
  const Row& at(int32_t s) const { return rows_[(size_t)s]; }

  // RowEngine._set: store the datum, hash it (document statistics updated),
  // write the index, then the lru evictions
  void set(const std::string& id, Datum&& d, bool bump = true) {
    MsgpackWriter w;
    write_datum(w, d);
    Row tmp;
    conv.hash((const uint8_t*)w.out.data(), w.out.size(), &tmp.idx, &tmp.val, bump);
    store(id, std::move(d), tmp.idx, tmp.val, bump);
  }

  // a row whose feature vector was hashed elsewhere (a MIX diff: the sender's
  // vector is kept, as rows.put_many does)
  void store(const std::string& id, Datum&& d, const std::vector<int32_t>& idx, const std::vector<float>& val,
             bool bump) {
    std::vector<int32_t> fi;
    std::vector<float> fv;
    fi.reserve(idx.size());
    fv.reserve(idx.size());
    for (size_t i = 0; i < idx.size(); ++i)
      if (idx[i] >= 0) { fi.push_back(idx[i]); fv.push_back(val[i]); }
    const int32_t s = assign(id);
    Row& r = rows_[(size_t)s];
    r.d = std::move(d);
    r.idx = std::move(fi);
    r.val = std::move(fv);
    r.live = true;
    if (bump) {
      version_[id] += 1;
      dirty_.insert(id);
      if (!removed_.empty()) removed_.erase(id);
    }
    if (lsh_) lsh_->set(s, idx, val);
    else pool_->set(s, idx, val);
    if (lru_) {
      touch(id);
      while ((int64_t)lru_order_.size() > max_size_) {
        const std::string victim = lru_order_.front();
        if (victim == id) break;
        remove(victim);
      }
    }
  }

  // batched writes (Model::write_many): the LSH index keeps the rows set
  // meanwhile on the host and writes them in one launch when it ends
  void defer_writes(bool on) {
    if (lsh_) lsh_->set_defer(on);
    else pool_->set_defer(on);
  }

  // called with the slot of every removed row (the LOF state's moved())
  std::function<void(int32_t)> on_remove;

  bool remove(const std::string& id, bool record = true) {
    auto it = slot_of_.find(id);
    if (it == slot_of_.end()) return false;
    const int32_t s = it->second.first;
    if (on_remove) on_remove(s);
    insertion_.erase(it->second.second);
    slot_of_.erase(it);
    Row& r = rows_[(size_t)s];
    r = Row();
    free_.push_back(s);
    if (record) {
      version_[id] += 1;
      removed_.insert(id);
      dirty_.erase(id);
    }
    if (lsh_) lsh_->remove(s);
    else pool_->remove(s);
    if (lru_) {
      auto l = lru_pos_.find(id);
      if (l != lru_pos_.end()) { lru_order_.erase(l->second); lru_pos_.erase(l); }
    }
    return true;
  }

  void clear() {
    rows_.clear();
    slot_of_.clear();
    insertion_.clear();
    free_.clear();
    version_.clear();
    dirty_.clear();
    removed_.clear();
    lru_order_.clear();
    lru_pos_.clear();
    if (lsh_) lsh_->clear();
    else pool_->clear();
    conv.clear();
  }

  std::vector<std::string> all_ids() const {
    std::vector<std::string> out;
    for (const Row& r : rows_)
      if (r.live) out.push_back(r.id);
    return out;
  }

  // k nearest of a hashed vector / a stored row -> (id, distance)
  std::vector<Hit> query_fv(const std::vector<int32_t>& idx, const std::vector<float>& val, int k) {
    if (nslots() == 0 || k <= 0) return {};
    return lsh_ ? lsh_->query_fv(idx, val, nslots(), k) : pool_->query_fv(idx, val, nslots(), k);
  }
  // several hashed vectors at one k: multi-query passes of up to 8 where
  // the index takes them (the LSH signature arguments hold 256 feature
  // slots per launch), one by one otherwise
  std::vector<std::vector<Hit>> query_fv_many(const std::vector<const std::vector<int32_t>*>& idx,
                                              const std::vector<const std::vector<float>*>& val, int k) {
    const size_t n = idx.size();
    std::vector<std::vector<Hit>> out(n);
    if (nslots() == 0 || k <= 0) return out;
    size_t i = 0;
    while (i < n) {
      size_t j = i + 1;
      size_t feats = idx[i]->size();
      while (j < n && j - i < (size_t)kQueryMax && (!lsh_ || feats + idx[j]->size() <= (size_t)kQuerySlots))
        feats += idx[j++]->size();
      std::vector<const std::vector<int32_t>*> bi(idx.begin() + i, idx.begin() + j);
      std::vector<const std::vector<float>*> bv(val.begin() + i, val.begin() + j);
      std::vector<std::vector<Hit>> r;
      const bool ok = j - i > 1 && (lsh_ ? lsh_->query_fv_many(bi, bv, nslots(), k, &r)
                                         : pool_->query_fv_many(bi, bv, nslots(), k, &r));
      if (ok) {
        for (size_t q = i; q < j; ++q) out[q] = std::move(r[q - i]);
      } else {
        for (size_t q = i; q < j; ++q) out[q] = query_fv(*idx[q], *val[q], k);
      }
      i = j;
    }
    return out;
  }
  std::vector<Hit> query_slot(int32_t s, int k) {
    if (nslots() == 0 || k <= 0) return {};
    return lsh_ ? lsh_->query_slot(s, nslots(), k) : pool_->query_slot(s, nslots(), k);
  }
  double similarity(float d) const { return lsh_ ? lsh_->similarity(d) : pool_->similarity(d); }

  // (id, score) of the hits whose slot still holds a row (row_engine._results)
  std::vector<std::pair<std::string, double>> results(const std::vector<Hit>& hits, bool similar) const {
    std::vector<std::pair<std::string, double>> out;
    for (const Hit& h : hits) {
      if (h.slot < 0 || h.slot >= nslots() || !rows_[(size_t)h.slot].live) continue;
      out.emplace_back(rows_[(size_t)h.slot].id, similar ? similarity(h.dist) : (double)h.dist);
    }
    return out;
  }

  double calc_similarity(const std::vector<int32_t>& ai, const std::vector<float>& av,
                         const std::vector<int32_t>& bi, const std::vector<float>& bv) const {
    if (lsh_) return lsh_->calc_similarity(ai, av, bi, bv);
    // recommender.py _dense + cosine / euclid in double, first-occurrence order
    auto dense = [](const std::vector<int32_t>& i, const std::vector<float>& v) {
      std::vector<std::pair<int32_t, double>> d;
      std::unordered_map<int32_t, size_t> at;
      for (size_t k = 0; k < i.size(); ++k) {
        if (i[k] < 0) continue;
        auto it = at.find(i[k]);
        if (it == at.end()) { at[i[k]] = d.size(); d.push_back({i[k], (double)v[k]}); }
        else d[it->second].second += (double)v[k];
      }
      return d;
    };
    const auto da = dense(ai, av), db = dense(bi, bv);
    std::unordered_map<int32_t, double> mb(db.begin(), db.end());
    double dot = 0.0, a2 = 0.0, b2 = 0.0;
    for (const auto& kv : da) {
      auto it = mb.find(kv.first);
      dot += kv.second * (it == mb.end() ? 0.0 : it->second);
    }
    for (const auto& kv : da) a2 += kv.second * kv.second;
    for (const auto& kv : db) b2 += kv.second * kv.second;
    if (method_ == "inverted_index_euclid") return -sqrt(std::max(0.0, a2 + b2 - 2 * dot));
    const double den = sqrt(a2) * sqrt(b2);
    return den > 0 ? dot / den : 0.0;
  }

  // ---------------------------------------------------------------- MIX
  // the row-diff protocol of jb_row_mix.hpp (parallel/row_mix.py) over this
  // store: the written rows' hashed vectors travel, receivers keep them
  size_t dirty_rows() const { return dirty_.size() + removed_.size(); }
  void pack_diff(MsgpackWriter& w) const { pack_row_diff(*this, w); }
  size_t apply_diffs(const std::vector<Value>& parts, std::vector<int32_t>* changed, bool forward = false) {
    // the LSH signatures of the applied rows: one staged launch at the end
    defer_writes(true);
    try {
      const size_t n = apply_row_diffs(*this, parts, changed, forward);
      defer_writes(false);
      return n;
    } catch (...) {
      defer_writes(false);
      throw;
    }
  }
  // store interface of pack_row_diff / apply_row_diffs
  std::vector<std::string> mix_ids() const {
    std::vector<std::string> ids;
    for (const auto& id : dirty_)
      if (slot_of_.count(id)) ids.push_back(id);
    std::sort(ids.begin(), ids.end());
    return ids;
  }
  std::vector<std::string> mix_removed() const {
    std::vector<std::string> rm(removed_.begin(), removed_.end());
    std::sort(rm.begin(), rm.end());
    return rm;
  }
  bool version_of(const std::string& id, uint64_t* v) const {
    auto it = version_.find(id);
    if (it == version_.end()) { *v = 0; return false; }
    *v = it->second;
    return true;
  }
  bool holds(const std::string& id) const { return slot_of_.count(id) != 0; }
  void row_view(const std::string& id, const Datum** d, const std::vector<int32_t>** ix,
                const std::vector<float>** vx) const {
    const Row& r = rows_[(size_t)slot_of_.at(id).first];
    *d = &r.d;
    *ix = &r.idx;
    *vx = &r.val;
  }
  int32_t slot_id(const std::string& id) const { return slot(id); }
  void store_mixed(const std::string& id, Datum&& d, const std::vector<int32_t>& idx,
                   const std::vector<float>& val, uint64_t v, bool forward) {
    store(id, std::move(d), idx, val, false);
    version_[id] = v;
    if (forward) {
      dirty_.insert(id);
      removed_.erase(id);
    }
  }
  void remove_mixed(const std::string& id, uint64_t v, bool forward) {
    remove(id, false);
    version_[id] = v;
    if (forward) {
      removed_.insert(id);
      dirty_.erase(id);
    }
  }
  bool weight_diff(int64_t* docs, int64_t* len, std::vector<int64_t>* idx, std::vector<int64_t>* cnt) const {
    if (!conv.uses_weights()) { *docs = *len = 0; return false; }
    conv.get_diff(docs, len, idx, cnt);
    return true;
  }
  void put_weight_diff(int64_t docs, int64_t len, const std::vector<int64_t>& idx, const std::vector<int64_t>& cnt,
                       bool keep_own = false) {
    conv.put_diff(docs, len, idx, cnt, keep_own);
  }
  void mix_done() {
    dirty_.clear();
    removed_.clear();
    conv.clear_diff();
  }

  // RowEngine.pack(): {"method", "rows": {id: [version, [sv, nv, bv]]}, "weights"}
  void pack(MsgpackWriter& w, const std::string& method_name) const {
    w.map(3);
    w.str("method");
    w.str(method_name);
    w.str("rows");
    w.map(slot_of_.size());
    for (const std::string& id : insertion_) {
      const Row& r = rows_[(size_t)slot_of_.at(id).first];
      w.str(id);
      w.arr(2);
      auto v = version_.find(id);
      w.sint(v == version_.end() ? 0 : (int64_t)v->second);
      w.arr(3);
      w.map(r.d.sv.size());
      for (const auto& kv : r.d.sv) { w.str(kv.first); w.str(kv.second); }
      w.map(r.d.nv.size());
      for (const auto& kv : r.d.nv) { w.str(kv.first); w.dbl(kv.second); }
      w.map(r.d.bv.size());
      for (const auto& kv : r.d.bv) { w.str(kv.first); w.bin(kv.second.data(), kv.second.size()); }
    }
    w.str("weights");
    conv.pack(w);
  }

  // RowEngine.unpack(): rows in file order, versions as stored, no
  // document-statistics updates (the weights come from the file)
  void unpack(const Value& obj) {
    const Value* rows = obj.get("rows");
    if (!rows || rows->kind != Value::MAP) throw std::runtime_error("broken model data: rows");
    clear();
    if (const Value* w = obj.get("weights"))
      if (w->kind != Value::NIL) conv.unpack(*w);
    for (const auto& kv : rows->o) {
      const Value& e = kv.second;
      if (e.kind != Value::ARR || e.a.size() != 2 || e.a[1].kind != Value::ARR || e.a[1].a.size() != 3)
        throw std::runtime_error("broken model data: row " + kv.first);
      Datum d;
      const Value& parts = e.a[1];
      for (const auto& x : parts.a[0].o) d.sv[x.first] = x.second.s;
      for (const auto& x : parts.a[1].o) d.nv[x.first] = x.second.num();
      for (const auto& x : parts.a[2].o) d.bv[x.first] = x.second.s;
      set(kv.first, std::move(d), false);
      version_[kv.first] = (uint64_t)e.a[0].num();
    }
  }

 private:
  int32_t assign(const std::string& id) {
    auto it = slot_of_.find(id);
    if (it != slot_of_.end()) return it->second.first;
    int32_t s;
    if (!free_.empty()) {
      s = free_.back();
      free_.pop_back();
    } else {
      s = (int32_t)rows_.size();
      rows_.emplace_back();
    }
    rows_[(size_t)s].id = id;
    insertion_.push_back(id);
    slot_of_[id] = {s, std::prev(insertion_.end())};
    return s;
  }

  void touch(const std::string& id) {
    auto l = lru_pos_.find(id);
    if (l != lru_pos_.end()) lru_order_.erase(l->second);
    lru_order_.push_back(id);
    lru_pos_[id] = std::prev(lru_order_.end());
  }

  std::string method_;
  hipStream_t stream_;
  std::unique_ptr<LshIndex> lsh_;
  std::unique_ptr<PoolIndex> pool_;
  std::deque<Row> rows_;   // (a deque: growth moves no rows and keeps references)
  std::list<std::string> insertion_;
  std::unordered_map<std::string, std::pair<int32_t, std::list<std::string>::iterator>> slot_of_;
  std::vector<int32_t> free_;
  std::unordered_map<std::string, uint64_t> version_;
  std::unordered_set<std::string> dirty_, removed_;   // since the last MIX
  bool lru_ = false;
  int64_t max_size_ = 0;
  std::list<std::string> lru_order_;
  std::unordered_map<std::string, std::list<std::string>::iterator> lru_pos_;
};

}  // namespace row
}  // namespace jb
