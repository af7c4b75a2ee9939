// The converter of the native linear servers (jubaclassifier,
// jubaregression): the fixed-slot host hasher (jb_hostfv.hpp) when the
// configuration fits the GPU request scan, else the wide rule set
// (jb_hostfv_wide.hpp: ngram / space splitters, tf / log_tf / idf / bm25
// weights, combination rules add / mul) with the document statistics of the
// global weights (WeightManager layout: df[H], diff[H], counts =
// [docs, total_len, diff_docs, diff_len]). Reference: the converter the
// engine servers build from the config, classifier_serv.cpp:111
// (make_fv_converter); config/classifier/default.json (bigram + idf) and
// arow_combinational_feature.json (mul) are the configurations this serves.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "jb_hostfv.hpp"
#include "jb_hostfv_wide.hpp"
#include "jb_server_common.hpp"
#include "jb_wide_rules.hpp"

namespace jb {
namespace srv {

struct WideRules {
  std::vector<HostRule> s, n, c;
  std::string blob;
  bool global = false;
  std::shared_ptr<WideExt> ext;   // plug-ins ("dynamic" types), filters, binary rules
};

// the converter section: fast rules, else wide rules (why: the reason neither fits)
inline bool build_linear_rules(const Value& conv, Rules* fast, bool* wide, WideRules* w, std::string* why) {
  std::string why_fast;
  *wide = false;
  if (build_rules(conv, fast, &why_fast)) return true;
  uint64_t H = fast->H;
  std::string why_wide;
  if (!jb::row::build_wide_rules(conv, &w->s, &w->n, &w->c, &w->blob, &H, &w->global, &why_wide, &w->ext)) {
    *why = why_fast + "; " + why_wide;
    return false;
  }
  fast->H = H;
  *wide = true;
  return true;
}

// The document statistics of idf / bm25 converters (WeightManager: df[H],
// diff[H] since the last MIX, counts = [docs, total_len, diff_docs,
// diff_len]) and their MIX: get_diff -> [docs, len, bin i64 idx, bin i64
// count]; put_diffs folds every member's (its own included).
struct DocStats {
  std::vector<int64_t> df, diff;
  int64_t counts[4] = {0, 0, 0, 0};

  void reset(uint64_t H) {
    df.assign(H, 0);
    diff.assign(H, 0);
    std::fill(counts, counts + 4, 0);
  }
  void clear() {
    std::fill(df.begin(), df.end(), 0);
    std::fill(diff.begin(), diff.end(), 0);
    std::fill(counts, counts + 4, 0);
  }
  void attach(HostFvWide* w) { w->set_weights(df.data(), diff.data(), counts); }

  std::string get_diff() const {
    MsgpackWriter u;
    u.arr(4);
    u.sint(counts[2]);
    u.sint(counts[3]);
    std::vector<int64_t> ix, cn;
    for (size_t i = 0; i < diff.size(); ++i)
      if (diff[i]) { ix.push_back((int64_t)i); cn.push_back(diff[i]); }
    u.bin(ix.data(), ix.size() * 8);
    u.bin(cn.data(), cn.size() * 8);
    return std::move(u.out);
  }
  // keep_own: one round of a push MIX (the own diff goes to the later
  // partners too; clear_diff() when the MIX ends) - see jb_row_engine.hpp put_diff
  void put_diffs(const std::vector<Value>& parts, bool keep_own = false) {
    if (df.empty()) return;
    int64_t docs = 0, len = 0;
    std::vector<int64_t> acc(df.size(), 0);
    for (const Value& d : parts) {
      if (d.kind != Value::ARR || d.a.size() != 4) throw std::runtime_error("mix: malformed weight diff");
      docs += (int64_t)d.a[0].num();
      len += (int64_t)d.a[1].num();
      const size_t n = std::min(d.a[2].s.size(), d.a[3].s.size()) / 8;
      for (size_t k = 0; k < n; ++k) {
        int64_t i, c;
        memcpy(&i, d.a[2].s.data() + 8 * k, 8);
        memcpy(&c, d.a[3].s.data() + 8 * k, 8);
        if (i >= 0 && (size_t)i < acc.size()) acc[(size_t)i] += c;
      }
    }
    counts[0] += docs - counts[2];
    counts[1] += len - counts[3];
    for (size_t i = 0; i < df.size(); ++i) df[i] = std::max<int64_t>(0, df[i] - diff[i] + acc[i]);
    if (keep_own) return;
    clear_diff();
  }
  void clear_diff() {
    std::fill(diff.begin(), diff.end(), 0);
    counts[2] = counts[3] = 0;
  }
  void put_diffs(const std::vector<std::string>& raw, bool keep_own = false) {
    std::vector<Value> parts;
    for (const auto& r : raw) parts.push_back(MsgpackReader((const uint8_t*)r.data(), r.size()).read());
    put_diffs(parts, keep_own);
  }
  // WeightManager.pack(): [doc_count, total_len, {"idx": [...], "df": [...]}]
  void pack(MsgpackWriter& u) const {
    u.arr(3);
    u.sint(counts[0]);
    u.sint(counts[1]);
    u.map(2);
    std::vector<int64_t> nz;
    for (size_t i = 0; i < df.size(); ++i)
      if (df[i]) nz.push_back((int64_t)i);
    u.str("idx");
    u.arr(nz.size());
    for (int64_t i : nz) u.sint(i);
    u.str("df");
    u.arr(nz.size());
    for (int64_t i : nz) u.sint(df[(size_t)i]);
  }
  void unpack(const Value* w) {
    clear();
    if (!w || w->kind != Value::ARR || w->a.size() != 3) return;
    const Value* ix = w->a[2].get("idx");
    const Value* dfv = w->a[2].get("df");
    if (!ix || !dfv || ix->kind != Value::ARR || dfv->kind != Value::ARR || ix->a.size() != dfv->a.size() ||
        ix->a.empty())
      return;
    if (df.empty()) throw std::runtime_error("model carries document frequencies the converter does not use");
    counts[0] = (int64_t)w->a[0].num();
    counts[1] = (int64_t)w->a[1].num();
    for (size_t k = 0; k < ix->a.size(); ++k) {
      const int64_t i = (int64_t)ix->a[k].num();
      if (i < 0 || (uint64_t)i >= df.size()) throw std::runtime_error("broken model data: weights index");
      df[(size_t)i] += (int64_t)dfv->a[k].num();
    }
  }
};

class LinearConv {
 public:
  void configure(const Rules& fast, bool wide, const WideRules& w) {
    H_ = fast.H;
    fast_.reset();
    wide_.reset();
    st_.df.clear();
    st_.diff.clear();
    std::fill(st_.counts, st_.counts + 4, 0);
    if (!wide) {
      fast_.reset(new HostFvHasher((const uint8_t*)fast.s.data(), (int)fast.s.size(), (const uint8_t*)fast.n.data(),
                                   (int)fast.n.size(), (const uint8_t*)fast.blob.data(), fast.blob.size(), H_));
      return;
    }
    wide_.reset(new HostFvWide((const uint8_t*)w.s.data(), (int)w.s.size(), (const uint8_t*)w.n.data(),
                               (int)w.n.size(), (const uint8_t*)w.c.data(), (int)w.c.size() / 2,
                               (const uint8_t*)w.blob.data(), w.blob.size(), H_));
    wide_->set_ext(w.ext);
    if (wide_->needs_weights()) {
      st_.reset(H_);
      st_.attach(wide_.get());
    }
  }
  bool wide() const { return (bool)wide_; }
  bool global() const { return !st_.df.empty(); }

  // one datum at the cursor (HostFvHasher::hash_datum contract: 0 ok, 1
  // malformed, 2 capacity); update: count it into the document statistics
  int hash_datum(Cursor& c, int32_t* idx, float* val, int64_t cap, int64_t* slots, bool update) {
    if (fast_) return fast_->hash_datum(c, idx, val, cap, slots);
    return wide_->hash_datum(c, idx, val, cap, slots, update);
  }
  // a list<datum> body (analysis: no statistics update)
  int hash_body(const uint8_t* p, size_t len, int32_t* idx, float* val, int64_t* row_ptr, int64_t max_samples,
                int64_t max_slots, int64_t* n, int64_t* slots) {
    if (fast_) return fast_->hash_body(p, len, idx, val, row_ptr, max_samples, max_slots, n, slots);
    return wide_->hash_body(p, len, idx, val, row_ptr, max_samples, max_slots, n, slots, false);
  }
  // the statistics updates of one request are undone if it fails
  void begin() { if (wide_) wide_->begin(); }
  void rollback() { if (wide_) wide_->rollback(); }

  void clear() { st_.clear(); }

  // WeightManager.pack() / unpack(), get_diff / put_diff (DocStats)
  void pack(MsgpackWriter& u) const { st_.pack(u); }
  void unpack(const Value* w) { st_.unpack(w); }
  std::string get_diff() const { return st_.get_diff(); }
  void put_diffs(const std::vector<std::string>& parts, bool keep_own = false) {
    if (!st_.df.empty()) st_.put_diffs(parts, keep_own);
  }
  void clear_diff() {
    if (!st_.df.empty()) st_.clear_diff();
  }
  int64_t docs() const { return st_.counts[0]; }

 private:
  uint64_t H_ = 1ull << 20;
  std::unique_ptr<HostFvHasher> fast_;
  std::unique_ptr<HostFvWide> wide_;
  DocStats st_;
};

}  // namespace srv
}  // namespace jb
