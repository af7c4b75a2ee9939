// jubaweight, native: the feature-weight server without Python.
//
// Reference: jubatus/server/server/weight_serv.cpp:30-110 - update(datum)
// converts with the global-weight statistics updated (document frequencies,
// document count and length), calc_weight(datum) converts without touching
// them; both return the weighted feature vector as list<feature> [key,
// value]; clear drops the statistics; "method" / "parameter" are accepted and
// ignored (weight_serv.cpp:33-36). Same semantics as models/weight.py over the
// native wide converter (csrc/native/jb_hostfv_wide.hpp: feature order,
// values in double, idf / bm25 against the document-frequency table); model
// files are shared with the Python server (Weight.pack(): the weight
// manager's [doc count, total length, {idx, df}]). Configurations outside the
// wide converter (filters, plug-ins, regex matchers) go to the Python server.
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "jb_host_server.hpp"
#include "jb_wide_rules.hpp"

namespace {

using namespace jb::srv;

struct WideConfig {
  std::vector<jb::HostRule> s, n, c;
  std::string blob;
  uint64_t H = 1ull << 20;      // fv_converter/converter.py DEFAULT_HASH_MAX_SIZE
  bool global = false;
  std::shared_ptr<jb::WideExt> ext;   // plug-ins, filters, binary rules
};

bool check_config(const std::string& text, std::string* why, WideConfig* out) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  const Value* conv = v.get("converter");
  if (!conv) { *why = "weight config requires converter"; return false; }
  WideConfig w;
  if (!jb::row::build_wide_rules(*conv, &w.s, &w.n, &w.c, &w.blob, &w.H, &w.global, why, &w.ext)) return false;
  if (out) *out = std::move(w);
  return true;
}

// a datum Value back to msgpack (the converter reads wire bytes)
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

class Weight : public HostEngine {
 public:
  explicit Weight(WideConfig cfg) : cfg_(std::move(cfg)) {
    hw_.reset(new jb::HostFvWide((const uint8_t*)cfg_.s.data(), (int)cfg_.s.size(),
                                 (const uint8_t*)cfg_.n.data(), (int)cfg_.n.size(),
                                 (const uint8_t*)cfg_.c.data(), (int)cfg_.c.size() / 2,
                                 (const uint8_t*)cfg_.blob.data(), cfg_.blob.size(), cfg_.H));
    hw_->set_ext(cfg_.ext);
    if (hw_->needs_weights()) {
      df_.assign(cfg_.H, 0);
      diff_.assign(cfg_.H, 0);
    }
    hw_->set_weights(df_.empty() ? nullptr : df_.data(), diff_.empty() ? nullptr : diff_.data(), counts_);
  }

  std::vector<HostMethod> methods() override {
    return {
        {"update", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) { convert(a[0], true, w); }},
        {"calc_weight", 2, false,
         [this](const std::vector<Value>& a, MsgpackWriter* w) { convert(a[0], false, w); }},
        {"clear", 1, true, [this](const std::vector<Value>&, MsgpackWriter* w) {
           clear();
           w->boolean(true);
         }},
    };
  }

  void clear() override {
    std::fill(df_.begin(), df_.end(), 0);
    std::fill(diff_.begin(), diff_.end(), 0);
    memset(counts_, 0, sizeof counts_);
  }

  std::string pack() override {
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(1);
    u.str("weights");
    u.arr(3);
    u.sint(counts_[0]);
    u.sint(counts_[1]);
    size_t nz = 0;
    for (int64_t x : df_) nz += x != 0;
    u.map(2);
    u.str("idx");
    u.arr(nz);
    for (size_t i = 0; i < df_.size(); ++i)
      if (df_[i]) u.uint(i);
    u.str("df");
    u.arr(nz);
    for (int64_t x : df_)
      if (x) u.sint(x);
    return std::move(u.out);
  }

  void unpack(const Value& obj) override {
    const Value* wv = obj.get("weights");
    if (!wv || wv->kind != Value::ARR || wv->a.size() != 3)
      throw std::runtime_error("broken model data: weight manager");
    clear();
    counts_[0] = (int64_t)wv->a[0].num();
    counts_[1] = (int64_t)wv->a[1].num();
    const Value* idx = wv->a[2].get("idx");
    const Value* dfv = wv->a[2].get("df");
    if (!idx || !dfv)
      throw std::runtime_error("model statistics are name-keyed: load them with the Python server");
    if (idx->a.size() != dfv->a.size()) throw std::runtime_error("broken model data: df table");
    for (size_t i = 0; i < idx->a.size(); ++i) {
      const uint64_t k = (uint64_t)idx->a[i].num();
      if (k >= df_.size()) throw std::runtime_error("broken model data: df index");
      df_[k] += (int64_t)dfv->a[i].num();
    }
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) override {
    st->emplace_back("weight_manager", "df");
    st->emplace_back("server_runtime", "native");
    st->emplace_back("converter", "native-wide");
    st->emplace_back("num_docs", std::to_string(counts_[0]));
  }

 private:
  void convert(const Value& datum, bool update, MsgpackWriter* w) {
    if (datum.kind != Value::ARR || datum.a.size() < 2) throw std::invalid_argument("datum expected");
    MsgpackWriter body;
    body.arr(1);
    put_value(body, datum);
    std::string names;
    std::vector<int64_t> name_end;
    idx_.resize(std::max<size_t>(idx_.size(), 256));
    val_.resize(idx_.size());
    int64_t rp[2] = {0, 0};
    int rc;
    for (;;) {
      int64_t n = 0, slots = 0;
      names.clear();
      name_end.clear();
      hw_->begin();
      hw_->set_sinks(&names, &name_end, nullptr);
      rc = hw_->hash_body((const uint8_t*)body.out.data(), body.out.size(), idx_.data(), val_.data(), rp, 1,
                          (int64_t)idx_.size(), &n, &slots, update);
      hw_->set_sinks(nullptr, nullptr, nullptr);
      if (rc == 2) {
        if (update && hw_->needs_weights()) hw_->rollback();
        idx_.resize(idx_.size() * 4);
        val_.resize(idx_.size());
        continue;
      }
      break;
    }
    if (rc) {
      if (update && hw_->needs_weights()) hw_->rollback();
      throw std::invalid_argument("malformed datum");
    }
    const int64_t slots = rp[1];
    w->arr((size_t)slots);
    int64_t st = 0;
    for (int64_t i = 0; i < slots; ++i) {
      w->arr(2);
      w->raw(names.data() + st, (size_t)(name_end[(size_t)i] - st));
      w->dbl((double)val_[(size_t)i]);
      st = name_end[(size_t)i];
    }
  }

  WideConfig cfg_;
  std::unique_ptr<jb::HostFvWide> hw_;
 public:
  // ---- MIX (models/weight.py: WeightManager get_diff / mix / put_diff): the
  // document statistics each member counted since the last MIX; the
  // cluster's sum replaces this member's contribution
  bool mixable() const override { return true; }
  std::string get_diff() override {
    MsgpackWriter u;
    u.arr(4);
    u.sint(counts_[2]);
    u.sint(counts_[3]);
    std::vector<int64_t> ix, cn;
    for (size_t i = 0; i < diff_.size(); ++i)
      if (diff_[i]) { ix.push_back((int64_t)i); cn.push_back(diff_[i]); }
    u.bin(ix.data(), ix.size() * 8);
    u.bin(cn.data(), cn.size() * 8);
    return std::move(u.out);
  }
  void put_diffs(const std::vector<Value>& parts) override { fold(parts, false); }
  // push MIX: the own counts go to every partner of the MIX (broadcast_mixer:
  // every member's exactly once), dropped when it ends
  void put_diffs_push(const std::vector<Value>& parts) override { fold(parts, true); }
  void push_done() override {
    std::fill(diff_.begin(), diff_.end(), 0);
    counts_[2] = counts_[3] = 0;
  }
  void fold(const std::vector<Value>& parts, bool keep_own) {
    int64_t docs = 0, len = 0;
    std::vector<int64_t> acc(df_.size(), 0);
    for (const Value& d : parts) {
      if (d.kind != Value::ARR || d.a.size() != 4) throw std::runtime_error("mix: malformed weight diff");
      docs += (int64_t)d.a[0].num();
      len += (int64_t)d.a[1].num();
      const std::string& ix = d.a[2].s;
      const std::string& cn = d.a[3].s;
      const size_t n = std::min(ix.size(), cn.size()) / 8;
      for (size_t k = 0; k < n; ++k) {
        int64_t i, c;
        memcpy(&i, ix.data() + 8 * k, 8);
        memcpy(&c, cn.data() + 8 * k, 8);
        if (i >= 0 && (size_t)i < acc.size()) acc[(size_t)i] += c;
      }
    }
    counts_[0] += docs - counts_[2];
    counts_[1] += len - counts_[3];
    for (size_t i = 0; i < df_.size(); ++i) df_[i] = std::max<int64_t>(0, df_[i] - diff_[i] + acc[i]);
    if (keep_own) return;
    std::fill(diff_.begin(), diff_.end(), 0);
    counts_[2] = counts_[3] = 0;
  }

 private:
  std::vector<int64_t> df_, diff_;
  int64_t counts_[4] = {0, 0, 0, 0};
  std::vector<int32_t> idx_;
  std::vector<float> val_;
};

}  // namespace

int main(int argc, char** argv) {
  return host_main(
      argc, argv, "weight",
      [](const std::string& text, std::string* why) { return check_config(text, why, nullptr); },
      [](const std::string& text) -> std::unique_ptr<HostEngine> {
        WideConfig cfg;
        std::string why;
        if (!check_config(text, &why, &cfg)) throw std::runtime_error(why);
        return std::unique_ptr<HostEngine>(new Weight(std::move(cfg)));
      },
      /*native_dist=*/true);
}
