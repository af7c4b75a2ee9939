// jubaburst, native: Kleinberg burst detection without Python.
//
// Reference: jubatus/server/server/burst_serv.cpp:44-246 (add_documents,
// get_result(_at), get_all_bursted_results(_at), keywords) over
// jubatus_core's burst; config config/burst/*.json. Same behaviour as
// models/burst.py (its docstring lists it): a window of window_batch_size
// batches of width batch_interval aligned to multiples of the interval, a
// document past the end slides the window, one older than its start is
// rejected; per keyword and batch d = documents, r = documents containing
// the keyword; two-state Viterbi with p0 = R/D, p1 = min(scaling p0,
// 1 - 1e-9), emission -ln(C(d,r) p^r (1-p)^(d-r)), entering the burst state
// costs gamma ln(n); bursting batches report cost(p0) - cost(p1), cut below
// a positive costcut_threshold; result_window_rotate_size past windows kept.
// Standalone: every keyword is processed here. Distributed (-z): a keyword
// is processed by its two CHT owners (replication 2, burst_serv.cpp:200-246;
// the processed set is re-derived when the ring changes) and the others get
// its result windows through MIX (keywords and the processed keywords'
// windows, models/burst.py get_diff / mix_diff / put_diff). Model files are
// shared with the Python server (Burst.pack()).
#include <math.h>

#include <algorithm>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "jb_host_server.hpp"

namespace {

using namespace jb::srv;

struct Params {
  int64_t window = 0, rotate = 5, max_reuse = 5;
  double interval = 0, costcut = -1;
};

bool parse_params(const std::string& text, Params* p, std::string* why) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  if (v.str_or("method", "") != "burst") { *why = "unsupported burst method: " + v.str_or("method", ""); return false; }
  const Value* par = v.get("parameter");
  auto num = [&](const char* k, double* out, bool required) {
    const Value* x = par ? par->get(k) : nullptr;
    if (!x) {
      if (required) *why = std::string("burst parameter '") + k + "' is required";
      return !required;
    }
    if (x->is_num()) *out = x->num();
    else if (x->kind == Value::STR) *out = atof(x->s.c_str());
    else { *why = k; return false; }
    return true;
  };
  double ws = 0, mr = 5, rot = 5;
  if (!num("window_batch_size", &ws, true) || !num("batch_interval", &p->interval, true) ||
      !num("max_reuse_batch_num", &mr, false) || !num("costcut_threshold", &p->costcut, false) ||
      !num("result_window_rotate_size", &rot, false))
    return false;
  p->window = (int64_t)ws;
  p->max_reuse = (int64_t)mr;
  p->rotate = (int64_t)rot;
  if (p->window <= 0 || !(p->interval > 0) || p->rotate <= 0) {
    *why = "window_batch_size, batch_interval and result_window_rotate_size must be positive";
    return false;
  }
  return true;
}

double cost(int64_t d, int64_t r, double p) {
  if (d == 0) return 0.0;
  const double lb = lgamma((double)d + 1) - lgamma((double)r + 1) - lgamma((double)(d - r) + 1);
  return -(lb + (double)r * log(p) + (double)(d - r) * log1p(-p));
}

// per-batch burst weights of one keyword (models/burst.py detect)
std::vector<double> detect(const std::vector<int64_t>& d, const std::vector<int64_t>& r, double scaling,
                           double gamma, double costcut) {
  const size_t n = d.size();
  int64_t D = 0, R = 0;
  for (size_t i = 0; i < n; ++i) { D += d[i]; R += r[i]; }
  std::vector<double> out(n, 0.0);
  if (n == 0 || D == 0 || R == 0 || R >= D) return out;
  const double p0 = (double)R / (double)D;
  const double p1 = std::min(scaling * p0, 1.0 - 1e-9);
  const double trans = n > 1 ? gamma * log((double)n) : gamma;
  std::vector<double> c0(n), c1(n);
  for (size_t i = 0; i < n; ++i) { c0[i] = cost(d[i], r[i], p0); c1[i] = cost(d[i], r[i], p1); }
  double b0 = c0[0], b1 = trans + c1[0];
  std::vector<std::pair<int, int>> back;
  for (size_t i = 1; i < n; ++i) {
    const int f0 = b0 <= b1 ? 0 : 1;
    const double v0 = b0 <= b1 ? b0 : b1;
    const int t1 = b0 + trans <= b1 ? 0 : 1;
    const double v1 = b0 + trans <= b1 ? b0 + trans : b1;
    back.emplace_back(f0, t1);
    b0 = v0 + c0[i];
    b1 = v1 + c1[i];
  }
  int state = b0 <= b1 ? 0 : 1;
  std::vector<int> states(n, 0);
  for (size_t i = n; i-- > 0;) {
    states[i] = state;
    if (i > 0) state = state == 0 ? back[i - 1].first : back[i - 1].second;
  }
  for (size_t i = 0; i < n; ++i) {
    double w = states[i] == 1 ? c0[i] - c1[i] : 0.0;
    if (costcut > 0 && w < costcut) w = 0.0;
    out[i] = std::max(w, 0.0);
  }
  return out;
}

struct Batch {
  int64_t d, r;
  double w;
};
struct Window {
  double start;
  std::vector<Batch> batches;
};

class Burst : public HostEngine {
 public:
  explicit Burst(const Params& p) : p_(p) { clear(); }

  std::vector<HostMethod> methods() override {
    return {
        {"add_documents", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           if (a[0].kind != Value::ARR) throw std::invalid_argument("list expected");
           rehash();
           int64_t n = 0;
           for (const Value& doc : a[0].a) {
             if (doc.kind != Value::ARR || doc.a.size() < 2) throw std::invalid_argument("document");
             if (add_document(arg_str(doc.a[1]), arg_num(doc.a[0]))) ++n;
           }
           if (n) calculate();
           w->sint(n);
         }},
        {"get_result", 2, false, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           write_window(w, result(arg_str(a[0])));
         }},
        {"get_result_at", 3, false, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           write_window(w, result_at(arg_str(a[0]), arg_num(a[1])));
         }},
        {"get_all_bursted_results", 1, false, [this](const std::vector<Value>&, MsgpackWriter* w) {
           bursted(w, false, 0.0);
         }},
        {"get_all_bursted_results_at", 2, false, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           bursted(w, true, arg_num(a[0]));
         }},
        {"get_all_keywords", 1, false, [this](const std::vector<Value>&, MsgpackWriter* w) {
           w->arr(order_.size());
           for (const auto& k : order_) {
             const auto& sg = kw_.at(k);
             w->arr(3);
             w->raw(k);
             w->dbl(sg.first);
             w->dbl(sg.second);
           }
         }},
        {"add_keyword", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const Value& k = a[0];
           if (k.kind != Value::ARR || k.a.size() != 3) throw std::invalid_argument("keyword_with_params");
           w->boolean(add_keyword(arg_str(k.a[0]), arg_num(k.a[1]), arg_num(k.a[2])));
         }},
        {"remove_keyword", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const std::string& k = arg_str(a[0]);
           if (!kw_.count(k)) { w->boolean(false); return; }
           kw_.erase(k);
           order_.erase(std::find(order_.begin(), order_.end(), k));
           r_.erase(k);
           results_.erase(k);
           proc_.erase(k);
           w->boolean(true);
         }},
        {"remove_all_keywords", 1, true, [this](const std::vector<Value>&, MsgpackWriter* w) {
           kw_.clear();
           order_.clear();
           r_.clear();
           results_.clear();
           proc_.clear();
           w->boolean(true);
         }},
        {"clear", 1, true, [this](const std::vector<Value>&, MsgpackWriter* w) {
           clear();
           w->boolean(true);
         }},
    };
  }

  // models/burst.py clear(): the window and the results; keywords stay
  void clear() override {
    has_start_ = false;
    start_ = 0;
    d_.assign((size_t)p_.window, 0);
    for (auto& kv : r_) kv.second.assign((size_t)p_.window, 0);
    results_.clear();
  }

  // models/burst.py pack()
  std::string pack() override {
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(6);
    u.str("keywords"); u.map(order_.size());
    for (const auto& k : order_) { u.str(k); u.arr(2); u.dbl(kw_.at(k).first); u.dbl(kw_.at(k).second); }
    std::vector<std::string> proc(proc_.begin(), proc_.end());   // sorted
    u.str("processed"); u.arr(proc.size());
    for (const auto& k : proc) u.str(k);
    u.str("start");
    if (has_start_) u.dbl(start_); else u.nil();
    u.str("d"); u.arr(d_.size());
    for (int64_t x : d_) u.sint(x);
    u.str("r"); u.map(order_.size());
    for (const auto& k : order_) {
      u.str(k);
      const auto& rr = r_.at(k);
      u.arr(rr.size());
      for (int64_t x : rr) u.sint(x);
    }
    u.str("results"); u.map(results_.size());
    for (const auto& k : order_) {
      auto it = results_.find(k);
      if (it == results_.end()) continue;
      u.str(k);
      u.arr(it->second.size());
      for (const Window& win : it->second) {
        u.arr(2);
        u.dbl(win.start);
        u.arr(win.batches.size());
        for (const Batch& b : win.batches) { u.arr(3); u.sint(b.d); u.sint(b.r); u.dbl(b.w); }
      }
    }
    return std::move(u.out);
  }

  void unpack(const Value& obj) override {
    const Value* kv = obj.get("keywords");
    const Value* st = obj.get("start");
    const Value* dv = obj.get("d");
    const Value* rv = obj.get("r");
    const Value* res = obj.get("results");
    if (!kv || kv->kind != Value::MAP || !dv || dv->kind != Value::ARR || !rv || rv->kind != Value::MAP || !res ||
        res->kind != Value::MAP)
      throw std::runtime_error("broken model data: burst");
    kw_.clear();
    order_.clear();
    r_.clear();
    results_.clear();
    proc_.clear();
    for (const auto& k : kv->o) {
      kw_[k.first] = {k.second.a.at(0).num(), k.second.a.at(1).num()};
      order_.push_back(k.first);
    }
    if (const Value* pv = obj.get("processed")) {
      if (pv->kind == Value::ARR)
        for (const Value& k : pv->a)
          if (k.is_str() && kw_.count(k.s)) proc_.insert(k.s);
    }
    has_start_ = st && st->is_num();
    start_ = has_start_ ? st->num() : 0.0;
    d_.clear();
    for (const Value& x : dv->a) d_.push_back((int64_t)x.num());
    d_.resize((size_t)p_.window, 0);
    for (const auto& k : rv->o) {
      std::vector<int64_t> rr;
      for (const Value& x : k.second.a) rr.push_back((int64_t)x.num());
      rr.resize((size_t)p_.window, 0);
      r_[k.first] = rr;
    }
    for (const auto& k : order_)
      if (!r_.count(k)) r_[k].assign((size_t)p_.window, 0);
    for (const auto& k : res->o) {
      std::vector<Window>& hist = results_[k.first];
      for (const Value& win : k.second.a) {
        Window wd{win.a.at(0).num(), {}};
        for (const Value& b : win.a.at(1).a)
          wd.batches.push_back({(int64_t)b.a.at(0).num(), (int64_t)b.a.at(1).num(), b.a.at(2).num()});
        hist.push_back(std::move(wd));
      }
    }
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) override {
    char b[64];
    st->emplace_back("num_keywords", std::to_string(kw_.size()));
    st->emplace_back("processed_keywords", std::to_string(proc_.size()));
    if (has_start_) { snprintf(b, sizeof b, "%.17g", start_); st->emplace_back("window_start", b); }
    else st->emplace_back("window_start", "None");
    st->emplace_back("window_batch_size", std::to_string(p_.window));
    snprintf(b, sizeof b, "%.17g", p_.interval);
    st->emplace_back("batch_interval", b);
  }

  // ---- distributed mode
  bool mixable() const override { return true; }
  bool uses_cht() const override { return true; }
  void attach(jb::mix::ClusterNode* node, const Args& a) override {
    node_ = node;
    loc_ = a.eth + "_" + std::to_string(a.port);
    ring_.clear();
  }
  // {"keywords": {k: [scaling, gamma]}, "results": {processed k: windows}}
  std::string get_diff() override {
    MsgpackWriter u;
    u.map(2);
    u.str("keywords");
    u.map(order_.size());
    for (const auto& k : order_) { u.str(k); u.arr(2); u.dbl(kw_.at(k).first); u.dbl(kw_.at(k).second); }
    u.str("results");
    size_t n = 0;
    for (const auto& k : order_) n += proc_.count(k) && results_.count(k);
    u.map(n);
    for (const auto& k : order_) {
      if (!proc_.count(k) || !results_.count(k)) continue;
      u.str(k);
      write_hist(&u, results_.at(k));
    }
    return std::move(u.out);
  }
  // mix_diff folded in rank order (a later member's entry wins), then
  // put_diff: new keywords join, windows of keywords not processed here
  // are taken
  void put_diffs(const std::vector<Value>& parts) override {
    std::vector<std::string> korder;
    std::unordered_map<std::string, std::pair<double, double>> kws;
    std::vector<std::string> rorder;
    std::unordered_map<std::string, const Value*> res;
    for (const Value& d : parts) {
      const Value* kv = d.get("keywords");
      const Value* rv = d.get("results");
      if (!kv || kv->kind != Value::MAP || !rv || rv->kind != Value::MAP)
        throw std::runtime_error("mix: malformed burst diff");
      for (const auto& k : kv->o) {
        if (!kws.count(k.first)) korder.push_back(k.first);
        kws[k.first] = {k.second.a.at(0).num(), k.second.a.at(1).num()};
      }
      for (const auto& k : rv->o) {
        if (!res.count(k.first)) rorder.push_back(k.first);
        res[k.first] = &k.second;
      }
    }
    for (const auto& k : korder)
      if (!kw_.count(k)) {
        kw_[k] = kws[k];
        order_.push_back(k);
        r_[k].assign((size_t)p_.window, 0);
      }
    for (const auto& k : rorder) {
      if (!kw_.count(k) || proc_.count(k)) continue;
      std::vector<Window> hist;
      for (const Value& win : res[k]->a) {
        Window wd{win.a.at(0).num(), {}};
        for (const Value& b : win.a.at(1).a)
          wd.batches.push_back({(int64_t)b.a.at(0).num(), (int64_t)b.a.at(1).num(), b.a.at(2).num()});
        hist.push_back(std::move(wd));
      }
      results_[k] = std::move(hist);
    }
  }

 private:
  // is this server one of the keyword's 2 CHT owners (standalone: always)
  bool will_process(const std::string& k) const {
    if (!node_ || ring_.empty()) return true;
    const std::string h = jb::Md5::hex(k);
    size_t i = (size_t)(std::lower_bound(ring_.begin(), ring_.end(), std::make_pair(h, std::string())) -
                        ring_.begin()) % ring_.size();
    for (int n = 0; n < 2; ++n, i = (i + 1) % ring_.size())
      if (ring_[i].second == loc_) return true;
    return false;
  }
  // the ring changed (a member joined / left): derive the processed set again
  void rehash() {
    if (!node_) return;
    auto ring = node_->cht_ring();
    if (ring == ring_) return;
    ring_ = std::move(ring);
    proc_.clear();
    for (const auto& k : order_)
      if (will_process(k)) proc_.insert(k);
  }

  bool add_keyword(const std::string& k, double scaling, double gamma) {
    if (kw_.count(k)) return false;
    if (!(scaling > 1.0) || !(gamma > 0.0)) throw EngineError("scaling_param must be > 1 and gamma > 0");
    rehash();
    kw_[k] = {scaling, gamma};
    order_.push_back(k);
    r_[k].assign((size_t)p_.window, 0);
    if (will_process(k)) proc_.insert(k);
    return true;
  }

  double window_end() const { return start_ + (double)p_.window * p_.interval; }

  bool add_document(const std::string& text, double pos) {
    const double last = floor(pos / p_.interval) * p_.interval;
    if (!has_start_) {
      start_ = last - (double)(p_.window - 1) * p_.interval;
      has_start_ = true;
    }
    if (pos < start_) return false;
    if (pos >= window_end()) {
      const double ns = last - (double)(p_.window - 1) * p_.interval;
      int64_t shift = (int64_t)llround((ns - start_) / p_.interval);
      shift = std::min(shift, p_.window);
      auto slide = [&](std::vector<int64_t>& v) {
        v.erase(v.begin(), v.begin() + shift);
        v.resize((size_t)p_.window, 0);
      };
      slide(d_);
      for (auto& kv : r_) slide(kv.second);
      start_ = ns;
    }
    int64_t i = (int64_t)floor((pos - start_) / p_.interval);
    i = std::min(i, p_.window - 1);
    d_[(size_t)i] += 1;
    for (auto& kv : r_)
      if (text.find(kv.first) != std::string::npos) kv.second[(size_t)i] += 1;
    return true;
  }

  void calculate() {
    if (!has_start_) return;
    for (const auto& k : order_) {
      if (!proc_.count(k)) continue;
      const auto& sg = kw_.at(k);
      const auto& rr = r_.at(k);
      const std::vector<double> w = detect(d_, rr, sg.first, sg.second, p_.costcut);
      Window win{start_, {}};
      for (size_t i = 0; i < (size_t)p_.window; ++i) win.batches.push_back({d_[i], rr[i], w[i]});
      std::vector<Window>& hist = results_[k];
      if (!hist.empty() && hist.back().start == start_) {
        hist.back() = std::move(win);
      } else {
        hist.push_back(std::move(win));
        if ((int64_t)hist.size() > p_.rotate) hist.erase(hist.begin(), hist.end() - p_.rotate);
      }
    }
  }

  Window result(const std::string& k) const {
    auto it = results_.find(k);
    return it == results_.end() || it->second.empty() ? Window{0.0, {}} : it->second.back();
  }

  Window result_at(const std::string& k, double pos) const {
    auto it = results_.find(k);
    if (it == results_.end()) return Window{0.0, {}};
    for (auto w = it->second.rbegin(); w != it->second.rend(); ++w)
      if (w->start <= pos && pos < w->start + (double)p_.window * p_.interval) return *w;
    return Window{0.0, {}};
  }

  static bool is_bursted(const Window& w) {
    for (const Batch& b : w.batches)
      if (b.w > 0) return true;
    return false;
  }

  void bursted(MsgpackWriter* w, bool at, double pos) const {
    std::vector<std::pair<std::string, Window>> out;
    for (const auto& k : order_) {
      Window win = at ? result_at(k, pos) : result(k);
      if (is_bursted(win)) out.emplace_back(k, std::move(win));
    }
    w->map(out.size());
    for (const auto& kv : out) {
      w->raw(kv.first);
      write_window(w, kv.second);
    }
  }

  static void write_hist(MsgpackWriter* u, const std::vector<Window>& hist) {
    u->arr(hist.size());
    for (const Window& win : hist) {
      u->arr(2);
      u->dbl(win.start);
      u->arr(win.batches.size());
      for (const Batch& b : win.batches) { u->arr(3); u->sint(b.d); u->sint(b.r); u->dbl(b.w); }
    }
  }

  static void write_window(MsgpackWriter* w, const Window& win) {
    w->arr(2);
    w->dbl(win.start);
    w->arr(win.batches.size());
    for (const Batch& b : win.batches) {
      w->arr(3);
      w->sint(b.d);
      w->sint(b.r);
      w->dbl(b.w);
    }
  }

  Params p_;
  jb::mix::ClusterNode* node_ = nullptr;
  std::string loc_;                                            // "ip_port" of this server
  std::vector<std::pair<std::string, std::string>> ring_;      // CHT vnodes seen last
  std::set<std::string> proc_;                                 // keywords processed here
  bool has_start_ = false;
  double start_ = 0;
  std::vector<int64_t> d_;
  std::unordered_map<std::string, std::pair<double, double>> kw_;
  std::vector<std::string> order_;                 // keyword insertion order (Python dict order)
  std::unordered_map<std::string, std::vector<int64_t>> r_;
  std::unordered_map<std::string, std::vector<Window>> results_;
};

}  // namespace

int main(int argc, char** argv) {
  return host_main(
      argc, argv, "burst",
      [](const std::string& text, std::string* why) {
        Params p;
        return parse_params(text, &p, why);
      },
      [](const std::string& text) -> std::unique_ptr<HostEngine> {
        Params p;
        std::string why;
        if (!parse_params(text, &p, &why)) throw std::runtime_error(why);
        return std::unique_ptr<HostEngine>(new Burst(p));
      },
      /*native_dist=*/true);
}
