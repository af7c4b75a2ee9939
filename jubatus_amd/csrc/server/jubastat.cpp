// jubastat, native: windowed per-key statistics without Python.
//
// Reference: jubatus/server/server/stat_serv.cpp:51-106 (window_size;
// push / sum / stddev / max / min / entropy / moment / clear) over
// jubatus_core's stat. Same semantics as models/stat.py (its docstring
// lists them): one global window of the last window_size pushes, per-key
// running n / sum / sum of squares, max / min recomputed from the window
// only when the leaving value was the extreme, entropy over the key
// distribution of the window (its key argument ignored, stat_serv.cpp:89-91),
// moment = mean of (v - center)^degree over the key's window values.
// Model files are shared with the Python server (Stat.pack()).
#include <math.h>

#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "jb_host_server.hpp"

namespace {

using namespace jb::srv;

struct KeyStat {
  int64_t n = 0;
  double s = 0, s2 = 0, mx = -INFINITY, mn = INFINITY;
};

bool check_config(const std::string& text, std::string* why, int64_t* window) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  const Value* w = v.get("window_size");
  if (!w) { *why = "stat config requires window_size"; return false; }
  int64_t ws = 0;
  if (w->kind == Value::INT) ws = w->i;
  else if (w->kind == Value::STR) ws = atoll(w->s.c_str());
  else if (w->kind == Value::DBL) ws = (int64_t)w->d;
  if (ws <= 0) { *why = "window_size must be positive"; return false; }
  if (window) *window = ws;
  return true;
}

class Stat : public HostEngine {
 public:
  explicit Stat(int64_t window) : window_size_(window) {}

  std::vector<HostMethod> methods() override {
    auto key_op = [this](const char* op, double (Stat::*fn)(const KeyStat&)) {
      return [this, op, fn](const std::vector<Value>& a, MsgpackWriter* w) {
        w->dbl((this->*fn)(get(op, arg_str(a[0]))));
      };
    };
    return {
        {"push", 3, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           push(arg_str(a[0]), arg_num(a[1]));
           w->boolean(true);
         }},
        {"sum", 2, false, key_op("sum", &Stat::f_sum)},
        {"stddev", 2, false, key_op("stddev", &Stat::f_stddev)},
        {"max", 2, false, key_op("max", &Stat::f_max)},
        {"min", 2, false, key_op("min", &Stat::f_min)},
        {"entropy", 2, false, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           arg_str(a[0]);
           w->dbl(entropy());
         }},
        {"moment", 4, false, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           w->dbl(moment(arg_str(a[0]), arg_int(a[1]), arg_num(a[2])));
         }},
        {"clear", 1, true, [this](const std::vector<Value>&, MsgpackWriter* w) {
           clear();
           w->boolean(true);
         }},
    };
  }

  void clear() override {
    window_.clear();
    stats_.clear();
    mixed_e_ = 0;
    mixed_n_ = 0;
  }

  std::string pack() override {
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(3);
    u.str("window_size"); u.uint((uint64_t)window_size_);
    u.str("window"); u.arr(window_.size());
    for (const auto& kv : window_) { u.arr(2); u.str(kv.first); u.dbl(kv.second); }
    u.str("mixed"); u.arr(2); u.dbl(mixed_e_); u.sint(mixed_n_);
    return std::move(u.out);
  }

  void unpack(const Value& obj) override {
    const Value* wv = obj.get("window");
    const Value* mv = obj.get("mixed");
    if (!wv || wv->kind != Value::ARR || !mv || mv->kind != Value::ARR || mv->a.size() != 2)
      throw std::runtime_error("broken model data: stat");
    clear();
    for (const Value& kv : wv->a) {
      if (kv.kind != Value::ARR || kv.a.size() != 2 || !kv.a[0].is_str() || !kv.a[1].is_num())
        throw std::runtime_error("broken model data: stat window");
      push(kv.a[0].s, kv.a[1].num());
    }
    mixed_e_ = mv->a[0].num();
    mixed_n_ = (int64_t)mv->a[1].num();
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) override {
    st->emplace_back("storage", "stat");
    st->emplace_back("window_size", std::to_string(window_size_));
    st->emplace_back("num_keys", std::to_string(stats_.size()));
    st->emplace_back("window_population", std::to_string(window_.size()));
  }

 private:
  void push(const std::string& key, double v) {
    window_.emplace_back(key, v);
    KeyStat& st = stats_[key];
    st.n += 1;
    st.s += v;
    st.s2 += v * v;
    st.mx = std::max(st.mx, v);
    st.mn = std::min(st.mn, v);
    if ((int64_t)window_.size() > window_size_) evict();
  }

  void evict() {
    const auto kv = window_.front();
    window_.pop_front();
    auto it = stats_.find(kv.first);
    KeyStat& st = it->second;
    st.n -= 1;
    if (st.n == 0) {
      stats_.erase(it);
      return;
    }
    st.s -= kv.second;
    st.s2 -= kv.second * kv.second;
    if (kv.second >= st.mx || kv.second <= st.mn) {
      st.mx = -INFINITY;
      st.mn = INFINITY;
      for (const auto& x : window_)
        if (x.first == kv.first) { st.mx = std::max(st.mx, x.second); st.mn = std::min(st.mn, x.second); }
    }
  }

  const KeyStat& get(const char* op, const std::string& key) const {
    auto it = stats_.find(key);
    if (it == stats_.end()) throw EngineError(std::string(op) + ": key " + key + " not found");
    return it->second;
  }

  double f_sum(const KeyStat& s) { return s.s; }
  double f_stddev(const KeyStat& s) {
    const double mean = s.s / (double)s.n;
    return sqrt(std::max(0.0, s.s2 / (double)s.n - mean * mean));
  }
  double f_max(const KeyStat& s) { return s.mx; }
  double f_min(const KeyStat& s) { return s.mn; }

  // ---- MIX (models/stat.py get_diff / mix_diff / put_diff): the cluster's
  // entropy terms sum over the members' windows
  bool mixable() const override { return true; }
  bool uses_cht() const override { return true; }
  std::string get_diff() override {
    MsgpackWriter w;
    w.arr(2);
    w.dbl(local_e());
    w.sint((int64_t)window_.size());
    return std::move(w.out);
  }
  void put_diffs(const std::vector<Value>& parts) override {
    double e = 0;
    int64_t n = 0;
    for (const Value& p : parts) {
      if (p.kind != Value::ARR || p.a.size() != 2) throw std::runtime_error("mix: malformed stat diff");
      e += p.a[0].num();
      n += (int64_t)p.a[1].num();
    }
    mixed_e_ = e;
    mixed_n_ = n;
  }

  double local_e() const {
    double e = 0;
    for (const auto& kv : stats_) e += (double)kv.second.n * log((double)kv.second.n);
    return e;
  }

  double entropy() const {
    double e;
    int64_t n;
    if (mixed_n_ > 0) {
      e = mixed_e_;
      n = mixed_n_;
    } else {
      e = local_e();
      n = (int64_t)window_.size();
    }
    if (n == 0) return 0.0;
    return log((double)n) - e / (double)n;
  }

  double moment(const std::string& key, int64_t degree, double center) const {
    const KeyStat& st = get("moment", key);
    if (degree < 0) throw EngineError("moment: negative degree");
    if (degree == 0) return 1.0;
    double acc = 0;
    for (const auto& x : window_)
      if (x.first == key) acc += pow(x.second - center, (double)degree);
    return acc / (double)st.n;
  }

  int64_t window_size_;
  std::deque<std::pair<std::string, double>> window_;
  std::unordered_map<std::string, KeyStat> stats_;
  double mixed_e_ = 0;
  int64_t mixed_n_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
  return host_main(
      argc, argv, "stat",
      [](const std::string& text, std::string* why) { return check_config(text, why, nullptr); },
      [](const std::string& text) -> std::unique_ptr<HostEngine> {
        int64_t w = 0;
        std::string why;
        if (!check_config(text, &why, &w)) throw std::runtime_error(why);
        return std::unique_ptr<HostEngine>(new Stat(w));
      },
      /*native_dist=*/true);
}
