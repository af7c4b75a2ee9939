// jubabandit, native: multi-armed bandits without Python.
//
// Reference: jubatus/server/server/bandit_serv.cpp:51-110 (register_arm,
// delete_arm, select_arm, register_reward, get_arm_info, reset, clear) over
// jubatus_core's bandit; configs config/bandit/*.json. Same rules as
// models/bandit.py (its docstring lists them): per player and arm
// (trial_count, weight = cumulative reward); assume_unrewarded counts a
// selection as a trial at once; ucb1 tries untried arms first (registration
// order) then argmax mean + sqrt(2 ln total / n); epsilon_greedy, softmax
// (P ~ exp(mean / tau)) and exp3 (P = (1-gamma) w / sum w + gamma / K, w_i *=
// exp(gamma r / (P_i K)) on reward, kept as log weights). Standalone only:
// the MIX deltas of the Python driver are folded into one table here, which
// is also what its pack() writes, so model files move both ways.
#include <math.h>

#include <algorithm>
#include <map>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "jb_host_server.hpp"

namespace {

using namespace jb::srv;

struct Params {
  std::string method;
  bool assume_unrewarded = false;
  double epsilon = 0.1, tau = 0.05, gamma = 0.1;
  bool has_seed = false;
  uint64_t seed = 0;
};

bool parse_params(const std::string& text, Params* p, std::string* why) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  p->method = v.str_or("method", "");
  if (p->method != "ucb1" && p->method != "epsilon_greedy" && p->method != "softmax" && p->method != "exp3") {
    *why = "unsupported bandit method: " + p->method;
    return false;
  }
  const Value* par = v.get("parameter");
  const Value* au = par ? par->get("assume_unrewarded") : nullptr;
  if (!au) { *why = "bandit parameter requires assume_unrewarded"; return false; }
  p->assume_unrewarded = au->kind == Value::BOOL ? au->b : (au->is_num() && au->num() != 0);
  auto num = [&](const char* k, double* out) {
    const Value* x = par->get(k);
    if (x && x->is_num()) *out = x->num();
  };
  num("epsilon", &p->epsilon);
  num("tau", &p->tau);
  num("gamma", &p->gamma);
  if (const Value* s = par->get("seed"); s && (s->kind == Value::INT || s->kind == Value::UINT)) {
    p->has_seed = true;
    p->seed = s->kind == Value::INT ? (uint64_t)s->i : s->u;
  }
  if (p->method == "epsilon_greedy" && !(p->epsilon >= 0 && p->epsilon <= 1)) {
    *why = "epsilon must be in [0, 1]";
    return false;
  }
  if (p->method == "softmax" && !(p->tau > 0)) { *why = "tau must be positive"; return false; }
  if (p->method == "exp3" && !(p->gamma > 0 && p->gamma <= 1)) { *why = "gamma must be in (0, 1]"; return false; }
  return true;
}

struct ArmInfo {
  int64_t n = 0;
  double w = 0;
};

class Bandit : public HostEngine {
 public:
  explicit Bandit(const Params& p) : p_(p), rng_(p.has_seed ? p.seed : std::random_device{}()) {}

  std::vector<HostMethod> methods() override {
    return {
        {"register_arm", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const std::string& arm = arg_str(a[0]);
           if (std::find(arms_.begin(), arms_.end(), arm) != arms_.end()) { w->boolean(false); return; }
           arms_.push_back(arm);
           w->boolean(true);
         }},
        {"delete_arm", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const std::string& arm = arg_str(a[0]);
           auto it = std::find(arms_.begin(), arms_.end(), arm);
           if (it == arms_.end()) { w->boolean(false); return; }
           arms_.erase(it);
           for (auto& kv : info_) kv.second.erase(arm);
           for (auto& kv : logw_) kv.second.erase(arm);
           for (auto& kv : dinfo_) kv.second.erase(arm);
           for (auto& kv : dlogw_) kv.second.erase(arm);
           w->boolean(true);
         }},
        {"select_arm", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const std::string& player = arg_str(a[0]);
           if (arms_.empty()) throw EngineError("select_arm: no arm registered");
           const std::string arm = choose(player);
           if (p_.assume_unrewarded) {
             info_[player][arm].n += 1;
             dinfo_[player][arm].n += 1;
           }
           w->raw(arm);
         }},
        {"register_reward", 4, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const std::string& player = arg_str(a[0]);
           const std::string& arm = arg_str(a[1]);
           const double r = arg_num(a[2]);
           auto it = std::find(arms_.begin(), arms_.end(), arm);
           if (it == arms_.end()) { w->boolean(false); return; }
           if (p_.method == "exp3") {
             const double pr = exp3_probs(player)[(size_t)(it - arms_.begin())];
             const double dl = p_.gamma * (r / pr) / (double)arms_.size();
             logw_[player][arm] += dl;
             dlogw_[player][arm] += dl;
           }
           for (ArmInfo* ai : {&info_[player][arm], &dinfo_[player][arm]}) {
             ai->n += p_.assume_unrewarded ? 0 : 1;
             ai->w += r;
           }
           w->boolean(true);
         }},
        {"get_arm_info", 2, false, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const std::string& player = arg_str(a[0]);
           w->map(arms_.size());
           for (const auto& arm : arms_) {
             const ArmInfo ai = get(player, arm);
             w->raw(arm);
             w->arr(2);
             w->sint(ai.n);
             w->dbl(ai.w);
           }
         }},
        {"reset", 2, true, [this](const std::vector<Value>& a, MsgpackWriter* w) {
           const std::string& player = arg_str(a[0]);
           info_.erase(player);
           logw_.erase(player);
           dinfo_.erase(player);
           dlogw_.erase(player);
           w->boolean(true);
         }},
        {"clear", 1, true, [this](const std::vector<Value>&, MsgpackWriter* w) {
           clear();
           w->boolean(true);
         }},
    };
  }

  void clear() override {
    arms_.clear();
    info_.clear();
    logw_.clear();
    dinfo_.clear();
    dlogw_.clear();
  }

  // ---- MIX (models/bandit.py get_diff / mix_diff / put_diff): each member
  // ships its arm list and the (trial, reward) / exp3 log-weight increments
  // since the last MIX; every member adds the cluster's increments
  bool mixable() const override { return true; }
  bool uses_cht() const override { return true; }
  std::string get_diff() override {
    MsgpackWriter u;
    u.arr(3);
    u.arr(arms_.size());
    for (const auto& a : arms_) u.str(a);
    u.map(dinfo_.size());
    for (const auto& pp : dinfo_) {
      u.str(pp.first);
      u.map(pp.second.size());
      for (const auto& aa : pp.second) {
        u.str(aa.first);
        u.arr(2);
        u.sint(aa.second.n);
        u.dbl(aa.second.w);
      }
    }
    u.map(dlogw_.size());
    for (const auto& pp : dlogw_) {
      u.str(pp.first);
      u.map(pp.second.size());
      for (const auto& aa : pp.second) { u.str(aa.first); u.dbl(aa.second); }
    }
    return std::move(u.out);
  }
  void put_diffs(const std::vector<Value>& parts) override {
    for (const Value& d : parts)
      if (d.kind != Value::ARR || d.a.size() != 3) throw std::runtime_error("mix: malformed bandit diff");
    for (const Value& d : parts)
      for (const Value& a : d.a[0].a)
        if (std::find(arms_.begin(), arms_.end(), a.s) == arms_.end()) arms_.push_back(a.s);
    // my totals already hold my increments: add everyone's, less mine
    for (const auto& pp : dinfo_)
      for (const auto& aa : pp.second) {
        ArmInfo& t = info_[pp.first][aa.first];
        t.n -= aa.second.n;
        t.w -= aa.second.w;
      }
    for (const auto& pp : dlogw_)
      for (const auto& aa : pp.second) logw_[pp.first][aa.first] -= aa.second;
    for (const Value& d : parts) {
      for (const auto& pp : d.a[1].o)
        for (const auto& aa : pp.second.o) {
          ArmInfo& t = info_[pp.first][aa.first];
          t.n += (int64_t)aa.second.a.at(0).num();
          t.w += aa.second.a.at(1).num();
        }
      for (const auto& pp : d.a[2].o)
        for (const auto& aa : pp.second.o) logw_[pp.first][aa.first] += aa.second.num();
    }
    dinfo_.clear();
    dlogw_.clear();
  }

  // models/bandit.py pack(): {"method", "arms", "info": {player: {arm: [n, w]}}, "exp3": {player: {arm: logw}}}
  std::string pack() override {
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(4);
    u.str("method"); u.str(p_.method);
    u.str("arms"); u.arr(arms_.size());
    for (const auto& a : arms_) u.str(a);
    u.str("info"); u.map(info_.size());
    for (const auto& pl : info_) {
      u.str(pl.first);
      u.map(pl.second.size());
      for (const auto& kv : pl.second) { u.str(kv.first); u.arr(2); u.sint(kv.second.n); u.dbl(kv.second.w); }
    }
    u.str("exp3"); u.map(logw_.size());
    for (const auto& pl : logw_) {
      u.str(pl.first);
      u.map(pl.second.size());
      for (const auto& kv : pl.second) { u.str(kv.first); u.dbl(kv.second); }
    }
    return std::move(u.out);
  }

  void unpack(const Value& obj) override {
    const Value* av = obj.get("arms");
    const Value* iv = obj.get("info");
    const Value* ev = obj.get("exp3");
    if (!av || av->kind != Value::ARR || !iv || iv->kind != Value::MAP || !ev || ev->kind != Value::MAP)
      throw std::runtime_error("broken model data: bandit");
    clear();
    for (const Value& a : av->a) arms_.push_back(a.s);
    for (const auto& pl : iv->o)
      for (const auto& kv : pl.second.o) {
        if (kv.second.kind != Value::ARR || kv.second.a.size() != 2)
          throw std::runtime_error("broken model data: arm_info");
        ArmInfo& ai = info_[pl.first][kv.first];
        ai.n = (int64_t)kv.second.a[0].num();
        ai.w = kv.second.a[1].num();
      }
    for (const auto& pl : ev->o)
      for (const auto& kv : pl.second.o) logw_[pl.first][kv.first] = kv.second.num();
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) override {
    st->emplace_back("method", p_.method);
    st->emplace_back("num_arms", std::to_string(arms_.size()));
    st->emplace_back("num_players", std::to_string(info_.size()));
  }

 private:
  ArmInfo get(const std::string& player, const std::string& arm) const {
    auto p = info_.find(player);
    if (p == info_.end()) return ArmInfo{};
    auto a = p->second.find(arm);
    return a == p->second.end() ? ArmInfo{} : a->second;
  }
  double mean(const std::string& player, const std::string& arm) const {
    const ArmInfo ai = get(player, arm);
    return ai.n > 0 ? ai.w / (double)ai.n : 0.0;
  }
  double logw(const std::string& player, const std::string& arm) const {
    auto p = logw_.find(player);
    if (p == logw_.end()) return 0.0;
    auto a = p->second.find(arm);
    return a == p->second.end() ? 0.0 : a->second;
  }
  std::vector<double> exp3_probs(const std::string& player) const {
    std::vector<double> lw;
    for (const auto& a : arms_) lw.push_back(logw(player, a));
    const double m = *std::max_element(lw.begin(), lw.end());
    double s = 0;
    for (double& x : lw) { x = exp(x - m); s += x; }
    const double k = (double)arms_.size();
    for (double& x : lw) x = (1.0 - p_.gamma) * x / s + p_.gamma / k;
    return lw;
  }
  size_t draw(const std::vector<double>& weights) {
    std::discrete_distribution<size_t> d(weights.begin(), weights.end());
    return d(rng_);
  }
  size_t argmax(const std::vector<double>& v) const {   // first index of the maximum
    size_t b = 0;
    for (size_t i = 1; i < v.size(); ++i)
      if (v[i] > v[b]) b = i;
    return b;
  }
  std::string choose(const std::string& player) {
    if (p_.method == "ucb1") {
      int64_t total = 0;
      for (const auto& a : arms_) {
        const ArmInfo ai = get(player, a);
        if (ai.n == 0) return a;
        total += ai.n;
      }
      std::vector<double> sc;
      for (const auto& a : arms_) {
        const ArmInfo ai = get(player, a);
        sc.push_back(ai.w / (double)ai.n + sqrt(2.0 * log((double)total) / (double)ai.n));
      }
      return arms_[argmax(sc)];
    }
    if (p_.method == "epsilon_greedy") {
      std::uniform_real_distribution<double> u(0.0, 1.0);
      if (u(rng_) < p_.epsilon) {
        std::uniform_int_distribution<size_t> pick(0, arms_.size() - 1);
        return arms_[pick(rng_)];
      }
      std::vector<double> m;
      for (const auto& a : arms_) m.push_back(mean(player, a));
      return arms_[argmax(m)];
    }
    if (p_.method == "softmax") {
      std::vector<double> m;
      for (const auto& a : arms_) m.push_back(mean(player, a) / p_.tau);
      const double mx = *std::max_element(m.begin(), m.end());
      for (double& x : m) x = exp(x - mx);
      return arms_[draw(m)];
    }
    return arms_[draw(exp3_probs(player))];
  }

  Params p_;
  std::mt19937_64 rng_;
  std::vector<std::string> arms_;
  std::map<std::string, std::map<std::string, ArmInfo>> info_;
  std::map<std::string, std::map<std::string, double>> logw_;
  // increments since the last MIX (distributed mode)
  std::map<std::string, std::map<std::string, ArmInfo>> dinfo_;
  std::map<std::string, std::map<std::string, double>> dlogw_;
};

}  // namespace

int main(int argc, char** argv) {
  return host_main(
      argc, argv, "bandit",
      [](const std::string& text, std::string* why) {
        Params p;
        return parse_params(text, &p, why);
      },
      [](const std::string& text) -> std::unique_ptr<HostEngine> {
        Params p;
        std::string why;
        if (!parse_params(text, &p, &why)) throw std::runtime_error(why);
        return std::unique_ptr<HostEngine>(new Bandit(p));
      },
      /*native_dist=*/true);
}
