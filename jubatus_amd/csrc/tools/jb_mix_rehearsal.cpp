// jb_mix_rehearsal: a host-only server process that runs the native model
// plane (csrc/native/jb_mix_group.hpp: coordinator membership, group epochs,
// control-plane star, trigger agreement, obsolete hand-over, watchdog) over a
// small linear model in host memory, with the same MIX protocol as the native
// jubaclassifier's device tables (label agreement by name, count deltas,
// touched-row union by MAX all-reduce, sparse / dense SUM all-reduce of
// [W | S] rows, fold T += mean - snapshot). Lets a CPU-only host rehearse the
// distributed protocol with any number of ranks (tests/test_native_mix.py).
//
// RPC (msgpack-RPC, first argument the cluster name as every server):
//   train(name, seed, n, nlabels) -> n   n pseudo-random updates
//   model(name) -> {label: [count, [W column], [S column]]}
//   do_mix(name) -> bool                 force a MIX and wait for it
//   get_status(name) -> {ident: {key: value}}
//
// With -R the process is a row engine instead (recommender / nearest_neighbor
// / anomaly): a host row store under the row-diff MIX protocol the native
// GPU row servers run (csrc/server/jb_row_mix.hpp - the same code):
//   put(name, seed, n, keys) -> n       n rows written (ids from a keyspace)
//   remove(name, id) -> bool
//   rows(name) -> {id: [version, x]}    the store (x: the row's "x" value)
//   apply_raw(name, bytes) -> n         apply one msgpack row diff as a MIX would
//
// usage: jb_mix_rehearsal -z host:port -n name -p port [-H rows] [-I ic_timeout]
//                         [-i interval_count] [-s interval_sec] [-Z zk_timeout] [-R]
#include <getopt.h>
#include <signal.h>

#include <map>
#include <set>
#include <unordered_map>
#include <unordered_set>

#include "jb_mix_group.hpp"
#include "jb_msgpack.hpp"
#include "jb_row_mix.hpp"
#include "jb_rpc.hpp"

namespace {

using jubatus_amd::mp::Value;
using jb::mix::Group;

std::string resp_ok(uint32_t id, const Value& v) {
  std::string o;
  o.push_back((char)0x94);
  o.push_back((char)0x01);
  jb::cc::put_u32(o, id);
  o.push_back((char)0xc0);
  jubatus_amd::mp::encode(v, o);
  return o;
}
std::string resp_err(uint32_t id, const std::string& msg) {
  std::string o;
  o.push_back((char)0x94);
  o.push_back((char)0x01);
  jb::cc::put_u32(o, id);
  jb::cc::put_raw(o, msg);
  o.push_back((char)0xc0);
  return o;
}

class HostModel : public jb::mix::Mixable {
 public:
  static constexpr int LC = 16;
  explicit HostModel(int64_t H) : H_(H), W_((size_t)H * LC, 0.f), S_((size_t)H * LC, 1.f), touched_((size_t)H, 1) {}

  int64_t train(uint64_t seed, int64_t n, int nlabels) {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
    for (int64_t i = 0; i < n; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      const int64_t row = (int64_t)(x % (uint64_t)H_);
      const std::string lab = "l" + std::to_string((x >> 20) % (uint64_t)std::max(1, nlabels));
      const int col = column(lab);
      if (col < 0) throw std::runtime_error("label table full");
      W_[(size_t)row * LC + col] += (float)((int64_t)((x >> 32) % 2001) - 1000) / 1000.f;
      S_[(size_t)row * LC + col] *= 0.9f;
      touched_[(size_t)row] = 1;
      counts_[col] += 1;
    }
    return n;
  }

  Value model() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<Value, Value>> m;
    for (size_t c = 0; c < names_.size(); ++c) {
      std::vector<Value> w, s;
      for (int64_t r = 0; r < H_; ++r) {
        w.push_back(Value::real(W_[(size_t)r * LC + c]));
        s.push_back(Value::real(S_[(size_t)r * LC + c]));
      }
      m.emplace_back(Value::str(names_[c]), Value::array({Value::uinteger(counts_[c]), Value::array(std::move(w)),
                                                          Value::array(std::move(s))}));
    }
    return Value::map(std::move(m));
  }

  // --------------------------------------------- the classifier's MIX, on the host
  uint64_t mix(Group& grp) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    std::string mine;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& n : names_) put_name(&mine, n);
    }
    const auto parts = star.allgather(mine, grp.deadline());
    std::vector<std::string> canon;
    std::set<std::string> seen;
    for (const auto& p : parts)
      for (auto& n : get_names(p))
        if (seen.insert(n).second) canon.push_back(n);
    const int Lc = (int)canon.size();
    std::vector<int> map(Lc);
    std::vector<int64_t> delta(Lc);
    std::vector<uint64_t> cur_at(Lc);
    std::vector<uint8_t> mark;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int c = 0; c < Lc; ++c) {
        map[c] = column(canon[c]);
        if (map[c] < 0) throw std::runtime_error("label table full");
        cur_at[c] = counts_[map[c]];
        delta[c] = (int64_t)cur_at[c] - (int64_t)base_[canon[c]];
      }
      mark.swap(touched_);
      touched_.assign((size_t)H_, 0);
    }
    star.allreduce_sum(delta.data(), (size_t)Lc, grp.deadline());
    pl.allreduce_max(mark.data(), mark.size(), grp.deadline());
    std::vector<int64_t> rows;
    for (int64_t r = 0; r < H_; ++r)
      if (mark[(size_t)r]) rows.push_back(r);
    const bool dense = (int64_t)rows.size() * 2 > H_;
    if (dense) {
      rows.resize((size_t)H_);
      for (int64_t r = 0; r < H_; ++r) rows[(size_t)r] = r;
    }
    uint64_t bytes = (uint64_t)H_ + 8ull * Lc;
    const size_t width = 2 * (size_t)Lc;
    std::vector<float> snap(rows.size() * width), red;
    if (!rows.empty() && Lc > 0) {
      {
        std::lock_guard<std::mutex> g(mu_);
        for (size_t i = 0; i < rows.size(); ++i)
          for (int c = 0; c < Lc; ++c) {
            snap[i * width + c] = W_[(size_t)rows[i] * LC + map[c]];
            snap[i * width + Lc + c] = S_[(size_t)rows[i] * LC + map[c]];
          }
      }
      red = snap;
      pl.allreduce_sum(red.data(), red.size(), grp.deadline());
      bytes += red.size() * 4;
      std::lock_guard<std::mutex> g(mu_);
      const float inv = 1.f / (float)grp.world();
      for (size_t i = 0; i < rows.size(); ++i)
        for (int c = 0; c < Lc; ++c) {
          W_[(size_t)rows[i] * LC + map[c]] += red[i * width + c] * inv - snap[i * width + c];
          S_[(size_t)rows[i] * LC + map[c]] += red[i * width + Lc + c] * inv - snap[i * width + Lc + c];
        }
    }
    std::lock_guard<std::mutex> g(mu_);
    for (int c = 0; c < Lc; ++c) {
      const uint64_t nb = (uint64_t)((int64_t)base_[canon[c]] + delta[c]);
      counts_[map[c]] = nb + (counts_[map[c]] - cur_at[c]);
      base_[canon[c]] = nb;
    }
    last_rows_ = rows.size();
    last_dense_ = dense;
    return bytes;
  }

  // --------------------------------------------- the classifier's push MIX, on the host
  // (jubaclassifier.cpp pair_mix: label agreement with the peer, the pair's
  // row union - kept for the MIX's later rounds - and the pairwise mean)
  bool push_mixable() const override { return true; }
  void push_begin() override {
    std::lock_guard<std::mutex> g(mu_);
    pmark_.swap(touched_);
    touched_.assign((size_t)H_, 0);
  }
  uint64_t pair_mix(Group& grp, int peer) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    const double dl = grp.deadline();
    std::string mine;
    if (peer >= 0) {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& n : names_) put_name(&mine, n);
    }
    const std::string theirs = pl.exchange_bytes(star, peer, mine, dl);
    if (peer < 0) {
      pl.pair_max(star, nullptr, 0, -1, dl);
      pl.exchange_bytes(star, -1, std::string(), dl);
      pl.pair_sum(star, nullptr, 0, -1, dl);
      return 0;
    }
    std::vector<std::string> canon;
    std::set<std::string> seen;
    for (const std::string* p : {grp.rank() < peer ? &mine : &theirs, grp.rank() < peer ? &theirs : &mine})
      for (auto& n : get_names(*p))
        if (seen.insert(n).second) canon.push_back(n);
    const int Lc = (int)canon.size();
    std::vector<int> map(Lc);
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int c = 0; c < Lc; ++c) {
        map[c] = column(canon[c]);
        if (map[c] < 0) throw std::runtime_error("label table full");
      }
    }
    pl.pair_max(star, pmark_.data(), pmark_.size(), peer, dl);
    std::vector<int64_t> rows;
    for (int64_t r = 0; r < H_; ++r)
      if (pmark_[(size_t)r]) rows.push_back(r);
    const size_t width = 2 * (size_t)Lc;
    std::vector<float> snap(rows.size() * width);
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i = 0; i < rows.size(); ++i)
        for (int c = 0; c < Lc; ++c) {
          snap[i * width + c] = W_[(size_t)rows[i] * LC + map[c]];
          snap[i * width + Lc + c] = S_[(size_t)rows[i] * LC + map[c]];
        }
    }
    const std::string ok = pl.exchange_bytes(star, peer, "1", dl);
    std::vector<float> red = snap;
    pl.pair_sum(star, red.data(), red.size(), ok == "1" ? peer : -1, dl);
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < rows.size(); ++i)
      for (int c = 0; c < Lc; ++c) {
        W_[(size_t)rows[i] * LC + map[c]] += red[i * width + c] * 0.5f - snap[i * width + c];
        S_[(size_t)rows[i] * LC + map[c]] += red[i * width + Lc + c] * 0.5f - snap[i * width + Lc + c];
      }
    last_rows_ = rows.size();
    last_dense_ = false;
    return (uint64_t)H_ + red.size() * 4;
  }

  void hand_over(Group& grp, int src, bool apply) override {
    std::string meta;
    std::vector<float> w, s;
    if (grp.rank() == src) {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t c = 0; c < names_.size(); ++c) {
        put_name(&meta, names_[c]);
        meta.append((const char*)&counts_[c], 8);
      }
      w = W_;
      s = S_;
    } else {
      w.assign(W_.size(), 0.f);
      s.assign(S_.size(), 0.f);
    }
    meta = grp.star().bcast_str(src, meta, grp.deadline());
    grp.plane().bcast(w.data(), w.size() * 4, src, grp.deadline());
    grp.plane().bcast(s.data(), s.size() * 4, src, grp.deadline());
    if (!apply || grp.rank() == src) return;
    std::lock_guard<std::mutex> g(mu_);
    names_.clear();
    counts_.assign(LC, 0);
    base_.clear();
    size_t o = 0;
    while (o < meta.size()) {
      const std::string n = take_name(meta, &o);
      uint64_t cnt;
      memcpy(&cnt, meta.data() + o, 8);
      o += 8;
      names_.push_back(n);
      counts_[names_.size() - 1] = cnt;
      base_[n] = cnt;
    }
    W_ = w;
    S_ = s;
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) {
    std::lock_guard<std::mutex> g(mu_);
    st->emplace_back("mix.last_rows", std::to_string(last_rows_));
    st->emplace_back("mix.last_mode", last_dense_ ? "dense" : "sparse");
    st->emplace_back("num_labels", std::to_string(names_.size()));
  }

 private:
  int column(const std::string& n) {   // mu_ held
    for (size_t c = 0; c < names_.size(); ++c)
      if (names_[c] == n) return (int)c;
    if ((int)names_.size() >= LC) return -1;
    names_.push_back(n);
    return (int)names_.size() - 1;
  }
  static void put_name(std::string* o, const std::string& n) {
    const uint32_t k = (uint32_t)n.size();
    o->append((const char*)&k, 4);
    *o += n;
  }
  static std::string take_name(const std::string& b, size_t* o) {
    uint32_t k;
    if (*o + 4 > b.size()) throw std::runtime_error("broken label list");
    memcpy(&k, b.data() + *o, 4);
    *o += 4;
    if (*o + k > b.size()) throw std::runtime_error("broken label list");
    std::string n = b.substr(*o, k);
    *o += k;
    return n;
  }
  static std::vector<std::string> get_names(const std::string& b) {
    std::vector<std::string> out;
    size_t o = 0;
    while (o < b.size()) out.push_back(take_name(b, &o));
    return out;
  }

  std::mutex mu_;
  int64_t H_;
  std::vector<float> W_, S_;
  std::vector<uint8_t> touched_, pmark_;   // pmark_: rows of the push MIX under way
  std::vector<std::string> names_;
  std::vector<uint64_t> counts_ = std::vector<uint64_t>(LC, 0);
  std::map<std::string, uint64_t> base_;
  uint64_t last_rows_ = 0;
  bool last_dense_ = false;
};

// A row store with versions (models/rows.py semantics) under the shared
// row-diff protocol: every write bumps the row's version and marks it
// written, a removal bumps it and records the removal.
class HostRowModel : public jb::mix::Mixable {
 public:
  struct Row {
    jb::row::Datum d;
    std::vector<int32_t> idx;
    std::vector<float> val;
    int32_t slot;
  };

  int64_t put(uint64_t seed, int64_t n, int64_t keys) {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 7;
    for (int64_t i = 0; i < n; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      const int64_t k = (int64_t)(x % (uint64_t)std::max<int64_t>(1, keys));
      const std::string id = "r" + std::to_string(k);
      Row r;
      r.d.sv["x"] = std::to_string(x % 100000);
      r.d.nv["v"] = (double)(x % 1000) / 10.0;
      r.idx = {(int32_t)(k % 97), (int32_t)(x % 1021)};
      r.val = {1.f, (float)(x % 7)};
      write(id, std::move(r));
      ++version_[id];
      dirty_.insert(id);
      removed_.erase(id);
    }
    return n;
  }
  bool remove(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    if (!rows_.erase(id)) return false;
    ++version_[id];
    removed_.insert(id);
    dirty_.erase(id);
    return true;
  }
  Value rows() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<Value, Value>> m;
    for (const auto& kv : rows_)
      m.emplace_back(Value::str(kv.first), Value::array({Value::uinteger(version_[kv.first]),
                                                          Value::str(kv.second.d.sv.at("x"))}));
    return Value::map(std::move(m));
  }

  uint64_t mix(Group& grp) override {
    std::lock_guard<std::mutex> g(mu_);
    jb::val::MsgpackWriter w;
    jb::row::pack_row_diff(*this, w);
    const auto raw = grp.plane().allgather_bytes(grp.star(), w.out, grp.deadline());
    std::vector<jb::val::Value> parts;
    for (const auto& r : raw) parts.push_back(jb::val::MsgpackReader((const uint8_t*)r.data(), r.size()).read());
    last_applied_ = jb::row::apply_row_diffs(*this, parts, nullptr);
    uint64_t bytes = 0;
    for (const auto& r : raw) bytes += r.size();
    return bytes;
  }
  // one peer diff applied as a MIX would (tests feed malformed diffs here)
  size_t apply_raw(const std::string& raw) {
    std::lock_guard<std::mutex> g(mu_);
    return jb::row::apply_row_diffs(*this, {jb::val::MsgpackReader((const uint8_t*)raw.data(), raw.size()).read()},
                                    nullptr);
  }
  // push mixers: the pair folds its two diffs, lower rank first
  uint64_t pair_mix(Group& grp, int peer) override {
    std::lock_guard<std::mutex> g(mu_);
    jb::val::MsgpackWriter w;
    if (peer >= 0) jb::row::pack_row_diff(*this, w);
    const std::string theirs = grp.plane().exchange_bytes(grp.star(), peer, w.out, grp.deadline());
    if (peer < 0) return 0;
    jb::val::Value a = jb::val::MsgpackReader((const uint8_t*)w.out.data(), w.out.size()).read();
    jb::val::Value b = jb::val::MsgpackReader((const uint8_t*)theirs.data(), theirs.size()).read();
    std::vector<jb::val::Value> parts;
    if (grp.rank() < peer) { parts.push_back(a); parts.push_back(b); }
    else { parts.push_back(b); parts.push_back(a); }
    last_applied_ = jb::row::apply_row_diffs(*this, parts, nullptr, /*forward=*/true);
    return w.out.size();
  }
  bool push_mixable() const override { return true; }
  void push_end() override {
    std::lock_guard<std::mutex> g(mu_);
    mix_done();
  }

  // obsolete protocol: rank src's whole store (every row as written) replaces mine
  void hand_over(Group& grp, int src, bool apply) override {
    std::lock_guard<std::mutex> g(mu_);
    jb::val::MsgpackWriter w;
    if (grp.rank() == src) {
      full_ = true;
      jb::row::pack_row_diff(*this, w);
      full_ = false;
    }
    const std::string got = grp.plane().bcast_bytes(grp.star(), src, w.out, grp.deadline());
    if (!apply || grp.rank() == src) return;
    rows_.clear();
    version_.clear();
    dirty_.clear();
    removed_.clear();
    jb::row::apply_row_diffs(*this, {jb::val::MsgpackReader((const uint8_t*)got.data(), got.size()).read()},
                             nullptr);
  }
  void status(std::vector<std::pair<std::string, std::string>>* st) {
    std::lock_guard<std::mutex> g(mu_);
    st->emplace_back("num_rows", std::to_string(rows_.size()));
    st->emplace_back("mix.last_rows_applied", std::to_string(last_applied_));
  }

  // ---- the store interface of jb_row_mix.hpp (mu_ held by the caller)
  std::vector<std::string> mix_ids() const {
    std::vector<std::string> ids;
    if (full_) {
      for (const auto& kv : rows_) ids.push_back(kv.first);
    } else {
      for (const auto& id : dirty_)
        if (rows_.count(id)) ids.push_back(id);
    }
    std::sort(ids.begin(), ids.end());
    return ids;
  }
  std::vector<std::string> mix_removed() const {
    if (full_) return {};
    std::vector<std::string> v(removed_.begin(), removed_.end());
    std::sort(v.begin(), v.end());
    return v;
  }
  bool version_of(const std::string& id, uint64_t* v) const {
    auto it = version_.find(id);
    if (it == version_.end()) { *v = 0; return false; }
    *v = it->second;
    return true;
  }
  bool holds(const std::string& id) const { return rows_.count(id) != 0; }
  void row_view(const std::string& id, const jb::row::Datum** d, const std::vector<int32_t>** ix,
                const std::vector<float>** vx) const {
    const Row& r = rows_.at(id);
    *d = &r.d;
    *ix = &r.idx;
    *vx = &r.val;
  }
  int32_t slot_id(const std::string& id) const {
    auto it = rows_.find(id);
    return it == rows_.end() ? -1 : it->second.slot;
  }
  void store_mixed(const std::string& id, jb::row::Datum&& d, const std::vector<int32_t>& idx,
                   const std::vector<float>& val, uint64_t v, bool forward) {
    Row r;
    r.d = std::move(d);
    r.idx = idx;
    r.val = val;
    write(id, std::move(r));
    version_[id] = v;
    if (forward) { dirty_.insert(id); removed_.erase(id); }
  }
  void remove_mixed(const std::string& id, uint64_t v, bool forward) {
    rows_.erase(id);
    version_[id] = v;
    if (forward) { removed_.insert(id); dirty_.erase(id); }
  }
  bool weight_diff(int64_t* docs, int64_t* len, std::vector<int64_t>*, std::vector<int64_t>*) const {
    *docs = *len = 0;
    return false;
  }
  void put_weight_diff(int64_t, int64_t, const std::vector<int64_t>&, const std::vector<int64_t>&, bool) {}
  void mix_done() {
    dirty_.clear();
    removed_.clear();
  }

 private:
  void write(const std::string& id, Row&& r) {
    auto it = rows_.find(id);
    r.slot = it != rows_.end() ? it->second.slot : next_slot_++;
    rows_[id] = std::move(r);
  }
  std::mutex mu_;
  std::unordered_map<std::string, Row> rows_;
  std::unordered_map<std::string, uint64_t> version_;
  std::unordered_set<std::string> dirty_, removed_;   // (sorted when packed)
  int32_t next_slot_ = 0;
  bool full_ = false;
  size_t last_applied_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
  std::string zk, name;
  int port = 0, H = 1024, ic = 10, icount = 0, isec = 0, zkt = 10;
  bool rows_mode = false;
  std::string kind = "linear_mixer";
  int c;
  while ((c = getopt(argc, argv, "z:n:p:H:I:i:s:Z:Rx:")) != -1) {
    switch (c) {
      case 'R': rows_mode = true; break;
      case 'x': kind = optarg; break;
      case 'z': zk = optarg; break;
      case 'n': name = optarg; break;
      case 'p': port = atoi(optarg); break;
      case 'H': H = atoi(optarg); break;
      case 'I': ic = atoi(optarg); break;
      case 'i': icount = atoi(optarg); break;
      case 's': isec = atoi(optarg); break;
      case 'Z': zkt = atoi(optarg); break;
      default: fprintf(stderr, "usage: %s -z zk -n name -p port [-H rows]\n", argv[0]); return 2;
    }
  }
  if (zk.empty() || name.empty() || port <= 0) {
    fprintf(stderr, "usage: %s -z zk -n name -p port [-H rows]\n", argv[0]);
    return 2;
  }
  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGTERM);
  sigaddset(&set, SIGINT);
  pthread_sigmask(SIG_BLOCK, &set, nullptr);
  signal(SIGPIPE, SIG_IGN);

  HostModel model(H);
  HostRowModel rmodel;
  jb::mix::Mixable* mixable = rows_mode ? (jb::mix::Mixable*)&rmodel : (jb::mix::Mixable*)&model;
  std::unique_ptr<jb::mix::LinearMixer> mixer;
  const std::string ident = "127.0.0.1_" + std::to_string(port);
  jb::RpcServer rpc(
      [&](const jb::RpcRequest& r) -> std::string {
        try {
          jubatus_amd::mp::Decoder d(r.params.data(), r.params.size());
          Value args;
          if (!d.next(args) || args.type != Value::ARRAY) return resp_err(r.msgid, "bad params");
          const auto& a = args.a;
          if (r.method == "train" && a.size() == 4) {
            const int64_t n = model.train(a[1].as_uint(), a[2].as_int(), (int)a[3].as_int());
            if (mixer) mixer->updated((uint64_t)n);
            return resp_ok(r.msgid, Value::integer(n));
          }
          if (r.method == "model") return resp_ok(r.msgid, model.model());
          if (r.method == "put" && a.size() == 4) {
            const int64_t n = rmodel.put(a[1].as_uint(), a[2].as_int(), a[3].as_int());
            if (mixer) mixer->updated((uint64_t)n);
            return resp_ok(r.msgid, Value::integer(n));
          }
          if (r.method == "remove" && a.size() == 2) {
            const bool ok = rmodel.remove(a[1].as_str());
            if (mixer && ok) mixer->updated(1);
            return resp_ok(r.msgid, Value::boolean(ok));
          }
          if (r.method == "rows") return resp_ok(r.msgid, rmodel.rows());
          if (r.method == "apply_raw" && a.size() == 2) {   // a peer's diff bytes, as a MIX receives them
            const std::string raw = a[1].as_str();
            return resp_ok(r.msgid, Value::integer((int64_t)rmodel.apply_raw(raw)));
          }
          if (r.method == "do_mix") return resp_ok(r.msgid, Value::boolean(mixer && mixer->do_mix()));
          if (r.method == "get_status") {
            std::vector<std::pair<std::string, std::string>> st;
            if (rows_mode) rmodel.status(&st);
            else model.status(&st);
            if (mixer) mixer->status(&st);
            std::vector<std::pair<Value, Value>> m;
            for (auto& kv : st) m.emplace_back(Value::str(kv.first), Value::str(kv.second));
            return resp_ok(r.msgid, Value::map({{Value::str(ident), Value::map(std::move(m))}}));
          }
          return resp_err(r.msgid, "no such method: " + r.method);
        } catch (const std::exception& e) {
          return resp_err(r.msgid, e.what());
        }
      },
      2, 0.0);
  rpc.listen("127.0.0.1", port);
  rpc.start();
  const char* type = rows_mode ? "recommender" : "classifier";
  jb::mix::ClusterNode node(zk, zkt, type, name);
  if (!node.config_rlock()) {
    fprintf(stderr, "failed to get config lock\n");
    return 1;
  }
  node.register_actor("127.0.0.1", port);
  jb::mix::MixerArgs ma;
  ma.kind = kind;
  ma.type = type;
  ma.name = name;
  ma.eth = "127.0.0.1";
  ma.port = port;
  ma.interval_sec = isec;
  ma.interval_count = icount;
  ma.interconnect_timeout = ic;
  mixer.reset(new jb::mix::LinearMixer(node.coord(), ma, mixable, [](Group& g, double) {
    return std::unique_ptr<jb::mix::Plane>(new jb::mix::HostPlane(&g.star()));
  }));
  mixer->start();
  fprintf(stderr, "jb_mix_rehearsal ready on %d\n", port);
  int sig = 0;
  while (sigwait(&set, &sig) != 0 || (sig != SIGTERM && sig != SIGINT)) {
  }
  mixer->stop();
  node.leave();
  rpc.stop();
  return 0;
}
