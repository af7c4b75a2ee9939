// RPC shell of the native host-engine servers (jubastat, jubabandit,
// jubaburst, jubagraph, jubaweight): the
// engines whose state is small per-key bookkeeping and stays on the host
// (SURVEY K14), served without Python. Reference: the generated
// <engine>_impl.cpp RPC tables and framework/server_base.cpp (save / load /
// get_status); the lock discipline of server_helper.hpp:296-303 (update =
// write lock, analysis = read lock) is a reader/writer mutex here.
//
// An engine supplies its methods (name, arity incl. the cluster name, update
// or analysis, handler writing the result), pack / unpack of its model
// payload (the same msgpack maps as the Python drivers, so model files move
// between the two servers) and its status keys.
//
// Distributed mode (-z, linear mixer): an engine that can mix supplies its
// diff and the fold of every member's diff (the Python drivers' get_diff /
// mix_diff / put_diff, folded in rank order on every member); the server
// joins the cluster (coordinator membership, config lock, actor node, CHT
// vnodes when the engine routes by CHT) and runs the native linear mixer
// (csrc/native/jb_mix_group.hpp): the diffs move as byte strings over the
// group's plane - the control plane for the host engines, RCCL all-gather
// for an engine with device state (clustering).
#pragma once
#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "jb_mix_group.hpp"
#include "jb_rpc.hpp"
#include "jb_server_common.hpp"
#include "jb_value.hpp"

namespace jb {
namespace srv {

struct HostMethod {
  std::string name;
  size_t arity;        // including the leading cluster name
  bool update;         // write lock + update_count
  std::function<void(const std::vector<Value>&, MsgpackWriter*)> fn;
  // optional zero-decode handler: the raw msgpack params array (arity
  // checked), for bulk payloads the engine reads in place (clustering push)
  std::function<void(const std::string&, MsgpackWriter*)> raw = nullptr;
  // the handler takes the model lock itself (HostEngine::set_lock): methods
  // that call other servers must not hold it meanwhile (graph_serv.cpp:
  // create_node / remove_node / create_edge)
  bool self_lock = false;
};

class HostEngine {
 public:
  virtual ~HostEngine() = default;
  virtual std::vector<HostMethod> methods() = 0;
  virtual std::string pack() = 0;                 // msgpack of the driver pack (bin types)
  virtual void unpack(const Value& obj) = 0;
  virtual void clear() = 0;
  virtual void status(std::vector<std::pair<std::string, std::string>>* st) = 0;
  // ---- distributed mode (model lock held exclusively by the caller)
  virtual bool mixable() const { return false; }
  virtual bool uses_cht() const { return false; }
  virtual std::string get_diff() { return std::string(); }            // msgpack
  virtual void put_diffs(const std::vector<Value>& parts) { (void)parts; }  // every rank's, rank order
  // one round of a push MIX ([own, partner] in rank order): engines whose
  // diffs are plain counts keep their own diff for the MIX's later partners
  // and drop it in push_done(); the default folds the pair like a linear MIX
  virtual void put_diffs_push(const std::vector<Value>& parts) { put_diffs(parts); }
  virtual void push_done() {}
  virtual std::unique_ptr<jb::mix::Plane> make_plane(jb::mix::Star& s, double dl) {
    (void)dl;
    return std::unique_ptr<jb::mix::Plane>(new jb::mix::HostPlane(&s));
  }
  // distributed mode: the cluster this server joined (its CHT, its
  // server-to-server peers) and its own address; called before serving and
  // again when a loaded model file replaces the engine
  virtual void attach(jb::mix::ClusterNode* node, const Args& a) {
    (void)node;
    (void)a;
  }
  // the server's model lock, for self_lock methods
  virtual void set_lock(std::shared_mutex* mu) { (void)mu; }
};

// a method error reported to the client as the message string
struct EngineError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class HostServer : public jb::mix::Mixable {
 public:
  // make(config text) -> engine, or throws (the config is validated first)
  using Factory = std::function<std::unique_ptr<HostEngine>(const std::string&)>;

  HostServer(const Args& a, const std::string& config, Factory make)
      : a_(a), config_(config), make_(std::move(make)) {
    eng_ = make_(config_);
    eng_->set_lock(&model_mu_);
    for (auto& m : eng_->methods()) table_.push_back(m);
  }

  void load_file(const std::string& path) { load_impl(path, true); }

  // distributed mode (-z): coordinator session, config read lock
  void join_cluster(std::unique_ptr<jb::mix::ClusterNode> node) {
    node_ = std::move(node);
    a_.connected_zookeeper = node_->connected();
    if (!node_->config_rlock()) throw std::runtime_error("failed to get config lock");
  }

  // ---- jb::mix::Mixable: one MIX / the obsolete hand-over (mixer thread)
  uint64_t mix(jb::mix::Group& g) override {
    std::unique_lock<std::shared_mutex> lk(model_mu_);
    const std::string mine = eng_->get_diff();
    const auto raw = g.plane().allgather_bytes(g.star(), mine, g.deadline());
    std::vector<Value> parts;
    uint64_t bytes = 0;
    for (const auto& r : raw) {
      parts.push_back(MsgpackReader((const uint8_t*)r.data(), r.size()).read());
      bytes += r.size();
    }
    eng_->put_diffs(parts);
    return bytes;
  }
  // push mixers: the pair folds its two diffs, lower rank first
  uint64_t pair_mix(jb::mix::Group& g, int peer) override {
    std::unique_lock<std::shared_mutex> lk(model_mu_);
    const std::string mine = peer >= 0 ? eng_->get_diff() : std::string();
    const std::string theirs = g.plane().exchange_bytes(g.star(), peer, mine, g.deadline());
    if (peer < 0) return 0;
    Value a = MsgpackReader((const uint8_t*)mine.data(), mine.size()).read();
    Value b = MsgpackReader((const uint8_t*)theirs.data(), theirs.size()).read();
    std::vector<Value> parts;
    if (g.rank() < peer) { parts.push_back(std::move(a)); parts.push_back(std::move(b)); }
    else { parts.push_back(std::move(b)); parts.push_back(std::move(a)); }
    eng_->put_diffs_push(parts);
    return mine.size();
  }
  bool push_mixable() const override { return true; }
  void push_end() override {
    std::unique_lock<std::shared_mutex> lk(model_mu_);
    eng_->push_done();
  }

  void hand_over(jb::mix::Group& g, int src, bool apply) override {
    std::string mine;
    if (g.rank() == src) {
      std::shared_lock<std::shared_mutex> lk(model_mu_);
      mine = eng_->pack();
    }
    const std::string got = g.plane().bcast_bytes(g.star(), src, mine, g.deadline());
    if (!apply || g.rank() == src) return;
    const Value v = MsgpackReader((const uint8_t*)got.data(), got.size()).read();
    if (v.kind != Value::ARR || v.a.size() != 2) throw std::runtime_error("hand-over: malformed model");
    std::unique_lock<std::shared_mutex> lk(model_mu_);
    eng_->unpack(v.a[1]);
  }

  int run() {
    rpc_.reset(new jb::RpcServer([this](const jb::RpcRequest& r) { return dispatch(r); }, a_.threads, 0.0));
    rpc_->set_io_threads(std::max(1, a_.threads / 4));
    int port;
    try {
      port = rpc_->listen(a_.bind, a_.port);
    } catch (const std::exception& e) {
      logf_("FATAL", "server failed to start: any process using port %d? (%s)", a_.port, e.what());
      return 1;
    }
    a_.port = port;
    if (node_) {
      std::unique_lock<std::shared_mutex> g(model_mu_);
      eng_->attach(node_.get(), a_);
    }
    logf_("INFO", "start listening at port %d", port);
    cs_.start_time = time(nullptr);
    rpc_->start();
    if (node_) {   // distributed mode: actor (+ CHT vnodes), then the mixer thread
      node_->register_actor(a_.eth, a_.port);
      if (eng_->uses_cht()) node_->register_cht(a_.eth, a_.port);
      jb::mix::MixerArgs ma;
      ma.kind = a_.mixer;
      ma.type = engine_name();
      ma.name = a_.name;
      ma.eth = a_.eth;
      ma.port = a_.port;
      ma.interval_sec = a_.interval_sec;
      ma.interval_count = a_.interval_count;
      ma.interconnect_timeout = a_.ic_timeout;
      mixer_.reset(new jb::mix::LinearMixer(node_->coord(), ma, this, [this](jb::mix::Group& g, double dl) {
        return eng_->make_plane(g.star(), dl);
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
  std::string local_path(const std::string& id) const {
    return a_.datadir + "/" + a_.eth + "_" + std::to_string(a_.port) + "_" + engine_name() + "_" + id +
           ".jubatus";
  }

  // elements of a params array header (-1: not an array)
  static int64_t params_count(const std::string& p) {
    if (p.empty()) return -1;
    const uint8_t t = (uint8_t)p[0];
    if ((t & 0xf0) == 0x90) return t & 0x0f;
    if (t == 0xdc && p.size() >= 3) return ((int64_t)(uint8_t)p[1] << 8) | (uint8_t)p[2];
    if (t == 0xdd && p.size() >= 5)
      return ((int64_t)(uint8_t)p[1] << 24) | ((int64_t)(uint8_t)p[2] << 16) | ((int64_t)(uint8_t)p[3] << 8) |
             (uint8_t)p[4];
    return -1;
  }

  std::string dispatch(const jb::RpcRequest& r) {
    for (const auto& x : table_) {
      if (x.name != r.method || !x.raw) continue;
      if (params_count(r.params) != (int64_t)x.arity)
        return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
      MsgpackWriter w;
      try {
        if (x.self_lock) {   // the handler takes model_mu_ itself (after its lock-free part)
          if (x.update) {
            if (mixer_) mixer_->updated(1);
            update_count_ += 1;
          }
          std::shared_lock<std::shared_mutex> life(life_mu_);   // (the engine is not replaced meanwhile)
          x.raw(r.params, &w);
        } else if (x.update) {
          if (mixer_) mixer_->updated(1);
          std::unique_lock<std::shared_mutex> g(model_mu_);
          update_count_ += 1;
          x.raw(r.params, &w);
        } else {
          std::shared_lock<std::shared_mutex> g(model_mu_);
          x.raw(r.params, &w);
        }
      } catch (const std::invalid_argument&) {
        return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
      } catch (const std::exception& e) {
        return r.notify ? std::string() : jb::val::response_msg(r.msgid, e.what());
      }
      return r.notify ? std::string() : jb::val::response_ok(r.msgid, w.out);
    }
    Value args;
    try {
      args = MsgpackReader((const uint8_t*)r.params.data(), r.params.size()).read();
    } catch (const std::exception&) {
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    }
    if (args.kind != Value::ARR) return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    MsgpackWriter w;
    try {
      const std::string& m = r.method;
      if (m == "do_mix" && mixer_) {
        if (args.a.size() != 1) return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
        w.boolean(mixer_->do_mix());
      } else if (m == "get_config" || m == "get_status" || m == "save" || m == "load") {
        const size_t want = (m == "save" || m == "load") ? 2 : 1;
        if (args.a.size() != want || (want == 2 && !args.a[1].is_str()))
          return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
        common(m, args, &w);
      } else {
        const HostMethod* hm = nullptr;
        for (const auto& x : table_)
          if (x.name == m) hm = &x;
        if (!hm) return r.notify ? std::string() : jb::val::response_code(r.msgid, kNoMethodError);
        if (args.a.size() != hm->arity)
          return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
        std::vector<Value> rest(args.a.begin() + 1, args.a.end());
        if (hm->self_lock) {
          if (hm->update) {
            if (mixer_) mixer_->updated(1);
            update_count_ += 1;
          }
          hm->fn(rest, &w);
        } else if (hm->update) {
          if (mixer_) mixer_->updated(1);
          std::unique_lock<std::shared_mutex> g(model_mu_);
          update_count_ += 1;
          hm->fn(rest, &w);
        } else {
          std::shared_lock<std::shared_mutex> g(model_mu_);
          hm->fn(rest, &w);
        }
      }
    } catch (const std::invalid_argument&) {
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    } catch (const std::exception& e) {
      return r.notify ? std::string() : jb::val::response_msg(r.msgid, e.what());
    }
    return r.notify ? std::string() : jb::val::response_ok(r.msgid, w.out);
  }

  void common(const std::string& m, const Value& args, MsgpackWriter* w) {
    if (m == "get_config") {
      w->raw(config_);
    } else if (m == "get_status") {
      std::vector<std::pair<std::string, std::string>> st;
      {
        std::lock_guard<std::mutex> g(st_mu_);
        common_status(a_, cs_, update_count_.load(), &st);
      }
      st.emplace_back("server_runtime", "native");
      {
        std::shared_lock<std::shared_mutex> g(model_mu_);
        eng_->status(&st);
      }
      if (mixer_) mixer_->status(&st);
      w->map(1);
      w->raw(ident());
      w->map(st.size());
      for (auto& kv : st) { w->raw(kv.first); w->raw(kv.second); }
    } else if (m == "save") {
      const std::string& id = args.a[1].s;
      if (id.empty()) throw std::runtime_error("empty id is not allowed");
      const std::string path = local_path(id);
      std::string user;
      {
        std::shared_lock<std::shared_mutex> g(model_mu_);
        user = eng_->pack();
      }
      write_model_file(path, engine_name(), id, config_, user);
      {
        std::lock_guard<std::mutex> g(st_mu_);
        cs_.last_saved = time(nullptr);
        cs_.last_saved_path = path;
      }
      logf_("INFO", "saved to %s", path.c_str());
      w->map(1);
      w->raw(ident());
      w->raw(path);
    } else {   // load
      if (args.a[1].s.empty()) throw std::runtime_error("empty id is not allowed");
      load_impl(local_path(args.a[1].s), false);
      w->boolean(true);
    }
  }

  void load_impl(const std::string& path, bool overwrite_config) {
    std::string bytes;
    if (!read_file(path, &bytes)) throw std::runtime_error("cannot open input file: " + path + ": " + strerror(errno));
    ModelFile mf;
    const std::string err = read_model_file(bytes, &mf);
    if (!err.empty()) throw std::runtime_error(err);
    if (mf.type != engine_name())
      throw std::runtime_error("invalid model type: saved type: " + mf.type + ", expected type: " + engine_name());
    if (!overwrite_config && !jb::val::same_config(mf.config, config_))
      throw std::runtime_error("model config mismatched with the running config");
    if (mf.user_version != 1)
      throw std::runtime_error("user data version mismatched: " + std::to_string(mf.user_version) +
                               ", current version: 1");
    std::unique_lock<std::shared_mutex> life(life_mu_);   // (no self-locking handler runs)
    std::unique_lock<std::shared_mutex> g(model_mu_);
    if (overwrite_config && !jb::val::same_config(mf.config, config_)) {
      eng_ = make_(mf.config);
      eng_->set_lock(&model_mu_);
      config_ = mf.config;
      table_.clear();
      for (auto& m : eng_->methods()) table_.push_back(m);
      if (node_) eng_->attach(node_.get(), a_);
    }
    eng_->unpack(mf.user);
    std::lock_guard<std::mutex> s(st_mu_);
    cs_.last_loaded = time(nullptr);
    cs_.last_loaded_path = path;
    logf_("INFO", "loaded from %s", path.c_str());
  }

  Args a_;
  std::string config_;
  Factory make_;
  std::unique_ptr<HostEngine> eng_;
  std::vector<HostMethod> table_;
  std::unique_ptr<jb::mix::ClusterNode> node_;
  std::unique_ptr<jb::mix::LinearMixer> mixer_;
  std::unique_ptr<jb::RpcServer> rpc_;
  std::shared_mutex model_mu_;
  std::shared_mutex life_mu_;   // shared: a self-locking raw handler runs; exclusive: the engine is replaced
  std::mutex st_mu_;
  CommonStatus cs_;
  std::atomic<uint64_t> update_count_{0};
};

// main() of a host-engine server: flags, config check (native vs Python),
// model file, serve
template <class Check>
int host_main(int argc, char** argv, const char* engine, Check check, HostServer::Factory make,
              bool native_dist = false) {
  set_engine(engine);
  Args a;
  std::string text;
  const int rc = startup(argc, argv, &a, &text, check, /*needs_gpu=*/false, native_dist, native_dist);
  if (rc >= 0) return rc;
  block_signals();
  logf_("INFO", "starting %s %s RPC server at %s:%d (native, host engine)", prog_name(), kVersion,
        a.eth.c_str(), a.port);
  try {
    HostServer srv(a, text, make);
    if (!a.zookeeper.empty())
      srv.join_cluster(std::unique_ptr<jb::mix::ClusterNode>(
          new jb::mix::ClusterNode(a.zookeeper, std::max(1, a.zk_timeout), engine, a.name)));
    if (!a.model_file.empty()) srv.load_file(a.model_file);
    return srv.run();
  } catch (const std::exception& e) {
    logf_("FATAL", "failed to start %s: %s", engine, e.what());
    return 1;
  }
}

// argument helpers for the handlers (std::invalid_argument -> ARGUMENT_ERROR)
inline const std::string& arg_str(const Value& v) {
  if (!v.is_str()) throw std::invalid_argument("string expected");
  return v.s;
}
inline double arg_num(const Value& v) {
  if (!v.is_num()) throw std::invalid_argument("number expected");
  return v.num();
}
inline int64_t arg_int(const Value& v) {
  if (v.kind == Value::INT) return v.i;
  if (v.kind == Value::UINT) return (int64_t)v.u;
  throw std::invalid_argument("integer expected");
}

}  // namespace srv
}  // namespace jb
