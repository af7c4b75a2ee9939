// jubagraph, native: the property graph engine without Python.
//
// Reference: jubatus/server/server/graph_serv.cpp:140-470 over jubatus_core's
// graph_wo_index; config config/graph/*.json (damping_factor, landmark_num).
// Same model as models/graph.py (its docstring lists it): nodes with string
// properties and in / out edge lists, edges (source, target, properties),
// node and edge ids from one counter (decimal strings for nodes); preset
// queries must be registered before they are answered, answers come from the
// index of the last update_index; centrality 0 = damped PageRank fixed point
// s = (1 - d) + d A^T (s / outdeg) on the query's subgraph; shortest path =
// hop-limited BFS over the indexed subgraph (edges in insertion order).
// Distributed (-z, graph_serv.cpp:150-330): node and edge ids come from the
// coordinator's id generator; create_node creates the node on its two CHT
// owners (create_node_here, server to server; the primary must succeed),
// remove_node tells every member (remove_global_node) after releasing the
// model lock, create_edge stores the edge here and replicates it to the
// source node's other owner (create_edge_here); the indices are built at MIX
// over the local graph plus every member's nodes and edges (models/graph.py
// get_diff / mix_diff / put_diff). Model files are shared with the Python
// server (Graph.pack()).
#include <math.h>

#include <algorithm>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "jb_host_server.hpp"

namespace {

using namespace jb::srv;

using Props = std::vector<std::pair<std::string, std::string>>;   // insertion order
using Cond = std::vector<std::pair<std::string, std::string>>;    // sorted
using QKey = std::pair<Cond, Cond>;                               // (edge, node) conditions

struct Node {
  Props p;
  std::vector<uint64_t> in, out;
};
struct Edge {
  uint64_t s, t;
  Props p;
};

std::string prop_get(const Props& p, const std::string& k, bool* found) {
  for (const auto& kv : p)
    if (kv.first == k) { *found = true; return kv.second; }
  *found = false;
  return std::string();
}

bool match(const Props& p, const Cond& c) {
  for (const auto& kv : c) {
    bool f;
    const std::string v = prop_get(p, kv.first, &f);
    if (!f || v != kv.second) return false;
  }
  return true;
}

std::string scalar(const Value& v) {   // a property value as Python's str() of it
  if (v.is_str()) return v.s;
  if (v.kind == Value::INT) return std::to_string(v.i);
  if (v.kind == Value::UINT) return std::to_string(v.u);
  if (v.kind == Value::BOOL) return v.b ? "True" : "False";
  if (v.kind == Value::DBL) { char b[40]; snprintf(b, sizeof b, "%.17g", v.d); return b; }
  throw std::invalid_argument("property value");
}

Props props_of(const Value& m) {
  Props out;
  if (m.kind == Value::NIL) return out;
  if (m.kind != Value::MAP) throw std::invalid_argument("property map expected");
  for (const auto& kv : m.o) out.emplace_back(kv.first, scalar(kv.second));
  return out;
}

Cond cond_of(const Value& list) {
  if (list.kind != Value::ARR) throw std::invalid_argument("query list expected");
  Cond c;
  for (const Value& x : list.a) {
    if (x.kind != Value::ARR || x.a.size() != 2) throw std::invalid_argument("query pair expected");
    c.emplace_back(scalar(x.a[0]), scalar(x.a[1]));
  }
  std::sort(c.begin(), c.end());
  return c;
}

QKey qkey(const Value& q) {
  if (q.kind != Value::ARR || q.a.size() != 2) throw std::invalid_argument("preset_query expected");
  return {cond_of(q.a[0]), cond_of(q.a[1])};
}

uint64_t node_id(const Value& v) {
  const std::string s = v.is_str() ? v.s : scalar(v);
  if (s.empty() || s.size() > 20 || !std::all_of(s.begin(), s.end(), ::isdigit))
    throw EngineError("invalid node id: '" + s + "'");
  return strtoull(s.c_str(), nullptr, 10);
}

uint64_t edge_id(const Value& v) {
  if (v.kind == Value::INT && v.i >= 0) return (uint64_t)v.i;
  if (v.kind == Value::UINT) return v.u;
  throw std::invalid_argument("edge id");
}

struct GraphParams {
  double damping = 0.9;
  int64_t landmark = 5;
};

bool parse_params(const std::string& text, GraphParams* p, std::string* why) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  if (v.str_or("method", "") != "graph_wo_index") {
    *why = "unsupported graph method: " + v.str_or("method", "");
    return false;
  }
  if (const Value* par = v.get("parameter")) {
    if (const Value* d = par->get("damping_factor")) p->damping = d->is_num() ? d->num() : atof(d->s.c_str());
    if (const Value* l = par->get("landmark_num"))
      p->landmark = (int64_t)(l->is_num() ? l->num() : atof(l->s.c_str()));
  }
  if (!(p->damping > 0 && p->damping < 1)) { *why = "damping_factor must be in (0, 1)"; return false; }
  return true;
}

class Graph : public HostEngine {
 public:
  explicit Graph(const GraphParams& p) : p_(p) {}

  std::vector<HostMethod> methods() override {
    using A = const std::vector<Value>&;
    HostMethod cn{"create_node", 1, true, [this](A, MsgpackWriter* w) {
      if (!node_) {
        std::unique_lock<std::shared_mutex> g(*mu_);
        const uint64_t id = next_id_++;
        create_node_here(id, true);
        w->raw(std::to_string(id));
        return;
      }
      const std::string sid = std::to_string(node_->create_id());
      const auto owners = node_->cht_find(sid, 2);
      selective_create(owners[0], sid);   // the primary must succeed
      for (size_t i = 1; i < owners.size(); ++i) {
        try {
          selective_create(owners[i], sid);
        } catch (const std::exception& e) {
          if (!strstr(e.what(), "exists"))
            logf_("WARN", "cannot create replica of node %s (%s): %s:%d", sid.c_str(), e.what(),
                  owners[i].first.c_str(), owners[i].second);
        }
      }
      w->raw(sid);
    }};
    cn.self_lock = true;
    HostMethod rn{"remove_node", 2, true, [this](A a, MsgpackWriter* w) {
      const uint64_t id = node_id(a[0]);
      {
        std::unique_lock<std::shared_mutex> g(*mu_);
        Node& n = node(id);
        if (!n.in.empty() || !n.out.empty())
          throw EngineError("cannot remove node " + std::to_string(id) + ": it has edges");
        nodes_.erase(id);
        node_order_.erase(std::find(node_order_.begin(), node_order_.end(), id));
        global_.erase(id);
      }
      if (node_) {   // every other member forgets it (no result awaited: rpc_no_result)
        for (const auto& m : node_->actors()) {
          if (is_me(m)) continue;
          try {
            MsgpackWriter p;
            p.arr(2);
            p.raw(name_);
            p.raw(std::to_string(id));
            peer_call(m, "remove_global_node", p.out);
          } catch (const std::exception& e) {
            logf_("INFO", "remove_global_node: %s", e.what());
          }
        }
      }
      w->boolean(true);
    }};
    rn.self_lock = true;
    HostMethod ce{"create_edge", 3, true, [this](A a, MsgpackWriter* w) {
      const Value& e = a[1];
      if (e.kind != Value::ARR || e.a.size() != 3) throw std::invalid_argument("edge expected");
      const uint64_t src = node_id(e.a[1]), tgt = node_id(e.a[2]);
      Props pr = props_of(e.a[0]);
      if (!node_) {
        std::unique_lock<std::shared_mutex> g(*mu_);
        const uint64_t eid = next_id_++;   // taken before the checks (graph_serv.cpp create_edge)
        if (!nodes_.count(src)) throw EngineError("unknown_id: source node " + std::to_string(src));
        if (!nodes_.count(tgt) && !global_.count(tgt))
          throw EngineError("unknown_id: target node " + std::to_string(tgt));
        put_edge(eid, src, tgt, std::move(pr));
        w->uint(eid);
        return;
      }
      const uint64_t eid = node_->create_id();
      const auto owners = node_->cht_find(std::to_string(src), 2);
      MsgpackWriter p;   // create_edge_here(name, eid, [prop, src, tgt])
      p.arr(3);
      p.raw(name_);
      p.uint(eid);
      p.arr(3);
      p.map(pr.size());
      for (const auto& kv : pr) { p.raw(kv.first); p.raw(kv.second); }
      p.raw(std::to_string(src));
      p.raw(std::to_string(tgt));
      {
        std::unique_lock<std::shared_mutex> g(*mu_);
        edge_here(eid, src, tgt, std::move(pr));
      }
      for (size_t i = 1; i < owners.size(); ++i) {
        if (is_me(owners[i])) continue;
        try {
          peer_call(owners[i], "create_edge_here", p.out);
        } catch (const std::exception& ex) {
          logf_("WARN", "cannot create replica of edge %llu (%s): %s:%d", (unsigned long long)eid, ex.what(),
                owners[i].first.c_str(), owners[i].second);
        }
      }
      w->uint(eid);
    }};
    ce.self_lock = true;
    return {
        cn,
        rn,
        ce,
        {"create_node_here", 2, true, [this](A a, MsgpackWriter* w) {
           create_node_here(node_id(a[0]), false);
           w->boolean(true);
         }},
        {"remove_global_node", 2, true, [this](A a, MsgpackWriter* w) {
           const uint64_t id = node_id(a[0]);
           global_.erase(id);
           if (remote_nodes_.erase(id))
             remote_order_.erase(std::find(remote_order_.begin(), remote_order_.end(), id));
           w->boolean(true);
         }},
        {"update_node", 3, true, [this](A a, MsgpackWriter* w) {
           node(node_id(a[0])).p = props_of(a[1]);
           w->boolean(true);
         }},
        {"get_node", 2, false, [this](A a, MsgpackWriter* w) {
           const Node& n = node(node_id(a[0]));
           w->arr(3);
           w->map(n.p.size());
           for (const auto& kv : n.p) { w->raw(kv.first); w->raw(kv.second); }
           w->arr(n.in.size());
           for (uint64_t e : n.in) w->uint(e);
           w->arr(n.out.size());
           for (uint64_t e : n.out) w->uint(e);
         }},
        {"create_edge_here", 3, true, [this](A a, MsgpackWriter* w) {
           const uint64_t eid = edge_id(a[0]);
           const Value& e = a[1];
           if (e.kind != Value::ARR || e.a.size() != 3) throw std::invalid_argument("edge expected");
           edge_here(eid, node_id(e.a[1]), node_id(e.a[2]), props_of(e.a[0]));
           w->boolean(true);
         }},
        {"update_edge", 4, true, [this](A a, MsgpackWriter* w) {
           const uint64_t eid = edge_id(a[1]);
           auto it = edges_.find(eid);
           if (it == edges_.end()) throw EngineError("unknown_id: edge " + std::to_string(eid));
           if (a[2].kind != Value::ARR || a[2].a.size() != 3) throw std::invalid_argument("edge expected");
           it->second.p = props_of(a[2].a[0]);
           w->boolean(true);
         }},
        {"remove_edge", 3, true, [this](A a, MsgpackWriter* w) {
           const uint64_t eid = edge_id(a[1]);
           auto it = edges_.find(eid);
           if (it == edges_.end()) throw EngineError("unknown_id: edge " + std::to_string(eid));
           const Edge e = it->second;
           edges_.erase(it);
           edge_order_.erase(std::find(edge_order_.begin(), edge_order_.end(), eid));
           auto drop = [eid](std::vector<uint64_t>& v) {
             auto f = std::find(v.begin(), v.end(), eid);
             if (f != v.end()) v.erase(f);
           };
           if (nodes_.count(e.s)) drop(nodes_[e.s].out);
           if (nodes_.count(e.t)) drop(nodes_[e.t].in);
           w->boolean(true);
         }},
        {"get_edge", 3, false, [this](A a, MsgpackWriter* w) {
           const uint64_t eid = edge_id(a[1]);
           const Edge* e = nullptr;
           auto it = edges_.find(eid);
           if (it != edges_.end()) e = &it->second;
           auto rt = remote_edges_.find(eid);
           if (!e && rt != remote_edges_.end()) e = &rt->second;
           if (!e) throw EngineError("unknown_id: edge " + std::to_string(eid));
           w->arr(3);
           w->map(e->p.size());
           for (const auto& kv : e->p) { w->raw(kv.first); w->raw(kv.second); }
           w->raw(std::to_string(e->s));
           w->raw(std::to_string(e->t));
         }},
        {"add_centrality_query", 2, true, [this](A a, MsgpackWriter* w) {
           cq_.insert(qkey(a[0]));
           w->boolean(true);
         }},
        {"add_shortest_path_query", 2, true, [this](A a, MsgpackWriter* w) {
           sq_.insert(qkey(a[0]));
           w->boolean(true);
         }},
        {"remove_centrality_query", 2, true, [this](A a, MsgpackWriter* w) {
           const QKey k = qkey(a[0]);
           cq_.erase(k);
           scores_.erase(k);
           w->boolean(true);
         }},
        {"remove_shortest_path_query", 2, true, [this](A a, MsgpackWriter* w) {
           const QKey k = qkey(a[0]);
           sq_.erase(k);
           sp_.erase(k);
           w->boolean(true);
         }},
        {"update_index", 1, true, [this](A, MsgpackWriter* w) {
           if (node_) throw EngineError("manual mix is available only in standalone mode.");
           update_index();
           w->boolean(true);
         }},
        {"get_centrality", 4, false, [this](A a, MsgpackWriter* w) {
           const uint64_t id = node_id(a[0]);
           const int64_t ctype = arg_int(a[1]);
           if (ctype != 0) throw EngineError("unknown centrality type: " + std::to_string(ctype));
           const QKey k = qkey(a[2]);
           if (!cq_.count(k)) throw EngineError("centrality query is not registered");
           auto sc = scores_.find(k);
           if (sc != scores_.end()) {
             auto it = sc->second.find(id);
             if (it != sc->second.end()) { w->dbl(it->second); return; }
           }
           if (nodes_.count(id) || remote_nodes_.count(id)) { w->dbl(0.0); return; }   // not indexed yet
           throw EngineError("unknown_id: node " + std::to_string(id));
         }},
        {"get_shortest_path", 2, false, [this](A a, MsgpackWriter* w) {
           const Value& q = a[0];
           if (q.kind != Value::ARR || q.a.size() != 4) throw std::invalid_argument("shortest_path_query");
           const auto path = shortest_path(node_id(q.a[0]), node_id(q.a[1]), arg_int(q.a[2]), qkey(q.a[3]));
           w->arr(path.size());
           for (uint64_t x : path) w->raw(std::to_string(x));
         }},
        {"clear", 1, true, [this](A, MsgpackWriter* w) {
           clear();
           w->boolean(true);
         }},
    };
  }

  void clear() override {
    nodes_.clear();
    node_order_.clear();
    edges_.clear();
    edge_order_.clear();
    remote_nodes_.clear();
    remote_order_.clear();
    remote_edges_.clear();
    remote_edge_order_.clear();
    global_.clear();
    cq_.clear();
    sq_.clear();
    scores_.clear();
    sp_.clear();
  }

  // models/graph.py pack(): nodes, edges, cq, sq, global, node_edges
  std::string pack() override {
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(6);
    u.str("nodes"); u.map(node_order_.size());
    for (uint64_t id : node_order_) write_props(&u, std::to_string(id), nodes_.at(id).p);
    u.str("edges"); u.map(edge_order_.size());
    for (uint64_t eid : edge_order_) write_edge(&u, eid, edges_.at(eid));
    write_queries(&u, "cq", cq_);
    write_queries(&u, "sq", sq_);
    std::vector<uint64_t> g(global_.begin(), global_.end());
    std::sort(g.begin(), g.end());
    u.str("global"); u.arr(g.size());
    for (uint64_t x : g) u.uint(x);
    u.str("node_edges"); u.map(node_order_.size());
    for (uint64_t id : node_order_) {
      const Node& n = nodes_.at(id);
      u.str(std::to_string(id));
      u.arr(2);
      u.arr(n.in.size());
      for (uint64_t e : n.in) u.uint(e);
      u.arr(n.out.size());
      for (uint64_t e : n.out) u.uint(e);
    }
    return std::move(u.out);
  }

  void unpack(const Value& obj) override {
    const Value* nv = obj.get("nodes");
    const Value* ev = obj.get("edges");
    const Value* ne = obj.get("node_edges");
    const Value* gv = obj.get("global");
    const Value* cv = obj.get("cq");
    const Value* sv = obj.get("sq");
    if (!nv || !ev || !ne || !gv || !cv || !sv) throw std::runtime_error("broken model data: graph");
    clear();
    for (const auto& kv : nv->o) {
      const uint64_t id = strtoull(kv.first.c_str(), nullptr, 10);
      Node n;
      n.p = props_of(kv.second);
      const Value* ie = ne->get(kv.first);
      if (ie && ie->kind == Value::ARR && ie->a.size() == 2) {
        for (const Value& x : ie->a[0].a) n.in.push_back((uint64_t)x.num());
        for (const Value& x : ie->a[1].a) n.out.push_back((uint64_t)x.num());
      }
      nodes_[id] = std::move(n);
      node_order_.push_back(id);
    }
    for (const auto& kv : ev->o) {
      const uint64_t eid = strtoull(kv.first.c_str(), nullptr, 10);
      edges_[eid] = Edge{(uint64_t)kv.second.a.at(0).num(), (uint64_t)kv.second.a.at(1).num(),
                         props_of(kv.second.a.at(2))};
      edge_order_.push_back(eid);
    }
    for (const Value& x : gv->a) global_.insert((uint64_t)x.num());
    for (const Value& q : cv->a) cq_.insert(qkey(q));
    for (const Value& q : sv->a) sq_.insert(qkey(q));
    uint64_t mx = 0;
    for (const auto& kv : nodes_) mx = std::max(mx, kv.first + 1);
    for (const auto& kv : edges_) mx = std::max(mx, kv.first + 1);
    next_id_ = std::max(next_id_, mx);
    update_index();
  }

  // ---- distributed mode
  void set_lock(std::shared_mutex* mu) override { mu_ = mu; }
  void attach(jb::mix::ClusterNode* node, const Args& a) override {
    node_ = node;
    eth_ = a.eth;
    port_ = a.port;
    name_ = a.name;
    ic_timeout_ = std::max(1, a.ic_timeout);
  }
  bool mixable() const override { return true; }
  bool uses_cht() const override { return true; }
  // models/graph.py get_diff: the local nodes (properties), edges and queries
  std::string get_diff() override {
    MsgpackWriter u;
    u.map(4);
    u.str("nodes"); u.map(node_order_.size());
    for (uint64_t id : node_order_) write_props(&u, std::to_string(id), nodes_.at(id).p);
    u.str("edges"); u.map(edge_order_.size());
    for (uint64_t eid : edge_order_) write_edge(&u, eid, edges_.at(eid));
    write_queries(&u, "cq", cq_);
    write_queries(&u, "sq", sq_);
    return std::move(u.out);
  }
  // mix_diff in rank order (a later member's entry wins), then put_diff: the
  // others' nodes and edges become the remote part, queries join, and the
  // indices are rebuilt over local + remote
  void put_diffs(const std::vector<Value>& parts) override {
    std::vector<uint64_t> norder, eorder;
    std::unordered_map<uint64_t, Props> nodes;
    std::unordered_map<uint64_t, Edge> edges;
    for (const Value& d : parts) {
      const Value* nv = d.get("nodes");
      const Value* ev = d.get("edges");
      const Value* cv = d.get("cq");
      const Value* sv = d.get("sq");
      if (!nv || !ev || !cv || !sv) throw std::runtime_error("mix: malformed graph diff");
      for (const auto& kv : nv->o) {
        const uint64_t id = strtoull(kv.first.c_str(), nullptr, 10);
        if (!nodes.count(id)) norder.push_back(id);
        nodes[id] = props_of(kv.second);
      }
      for (const auto& kv : ev->o) {
        const uint64_t eid = strtoull(kv.first.c_str(), nullptr, 10);
        if (!edges.count(eid)) eorder.push_back(eid);
        edges[eid] = Edge{(uint64_t)kv.second.a.at(0).num(), (uint64_t)kv.second.a.at(1).num(),
                          props_of(kv.second.a.at(2))};
      }
      for (const Value& q : cv->a) cq_.insert(qkey(q));
      for (const Value& q : sv->a) sq_.insert(qkey(q));
    }
    remote_nodes_.clear();
    remote_order_.clear();
    for (uint64_t id : norder)
      if (!nodes_.count(id)) {
        remote_nodes_[id] = std::move(nodes[id]);
        remote_order_.push_back(id);
        global_.insert(id);
      }
    remote_edges_.clear();
    remote_edge_order_.clear();
    for (uint64_t eid : eorder)
      if (!edges_.count(eid)) {
        remote_edges_[eid] = std::move(edges[eid]);
        remote_edge_order_.push_back(eid);
      }
    update_index();
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) override {
    st->emplace_back("local_node_num", std::to_string(nodes_.size()));
    st->emplace_back("global_node_num", std::to_string(global_.size()));
    st->emplace_back("local_edge_num", std::to_string(edges_.size()));
    st->emplace_back("centrality_query_num", std::to_string(cq_.size()));
    st->emplace_back("shortest_path_query_num", std::to_string(sq_.size()));
  }

 private:
  static void write_props(MsgpackWriter* u, const std::string& key, const Props& p) {
    u->str(key);
    u->map(p.size());
    for (const auto& kv : p) { u->str(kv.first); u->str(kv.second); }
  }
  static void write_edge(MsgpackWriter* u, uint64_t eid, const Edge& e) {
    u->str(std::to_string(eid));
    u->arr(3);
    u->uint(e.s);
    u->uint(e.t);
    u->map(e.p.size());
    for (const auto& kv : e.p) { u->str(kv.first); u->str(kv.second); }
  }
  static void write_queries(MsgpackWriter* u, const char* name, const std::set<QKey>& qs) {
    u->str(name);
    u->arr(qs.size());
    for (const QKey& k : qs) {
      u->arr(2);
      for (const Cond* c : {&k.first, &k.second}) {
        u->arr(c->size());
        for (const auto& kv : *c) { u->arr(2); u->str(kv.first); u->str(kv.second); }
      }
    }
  }

  bool is_me(const std::pair<std::string, int>& hp) const { return hp.first == eth_ && hp.second == port_; }

  // a server-to-server call (interconnect timeout); throws on any error
  void peer_call(const std::pair<std::string, int>& hp, const char* method, const std::string& params) {
    jb::cc::Conn c(hp.first, hp.second, ic_timeout_);
    const double dl = jb::cc::now_s() + ic_timeout_;
    const uint32_t mid = c.send_request(method, params, dl);
    jb::cc::CallResult res;
    c.recv_response(mid, dl, &res);
    if (!res.transport_ok) throw std::runtime_error(res.transport_error);
    if (!res.err.empty()) {
      const Value e = MsgpackReader((const uint8_t*)res.err.data(), res.err.size()).read();
      throw std::runtime_error(e.is_str() ? e.s : std::string("remote error"));
    }
  }

  // create_node_here on one owner (this server under the model lock, else by RPC)
  void selective_create(const std::pair<std::string, int>& owner, const std::string& sid) {
    if (is_me(owner)) {
      std::unique_lock<std::shared_mutex> g(*mu_);
      create_node_here(strtoull(sid.c_str(), nullptr, 10), false);
      return;
    }
    MsgpackWriter p;
    p.arr(2);
    p.raw(name_);
    p.raw(sid);
    peer_call(owner, "create_node_here", p.out);
  }

  // replica path: the source node is created when missing, no target check
  void edge_here(uint64_t eid, uint64_t src, uint64_t tgt, Props pr) {
    if (!nodes_.count(src)) { nodes_[src] = Node{}; node_order_.push_back(src); }
    put_edge(eid, src, tgt, std::move(pr));
  }

  Node& node(uint64_t id) {
    auto it = nodes_.find(id);
    if (it == nodes_.end()) throw EngineError("unknown_id: node " + std::to_string(id));
    return it->second;
  }

  void create_node_here(uint64_t id, bool strict) {
    if (nodes_.count(id)) {
      if (strict) throw EngineError("local_node_exists: " + std::to_string(id));
      return;
    }
    nodes_[id] = Node{};
    node_order_.push_back(id);
    global_.insert(id);
  }

  void put_edge(uint64_t eid, uint64_t src, uint64_t tgt, Props p) {
    if (edges_.count(eid)) throw EngineError("edge " + std::to_string(eid) + " already exists");
    edges_[eid] = Edge{src, tgt, std::move(p)};
    edge_order_.push_back(eid);
    nodes_[src].out.push_back(eid);
    auto t = nodes_.find(tgt);
    if (t != nodes_.end()) t->second.in.push_back(eid);
  }

  // nodes of the query (sorted) and its edges in insertion order
  // (models/graph.py _all: the remote part from the last MIX, then the local
  // graph over it)
  void subgraph(const QKey& k, std::vector<uint64_t>* ids, std::vector<std::pair<uint64_t, uint64_t>>* es) const {
    std::unordered_set<uint64_t> keep;
    for (const auto& kv : nodes_)
      if (match(kv.second.p, k.second)) { keep.insert(kv.first); ids->push_back(kv.first); }
    for (const auto& kv : remote_nodes_)
      if (match(kv.second, k.second)) { keep.insert(kv.first); ids->push_back(kv.first); }
    std::sort(ids->begin(), ids->end());
    for (const auto* order : {&remote_edge_order_, &edge_order_}) {
      const auto& tab = order == &edge_order_ ? edges_ : remote_edges_;
      for (uint64_t eid : *order) {
        const Edge& e = tab.at(eid);
        if (keep.count(e.s) && keep.count(e.t) && match(e.p, k.first)) es->emplace_back(e.s, e.t);
      }
    }
  }

  void update_index() {
    scores_.clear();
    for (const QKey& k : cq_) {
      std::vector<uint64_t> ids;
      std::vector<std::pair<uint64_t, uint64_t>> es;
      subgraph(k, &ids, &es);
      std::unordered_map<uint64_t, size_t> pos;
      for (size_t i = 0; i < ids.size(); ++i) pos[ids[i]] = i;
      const size_t n = ids.size();
      std::vector<double> outdeg(n, 0.0), s(n, 1.0), contrib(n);
      std::vector<std::pair<size_t, size_t>> e2;
      for (const auto& e : es) {
        e2.emplace_back(pos[e.first], pos[e.second]);
        outdeg[pos[e.first]] += 1;
      }
      for (int it = 0; it < 200 && n; ++it) {
        std::fill(contrib.begin(), contrib.end(), 0.0);
        for (const auto& e : e2) contrib[e.second] += s[e.first] / outdeg[e.first];
        double diff = 0;
        for (size_t i = 0; i < n; ++i) {
          const double ns = (1.0 - p_.damping) + p_.damping * contrib[i];
          diff = std::max(diff, fabs(ns - s[i]));
          s[i] = ns;
        }
        if (diff < 1e-10) break;
      }
      auto& out = scores_[k];
      for (size_t i = 0; i < n; ++i) out[ids[i]] = s[i];
    }
    sp_.clear();
    for (const QKey& k : sq_) {
      std::vector<uint64_t> ids;
      std::vector<std::pair<uint64_t, uint64_t>> es;
      subgraph(k, &ids, &es);
      auto& adj = sp_[k];
      for (uint64_t id : ids) adj[id];
      for (const auto& e : es) adj[e.first].push_back(e.second);
    }
  }

  std::vector<uint64_t> shortest_path(uint64_t src, uint64_t tgt, int64_t max_hop, const QKey& k) const {
    if (!sq_.count(k)) throw EngineError("shortest path query is not registered");
    auto ai = sp_.find(k);
    if (ai == sp_.end()) return {};
    const auto& adj = ai->second;
    if (!adj.count(src) || !adj.count(tgt)) return {};
    std::unordered_map<uint64_t, uint64_t> prev;
    std::unordered_set<uint64_t> seen{src};
    std::deque<std::pair<uint64_t, int64_t>> frontier{{src, 0}};
    while (!frontier.empty()) {
      const auto [u, h] = frontier.front();
      frontier.pop_front();
      if (u == tgt) {
        std::vector<uint64_t> path{u};
        uint64_t x = u;
        while (x != src) { x = prev.at(x); path.push_back(x); }
        std::reverse(path.begin(), path.end());
        return path;
      }
      if (h >= max_hop) continue;
      for (uint64_t v : adj.at(u))
        if (!seen.count(v)) {
          seen.insert(v);
          prev[v] = u;
          frontier.emplace_back(v, h + 1);
        }
    }
    return {};
  }

  GraphParams p_;
  std::shared_mutex* mu_ = nullptr;          // the server's model lock (self_lock methods)
  jb::mix::ClusterNode* node_ = nullptr;     // distributed mode
  std::string eth_, name_;
  int port_ = 0;
  double ic_timeout_ = 10;
  uint64_t next_id_ = 0;
  std::unordered_map<uint64_t, Node> nodes_;
  std::vector<uint64_t> node_order_;
  std::unordered_map<uint64_t, Edge> edges_;
  std::vector<uint64_t> edge_order_;
  std::unordered_set<uint64_t> global_;
  std::unordered_map<uint64_t, Props> remote_nodes_;   // the other members' (last MIX)
  std::vector<uint64_t> remote_order_;
  std::unordered_map<uint64_t, Edge> remote_edges_;
  std::vector<uint64_t> remote_edge_order_;
  std::set<QKey> cq_, sq_;
  std::map<QKey, std::unordered_map<uint64_t, double>> scores_;
  std::map<QKey, std::unordered_map<uint64_t, std::vector<uint64_t>>> sp_;
};

}  // namespace

int main(int argc, char** argv) {
  return host_main(
      argc, argv, "graph",
      [](const std::string& text, std::string* why) {
        GraphParams p;
        return parse_params(text, &p, why);
      },
      [](const std::string& text) -> std::unique_ptr<HostEngine> {
        GraphParams p;
        std::string why;
        if (!parse_params(text, &p, &why)) throw std::runtime_error(why);
        return std::unique_ptr<HostEngine>(new Graph(p));
      },
      /*native_dist=*/true);
}
