"""Property graph with preset-query indices (jubagraph, graph_wo_index).

Reference: jubatus/server/server/graph_serv.cpp:140-470 over jubatus_core's
graph_wo_index (EXTERNAL); config config/graph/graph_wo_index.json
(damping_factor, landmark_num). Model:
* nodes (uint64 ids, string properties, in/out edge id lists) and edges
  (id, source, target, properties); node and edge ids share one generator;
* ``preset_query{edge_query, node_query}``: lists of (key, value) property
  constraints; a centrality / shortest-path query must be registered
  (add_*_query) before it is answered, and answers come from the index
  built at the last ``update_index`` (standalone) or MIX (distributed);
* centrality type 0 = eigen score: the damped PageRank fixed point
  s = (1 - d) + d * A^T (s / outdeg) on the query's node/edge subgraph
  (unnormalised, starting from 1 - scores are ~1 on average);
* shortest path: hop-limited BFS over the query's indexed subgraph
  (exact - the reference's landmark index approximates it; ``landmark_num``
  is accepted); an empty list when unreachable within ``max_hop``;
* global nodes: nodes known from other servers (create_edge targets, MIX);
  ``remove_global_node`` drops one everywhere.
Errors: unknown ids raise ``unknown_id``; creating an existing node raises
``local_node_exists``; removing a node that still has edges raises.
MIX: servers exchange their local nodes / edges; every server rebuilds the
indices over the union (get_diff / mix_diff / put_diff).
"""
from __future__ import annotations

import threading
from collections import deque

import numpy as np


class GraphError(RuntimeError):
    pass


class UnknownId(GraphError):
    def __init__(self, what: str, i: int):
        super().__init__(f"unknown_id: {what} {i}")


class LocalNodeExists(GraphError):
    def __init__(self, i: int):
        super().__init__(f"local_node_exists: {i}")


def _qkey(q) -> tuple:
    """Canonical, hashable form of a preset_query [[edge (k, v)...], [node (k, v)...]]."""
    eq, nq = q
    return (tuple(sorted((str(a), str(b)) for a, b in eq)), tuple(sorted((str(a), str(b)) for a, b in nq)))


def _match(props: dict, cond: tuple) -> bool:
    return all(props.get(k) == v for k, v in cond)


class Graph:
    def __init__(self, method: str, parameter: dict | None):
        if method != "graph_wo_index":
            raise ValueError(f"unsupported graph method: {method}")
        p = dict(parameter or {})
        self.damping = float(p.get("damping_factor", 0.9))
        self.landmark_num = int(p.get("landmark_num", 5))
        if not 0.0 < self.damping < 1.0:
            raise ValueError("damping_factor must be in (0, 1)")
        self._lock = threading.RLock()
        self.clear()

    def clear(self) -> None:
        with getattr(self, "_lock", threading.RLock()):
            self.nodes: dict[int, dict] = {}          # id -> {"p": {}, "in": [], "out": []}
            self.edges: dict[int, tuple[int, int, dict]] = {}
            self.global_nodes: set[int] = set()
            self.centrality_queries: set[tuple] = set()
            self.sp_queries: set[tuple] = set()
            self.remote_nodes: dict[int, dict] = {}   # from MIX
            self.remote_edges: dict[int, tuple[int, int, dict]] = {}
            self.scores: dict[tuple, dict[int, float]] = {}
            self.sp_index: dict[tuple, dict[int, list[int]]] = {}

    # ------------------------------------------------------------- nodes
    def create_node_here(self, nid: int) -> None:
        with self._lock:
            if nid in self.nodes:
                raise LocalNodeExists(nid)
            self.nodes[nid] = {"p": {}, "in": [], "out": []}
            self.global_nodes.add(nid)

    create_node = create_node_here

    def _node(self, nid: int) -> dict:
        n = self.nodes.get(nid)
        if n is None:
            raise UnknownId("node", nid)
        return n

    def update_node(self, nid: int, prop: dict) -> None:
        with self._lock:
            self._node(nid)["p"] = {str(k): str(v) for k, v in prop.items()}

    def remove_node(self, nid: int) -> None:
        with self._lock:
            n = self._node(nid)
            if n["in"] or n["out"]:
                raise GraphError(f"cannot remove node {nid}: it has edges")
            del self.nodes[nid]
            self.global_nodes.discard(nid)

    def remove_global_node(self, nid: int) -> None:
        with self._lock:
            self.global_nodes.discard(nid)
            self.remote_nodes.pop(nid, None)

    def get_node(self, nid: int) -> dict:
        with self._lock:
            n = self._node(nid)
            return {"property": dict(n["p"]), "in_edges": list(n["in"]), "out_edges": list(n["out"])}

    # ------------------------------------------------------------- edges
    def create_edge_here(self, eid: int, src: int, tgt: int, prop: dict) -> None:
        """replica path: the source node is created when missing"""
        with self._lock:
            if src not in self.nodes:
                self.nodes[src] = {"p": {}, "in": [], "out": []}
            self._put_edge(eid, src, tgt, prop)

    def create_edge(self, eid: int, src: int, tgt: int, prop: dict) -> None:
        with self._lock:
            if src not in self.nodes:
                raise UnknownId("source node", src)
            if tgt not in self.nodes and tgt not in self.global_nodes:
                raise UnknownId("target node", tgt)
            self._put_edge(eid, src, tgt, prop)

    def _put_edge(self, eid, src, tgt, prop) -> None:
        if eid in self.edges:
            raise GraphError(f"edge {eid} already exists")
        self.edges[eid] = (src, tgt, {str(k): str(v) for k, v in prop.items()})
        self.nodes[src]["out"].append(eid)
        if tgt in self.nodes:
            self.nodes[tgt]["in"].append(eid)

    def update_edge(self, eid: int, prop: dict) -> None:
        with self._lock:
            if eid not in self.edges:
                raise UnknownId("edge", eid)
            s, t, _ = self.edges[eid]
            self.edges[eid] = (s, t, {str(k): str(v) for k, v in prop.items()})

    def remove_edge(self, eid: int) -> None:
        with self._lock:
            e = self.edges.pop(eid, None)
            if e is None:
                raise UnknownId("edge", eid)
            s, t, _ = e
            if s in self.nodes and eid in self.nodes[s]["out"]:
                self.nodes[s]["out"].remove(eid)
            if t in self.nodes and eid in self.nodes[t]["in"]:
                self.nodes[t]["in"].remove(eid)

    def get_edge(self, eid: int) -> tuple[dict, int, int]:
        with self._lock:
            e = self.edges.get(eid) or self.remote_edges.get(eid)
            if e is None:
                raise UnknownId("edge", eid)
            return dict(e[2]), e[0], e[1]

    # ----------------------------------------------------------- queries
    def add_centrality_query(self, q) -> None:
        with self._lock:
            self.centrality_queries.add(_qkey(q))

    def add_shortest_path_query(self, q) -> None:
        with self._lock:
            self.sp_queries.add(_qkey(q))

    def remove_centrality_query(self, q) -> None:
        with self._lock:
            k = _qkey(q)
            self.centrality_queries.discard(k)
            self.scores.pop(k, None)

    def remove_shortest_path_query(self, q) -> None:
        with self._lock:
            k = _qkey(q)
            self.sp_queries.discard(k)
            self.sp_index.pop(k, None)

    def _all(self):
        nodes = dict(self.remote_nodes)
        nodes.update({i: n["p"] for i, n in self.nodes.items()})
        edges = dict(self.remote_edges)
        edges.update(self.edges)
        return nodes, edges

    def _subgraph(self, key: tuple, nodes, edges):
        eq, nq = key
        keep = {i for i, p in nodes.items() if _match(p, nq)}
        es = [(s, t) for s, t, p in edges.values() if s in keep and t in keep and _match(p, eq)]
        return sorted(keep), es

    def _pagerank(self, ids: list[int], es: list[tuple[int, int]]) -> dict[int, float]:
        if not ids:
            return {}
        pos = {n: i for i, n in enumerate(ids)}
        src = np.array([pos[s] for s, _ in es], dtype=np.int64)
        dst = np.array([pos[t] for _, t in es], dtype=np.int64)
        outdeg = np.bincount(src, minlength=len(ids)).astype(np.float64)
        s = np.ones(len(ids))
        for _ in range(200):
            contrib = np.zeros(len(ids))
            if len(es):
                np.add.at(contrib, dst, s[src] / outdeg[src])
            ns = (1.0 - self.damping) + self.damping * contrib
            if np.max(np.abs(ns - s)) < 1e-10:
                s = ns
                break
            s = ns
        return {n: float(s[i]) for n, i in pos.items()}

    def update_index(self) -> None:
        with self._lock:
            nodes, edges = self._all()
            self.scores = {}
            for key in self.centrality_queries:
                ids, es = self._subgraph(key, nodes, edges)
                self.scores[key] = self._pagerank(ids, es)
            self.sp_index = {}
            for key in self.sp_queries:
                ids, es = self._subgraph(key, nodes, edges)
                adj: dict[int, list[int]] = {i: [] for i in ids}
                for s, t in es:
                    adj[s].append(t)
                self.sp_index[key] = adj

    def get_centrality(self, nid: int, ctype: int, q) -> float:
        with self._lock:
            if ctype != 0:
                raise GraphError(f"unknown centrality type: {ctype}")
            key = _qkey(q)
            if key not in self.centrality_queries:
                raise GraphError("centrality query is not registered")
            sc = self.scores.get(key, {})
            if nid not in sc:
                if nid in self.nodes or nid in self.remote_nodes:
                    return 0.0   # not indexed yet (update_index / MIX pending)
                raise UnknownId("node", nid)
            return sc[nid]

    def get_shortest_path(self, src: int, tgt: int, max_hop: int, q) -> list[int]:
        with self._lock:
            key = _qkey(q)
            if key not in self.sp_queries:
                raise GraphError("shortest path query is not registered")
            adj = self.sp_index.get(key, {})
            if src not in adj or tgt not in adj:
                return []
            prev = {src: None}
            frontier = deque([(src, 0)])
            while frontier:
                u, h = frontier.popleft()
                if u == tgt:
                    path = []
                    while u is not None:
                        path.append(u)
                        u = prev[u]
                    return path[::-1]
                if h >= max_hop:
                    continue
                for v in adj[u]:
                    if v not in prev:
                        prev[v] = u
                        frontier.append((v, h + 1))
            return []

    # ----------------------------------------------------------------- MIX
    def get_diff(self) -> dict:
        with self._lock:
            return {"nodes": {str(i): n["p"] for i, n in self.nodes.items()},
                    "edges": {str(e): [s, t, p] for e, (s, t, p) in self.edges.items()},
                    "cq": [list(map(list, k)) for k in self.centrality_queries],
                    "sq": [list(map(list, k)) for k in self.sp_queries]}

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        out = {"nodes": dict(a["nodes"]), "edges": dict(a["edges"]),
               "cq": list(a["cq"]), "sq": list(a["sq"])}
        out["nodes"].update(b["nodes"])
        out["edges"].update(b["edges"])
        out["cq"] += [q for q in b["cq"] if q not in out["cq"]]
        out["sq"] += [q for q in b["sq"] if q not in out["sq"]]
        return out

    def put_diff(self, mixed: dict) -> bool:
        with self._lock:
            self.remote_nodes = {int(i): {str(k): str(v) for k, v in p.items()}
                                 for i, p in mixed["nodes"].items() if int(i) not in self.nodes}
            self.remote_edges = {int(e): (int(v[0]), int(v[1]), dict(v[2]))
                                 for e, v in mixed["edges"].items() if int(e) not in self.edges}
            self.global_nodes |= set(self.remote_nodes)
            for q in mixed["cq"]:
                self.centrality_queries.add(_qkey(q))
            for q in mixed["sq"]:
                self.sp_queries.add(_qkey(q))
            self.update_index()
            return True

    def pack(self) -> dict:
        with self._lock:
            d = self.get_diff()
            d["global"] = sorted(self.global_nodes)
            d["node_edges"] = {str(i): [n["in"], n["out"]] for i, n in self.nodes.items()}
            return d

    def unpack(self, obj: dict) -> None:
        with self._lock:
            self.clear()
            for i, p in obj["nodes"].items():
                ine, oute = obj["node_edges"][i]
                self.nodes[int(i)] = {"p": dict(p), "in": list(ine), "out": list(oute)}
            self.edges = {int(e): (int(v[0]), int(v[1]), dict(v[2])) for e, v in obj["edges"].items()}
            self.global_nodes = set(obj["global"])
            self.centrality_queries = {_qkey(q) for q in obj["cq"]}
            self.sp_queries = {_qkey(q) for q in obj["sq"]}
            self.update_index()

    def get_status(self) -> dict[str, str]:
        return {"local_node_num": str(len(self.nodes)), "global_node_num": str(len(self.global_nodes)),
                "local_edge_num": str(len(self.edges)),
                "centrality_query_num": str(len(self.centrality_queries)),
                "shortest_path_query_num": str(len(self.sp_queries))}
