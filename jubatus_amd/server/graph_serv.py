"""jubagraph glue (reference jubatus/server/server/graph_serv.cpp:140-470).

Node ids travel as decimal strings, edge ids as uint64; node and edge ids
come from one id generator (standalone counter / coordinator sequence).
Distributed mode (graph_serv.cpp:150-330):
* ``create_node``: the node is created on its two CHT owners
  (``create_node_here``; the primary must succeed, replica failures are
  logged, "already exists" passes);
* ``remove_node``: local removal, then ``remove_global_node`` to every
  member (after releasing the lock, as the reference does);
* ``create_edge``: stored here (the proxy routes by the source node) and
  replicated to the source's other owner with ``create_edge_here``;
* ``update_index`` is standalone only - a cluster builds indices at MIX.
"""
from __future__ import annotations

from ..common.cht import CHT
from ..common.idgen import create_id_generator
from ..common.membership import get_all_nodes
from ..common.mprpc import RpcClient, RpcMClient
from ..framework.engine_serv import EngineServ
from ..models.graph import Graph, GraphError, LocalNodeExists
from ..utils import logger

log = logger.get_logger("graph")


def _n2i(nid) -> int:
    if isinstance(nid, bytes):
        nid = nid.decode()
    try:
        v = int(nid)
    except (TypeError, ValueError) as e:
        raise GraphError(f"invalid node id: {nid!r}") from e
    if v < 0:
        raise GraphError(f"invalid node id: {nid!r}")
    return v


def _props(p) -> dict:
    return {(k.decode() if isinstance(k, bytes) else str(k)): (v.decode() if isinstance(v, bytes) else str(v))
            for k, v in (p or {}).items()}


class GraphServ(EngineServ):
    type_name = "graph"

    def __init__(self, argv, coord=None):
        super().__init__(argv, coord)
        self.idgen = create_id_generator(argv, coord)

    def uses_gpu(self) -> bool:
        return False

    def build_driver(self, cfg: dict):
        return Graph(cfg.get("method"), cfg.get("parameter"))

    def _is_me(self, hp) -> bool:
        a = self.argv()
        return hp[0] == a.eth and int(hp[1]) == a.port

    def _owners(self, key: str, n: int = 2):
        owners = CHT(self.coord, self.type_name, self.argv().name).find(key, n)
        if not owners:
            raise RuntimeError(f"no server found in cht: {self.argv().name}")
        return owners

    # ---------------------------------------------------------------- nodes
    def create_node(self) -> str:
        self.check_set_config()
        nid = int(self.idgen.generate())
        sid = str(nid)
        if self.argv().is_standalone():
            with self.rw_mutex.write():
                self.event_model_updated()
                self.driver.create_node(nid)
            return sid
        owners = self._owners(sid)
        self._selective_create_node(owners[0], sid)
        for o in owners[1:]:
            try:
                self._selective_create_node(o, sid)
            except Exception as e:  # noqa: BLE001 - replica is best effort
                if "exists" not in str(e):
                    log.warning("cannot create replica of node %s (%s): %s:%d", sid, e, o[0], o[1])
        return sid

    def _selective_create_node(self, owner, sid: str) -> None:
        if self._is_me(owner):
            with self.rw_mutex.write():
                self.event_model_updated()
                self.create_node_here(sid)
            return
        with RpcClient(owner[0], owner[1], self.argv().interconnect_timeout) as c:
            c.call("create_node_here", self.argv().name, sid)

    def create_node_here(self, nid) -> bool:
        self.check_set_config()
        try:
            self.driver.create_node_here(_n2i(nid))
        except LocalNodeExists:
            pass
        return True

    def update_node(self, nid, prop) -> bool:
        self.check_set_config()
        self.driver.update_node(_n2i(nid), _props(prop))
        return True

    def remove_node(self, nid) -> bool:
        self.check_set_config()
        i = _n2i(nid)
        with self.rw_mutex.write():
            self.event_model_updated()
            self.driver.remove_node(i)
        if not self.argv().is_standalone():
            members = [m for m in get_all_nodes(self.coord, self.type_name, self.argv().name)
                       if not self._is_me(m)]
            if members:
                try:
                    RpcMClient(members, self.argv().interconnect_timeout).call(
                        "remove_global_node", self.argv().name, str(i))
                except Exception as e:  # noqa: BLE001 - reference passes rpc_no_result
                    log.info("remove_global_node: %s", e)
        return True

    def remove_global_node(self, nid) -> bool:
        self.check_set_config()
        self.driver.remove_global_node(_n2i(nid))
        return True

    def get_node(self, nid):
        self.check_set_config()
        n = self.driver.get_node(_n2i(nid))
        return [n["property"], n["in_edges"], n["out_edges"]]

    # ---------------------------------------------------------------- edges
    def create_edge(self, nid, e) -> int:
        self.check_set_config()
        prop, src, tgt = _props(e[0]), _n2i(e[1]), _n2i(e[2])
        eid = int(self.idgen.generate())
        if self.argv().is_standalone():
            with self.rw_mutex.write():
                self.event_model_updated()
                self.driver.create_edge(eid, src, tgt, prop)
            return eid
        owners = self._owners(str(src))
        with self.rw_mutex.write():
            self.event_model_updated()
            self.driver.create_edge_here(eid, src, tgt, prop)
        for o in owners[1:]:
            if self._is_me(o):
                continue
            try:
                with RpcClient(o[0], o[1], self.argv().interconnect_timeout) as c:
                    c.call("create_edge_here", self.argv().name, eid, [prop, str(src), str(tgt)])
            except Exception as ex:  # noqa: BLE001 - replica is best effort
                log.warning("cannot create replica of edge %d (%s): %s:%d", eid, ex, o[0], o[1])
        return eid

    def create_edge_here(self, eid: int, e) -> bool:
        self.check_set_config()
        self.driver.create_edge_here(int(eid), _n2i(e[1]), _n2i(e[2]), _props(e[0]))
        return True

    def update_edge(self, nid, eid: int, e) -> bool:
        self.check_set_config()
        self.driver.update_edge(int(eid), _props(e[0]))
        return True

    def remove_edge(self, nid, eid: int) -> bool:
        self.check_set_config()
        self.driver.remove_edge(int(eid))
        return True

    def get_edge(self, nid, eid: int):
        self.check_set_config()
        prop, s, t = self.driver.get_edge(int(eid))
        return [prop, str(s), str(t)]

    # -------------------------------------------------------------- queries
    def get_centrality(self, nid, ctype: int, q) -> float:
        self.check_set_config()
        return float(self.driver.get_centrality(_n2i(nid), int(ctype), q))

    def add_centrality_query(self, q) -> bool:
        self.check_set_config()
        self.driver.add_centrality_query(q)
        return True

    def add_shortest_path_query(self, q) -> bool:
        self.check_set_config()
        self.driver.add_shortest_path_query(q)
        return True

    def remove_centrality_query(self, q) -> bool:
        self.check_set_config()
        self.driver.remove_centrality_query(q)
        return True

    def remove_shortest_path_query(self, q) -> bool:
        self.check_set_config()
        self.driver.remove_shortest_path_query(q)
        return True

    def get_shortest_path(self, req):
        self.check_set_config()
        src, tgt, max_hop, q = req[0], req[1], int(req[2]), req[3]
        return [str(x) for x in self.driver.get_shortest_path(_n2i(src), _n2i(tgt), max_hop, q)]

    def update_index(self) -> bool:
        if not self.argv().is_standalone():
            raise RuntimeError("manual mix is available only in standalone mode.")
        self.check_set_config()
        self.driver.update_index()
        return True
