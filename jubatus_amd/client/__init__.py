"""Python client library (reference C35: jubatus/client/*.hpp, the generated
per-engine clients; same method names, argument order and wire types).

    from jubatus_amd.client import Classifier, Datum
    c = Classifier("127.0.0.1", 9199, "cluster-name")
    c.train([("spam", Datum({"text": "buy now"}))])
    c.classify([Datum({"text": "hello"})])   # -> [[EstimateResult(label, score), ...]]

Every call sends the cluster name as the first argument (the proxy routes on
it). Engine methods come from the IDL table (idl/specs.py).
"""
from __future__ import annotations

from dataclasses import dataclass, fields, is_dataclass
from typing import Any

from ..common.mprpc import RpcClient
from ..fv_converter.datum import Datum
from ..idl import specs

__all__ = ["Client", "Datum", "EstimateResult", "LabeledDatum", "ScoredDatum", "IdWithScore",
           "WeightedDatum", "Feature", "ArmInfo", "Document", "KeywordWithParams", "Batch",
           "Window", "Node", "Edge", "Query", "PresetQuery", "ShortestPathQuery"] + \
          [n.title().replace("_", "") for n in specs.ENGINES]


# ------------------------------------------------------------- wire types
@dataclass
class EstimateResult:
    label: str
    score: float


@dataclass
class LabeledDatum:
    label: str
    data: Datum


@dataclass
class ScoredDatum:
    score: float
    data: Datum


@dataclass
class IdWithScore:
    id: str
    score: float


@dataclass
class WeightedDatum:
    weight: float
    point: Datum


@dataclass
class Feature:
    key: str
    value: float


@dataclass
class ArmInfo:
    trial_count: int
    weight: float


@dataclass
class Document:
    pos: float
    text: str


@dataclass
class KeywordWithParams:
    keyword: str
    scaling_param: float
    gamma: float


@dataclass
class Batch:
    all_data_count: int
    relevant_data_count: int
    burst_weight: float


@dataclass
class Window:
    start_pos: float
    batches: list


@dataclass
class Query:
    from_id: str
    to_id: str


@dataclass
class PresetQuery:
    edge_query: list
    node_query: list


@dataclass
class Edge:
    property: dict
    source: str
    target: str


@dataclass
class Node:
    property: dict
    in_edges: list
    out_edges: list


@dataclass
class ShortestPathQuery:
    source: str
    target: str
    max_hop: int
    query: PresetQuery


def to_wire(x: Any) -> Any:
    if isinstance(x, Datum):
        return x.to_msgpack()
    if is_dataclass(x):
        return [to_wire(getattr(x, f.name)) for f in fields(x)]
    if isinstance(x, dict):
        return {k: to_wire(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [to_wire(v) for v in x]
    return x


def _conv(ret: str, v: Any) -> Any:
    """Convert a wire result of IDL type ``ret`` to client objects."""
    if v is None:
        return v
    r = ret.replace(" ", "")
    if r.startswith("list<") and r.endswith(">"):
        inner = r[5:-1]
        return [_conv(inner, x) for x in v]
    if r.startswith("map<string,") and r.endswith(">"):
        inner = r[len("map<string,"):-1]
        return {k: _conv(inner, x) for k, x in v.items()}
    simple = {"estimate_result": EstimateResult, "id_with_score": IdWithScore,
              "feature": Feature, "arm_info": ArmInfo, "keyword_with_params": KeywordWithParams}
    if r in simple:
        return simple[r](*v)
    if r == "datum":
        return Datum.from_msgpack(v)
    if r == "weighted_datum":
        return WeightedDatum(v[0], Datum.from_msgpack(v[1]))
    if r == "window":
        return Window(v[0], [Batch(*b) for b in v[1]])
    if r == "node":
        return Node(v[0], list(v[1]), list(v[2]))
    if r == "edge":
        return Edge(v[0], v[1], v[2])
    return v


class Client:
    """Common methods (reference client/common/client.hpp:29-85)."""

    engine = ""

    def __init__(self, host: str, port: int, name: str, timeout: float = 10.0):
        self._c = RpcClient(host, port, timeout)
        self.name = name

    def get_name(self) -> str:
        return self.name

    def set_name(self, name: str) -> None:
        self.name = name

    def get_client(self) -> RpcClient:
        return self._c

    def close(self) -> None:
        self._c.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def call(self, method: str, *args: Any) -> Any:
        return self._c.call(method, self.name, *[to_wire(a) for a in args])

    def get_config(self) -> str:
        return self.call("get_config")

    def save(self, id: str) -> dict:
        return self.call("save", id)

    def load(self, id: str) -> bool:
        return self.call("load", id)

    def get_status(self) -> dict:
        return self.call("get_status")

    def do_mix(self) -> bool:
        return self.call("do_mix")

    def get_proxy_status(self) -> dict:
        return self.call("get_proxy_status")


def _make_method(m: specs.Method):
    def method(self, *args):
        if len(args) != len(m.args):
            raise TypeError(f"{m.name}() takes {len(m.args)} arguments ({len(args)} given)")
        return _conv(m.ret, self.call(m.name, *args))
    method.__name__ = m.name
    method.__doc__ = f"{m.ret} {m.name}({', '.join(m.args)})  [{m.routing}, {m.lock}, {m.agg}]"
    return method


def _make_client(engine: str):
    ns = {"engine": engine}
    for m in specs.SERVICES[engine]:
        if m.routing != "internal":
            ns[m.name] = _make_method(m)
    return type(engine.title().replace("_", ""), (Client,), ns)


Classifier = _make_client("classifier")
Regression = _make_client("regression")
Recommender = _make_client("recommender")
NearestNeighbor = _make_client("nearest_neighbor")
Anomaly = _make_client("anomaly")
Clustering = _make_client("clustering")
Graph = _make_client("graph")
Bandit = _make_client("bandit")
Burst = _make_client("burst")
Stat = _make_client("stat")
Weight = _make_client("weight")


def _train_classifier(self, data):
    wire = []
    for x in data:
        if isinstance(x, LabeledDatum):
            wire.append([x.label, x.data.to_msgpack()])
        else:
            lab, d = x
            wire.append([lab, (d if isinstance(d, Datum) else Datum(d)).to_msgpack()])
    return self.call("train", wire)


Classifier.train = _train_classifier
