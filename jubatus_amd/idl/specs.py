"""Service definitions of the 11 engines (the IDL contract).

Reference: jubatus/server/server/*.idl and the decorator semantics of the
jenerator (tools/jenerator/src/syntax.ml:111-130, cpp.ml:558-603):

* routing  random | broadcast | cht(n) | internal     (#@cht means cht(2))
* lock     update (write lock + event_model_updated) | analysis (read lock) | nolock
* agg      pass | all_and | all_or | merge | concat | add

Every public method takes the cluster ``name`` as a leading argument on the
wire (the proxy routes on it; servers ignore it). ``args`` below lists the
arguments *after* ``name``. This table drives the server dispatch
(framework/server_helper.py), the proxy routing (framework/proxy.py), the
client stubs (client/) and the generated API reference (idl/gen_docs.py).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Method:
    name: str
    args: tuple[str, ...]      # "name:type"
    ret: str
    routing: str               # random | broadcast | cht | internal
    lock: str                  # update | analysis | nolock
    agg: str = "pass"
    cht_n: int = 2
    doc: str = ""

    @property
    def arity(self) -> int:
        return len(self.args) + 1  # + cluster name


def split_args(spec: str) -> tuple[str, ...]:
    """split "a:t1, b:map<string,string>" on top-level commas only"""
    out, depth, cur = [], 0, ""
    for ch in spec:
        depth += (ch == "<") - (ch == ">")
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    out.append(cur.strip())
    return tuple(a for a in out if a)


def M(name, args, ret, routing, lock, agg="pass", cht_n=2, doc=""):
    if isinstance(args, str):
        args = split_args(args)
    return Method(name, tuple(args), ret, routing, lock, agg, cht_n, doc)


# message types per engine (the reference IDLs' ``message`` blocks; field
# order is the wire order). ``datum`` is built in.
MESSAGES: dict[str, tuple[tuple[str, tuple[str, ...]], ...]] = {
    "classifier": (("estimate_result", ("label:string", "score:double")),
                   ("labeled_datum", ("label:string", "data:datum"))),
    "regression": (("scored_datum", ("score:float", "data:datum")),),
    "recommender": (("id_with_score", ("id:string", "score:float")),),
    "nearest_neighbor": (("id_with_score", ("id:string", "score:float")),),
    "anomaly": (("id_with_score", ("id:string", "score:float")),),
    "clustering": (("weighted_datum", ("weight:double", "point:datum")),),
    "graph": (("node", ("property:map<string,string>", "in_edges:list<ulong>", "out_edges:list<ulong>")),
              ("query", ("from_id:string", "to_id:string")),
              ("preset_query", ("edge_query:list<query>", "node_query:list<query>")),
              ("edge", ("property:map<string,string>", "source:string", "target:string")),
              ("shortest_path_query", ("source:string", "target:string", "max_hop:uint",
                                       "query:preset_query"))),
    "bandit": (("arm_info", ("trial_count:int", "weight:double")),),
    "burst": (("keyword_with_params", ("keyword:string", "scaling_param:double", "gamma:double")),
              ("batch", ("all_data_count:int", "relevant_data_count:int", "burst_weight:double")),
              ("window", ("start_pos:double", "batches:list<batch>")),
              ("document", ("pos:double", "text:string"))),
    "stat": (),
    "weight": (("feature", ("key:string", "value:float")),),
}


# methods every engine has (framework + generated impl; proxy.cpp:43-66)
COMMON = (
    M("get_config", "", "string", "random", "analysis"),
    M("save", "id:string", "map<string,string>", "broadcast", "analysis", "merge"),
    M("load", "id:string", "bool", "broadcast", "update", "all_and"),
    M("get_status", "", "map<string,map<string,string>>", "broadcast", "analysis", "merge"),
)

SERVICES: dict[str, tuple[Method, ...]] = {
    # classifier.idl:41-80 (every method NOLOCK at the impl: classifier_impl.cpp:54-83)
    "classifier": (
        M("train", "data:list<labeled_datum>", "int", "random", "nolock"),
        M("classify", "data:list<datum>", "list<list<estimate_result>>", "random", "nolock"),
        M("get_labels", "", "map<string,ulong>", "random", "nolock"),
        M("set_label", "new_label:string", "bool", "broadcast", "nolock", "all_and"),
        M("clear", "", "bool", "broadcast", "nolock", "all_and"),
        M("delete_label", "target_label:string", "bool", "broadcast", "nolock", "all_or"),
    ),
    # regression.idl:25-31
    "regression": (
        M("train", "train_data:list<scored_datum>", "int", "random", "update"),
        M("estimate", "estimate_data:list<datum>", "list<float>", "random", "analysis"),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
    ),
    # recommender.idl:25-55
    "recommender": (
        M("clear_row", "id:string", "bool", "cht", "update", "all_and"),
        M("update_row", "id:string, row:datum", "bool", "cht", "update", "all_and"),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
        M("complete_row_from_id", "id:string", "datum", "cht", "analysis"),
        M("complete_row_from_datum", "row:datum", "datum", "random", "analysis"),
        M("similar_row_from_id", "id:string, size:uint", "list<id_with_score>", "cht", "analysis"),
        M("similar_row_from_datum", "row:datum, size:uint", "list<id_with_score>", "random", "analysis"),
        M("decode_row", "id:string", "datum", "cht", "analysis"),
        M("get_all_rows", "", "list<string>", "random", "analysis"),
        M("calc_similarity", "lhs:datum, rhs:datum", "float", "random", "analysis"),
        M("calc_l2norm", "row:datum", "float", "random", "analysis"),
    ),
    # nearest_neighbor.idl:8-26 (analysis methods lock-free: ChangeLog.rst:102)
    "nearest_neighbor": (
        M("clear", "", "bool", "broadcast", "update", "all_and"),
        M("set_row", "id:string, d:datum", "bool", "cht", "update", "pass", cht_n=1),
        M("neighbor_row_from_id", "id:string, size:uint", "list<id_with_score>", "random", "nolock"),
        M("neighbor_row_from_datum", "query:datum, size:uint", "list<id_with_score>", "random", "nolock"),
        M("similar_row_from_id", "id:string, ret_num:uint", "list<id_with_score>", "random", "nolock"),
        M("similar_row_from_datum", "query:datum, ret_num:uint", "list<id_with_score>", "random", "nolock"),
        M("get_all_rows", "", "list<string>", "random", "nolock"),
    ),
    # anomaly.idl:26-49
    "anomaly": (
        M("clear_row", "id:string", "bool", "cht", "update", "all_and"),
        M("add", "row:datum", "id_with_score", "random", "nolock"),
        M("update", "id:string, row:datum", "float", "cht", "update"),
        M("overwrite", "id:string, row:datum", "float", "cht", "update"),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
        M("calc_score", "row:datum", "float", "random", "analysis"),
        M("get_all_rows", "", "list<string>", "random", "analysis"),
    ),
    # clustering.idl:26-44
    "clustering": (
        M("push", "points:list<datum>", "bool", "random", "update"),
        M("get_revision", "", "uint", "random", "analysis"),
        M("get_core_members", "", "list<list<weighted_datum>>", "random", "analysis"),
        M("get_k_center", "", "list<datum>", "random", "analysis"),
        M("get_nearest_center", "point:datum", "datum", "random", "analysis"),
        M("get_nearest_members", "point:datum", "list<weighted_datum>", "random", "analysis"),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
    ),
    # graph.idl:54-105
    "graph": (
        M("create_node", "", "string", "random", "nolock"),
        M("remove_node", "node_id:string", "bool", "cht", "nolock"),
        M("update_node", "node_id:string, property:map<string,string>", "bool", "cht", "update", "all_and"),
        M("create_edge", "node_id:string, e:edge", "ulong", "cht", "nolock", "pass", cht_n=1),
        M("update_edge", "node_id:string, edge_id:ulong, e:edge", "bool", "cht", "update", "all_and"),
        M("remove_edge", "node_id:string, edge_id:ulong", "bool", "cht", "update", "all_and"),
        M("get_centrality", "node_id:string, centrality_type:int, query:preset_query", "double",
          "random", "analysis"),
        M("add_centrality_query", "query:preset_query", "bool", "broadcast", "update", "all_and"),
        M("add_shortest_path_query", "query:preset_query", "bool", "broadcast", "update", "all_and"),
        M("remove_centrality_query", "query:preset_query", "bool", "broadcast", "update", "all_and"),
        M("remove_shortest_path_query", "query:preset_query", "bool", "broadcast", "update", "all_and"),
        M("get_shortest_path", "query:shortest_path_query", "list<string>", "random", "analysis"),
        M("update_index", "", "bool", "broadcast", "update", "all_and"),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
        M("get_node", "node_id:string", "node", "cht", "analysis"),
        M("get_edge", "node_id:string, edge_id:ulong", "edge", "cht", "analysis"),
        M("create_node_here", "node_id:string", "bool", "internal", "update"),
        M("remove_global_node", "node_id:string", "bool", "internal", "update"),
        M("create_edge_here", "edge_id:ulong, e:edge", "bool", "internal", "update"),
    ),
    # bandit.idl:17-91
    "bandit": (
        M("register_arm", "arm_id:string", "bool", "broadcast", "update", "all_and"),
        M("delete_arm", "arm_id:string", "bool", "broadcast", "update", "all_and"),
        M("select_arm", "player_id:string", "string", "cht", "update", "pass", cht_n=1),
        M("register_reward", "player_id:string, arm_id:string, reward:double", "bool", "cht",
          "update", "all_and", cht_n=1),
        M("get_arm_info", "player_id:string", "map<string,arm_info>", "cht", "analysis", "pass", cht_n=1),
        M("reset", "player_id:string", "bool", "broadcast", "update", "all_or"),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
    ),
    # burst.idl:42-69
    "burst": (
        M("add_documents", "data:list<document>", "int", "broadcast", "update", "pass"),
        M("get_result", "keyword:string", "window", "cht", "analysis"),
        M("get_result_at", "keyword:string, pos:double", "window", "cht", "analysis"),
        M("get_all_bursted_results", "", "map<string,window>", "broadcast", "analysis", "merge"),
        M("get_all_bursted_results_at", "pos:double", "map<string,window>", "broadcast", "analysis", "merge"),
        M("get_all_keywords", "", "list<keyword_with_params>", "random", "analysis"),
        M("add_keyword", "keyword:keyword_with_params", "bool", "broadcast", "update", "all_and"),
        M("remove_keyword", "keyword:string", "bool", "broadcast", "update", "all_and"),
        M("remove_all_keywords", "", "bool", "broadcast", "update", "all_and"),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
    ),
    # stat.idl:20-36
    "stat": (
        M("push", "key:string, value:double", "bool", "cht", "update", "all_and", cht_n=1),
        M("sum", "key:string", "double", "cht", "analysis", "pass", cht_n=1),
        M("stddev", "key:string", "double", "cht", "analysis", "pass", cht_n=1),
        M("max", "key:string", "double", "cht", "analysis", "pass", cht_n=1),
        M("min", "key:string", "double", "cht", "analysis", "pass", cht_n=1),
        M("entropy", "key:string", "double", "cht", "analysis", "pass", cht_n=1),
        M("moment", "key:string, degree:int, center:double", "double", "cht", "analysis", "pass", cht_n=1),
        M("clear", "", "bool", "broadcast", "update", "all_and"),
    ),
    # weight.idl:24-30
    "weight": (
        M("update", "d:datum", "list<feature>", "random", "nolock"),
        M("calc_weight", "d:datum", "list<feature>", "random", "nolock"),
        M("clear", "", "bool", "broadcast", "nolock", "all_and"),
    ),
}

# engines whose servers register on the consistent hash ring (use_cht =
# "service has any cht method", cpp.ml:579-603)
def uses_cht(engine: str) -> bool:
    return any(m.routing == "cht" for m in SERVICES[engine])


def methods(engine: str) -> tuple[Method, ...]:
    return COMMON + SERVICES[engine]


ENGINES = tuple(SERVICES)
