"""stat / weight / bandit / burst / graph engines: model semantics and the
servers end to end (reference client_test/{stat,graph}_test.cpp API coverage
plus numeric checks of our own: window eviction, entropy, UCB1 order, exp3
updates, Kleinberg bursts, PageRank fixed point, hop-limited paths)."""
import json
import math

import pytest

from helpers import config_path, start_standalone
from jubatus_amd.client import (ArmInfo, Bandit, Batch, Burst, Datum, Document, Edge, Feature, Graph,
                                KeywordWithParams, Node, PresetQuery, Query, ShortestPathQuery, Stat,
                                Weight, Window)
from jubatus_amd.models.bandit import Bandit as BanditModel
from jubatus_amd.models.burst import Burst as BurstModel
from jubatus_amd.models.burst import detect
from jubatus_amd.models.graph import Graph as GraphModel
from jubatus_amd.models.graph import GraphError, UnknownId
from jubatus_amd.models.stat import Stat as StatModel
from jubatus_amd.models.stat import StatError


# ------------------------------------------------------------------ stat
def test_stat_window_and_moments():
    s = StatModel(4)
    for k, v in [("a", 1.0), ("a", 5.0), ("b", 2.0), ("a", 3.0)]:
        s.push(k, v)
    assert s.sum("a") == 9.0 and s.max("a") == 5.0 and s.min("a") == 1.0
    assert s.stddev("a") == pytest.approx(math.sqrt((1 + 25 + 9) / 3 - 9))
    assert s.moment("a", 2, 3.0) == pytest.approx((4 + 4 + 0) / 3)
    assert s.moment("a", 0, 7.0) == 1.0
    s.push("b", 4.0)             # evicts a=1 -> min recomputed
    assert s.min("a") == 3.0 and s.sum("a") == 8.0
    # entropy over the window's key distribution {a:2, b:2}
    assert s.entropy() == pytest.approx(math.log(2))
    s.push("c", 1.0)
    s.push("c", 1.0)
    s.push("c", 1.0)             # window = b, c, c, c
    with pytest.raises(StatError):
        s.sum("a")
    with pytest.raises(StatError):
        s.moment("b", -1, 0.0)


def test_stat_mix_entropy():
    a, b = StatModel(10), StatModel(10)
    a.push("x", 1)
    a.push("x", 1)
    b.push("y", 1)
    b.push("y", 1)
    m = StatModel.mix_diff(a.get_diff(), b.get_diff())
    a.put_diff(m)
    assert a.entropy() == pytest.approx(math.log(2))


def test_stat_server(tmp_path):
    h = start_standalone("stat", config_path("stat/stat.json"), tmp_path)
    try:
        with Stat("127.0.0.1", h.argv.port, "") as c:
            assert c.get_config()
            st = list(c.get_status().values())[0]
            assert st["type"] == "stat"
            for v in (1.0, 2.0, 3.0):
                assert c.push("k", v) is True
            assert c.sum("k") == 6.0 and c.max("k") == 3.0 and c.min("k") == 1.0
            assert c.stddev("k") == pytest.approx(math.sqrt(2 / 3))
            assert c.moment("k", 1, 1.0) == pytest.approx(1.0)
            assert c.entropy("ignored") == pytest.approx(0.0)
            with pytest.raises(Exception):
                c.sum("missing")
            assert len(c.save("s")) == 1
            assert c.clear() is True
            assert c.load("s") is True and c.sum("k") == 6.0
    finally:
        h.stop()


# ---------------------------------------------------------------- weight
def test_weight_server(tmp_path):
    cfg = json.dumps({"converter": {"string_rules": [{"key": "*", "type": "space",
                                                       "sample_weight": "tf", "global_weight": "idf"}],
                                    "num_rules": [{"key": "*", "type": "num"}]}})
    h = start_standalone("weight", cfg, tmp_path)
    try:
        with Weight("127.0.0.1", h.argv.port, "") as c:
            f = c.update(Datum({"t": "hello world", "n": 2.0}))
            assert all(isinstance(x, Feature) for x in f)
            d = {x.key: x.value for x in f}
            assert d["n@num"] == 2.0
            c.update(Datum({"t": "hello there"}))
            w = {x.key: x.value for x in c.calc_weight(Datum({"t": "hello world"}))}
            # idf(hello) = log(2/2) = 0 < idf(world) = log(2/1)
            assert w["t$hello@space#tf/idf"] == pytest.approx(0.0)
            assert w["t$world@space#tf/idf"] == pytest.approx(math.log(2))
            before = c.calc_weight(Datum({"t": "x y"}))
            assert c.calc_weight(Datum({"t": "x y"})) == before     # calc_weight does not update
            assert c.clear() is True
    finally:
        h.stop()


# ---------------------------------------------------------------- bandit
def test_ucb1_tries_every_arm_then_exploits():
    b = BanditModel("ucb1", {"assume_unrewarded": False})
    for a in ("a", "b", "c"):
        assert b.register_arm(a)
    assert not b.register_arm("a")
    seen = []
    for _ in range(3):
        arm = b.select_arm("p")
        seen.append(arm)
        b.register_reward("p", arm, 1.0 if arm == "b" else 0.0)
    assert seen == ["a", "b", "c"]
    picks = []
    for _ in range(30):
        arm = b.select_arm("p")
        picks.append(arm)
        b.register_reward("p", arm, 1.0 if arm == "b" else 0.0)
    assert picks.count("b") > 20
    info = b.get_arm_info("p")
    assert sum(n for n, _ in info.values()) == 33 and info["b"][1] == info["b"][0]


def test_assume_unrewarded_counts_on_select():
    b = BanditModel("epsilon_greedy", {"assume_unrewarded": True, "epsilon": 0.5, "seed": 3})
    b.register_arm("x")
    b.select_arm("p")
    assert b.get_arm_info("p")["x"] == (1, 0.0)
    b.register_reward("p", "x", 2.0)
    assert b.get_arm_info("p")["x"] == (1, 2.0)
    assert b.register_reward("p", "nope", 1.0) is False


def test_exp3_and_softmax_prefer_rewarded_arm():
    for method, p in (("exp3", {"gamma": 0.2}), ("softmax", {"tau": 0.1})):
        b = BanditModel(method, {"assume_unrewarded": False, "seed": 0, **p})
        b.register_arm("good")
        b.register_arm("bad")
        for _ in range(300):
            arm = b.select_arm("u")
            b.register_reward("u", arm, 1.0 if arm == "good" else 0.0)
        info = b.get_arm_info("u")
        assert info["good"][0] > info["bad"][0]


def test_bandit_mix_sums_deltas():
    a = BanditModel("ucb1", {"assume_unrewarded": False})
    b = BanditModel("ucb1", {"assume_unrewarded": False})
    for m in (a, b):
        m.register_arm("x")
    a.register_reward("p", "x", 1.0)
    b.register_reward("p", "x", 3.0)
    mixed = BanditModel.mix_diff(a.get_diff(), b.get_diff())
    a.put_diff(mixed)
    b.put_diff(mixed)
    assert a.get_arm_info("p") == b.get_arm_info("p") == {"x": (2, 4.0)}
    a.register_reward("p", "x", 1.0)
    assert a.get_arm_info("p") == {"x": (3, 5.0)}


@pytest.mark.parametrize("cfg", ["ucb1", "epsilon_greedy", "softmax", "exp3"])
def test_bandit_server(tmp_path, cfg):
    h = start_standalone("bandit", config_path(f"bandit/{cfg}.json"), tmp_path)
    try:
        with Bandit("127.0.0.1", h.argv.port, "") as c:
            with pytest.raises(Exception):
                c.select_arm("p")
            assert c.register_arm("a1") and c.register_arm("a2")
            arm = c.select_arm("p")
            assert arm in ("a1", "a2")
            assert c.register_reward("p", arm, 1.0) is True
            info = c.get_arm_info("p")
            assert set(info) == {"a1", "a2"} and all(isinstance(v, ArmInfo) for v in info.values())
            assert info[arm].weight == 1.0
            assert c.delete_arm("a2") is True and c.delete_arm("a2") is False
            assert c.reset("p") is True and c.get_arm_info("p")["a1"].trial_count == 0
            c.save("b")
            assert c.clear() is True
            assert c.load("b") is True
    finally:
        h.stop()


# ----------------------------------------------------------------- burst
def test_detect_finds_burst():
    d = [100] * 10
    r = [5, 5, 5, 5, 5, 40, 45, 5, 5, 5]
    w = detect(d, r, 2.0, 1.0)
    assert w[5] > 0 and w[6] > 0
    assert all(x == 0 for i, x in enumerate(w) if i not in (5, 6))
    assert detect([10] * 4, [0] * 4, 2.0, 1.0) == [0.0] * 4


def test_burst_window_slides_and_rejects_old():
    b = BurstModel("burst", {"window_batch_size": 5, "batch_interval": 10, "max_reuse_batch_num": 5,
                             "costcut_threshold": -1, "result_window_rotate_size": 3})
    assert b.add_keyword("fire", 2.0, 1.0)
    assert not b.add_keyword("fire", 2.0, 1.0)
    assert b.add_document("nothing", 45.0)          # window [0, 50)
    assert b.start == 0.0
    for i in range(50):
        b.add_document("fire here" if 40 <= i < 48 else "calm", float(i))
    b.calculate_results()
    start, batches = b.get_result("fire")
    assert start == 0.0 and len(batches) == 5
    assert batches[4][1] == 8 and batches[4][2] > 0
    assert "fire" in b.get_all_bursted_results()
    assert b.add_document("calm", 75.0)             # slides to [30, 80)
    b.calculate_results()
    assert b.get_result("fire")[0] == 30.0
    assert not b.add_document("too old", 5.0)
    assert b.get_result_at("fire", 5.0)[0] == 0.0   # the old window is kept
    assert b.get_result("unknown") == (0.0, [])


def test_burst_server(tmp_path):
    h = start_standalone("burst", config_path("burst/burst.json"), tmp_path)
    try:
        with Burst("127.0.0.1", h.argv.port, "") as c:
            assert c.add_keyword(KeywordWithParams("jubatus", 2.0, 1.0)) is True
            kws = c.get_all_keywords()
            assert [k.keyword for k in kws] == ["jubatus"]
            docs = [Document(float(t), "jubatus rocks" if 40 <= t < 50 and t % 2 else "nothing")
                    for t in range(50)]
            assert c.add_documents(docs) == 50
            w = c.get_result("jubatus")
            assert isinstance(w, Window) and len(w.batches) == 5
            assert all(isinstance(x, Batch) for x in w.batches)
            assert w.batches[4].relevant_data_count == 5 and w.batches[4].burst_weight > 0
            assert "jubatus" in c.get_all_bursted_results()
            assert c.get_result_at("jubatus", 45.0).start_pos == w.start_pos
            assert "jubatus" in c.get_all_bursted_results_at(45.0)
            c.save("b")
            assert c.remove_keyword("jubatus") is True and c.get_all_keywords() == []
            assert c.load("b") is True and len(c.get_all_keywords()) == 1
            assert c.remove_all_keywords() is True
            assert c.clear() is True
    finally:
        h.stop()


# ----------------------------------------------------------------- graph
Q0 = [[], []]


def test_pagerank_and_paths():
    g = GraphModel("graph_wo_index", {"damping_factor": 0.85, "landmark_num": 5})
    for i in range(4):
        g.create_node(i)
    g.update_node(0, {"kind": "hub"})
    eid = 100
    for s, t in [(1, 0), (2, 0), (3, 0), (0, 1)]:
        g.create_edge(eid, s, t, {"rel": "x"})
        eid += 1
    g.add_centrality_query(Q0)
    g.add_shortest_path_query(Q0)
    g.update_index()
    sc = {i: g.get_centrality(i, 0, Q0) for i in range(4)}
    # fixed point check: s = 0.15 + 0.85 * sum_in s(src) / outdeg(src)
    assert sc[0] == pytest.approx(0.15 + 0.85 * (sc[1] + sc[2] + sc[3]), rel=1e-6)
    assert sc[0] > sc[1] > sc[2]
    assert g.get_shortest_path(2, 1, 5, Q0) == [2, 0, 1]
    assert g.get_shortest_path(2, 1, 1, Q0) == []
    assert g.get_shortest_path(0, 3, 5, Q0) == []
    # node-property filtered query: only "hub" survives
    qn = [[], [["kind", "hub"]]]
    g.add_centrality_query(qn)
    g.update_index()
    assert g.get_centrality(0, 0, qn) == pytest.approx(0.15)
    with pytest.raises(GraphError):
        g.get_centrality(0, 0, [[["rel", "y"]], []])   # not registered
    with pytest.raises(GraphError):
        g.remove_node(0)                               # has edges
    with pytest.raises(UnknownId):
        g.get_node(99)
    g.remove_edge(103)
    assert g.get_node(0)["out_edges"] == []


def test_graph_mix_union():
    a = GraphModel("graph_wo_index", {})
    b = GraphModel("graph_wo_index", {})
    a.create_node(1)
    b.create_node(2)
    a.global_nodes.add(2)
    a.create_edge(10, 1, 2, {})
    a.add_shortest_path_query(Q0)
    m = GraphModel.mix_diff(a.get_diff(), b.get_diff())
    a.put_diff(m)
    b.put_diff(m)
    assert b.get_shortest_path(1, 2, 3, Q0) == [1, 2]
    assert b.get_edge(10) == ({}, 1, 2)


def test_graph_server(tmp_path):
    h = start_standalone("graph", config_path("graph/graph_wo_index.json"), tmp_path)
    try:
        with Graph("127.0.0.1", h.argv.port, "") as c:
            st = list(c.get_status().values())[0]
            assert st["type"] == "graph"
            n = [c.create_node() for _ in range(3)]
            assert len(set(n)) == 3
            assert c.update_node(n[0], {"color": "red"}) is True
            e1 = c.create_edge(n[0], Edge({"w": "1"}, n[0], n[1]))
            e2 = c.create_edge(n[1], Edge({}, n[1], n[2]))
            assert c.get_edge(n[0], e1) == Edge({"w": "1"}, n[0], n[1])
            node = c.get_node(n[1])
            assert isinstance(node, Node) and node.in_edges == [e1] and node.out_edges == [e2]
            q = PresetQuery([], [])
            assert c.add_centrality_query(q) and c.add_shortest_path_query(q)
            assert c.update_index() is True
            assert c.get_centrality(n[2], 0, q) > c.get_centrality(n[0], 0, q)
            with pytest.raises(Exception):
                c.get_centrality(n[2], 1, q)
            assert c.get_shortest_path(ShortestPathQuery(n[0], n[2], 10, q)) == n
            assert c.update_edge(n[0], e1, Edge({"w": "2"}, n[0], n[1])) is True
            assert c.get_edge(n[0], e1).property == {"w": "2"}
            c.save("g")
            assert c.remove_edge(n[1], e2) is True
            assert c.remove_centrality_query(q) and c.remove_shortest_path_query(q)
            assert c.clear() is True
            assert c.load("g") is True
            assert c.get_node(n[1]).out_edges == [e2]
            with pytest.raises(Exception):
                c.get_node("999999")
            _ = Query("a", "b")
    finally:
        h.stop()
