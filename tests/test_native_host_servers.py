"""Native host-engine servers (csrc/server/jb_host_server.hpp: jubastat):
no Python and no GPU in the process, so these run on the CPU. Every call is
checked against the Python driver fed the same sequence (models/stat.py),
including the error messages, and model files move both ways."""
import json
import os
import random
import socket
import subprocess
import time

import pytest

from helpers import ROOT, config_path
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcMethodNotFound, RpcTimeoutError, RpcTypeError

NATIVE_BIN = os.path.join(ROOT, "jubatus_amd", "native_bin")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def stat_server(tmp_path):
    port = _free_port()
    cfg = tmp_path / "stat.json"
    cfg.write_text(json.dumps({"window_size": 16}))
    p = subprocess.Popen([os.path.join(NATIVE_BIN, "jubastat"), "-p", str(port), "-b", "127.0.0.1",
                          "-f", str(cfg), "-d", str(tmp_path)], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT)
    deadline = time.time() + 30
    while True:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            break
        except (OSError, RpcIOError, RpcTimeoutError):
            assert p.poll() is None and time.time() < deadline, p.stdout.read()
            time.sleep(0.1)
    yield port, str(cfg)
    p.terminate()
    p.wait(timeout=30)


def _call(c, m, *a):
    try:
        return ("ok", c.call(m, "", *a))
    except RpcTypeError:
        return ("arg", None)
    except Exception as e:  # noqa: BLE001 - application error text
        return ("err", str(e))


def test_native_stat_matches_python_driver(stat_server):
    from jubatus_amd.models.stat import Stat, StatError
    port, _ = stat_server
    ref = Stat(16)
    rng = random.Random(0)
    keys = ["a", "b", "c", "d"]
    with RpcClient("127.0.0.1", port, 10.0) as c:
        for step in range(400):
            op = rng.choice(["push"] * 4 + ["sum", "stddev", "max", "min", "entropy", "moment"])
            k = rng.choice(keys + ["zz"])
            if op == "push":
                v = rng.uniform(-10, 10)
                assert c.call("push", "", k, v) is ref.push(k, v)
                continue
            args = (k, rng.randrange(0, 4), rng.uniform(-1, 1)) if op == "moment" else (k,)
            got = _call(c, op, *args)
            try:
                want = ("ok", ref.entropy() if op == "entropy" else getattr(ref, op)(*args))
            except StatError as e:
                want = ("err", str(e))
            assert got[0] == want[0], (step, op, got, want)
            if got[0] == "ok":
                assert got[1] == pytest.approx(want[1], rel=1e-9, abs=1e-9), (step, op, args)
            else:
                assert want[1] in got[1]
        (_, st), = c.call("get_status", "").items()
        st = {(k.decode() if isinstance(k, bytes) else k): v for k, v in st.items()}
        assert st["server_runtime"] == "native" and st["window_size"] == "16"
        from test_status_keys import COMMON, DISTRIBUTED
        assert not [k for k in COMMON if k not in st]
        assert not [k for k in DISTRIBUTED if k in st]
        assert int(st["window_population"]) == 16
        assert _call(c, "moment", "a", -1, 0.0)[0] in ("err", "arg") or "a" not in ref.stats
        with pytest.raises(RpcMethodNotFound):
            c.call("no_such", "")
        assert _call(c, "push", "a")[0] == "arg"           # arity
        assert _call(c, "push", "a", "x")[0] == "arg"      # type


def test_native_stat_model_files_both_ways(stat_server, tmp_path):
    from jubatus_amd.framework import save_load
    from jubatus_amd.models.stat import Stat
    port, cfg = stat_server
    text = open(cfg).read()
    with RpcClient("127.0.0.1", port, 10.0) as c:
        for i in range(40):
            c.call("push", "", f"k{i % 3}", float(i))
        (ident, path), = c.call("save", "", "m").items()
        path = path.decode() if isinstance(path, bytes) else path
        ident = ident.decode() if isinstance(ident, bytes) else ident
        with open(path, "rb") as f:
            _, pack = save_load.load_server(f, "stat", text, 1, False)
        ref = Stat(16)
        ref.unpack(pack)
        assert c.call("sum", "", "k1") == pytest.approx(ref.sum("k1"))
        assert c.call("clear", "") is True
        with pytest.raises(Exception):
            c.call("sum", "", "k1")
        assert c.call("load", "", "m") is True
        assert c.call("max", "", "k2") == pytest.approx(ref.max("k2"))
        ref2 = Stat(16)
        for i in range(10):
            ref2.push("p", float(i * i))
        with open(os.path.join(os.path.dirname(path), f"{ident}_stat_py.jubatus"), "wb") as f:
            save_load.save_server(f, "stat", "py", text, 1, ref2.pack())
        assert c.call("load", "", "py") is True
        assert c.call("stddev", "", "p") == pytest.approx(ref2.stddev("p"))
        assert c.call("entropy", "", "ignored") == pytest.approx(ref2.entropy())


def test_native_stat_config_check(tmp_path):
    p = tmp_path / "s.json"
    exe = os.path.join(NATIVE_BIN, "jubastat")
    for cfg, want in ((config_path("stat/default.json"), "native"),):
        r = subprocess.run([exe, "--native-check", "-f", cfg], capture_output=True, text=True, timeout=30)
        assert r.stdout.strip() == want
    p.write_text("{}")
    r = subprocess.run([exe, "--native-check", "-f", str(p)], capture_output=True, text=True, timeout=30)
    assert "window_size" in r.stdout


# ------------------------------------------------------------------ bandit
def _start(exe, cfg_obj, tmp_path):
    port = _free_port()
    cfg = tmp_path / "cfg.json"
    cfg.write_text(json.dumps(cfg_obj))
    p = subprocess.Popen([os.path.join(NATIVE_BIN, exe), "-p", str(port), "-b", "127.0.0.1",
                          "-f", str(cfg), "-d", str(tmp_path)], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT)
    deadline = time.time() + 30
    while True:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            return p, port, str(cfg)
        except (OSError, RpcIOError, RpcTimeoutError):
            assert p.poll() is None and time.time() < deadline, p.stdout.read()
            time.sleep(0.1)


def _norm(x):
    if isinstance(x, bytes):
        return x.decode()
    if isinstance(x, dict):
        return {_norm(k): _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    return x


@pytest.mark.parametrize("unrewarded", [False, True])
def test_native_bandit_ucb1_matches_python_driver(tmp_path, unrewarded):
    """ucb1 is deterministic: the native server and the Python driver pick
    the same arms and keep the same arm_info for the same reward stream"""
    from jubatus_amd.models.bandit import Bandit
    cfg = {"method": "ucb1", "parameter": {"assume_unrewarded": unrewarded}}
    p, port, _ = _start("jubabandit", cfg, tmp_path)
    ref = Bandit("ucb1", cfg["parameter"])
    rng = random.Random(3)
    try:
        with RpcClient("127.0.0.1", port, 10.0) as c:
            assert _call(c, "select_arm", "p")[0] == "err"      # no arm
            for a in ("a0", "a1", "a2"):
                assert c.call("register_arm", "", a) is True and ref.register_arm(a)
            assert c.call("register_arm", "", "a1") is False
            truth = {"a0": 0.2, "a1": 0.8, "a2": 0.5}
            for _ in range(200):
                player = rng.choice(["p", "q"])
                arm = _norm(c.call("select_arm", "", player))
                assert arm == ref.select_arm(player)
                r = 1.0 if rng.random() < truth[arm] else 0.0
                assert c.call("register_reward", "", player, arm, r) is True
                ref.register_reward(player, arm, r)
            for player in ("p", "q"):
                got = _norm(c.call("get_arm_info", "", player))
                want = {a: [n, w] for a, (n, w) in ref.get_arm_info(player).items()}
                assert got == want
            assert c.call("register_reward", "", "p", "nope", 1.0) is False
            assert c.call("delete_arm", "", "a2") is True and ref.delete_arm("a2")
            assert sorted(_norm(c.call("get_arm_info", "", "p"))) == ["a0", "a1"]
            assert c.call("reset", "", "p") is True and ref.reset("p")
            assert _norm(c.call("get_arm_info", "", "p")) == {"a0": [0, 0.0], "a1": [0, 0.0]}
            (_, st), = _norm(c.call("get_status", "")).items()
            assert st["server_runtime"] == "native" and st["num_arms"] == "2"
    finally:
        p.terminate()
        p.wait(timeout=30)


@pytest.mark.parametrize("method,param", [("epsilon_greedy", {"epsilon": 0.1}), ("softmax", {"tau": 0.05}),
                                          ("exp3", {"gamma": 0.1})])
def test_native_bandit_randomized_methods_learn(tmp_path, method, param):
    cfg = {"method": method, "parameter": {"assume_unrewarded": False, "seed": 7, **param}}
    p, port, text = _start("jubabandit", cfg, tmp_path)
    rng = random.Random(5)
    try:
        with RpcClient("127.0.0.1", port, 10.0) as c:
            for a in ("bad", "good"):
                c.call("register_arm", "", a)
            picks = []
            for _ in range(600):
                arm = _norm(c.call("select_arm", "", "u"))
                picks.append(arm)
                c.call("register_reward", "", "u", arm, 1.0 if (arm == "good") == (rng.random() < 0.9) else 0.0)
            assert picks[-200:].count("good") > 120, (method, picks[-200:].count("good"))
            # model file -> the Python driver
            from jubatus_amd.framework import save_load
            from jubatus_amd.models.bandit import Bandit
            (_, path), = _norm(c.call("save", "", "b")).items()
            with open(path, "rb") as f:
                _, pack = save_load.load_server(f, "bandit", open(text).read(), 1, False)
            ref = Bandit(method, cfg["parameter"])
            ref.unpack(pack)
            want = {a: [n, w] for a, (n, w) in ref.get_arm_info("u").items()}
            assert _norm(c.call("get_arm_info", "", "u")) == want
            assert c.call("clear", "") is True
            assert _norm(c.call("get_arm_info", "", "u")) == {}
            assert c.call("load", "", "b") is True
            assert _norm(c.call("get_arm_info", "", "u")) == want
    finally:
        p.terminate()
        p.wait(timeout=30)


# ------------------------------------------------------------------- burst
def _flat(x):
    if isinstance(x, (list, tuple)):
        return [v for e in x for v in _flat(e)]
    return [x]


def _same(a, b):
    fa, fb = _flat(a), _flat(b)
    assert len(fa) == len(fb), (a, b)
    assert fa == pytest.approx(fb, rel=1e-9, abs=1e-9), (a, b)
    return True


def test_native_burst_matches_python_driver(tmp_path):
    from jubatus_amd.framework import save_load
    from jubatus_amd.models.burst import Burst
    from jubatus_amd.server.burst_serv import _window
    cfg = json.load(open(config_path("burst/burst.json")))
    p, port, text = _start("jubaburst", cfg, tmp_path)
    ref = Burst(cfg["method"], cfg["parameter"])
    rng = random.Random(11)
    try:
        with RpcClient("127.0.0.1", port, 10.0) as c:
            for kw, s, g in (("fire", 2.0, 1.0), ("quake", 3.0, 0.5), ("rain", 2.5, 1.0)):
                assert c.call("add_keyword", "", [kw, s, g]) is True
                ref.add_keyword(kw, s, g)
            assert c.call("add_keyword", "", ["fire", 2.0, 1.0]) is False
            assert _call(c, "add_keyword", ["bad", 0.5, 1.0])[0] == "err"
            pos = 0.0
            seen = 0
            for step in range(120):
                docs = []
                for _ in range(rng.randrange(1, 6)):
                    pos += rng.uniform(0, 3)
                    burst = 40 < step < 70
                    words = ["fire" if rng.random() < (0.8 if burst else 0.1) else "calm",
                             "quake" if rng.random() < 0.2 else "", "rain" if rng.random() < 0.3 else ""]
                    docs.append([pos - rng.uniform(0, 60) if rng.random() < 0.05 else pos, " ".join(words)])
                n = c.call("add_documents", "", docs)
                want = sum(ref.add_document(t, float(ps)) for ps, t in docs)
                if want:
                    ref.calculate_results()
                assert n == want
                if step % 10 == 9:
                    for kw in ("fire", "quake", "rain", "none"):
                        assert _same(_norm(c.call("get_result", "", kw)), _window(ref.get_result(kw)))
                        q = pos - rng.uniform(0, 40)
                        assert _same(_norm(c.call("get_result_at", "", kw, q)), _window(ref.get_result_at(kw, q)))
                    got = _norm(c.call("get_all_bursted_results", ""))
                    want_b = {k: _window(v) for k, v in ref.get_all_bursted_results().items()}
                    assert sorted(got) == sorted(want_b)
                    seen += len(got)
                    for k in got:
                        assert _same(got[k], want_b[k])
            assert seen > 0                      # bursts were detected and compared
            q = pos - 30.0
            got = _norm(c.call("get_all_bursted_results_at", "", q))
            assert sorted(got) == sorted(ref.get_all_bursted_results_at(q))
            assert _norm(c.call("get_all_keywords", "")) == [[k, s, g] for k, s, g in ref.get_all_keywords()]
            (ident, path), = _norm(c.call("save", "", "b")).items()
            with open(path, "rb") as f:
                _, pack = save_load.load_server(f, "burst", open(text).read(), 1, False)
            ref2 = Burst(cfg["method"], cfg["parameter"])
            ref2.unpack(pack)
            assert _same(_window(ref2.get_result("fire")), _window(ref.get_result("fire")))
            assert c.call("remove_keyword", "", "rain") is True and c.call("remove_keyword", "", "rain") is False
            assert c.call("clear", "") is True
            assert _norm(c.call("get_result", "", "fire")) == [0.0, []]
            assert c.call("load", "", "b") is True
            assert _same(_norm(c.call("get_result", "", "fire")), _window(ref.get_result("fire")))
            with open(os.path.join(os.path.dirname(path), f"{ident}_burst_py.jubatus"), "wb") as f:
                save_load.save_server(f, "burst", "py", open(text).read(), 1, ref.pack())
            assert c.call("remove_all_keywords", "") is True
            assert c.call("load", "", "py") is True
            assert _norm(c.call("get_all_keywords", "")) == [[k, s, g] for k, s, g in ref.get_all_keywords()]
            (_, st), = _norm(c.call("get_status", "")).items()
            assert st["server_runtime"] == "native" and st["num_keywords"] == "3"
    finally:
        p.terminate()
        p.wait(timeout=30)


# ------------------------------------------------------------------- graph
def _both(tmp_path, engine, cfg_file):
    """(native port, Python server helper) serving the same config"""
    from helpers import start_standalone
    p, port, _ = _start(f"juba{engine}", json.load(open(cfg_file)), tmp_path / "n" if False else tmp_path)
    (tmp_path / "py").mkdir()
    h = start_standalone(engine, cfg_file, tmp_path / "py")
    return p, port, h


def test_native_graph_matches_python_server(tmp_path):
    """the same RPC sequence against the native and the Python jubagraph:
    identical answers and error classes (ids, properties, edges, centrality,
    shortest paths, queries, removal rules)"""
    p, nport, h = _both(tmp_path, "graph", config_path("graph/default.json"))
    rng = random.Random(2)
    try:
        with RpcClient("127.0.0.1", nport, 10.0) as n, RpcClient("127.0.0.1", h.argv.port, 10.0) as y:
            def both(m, *a, same=True):
                rn, ry = _call(n, m, *a), _call(y, m, *a)
                assert rn[0] == ry[0], (m, a, rn, ry)
                if same and rn[0] == "ok":
                    if isinstance(ry[1], float):
                        assert rn[1] == pytest.approx(ry[1], rel=1e-9), (m, a)
                    else:
                        assert _norm(rn[1]) == _norm(ry[1]), (m, a)
                return _norm(rn[1])
            ids = [both("create_node") for _ in range(12)]
            for i in ids:
                both("update_node", i, {"kind": rng.choice(["a", "b"]), "w": str(rng.randrange(3))})
            q_all = [[], []]
            q_a = [[["t", "x"]], [["kind", "a"]]]
            for q in (q_all, q_a):
                both("add_centrality_query", q)
                both("add_shortest_path_query", q)
            eids = []
            for _ in range(30):
                s, t = rng.choice(ids), rng.choice(ids)
                eids.append(both("create_edge", s, [{"t": rng.choice(["x", "y"])}, s, t]))
            both("create_edge", ids[0], [{}, ids[0], "999"])           # unknown target
            both("create_edge", "999", [{}, "999", ids[0]])            # unknown source
            both("get_centrality", ids[0], 0, q_all)                   # before update_index
            both("update_index")
            for i in ids:
                for q in (q_all, q_a):
                    both("get_centrality", i, 0, q)
                both("get_node", i)
            both("get_centrality", ids[0], 1, q_all)                   # unknown type
            both("get_centrality", ids[0], 0, [[["no", "pe"]], []])    # unregistered
            for _ in range(20):
                s, t = rng.choice(ids), rng.choice(ids)
                for q in (q_all, q_a):
                    both("get_shortest_path", [s, t, rng.randrange(1, 5), q])
            both("get_shortest_path", [ids[0], ids[1], 3, [[["x", "y"]], []]])
            for e in eids[:5]:
                both("get_edge", ids[0], e)
                both("update_edge", ids[0], e, [{"t": "z"}, "0", "0"])
                both("get_edge", ids[0], e)
            both("get_edge", ids[0], 10 ** 6)
            both("remove_node", ids[0])                                # has edges
            lonely = both("create_node")
            both("remove_node", lonely)
            both("get_node", lonely)
            for e in eids[5:10]:
                both("remove_edge", ids[0], e)
            both("remove_edge", ids[0], eids[5])
            both("remove_centrality_query", q_a)
            both("get_centrality", ids[1], 0, q_a)
            both("get_node", "not-an-id")
            both("update_index")
            for i in ids[1:4]:
                both("get_centrality", i, 0, q_all)
            # model files: native save -> native load and Python load of the same file
            (_, path), = _norm(n.call("save", "", "g")).items()
            from jubatus_amd.framework import save_load
            from jubatus_amd.models.graph import Graph
            with open(path, "rb") as f:
                _, pack = save_load.load_server(f, "graph", open(config_path("graph/default.json")).read(), 1,
                                                False)
            ref = Graph("graph_wo_index", {})
            ref.unpack(pack)
            assert ref.get_centrality(int(ids[2]), 0, q_all) == pytest.approx(
                n.call("get_centrality", "", ids[2], 0, q_all))
            assert n.call("clear", "") is True
            assert n.call("load", "", "g") is True
            assert _norm(n.call("get_node", "", ids[3])) == _norm(y.call("get_node", "", ids[3]))
            (_, st), = _norm(n.call("get_status", "")).items()
            assert st["server_runtime"] == "native" and st["local_node_num"] == "12"
    finally:
        h.stop()
        p.terminate()
        p.wait(timeout=30)
