"""Distributed mode of the native host-engine servers on the CPU (no GPU, no
Python in the server processes): two jubastat / jubabandit / jubaweight
servers join a cluster through the native coordinator, register their actor
(and CHT vnodes for the CHT-routed engines), and mix with the native linear
mixer over the control plane (csrc/server/jb_host_server.hpp). After a MIX
both answer as one server holding everything would: stat's entropy over the
cluster's windows, bandit's summed arm statistics, weight's document
frequencies. Reference: linear_mixer.cpp:358-544 and the Python drivers'
get_diff / mix_diff / put_diff (models/{stat,bandit,weight}.py)."""
import json
import math
import os
import socket
import subprocess
import tempfile
import time

import pytest

from jubatus_amd.client import Client, Datum
from jubatus_amd.common import config as zkconfig
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import NativeCoordinator, native_available
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import wait_server

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = os.path.join(ROOT, "jubatus_amd", "native_bin")

pytestmark = pytest.mark.skipif(not (native_available() and os.path.exists(os.path.join(NB, "jubastat"))),
                                reason="native binaries not built")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def coord():
    srv = NativeCoordinator(0, "127.0.0.1")
    yield srv
    srv.stop()


def status(c):
    (_, st), = c.get_status().items()
    return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
            for k, v in st.items()}


class Cluster:
    def __init__(self, coord, engine, name, cfg, n=2, extra=(), mixer="linear_mixer", start=True):
        self.ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
        zkconfig.config_tozk(self.ls, engine, name, json.dumps(cfg))
        self.engine, self.name, self.coord, self.mixer = engine, name, coord, mixer
        self.extra = tuple(extra) + (("-x", mixer) if mixer != "linear_mixer" else ())
        self.ports, self.procs, self.c = [], [], []
        for _ in range(n if start else 0):
            self.add()
        if start:
            self.wait_group(n)

    def add(self):
        p = free_port()
        log = open(os.path.join(tempfile.gettempdir(), f"hostdist_{self.name}_{p}.log"), "wb")
        self.procs.append(subprocess.Popen(
            [os.path.join(NB, f"juba{self.engine}"), "-z", f"127.0.0.1:{self.coord.port}", "-n", self.name,
             "-p", str(p), "-b", "127.0.0.1", "-s", "0", "-i", "0", "-I", "5", "-Z", "5", *self.extra],
            stdout=subprocess.DEVNULL, stderr=log))
        assert wait_server("127.0.0.1", p, 60)
        self.ports.append(p)
        self.c.append(Client("127.0.0.1", p, self.name, timeout=30.0))
        return self.c[-1]

    def wait_group(self, n):
        k = self.mixer
        deadline = time.time() + 60
        while time.time() < deadline:
            sts = [status(c) for c in self.c]
            if all(s.get(f"{k}.group_size") == str(n) and s.get(f"{k}.is_obsolete") == "0" for s in sts):
                return
            time.sleep(0.2)
        raise AssertionError("group did not form")

    def mix(self, at_least=1):
        assert self.c[0].do_mix() is True
        deadline = time.time() + 20
        while time.time() < deadline:
            if all(int(status(c).get(f"{self.mixer}.mix_count", "0")) >= at_least for c in self.c):
                return
            time.sleep(0.1)

    def close(self):
        for c in self.c:
            c.close()
        for p in self.procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    p.kill()
        self.ls.close()


def test_native_stat_distributed_entropy(coord):
    cl = Cluster(coord, "stat", "sdist", {"window_size": 64})
    try:
        st = status(cl.c[0])
        assert st["server_runtime"] == "native" and st["linear_mixer.runtime"] == "native"
        assert st["is_standalone"] == "0"
        assert st["use_cht"] == "1"      # server_helper<stat_serv>(a, true) (stat_impl.cpp:20)
        # CHT-routed engine: 8 vnodes per server
        assert len(cl.ls.list(mb.build_actor_path("stat", "sdist") + "/cht")) == 16
        keys = {}
        for i in range(20):
            k = f"k{i % 5}"
            # cht(1): a key lives on one server (k0, k1 here; the rest there)
            cl.c[0 if k in ("k0", "k1") else 1].call("push", k, float(i))
            keys[k] = keys.get(k, 0) + 1
        cl.mix()
        n = sum(keys.values())
        want = math.log(n) - sum(c * math.log(c) for c in keys.values()) / n
        for c in cl.c:
            assert abs(c.call("entropy", "k0") - want) < 1e-9
    finally:
        cl.close()


def test_native_bandit_distributed_arm_info(coord):
    cl = Cluster(coord, "bandit", "bdist", {"method": "ucb1", "parameter": {"assume_unrewarded": False}})
    try:
        a, b = cl.c
        a.call("register_arm", "x")
        b.call("register_arm", "y")
        for _ in range(3):
            a.call("register_reward", "p", "x", 1.0)
        b.call("register_arm", "x")
        b.call("register_reward", "p", "x", 0.5)
        b.call("register_reward", "p", "y", 2.0)
        cl.mix()
        want = {"x": [4, 3.5], "y": [1, 2.0]}
        for c in cl.c:
            info = {(k.decode() if isinstance(k, bytes) else k): list(v)
                    for k, v in c.call("get_arm_info", "p").items()}
            assert info == want, info
        # increments after the MIX are shipped once, not again
        a.call("register_reward", "p", "y", 1.0)
        cl.mix()
        for c in cl.c:
            info = {(k.decode() if isinstance(k, bytes) else k): list(v)
                    for k, v in c.call("get_arm_info", "p").items()}
            assert info["y"] == [2, 3.0] and info["x"] == [4, 3.5], info
    finally:
        cl.close()


def test_native_weight_distributed_idf(coord):
    cfg = json.load(open(os.path.join(ROOT, "config/weight/default.json")))
    cl = Cluster(coord, "weight", "wdist", cfg)
    solo_port = free_port()
    cfg_path = os.path.join(tempfile.gettempdir(), f"wsolo_{solo_port}.json")
    json.dump(cfg, open(cfg_path, "w"))
    solo = subprocess.Popen([os.path.join(NB, "jubaweight"), "-f", cfg_path, "-p", str(solo_port), "-b", "127.0.0.1"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        assert wait_server("127.0.0.1", solo_port, 60)
        s = Client("127.0.0.1", solo_port, "", timeout=30.0)
        docs = [Datum({"text": "the quick brown fox"}), Datum({"text": "the lazy dog"}),
                Datum({"text": "quick quick fox"}), Datum({"text": "a dog and a fox"})]
        for i, d in enumerate(docs):
            cl.c[i % 2].call("update", d)
            s.call("update", d)
        cl.mix()
        q = Datum({"text": "quick dog"})
        want = sorted((k, round(v, 5)) for k, v in s.call("calc_weight", q))
        for c in cl.c:
            got = sorted((k, round(v, 5)) for k, v in c.call("calc_weight", q))
            assert got == want, (got, want)
        s.close()
    finally:
        if solo.poll() is None:
            solo.terminate()
            solo.wait(timeout=15)
        cl.close()


def test_native_burst_distributed_keywords(coord):
    """three jubaburst servers: the proxy broadcasts keywords and documents,
    each keyword is processed by its 2 CHT owners, and after a MIX every
    server answers get_result for every keyword as one standalone server
    does (reference burst_serv.cpp:200-246, models/burst.py MIX)."""
    cfg = json.load(open(os.path.join(ROOT, "config/burst/default.json")))
    cl = Cluster(coord, "burst", "budist", cfg, n=3)
    solo_port = free_port()
    cfg_path = os.path.join(tempfile.gettempdir(), f"busolo_{solo_port}.json")
    json.dump(cfg, open(cfg_path, "w"))
    solo = subprocess.Popen([os.path.join(NB, "jubaburst"), "-f", cfg_path, "-p", str(solo_port), "-b", "127.0.0.1"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        assert wait_server("127.0.0.1", solo_port, 60)
        s = Client("127.0.0.1", solo_port, "", timeout=30.0)
        kws = [f"kw{i}" for i in range(12)]
        for k in kws:
            for c in cl.c + [s]:
                assert c.call("add_keyword", [k, 2.0, 1.0]) is True
        import random
        rng = random.Random(3)
        docs = []
        for t in range(400):
            words = [rng.choice(kws) for _ in range(rng.randint(0, 2))]
            if t > 300 and rng.random() < 0.6:
                words.append("kw3")          # a burst late in the stream
            docs.append([float(t) * 0.25, " ".join(words) or "nothing"])
        for i in range(0, len(docs), 50):
            for c in cl.c + [s]:
                assert c.call("add_documents", docs[i:i + 50]) == 50
        procs = [int(status(c)["processed_keywords"]) for c in cl.c]
        # 2 consecutive vnodes per keyword (a server may own both: cht.cpp:107-143)
        assert len(kws) <= sum(procs) <= 2 * len(kws) and min(procs) < len(kws), procs
        cl.mix()
        for k in kws:
            want = s.call("get_result", k)
            for c in cl.c:
                got = c.call("get_result", k)
                assert got == want, (k, got, want)
        assert s.call("get_all_bursted_results") == cl.c[0].call("get_all_bursted_results")
        s.close()
    finally:
        if solo.poll() is None:
            solo.terminate()
            solo.wait(timeout=15)
        cl.close()


def test_native_graph_distributed_replicated_writes(coord):
    """three jubagraph servers: create_node lands on the node's two CHT
    owners (server-to-server create_node_here), create_edge is replicated to
    the source's other owner, and after a MIX every server answers
    centrality and shortest path over the whole graph as one standalone
    server does (graph_serv.cpp:150-330, models/graph.py MIX)."""
    from jubatus_amd.common.cht import CHT
    cfg = json.load(open(os.path.join(ROOT, "config/graph/default.json")))
    cl = Cluster(coord, "graph", "gdist", cfg, n=3)
    solo_port = free_port()
    cfg_path = os.path.join(tempfile.gettempdir(), f"gsolo_{solo_port}.json")
    json.dump(cfg, open(cfg_path, "w"))
    solo = subprocess.Popen([os.path.join(NB, "jubagraph"), "-f", cfg_path, "-p", str(solo_port), "-b", "127.0.0.1"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    dec = lambda x: x.decode() if isinstance(x, bytes) else x
    try:
        assert wait_server("127.0.0.1", solo_port, 60)
        s = Client("127.0.0.1", solo_port, "", timeout=30.0)
        by_port = dict(zip(cl.ports, cl.c))
        cht = CHT(cl.ls, "graph", "gdist")
        ids, sids = [], []
        for i in range(8):
            nid = dec(cl.c[i % 3].call("create_node"))
            ids.append(nid)
            sids.append(dec(s.call("create_node")))
            owners = {int(p) for _, p in cht.find(nid, 2)}
            for p in owners:                      # the node is on each of its owners
                assert by_port[p].call("get_node", nid) is not None
        assert len(set(ids)) == len(ids)
        edges = [(i, (i + 1) % 8) for i in range(8)] + [(0, 4), (2, 6), (5, 1)]
        for a, b in edges:
            src_owner = int(cht.find(ids[a], 2)[0][1])   # the proxy routes by the source node
            eid = by_port[src_owner].call("create_edge", ids[a], [{}, ids[a], ids[b]])
            s.call("create_edge", sids[a], [{}, sids[a], sids[b]])
            for _, p in cht.find(ids[a], 2):   # stored on both owners of the source
                assert by_port[int(p)].call("get_edge", ids[a], eid) is not None
        q = [[], []]
        for c in cl.c + [s]:
            assert c.call("add_centrality_query", q) is True
            assert c.call("add_shortest_path_query", q) is True
        with pytest.raises(Exception):
            cl.c[0].call("update_index")
        assert s.call("update_index") is True
        cl.mix()
        for i in range(8):
            want = s.call("get_centrality", sids[i], 0, q)
            for c in cl.c:
                assert abs(c.call("get_centrality", ids[i], 0, q) - want) < 1e-9
        want = [sids.index(dec(x)) for x in s.call("get_shortest_path", [sids[0], sids[6], 10, q])]
        for c in cl.c:
            got = [ids.index(dec(x)) for x in c.call("get_shortest_path", [ids[0], ids[6], 10, q])]
            assert got == want, (got, want)
        # remove_node reaches every member's global node set
        lone = dec(cl.c[1].call("create_node"))
        before = [int(status(c)["global_node_num"]) for c in cl.c]
        owner = int(cht.find(lone, 2)[0][1])
        assert by_port[owner].call("remove_node", lone) is True
        after = [int(status(c)["global_node_num"]) for c in cl.c]
        oi = cl.ports.index(owner)
        assert all(a <= b for a, b in zip(after, before)) and after[oi] < before[oi]
        s.close()
    finally:
        if solo.poll() is None:
            solo.terminate()
            solo.wait(timeout=15)
        cl.close()


def test_native_weight_broadcast_mixer_idf_three_members(coord):
    """push MIX of the document statistics: with broadcast_mixer
    every pair meets once per MIX and each member's own counts go to every
    partner, so three members end with the statistics of all documents -
    calc_weight equals a server that saw every document"""
    cfg = json.load(open(os.path.join(ROOT, "config/weight/default.json")))
    cl = Cluster(coord, "weight", "wbc", cfg, n=3, mixer="broadcast_mixer")
    solo_port = free_port()
    cfg_path = os.path.join(tempfile.gettempdir(), f"wbsolo_{solo_port}.json")
    json.dump(cfg, open(cfg_path, "w"))
    solo = subprocess.Popen([os.path.join(NB, "jubaweight"), "-f", cfg_path, "-p", str(solo_port), "-b", "127.0.0.1"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        assert wait_server("127.0.0.1", solo_port, 60)
        s = Client("127.0.0.1", solo_port, "", timeout=30.0)
        docs = [Datum({"text": t}) for t in ("the quick brown fox", "the lazy dog", "quick quick fox",
                                             "a dog and a fox", "brown dog", "the end")]
        for i, d in enumerate(docs):
            cl.c[i % 3].call("update", d)
            s.call("update", d)
        cl.mix()
        q = Datum({"text": "quick dog the fox"})
        want = sorted((k, round(v, 5)) for k, v in s.call("calc_weight", q))
        for c in cl.c:
            got = sorted((k, round(v, 5)) for k, v in c.call("calc_weight", q))
            assert got == want, (got, want)
        # a second MIX with nothing new changes nothing (no double counting)
        cl.mix(at_least=2)
        for c in cl.c:
            assert sorted((k, round(v, 5)) for k, v in c.call("calc_weight", q)) == want
        s.close()
    finally:
        if solo.poll() is None:
            solo.terminate()
            solo.wait(timeout=15)
        cl.close()


def test_native_random_mixer_late_members_agree_round(coord):
    """push mixers pair members by the MIX round number; a member
    that mixed alone before the others joined has a higher count. The count
    is agreed in the MIX trigger, so three members with different counts
    still pair up and every MIX completes"""
    cfg = json.load(open(os.path.join(ROOT, "config/weight/default.json")))
    cl = Cluster(coord, "weight", "wrm", cfg, n=0, mixer="random_mixer", start=False)
    try:
        a = cl.add()
        cl.wait_group(1)
        for _ in range(3):                      # solo MIXes: a's count moves ahead
            assert a.do_mix() is True
        assert int(status(a)["random_mixer.mix_count"]) >= 3
        cl.add()
        cl.add()
        cl.wait_group(3)
        for d in ("alpha beta", "beta gamma", "gamma delta"):
            for c in cl.c:
                c.call("update", Datum({"text": d}))
        counts = [int(status(c)["random_mixer.mix_count"]) for c in cl.c]
        for _ in range(3):
            assert cl.c[1].do_mix() is True
        deadline = time.time() + 20
        while True:
            after = [int(status(c)["random_mixer.mix_count"]) for c in cl.c]
            if len(set(after)) == 1 or time.time() > deadline:
                break
            time.sleep(0.1)
        assert len(set(after)) == 1 and after[0] >= max(counts) + 3, (counts, after)
        assert all(status(c)["random_mixer.watchdog_aborts"] == "0" for c in cl.c)
    finally:
        cl.close()
