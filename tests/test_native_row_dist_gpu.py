"""Distributed mode of the native row servers (no Python in the server
process): two jubaanomaly / jubarecommender servers on this box's GPU join a
cluster through the native coordinator, register CHT vnodes, and mix their
row stores with the row-diff MIX (csrc/server/jb_row_mix.hpp) over the staged
host plane (both share one GPU; between GPUs the same bytes move by RCCL
all-gather). Anomaly adds take a cluster-wide id from the coordinator and go
to the id's CHT owners (server-to-server update). After a MIX the LOF scores
equal those of one standalone server holding the same rows. Reference:
linear_mixer.cpp:358-544, anomaly_serv.cpp:178-211,275-297, cht.cpp:107-143."""
import json
import os
import random
import socket
import subprocess
import tempfile
import time

import pytest

from jubatus_amd.client import Client, Datum
from jubatus_amd.common import config as zkconfig
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import NativeCoordinator
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import wait_server

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = os.path.join(ROOT, "jubatus_amd", "native_bin")


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


def spawn(exe, args, tag):
    log = open(os.path.join(tempfile.gettempdir(), f"row_dist_{tag}.log"), "wb")
    return subprocess.Popen([os.path.join(NB, exe), *args], stdout=subprocess.DEVNULL, stderr=log)


def stop(procs):
    for p in procs:
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()


def status(c):
    (_, st), = c.get_status().items()
    return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
            for k, v in st.items()}


def wait_group(clients, n, timeout=90):
    deadline = time.time() + timeout
    while time.time() < deadline:
        sts = [status(c) for c in clients]
        if all(st.get("linear_mixer.group_size") == str(n) and st.get("linear_mixer.is_obsolete") == "0"
               for st in sts):
            return True
        time.sleep(0.2)
    return False


def _cluster(coord, engine, name, cfg_path, n=2):
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    zkconfig.config_tozk(ls, engine, name, open(cfg_path).read())
    ports = [free_port() for _ in range(n)]
    procs = [spawn(f"juba{engine}", ["-z", f"127.0.0.1:{coord.port}", "-n", name, "-p", str(p), "-b", "127.0.0.1",
                                     "-s", "0", "-i", "0", "-I", "10", "-Z", "5"], f"{name}_{p}") for p in ports]
    for p in ports:
        assert wait_server("127.0.0.1", p, 90)
    clients = [Client("127.0.0.1", p, name, timeout=60.0) for p in ports]
    assert wait_group(clients, n)
    return ls, ports, procs, clients


def _point(rng):
    return Datum({"x": rng.gauss(0, 1), "y": rng.gauss(0, 1), "z": rng.gauss(0, 1)})


def test_native_anomaly_distributed_add_mix_equals_one_node(coord):
    # inverted_index_euclid: exact distances (an LSH backend's quantized
    # distances tie, and ties break by slot order, which differs between a
    # server that was sent rows by a MIX and one that added them itself)
    cfg_path = os.path.join(ROOT, "config/anomaly/default.json")
    ls, ports, procs, (a, b) = _cluster(coord, "anomaly", "adist", cfg_path)
    solo_port = free_port()
    solo = spawn("jubaanomaly", ["-f", cfg_path, "-p", str(solo_port), "-b", "127.0.0.1"], f"solo_{solo_port}")
    procs.append(solo)
    try:
        assert wait_server("127.0.0.1", solo_port, 90)
        s = Client("127.0.0.1", solo_port, "", timeout=60.0)
        rng = random.Random(5)
        ids = []
        for i in range(120):
            d = _point(rng)
            rid, _ = (a if i % 2 == 0 else b).call("add", d)       # cluster-wide id, CHT owners
            rid = rid.decode() if isinstance(rid, bytes) else rid
            ids.append(rid)
            s.call("update", rid, d)                              # the one-node oracle
        assert len(set(ids)) == len(ids)
        for st in (status(a), status(b)):
            assert st["server_runtime"] == "native" and st["linear_mixer.runtime"] == "native"
            assert st["is_standalone"] == "0"
        assert a.do_mix() is True
        deadline = time.time() + 30
        while time.time() < deadline and int(status(b).get("linear_mixer.mix_count", "0")) < 1:
            time.sleep(0.1)
        rows = [sorted(x.decode() if isinstance(x, bytes) else x for x in c.call("get_all_rows"))
                for c in (a, b, s)]
        assert rows[0] == rows[1] == rows[2] == sorted(ids)
        # the LOF tables (kdist / lrd) of a server that inserted rows one by
        # one are incremental; a MIX re-derives them from the mixed rows, as a
        # model load does: the oracle reloads its own model first
        (_, path), = s.save("lof_oracle").items()
        assert s.load("lof_oracle") is True
        q = random.Random(9)
        for _ in range(20):
            d = _point(q)
            want = s.call("calc_score", d)
            for c in (a, b):
                got = c.call("calc_score", d)
                assert abs(got - want) <= 1e-4 * max(1.0, abs(want)), (got, want)
        # CHT vnodes: 8 per server
        assert len(ls.list(mb.build_actor_path("anomaly", "adist") + "/cht")) == 16
        for c in (a, b, s):
            c.close()
    finally:
        stop(procs)
        ls.close()


def test_native_recommender_distributed_mix(coord):
    cfg_path = os.path.join(ROOT, "config/recommender/euclid_lsh.json")
    ls, ports, procs, (a, b) = _cluster(coord, "recommender", "rdist", cfg_path)
    try:
        rng = random.Random(3)
        for i in range(50):
            (a if i < 25 else b).call("update_row", f"r{i}", _point(rng))
        a.call("update_row", "r3", Datum({"x": 9.0, "y": 9.0, "z": 9.0}))   # a newer version of a's row
        b.call("clear_row", "r30")
        assert b.do_mix() is True
        deadline = time.time() + 30
        while time.time() < deadline and int(status(a).get("linear_mixer.mix_count", "0")) < 1:
            time.sleep(0.1)
        want = sorted(f"r{i}" for i in range(50) if i != 30)
        for c in (a, b):
            got = sorted(x.decode() if isinstance(x, bytes) else x for x in c.call("get_all_rows"))
            assert got == want
        da = a.call("decode_row", "r3")
        db = b.call("decode_row", "r3")
        assert da == db
        ra = a.call("similar_row_from_id", "r7", 5)
        rb = b.call("similar_row_from_id", "r7", 5)
        assert [x[0] for x in ra] == [x[0] for x in rb]
        st = status(a)
        assert int(st["linear_mixer.last_mix_bytes"]) > 0
        for c in (a, b):
            c.close()
    finally:
        stop(procs)
        ls.close()


def test_native_clustering_distributed_mix_agrees(coord):
    """two native jubaclustering servers (kmeans.json: 1000-point buckets)
    each push their own points; after a MIX both cluster the union of the
    members' coresets in the same order from the same revision: the same
    k centers (clustering_serv.cpp:108-142; BASELINE config #5)"""
    cfg_path = os.path.join(ROOT, "config/clustering/kmeans.json")
    ls, ports, procs, (a, b) = _cluster(coord, "clustering", "cdist", cfg_path)
    try:
        rng = random.Random(11)
        centers = [(0.0, 0.0), (10.0, 0.0), (0.0, 10.0)]

        def pts(n, which):
            out = []
            for _ in range(n):
                cx, cy = centers[rng.choice(which)]
                out.append(Datum({"x": cx + rng.gauss(0, 0.5), "y": cy + rng.gauss(0, 0.5)}))
            return out
        assert a.call("push", pts(1000, [0, 1])) is True      # a closes one bucket
        assert b.call("push", pts(1000, [1, 2])) is True
        assert a.do_mix() is True
        deadline = time.time() + 30
        while time.time() < deadline and int(status(b).get("linear_mixer.mix_count", "0")) < 1:
            time.sleep(0.1)
        ca = sorted((round(d[1][0][1], 3), round(d[1][1][1], 3)) for d in a.call("get_k_center"))
        cb = sorted((round(d[1][0][1], 3), round(d[1][1][1], 3)) for d in b.call("get_k_center"))
        assert ca == cb, (ca, cb)
        # every true center is found (a's and b's data together)
        for cx, cy in centers:
            assert min(abs(x - cx) + abs(y - cy) for x, y in ca) < 1.5, ca
        sa = status(a)
        assert sa["linear_mixer.runtime"] == "native" and int(sa["linear_mixer.last_mix_bytes"]) > 0
    finally:
        stop(procs)
        ls.close()
