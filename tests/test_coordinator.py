"""Coordinator / lock_service / membership / CHT / config / idgen (reference
tests: zk_test.cpp:69-227, membership_test.cpp, cht_test.cpp, config_test.cpp,
global_id_generator_test.cpp - here against our own coordinator)."""
import threading
import time

import pytest

from jubatus_amd.common import cht as chtmod
from jubatus_amd.common import config as zkconfig
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import CoordinatorServer, NativeCoordinator
from jubatus_amd.common.idgen import CoordinatorIdGenerator, StandaloneIdGenerator
from jubatus_amd.common.lock_service import (CachedLockService, CoordinatorClient, LocalLockService,
                                             LockServiceMutex, ZNodeStore)


@pytest.fixture
def coord():
    srv = CoordinatorServer(0, "127.0.0.1").start()
    yield srv
    srv.stop()


@pytest.fixture(scope="module")
def native_coord():
    srv = NativeCoordinator(0, "127.0.0.1")
    yield srv
    srv.stop()


@pytest.fixture(params=["local", "remote", "native"])
def ls(request, coord, native_coord):
    if request.param == "local":
        s = LocalLockService(ZNodeStore())
    elif request.param == "remote":
        s = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=2.0)
    else:
        s = CoordinatorClient(f"127.0.0.1:{native_coord.port}", timeout=2.0)
        for top in s.list("/"):              # module-scoped server: start from an empty tree
            _rm_tree(s, "/" + top)
    yield s
    s.close()


def _rm_tree(s, path):
    for c in s.list(path):
        _rm_tree(s, f"{path}/{c}")
    s.remove(path)


def test_native_coordinator_sessions_and_errors(native_coord):
    """native server: ephemerals die with the session (close and TTL expiry),
    NO_METHOD / ARGUMENT errors like the reference rpc_server"""
    from jubatus_amd.common.mprpc import RpcClient, RpcMethodNotFound, RpcTypeError
    a = CoordinatorClient(f"127.0.0.1:{native_coord.port}", timeout=0.6)
    b = CoordinatorClient(f"127.0.0.1:{native_coord.port}", timeout=2.0)
    b.create("/nat")
    assert a.create("/nat/e", "x", True) and b.exists("/nat/e")
    assert not a.create("/nat/e/child")                 # no children under ephemerals
    a._stop.set()                                       # stop heartbeating: TTL expiry
    deadline = time.time() + 5
    while b.exists("/nat/e") and time.time() < deadline:
        time.sleep(0.05)
    assert not b.exists("/nat/e")
    c = RpcClient("127.0.0.1", native_coord.port, timeout=2.0)
    with pytest.raises(RpcMethodNotFound):
        c.call("no_such_method")
    with pytest.raises(RpcTypeError):
        c.call("create", "not-a-sid", "/p", "", False)
    assert c.call("dump")["/nat"] == ""
    b.close()


def test_create_exists_remove(ls):
    assert ls.create("/a") and ls.create("/a")          # existing persistent: ok
    assert not ls.create("/x/y")                        # missing parent
    assert ls.create("/a/b", "payload") and ls.read("/a/b") == "payload"
    assert ls.set("/a/b", "v2") and ls.read("/a/b") == "v2"
    assert ls.list("/a") == ["b"]
    assert ls.exists("/a/b") and ls.remove("/a/b") and not ls.exists("/a/b")
    assert ls.remove("/a/b")                            # removing a missing node is ok
    assert ls.read("/nope") is None


def test_seq_and_id(ls):
    ls.create("/s")
    p1, p2 = ls.create_seq("/s/n_"), ls.create_seq("/s/n_")
    assert p1 == "/s/n_0000000000" and p2 == "/s/n_0000000001"
    ls.create("/id", "")
    a, b = ls.create_id("/id", 3), ls.create_id("/id", 3)
    assert b == a + 1 and (a >> 32) == 3
    assert ls.hd_list("/s") == "n_0000000000"


def test_ephemeral_dies_with_session(coord):
    a = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=1.0)
    b = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=1.0)
    a.create("/e")
    assert a.create("/e/n1", "x", True)
    assert not a.create("/e/n1", "x", True)             # ephemeral create of existing fails
    assert b.exists("/e/n1")
    fired = threading.Event()
    b.bind_delete_watcher("/e/n1", lambda p: fired.set())
    a.close()
    assert fired.wait(3.0)
    assert not b.exists("/e/n1")
    b.close()


def test_session_expiry_runs_cleanup(coord):
    c = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=0.5)
    cleaned = threading.Event()
    c.push_cleanup(cleaned.set)
    c.create("/eph_parent")
    c.create("/eph_parent/me", "", True)
    coord.store.close_session(c.sid)                    # coordinator forgets the session
    assert cleaned.wait(3.0)
    c.close()


def test_child_and_data_watchers(ls):
    ls.create("/w")
    got = []
    ev = threading.Event()
    ls.bind_child_watcher("/w", lambda p: (got.append(("child", p)), ev.set()))
    ls.create("/w/c1")
    assert ev.wait(3.0)
    ev.clear()
    ls.bind_watcher("/w", lambda p: (got.append(("data", p)), ev.set()))
    ls.set("/w", "new")
    assert ev.wait(3.0)
    assert ("child", "/w") in got and ("data", "/w") in got


def test_mutex(ls):
    ls.create("/lk")
    m1, m2 = LockServiceMutex(ls, "/lk/l"), LockServiceMutex(ls, "/lk/l")
    assert m1.try_lock()
    assert not m2.try_lock() and not m2.try_rlock()
    m1.unlock()
    r1, r2 = LockServiceMutex(ls, "/lk/l"), LockServiceMutex(ls, "/lk/l")
    assert r1.try_rlock() and r2.try_rlock()            # shared readers
    assert not m2.try_lock()
    r1.unlock(); r2.unlock()
    assert m2.try_lock()


def test_membership_paths(ls):
    # reference membership_test.cpp
    assert mb.build_loc_str("127.0.0.1", 9199) == "127.0.0.1_9199"
    assert mb.build_loc_str("127.0.0.1", 9199, 3) == "127.0.0.1_9199_3"
    assert mb.revert("127.0.0.1_9199") == ("127.0.0.1", 9199)
    assert mb.build_actor_path("classifier", "t") == "/jubatus/actors/classifier/t"
    assert mb.build_config_path("classifier", "t") == "/jubatus/config/classifier/t"
    mb.prepare_jubatus(ls, "classifier", "t")
    mb.register_actor(ls, "classifier", "t", "127.0.0.1", 9199)
    mb.register_active(ls, "classifier", "t", "127.0.0.1", 9199)
    assert mb.get_all_nodes(ls, "classifier", "t") == [("127.0.0.1", 9199)]
    assert mb.get_all_actives(ls, "classifier", "t") == [("127.0.0.1", 9199)]
    mb.unregister_active(ls, "classifier", "t", "127.0.0.1", 9199)
    assert mb.get_all_actives(ls, "classifier", "t") == []


def test_cht(ls):
    # reference cht_test.cpp: make_hash is md5 hex
    assert chtmod.make_hash("hoge") == __import__("hashlib").md5(b"hoge").hexdigest()
    mb.prepare_jubatus(ls, "anomaly", "c")
    chtmod.CHT.setup_cht_dir(ls, "anomaly", "c")
    c = chtmod.CHT(ls, "anomaly", "c")
    for p in (9001, 9002, 9003):
        c.register_node("127.0.0.1", p)
    assert len(ls.list(c.path)) == 3 * chtmod.NUM_VSERV
    owners = c.find("row-42", 2)
    assert len(owners) == 2 and all(h == "127.0.0.1" for h, _ in owners)
    assert c.find("row-42", 2) == owners                # deterministic
    # keys spread over every server
    seen = {c.find(f"k{i}", 1)[0][1] for i in range(200)}
    assert seen == {9001, 9002, 9003}
    c.unregister_node("127.0.0.1", 9002)
    assert all(p != 9002 for _, p in (c.find(f"k{i}", 1)[0] for i in range(50)))


def test_config_roundtrip_and_lock(ls):
    zkconfig.config_tozk(ls, "classifier", "t", '{"method": "PA"}')
    assert zkconfig.config_fromzk(ls, "classifier", "t") == '{"method": "PA"}'
    with pytest.raises(zkconfig.ConfigError):
        zkconfig.config_tozk(ls, "classifier", "t", "{bad json")
    lock = zkconfig.get_config_lock(ls, "classifier", "t")   # a running server's read lock
    with pytest.raises(zkconfig.ConfigError):
        zkconfig.config_tozk(ls, "classifier", "t", '{"method": "AROW"}')
    lock.unlock()
    mb.register_actor(ls, "classifier", "t", "127.0.0.1", 1)  # a server is running
    with pytest.raises(zkconfig.ConfigError):
        zkconfig.remove_config_fromzk(ls, "classifier", "t")
    mb.unregister_actor(ls, "classifier", "t", "127.0.0.1", 1)
    zkconfig.remove_config_fromzk(ls, "classifier", "t")
    with pytest.raises(zkconfig.ConfigError):
        zkconfig.config_fromzk(ls, "classifier", "t")


def test_idgen(ls):
    g = StandaloneIdGenerator()
    assert [g.generate() for _ in range(3)] == [0, 1, 2]
    mb.prepare_jubatus(ls, "anomaly", "t")
    z = CoordinatorIdGenerator(ls, "anomaly", "t")
    ids = [z.generate() for _ in range(5)]
    assert ids == sorted(set(ids))


def test_cached_lock_service(ls):
    c = CachedLockService(ls)
    ls.create("/cc")
    assert c.list("/cc") == []
    ls.create("/cc/x")
    deadline = time.time() + 3
    while c.list("/cc") != ["x"] and time.time() < deadline:
        time.sleep(0.05)
    assert c.list("/cc") == ["x"]


def test_coordinator_twins_agree_op_by_op(coord, native_coord):
    """the Python coordinator (common/coordinator.py, the test harness and
    fallback) and the native one (csrc/coord/jubacoordinator.cpp, production)
    answer a seeded random sequence of lock_service operations identically,
    call by call"""
    import random
    py = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=2.0)
    na = CoordinatorClient(f"127.0.0.1:{native_coord.port}", timeout=2.0)
    for s in (py, na):
        for top in s.list("/"):
            _rm_tree(s, "/" + top)
        s.create("/twin")
    rng = random.Random(7)
    names = ["/twin/a", "/twin/b", "/twin/a/x", "/twin/b/y", "/twin/c", "/twin/a/x/z"]
    for step in range(400):
        op = rng.choice(["create", "create_eph", "set", "read", "exists", "list", "remove", "seq", "id"])
        p = rng.choice(names)
        val = f"v{rng.randrange(5)}"
        res = []
        for s in (py, na):
            if op == "create":
                r = s.create(p, val)
            elif op == "create_eph":
                r = s.create(p, val, True)
            elif op == "set":
                r = s.set(p, val)
            elif op == "read":
                r = s.read(p)
            elif op == "exists":
                r = s.exists(p)
            elif op == "list":
                r = sorted(s.list(p))
            elif op == "remove":
                r = s.remove(p)
            elif op == "seq":
                r = s.create_seq(p + "/q_")
            else:
                r = s.create_id(p, 1) if s.exists(p) else None
            res.append(r)
        assert res[0] == res[1], (step, op, p, res)
    assert sorted(py.list("/twin")) == sorted(na.list("/twin"))
    py.close()
    na.close()
