"""Multi-process cluster on one host (reference strategy: several servers on
localhost ports + a local coordinator, client_test/envdef.sample.py:13-18).

Two jubaclassifier processes (host backend, gloo process group) join a
cluster through our coordinator; training lands on one server only and a
MIX makes the other one learn it: linear_mixer (all-reduce mean) and the
push mixers (pairwise send/recv)."""
import os
import socket
import subprocess
import tempfile
import sys
import time

import pytest

from jubatus_amd.client import Classifier, Datum
from jubatus_amd.common import config as zkconfig
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import CoordinatorServer, NativeCoordinator, native_available
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import wait_server

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(params=["native"])
def coord(request):
    # the production coordinator: native C++ server (csrc/coord), no Python
    srv = NativeCoordinator(0, "127.0.0.1") if native_available() else \
        CoordinatorServer(0, "127.0.0.1").start()
    yield srv
    srv.stop()


LOGDIR = os.environ.get("JUBATUS_TEST_LOGDIR", tempfile.gettempdir())


def spawn(engine, zport, name, port, mixer="linear_mixer", extra=(), env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT, JUBATUS_FORCE_CPU="1", **(env_extra or {}))
    cmd = [sys.executable, "-m", "jubatus_amd.cmd.server", engine, "-z", f"127.0.0.1:{zport}",
           "-n", name, "-p", str(port), "-b", "127.0.0.1", "-x", mixer, "-s", "0", "-i", "0",
           "-I", "5", "--cpu", *extra]
    log = open(os.path.join(LOGDIR, f"{engine}_{name}_{port}.log"), "wb")
    return subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=log)


def wait_actives(ls, engine, name, n, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if len(mb.get_all_actives(ls, engine, name)) >= n:
            return True
        time.sleep(0.2)
    return False


@pytest.mark.parametrize("mixer", ["linear_mixer", "skip_mixer", "random_mixer", "broadcast_mixer"])
def test_two_server_mix(coord, mixer):
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = f"dist_{mixer}"
    zkconfig.config_tozk(ls, "classifier", name, open(os.path.join(ROOT, "config/classifier/arow.json")).read())
    ports = [free_port(), free_port()]
    procs = [spawn("classifier", coord.port, name, p, mixer) for p in ports]
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 60), "server did not start"
        assert wait_actives(ls, "classifier", name, 2), "servers did not become active"
        a = Classifier("127.0.0.1", ports[0], name)
        b = Classifier("127.0.0.1", ports[1], name)
        a.train([("pos", Datum({"w": "good"})), ("neg", Datum({"w": "bad"}))] * 3)
        assert b.get_labels() == {}
        assert a.do_mix() is True
        deadline = time.time() + 20
        key = f"{mixer}.mix_count"
        while int(list(b.get_status().values())[0][key]) < 1 and time.time() < deadline:
            time.sleep(0.2)
        assert set(b.get_labels()) == {"pos", "neg"}
        top = max(b.classify([Datum({"w": "good"})])[0], key=lambda e: e.score)
        assert top.label == "pos"
        if mixer == "linear_mixer":
            # model averaging: both servers hold the same model after the MIX
            sa = {e.label: e.score for e in a.classify([Datum({"w": "good"})])[0]}
            sb = {e.label: e.score for e in b.classify([Datum({"w": "good"})])[0]}
            assert sa.keys() == sb.keys()
            assert all(abs(sa[k] - sb[k]) < 1e-5 for k in sa)
            assert b.get_labels() == {"pos": 3, "neg": 3}  # counts mixed (sum of deltas)
        st = list(b.get_status().values())[0]
        assert st["mixer"] == mixer and st["is_standalone"] == "0"
        # distributed-mode keys (reference client_test/status_test.hpp:47-56)
        for k in ("connected_zookeeper", "interconnect_timeout", "interval_count", "interval_sec",
                  "mixer", "name", "use_cht", "zk", "zookeeper_timeout"):
            assert k in st, k
        assert int(st[f"{mixer}.mix_count"]) >= 1
        a.close()
        b.close()
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
        ls.close()


def test_server_self_fences_when_actor_deleted(coord):
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    zkconfig.config_tozk(ls, "classifier", "fence", open(os.path.join(ROOT, "config/classifier/pa.json")).read())
    port = free_port()
    p = spawn("classifier", coord.port, "fence", port)
    try:
        assert wait_server("127.0.0.1", port, 60)
        assert wait_actives(ls, "classifier", "fence", 1)
        ls.remove(f"/jubatus/actors/classifier/fence/nodes/127.0.0.1_{port}")
        p.wait(timeout=30)   # stops itself (server_helper.cpp:91-94)
        assert p.returncode == 0
    finally:
        if p.poll() is None:
            p.kill()
        ls.close()


class _NativeProxy:
    """csrc/proxy/jubaproxy.cpp as a child process"""

    def __init__(self, engine, zport):
        from jubatus_amd import build_ext
        exe = os.path.join(build_ext.NATIVE_BIN, "jubaproxy")
        if not os.access(exe, os.X_OK):
            build_ext.build_tools()
        self.port = free_port()
        self.proc = subprocess.Popen([exe, engine, "-p", str(self.port), "-b", "127.0.0.1",
                                      "-z", f"127.0.0.1:{zport}", "-I", "5"],
                                     stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        line = self.proc.stdout.readline()
        assert line.startswith("jubaproxy ready"), line

    def stop(self):
        self.proc.terminate()
        self.proc.wait(10)


def _start_proxy(impl, engine, zport):
    if impl == "native":
        return _NativeProxy(engine, zport)
    from jubatus_amd.framework.proxy import Proxy
    from jubatus_amd.framework.server_util import ProxyArgv
    pa = ProxyArgv(type=engine, port=0, bind_address="127.0.0.1", eth="127.0.0.1",
                   z=f"127.0.0.1:{zport}", program_name=f"juba{engine}_proxy")
    proxy = Proxy(pa)
    proxy.start(block=False)
    proxy.port = pa.port
    return proxy


@pytest.mark.parametrize("impl", ["python", "native"])
def test_proxy_routing(coord, impl):
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = "viaproxy"
    zkconfig.config_tozk(ls, "classifier", name, open(os.path.join(ROOT, "config/classifier/pa.json")).read())
    ports = [free_port(), free_port()]
    procs = [spawn("classifier", coord.port, name, p) for p in ports]
    proxy = _start_proxy(impl, "classifier", coord.port)

    class pa:  # noqa: N801
        port = proxy.port
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 60)
        assert wait_actives(ls, "classifier", name, 2)
        c = Classifier("127.0.0.1", pa.port, name)
        for _ in range(10):  # random routing spreads the requests
            assert c.train([("a", Datum({"k": "x"})), ("b", Datum({"k": "y"}))]) == 2
        st = c.get_status()                      # broadcast + merge
        assert len(st) == 2
        assert sum(int(s["update_count"]) for s in st.values()) == 10
        assert c.set_label("z") is True          # broadcast + all_and
        assert all("z" in Classifier("127.0.0.1", p, name).get_labels() for p in ports)
        saved = c.save("px")                     # broadcast + merge
        assert len(saved) == 2
        assert c.load("px") is True
        ps = c.get_proxy_status()
        (k, v), = ps.items()
        assert int(v["request_count"]) >= 14 and int(v["forward_count"]) >= 16
        from jubatus_amd.common.mprpc import RpcCallError
        with pytest.raises(RpcCallError):
            Classifier("127.0.0.1", pa.port, "no_such_cluster").get_config()
        c.close()
    finally:
        proxy.stop()
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
        ls.close()


def test_native_proxy_cht_routing(coord):
    """cht(2) methods reach the two CHT owners of the row id; random analysis
    methods see the row (recommender, native proxy)"""
    from jubatus_amd.client import Recommender
    from jubatus_amd.common.cht import CHT
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = "chtproxy"
    zkconfig.config_tozk(ls, "recommender", name,
                         open(os.path.join(ROOT, "config/recommender/inverted_index.json")).read())
    ports = []
    while len(ports) < 3:
        p = free_port()
        if p not in ports:
            ports.append(p)
    procs = [spawn("recommender", coord.port, name, p) for p in ports]
    proxy = _NativeProxy("recommender", coord.port)
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 60)
        assert wait_actives(ls, "recommender", name, 3)
        r = Recommender("127.0.0.1", proxy.port, name)
        for i in range(12):
            assert r.update_row(f"row{i}", Datum({"a": float(i), "b": 1.0})) is True
        cht = CHT(ls, "recommender", name)
        for i in range(12):
            owners = {p for _, p in cht.find(f"row{i}", 2)}
            for p in ports:
                rows = Recommender("127.0.0.1", p, name).get_all_rows()
                assert (f"row{i}" in rows) == (p in owners), (i, p, owners)
        assert r.decode_row("row3").num_values                    # cht analysis
        assert r.clear() is True                                   # broadcast all_and
        r.close()
    finally:
        proxy.stop()
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
        ls.close()


def test_rank_killed_mid_mix_survivor_recovers(coord):
    """fault injection kills one server when its first MIX reaches the
    all-reduce; the survivor re-forms the group alone, keeps serving and
    keeps its model (SURVEY §5.3 elastic recovery)."""
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = "faulty"
    zkconfig.config_tozk(ls, "classifier", name, open(os.path.join(ROOT, "config/classifier/pa.json")).read())
    ports = [free_port(), free_port()]
    fast = ("-Z", "2")   # short coordinator session: the dead rank's nodes expire quickly
    good = spawn("classifier", coord.port, name, ports[0], extra=fast)
    bad = spawn("classifier", coord.port, name, ports[1], extra=fast,
                env_extra={"JUBATUS_FAULT": "mix_kill:phase=allreduce,at=1"})
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 60)
        assert wait_actives(ls, "classifier", name, 2)
        a = Classifier("127.0.0.1", ports[0], name, timeout=90.0)
        a.train([("pos", Datum({"w": "good"})), ("neg", Datum({"w": "bad"}))] * 3)
        try:
            a.do_mix()                  # the faulty rank dies inside this MIX
        except Exception:
            pass
        bad.wait(timeout=60)
        assert bad.returncode == 17
        deadline = time.time() + 120
        ok = False
        while time.time() < deadline:
            try:
                if a.do_mix():          # alone again: the mixer runs and reports success
                    ok = True
                    break
            except Exception:
                pass
            time.sleep(0.5)
        assert ok
        top = max(a.classify([Datum({"w": "good"})])[0], key=lambda e: e.score)
        assert top.label == "pos"
        a.close()
    finally:
        for p in (good, bad):
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    p.kill()
        ls.close()


def test_stalled_rank_watchdog_aborts_and_regroups(coord):
    """one server stalls its first MIX past --interconnect_timeout (fault
    mix_hang): the other one's watchdog aborts the group instead of hanging,
    keeps serving, and the two re-form a group whose next MIX succeeds
    (reference: interconnect_timeout bounds server-to-server calls,
    server_util.cpp:190-194; failed peers are skipped, linear_mixer.cpp:455-489)."""
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = "stall"
    zkconfig.config_tozk(ls, "classifier", name, open(os.path.join(ROOT, "config/classifier/pa.json")).read())
    ports = [free_port(), free_port()]
    good = spawn("classifier", coord.port, name, ports[0], extra=("-I", "2"))
    slow = spawn("classifier", coord.port, name, ports[1], extra=("-I", "2"),
                 env_extra={"JUBATUS_FAULT": "mix_hang:phase=allreduce,at=1,ms=7000"})
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 60)
        assert wait_actives(ls, "classifier", name, 2)
        a = Classifier("127.0.0.1", ports[0], name, timeout=90.0)
        a.train([("pos", Datum({"w": "good"})), ("neg", Datum({"w": "bad"}))] * 3)
        t0 = time.time()
        try:
            a.do_mix()                  # the slow rank stalls inside this MIX
        except Exception:
            pass
        # the survivor is not stuck: it serves while the group is aborted
        assert max(a.classify([Datum({"w": "good"})])[0], key=lambda e: e.score).label == "pos"
        deadline = time.time() + 120
        ok = False
        while time.time() < deadline:
            try:
                if a.do_mix():
                    st = list(a.get_status().values())[0]
                    if st.get("linear_mixer.group_size") == "2":
                        ok = True
                        break
            except Exception:
                pass
            time.sleep(0.5)
        assert ok, "no MIX with both members after the stall"
        st = list(a.get_status().values())[0]
        assert int(st["linear_mixer.watchdog_aborts"]) >= 1
        assert time.time() - t0 < 120
        b = Classifier("127.0.0.1", ports[1], name, timeout=30.0)
        top = max(b.classify([Datum({"w": "good"})])[0], key=lambda e: e.score)
        assert top.label == "pos"       # the mixed model reached the stalled rank
        a.close()
        b.close()
    finally:
        for p in (good, slow):
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    p.kill()
        ls.close()
