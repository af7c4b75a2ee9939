"""Operations tools: jubaconv, jubaconfig, jubavisor + jubactl (cluster
start / status / save / load / stop through the supervisor), jubadump
(reference C31-C34; the reference's own jubavisor test is empty, so this is
our coverage)."""
import io
import json
import os
import socket
import subprocess
import time

import pytest

from jubatus_amd.cmd import jubaconfig, jubaconv, jubactl, jubadump
from jubatus_amd.cmd.jubavisor import Jubavisor, argv_from_wire, argv_to_wire, split_server_name
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import CoordinatorServer
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import RpcClient, RpcMethodNotFound, RpcServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE_BIN_DIR = os.path.join(ROOT, "jubatus_amd", "native_bin")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def free_port_block(n: int = 4) -> int:
    """a free port whose next n ports are free too (jubavisor hands its
    children the ports after its own)"""
    for _ in range(200):
        base = free_port()
        socks = []
        try:
            for q in range(base, base + n + 1):
                s = socket.socket()
                socks.append(s)
                s.bind(("127.0.0.1", q))
            return base
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    raise RuntimeError("no free port block")


@pytest.fixture
def coord():
    srv = CoordinatorServer(0, "127.0.0.1").start()
    yield srv
    srv.stop()


def test_jubaconv_json_datum_fv(tmp_path):
    js = '{"user": {"name": "taro", "age": 31, "tags": ["a", "b"], "vip": true, "x": null}}'
    out = io.StringIO()
    assert jubaconv.main(["-i", "json", "-o", "datum"], stdin=io.StringIO(js), out=out) == 0
    d = json.loads(out.getvalue())
    assert ["/user/name", "taro"] in d["string_values"] and ["/user/tags[1]", "b"] in d["string_values"]
    assert ["/user/age", 31.0] in d["num_values"] and ["/user/vip", 1.0] in d["num_values"]
    cfg = tmp_path / "c.json"
    cfg.write_text(json.dumps({"converter": {"string_rules": [{"key": "*", "type": "str",
                                                                "sample_weight": "bin", "global_weight": "bin"}],
                                              "num_rules": [{"key": "*", "type": "num"}]}}))
    out = io.StringIO()
    assert jubaconv.main(["-o", "fv", "-c", str(cfg)], stdin=io.StringIO(js), out=out) == 0
    lines = out.getvalue().splitlines()
    assert "/user/name$taro@str#bin/bin: 1" in lines and "/user/age@num: 31" in lines
    out = io.StringIO()
    assert jubaconv.main(["-i", "datum", "-o", "fv", "-c", str(cfg)],
                         stdin=io.StringIO(json.dumps(d)), out=out) == 0
    assert "/user/age@num: 31" in out.getvalue().splitlines()
    assert jubaconv.main(["-i", "datum", "-o", "json"], stdin=io.StringIO(json.dumps(d)), out=io.StringIO()) == -1


def test_jubaconfig(coord):
    zk = f"127.0.0.1:{coord.port}"
    out = []
    cfg = os.path.join(ROOT, "config/classifier/pa.json")
    assert jubaconfig.main(["-c", "write", "-f", cfg, "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 0
    assert jubaconfig.main(["-c", "read", "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 0
    assert json.loads(out[-1])["method"] == "PA"
    out.clear()
    assert jubaconfig.main(["-c", "list", "-z", zk], out=out.append) == 0
    assert out[0] == "config of classifier/c1:"
    assert jubaconfig.main(["-c", "delete", "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 0
    assert jubaconfig.main(["-c", "read", "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 1


def test_jubavisor_wire_helpers():
    assert split_server_name("jubaclassifier/foo") == ("jubaclassifier", "foo")
    with pytest.raises(ValueError):
        split_server_name("classifier")
    d = {"port": 1, "name": "x", "mixer": "linear_mixer", "daemon": False}
    assert argv_from_wire(argv_to_wire(d))["mixer"] == "linear_mixer"
    assert jubactl.split_counts(5, 2) == [3, 2] and jubactl.split_counts(0, 3) == [1, 1, 1]


def _cluster_roundtrip(zk, ls, tmp_path, gpus=0):
    """jubactl start 2 / status / save / load / stop against the registered supervisor(s);
    gpus > 0: the supervisor hands out one device per child (--gpu), visible in get_status"""
    out = []
    assert jubaconfig.main(["-c", "write", "-f", os.path.join(ROOT, "config/classifier/arow.json"),
                            "-t", "classifier", "-n", "cl", "-z", zk], out=out.append) == 0
    common = ["-s", "jubaclassifier", "-n", "cl", "-t", "classifier", "-z", zk]
    assert jubactl.main(["-c", "start", "-N", "2", "-D", str(tmp_path), "-S", "0", "-I", "0", *common]) == 0
    nodes_path = mb.build_actor_path("classifier", "cl") + "/nodes"
    deadline = time.time() + 90
    while len(ls.list(nodes_path)) < 2 and time.time() < deadline:
        time.sleep(0.3)
    nodes = ls.list(nodes_path)
    assert len(nodes) == 2, nodes
    assert jubactl.main(["-c", "status", *common]) == 0
    if gpus:
        seen = []
        for n in nodes:
            host, port = n.rsplit("_", 1)
            with RpcClient(host, int(port), 10.0) as c:
                st = c.call("get_status", "cl")
            st = {k.decode() if isinstance(k, bytes) else k: v for k, v in st.items()}
            v = list(st.values())[0]
            v = {(k.decode() if isinstance(k, bytes) else k): (x.decode() if isinstance(x, bytes) else x)
                 for k, x in v.items()}
            seen.append(v["gpu"])
        assert sorted(seen) == ["0", "1"], seen
    assert jubactl.main(["-c", "save", "-i", "m1", *common]) == 0
    saved = [f for f in os.listdir(tmp_path) if f.endswith("m1.jubatus")]
    assert len(saved) == 2, os.listdir(tmp_path)
    assert jubactl.main(["-c", "load", "-i", "m1", *common]) == 0
    # jubadump reads one of the saved models
    dumped = jubadump.dump(os.path.join(tmp_path, saved[0]))
    assert dumped["system"]["type"] == "classifier" and dumped["model"]["method"] == "AROW"
    assert jubactl.main(["-c", "stop", *common]) == 0
    deadline = time.time() + 30
    while ls.list(nodes_path) and time.time() < deadline:
        time.sleep(0.3)
    assert ls.list(nodes_path) == []


def test_jubavisor_jubactl_cluster(coord, tmp_path, monkeypatch):
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    zk = f"127.0.0.1:{coord.port}"
    vport = free_port_block()
    visor = Jubavisor(zk, vport, max_children=4, listen_addr="127.0.0.1", gpus=2)
    rpc = RpcServer(2)
    rpc.add("start", visor.start, arity=3)
    rpc.add("stop", visor.stop, arity=2)
    rpc.listen(vport, "127.0.0.1")
    rpc.start()
    ls = CoordinatorClient(zk, timeout=5.0)
    try:
        _cluster_roundtrip(zk, ls, tmp_path, gpus=2)
    finally:
        rpc.stop()
        visor.close()
        ls.close()


def _native_visor(zk, vport, tmp_path, maxc=4, gpus=None):
    exe = os.path.join(NATIVE_BIN_DIR, "jubavisor")
    if not os.access(exe, os.X_OK):
        pytest.skip("native jubavisor not built (python -m jubatus_amd.build_ext)")
    err = open(tmp_path / "visor.err", "w")
    extra = ["-G", str(gpus)] if gpus is not None else []
    p = subprocess.Popen([exe, "-p", str(vport), "-z", zk, "-m", str(maxc), "-b", "127.0.0.1", *extra],
                         stdout=subprocess.PIPE, stderr=err, text=True)
    line = p.stdout.readline()
    assert line.startswith("jubavisor ready"), (line, (tmp_path / "visor.err").read_text())
    return p, err


def test_native_jubavisor_jubactl_cluster(coord, tmp_path, monkeypatch):
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    zk = f"127.0.0.1:{coord.port}"
    vport = free_port_block()
    proc, err = _native_visor(zk, vport, tmp_path, gpus=2)
    ls = CoordinatorClient(zk, timeout=5.0)
    try:
        assert ls.list(mb.JUBAVISOR_BASE_PATH) == [f"127.0.0.1_{vport}"]
        _cluster_roundtrip(zk, ls, tmp_path, gpus=2)
    finally:
        proc.terminate()
        rc = proc.wait(30)
        err.close()
        ls.close()
    assert rc == 0, (tmp_path / "visor.err").read_text()[-2000:]


def test_native_jubavisor_rpc_errors_and_shutdown(coord, tmp_path, monkeypatch):
    """bad names / arity, pool exhaustion, and SIGTERM stopping the children"""
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    zk = f"127.0.0.1:{coord.port}"
    vport = free_port_block(1)
    proc, err = _native_visor(zk, vport, tmp_path, maxc=1)
    ls = CoordinatorClient(zk, timeout=5.0)
    argv = argv_to_wire({"threadnum": 2, "timeout": 10, "interval_sec": 0, "interval_count": 0,
                         "datadir": str(tmp_path), "mixer": "linear_mixer"})
    assert jubaconfig.main(["-c", "write", "-f", os.path.join(ROOT, "config/classifier/pa.json"),
                            "-t", "classifier", "-n", "cx", "-z", zk], out=lambda *a, **k: None) == 0
    try:
        with RpcClient("127.0.0.1", vport, 10.0) as c:
            assert c.call("start", "classifier", 1, argv) == -1          # not juba<engine>/<name>
            assert c.call("start", "jubaclassifier/", 1, argv) == -1
            assert c.call("stop", "nothing", 1) == -1
            assert c.call("stop", "jubaclassifier/none", 1) == 0
            with pytest.raises(RpcMethodNotFound):
                c.call("restart", "jubaclassifier/x", 1)
            with pytest.raises(Exception):
                c.call("start", "jubaclassifier/x")                       # arity
            assert c.call("start", "jubaclassifier/cx", 2, argv) == -1    # pool of 1 port
            assert c.call("start", "jubaclassifier/cx", 1, argv) == 0
        nodes_path = mb.build_actor_path("classifier", "cx") + "/nodes"
        deadline = time.time() + 90
        while not ls.list(nodes_path) and time.time() < deadline:
            time.sleep(0.3)
        assert ls.list(nodes_path) == [f"127.0.0.1_{vport + 1}"]
    finally:
        proc.terminate()          # the supervisor takes its children down with it
        rc = proc.wait(30)
        err.close()
    deadline = time.time() + 30
    while ls.list(nodes_path) and time.time() < deadline:
        time.sleep(0.3)
    assert ls.list(nodes_path) == []
    assert ls.list(mb.JUBAVISOR_BASE_PATH) == []
    ls.close()
    assert rc == 0


def test_codestyle_clean():
    """tools/codestyle.py (include guards, whitespace, line length, unused
    imports) finds nothing in the tree"""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "codestyle.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]


def test_man_pages_current():
    """man/*.{1,8} are rendered from the tools' own --help (tools/gen_man.py)"""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_man.py"), "--check"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
