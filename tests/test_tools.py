"""Operations tools: jubaconv, jubaconfig, jubavisor + jubactl (cluster
start / status / save / load / stop through the supervisor), jubadump
(reference C31-C34; the reference's own jubavisor test is empty, so this is
our coverage)."""
import io
import json
import os
import socket
import time

import pytest

from jubatus_amd.cmd import jubaconfig, jubaconv, jubactl, jubadump
from jubatus_amd.cmd.jubavisor import Jubavisor, argv_from_wire, argv_to_wire, split_server_name
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import CoordinatorServer
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import RpcServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


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


def test_jubavisor_jubactl_cluster(coord, tmp_path, monkeypatch):
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    zk = f"127.0.0.1:{coord.port}"
    vport = free_port()
    visor = Jubavisor(zk, vport, max_children=4, listen_addr="127.0.0.1")
    rpc = RpcServer(2)
    rpc.add("start", visor.start, arity=3)
    rpc.add("stop", visor.stop, arity=2)
    rpc.listen(vport, "127.0.0.1")
    rpc.start()
    ls = CoordinatorClient(zk, timeout=5.0)
    out = []
    try:
        assert jubaconfig.main(["-c", "write", "-f", os.path.join(ROOT, "config/classifier/arow.json"),
                                "-t", "classifier", "-n", "cl", "-z", zk], out=out.append) == 0
        common = ["-s", "jubaclassifier", "-n", "cl", "-t", "classifier", "-z", zk]
        assert jubactl.main(["-c", "start", "-N", "2", "-D", str(tmp_path), "-S", "0", "-I", "0", *common]) == 0
        deadline = time.time() + 90
        while len(ls.list(mb.build_actor_path("classifier", "cl") + "/nodes")) < 2 and time.time() < deadline:
            time.sleep(0.3)
        nodes = ls.list(mb.build_actor_path("classifier", "cl") + "/nodes")
        assert len(nodes) == 2, nodes
        assert jubactl.main(["-c", "status", *common]) == 0
        assert jubactl.main(["-c", "save", "-i", "m1", *common]) == 0
        saved = [f for f in os.listdir(tmp_path) if f.endswith("m1.jubatus")]
        assert len(saved) == 2, os.listdir(tmp_path)
        assert jubactl.main(["-c", "load", "-i", "m1", *common]) == 0
        # jubadump reads one of the saved models
        dumped = jubadump.dump(os.path.join(tmp_path, saved[0]))
        assert dumped["system"]["type"] == "classifier" and dumped["model"]["method"] == "AROW"
        assert jubactl.main(["-c", "stop", *common]) == 0
        deadline = time.time() + 30
        while ls.list(mb.build_actor_path("classifier", "cl") + "/nodes") and time.time() < deadline:
            time.sleep(0.3)
        assert ls.list(mb.build_actor_path("classifier", "cl") + "/nodes") == []
    finally:
        rpc.stop()
        visor.close()
        ls.close()
